#!/bin/bash
# rocprofv3 kernel statistics of the cfg5 device-resident bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/p5; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 bench.py --config 5 --mode device \
  --steps 2 --warmup 1 --no-cpu --no-variants > $O/bench.json 2> $O/bench.err
rc=$?; echo "rc=$rc"
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/p5/kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:22]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):5d} calls {float(r["AverageNs"])/1e6:8.3f} ms avg  {r["Name"][:90]}')
PY
exit $rc
