#!/bin/bash
# rocprofv3 kernel stats of one bench step (after one warmup) per variant;
# VARIANTS = space-separated env assignments (use "-" for the default).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ks
i=0
for v in ${VARIANTS:--}; do
  i=$((i+1))
  ( [ "$v" != "-" ] && export ${v//,/ }
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ks/v$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu ${BENCH_ARGS:-} > gpurun_out/ks/v$i.json 2> gpurun_out/ks/v$i.err )
  rc=$?; echo "== variant $i ($v) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/ks/v$i.err; exit $rc; }
  python3 -c "
import json;d=json.load(open('gpurun_out/ks/v$i.json'));print(round(d['value']/1e9,2),'e9', round(d['ms_per_step'],2),'ms')"
  f=$(find gpurun_out/ks/v$i -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print(f"{float(r['AverageNs'])/1e6:9.3f} ms x{r['Calls']:>3}  {r['Name'][:90]}")
PY
done
