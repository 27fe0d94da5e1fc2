#!/bin/bash
# The radix scatter's speed by output position inside a large allocation
# (tools/rp_bench layout -3): input region 0, output region r of R, in a few
# processes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/rpsweep; mkdir -p $O
R=${R:-14}; N=${N:-150000000}
PAIRS=$(python3 -c "print(','.join(f'0:{r}' for r in range($R)))")
for p in 1 2 3; do
  RP_NREG=$R RP_PAIRS=$PAIRS RP_NOCHECK=1 timeout -k 10 200 ./tools/rp_bench $N 2 3 1 48 -3 > $O/proc$p.txt 2>&1
  rc=$?; echo "process $p rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/proc$p.txt; exit $rc; }
  python3 -c "
import json
rows=[json.loads(l) for l in open('$O/proc$p.txt') if l.startswith('{')]
print(' '.join(f\"{r['pair'][1]}:{r['avg_ms']}\" for r in rows))"
done
