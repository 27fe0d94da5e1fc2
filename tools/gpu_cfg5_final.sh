#!/bin/bash
# cfg5 device-resident bench on the final tree (with the CPU baseline), twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/cfg5f; mkdir -p $O
for r in 1 2; do
  timeout -k 10 600 python3 bench.py --config 5 --steps 5 --warmup 2 --no-e2e --no-variants > $O/cfg5_$r.json 2> $O/cfg5_$r.err
  rc=$?; echo "cfg5 run $r rc=$rc"; cut -c1-200 $O/cfg5_$r.json; [ $rc -eq 0 ] || { tail -5 $O/cfg5_$r.err; exit $rc; }
done
