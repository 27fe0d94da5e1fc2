#!/bin/bash
# cfg3 and cfg4 per-GPU shards at N = 1 (their 8-GPU runs are the driver's)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/cfg34; mkdir -p $O
timeout -k 10 600 python3 bench.py --config 3 --steps 5 --warmup 2 --no-cpu --no-variants --no-e2e > $O/cfg3.json 2> $O/cfg3.err
rc=$?; echo "cfg3 rc=$rc"; cut -c1-260 $O/cfg3.json; [ $rc -eq 0 ] || { tail -5 $O/cfg3.err; exit $rc; }
timeout -k 10 900 python3 bench.py --config 4 --steps 3 --warmup 1 --no-variants > $O/cfg4.json 2> $O/cfg4.err
rc=$?; echo "cfg4 rc=$rc"; cut -c1-260 $O/cfg4.json; [ $rc -eq 0 ] || { tail -5 $O/cfg4.err; exit $rc; }
