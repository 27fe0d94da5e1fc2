#!/bin/bash
# Round-4 late check: the full GPU suite and the cfg4 per-GPU shard (one skm
# batch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 bench.py --config 4 --steps 3 --warmup 1 --no-variants > $O/cfg4.json 2> $O/cfg4.err
rc=$?; echo "cfg4 rc=$rc"; cut -c1-300 $O/cfg4.json; [ $rc -eq 0 ] || { tail -5 $O/cfg4.err; exit $rc; }
