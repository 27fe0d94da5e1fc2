#!/bin/bash
# cfg4 shard, one device step with KC_DEBUG (P5 passes / aborts / max m per
# launch) in one batch and, for comparison, in safe batches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/cfg4dbg; mkdir -p $O
KC_DEBUG=1 timeout -k 10 600 python3 bench.py --config 4 --steps 1 --warmup 0 --no-cpu --no-e2e --no-variants > $O/big.json 2> $O/big.err
rc=$?; echo "big rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/big.err; exit $rc; }
KC_SKM_SAFE_BATCH=1 KC_DEBUG=1 timeout -k 10 600 python3 bench.py --config 4 --steps 1 --warmup 0 --no-cpu --no-e2e --no-variants > $O/safe.json 2> $O/safe.err
rc=$?; echo "safe rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/safe.err; exit $rc; }
grep -h "skm F records\|dedup\|P5" $O/big.err | tail -6; echo ---; grep -h "skm F records\|dedup\|P5" $O/safe.err | tail -8
