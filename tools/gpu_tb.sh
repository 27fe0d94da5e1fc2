#!/bin/bash
# GPU suite then one default bench line (no CPU baseline). Output under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.load(open('gpurun_out/bench.json'))
print(d['value']/1e9, d['ms_per_step'], d['breakdown_ms_per_step'])" 
exit $rc
