#!/bin/bash
# GPU suite (no full-size), full bench with CPU baseline, rocprof kernel stats,
# PMC passes. Everything lands in gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q -k "not full_size" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh || exit $?
bash tools/gpu_pmc.sh || exit $?
timeout -k 10 600 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench default rc=$rc"; cat gpurun_out/bench_default.json
exit $rc
