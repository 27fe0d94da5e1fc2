#!/bin/bash
# GPU suite, then the default bench line and a rocprofv3 kernel-stats run of
# the bench (tools/gpu_prof.sh). Output under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench default rc=$rc"; cut -c1-400 gpurun_out/bench_default.json
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh
