#!/bin/bash
# Iteration pass: GPU parity tests (fast subset), then full-size bench + rocprof stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q -k "not full_size" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh
