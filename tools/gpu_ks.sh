#!/bin/bash
# Key-space exchange: new GPU tests first, then the whole GPU suite (minus the
# full-size case), then the 2-rank rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -m pytest tests -m gpu -x -q -k "keyspace or merge_records" > gpurun_out/pytest_ks.log 2>&1
rc=$?; echo "pytest ks rc=$rc"; tail -30 gpurun_out/pytest_ks.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q -k "not full_size" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_dist.sh
