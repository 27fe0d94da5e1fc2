#!/bin/bash
# GPU test run on the box: the given pytest selection (default: the whole -m gpu
# suite, the ingest tests first), each test bounded, output under gpurun_out/t.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/t
SEL="${@:-tests/test_gpu_ingest.py tests}"
timeout -k 10 1000 python3 -u -m pytest $SEL -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/t/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t/pytest.log
[ $rc -eq 0 ] || grep -B2 -A40 "Error\|FAILED\|assert" gpurun_out/t/pytest.log | head -80
exit $rc
