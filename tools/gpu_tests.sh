#!/bin/bash
# GPU test run on the box: the given pytest selection (default: the whole -m gpu
# suite, the ingest tests first), each test bounded, output under gpurun_out/t.
# A heartbeat file keeps long single tests (the full-size parity checks run
# minutes of CPU oracle work) visible to the box's silence check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/t
(while sleep 50; do date +%T >> gpurun_out/t/heartbeat; done) &
HB=$!
if [ $# -eq 0 ]; then set -- tests/test_gpu_ingest.py tests; fi
timeout -k 10 1150 python3 -u -m pytest "$@" -x -q -m gpu --timeout 180 --timeout-method thread --durations=25 > gpurun_out/t/pytest.log 2>&1
rc=$?; kill $HB; echo "pytest rc=$rc"; tail -30 gpurun_out/t/pytest.log
[ $rc -eq 0 ] || grep -B2 -A40 "Error\|FAILED\|assert" gpurun_out/t/pytest.log | head -80
exit $rc
