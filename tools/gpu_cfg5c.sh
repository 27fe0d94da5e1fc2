#!/bin/bash
# Selected parity tests (-k expression in $1), cfg5 trace (auto), then the
# parity / skm / ingest GPU files.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/c5c; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "$1" > $O/sel.log 2>&1
rc=$?; tail -15 $O/sel.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_cfg5b.sh auto || exit $?
[ "$2" = "quick" ] && exit 0
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_skm.py tests/test_gpu_ingest.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
