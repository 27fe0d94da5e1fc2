#!/bin/bash
# fq_encode_k tuning: the encode parity tests on the in-tree library, then a
# same-box A/B of library variants (LIBS) on the cfg2 device-resident bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${OUT:-fqab}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fq_encode.py tests/test_gpu_ingest.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS="${LIBS:-fqold fqb256 fqb512w6 fqb256w8 fqh8b256 main}" CFG=2 STEPS=${STEPS:-5} OUT=${OUT:-fqab} bash tools/gpu_ab_lib.sh
