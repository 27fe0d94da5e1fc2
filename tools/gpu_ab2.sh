#!/bin/bash
# The large-batch skm tests, then a same-box A/B of fq_encode_k and P5a
# geometries (library variants) on the cfg2 device-resident bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/ab2; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_skm.py -k "large_batch or many_batches or pool_overflow or weighted_spill" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS="${LIBS:-fqh8b256 fqh8b128 fqh8b64 fqh8x8 p5a1024 p5a512h p5a1024h p5a256h}" CFG=2 STEPS=5 OUT=ab2 bash tools/gpu_ab_lib.sh
