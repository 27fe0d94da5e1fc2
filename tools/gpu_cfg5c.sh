#!/bin/bash
# cfg5 trace (auto), P5 fixed cost (experiment build, KC_P5_SKIP=1), then the
# segment-sort / pre-split parity tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/c5c; mkdir -p $O
bash tools/gpu_cfg5b.sh auto || exit $?
KC_LIB=$PWD/kmer-counter_amd/variants/exp/libkc_hip.so KC_P5_SKIP=1 KC_DEBUG=1 timeout -k 10 300 python3 -u bench.py \
  --config 5 --mode device --steps 1 --warmup 0 --no-cpu --no-variants > $O/skip.json 2> $O/skip.err
echo "skip rc=$?"; grep "kc: P5" $O/skip.err | head -4
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_skm.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
