#!/bin/bash
# Same-box A/B of variant libraries (tools/build_variant.sh with
# VARIANT_DIR=kmer-counter_amd/abvar): the skm/parity GPU tests on the first
# variant named in VT (optional), then the device-resident bench alternating
# the variants (AB_REPS repetitions, AB_CONFIG).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/abv; mkdir -p $O
if [ -n "$VT" ]; then
  KC_LIB=$PWD/kmer-counter_amd/abvar/$VT/libkc_hip.so timeout -k 10 900 python3 -u -m pytest ${VTESTS:-tests/test_gpu_skm.py} -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_$VT.log 2>&1
  rc=$?; echo "pytest $VT rc=$rc"; tail -2 $O/pytest_$VT.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" $O/pytest_$VT.log | head -60; exit $rc; }
fi
for rep in $(seq 1 ${AB_REPS:-2}); do
  for v in $AB; do
    KC_TEST_HOOKS=1 KC_LIB=$PWD/kmer-counter_amd/abvar/$v/libkc_hip.so timeout -k 10 300 python3 bench.py --config ${AB_CONFIG:-2} --steps ${AB_STEPS:-5} --warmup 2 --no-cpu --no-e2e --no-variants > $O/$v.$rep.json 2> $O/$v.$rep.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -5 $O/$v.$rep.err; exit $rc; }
    python3 -c "
import json; d=json.loads(open('$O/$v.$rep.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']
b=d['device_resident']['breakdown_ms_per_step']
print('$v', $rep, round(d['value']/1e9,2), 'e9', round(d['ms_per_step'],2), 'ms idx', round(b['fastq_index'],2), 'fin', round(b['finish'],2), {t: k[t]['ms_per_step'] for t in k})"
  done
done
