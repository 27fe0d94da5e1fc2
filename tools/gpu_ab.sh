#!/bin/bash
# Same-box A/B of library paths on the device-resident bench. Optional
# pytest selection first (AB_TESTS), then for each repetition every variant
# of AB (space-separated name=VAR:VAL,VAR:VAL ...; test hooks need
# KC_TEST_HOOKS=1, which the variants get) in its own process; prints value,
# ms/step, FASTQ index time and the per-kernel ms/step of each run.
#   AB="base= nolb=KC_NO_FQ_LB:1" AB_TESTS="tests/test_gpu_fq_encode.py" bash tools/gpu_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
if [ -n "$AB_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest $AB_TESTS -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" $O/pytest.log | head -80; exit $rc; }
fi
for rep in $(seq 1 ${AB_REPS:-2}); do
  for spec in $AB; do
    name=${spec%%=*}; envs=${spec#*=}
    ( export KC_TEST_HOOKS=1
      for kv in ${envs//,/ }; do export "${kv%%:*}=${kv#*:}"; done
      timeout -k 10 300 python3 bench.py --config ${AB_CONFIG:-2} --steps ${AB_STEPS:-5} --warmup 2 --no-cpu --no-e2e --no-variants > $O/$name.$rep.json 2> $O/$name.$rep.err )
    rc=$?; [ $rc -eq 0 ] || { echo "bench $name rc=$rc"; tail -5 $O/$name.$rep.err; exit $rc; }
    python3 -c "
import json; d=json.loads(open('$O/$name.$rep.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']
b=d['device_resident']['breakdown_ms_per_step']
print('$name', $rep, round(d['value']/1e9,2), 'e9', round(d['ms_per_step'],2), 'ms idx', round(b['fastq_index'],2), 'fin', round(b['finish'],2), {t: k[t]['ms_per_step'] for t in k})"
  done
done
