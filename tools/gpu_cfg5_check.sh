#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/c5; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fq_encode.py tests/test_gpu_parity.py tests/test_varlen.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" $O/pytest.log | head -60; exit $rc; }
for rep in 1 2; do
  timeout -k 10 600 python3 bench.py --config 5 --steps 5 --warmup 2 --no-e2e --no-cpu --no-variants > $O/cfg5.$rep.json 2> $O/cfg5.$rep.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 $O/cfg5.$rep.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('$O/cfg5.$rep.json').read().strip().splitlines()[-1]); print('cfg5', $rep, round(d['value']/1e9,2), round(d['ms_per_step'],2), d['device_resident']['breakdown_ms_per_step'])"
done
