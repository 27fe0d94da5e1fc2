#!/bin/bash
# One iteration: selected parity tests ($1, -k), cfg5 trace, cfg2 device bench,
# sort_runs phase ticks, then the parity / skm / ingest GPU files ($2 != quick).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/it; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "$1" > $O/sel.log 2>&1
rc=$?; tail -3 $O/sel.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_cfg5b.sh auto || exit $?
timeout -k 10 300 python3 -u bench.py --config 2 --mode device --steps 3 --warmup 1 --no-cpu --no-variants \
  > $O/cfg2.json 2> $O/cfg2.err
rc=$?; echo "cfg2 rc=$rc"; [ $rc -ne 0 ] && tail -5 $O/cfg2.err && exit $rc
python3 -c "
import json; d=json.loads(open('$O/cfg2.json').read()); r=d['device_resident']
print('cfg2', d['value'], r['ms_per_step'], r['breakdown_ms_per_step'])"
bash tools/gpu_srprof.sh > /dev/null && grep sort_runs gpurun_out/sr/b.json
[ "$2" = "quick" ] && exit 0
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_skm.py tests/test_gpu_ingest.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
