#!/bin/bash
# cfg5 (k=55, 20M iid reads, 48 GiB working set: spill runs) device-resident:
# default engine, then the key-prefix engine forced; KC_DEBUG P5 lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/c5; mkdir -p $O
if [ "$1" = "tests" ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -B2 -A30 "Error\|FAILED" $O/pytest.log | head -60; exit $rc; }
fi
for eng in auto partition; do
  KC_DEBUG=1 timeout -k 10 600 python3 -u bench.py --config 5 --mode device --engine $eng --steps 2 --warmup 1 --no-cpu --no-variants > $O/bench_$eng.json 2> $O/bench_$eng.err
  rc=$?; echo "cfg5 $eng rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench_$eng.json').read()); r=d['device_resident']
print(d['value'], r['ms_per_step'], r['breakdown_ms_per_step'], d['spill_runs'])"
  [ $rc -eq 0 ] || { tail -20 $O/bench_$eng.err; exit $rc; }
done
