#!/bin/bash
# Round-3 iteration on the box: ingest tests, the default (end-to-end cfg2)
# bench line, then cfg5 device-resident with KC_DEBUG (P5 passes) and trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/i; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ingest.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -B2 -A30 "Error\|FAILED" $O/pytest.log | head -60; exit $rc; }
timeout -k 10 600 python3 -u bench.py --steps 2 --warmup 1 > $O/bench2.json 2> $O/bench2.err
rc=$?; echo "bench cfg2 rc=$rc"; cut -c1-1500 $O/bench2.json; [ $rc -eq 0 ] || { tail -20 $O/bench2.err; exit $rc; }
KC_DEBUG=1 KC_TRACE=1 timeout -k 10 600 python3 -u bench.py --config 5 --mode device --steps 1 --warmup 1 --no-cpu --no-variants > $O/bench5.json 2> $O/bench5.err
rc=$?; echo "bench cfg5 rc=$rc"; cut -c1-2500 $O/bench5.json; [ $rc -eq 0 ] || { tail -20 $O/bench5.err; exit $rc; }
exit 0
