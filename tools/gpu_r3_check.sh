#!/bin/bash
# Round-3 check on the box: the whole -m gpu suite, the default cfg2 bench line
# (end-to-end), then the cfg5 device-resident line with phase tracing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/c; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -B2 -A30 "Error\|FAILED" $O/pytest.log | head -60; exit $rc; }
fi
timeout -k 10 600 python3 -u bench.py --steps 3 --warmup 1 ${BENCH2_ARGS} > $O/bench2.json 2> $O/bench2.err
rc=$?; echo "bench cfg2 rc=$rc"; cut -c1-600 $O/bench2.json; [ $rc -eq 0 ] || { tail -20 $O/bench2.err; exit $rc; }
KC_TRACE=1 timeout -k 10 600 python3 -u bench.py --config 5 --mode device --steps 3 --warmup 1 --no-cpu --no-variants > $O/bench5.json 2> $O/bench5.err
rc=$?; echo "bench cfg5 rc=$rc"; cut -c1-2500 $O/bench5.json; [ $rc -eq 0 ] || { tail -20 $O/bench5.err; exit $rc; }
exit 0
