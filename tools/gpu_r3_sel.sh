#!/bin/bash
# Selected GPU tests (pytest -k expression in $SEL_K, files in $SEL_F), then
# optionally the cfg5 device-resident line ($CFG5=1) with debug output.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest ${SEL_F:-tests} -x -v -m gpu -k "${SEL_K}" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -40; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B2 -A40 "Error\|FAILED\|assert" $O/pytest.log | head -120; exit $rc; }
if [ -n "$CFG5" ]; then
KC_DEBUG=1 KC_TRACE=1 timeout -k 10 600 python3 -u bench.py --config 5 --mode device --steps 3 --warmup 1 --no-cpu --no-variants > $O/bench5.json 2> $O/bench5.err
rc=$?; echo "bench cfg5 rc=$rc"; cut -c1-3000 $O/bench5.json; [ $rc -eq 0 ] || { tail -30 $O/bench5.err; exit $rc; }
fi
exit 0
