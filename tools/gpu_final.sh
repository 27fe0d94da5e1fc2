#!/bin/bash
# End-of-round evidence: the driver's GPU test command, smoke(), the round
# profiles (PMC traffic passes, bench line with CPU baseline, rocprof stats),
# then the cfg2v (variable-length) bench line with its CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/final/pytest_gpu.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" gpurun_out/final/pytest_gpu.log | head -60; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/final/smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_round.sh || exit $?
timeout -k 10 600 python3 bench.py --min-read-length 50 > gpurun_out/final/bench_varlen.json 2> gpurun_out/final/bench_varlen.err
rc=$?; echo "varlen bench rc=$rc"; cut -c1-400 gpurun_out/final/bench_varlen.json
exit $rc
