#!/bin/bash
# GPU tests (optional) then the default bench line (end-to-end cfg2) on the box.
# usage: tools/gpu_bench_e2e.sh [tests|tests:<pytest selection>|notests] [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/b
if [ "${1%%:*}" = "tests" ]; then
  SEL=tests; [ "$1" != "tests" ] && SEL="${1#tests:}"
  timeout -k 10 900 python3 -u -m pytest $SEL -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/b/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/b/pytest.log
  [ $rc -eq 0 ] || { grep -B2 -A30 "Error\|FAILED" gpurun_out/b/pytest.log | head -60; exit $rc; }
fi
shift
timeout -k 10 900 python3 -u bench.py "$@" > gpurun_out/b/bench.json 2> gpurun_out/b/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-3000 gpurun_out/b/bench.json
[ $rc -eq 0 ] || tail -30 gpurun_out/b/bench.err
exit $rc
