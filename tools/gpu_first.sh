#!/bin/bash
# First GPU pass: smoke, parity tests (not the full-size one), a short bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q -k "not full_size" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --reads 5000000 --steps 2 --warmup 1 --cpu-reads 200000 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_small.json; tail -5 gpurun_out/bench_small.err
exit $rc
