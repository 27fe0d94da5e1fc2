#!/bin/bash
# Sub-range P5 tests, GPU suite, cfg5 (partition engine, then the table engine
# with a small gpuMemoryLimit = forced spill), cfg2 regression check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -m pytest tests -m gpu -x -q -k "subrange" > gpurun_out/pytest_sub.log 2>&1
rc=$?; echo "pytest sub rc=$rc"; tail -30 gpurun_out/pytest_sub.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q -k "not full_size" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --config 5 --steps 1 --warmup 1 --no-cpu > gpurun_out/cfg5_part.json 2> gpurun_out/cfg5_part.err
rc=$?; echo "cfg5 partition rc=$rc"; cat gpurun_out/cfg5_part.json; tail -5 gpurun_out/cfg5_part.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/cfg2.json 2> gpurun_out/cfg2.err
rc=$?; echo "cfg2 rc=$rc"; cat gpurun_out/cfg2.json; tail -5 gpurun_out/cfg2.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --config 5 --engine table --mem 17179869184 --steps 1 --warmup 0 --no-cpu > gpurun_out/cfg5_table.json 2> gpurun_out/cfg5_table.err
rc=$?; echo "cfg5 table rc=$rc"; cat gpurun_out/cfg5_table.json; tail -5 gpurun_out/cfg5_table.err
exit $rc
