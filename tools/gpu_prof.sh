#!/bin/bash
# Full-size bench + rocprofv3 kernel-trace stats of the same command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
READS=${READS:-50000000}
timeout -k 10 600 python3 bench.py --reads $READS --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_full.json; tail -5 gpurun_out/bench_full.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --reads $READS --steps 1 --warmup 1 --no-cpu > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
find gpurun_out/prof -name '*stats*' | head
for f in $(find gpurun_out/prof -name '*kernel_stats.csv'); do cut -d, -f1-8 "$f" | head -30; done
exit $rc
