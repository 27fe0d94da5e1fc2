#!/bin/bash
# Kernel trace of one cfg5 step (partition engine).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python3 bench.py --config 5 --steps 1 --warmup 0 --no-cpu > gpurun_out/prof5.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof5.log
for f in $(find gpurun_out/prof5 -name '*kernel_stats.csv'); do cut -d, -f1-8 "$f" | head -30; done
f=$(find gpurun_out/prof5 -name '*kernel_trace.csv' | head -1)
grep -n count_buckets "$f" | cut -c1-300 | head
exit $rc
