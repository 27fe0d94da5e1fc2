#!/bin/bash
# Kernel trace (timestamps) of the cfg2 device-resident step: the last step's
# kernels and the gaps between them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/trace; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- python3 bench.py --config ${CFG:-2} --steps 3 --warmup 1 --no-cpu --no-e2e --no-variants > $O/bench.json 2> $O/bench.err
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench.err; exit $rc; }
for f in $(find $O/p -name '*kernel_trace.csv'); do cp "$f" $O/kernel_trace.csv; done
for f in $(find $O/p -name '*kernel_stats.csv'); do cp "$f" $O/kernel_stats.csv; done
ls -la $O
