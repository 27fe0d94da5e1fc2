#!/bin/bash
# The driver's exact bench command on the committed tree, then a kernel
# trace of the cfg5 device step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/drv; mkdir -p $O
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench_driver.json; [ $rc -eq 0 ] || { tail -20 $O/bench_driver.err; exit $rc; }
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof5 -o run --output-format csv -- python3 bench.py --config 5 --steps 3 --warmup 1 --no-cpu --no-e2e --no-variants > $O/prof5.json 2> $O/prof5.err
rc=$?; echo "rocprof cfg5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for f in $(find $O/prof5 -name '*kernel_stats.csv'); do cp "$f" $O/kernel_stats_cfg5.csv; done
