#!/bin/bash
# Round evidence on one box: the driver's exact bench command under
# rocprofv3 --kernel-trace --stats (the line's HIP-event kernel times and the
# trace come from the same process), PMC passes at cfg2 (one counter group
# per rocprofv3 run, --kernel-trace only), cfg5 in two fresh processes with
# the CPU baseline, and the cfg3 per-GPU shard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/ev; mkdir -p $O
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/drv -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
rc=$?; echo "driver cmd under rocprof rc=$rc"; cut -c1-300 $O/bench_driver.json; [ $rc -eq 0 ] || { tail -20 $O/bench_driver.err; exit $rc; }
for f in $(find $O/drv -name '*kernel_stats.csv'); do cp "$f" $O/kernel_stats_driver_cmd.csv; done
OUT=gpurun_out/pmc bash tools/gpu_pmc.sh > $O/pmc_cfg2.txt 2>&1 || { tail -20 $O/pmc_cfg2.txt; exit 1; }
tail -3 $O/pmc_cfg2.txt
for rep in 1 2; do
  timeout -k 10 600 python3 bench.py --config 5 --steps 5 --warmup 2 --no-e2e > $O/bench_cfg5.$rep.json 2> $O/bench_cfg5.$rep.err
  rc=$?; echo "cfg5 $rep rc=$rc"; cut -c1-200 $O/bench_cfg5.$rep.json; [ $rc -eq 0 ] || { tail -5 $O/bench_cfg5.$rep.err; exit $rc; }
done
timeout -k 10 600 python3 bench.py --config 3 --steps 5 --warmup 2 --no-variants > $O/bench_cfg3.json 2> $O/bench_cfg3.err
rc=$?; echo "cfg3 rc=$rc"; cut -c1-200 $O/bench_cfg3.json
exit $rc
