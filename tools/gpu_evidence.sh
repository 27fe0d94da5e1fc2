#!/bin/bash
# Round evidence on one box: PMC passes at cfg2 and cfg5 (one counter group
# per rocprofv3 run, --kernel-trace only), the driver's exact bench command,
# and a kernel trace (rocprofv3 --kernel-trace --stats) of the cfg2 and cfg5
# device steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/ev; mkdir -p $O
OUT=gpurun_out/pmc bash tools/gpu_pmc.sh > $O/pmc_cfg2.txt 2>&1 || { tail -20 $O/pmc_cfg2.txt; exit 1; }
tail -3 $O/pmc_cfg2.txt
bash tools/gpu_pmc5.sh > $O/pmc_cfg5.txt 2>&1 || { tail -20 $O/pmc_cfg5.txt; exit 1; }
tail -3 $O/pmc_cfg5.txt
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench_driver.json; [ $rc -eq 0 ] || { tail -20 $O/bench_driver.err; exit $rc; }
export TMPDIR=/tmp
for c in 2 5; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof$c -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-e2e --no-variants > $O/prof$c.json 2> $O/prof$c.err
  rc=$?; echo "rocprof cfg$c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  for f in $(find $O/prof$c -name '*kernel_stats.csv'); do cp "$f" $O/kernel_stats_cfg$c.csv; done
done
timeout -k 10 600 python3 bench.py --config 5 --steps 5 --warmup 2 --no-e2e > $O/bench_cfg5.json 2> $O/bench_cfg5.err
rc=$?; echo "cfg5 rc=$rc"; cut -c1-300 $O/bench_cfg5.json
exit $rc
