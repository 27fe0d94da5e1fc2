#!/bin/bash
# Round evidence, in two calls:
#   part cfg2: PMC traffic passes, the default (end-to-end) bench line with CPU
#              baselines and host variants, rocprof kernel stats (gpu_round.sh)
#   part cfg5: the cfg5 device-resident line, its rocprof kernel stats, its PMC
#              passes (gpu_pmc5.sh), then the 2-rank gloo rehearsal (gpu_dist.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
case "${1:-cfg2}" in
cfg2)
  bash tools/gpu_round.sh ;;
cfg5)
  O=gpurun_out/round; mkdir -p $O
  timeout -k 10 600 python3 bench.py --config 5 --mode device --steps 3 --warmup 1 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
  rc=$?; echo "cfg5 rc=$rc"; cut -c1-400 $O/bench_cfg5.json; [ $rc -eq 0 ] || { tail -5 $O/bench_cfg5.err; exit $rc; }
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof5 -o run --output-format csv -- python3 bench.py --config 5 \
    --mode device --steps 2 --warmup 1 --no-cpu --no-variants > $O/prof5.json 2> $O/prof5.err
  rc=$?; echo "rocprof cfg5 rc=$rc"
  for f in $(find $O/prof5 -name '*kernel_stats.csv'); do cp "$f" $O/kernel_stats_cfg5.csv; done
  [ $rc -eq 0 ] || exit $rc
  bash tools/gpu_pmc5.sh || exit $?
  bash tools/gpu_dist.sh ;;
esac
