#!/bin/bash
# Final check on one box: the full GPU suite, smoke(), the driver's exact bench
# command, a kernel trace of the cfg2 device step, and the cfg4 per-GPU shard
# (one skm batch). A heartbeat file keeps the long full-size tests visible.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
(while sleep 50; do date +%T >> $O/heartbeat; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread --durations=15 > $O/pytest.log 2>&1
rc=$?; tail -20 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench_driver.json; [ $rc -eq 0 ] || { tail -20 $O/bench_driver.err; exit $rc; }
[ -n "$NO_PROF" ] && exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof2 -o run --output-format csv -- python3 bench.py --config 2 --steps 3 --warmup 1 --no-cpu --no-e2e --no-variants > $O/prof2.json 2> $O/prof2.err
rc=$?; echo "rocprof cfg2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for f in $(find $O/prof2 -name '*kernel_stats.csv'); do cp "$f" $O/kernel_stats_cfg2.csv; done
timeout -k 10 900 python3 bench.py --config 4 --steps 3 --warmup 1 --no-variants > $O/cfg4.json 2> $O/cfg4.err
rc=$?; echo "cfg4 rc=$rc"; cut -c1-300 $O/cfg4.json; [ $rc -eq 0 ] || { tail -5 $O/cfg4.err; exit $rc; }
