#!/bin/bash
# Round-4 first lease: the driver's exact bench command (no environment
# overrides), the output-write probe, then the GPU test suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4a; mkdir -p $O
df -h /tmp /dev/shm . > $O/df.txt 2>&1; echo "TMPDIR=${TMPDIR:-unset}" >> $O/df.txt; cat $O/df.txt
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench_driver.json
[ $rc -eq 0 ] || { tail -30 $O/bench_driver.err; exit $rc; }
g++ -O2 -std=c++17 -pthread -o $O/write_probe tools/write_probe.cpp 2>/dev/null
for d in /tmp /dev/shm; do timeout -k 10 200 $O/write_probe $d 3.4 16 > $O/write_probe_$(basename $d).txt 2>&1; echo "probe $d rc=$?"; done
cat $O/write_probe_*.txt
timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || grep -B2 -A40 "Error\|FAILED\|assert" $O/pytest.log | head -80
exit $rc
