#!/bin/bash
# Variable-length reads: GPU parity tests, then the cfg2v
# bench line (reads of 50..150 bp from the cfg2 genome, KC_FLAG_VARLEN) with
# its CPU baseline, then rocprofv3 kernel stats of the same command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/varlen
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_varlen.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest.log | head -60; exit $rc; }
timeout -k 10 600 python3 bench.py --min-read-length ${LMIN:-50} > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-900 $O/bench.json
[ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --min-read-length ${LMIN:-50} --steps 3 --warmup 1 --no-cpu > $O/prof.json 2> $O/prof.err
rc=$?; echo "rocprof rc=$rc"
for f in $(find $O/prof -name '*kernel_stats.csv'); do cp "$f" $O/kernel_stats.csv; cut -d, -f1-4 "$f" | head -16; done
exit $rc
