#!/bin/bash
# Round-4 lease: GPU test suite, cfg2 device line + kernel trace, cfg5 line
# with its CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4b; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest ${PYSEL:-tests} -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -B2 -A30 "Error\|FAILED\|assert" $O/pytest.log | head -60; exit $rc; }
timeout -k 10 600 python3 bench.py --steps 10 --warmup 3 --no-e2e --no-variants --no-cpu > $O/bench_cfg2.json 2> $O/bench_cfg2.err
rc=$?; echo "cfg2 rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench_cfg2.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps(d['device_resident']['breakdown_ms_per_step']))"
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-variants > $O/prof.json 2> $O/prof.err
rc=$?; echo "rocprof rc=$rc"
for f in $(find $O/prof -name '*kernel_stats.csv'); do cp "$f" $O/kernel_stats_cfg2.csv; cut -d, -f1-4 "$f" | head -30; done
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --config 5 --steps 5 --warmup 2 --no-e2e > $O/bench_cfg5.json 2> $O/bench_cfg5.err
rc=$?; echo "cfg5 rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench_cfg5.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps(d['device_resident']['breakdown_ms_per_step']), json.dumps(d['cpu_baseline'])[:200])"
exit $rc
