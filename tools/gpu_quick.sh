#!/bin/bash
# Quick lease: a pytest selection (PYSEL), the cfg2 device line and a kernel
# trace of it (kernel stats csv), optionally cfg5 (CFG5=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${OUT:-q}; mkdir -p $O
if [ -n "$PYSEL" ]; then
  timeout -k 10 900 python3 -u -m pytest $PYSEL -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
  [ $rc -eq 0 ] || { grep -B2 -A30 "Error\|FAILED\|assert" $O/pytest.log | head -60; exit $rc; }
fi
timeout -k 10 600 python3 bench.py --steps 10 --warmup 3 --no-e2e --no-variants --no-cpu > $O/bench_cfg2.json 2> $O/bench_cfg2.err
rc=$?; echo "cfg2 rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench_cfg2.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps(d['device_resident']['breakdown_ms_per_step']))"
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-variants > $O/prof.json 2> $O/prof.err
rc=$?; echo "rocprof rc=$rc"
for f in $(find $O/prof -name '*kernel_stats.csv'); do cp "$f" $O/kernel_stats_cfg2.csv; done
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/kernel_stats_cfg2.csv')))[:14]: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e6,3))"
[ $rc -eq 0 ] || exit $rc
if [ -n "$CFG5" ]; then
  timeout -k 10 600 python3 bench.py --config 5 --steps 5 --warmup 2 --no-e2e --no-cpu --no-variants > $O/bench_cfg5.json 2> $O/bench_cfg5.err
  rc=$?; echo "cfg5 rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench_cfg5.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps(d['device_resident']['breakdown_ms_per_step']))"
fi
exit $rc
