#!/bin/bash
# Iteration: GPU tests (filter TESTK), cfg2 bench, rocprofv3 kernel stats of the same bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/t
O=gpurun_out/t
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -k "${TESTK:-not full_size}" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit $rc; }
KC_DEBUG=1 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu ${BARGS:-} > $O/cfg2.json 2> $O/cfg2.err
rc=$?; echo "cfg2 rc=$rc"; python3 -c "import json;d=json.load(open('$O/cfg2.json'));print(round(d['value']/1e9,2),'G/s',round(d['ms_per_step'],2),'ms',d['engines_used'] if 'engines_used' in d else '')"
[ $rc -eq 0 ] || { tail -20 $O/cfg2.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu ${BARGS:-} > $O/prof.json 2> $O/prof.err
rc=$?; echo "rocprof rc=$rc"
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/t/prof/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(f"{float(r['AverageNs'])/1e6:9.3f} ms x{r['Calls']:>4}  {r['Name'][:70]}")
PY
exit $rc
