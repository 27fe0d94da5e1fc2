#!/bin/bash
# Quick P2 write-traffic check: bench + WRITE_SIZE pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/p2w
timeout -k 10 300 python3 -m pytest tests -m gpu -x -q -k "not full_size" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/p2w/b.json 2> gpurun_out/p2w/b.err
rc=$?; python3 -c "import json;d=json.load(open('gpurun_out/p2w/b.json'));print(round(d['value']/1e9,2),'G/s',round(d['ms_per_step'],1),'ms',d['breakdown_ms_per_step'])"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/p2w/w -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/p2w/w.log 2>&1
rc=$?; echo "pmc rc=$rc"
python3 - <<'PY'
import csv,glob,collections
t=collections.defaultdict(float)
for f in glob.glob('gpurun_out/p2w/w/**/*counter_collection.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        t[r['Kernel_Name'][:50]]+=float(r['Counter_Value'])*1024/1e9
for k,v in sorted(t.items(),key=lambda x:-x[1])[:6]: print(f"{k:50s} {v:8.2f} GB")
PY
exit $rc
