#!/bin/bash
# GPU suite (no full-size), cfg2 bench, cfg5 bench (1 step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q -k "not full_size" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log | grep -v "^\s*$" | tail -8
[ $rc -eq 0 ] || exit $rc
KC_DEBUG=1 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/cfg2.json 2> gpurun_out/cfg2.err
rc=$?; echo "cfg2 rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/cfg2.json'));print(round(d['value']/1e9,2),'G/s',round(d['ms_per_step'],1),'ms',{k:(round(v,1) if isinstance(v,float) else v) for k,v in d['breakdown_ms_per_step'].items()})"
[ $rc -eq 0 ] || exit $rc
if [ -z "$NO5" ]; then
KC_DEBUG=1 timeout -k 10 300 python3 bench.py --config 5 --steps 1 --warmup 1 --no-cpu > gpurun_out/cfg5.json 2> gpurun_out/cfg5.err
rc=$?; echo "cfg5 rc=$rc"; grep "kc: P5" gpurun_out/cfg5.err | tail -2; python3 -c "import json;d=json.load(open('gpurun_out/cfg5.json'));print(round(d['value']/1e9,2),'G/s',round(d['ms_per_step'],1),'ms',{k:(round(v,1) if isinstance(v,float) else v) for k,v in d['breakdown_ms_per_step'].items()})"
fi
exit $rc
