#!/bin/bash
# skm tests + cfg2 bench for both engines (and optional PMC of skm).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_skm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_skm.log 2>&1
rc=$?; echo "pytest skm rc=$rc"; tail -2 gpurun_out/pytest_skm.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" gpurun_out/pytest_skm.log | head -60; exit $rc; }
for eng in ${ENGINES:-skm partition}; do
KC_DEBUG=1 timeout -k 10 300 python3 bench.py --engine $eng --steps 3 --warmup 1 --no-cpu > gpurun_out/cfg2_$eng.json 2> gpurun_out/cfg2_$eng.err
rc=$?; echo "cfg2 $eng rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/cfg2_$eng.json'));print(round(d['value']/1e9,2),'G/s',round(d['ms_per_step'],1),'ms',{k:(round(v,1) if isinstance(v,float) else v) for k,v in d['breakdown_ms_per_step'].items()})"
[ $rc -eq 0 ] || { tail -20 gpurun_out/cfg2_$eng.err; exit $rc; }
done
grep "kc: skm" gpurun_out/cfg2_skm.err | tail -1
[ -z "$PMC" ] && exit 0
OUT=gpurun_out/pmc_skm READS=10000000 ARGS="--engine skm" bash tools/gpu_pmc.sh 2>&1 | grep -A3 "count_skm\|skm_front\|rp_scatter"
