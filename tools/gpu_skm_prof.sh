#!/bin/bash
# skm engine: parity tests, cfg2 bench, PMC passes (wave-cycle split and
# instruction mix) at 10M reads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_skm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_skm.log 2>&1
rc=$?; echo "pytest skm rc=$rc"; tail -2 gpurun_out/pytest_skm.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" gpurun_out/pytest_skm.log | head -60; exit $rc; }
KC_DEBUG=1 timeout -k 10 300 python3 bench.py --engine skm --steps 3 --warmup 1 --no-cpu > gpurun_out/cfg2_skm.json 2> gpurun_out/cfg2_skm.err
rc=$?; echo "cfg2 skm rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/cfg2_skm.json'));print(round(d['value']/1e9,2),'G/s',round(d['ms_per_step'],1),'ms',{k:(round(v,1) if isinstance(v,float) else v) for k,v in d['breakdown_ms_per_step'].items()})"
[ $rc -eq 0 ] || { tail -20 gpurun_out/cfg2_skm.err; exit $rc; }
grep "kc: skm" gpurun_out/cfg2_skm.err | tail -1
[ -n "$NOPMC" ] && exit 0
OUT=gpurun_out/pmc_skm READS=10000000 ARGS="--engine skm" bash tools/gpu_pmc.sh 2>&1 | grep -v "^wrote" | head -60
