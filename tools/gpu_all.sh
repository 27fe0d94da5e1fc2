#!/bin/bash
# Full GPU parity suite (no full-size), then cfg2 and cfg5 benches for the given engines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -k "not full_size" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/pytest_gpu.log | head -80; exit $rc; }
for eng in ${ENGINES:-skm}; do
for cfg in ${CFGS:-2 5}; do
KC_DEBUG=1 timeout -k 10 300 python3 bench.py --engine $eng --config $cfg --steps 2 --warmup 1 --no-cpu > gpurun_out/cfg${cfg}_$eng.json 2> gpurun_out/cfg${cfg}_$eng.err
rc=$?; echo "cfg$cfg $eng rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/cfg${cfg}_$eng.json'));print(round(d['value']/1e9,2),'G/s',round(d['ms_per_step'],1),'ms',{k:(round(v,1) if isinstance(v,float) else v) for k,v in d['breakdown_ms_per_step'].items()})"
[ $rc -eq 0 ] || { tail -20 gpurun_out/cfg${cfg}_$eng.err; exit $rc; }
grep "kc: skm\|kc: P5" gpurun_out/cfg${cfg}_$eng.err | tail -1
done
done
