#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "keyspace_split and skm" --timeout 120 --timeout-method thread > gpurun_out/ks1.log 2>&1; echo "ks skm only rc=$?"; tail -3 gpurun_out/ks1.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "keyspace_split and partition" --timeout 120 --timeout-method thread > gpurun_out/ks2.log 2>&1; echo "ks part only rc=$?"; tail -3 gpurun_out/ks2.log
for eng in skm partition; do
KC_DEBUG=1 timeout -k 10 300 python3 bench.py --engine $eng --steps 3 --warmup 1 --no-cpu > gpurun_out/cfg2_$eng.json 2> gpurun_out/cfg2_$eng.err
rc=$?; echo "cfg2 $eng rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/cfg2_$eng.json'));print(round(d['value']/1e9,2),'G/s',round(d['ms_per_step'],1),'ms',{k:(round(v,1) if isinstance(v,float) else v) for k,v in d['breakdown_ms_per_step'].items()})"
[ $rc -eq 0 ] || { tail -20 gpurun_out/cfg2_$eng.err; exit $rc; }
done
grep "kc: skm" gpurun_out/cfg2_skm.err | tail -2
