#!/bin/bash
# F3 with per-read lengths: parity (varlen + skm + fused index), then the cfg2
# and cfg2v bench lines (no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/f3v
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_varlen.py tests/test_gpu_skm.py tests/test_gpu_fq_encode.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest.log | head -60; exit $rc; }
for a in "" "--min-read-length 50"; do
  timeout -k 10 300 python3 bench.py --no-cpu $a > $O/b.json 2> $O/b.err
  rc=$?; [ $rc -eq 0 ] || { tail -20 $O/b.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('$a', round(d['value']/1e9,2),'G/s',round(d['ms_per_step'],2),'ms',{k:v['avg_launch_ms'] for k,v in d['roofline']['kernels'].items()}, d['breakdown_ms_per_step']['fastq_index'])"
done
