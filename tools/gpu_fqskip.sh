#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for sk in 0 1 2 3; do
KC_FQ_SKIP=$sk timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/fq$sk.json 2> gpurun_out/fq$sk.err
echo "skip=$sk rc=$? $(python3 -c "import json;d=json.load(open('gpurun_out/fq$sk.json'));print(d['breakdown_ms_per_step']['fastq_index'])" 2>&1 | tail -1)"
done
KC_NO_FUSED_ENCODE=1 timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/fqold.json 2> gpurun_out/fqold.err
echo "old rc=$? $(python3 -c "import json;d=json.load(open('gpurun_out/fqold.json'));print(d['breakdown_ms_per_step']['fastq_index'], d['breakdown_ms_per_step']['partition_passes'][0]-d['breakdown_ms_per_step']['partition_passes'][1])" 2>&1 | tail -1)"
exit 0
