#!/bin/bash
# P5 timing ablation (results invalid under KC_P5_SKIP; timing only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for sk in ${SKIPS:-0 1 3 7}; do
KC_DEBUG=1 KC_P5_SKIP=$sk timeout -k 10 120 python3 bench.py --engine skm --steps 2 --warmup 1 --no-cpu > gpurun_out/p5skip$sk.json 2> gpurun_out/p5skip$sk.err
rc=$?; echo "skip=$sk rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/p5skip$sk.json'));print(d['breakdown_ms_per_step']['partition_passes'])" 2>&1 | tail -1)"
grep "kc: skm" gpurun_out/p5skip$sk.err | tail -1
done
exit 0
