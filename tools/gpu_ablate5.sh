#!/bin/bash
# P5 timing ablation (KC_P5_SKIP=1: no LDS inserts; output invalid, timing only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
KC_P5_SKIP=1 timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/abl5.json 2> gpurun_out/abl5.err
rc=$?; echo "p5skip rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/abl5.json'));print(d['breakdown_ms_per_step'])")"
exit $rc
