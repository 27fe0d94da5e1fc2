#!/bin/bash
# P2 timing ablations (results invalid under KC_P2_SKIP; timing only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for sk in 1 2 4; do
KC_P2_SKIP=$sk timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/abl$sk.json 2> gpurun_out/abl$sk.err
rc=$?; echo "skip=$sk rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/abl$sk.json'));print(d['breakdown_ms_per_step']['partition_passes'])")"
[ $rc -eq 0 ] || exit $rc
done
