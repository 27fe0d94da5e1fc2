#!/bin/bash
# F timing ablations (results invalid under KC_F_SKIP; timing only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for sk in 0 1 3 7 15 2 8; do
KC_F_SKIP=$sk timeout -k 10 120 python3 bench.py --engine skm --steps 2 --warmup 1 --no-cpu > gpurun_out/fskip$sk.json 2> gpurun_out/fskip$sk.err
rc=$?; echo "skip=$sk rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/fskip$sk.json'));print(d['breakdown_ms_per_step']['partition_passes'])" 2>&1 | tail -1)"
done
exit 0
