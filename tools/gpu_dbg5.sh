#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
KC_DEBUG=1 timeout -k 10 300 python3 bench.py --config 5 --steps 1 --warmup 0 --no-cpu ${EXTRA} > gpurun_out/dbg5.json 2> gpurun_out/dbg5.err
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/dbg5.err | tail; python3 -c "import json;d=json.load(open('gpurun_out/dbg5.json'));print(d['ms_per_step'], d['breakdown_ms_per_step'])"
exit $rc
