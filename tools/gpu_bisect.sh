#!/bin/bash
# Runs one GPU test selection under several environment settings; stops on a
# crash or time limit (exit >= 124), continues past ordinary test failures.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/bis; mkdir -p $O
sel="$1"; shift
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs KC_DEBUG=1 timeout -k 10 200 python3 -u -m pytest -x -q -s --timeout 120 -m gpu tests/test_gpu_parity.py \
    -k "$sel" > $O/r$i.log 2>&1
  rc=$?
  echo "[$envs] rc=$rc: $(grep -E 'passed|failed' $O/r$i.log | tail -1)"
  grep -E "kc: P5" $O/r$i.log | tail -3
  [ $rc -ge 124 ] && exit $rc
done
exit 0
