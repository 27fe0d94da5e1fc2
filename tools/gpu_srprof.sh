#!/bin/bash
# sort_runs_k phase ticks (experiment build prints block 0's totals per launch)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/sr; mkdir -p $O
KC_LIB=$PWD/kmer-counter_amd/variants/exp/libkc_hip.so KC_DEBUG=1 timeout -k 10 300 python3 -u bench.py \
  --config 5 --mode device --steps 1 --warmup 0 --no-cpu --no-variants > $O/b.json 2> $O/b.err
rc=$?; echo "rc=$rc"; grep "sort_runs\|P5s" $O/b.err | head; exit $rc
