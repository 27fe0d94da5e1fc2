#!/bin/bash
# P2 (count_front scatter sink) ablation at cfg5 on the experiment build:
# KC_P2_SKIP 16 = full P2 then stop, 1 = no flush stores, 2 = no staging, 4 = no sink
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/p2abl; mkdir -p $O
for v in 16 1 2 4 16; do
  KC_LIB=$PWD/kmer-counter_amd/variants/exp/libkc_hip.so KC_P2_SKIP=$v timeout -k 10 300 python3 -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu --no-variants --no-e2e > $O/s$v.json 2> $O/s$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "skip $v rc=$rc"; tail -5 $O/s$v.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('$O/s$v.json').read().splitlines()[-1])
b=d['device_resident']['breakdown_ms_per_step']; print('P2_SKIP=$v', round(d['ms_per_step'],2), b['partition_passes'])"
done
