#!/bin/bash
# cfg5 device-resident comparison on one box: key-range passes (default, and
# at least 4 / 8 passes) vs read batches + merge (KC_NO_KEY_PASSES).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
for v in ${AB_SET:-passes passes4 passes8 batches}; do
  unset KC_NO_KEY_PASSES KC_KEY_PASSES_MIN
  case $v in batches) export KC_NO_KEY_PASSES=1;; passes4) export KC_KEY_PASSES_MIN=4;; passes8) export KC_KEY_PASSES_MIN=8;; esac
  timeout -k 10 300 python3 -u bench.py --config 5 --mode device --steps 3 --warmup 1 --no-cpu --no-variants > $O/$v.json 2> $O/$v.err
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/$v.err; exit $rc; }
  python3 -c "
import json,sys; d=json.loads(open('$O/$v.json').read().splitlines()[-1])
b=d['device_resident']['breakdown_ms_per_step']; print('$v', round(d['ms_per_step'],2), b['partition_passes'], 'p3b', b['p3b_presplit (in partition_passes[2])'], 'fin', round(b['finish'],2), 'idx', round(b['fastq_index'],2))"
done
