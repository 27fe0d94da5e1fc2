#!/bin/bash
# Same-box A/B of library builds (KC_LIB) on the device-resident bench:
# LIBS entries are variant names (main = the in-tree library); CFG = 2 or 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${OUT:-abl}; mkdir -p $O
for rep in 1 2; do
for v in ${LIBS:-main rpdyn}; do
  lib=""; [ $v = main ] || lib=$PWD/kmer-counter_amd/variants/$v/libkc_hip.so
  for c in ${CFG:-2 5}; do
    KC_LIB=$lib timeout -k 10 300 python3 -u bench.py --config $c --steps ${STEPS:-5} --warmup 2 --no-cpu --no-variants --no-e2e > $O/$v.$c.$rep.json 2> $O/$v.$c.$rep.err
    rc=$?; [ $rc -eq 0 ] || { echo "$v cfg$c rc=$rc"; tail -5 $O/$v.$c.$rep.err; exit $rc; }
    python3 -c "
import json; d=json.loads(open('$O/$v.$c.$rep.json').read().splitlines()[-1])
b=d['device_resident']['breakdown_ms_per_step']; print('$v cfg$c', round(d['ms_per_step'],2), 'fq', round(b['fastq_index'],2), b['partition_passes'], 'p3b', b['p3b_presplit (in partition_passes[2])'], 'fin', round(b['finish'],2))"
  done
done
done
