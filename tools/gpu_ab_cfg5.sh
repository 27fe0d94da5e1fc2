#!/bin/bash
# cfg5 device-resident A/B on one box: AB_SET names env settings (name=VAR,VAR2 or name=)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${OUT:-ab5}; mkdir -p $O
for spec in ${AB_SET:-base= nodigs=KC_P2_NO_DIGS nodual=KC_NO_DUAL_PASS}; do
  name=${spec%%=*}; vars=${spec#*=}
  ( for v in ${vars//,/ }; do export $v=1; done
    timeout -k 10 300 python3 -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu --no-variants --no-e2e > $O/$name.json 2> $O/$name.err )
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/$name.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('$O/$name.json').read().splitlines()[-1])
b=d['device_resident']['breakdown_ms_per_step']; print('$name', round(d['ms_per_step'],2), b['partition_passes'], 'p3b', b['p3b_presplit (in partition_passes[2])'], 'idx', round(b['fastq_index'],2))"
done
