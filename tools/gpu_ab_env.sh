#!/bin/bash
# Same-box A/B of environment settings on the device-resident bench:
# AB_SET entries name=VAR[,VAR2] (name= : defaults); CFG = 2 or 5; REPS rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${OUT:-abe}; mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
for spec in ${AB_SET}; do
  name=${spec%%=*}; vars=${spec#*=}
  ( for v in ${vars//,/ }; do export $v=1; done
    timeout -k 10 300 python3 -u bench.py --config ${CFG:-2} --steps ${STEPS:-10} --warmup 2 --no-cpu --no-variants --no-e2e > $O/$name.$rep.json 2> $O/$name.$rep.err )
  rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 $O/$name.$rep.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('$O/$name.$rep.json').read().splitlines()[-1])
b=d['device_resident']['breakdown_ms_per_step']; print('$name', round(d['ms_per_step'],2), b['partition_passes'], 'p5a', b['p5a_dedup'], 'fin', round(b['finish'],2))"
done
done
