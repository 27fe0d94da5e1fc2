#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) on a reduced cfg2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
READS=${READS:-10000000}
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc/g$i -o p -- python3 bench.py --reads $READS --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc/g$i.log 2>&1
  rc=$?; echo "group $i rc=$rc: $grp"
  [ $rc -eq 0 ] || exit $rc
done
