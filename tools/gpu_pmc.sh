#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only, never
# combined with sys/runtime traces) on the bench workload; summarised by
# tools/pmc_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
READS=${READS:-50000000}
ARGS=${ARGS:-}
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/g$i -o p -- python3 bench.py --reads $READS --steps 1 --warmup 0 --no-cpu --no-e2e --no-variants $ARGS > $OUT/g$i.log 2>&1
  rc=$?; echo "group $i rc=$rc: $grp"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $OUT $READS ${K:-31}
