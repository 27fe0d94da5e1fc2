#!/bin/bash
# SQ counter groups (wave-cycle split, instruction mix) for one kernel per
# variant (VARIANTS = space-separated env assignments, "-" = default; KNAME =
# kernel name substring), 10M reads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
i=0
for v in ${VARIANTS:--}; do
  i=$((i+1))
  OUT=gpurun_out/pmcv/v$i
  mkdir -p $OUT
  g=0
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
    g=$((g+1))
    ( [ "$v" != "-" ] && export ${v//,/ }
      timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/g$g -o p -- python3 bench.py --reads ${READS:-10000000} --steps 1 --warmup 0 --no-cpu --engine skm > $OUT/g$g.log 2>&1 )
    rc=$?
    [ $rc -eq 0 ] || { echo "variant $i group $g rc=$rc"; tail -5 $OUT/g$g.log; exit $rc; }
  done
  echo "== variant $i ($v)"
  python3 tools/pmc_summary.py $OUT ${READS:-10000000} 31 2>&1 | grep -A3 "${KNAME:-front}"
done
