#!/bin/bash
# PMC passes over the cfg5 device-resident bench (one rocprofv3 run per counter
# group, --kernel-trace only): HBM read, HBM write, SQ wave-cycle split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/pmc5; mkdir -p $O
i=0
for grp in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE" \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/g$i -o p -- python3 bench.py \
    --config 5 --steps 1 --warmup 0 --no-cpu --no-variants --no-e2e > $O/g$i.log 2>&1
  rc=$?; echo "pmc group $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $O 20000000 55 pmc_cfg5.json > $O/summary.txt 2>&1; rc=$?
head -60 $O/summary.txt
exit $rc
