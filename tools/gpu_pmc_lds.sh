set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for v in base noswz; do
  O=gpurun_out/pmclds_$v; mkdir -p $O
  if [ $v = noswz ]; then export KC_LIB=kmer-counter_amd/ab/noswz/libkc_hip.so; else unset KC_LIB; fi
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $O/g1 -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-variants > $O/g1.log 2>&1
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/g1.log; exit $rc; }
  python3 tools/pmc_summary.py $O 50000000 31 r05_pmc_lds_$v.json > $O/summary.txt 2>&1
  grep -A3 "count_skm_k<1>\|count_rec_k\|count_skm_kILi1" $O/summary.txt | head -12
done
