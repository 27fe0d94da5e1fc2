#!/bin/bash
# rp_scatter_k variants through tools/rp_bench (random records, HIP events);
# RP_SET entries: <variant>[:emit 0|1]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/rpab; mkdir -p $O
for spec in ${RP_SET:-main main:0 rp1 rp1:0 rpnt rpnt:0}; do
  v=${spec%%:*}; e=1; [ "$spec" = "$v" ] || e=${spec#*:}; sh=${e#*/}; e=${e%%/*}; [ "$sh" = "$e" ] && sh=48
  d=kmer-counter_amd; [ $v = main ] || d=kmer-counter_amd/variants/$v
  LD_LIBRARY_PATH=$d timeout -k 10 120 ./tools/rp_bench ${RP_N:-592344064} ${RP_NW:-2} 5 $e $sh > $O/$v.$e.json 2> $O/$v.$e.err
  rc=$?; echo "$spec rc=$rc $(cat $O/$v.$e.json)"; [ $rc -eq 0 ] || { tail -5 $O/$v.$e.err; exit $rc; }
done
