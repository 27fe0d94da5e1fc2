#!/bin/bash
# Process-to-process spread of the radix scatter (S at cfg2 size) and its
# dependence on where the output buffer sits relative to the input:
# rp_bench in separate processes, two allocations vs one with an offset.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/rplay; mkdir -p $O
for rep in ${REPS:-1 2 3}; do
for lay in ${LAYOUTS:--1 0 4096 65536 1052672}; do
  LD_LIBRARY_PATH=kmer-counter_amd timeout -k 10 120 ./tools/rp_bench 592344064 2 5 1 48 $lay > $O/l$lay.$rep.json 2> $O/l$lay.$rep.err
  rc=$?; echo "layout $lay rep $rep rc=$rc $(cat $O/l$lay.$rep.json)"; [ $rc -eq 0 ] || { tail -5 $O/l$lay.$rep.err; exit $rc; }
done
done
