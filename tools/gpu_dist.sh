#!/bin/bash
# Rehearsal of the multi-rank bench path on one GPU: 2 ranks, gloo (RCCL
# refuses two ranks on one device), each rank its own device context on GPU 0;
# the end-to-end step with the key-space all-to-all (part files), then
# read-shard with the runs gathered and merged on rank 0's device, then cfg3 as
# stated (read-shard, run files, host k-way merge on rank 0). Every line
# carries rank 0's CPU baseline (timed after the timed region at every N).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/dist
for x in ${XCH:-alltoall none files}; do
  KC_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --reads 4000000 --mem 17179869184 --exchange $x --cpu-reads 300000 --no-variants > gpurun_out/dist/bench_dist2_$x.json 2> gpurun_out/dist/bench_dist2_$x.err
  rc=$?; echo "dist $x rc=$rc"; cut -c1-1200 gpurun_out/dist/bench_dist2_$x.json; tail -3 gpurun_out/dist/bench_dist2_$x.err
  [ $rc -eq 0 ] || exit $rc
done
