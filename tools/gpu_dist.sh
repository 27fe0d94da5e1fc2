#!/bin/bash
# Rehearsal of the multi-rank bench path on one GPU (2 ranks, gloo for the
# host-side barrier/max; each rank its own device context on GPU 0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
KC_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --reads 4000000 --mem 17179869184 > gpurun_out/bench_dist2.json 2> gpurun_out/bench_dist2.err
rc=$?; echo "dist rc=$rc"; cat gpurun_out/bench_dist2.json; tail -3 gpurun_out/bench_dist2.err
exit $rc
