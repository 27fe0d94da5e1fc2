#!/bin/bash
# cfg3 rehearsal at full shard size on one GPU: N ranks over gloo (RCCL
# refuses two ranks on one device), each a full 50M-read cfg3 shard in HBM
# with a working set that lets N contexts share the GPU; the run files and the
# host merge shared by the ranks, then rank 0's merge of the same files.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/cfg3r; mkdir -p $O
N=${N:-4}; MEM=${MEM:-$((40<<30))}
for fm in ${FM:-ranks rank0}; do
  KC_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29541 bench.py --config 3 --gpus $N --steps ${STEPS:-3} --warmup 1 --mem $MEM --files-merge $fm --cpu-reads 300000 --no-variants > $O/bench_cfg3_dist${N}_$fm.json 2> $O/bench_cfg3_dist${N}_$fm.err
  rc=$?; echo "cfg3 $N-rank $fm rc=$rc"; python3 -c "
import json; d=json.loads(open('$O/bench_cfg3_dist${N}_$fm.json').read().strip().splitlines()[-1]); print(round(d['value']/1e9,2), 'e9', round(d['ms_per_step'],1), 'ms', d['device_resident']['breakdown_ms_per_step'])"; tail -3 $O/bench_cfg3_dist${N}_$fm.err
  [ $rc -eq 0 ] || exit $rc
done
