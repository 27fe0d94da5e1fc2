#!/bin/bash
# Round 6: the multi-rank tests (2, 3 and 8 ranks over gloo on the one GPU,
# the full-size cfg3 shards with the shared host merge), cfg5 at the bench's
# 48 GiB, then the 2-rank cfg3 bench rehearsal at full shard size with the
# merge shared by the ranks and with rank 0's merge.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6d; mkdir -p $O
(while sleep 50; do date +%T >> $O/heartbeat; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python3 -u -m pytest ${TESTS:-tests/test_dist_gpu.py "tests/test_gpu_parity.py::test_config5_full_size_properties[bench_48GiB]"} -x -v -rP -m gpu --timeout 300 --timeout-method thread --durations=20 > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|cfg3 full" $O/pytest.log | cut -c1-600 | tail -30; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAILED" $O/pytest.log | head -80; exit $rc; }
[ -n "$NO_BENCH" ] && exit 0
for fm in ${FM:-ranks rank0}; do
  KC_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --config 3 --gpus 2 --steps 3 --warmup 1 --mem $((90<<30)) --files-merge $fm --cpu-reads 300000 --no-variants > $O/bench_cfg3_dist2_$fm.json 2> $O/bench_cfg3_dist2_$fm.err
  rc=$?; echo "cfg3 2-rank $fm rc=$rc"; cut -c1-400 $O/bench_cfg3_dist2_$fm.json; python3 -c "
import json; d=json.loads(open('$O/bench_cfg3_dist2_$fm.json').read().strip().splitlines()[-1]); print(d['device_resident']['breakdown_ms_per_step'])"; tail -3 $O/bench_cfg3_dist2_$fm.err
  [ $rc -eq 0 ] || exit $rc
done
