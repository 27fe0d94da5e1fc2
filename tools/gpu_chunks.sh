#!/bin/bash
# Chunk-path GPU tests, then the default bench (host variants: reference chunks)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/ch; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_ingest.py -k "chunk or checkpoint or rollback or batch or file" > $O/sel.log 2>&1
rc=$?; tail -3 $O/sel.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py --no-cpu > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && tail -5 $O/bench.err && exit $rc
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['end_to_end']['phases_ms_rank0'])
print(d['host_variants']['reference_chunks']); print(d['host_variants']['host_memory']['value'])"
