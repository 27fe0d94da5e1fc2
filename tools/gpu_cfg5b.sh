#!/bin/bash
# cfg5 device-resident with KC_DEBUG + KC_TRACE (finish phases); engines given as args
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/c5b; mkdir -p $O
for eng in "$@"; do
  KC_DEBUG=1 KC_TRACE=1 timeout -k 10 300 python3 -u bench.py --config 5 --mode device --steps 1 --warmup 1 --no-cpu \
    --no-variants --engine $eng > $O/bench_$eng.json 2> $O/bench_$eng.err
  rc=$?; echo "cfg5 $eng rc=$rc"; [ $rc -ne 0 ] && tail -5 $O/bench_$eng.err && exit $rc
  python3 -c "
import json; d=json.loads(open('$O/bench_$eng.json').read()); r=d['device_resident']
print(d['value'], r['ms_per_step'], r['breakdown_ms_per_step'], d['spill_runs'])"
  grep -v "download piece\|reader block\|block " $O/bench_$eng.err | tail -22 | cut -c1-160
done
