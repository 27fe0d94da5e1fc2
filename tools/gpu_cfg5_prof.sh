#!/bin/bash
# cfg5 device step under rocprofv3 --kernel-trace --stats, one-pass index vs
# the two-kernel index (KC_NO_FQ_SPEC=1), one process each, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/c5p; mkdir -p $O
for v in spec nospec; do
  if [ $v = nospec ]; then export KC_TEST_HOOKS=1 KC_NO_FQ_SPEC=1; else unset KC_NO_FQ_SPEC; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 bench.py --config 5 --steps 3 --warmup 1 --no-cpu --no-e2e --no-variants > $O/$v.json 2> $O/$v.err
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$v.err; exit $rc; }
  for f in $(find $O/$v -name '*kernel_stats.csv'); do cp "$f" $O/stats_$v.csv; done
done
