#!/bin/bash
# S's scatter alone (tools/rp_bench, cfg2 size) in several processes: six
# (input, output) region pairs x digit-region pads, to see whether gaps
# between the 256 output digit regions change the per-process slow mode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/rppad; mkdir -p $O
for p in 1 2 3 4; do
  RP_NREG=${NREG:-3} RP_NOCHECK=1 RP_PADS=${PADS:-0,97,4099,65537} timeout -k 10 200 ./tools/rp_bench 592344064 2 3 1 48 -3 > $O/proc$p.txt 2>&1
  rc=$?; echo "process $p rc=$rc"; [ $rc -eq 0 ] || { cat $O/proc$p.txt | tail -5; exit $rc; }
  python3 -c "
import json
rows=[json.loads(l) for l in open('$O/proc$p.txt') if l.startswith('{')]
for pad in sorted(set(r['pad'] for r in rows)):
    print(' pad', pad, ' '.join(f\"{r['pair']}:{r['avg_ms']}\" for r in rows if r['pad']==pad))"
done
