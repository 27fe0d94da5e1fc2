#!/bin/bash
# The radix scatter (S size) into a plain allocation, into virtual-memory
# mapped chunks in creation order, and into the same chunks shuffled
# (tools/rp_bench layout -4), several processes per chunk size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/rpvmm; mkdir -p $O
N=${N:-592344064}
for ch in ${CHUNKS:-64 2}; do
  for p in 1 2 3; do
    chk=1; [ $p -eq 1 ] && [ $ch = "${CHUNKS%% *}" ] && chk=
    ( [ -n "$chk" ] && export RP_NOCHECK=1
      RP_CHUNK_MB=$ch RP_SWEEPS=2 timeout -k 10 300 ./tools/rp_bench $N 2 3 1 48 -4 > $O/c$ch.p$p.txt 2> $O/c$ch.p$p.err )
    rc=$?; echo "chunk $ch MB process $p rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/c$ch.p$p.err; exit $rc; }
    python3 -c "
import json
rows=[json.loads(l) for l in open('$O/c$ch.p$p.txt') if l.startswith('{')]
print(' '.join(f\"{['plain','vmm','shuf'][r['pair'][1]]}:{r['avg_ms']}\" for r in rows))"
  done
done
