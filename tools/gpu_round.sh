#!/bin/bash
# Round evidence for the default engine at cfg2: PMC traffic passes (FETCH_SIZE,
# WRITE_SIZE; each its own rocprofv3 run), then the default bench line (with
# cpu_baseline, traffic read from the PMC summary just written), then a
# rocprofv3 --kernel-trace --stats run of the same bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/round/pmc
O=gpurun_out/round
i=0
for grp in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/pmc/g$i -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/pmc/g$i.log 2>&1
  rc=$?; echo "pmc group $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $O/pmc 50000000 31 > $O/pmc_summary.txt 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json | cut -c1-600
[ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $O/prof.json 2> $O/prof.err
rc=$?; echo "rocprof rc=$rc"
for f in $(find $O/prof -name '*kernel_stats.csv'); do cp "$f" $O/kernel_stats.csv; cut -d, -f1-8 "$f" | head -25; done
exit $rc
