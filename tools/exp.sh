#!/bin/bash
# dev: headline bench per variant library (madraft_amd/lib/var/<name>.so), two alternating
# rounds, then section profiles of the MR_PROF variants named in $PROFS
# usage: bash tools/exp.sh <outdir> <name1> <name2> ...   (extra bench args in $BARGS)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; shift; mkdir -p $O
V=$PWD/madraft_amd/lib/var
for r in 1 2; do
  for f in "$@"; do
    MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --variant '' $BARGS > $O/bench_$f.json 2> $O/bench_$f.err || { echo "FAIL $f"; tail -5 $O/bench_$f.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], 'ms/launch %.2f' % d['roofline']['avg_launch_ms'], 'Gev/s %.3f' % (d['events_per_sec']/1e9), 'ev/seed', d['events_per_seed'])" | tee -a $O/summary.txt
  done
done
for p in $PROFS; do
  MADRAFT_HIP_LIB=$V/$p.so timeout -k 10 300 python tools/prof.py > $O/prof_$p.txt 2>&1 || { echo "PROF FAIL $p"; tail $O/prof_$p.txt; exit 1; }
  cat $O/prof_$p.txt
done
