#!/bin/bash
# same-box A/B of bench.py's pipelined steps (--pipeline 2: step j + 1 submitted before step j
# is finished, two batches on two streams) against one batch at a time (--pipeline 1), headline
# and crash variant. usage: bash tools/r06_pipe.sh <tag> [library]
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; mkdir -p $O
LIBARG=${2:+MADRAFT_HIP_LIB=$2}
for r in 1 2; do
  for p in 1 2; do
    for t in figure_8_unreliable_2c figure_8_unreliable_crash; do
      env $LIBARG timeout -k 10 300 python bench.py --test $t --steps ${STEPS:-20} --warmup 3 --pipeline $p \
        --no-cpu-baseline --variant '' --million 0 > $O/b_${t}_p$p.json 2> $O/b_${t}_p$p.err \
        || { echo "BENCH FAIL $t p$p"; tail -5 $O/b_${t}_p$p.err; exit 1; }
      python -c "import json; d=json.loads(open('$O/b_${t}_p$p.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$r $t pipeline $p', d['value'], 'ms/step', d['ms_per_step'], 'ms/launch %.2f' % r['avg_launch_ms'], 'frac', r['frac'], 'ev/seed', d['events_per_seed'])" | tee -a $O/summary.txt
    done
  done
done
