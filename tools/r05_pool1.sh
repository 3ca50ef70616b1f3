#!/bin/bash
# round 5, first pool-kernel pass: parity of the pool kernel on the Raft scenarios, then a
# same-library A/B (MR_POOL=0: step_kernel, 1: pool_kernel) of the headline and configs 2 / 3'.
# usage: bash tools/r05_pool1.sh <tag>
cd "$GRAFT_REPO_ROOT"; T=${1:-r05p1}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "${PTEST:-test_scenario_bit_exact and (figure_8 or fail_agree or initial_election or snapshot_basic or persist2)}" \
  > $O/parity.log 2>&1 || { echo "PARITY FAIL"; grep -E "FAILED|Error|assert" $O/parity.log | head -20; tail -5 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for r in 1 2; do
  for p in 0 1; do
    MR_POOL=$p timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --variant '' --million 0 \
      > $O/b_$p.json 2> $O/b_$p.err || { echo "BENCH FAIL pool=$p"; tail -5 $O/b_$p.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_$p.json').read().strip().splitlines()[-1]); print('$r pool=$p', d['value'], 'ms/launch %.2f' % d['roofline']['avg_launch_ms'], 'ev/seed', d['events_per_seed'])" | tee -a $O/summary.txt
  done
done
for p in 0 1; do
  MR_POOL=$p timeout -k 10 400 python tools/cfg_ab.py pool=$p C2,C3c >> $O/summary.txt 2> $O/cfg_$p.err || { echo "CFG FAIL pool=$p"; tail -5 $O/cfg_$p.err; exit 1; }
done
cat $O/summary.txt
