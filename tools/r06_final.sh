#!/bin/bash
# round-6 evidence pass on the committed tree: GPU suite, smoke, bench (the driver's command
# shape, with config 3's 1M jobs), rocprofv3 kernel stats, PMC passes -> profiles/pmc_<tag>.json
# (stamped with the library hash; traffic + divergence + LDS counters), the BASELINE configs
# table. usage: PARTS="suite bench pmc configs" bash tools/r05_final.sh <tag>
# (one gpurun call is at most 20 minutes: run the parts in two calls)
cd "$GRAFT_REPO_ROOT"; T=${1:-r06}; O=gpurun_out/$T; mkdir -p $O
PARTS=${PARTS:-suite bench pmc configs}
has() { case " $PARTS " in *" $1 "*) return 0;; esac; return 1; }
if has suite; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { echo "GPU tests FAILED"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -3 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke FAILED"; cat $O/smoke.txt; exit 1; }
  cat $O/smoke.txt
fi
if has bench; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench FAILED"; tail $O/bench.err; exit 1; }
  cat $O/bench.json
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run \
    -- python3 bench.py --no-cpu-baseline --variant= --million 0 --steps 5 --warmup 1 > $O/kt.log 2>&1 || { echo "kernel trace FAILED"; tail $O/kt.log; exit 1; }
  find $O/kt -name "*kernel_stats.csv" -exec cat {} \; | head -5
fi
if has pmc; then
  bash tools/pmc.sh $O/pmc --variant= --steps 1 --warmup 0 --pipeline 1 || { echo "pmc FAILED"; exit 1; }
  python tools/pmc_sum.py $O/pmc --json $O/pmc_$T.json > $O/pmc_summary.txt 2>&1; tail -8 $O/pmc_summary.txt
fi
if has configs; then
  timeout -k 10 1000 python tools/configs.py 6 > $O/configs.txt 2> $O/configs.err || { echo "configs FAILED"; tail $O/configs.err; }
  cat $O/configs.txt
fi
