#!/bin/bash
# round-4 evidence pass on the committed tree: GPU suite, smoke, bench (the driver's command
# shape, with config 3's 1M jobs), rocprofv3 kernel stats, PMC passes -> profiles/pmc_<tag>.json
# (stamped with the library hash; traffic + divergence + LDS counters), the BASELINE configs
# table. usage: bash tools/r04_final.sh <tag>
cd "$GRAFT_REPO_ROOT"; T=${1:-r04}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "GPU tests FAILED"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -3 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke FAILED"; cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run \
  -- python3 bench.py --no-cpu-baseline --variant= --million 0 --steps 5 --warmup 1 > $O/kt.log 2>&1 || { echo "kernel trace FAILED"; tail $O/kt.log; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cat {} \; | head -5
bash tools/pmc.sh $O/pmc --variant= --steps 1 --warmup 0 || { echo "pmc FAILED"; exit 1; }
python tools/pmc_sum.py $O/pmc --json $O/pmc_$T.json > $O/pmc_summary.txt 2>&1; tail -8 $O/pmc_summary.txt
if [ -z "$NO_CONFIGS" ]; then
  timeout -k 10 900 python tools/configs.py 6 > $O/configs.txt 2> $O/configs.err || { echo "configs FAILED"; tail $O/configs.err; }
  cat $O/configs.txt
fi
