#!/bin/bash
# full GPU suite + smoke + a short bench of the committed library. usage: bash tools/r05_suite.sh <tag>
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r05suite}; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "GPU tests FAILED"; grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; tail -3 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke FAILED"; cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --million 0 > $O/bench.json 2> $O/bench.err || { echo "bench FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench.json
