#!/bin/bash
# round-3 evidence pass on the committed tree: GPU suite, smoke, bench (driver's command),
# rocprofv3 kernel stats, PMC passes -> profiles/pmc_r03.json (stamped), configs table
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r03f
O=gpurun_out/r03f
V=$PWD/madraft_amd/lib/var
for r in 1 2; do
  for f in b0.so pol.so; do
    MADRAFT_HIP_LIB=$V/$f timeout -k 10 300 python tools/cfg_ab.py $f C2,C3,C3c,C5 >> $O/policy_ab.txt 2>> $O/policy_ab.err || { echo "FAIL $f"; tail $O/policy_ab.err; exit 1; }
  done
done
cat $O/policy_ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "GPU tests FAILED"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -5 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke FAILED"; cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench.json
