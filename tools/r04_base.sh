#!/bin/bash
# round-4 first GPU pass: GPU suite on the committed tree, bench, divergence / LDS counter
# calibration (tools/valu_calib) and the step kernel's divergence / LDS counters.
# usage: bash tools/r04_base.sh <tag>
cd "$GRAFT_REPO_ROOT"; T=${1:-r04a}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "GPU tests FAILED"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -3 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $O/calib -o run -- ./tools/valu_calib > $O/calib.log 2>&1 || { echo "calib FAILED"; tail $O/calib.log; exit 1; }
PMC_GROUPS="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU" \
  bash tools/pmc.sh $O/pmc --variant= --steps 1 --warmup 0 || { echo "pmc FAILED"; exit 1; }
python tools/pmc_sum.py $O/pmc > $O/pmc_summary.txt 2>&1; cat $O/pmc_summary.txt
