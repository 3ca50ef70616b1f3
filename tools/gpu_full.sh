#!/bin/bash
# Full GPU evidence pass on the box: parity tests, bench line, rocprofv3
# kernel-trace stats and PMC passes, all under gpurun_out/$TAG*.
# usage (from gpurun): TAG=r01_v5 bash tools/gpu_full.sh
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r01}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1
fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run \
  -- python3 bench.py --no-cpu-baseline --variant= --steps 2 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/${TAG}_kt.log 2>&1
if [ -z "$SKIP_PMC" ]; then
  PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU;SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM;TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
    bash tools/pmc.sh gpurun_out/${TAG}_pmc --variant= --steps 1 --warmup 0 ${BENCH_ARGS:-}
fi
