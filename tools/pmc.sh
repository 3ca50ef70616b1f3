#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over a short bench run.
# usage: bash tools/pmc.sh <outdir> [bench args...]; PMC_GROUPS="g1;g2;..." overrides the groups
set -e
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
DEF="FETCH_SIZE;WRITE_SIZE;TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum;TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum;TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU;SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM;TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE;SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"
IFS=';' read -ra groups <<< "${PMC_GROUPS:-$DEF}"
i=0
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$out/p$i" -o run -- python3 bench.py --no-cpu-baseline --million 0 "$@" > "$out/p$i.log" 2>&1
done
