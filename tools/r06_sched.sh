#!/bin/bash
# LLVM AMDGPU machine-scheduler strategy: default (SB) vs max-memory-clause (SMC) vs max-ilp (SILP)
# on the headline and its crash variant; parity of each variant first
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06_sched; mkdir -p $O; V=$PWD/madraft_amd/lib/var
for v in SMC SILP; do
MADRAFT_HIP_LIB=$V/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "test_scenario_bit_exact[figure_8_unreliable_2c] or test_scenario_bit_exact[figure_8_unreliable_crash]" > $O/parity_$v.log 2>&1 || { echo "PARITY FAIL $v"; tail -30 $O/parity_$v.log; exit 1; }
tail -1 $O/parity_$v.log
done
for r in 1 2; do for v in SB SMC SILP; do
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py figure_8_unreliable_2c 131072 0 6 1 2>&1 | tail -1 | tee -a $O/sched.txt || exit 1
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py figure_8_unreliable_crash 131072 0 6 1 2>&1 | tail -1 | tee -a $O/sched.txt || exit 1
done; done
