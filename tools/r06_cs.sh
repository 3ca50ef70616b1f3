#!/bin/bash
# code size of the pool kernel (66 KB for the headline's, the instruction cache is 64 KB per two
# CUs): -O3 (CB) vs -Os (COS) vs -fno-unroll-loops (CNU) vs -O2 (CO2), headline + crash variant
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06_cs; mkdir -p $O; V=$PWD/madraft_amd/lib/var
for v in COS CNU CO2; do
MADRAFT_HIP_LIB=$V/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "test_scenario_bit_exact[figure_8_unreliable_2c] or test_scenario_bit_exact[figure_8_unreliable_crash]" > $O/parity_$v.log 2>&1 || { echo "PARITY FAIL $v"; tail -30 $O/parity_$v.log; exit 1; }
tail -1 $O/parity_$v.log
done
for r in 1 2; do for v in CB COS CNU CO2; do
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py figure_8_unreliable_2c 131072 0 6 1 2>&1 | tail -1 | tee -a $O/cs.txt || exit 1
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py figure_8_unreliable_crash 131072 0 6 1 2>&1 | tail -1 | tee -a $O/cs.txt || exit 1
done; done
