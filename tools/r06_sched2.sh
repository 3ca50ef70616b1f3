#!/bin/bash
# max-memory-clause machine scheduling (SMC2) vs the default (SB2) on config 4, config 5 and the two
# 15-client linearizable bodies; parity of SMC2 first
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06_sched2; mkdir -p $O; V=$PWD/madraft_amd/lib/var
A=persist_partition_unreliable_linearizable_3a
T=snapshot_unreliable_recover_concurrent_partition_linearizable_3b
MADRAFT_HIP_LIB=$V/SMC2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "test_scenario_bit_exact[snapshot_install_unreliable_2d] or test_scenario_bit_exact[unreliable_3a] or test_scenario_bit_exact[$A] or test_scenario_bit_exact[$T] or test_linearizable_kv_15_clients_7_servers or (seven_server_pool and not crash)" > $O/parity.log 2>&1 || { echo "PARITY FAIL"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for r in 1 2; do for v in SB2 SMC2; do
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py snapshot_install_unreliable_2d 262144 7 2 1 2>&1 | tail -1 | tee -a $O/sched2.txt || exit 1
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py unreliable_3a 65536 0 3 1 2>&1 | tail -1 | tee -a $O/sched2.txt || exit 1
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py $A 65536 0 2 1 2>&1 | tail -1 | tee -a $O/sched2.txt || exit 1
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py $T 65536 0 2 1 2>&1 | tail -1 | tee -a $O/sched2.txt || exit 1
done; done
