#!/bin/bash
# the tie-break of the earliest-message rescan with the tied slots' sequence numbers loaded four per
# trip (TB) vs one round trip per tied slot (BASE = HEAD's sources); TB also has InstallSnapshot's
# copy back at 4 quads. Parity of TB first, then two same-box rounds on four BASELINE configs.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06_tb; mkdir -p $O; V=$PWD/madraft_amd/lib/var
T=snapshot_unreliable_recover_concurrent_partition_linearizable_3b
MADRAFT_HIP_LIB=$V/TB.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "test_scenario_bit_exact[figure_8_unreliable_2c] or test_scenario_bit_exact[snapshot_install_unreliable_2d] or test_scenario_bit_exact[unreliable_3a] or test_scenario_bit_exact[$T] or test_linearizable_kv_15_clients_7_servers[$T] or (seven_server_pool and not crash)" > $O/parity.log 2>&1 || { echo "PARITY FAIL"; tail -30 $O/parity.log; exit 1; }
grep -c PASSED $O/parity.log; tail -1 $O/parity.log
for r in 1 2; do for v in BASE TB; do
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py figure_8_unreliable_2c 131072 0 6 1 2>&1 | tail -1 | tee -a $O/tb.txt || exit 1
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py snapshot_install_unreliable_2d 262144 7 2 1 2>&1 | tail -1 | tee -a $O/tb.txt || exit 1
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py unreliable_3a 65536 0 3 1 2>&1 | tail -1 | tee -a $O/tb.txt || exit 1
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py $T 65536 0 2 1 2>&1 | tail -1 | tee -a $O/tb.txt || exit 1
done; done
