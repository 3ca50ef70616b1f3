#!/bin/bash
# the 15-client 3B body: snapshot and install copies in 8-quad chunks (KB8, as committed) vs the
# install copy back at 4 (KI4); then KI4's section profile (HPKI4)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06_ki; mkdir -p $O; V=$PWD/madraft_amd/lib/var
T=snapshot_unreliable_recover_concurrent_partition_linearizable_3b
MADRAFT_HIP_LIB=$V/KI4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "test_scenario_bit_exact[$T] or test_linearizable_kv_15_clients_7_servers[$T]" > $O/parity.log 2>&1 || { echo "PARITY FAIL"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for r in 1 2 3; do for v in KB8 KI4; do
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py $T 65536 0 2 1 2>&1 | tail -1 | tee -a $O/ki.txt || exit 1
done; done
MADRAFT_HIP_LIB=$V/HPKI4.so timeout -k 10 300 python tools/prof.py $T 65536 > $O/prof_ki4.txt 2>&1; tail -12 $O/prof_ki4.txt
