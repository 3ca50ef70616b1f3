#!/bin/bash
# the 15-client 3B body: the persisted snapshot's copy with non-temporal stores (NT, source copy) vs
# ordinary stores (NB, the committed sources); parity of NT first, three same-box rounds
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06_nt; mkdir -p $O; V=$PWD/madraft_amd/lib/var
T=snapshot_unreliable_recover_concurrent_partition_linearizable_3b
MADRAFT_HIP_LIB=$V/NT.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "test_scenario_bit_exact[$T] or test_linearizable_kv_15_clients_7_servers[$T]" > $O/parity.log 2>&1 || { echo "PARITY FAIL"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for r in 1 2 3; do for v in NB NT; do
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py $T 65536 0 2 1 2>&1 | tail -1 | tee -a $O/nt.txt || exit 1
done; done
