#!/bin/bash
# KV snapshot copy chunk: 4 quads (K4, as committed) vs 8 (K8) vs 16 (K16) on the snapshotting
# kvraft bodies (3B linearizable, 3B) — parity of K8 / K16 first, then two same-box rounds
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06_kc; mkdir -p $O; V=$PWD/madraft_amd/lib/var
T=snapshot_unreliable_recover_concurrent_partition_linearizable_3b
U=snapshot_unreliable_recover_concurrent_partition_3b
for v in K8 K16; do
MADRAFT_HIP_LIB=$V/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "test_scenario_bit_exact[$T] or test_linearizable_kv_15_clients_7_servers[$T] or test_scenario_bit_exact[$U]" > $O/parity_$v.log 2>&1 || { echo "PARITY FAIL $v"; tail -30 $O/parity_$v.log; exit 1; }
tail -1 $O/parity_$v.log
done
for r in 1 2; do for v in K4 K8 K16; do
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py $T 65536 0 2 1 2>&1 | tail -1 | tee -a $O/kc.txt || exit 1
done; done
for v in K4 K8 K16; do
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py $U 65536 0 2 1 2>&1 | tail -1 | tee -a $O/kc.txt || exit 1
done
