#!/bin/bash
# the service pool's applier continuation (KVAP) against the committed sources (KVB): kvraft parity
# on the variant, then configs 5 / 5-lin on both (pool kernel, pipelined steps)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06_kvap; mkdir -p $O
V=$PWD/madraft_amd/lib/var
MADRAFT_HIP_LIB=$V/KVAP.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "test_scenario_bit_exact[unreliable_3a] or test_scenario_bit_exact[persist_partition_unreliable_linearizable_3a] or test_scenario_bit_exact[snapshot_unreliable_recover_concurrent_partition_linearizable_3b] or test_linearizable_kv_15_clients_7_servers or test_linearizability_checker_bit_exact[unreliable_3a" \
  > $O/parity.log 2>&1 || { echo "PARITY FAIL"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for r in 1 2; do for v in KVB KVAP; do
  for t in unreliable_3a persist_partition_unreliable_linearizable_3a snapshot_unreliable_recover_concurrent_partition_linearizable_3b; do
    MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py $t 65536 0 2 1 2>&1 | tail -1 | tee -a $O/kv.txt || exit 1
  done
done; done
