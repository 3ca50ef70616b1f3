#!/bin/bash
# the KV snapshot copy with the next chunk's loads issued before the current chunk's stores (K47P)
# vs as committed (K47B), on the snapshotting 15-client linearizable 3B body
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06_k47p; mkdir -p $O; V=$PWD/madraft_amd/lib/var
T=snapshot_unreliable_recover_concurrent_partition_linearizable_3b
MADRAFT_HIP_LIB=$V/K47P.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "test_scenario_bit_exact[$T] or test_linearizable_kv_15_clients_7_servers[$T]" > $O/parity.log 2>&1 || { echo "PARITY FAIL"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for r in 1 2; do for v in K47B K47P; do
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py $T 65536 0 2 1 2>&1 | tail -1 | tee -a $O/kv.txt || exit 1
done; done
