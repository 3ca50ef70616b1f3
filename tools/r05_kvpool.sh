#!/bin/bash
# the service pool (MR_POOL=2 units): parity of variant $2 on the kvraft / shard_ctrler tests it
# holds, then configs 5 / 5-lin on it with the pool (MR_POOL=1) and without (MR_POOL=0)
cd "$GRAFT_REPO_ROOT"; T=$1; f=$2; O=gpurun_out/$T; mkdir -p $O; V=$PWD/madraft_amd/lib/var
IDS="tests/test_gpu_parity.py::test_scenario_bit_exact[unreliable_3a] tests/test_gpu_parity.py::test_scenario_bit_exact[persist_partition_unreliable_linearizable_3a] tests/test_gpu_parity.py::test_scenario_bit_exact[snapshot_unreliable_recover_concurrent_partition_linearizable_3b] tests/test_gpu_parity.py::test_scenario_bit_exact[basic_4a] tests/test_gpu_parity.py::test_scenario_bit_exact[unreliable_one_key_3a] tests/test_gpu_parity.py::test_linearizable_kv_15_clients_7_servers tests/test_gpu_parity.py::test_kv_unreliable_traced tests/test_kv_trace.py::test_gpu_kv_applies_hold[unreliable_3a] tests/test_kv_trace.py::test_gpu_kv_applies_hold[persist_partition_unreliable_linearizable_3a] tests/test_kv_trace.py::test_gpu_kv_applies_at_baseline_size tests/test_kv_trace.py::test_gpu_kv_replay_catches_duplicate_appends"
MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $IDS > $O/parity_$f.log 2>&1 || { echo "PARITY FAIL $f"; grep -E "FAILED|Error|assert" $O/parity_$f.log | head -20; tail -30 $O/parity_$f.log; exit 1; }
echo "$f parity: $(tail -1 $O/parity_$f.log)"
for r in 1 2; do
  for p in 1 0; do
    MR_POOL=$p MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 400 python tools/cfg_ab.py "$f-pool$p" ${CFGS:-C5,C5L,C5L3b} 2>&1 | grep -v amdgpu.ids | tee -a $O/summary.txt || exit 1
  done
done
