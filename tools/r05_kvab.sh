#!/bin/bash
# kvraft kernels: divergence counters, then same-box A/B of library variants on configs 5 / 5-lin
# (parity of each variant on the kvraft parity tests first). usage: bash tools/r05_kvab.sh <tag> <v1> <v2> ...
cd "$GRAFT_REPO_ROOT"; T=$1; shift; O=gpurun_out/$T; mkdir -p $O; V=$PWD/madraft_amd/lib/var
[ -n "$NOPMC" ] || bash tools/r05_kvpmc.sh ${T}_pmc || exit 1
for f in "$@"; do
  IDS="tests/test_gpu_parity.py::test_scenario_bit_exact[unreliable_3a] tests/test_gpu_parity.py::test_scenario_bit_exact[persist_partition_unreliable_linearizable_3a] tests/test_gpu_parity.py::test_scenario_bit_exact[snapshot_unreliable_recover_concurrent_partition_linearizable_3b] tests/test_gpu_parity.py::test_linearizable_kv_15_clients_7_servers tests/test_gpu_parity.py::test_kv_unreliable_traced tests/test_kv_trace.py::test_gpu_kv_applies_hold[unreliable_3a] tests/test_kv_trace.py::test_gpu_kv_applies_at_baseline_size tests/test_kv_trace.py::test_gpu_kv_replay_catches_duplicate_appends"
  MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread ${PIDS:-$IDS} > $O/parity_$f.log 2>&1 || { echo "PARITY FAIL $f"; tail -15 $O/parity_$f.log; exit 1; }
  echo "$f parity: $(tail -1 $O/parity_$f.log)"
done
for r in 1 2; do
  for f in "$@"; do
    MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 400 python tools/cfg_ab.py $f ${CFGS:-C5,C5L,C5L3b} 2>&1 | tee -a $O/summary.txt || exit 1
  done
done
