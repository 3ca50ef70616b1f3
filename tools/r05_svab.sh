#!/bin/bash
# same-box A/B of service-pool variants on configs 5 / 5-lin (parity on the kvraft tests first)
cd "$GRAFT_REPO_ROOT"; T=$1; shift; O=gpurun_out/$T; mkdir -p $O; V=$PWD/madraft_amd/lib/var
IDS="tests/test_gpu_parity.py::test_scenario_bit_exact[unreliable_3a] tests/test_gpu_parity.py::test_scenario_bit_exact[persist_partition_unreliable_linearizable_3a] tests/test_gpu_parity.py::test_scenario_bit_exact[snapshot_unreliable_recover_concurrent_partition_linearizable_3b] tests/test_gpu_parity.py::test_linearizable_kv_15_clients_7_servers tests/test_gpu_parity.py::test_kv_unreliable_traced"
for f in "$@"; do
  MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $IDS > $O/parity_$f.log 2>&1 || { echo "PARITY FAIL $f"; tail -20 $O/parity_$f.log; exit 1; }
  echo "$f parity: $(tail -1 $O/parity_$f.log)"
done
for r in 1 2; do
  for f in "$@"; do
    MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 400 python tools/cfg_ab.py $f ${CFGS:-C5,C5L,C5L3b} 2>&1 | grep -v amdgpu.ids | tee -a $O/summary.txt || exit 1
  done
done
