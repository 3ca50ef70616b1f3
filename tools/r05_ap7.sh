#!/bin/bash
# A/B: the 7-server Raft pool with auto-streaming (AP7) against the step kernel (CUR) on config 4;
# parity of AP7 on the 2D tests at 7 servers first
cd "$GRAFT_REPO_ROOT"; T=$1; O=gpurun_out/$T; mkdir -p $O; V=$PWD/madraft_amd/lib/var
MADRAFT_HIP_LIB=$V/AP7.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "snapshot_7_nodes or (test_scenario_bit_exact and _2d)" > $O/parity_AP7.log 2>&1 || { echo "PARITY FAIL"; tail -30 $O/parity_AP7.log; exit 1; }
echo "AP7 parity: $(tail -1 $O/parity_AP7.log)"
MADRAFT_HIP_LIB=$V/AP7.so timeout -k 10 300 python -c "
from madraft_amd import sim
with sim.Batch('snapshot_install_unreliable_2d', 4096, nodes=7) as b:
    print('kernel at 7 servers:', b.kernel)"
for r in 1 2; do
  for f in CUR AP7; do
    MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 400 python tools/cfg_ab.py $f C4 2>&1 | grep -v amdgpu.ids | tee -a $O/summary.txt || exit 1
  done
done
