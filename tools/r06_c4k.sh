#!/bin/bash
# config 4 on the 7-server pool: fine kinds (C4F) / node timers in a kind of their own (C4T) vs as
# committed (C4X)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06_c4k; mkdir -p $O; V=$PWD/madraft_amd/lib/var
T=snapshot_install_unreliable_2d
for v in C4F C4T; do
  MADRAFT_HIP_LIB=$V/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "(seven_server and not crash) or snapshot_7" > $O/parity_$v.log 2>&1 || { echo "PARITY FAIL $v"; tail -30 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
for r in 1 2; do for v in C4X C4F C4T; do
  MADRAFT_HIP_LIB=$V/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py $T 262144 7 2 1 2>&1 | tail -1 | tee -a $O/c4.txt || exit 1
done; done
