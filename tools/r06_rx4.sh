#!/bin/bash
# A/B of the four-slot rescan in the pool kernels: headline + crash variant, then config 4
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06_rx4; mkdir -p $O
TESTS="figure_8_unreliable_2c figure_8_unreliable_crash" ROUNDS=2 STEPS=5 BARGS="--pipeline 1" bash tools/ab.sh r06_rx4 B10 RX4 || exit 1
for r in 1 2; do for v in C4B10 C4RX4; do
  MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py snapshot_install_unreliable_2d 262144 7 2 1 2>&1 | tail -1 | tee -a $O/c4.txt || exit 1
done; done
