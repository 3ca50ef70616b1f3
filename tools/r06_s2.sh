#!/bin/bash
# round-6 session 2: the 7-server pool's parity tests on the product library, A/B of the
# AppendEntries-long queue (AEL) on the headline, config 4 variants, the AEL section profile
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06_s2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_guard.py -x -v --timeout 300 --timeout-method thread \
  -k "seven_server or snapshot_7 or baseline_sizes or pool_workgroup or pool_and_step or planted" > $O/pytest.log 2>&1 \
  || { echo "pytest FAILED"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TESTS="figure_8_unreliable_2c figure_8_unreliable_crash" ROUNDS=2 STEPS=5 BARGS="--pipeline 1" bash tools/ab.sh r06_s2/ab BASE7 AEL || exit 1
for v in C4B C4AEL C4COOP C4AC6; do
  MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/$v.so POOLS=1 timeout -k 10 300 python tools/r06_cfg_ab.py snapshot_install_unreliable_2d 262144 7 2 1 2>&1 | tail -1 | tee -a $O/c4.txt || exit 1
done
MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/AELP.so timeout -k 10 180 python tools/prof.py figure_8_unreliable_2c 131072 > $O/prof_ael.txt 2>&1 || { echo "PROF FAIL"; tail $O/prof_ael.txt; exit 1; }
tail -8 $O/prof_ael.txt
