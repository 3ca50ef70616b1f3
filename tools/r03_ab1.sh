#!/bin/bash
# A/B: round-2 head (h0) vs phase-split kernel without (n0) / with (n1) cooperative draws; parity
# of n1 on the headline scenario's tests first
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r03ab1
O=gpurun_out/r03ab1
V=$PWD/madraft_amd/lib/var
MADRAFT_HIP_LIB=$V/n1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "figure_8_unreliable_2c and not eight" > $O/parity_n1.log 2>&1 || { echo "parity n1 FAILED"; tail -30 $O/parity_n1.log; exit 1; }
tail -3 $O/parity_n1.log
for r in 1 2; do
  for f in ${AB:-h0.so n0.so n1.so}; do
    MADRAFT_HIP_LIB=$V/$f timeout -k 10 240 python tools/occ.py $f 32 131072 figure_8_unreliable_2c >> $O/ab.txt 2>> $O/ab.err || { echo "FAIL $f"; cat $O/ab.err | tail; exit 1; }
  done
done
cat $O/ab.txt
