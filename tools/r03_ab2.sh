#!/bin/bash
# full GPU suite on the product library, then A/B of AE-class / tester-prefetch variants
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r03ab2
O=gpurun_out/r03ab2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -eq 0 ] || { echo "GPU tests FAILED rc=$rc"; grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; exit 1; }
V=$PWD/madraft_amd/lib/var
for r in 1 2; do
  for f in ${AB:-b0.so ae2.so ae3.so tp.so ps.so}; do
    MADRAFT_HIP_LIB=$V/$f timeout -k 10 300 python tools/cfg_ab.py $f ${CFGS:-C2,C3,C3c,C5} >> $O/cfg.txt 2>> $O/cfg.err || { echo "FAIL $f"; tail $O/cfg.err; exit 1; }
  done
done
cat $O/cfg.txt
for r in 1 2; do
  for f in b0.so x1.so x2.so; do
    MADRAFT_HIP_LIB=$V/$f timeout -k 10 240 python tools/occ.py $f 32 131072 figure_8_unreliable_2c >> $O/cost.txt 2>> $O/cost.err || { echo "FAIL $f"; tail $O/cost.err; exit 1; }
  done
done
cat $O/cost.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in "scatter16 64" "stream16 4096"; do
  n=${m%% *}
  timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace --output-format csv -d $O/cal_$n -o run -- build/memlat $m > $O/cal_$n.log 2>&1 || echo "cal $n failed"
done
