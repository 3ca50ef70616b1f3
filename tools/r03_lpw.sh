#!/bin/bash
# lanes-per-wave: parity on the A/B library, then throughput per config; counter names for FETCH
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r03lpw
O=gpurun_out/r03lpw
V=$PWD/madraft_amd/lib/var
MADRAFT_HIP_LIB=$V/lp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "lanes_per_wave" > $O/parity.log 2>&1 || { echo "parity FAILED"; tail -30 $O/parity.log; exit 1; }
tail -3 $O/parity.log
for r in 1 2; do
  MADRAFT_HIP_LIB=$V/lp.so timeout -k 10 200 python tools/lpw_ab.py r$r C2 64,32,16 >> $O/ab.txt 2>> $O/ab.err || { echo "C2 fail"; tail $O/ab.err; exit 1; }
  MADRAFT_HIP_LIB=$V/lp.so timeout -k 10 200 python tools/lpw_ab.py r$r C3 64,32 >> $O/ab.txt 2>> $O/ab.err || { echo "C3 fail"; tail $O/ab.err; exit 1; }
  MADRAFT_HIP_LIB=$V/lp.so timeout -k 10 200 python tools/lpw_ab.py r$r C5 64,32 >> $O/ab.txt 2>> $O/ab.err || { echo "C5 fail"; tail $O/ab.err; exit 1; }
done
cat $O/ab.txt
timeout -k 10 60 rocprofv3 --list-avail > $O/counters.txt 2>&1 || true
grep -E "TCC_EA0_(RD|WR)REQ" $O/counters.txt | head -20 || true
