#!/bin/bash
# AE sub-class rules for every 64-bit-key scenario (r16/r32: only with >= 16/32 other node events;
# k5: only AppendEntries of >= 5 entries; k1: only ones with entries) vs the current gate (b0);
# then a trial of the request-size PMC passes on the product library
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r03ab3
O=gpurun_out/r03ab3
V=$PWD/madraft_amd/lib/var
for r in 1 2; do
  for f in b0.so r16.so r32.so k5.so k1.so; do
    MADRAFT_HIP_LIB=$V/$f timeout -k 10 300 python tools/cfg_ab.py $f C2,C3,C3c,C5 >> $O/cfg.txt 2>> $O/cfg.err || { echo "FAIL $f"; tail $O/cfg.err; exit 1; }
  done
done
cat $O/cfg.txt
bash tools/pmc.sh $O/pmc --variant= --steps 1 --warmup 0 || { echo "pmc failed"; exit 1; }
python tools/pmc_sum.py $O/pmc > $O/pmc_summary.txt 2>&1
cat $O/pmc_summary.txt
