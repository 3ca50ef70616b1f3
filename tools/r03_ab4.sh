#!/bin/bash
# AE sub-class for every scenario with >= 32 / 40 / 48 other node events (r32/r40/r48) and the
# next-event prefetch (nf1: node record, nf2: + message record) vs the current tree (b0)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r03ab4
O=gpurun_out/r03ab4
V=$PWD/madraft_amd/lib/var
for r in 1 2; do
  for f in b0.so r32.so r40.so r48.so; do
    MADRAFT_HIP_LIB=$V/$f timeout -k 10 300 python tools/cfg_ab.py $f C3,C3c,C5 >> $O/cfg.txt 2>> $O/cfg.err || { echo "FAIL $f"; tail $O/cfg.err; exit 1; }
  done
  for f in b0.so nf1.so nf2.so wp.so; do
    MADRAFT_HIP_LIB=$V/$f timeout -k 10 300 python tools/cfg_ab.py $f C2,C3,C3c >> $O/pf.txt 2>> $O/cfg.err || { echo "FAIL $f"; tail $O/cfg.err; exit 1; }
  done
done
cat $O/cfg.txt $O/pf.txt
