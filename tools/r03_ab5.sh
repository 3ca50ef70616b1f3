#!/bin/bash
# A/B of variant libraries on configs 2, 3, 3c, 5 (two alternating runs)
# usage: bash tools/r03_ab5.sh <outdir> <lib1> <lib2> ...  (names under madraft_amd/lib/var/)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; shift; mkdir -p $O
V=$PWD/madraft_amd/lib/var
for r in 1 2; do
  for f in "$@"; do
    MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 300 python tools/cfg_ab.py $f ${CFGS:-C2,C3,C3c,C5} >> $O/ab.txt 2>> $O/ab.err || { echo "FAIL $f"; tail $O/ab.err; exit 1; }
  done
done
cat $O/ab.txt
