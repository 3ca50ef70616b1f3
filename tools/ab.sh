#!/bin/bash
# dev A/B on the GPU box: tools/occ.py over variant libraries (madraft_amd/lib/var/<name>.so)
# usage: AB="a.so b.so" SIZES=131072 M=32 bash tools/ab.sh
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=$PWD/madraft_amd/lib/var
for r in 1 2; do
  for f in ${AB}; do
    MADRAFT_HIP_LIB=$V/$f timeout -k 10 240 python tools/occ.py $f ${M:-32} ${SIZES:-131072} ${TEST:-figure_8_unreliable_2c} >> gpurun_out/ab.txt 2>> gpurun_out/ab.err || { echo "FAIL $f" >> gpurun_out/ab.txt; exit 1; }
  done
done
cat gpurun_out/ab.txt
