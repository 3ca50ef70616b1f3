#!/bin/bash
# dev experiment pass on the GPU box: section profiles of a -DMR_PROF build at
# several batch sizes, then benches of the variant libraries in madraft_amd/lib/var/
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$PWD/madraft_amd/lib/var
for n in ${PROF_SIZES:-}; do
  MADRAFT_HIP_LIB=$V/prof.so timeout -k 10 300 python tools/prof.py figure_8_unreliable_2c $n > gpurun_out/prof_$n.txt 2>&1
done
bash tools/bench_variants.sh ${BENCH:-}
