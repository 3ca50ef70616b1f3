#!/bin/bash
# dev A/B run on the GPU box: parity of the default library, section profiles, variant benches
set -e
cd $GRAFT_REPO_ROOT
V=$PWD/madraft_amd/lib/var
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_default.log 2>&1
for p in ${PROFS:-}; do
  MADRAFT_HIP_LIB=$V/$p timeout -k 10 300 python tools/prof.py > gpurun_out/prof_$p.txt 2>&1
done
bash tools/bench_variants.sh ${BENCH:-}
