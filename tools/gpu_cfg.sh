#!/bin/bash
# dev GPU pass: BASELINE configs 2-5 (GPU only) for variant libraries, two alternating rounds
# usage (from gpurun): AB="h0.so s4.so" TAG=x bash tools/gpu_cfg.sh
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=$PWD/madraft_amd/lib/var
for r in 1 2; do
  for f in ${AB}; do
    MADRAFT_HIP_LIB=$V/$f timeout -k 10 300 python tools/cfg_ab.py $f ${CFGS:-C2,C3,C3c,C4,C5} \
      >> gpurun_out/${TAG}_cfg.txt 2>> gpurun_out/${TAG}_cfg.err || { echo "FAIL $f"; exit 1; }
  done
done
cat gpurun_out/${TAG}_cfg.txt
