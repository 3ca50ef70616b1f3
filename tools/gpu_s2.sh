#!/bin/bash
# dev GPU pass: parity suite on the default library, then A/B of variant libraries
# usage (from gpurun): AB="v0.so v1.so" TAG=r02_s2 bash tools/gpu_s2.sh
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-dev}
if [ -x build/philox_bench ]; then
  timeout -k 10 60 build/philox_bench > gpurun_out/${TAG}_philox.txt 2>&1
fi
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  tail -3 gpurun_out/${TAG}_pytest_gpu.log
fi
V=$PWD/madraft_amd/lib/var
for r in 1 2; do
  for f in ${AB}; do
    MADRAFT_HIP_LIB=$V/$f timeout -k 10 240 python tools/occ.py $f ${M:-32} ${SIZES:-131072} \
      ${TEST:-figure_8_unreliable_2c} >> gpurun_out/${TAG}_ab.txt 2>> gpurun_out/${TAG}_ab.err
  done
done
cat gpurun_out/${TAG}_ab.txt
