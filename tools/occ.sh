#!/bin/bash
# dev occupancy experiment on the GPU box (tools/occ.py over madraft_amd/lib/var/*.so)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=$PWD/madraft_amd/lib/var
run() { MADRAFT_HIP_LIB=$V/$1 timeout -k 10 240 python tools/occ.py $1 $2 $3 >> gpurun_out/occ.txt 2>> gpurun_out/occ.err || { echo "FAIL $1 $2 $3" >> gpurun_out/occ.txt; exit 1; }; }
run base.so 32 131072
run base.so 16 131072,196608
run w3.so 16 131072,196608
run w3lean.so 16 131072,196608
run w4lean.so 12 196608,262144
cat gpurun_out/occ.txt
