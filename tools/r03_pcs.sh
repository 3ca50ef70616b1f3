#!/bin/bash
# PC sampling of the headline step kernel (library variant with line tables: pcs.so)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r03pcs
O=gpurun_out/r03pcs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/${LIB:-pcs}.so timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled \
  --pc-sampling-method ${METHOD:-host_trap} --pc-sampling-unit ${UNIT:-time} --pc-sampling-interval ${IVL:-100} \
  --output-format csv -d $O/raw -o run -- python3 bench.py --steps 1 --warmup 0 --variant= --no-cpu-baseline \
  > $O/run.log 2>&1 || { echo "pc sampling run failed"; tail -30 $O/run.log; exit 1; }
find $O/raw -name "*.csv" | head -20
f=$(find $O/raw -name "*pc_sampling*.csv" | head -1)
[ -n "$f" ] || { echo "no pc sampling csv"; exit 1; }
ls -la $f
python tools/pc_sum.py $f 120 > $O/summary.txt 2>&1
head -c 200000 $f > $O/head.csv
gzip -c $f > $O/pcs.csv.gz
ls -la $O
head -60 $O/summary.txt
