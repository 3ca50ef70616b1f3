#!/bin/bash
# round-3 evidence pass, part 2: rocprofv3 kernel stats, PMC passes -> pmc_r03.json (stamped with
# the library hash), the BASELINE configs table
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r03f
O=gpurun_out/r03f
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
# dependent-load latency at the step kernel's 26.8 GB footprint vs the number of lanes in flight
for L in 256 1024 8192 32768 65536 131072; do
  timeout -k 10 120 build/memlat chase $((26843545600 / L / 16 * 16)) 1000 1 $L >> $O/latency_vs_lanes.txt 2>&1 || { echo "chase $L failed"; exit 1; }
done
cat $O/latency_vs_lanes.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run \
  -- python3 bench.py --no-cpu-baseline --variant= --steps 5 --warmup 1 > $O/kt.log 2>&1 || { echo "kernel trace FAILED"; tail $O/kt.log; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cat {} \; | head -5
bash tools/pmc.sh $O/pmc --variant= --steps 1 --warmup 0 || { echo "pmc FAILED"; exit 1; }
python tools/pmc_sum.py $O/pmc --json $O/pmc_r03.json > $O/pmc_summary.txt 2>&1; cat $O/pmc_summary.txt | tail -4
timeout -k 10 900 python tools/configs.py 6 > $O/configs.txt 2> $O/configs.err || { echo "configs FAILED"; tail $O/configs.err; }
cat $O/configs.txt
