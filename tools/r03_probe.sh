#!/bin/bash
# round-3 first GPU pass: host probe, memory-shape micro-benchmarks (+ FETCH_SIZE calibration),
# baseline bench of the round-2 tree
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r03p
O=gpurun_out/r03p
python tools/probe_host.py > $O/host.txt 2>&1
for b in 1024 4096 16384 65536 204800; do
  for ch in 1 4; do
    timeout -k 10 120 build/memlat chase $b 2000 $ch >> $O/chase.txt 2>&1 || { echo "chase $b $ch failed"; exit 1; }
  done
done
cat $O/chase.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/sc_f -o run -- build/memlat scatter16 64 > $O/sc_f.log 2>&1 || { echo "pmc scatter failed"; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/st_f -o run -- build/memlat stream16 4096 > $O/st_f.log 2>&1 || { echo "pmc stream failed"; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace --output-format csv -d $O/sc_r -o run -- build/memlat scatter16 64 > $O/sc_r.log 2>&1 || echo "rdreq pass failed (counter names?)"
cat $O/sc_f.log $O/st_f.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
cat $O/bench.json
