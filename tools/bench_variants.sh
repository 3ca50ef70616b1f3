#!/bin/bash
for f in "$@"; do
  MADRAFT_HIP_LIB=$PWD/madraft_amd/lib/var/$f timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$f.log 2>&1 || { echo "$f FAILED"; continue; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], 'Gev/s %.3f' % (d['events_per_sec']/1e9), 'ev/seed', d['events_per_seed'], d['roofline']['launches'])"
done
