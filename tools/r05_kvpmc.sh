#!/bin/bash
# issue / divergence / wait counters of the kvraft step kernels (configs 5 and 5-lin).
# usage: bash tools/r05_kvpmc.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r05kvpmc}; mkdir -p $O
G1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for t in unreliable_3a persist_partition_unreliable_linearizable_3a; do
  timeout -s KILL 180 rocprofv3 --pmc $G1 --kernel-trace --output-format csv -d $O/$t -o run -- python3 bench.py --test $t --clusters 65536 --no-cpu-baseline --variant= --million 0 --steps 1 --warmup 0 > $O/$t.log 2>&1 || { echo "PMC FAIL $t"; tail -3 $O/$t.log; exit 1; }
  python - $O $t <<'PY'
import csv, glob, sys, collections, json
O, t = sys.argv[1], sys.argv[2]
a = collections.defaultdict(float)
for f in glob.glob(f"{O}/{t}/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "step_kernel" in r["Kernel_Name"] or "pool_kernel" in r["Kernel_Name"]:
            a[r["Counter_Name"]] += float(r["Counter_Value"])
ev = None
for line in open(f"{O}/{t}.log"):
    if line.startswith("{"):
        d = json.loads(line); ev = d["events_per_seed"] * d["config"]["clusters_total"]
print(t, f"VALU/ev {a['SQ_INSTS_VALU']/ev:.1f} SALU/ev {a['SQ_INSTS_SALU']/ev:.1f} "
      f"lanes/VALU {a['SQ_THREAD_CYCLES_VALU']/max(1,a['SQ_ACTIVE_INST_VALU']):.2f} wait {a['SQ_WAIT_ANY']/a['SQ_WAVE_CYCLES']:.3f} "
      f"active {a['SQ_ACTIVE_INST_ANY']/a['SQ_WAVE_CYCLES']:.3f}")
PY
done
