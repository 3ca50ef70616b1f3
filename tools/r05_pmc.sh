#!/bin/bash
# issue / divergence / wait counters of the headline kernel, step_kernel (MR_POOL=0) vs
# pool_kernel (MR_POOL=1), same library. usage: bash tools/r05_pmc.sh <tag> [lib]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-r05pmc}; mkdir -p $O
LIB=${2:-$PWD/madraft_amd/lib/libmadraft_hip.so}
G1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
G2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM"
for p in ${POOLS:-0 1}; do
  i=0
  for g in "$G1" "$G2"; do
    i=$((i+1))
    MR_POOL=$p MADRAFT_HIP_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $O/pool${p}_g$i -o run -- python3 bench.py --no-cpu-baseline --variant= --million 0 --steps 1 --warmup 0 > $O/pool${p}_g$i.log 2>&1 || { echo "PMC FAIL pool=$p g$i"; tail -3 $O/pool${p}_g$i.log; exit 1; }
  done
  python - $O $p <<'PY'
import csv, glob, sys, collections, json
O, p = sys.argv[1], sys.argv[2]
a = collections.defaultdict(float)
for f in glob.glob(f"{O}/pool{p}_g*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "step_kernel" in r["Kernel_Name"] or "pool_kernel" in r["Kernel_Name"]:
            a[r["Counter_Name"]] += float(r["Counter_Value"])
ev = None
for line in open(f"{O}/pool{p}_g1.log"):
    if line.startswith("{"):
        d = json.loads(line); ev = d["events_per_seed"] * d["config"]["clusters_total"]
print(f"pool={p}", " ".join(f"{k}={v:.4g}" for k, v in sorted(a.items())))
print(f"pool={p} per event: VALU {a['SQ_INSTS_VALU']/ev:.1f} SALU {a['SQ_INSTS_SALU']/ev:.1f} LDS {a['SQ_INSTS_LDS']/ev:.1f} "
      f"VMEM_RD {a['SQ_INSTS_VMEM_RD']/ev:.2f} VMEM_WR {a['SQ_INSTS_VMEM_WR']/ev:.2f} BR {a['SQ_INSTS_BRANCH']/ev:.1f}; "
      f"lanes/VALU {a['SQ_THREAD_CYCLES_VALU']/max(1,a['SQ_ACTIVE_INST_VALU']):.2f} wait {a['SQ_WAIT_ANY']/a['SQ_WAVE_CYCLES']:.3f} "
      f"active {a['SQ_ACTIVE_INST_ANY']/a['SQ_WAVE_CYCLES']:.3f} lds_conf/LDS {a['SQ_LDS_BANK_CONFLICT']/max(1,a['SQ_INSTS_LDS']):.2f}")
PY
done
