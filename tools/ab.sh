#!/bin/bash
# same-box A/B of variant libraries (madraft_amd/lib/var/<name>.so, tools/var.py): a parity
# smoke per variant (GPU vs oracle, $PTEST), then $ROUNDS alternating rounds of bench.py on each
# test in $TESTS. usage: bash tools/ab.sh <outdir> <name1> <name2> ...
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; shift; mkdir -p $O
V=$PWD/madraft_amd/lib/var
TESTS=${TESTS:-figure_8_unreliable_2c}
PTEST=${PTEST:-"test_scenario_bit_exact and (figure_8_unreliable_2c or figure_8_unreliable_crash)"}
for f in "$@"; do
  case " $NOPAR " in *" $f "*) echo "$f parity: skipped (timing-only variant)"; continue;; esac
  if [ -n "$PIDS" ]; then set -- "$@"; PARGS=($PIDS); else PARGS=(tests/test_gpu_parity.py -k "$PTEST"); fi
  MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread "${PARGS[@]}" > $O/parity_$f.log 2>&1 || { echo "PARITY FAIL $f"; tail -15 $O/parity_$f.log; exit 1; }
  echo "$f parity: $(tail -1 $O/parity_$f.log)"
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for t in $TESTS; do
    for f in "$@"; do
      MADRAFT_HIP_LIB=$V/$f.so timeout -k 10 300 python bench.py --test $t --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --variant '' --million 0 $BARGS > $O/b_${t}_$f.json 2> $O/b_${t}_$f.err || { echo "BENCH FAIL $f $t"; tail -5 $O/b_${t}_$f.err; exit 1; }
      python -c "import json; d=json.loads(open('$O/b_${t}_$f.json').read().strip().splitlines()[-1]); print('$r $t $f', d['value'], 'ms/launch %.2f' % d['roofline']['avg_launch_ms'], 'ev/seed', d['events_per_seed'])" | tee -a $O/summary.txt
    done
  done
done
if [ -n "$PMC" ]; then  # one counter pass per variant: issued instructions, divergence, waits
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  for f in "$@"; do
    MADRAFT_HIP_LIB=$V/$f.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/pmc_$f -o run -- python3 bench.py --no-cpu-baseline --variant= --million 0 --steps 1 --warmup 0 $BARGS > $O/pmc_$f.log 2>&1 || { echo "PMC FAIL $f"; tail -3 $O/pmc_$f.log; exit 1; }
    python - "$O/pmc_$f" "$f" <<'PY' | tee -a $O/summary.txt
import csv, glob, sys, collections, json
a = collections.defaultdict(float)
for p in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "step_kernel" in r["Kernel_Name"] or "pool_kernel" in r["Kernel_Name"]:
            a[r["Counter_Name"]] += float(r["Counter_Value"])
ev = None
for line in open(sys.argv[1] + ".log"):
    if line.startswith("{"):
        d = json.loads(line); ev = d["events_per_seed"] * d["config"]["clusters_total"]
print(sys.argv[2], "VALU/ev %.2f SALU/ev %.2f lanes/VALU %.2f wait %.3f active %.3f" % (
    a["SQ_INSTS_VALU"] / ev, a["SQ_INSTS_SALU"] / ev, a["SQ_THREAD_CYCLES_VALU"] / a["SQ_ACTIVE_INST_VALU"],
    a["SQ_WAIT_ANY"] / a["SQ_WAVE_CYCLES"], a["SQ_ACTIVE_INST_ANY"] / a["SQ_WAVE_CYCLES"]))
PY
  done
fi

