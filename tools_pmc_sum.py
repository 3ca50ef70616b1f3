"""Summarise rocprofv3 --pmc passes (tools_pmc.sh output) for step_kernel."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
agg = collections.defaultdict(float)
disp = 0
for p in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    ids = set()
    for r in csv.DictReader(open(p)):
        if "step_kernel" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        ids.add(r["Dispatch_Id"])
    disp = max(disp, len(ids))
wc = agg.get("SQ_WAVE_CYCLES", 1)
print(f"dispatches={disp}")
for k in sorted(agg):
    print(f"{k:28s} {agg[k]:.4g}")
if "SQ_WAIT_ANY" in agg:
    print(f"wait_any/wave_cycles = {agg['SQ_WAIT_ANY'] / wc:.3f}  active/wave_cycles = {agg['SQ_ACTIVE_INST_ANY'] / wc:.3f}")
if "FETCH_SIZE" in agg:
    print(f"HBM bytes (FETCH*2 corrected + WRITE) = {(2 * agg['FETCH_SIZE'] + agg.get('WRITE_SIZE', 0)) * 1024:.4g}")
