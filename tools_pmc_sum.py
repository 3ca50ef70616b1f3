"""Summarise rocprofv3 --pmc passes (tools_pmc.sh output) for step_kernel.

usage: python tools_pmc_sum.py <pmc_dir> [--json out.json --test T --clusters C]

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a coalesced read, so it is
doubled. With --json the per-launch traffic is written in the form bench.py's
roofline.traffic reads (profiles/pmc_*.json).
"""
import argparse
import collections
import csv
import glob
import json

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--json")
ap.add_argument("--test", default="figure_8_unreliable_2c")
ap.add_argument("--clusters", type=int, default=131072)
a = ap.parse_args()

agg = collections.defaultdict(float)
disp = {}
for p in sorted(glob.glob(f"{a.dir}/p*/run_counter_collection.csv")):
    ids = set()
    for r in csv.DictReader(open(p)):
        if "step_kernel" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        ids.add(r["Dispatch_Id"])
    for k in {r for r in agg}:
        disp.setdefault(k, len(ids))
nd = max(disp.values()) if disp else 0
wc = agg.get("SQ_WAVE_CYCLES", 1)
print(f"dispatches={nd}")
for k in sorted(agg):
    print(f"{k:28s} {agg[k]:.4g}")
if "SQ_WAIT_ANY" in agg:
    print(f"wait_any/wave_cycles = {agg['SQ_WAIT_ANY'] / wc:.3f}  "
          f"active/wave_cycles = {agg['SQ_ACTIVE_INST_ANY'] / wc:.3f}")
if "FETCH_SIZE" in agg:
    rd = 2 * agg["FETCH_SIZE"] * 1024
    wr = agg.get("WRITE_SIZE", 0) * 1024
    per = (rd + wr) / max(disp.get("FETCH_SIZE", nd), 1)
    print(f"HBM bytes (2*FETCH_SIZE + WRITE_SIZE, KiB->B) = {rd + wr:.4g}; per launch {per:.4g}")
    if a.json:
        json.dump({"test": a.test, "clusters": a.clusters, "kernel": "step_kernel", "abi": 3,
                   "dispatches": disp.get("FETCH_SIZE", nd), "hbm_read_bytes": rd,
                   "hbm_write_bytes": wr, "hbm_bytes_per_launch": per,
                   "counters": dict(agg),
                   "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; "
                             "FETCH doubled per MI355X_MICROARCH.md HBM section"},
                  open(a.json, "w"), indent=1)
