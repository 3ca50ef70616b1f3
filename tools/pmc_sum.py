"""Summarise rocprofv3 --pmc passes (tools/pmc.sh output) for step_kernel.

usage: python tools/pmc_sum.py <pmc_dir> [--json out.json --test T --clusters C]

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; FETCH_SIZE is scaled by --fetch-factor (the guide's 2 for wide coalesced
streaming reads; DESIGN.md §6.2 records what tools/memlat.hip measured for this
kernel's scattered record reads). With --json the per-launch traffic is written in
the form bench.py's roofline.traffic reads (profiles/pmc_*.json), stamped with the
lib_sha16 the profiled bench runs printed: bench.py uses a record only for that build.
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
ap.add_argument("--fetch-factor", type=float, default=2.0)
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
libs = set()
for p in glob.glob(f"{a.dir}/p*.log"):
    for line in open(p, errors="replace"):
        if line.startswith("{") and "lib_sha16" in line:
            try:
                libs.add(json.loads(line)["lib_sha16"])
            except ValueError:
                pass
if len(libs) > 1:
    raise SystemExit(f"PMC passes of different library builds: {sorted(libs)}")
lib = libs.pop() if libs else None
print(f"lib_sha16={lib}")
if "FETCH_SIZE" in agg:
    rd = a.fetch_factor * agg["FETCH_SIZE"] * 1024
    wr = agg.get("WRITE_SIZE", 0) * 1024
    per = (rd + wr) / max(disp.get("FETCH_SIZE", nd), 1)
    print(f"HBM bytes ({a.fetch_factor:g}*FETCH_SIZE + WRITE_SIZE, KiB->B) = {rd + wr:.4g}; "
          f"per launch {per:.4g}")
    if a.json:
        if lib is None:
            raise SystemExit("no lib_sha16 in the bench logs: cannot stamp the record")
        json.dump({"test": a.test, "clusters": a.clusters, "kernel": "step_kernel", "abi": 3,
                   "lib_sha16": lib, "fetch_factor": a.fetch_factor,
                   "dispatches": disp.get("FETCH_SIZE", nd), "hbm_read_bytes": rd,
                   "hbm_write_bytes": wr, "hbm_bytes_per_launch": per,
                   "counters": dict(agg),
                   "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; "
                             f"FETCH_SIZE x {a.fetch_factor:g} (DESIGN.md 6.2)"},
                  open(a.json, "w"), indent=1)
