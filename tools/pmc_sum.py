"""Summarise rocprofv3 --pmc passes (tools/pmc.sh output) for pool_kernel / step_kernel.

usage: python tools/pmc_sum.py <pmc_dir> [--json out.json --test T --clusters C]

HBM traffic per launch, from the L2's fabric request counters (one pass per counter group):
reads = 128 x TCC_EA0_RDREQ_128B + 64 x _64B + 32 x _32B, writes = 64 x TCC_EA0_WRREQ_64B +
32 x (TCC_EA0_WRREQ - _64B). profiles/r03_fetch_calibration.txt: every read request of the
step kernel's shapes (scattered 16-B records and coalesced words) is a whole 128-B line, and
FETCH_SIZE (= RDREQ x 64 B) undercounts it by exactly 2 — the MI355X_MICROARCH.md doubling —
so FETCH_SIZE x 2 + WRITE_SIZE is printed beside it as a cross-check. With --json the record
bench.py's roofline.traffic reads (profiles/pmc_*.json) is written, stamped with the
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
a = ap.parse_args()

agg = collections.defaultdict(float)
disp = {}
kernels = set()
for p in sorted(glob.glob(f"{a.dir}/p*/run_counter_collection.csv")):
    ids, names = set(), set()
    for r in csv.DictReader(open(p)):
        if "step_kernel" not in r["Kernel_Name"] and "pool_kernel" not in r["Kernel_Name"]:
            continue
        kernels.add("pool_kernel" if "pool_kernel" in r["Kernel_Name"] else "step_kernel")
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        ids.add(r["Dispatch_Id"])
        names.add(r["Counter_Name"])
    for k in names:
        disp[k] = len(ids)
nd = max(disp.values()) if disp else 0
wc = agg.get("SQ_WAVE_CYCLES", 1)
print(f"dispatches={nd}")
for k in sorted(agg):
    print(f"{k:32s} {agg[k]:.4g}")
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


def per_launch(name):
    return agg[name] / max(disp.get(name, nd), 1)


kernel = "/".join(sorted(kernels))
out = {"test": a.test, "clusters": a.clusters, "kernel": kernel, "abi": 4, "lib_sha16": lib,
       "counters": dict(agg), "dispatches": disp}
if "FETCH_SIZE" in agg and "WRITE_SIZE" in agg:
    fs = 2 * per_launch("FETCH_SIZE") * 1024 + per_launch("WRITE_SIZE") * 1024
    out["fetch2_write_bytes_per_launch"] = fs
    print(f"2 x FETCH_SIZE + WRITE_SIZE per launch = {fs:.4g} B")
req = ("TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum")
if all(k in agg for k in req):
    rd = (128 * per_launch("TCC_EA0_RDREQ_128B_sum") + 64 * per_launch("TCC_EA0_RDREQ_64B_sum")
          + 32 * (per_launch("TCC_EA0_RDREQ_32B_sum") if "TCC_EA0_RDREQ_32B_sum" in agg else 0))
    w64 = per_launch("TCC_EA0_WRREQ_64B_sum")
    wr = 64 * w64 + 32 * (per_launch("TCC_EA0_WRREQ_sum") - w64)
    out.update(hbm_read_bytes=rd, hbm_write_bytes=wr, hbm_bytes_per_launch=rd + wr,
               method="rocprofv3 --pmc, one pass per group: reads 128/64/32 x TCC_EA0_RDREQ_"
                      "{128B,64B,32B}, writes 64 x WRREQ_64B + 32 x the rest (DESIGN.md 6.2)")
    print(f"request-size HBM bytes per launch: read {rd:.4g} + write {wr:.4g} = {rd + wr:.4g}")
elif "fetch2_write_bytes_per_launch" in out:
    out.update(hbm_bytes_per_launch=out["fetch2_write_bytes_per_launch"],
               method="rocprofv3 --pmc FETCH_SIZE x 2 + WRITE_SIZE (profiles/r03_fetch_calibration.txt)")
# divergence and LDS (north_star: "LDS bank-conflict and wavefront-divergence counters"):
# SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU is the mean number of active lanes per VALU
# instruction — calibrated on this pool with tools/valu_calib.hip (64 / 32 / 16 / 4 / 1 active
# lanes read 64.0 / 32.0 / 16.1 / 4.1 / 1.08, profiles/r04_valu_calib.txt) — so / 64 is the
# thread-level VALU utilisation; SQ_LDS_BANK_CONFLICT counts the extra LDS cycles bank conflicts
# cost, over SQ_LDS_IDX_ACTIVE (all LDS-array cycles)
if "SQ_THREAD_CYCLES_VALU" in agg and "SQ_ACTIVE_INST_VALU" in agg:
    out["valu_lane_util"] = agg["SQ_THREAD_CYCLES_VALU"] / agg["SQ_ACTIVE_INST_VALU"] / 64.0
    print(f"valu_lane_util = {out['valu_lane_util']:.4f} "
          f"({agg['SQ_THREAD_CYCLES_VALU'] / agg['SQ_ACTIVE_INST_VALU']:.2f} active lanes per VALU instruction)")
if "SQ_LDS_BANK_CONFLICT" in agg:
    out["lds_bank_conflicts_per_launch"] = per_launch("SQ_LDS_BANK_CONFLICT")
    if agg.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_frac"] = agg["SQ_LDS_BANK_CONFLICT"] / agg["SQ_LDS_IDX_ACTIVE"]
    print(f"lds_bank_conflicts per launch = {out['lds_bank_conflicts_per_launch']:.4g}")
for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU"):
    if k in agg:
        out[k.lower() + "_per_launch"] = per_launch(k)
if a.json:
    if lib is None:
        raise SystemExit("no lib_sha16 in the bench logs: cannot stamp the record")
    if "hbm_bytes_per_launch" not in out:
        raise SystemExit("no traffic counters in these passes")
    json.dump(out, open(a.json, "w"), indent=1)
