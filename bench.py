"""bench.py — seeds/sec & simulated Raft events/sec on 5-node figure_8_unreliable_2c.

BASELINE.json metric; config 3 = 1,048,576 clusters sharded across 8 MI355X,
i.e. 131,072 clusters (seeds) per GPU — weak scaling, per-GPU work fixed.
A step = reset every cluster of this rank's batch to RaftTester::new state with
fresh seeds (device-side), then run the whole test (src/raft/tests.rs:688-741)
for all of them to a verdict. Inputs (seeds) are generated on the device; all
state is resident in HBM before the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--clusters C]
For N > 1 the driver runs it under torch.distributed.run (one rank per GPU).
Rank 0 prints ONE JSON line.
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import time

import torch  # first: our library then shares torch's HIP runtime (same SONAME)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from madraft_amd import _abi, sim  # noqa: E402
from madraft_amd import dist as mdist  # noqa: E402

METRIC = "seeds/sec & simulated Raft events/sec, 5-node figure8_unreliable, 1-8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def bytes_per_event(n):
    """SURVEY.md §8d algorithmic bytes per event: node SoA read + write
    (2 * (32 + 8N)) + one 32-B message slot written at send and read at
    delivery (64); + 12 B per log entry shipped (counted separately)."""
    return 2 * (32 + 8 * n) + 64


def cpu_baseline(test, seeds_per_proc, procs, safety=False):
    """The oracle CLI (madsim-like scalar DES) — MADSIM_TEST_NUM seeds per
    process, one process per host core, like `MADSIM_TEST_NUM=N cargo test`."""
    exe = os.path.join(ROOT, "oracle", "_build", "mr_oracle")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    t0 = time.perf_counter()
    ps = []
    for k in range(procs):
        env = dict(os.environ, MADSIM_TEST_SEED=str(_abi.README_SEED + 10_000_000 + k * seeds_per_proc),
                   MADSIM_TEST_NUM=str(seeds_per_proc))
        ps.append(subprocess.Popen([exe, test] + (["--safety"] if safety else []), env=env,
                                   stdout=subprocess.PIPE,
                                   stderr=subprocess.DEVNULL, text=True))
    outs = [json.loads(p.communicate()[0].strip().splitlines()[-1]) for p in ps]
    wall = time.perf_counter() - t0
    seeds = sum(o["seeds"] for o in outs)
    events = sum(o["events"] for o in outs)
    return {"value": round(seeds / wall, 1), "unit": "seeds/s", "cores": procs, "kind": "port",
            "events_per_sec": round(events / wall, 1), "wall_s": round(wall, 3),
            "sample": f"{procs} processes x {seeds_per_proc} seeds of {test} "
                      f"(oracle/mr_oracle{' --safety' if safety else ''}, "
                      f"MADSIM_TEST_NUM={seeds_per_proc} each)"}


def load_pmc(test, clusters):
    """HBM traffic per step-kernel launch from the committed rocprofv3 --pmc
    summary of the same workload (profiles/pmc_*.json), or None."""
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if d.get("test") == test and d.get("clusters") == clusters:
            best = d
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--clusters", type=int, default=131072, help="clusters (seeds) per GPU")
    ap.add_argument("--test", default="figure_8_unreliable_2c")
    ap.add_argument("--cpu-seeds", type=int, default=20000, help="cpu_baseline seeds per process")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-safety", action="store_true",
                    help="without the per-event Raft invariant checks (MR_F_SAFETY)")
    ap.add_argument("--pipeline", action="store_true",
                    help="two batches, step i+1 queued while step i runs (A/B: 5 %% slower)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) or gloo (one-GPU rehearsal)")
    a = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0)) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)  # RCCL over xGMI
        else:  # rehearsal of the N>1 path on one GPU (tests): counters all-reduced on the host
            dist.init_process_group(a.dist_backend)
            dev = torch.device("cpu")

    def barrier():
        if world > 1:
            dist.barrier()

    total = a.clusters * world
    base, count = mdist.shard(total, world, rank)
    mk = lambda: sim.Batch(a.test, count, _abi.README_SEED, cluster_base=base, device=local,
                           safety=not a.no_safety)
    # --pipeline: two batches on their own streams, step i+1 queued while step i runs so its
    # waves take the CUs step i's early-finishing waves free (mr_batch_submit / finish).
    # Measured 545 K vs 576 K seeds/s without: off by default.
    bufs = [mk(), mk()] if a.pipeline else [mk()]
    b = bufs[0]
    n = int(b.cfg.n_nodes)

    def run_steps(first, k, acc):
        """steps first..first+k-1, each a fresh batch of seeds, pipelined over `bufs`."""
        if k <= 0:
            return
        bufs[0].submit(_abi.README_SEED + first * total)
        for j in range(k):
            if j + 1 < k:
                bufs[(j + 1) % 2].submit(_abi.README_SEED + (first + j + 1) * total)
            st, c = bufs[j % 2].finish()
            acc.append((st, c))

    def run_steps_serial(first, k, acc):
        for j in range(k):
            b.submit(_abi.README_SEED + (first + j) * total)
            acc.append(b.finish())

    go = run_steps if a.pipeline else run_steps_serial
    go(0, a.warmup, [])
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    acc = []
    go(a.warmup, a.steps, acc)
    kernel_ms = 0.0
    launches = events = shipped = passed = done = 0
    for st, c in acc:  # counters were read inside the timed region (verdict collection)
        kernel_ms += st["kernel_ms"]
        launches += st["launches"]
        events += c["events"]
        shipped += c["entries_shipped"]
        passed += c["passed"]
        done += c["done"]
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    r0_events, r0_shipped = events, shipped
    last = acc[-1][1]
    if world > 1:
        elapsed = mdist.allreduce_max(elapsed, device=dev)
        tot = mdist.allreduce_counters({**last, "events": events, "entries_shipped": shipped,
                                        "passed": passed, "done": done}, device=dev)
        events, shipped, passed, done = (tot["events"], tot["entries_shipped"], tot["passed"],
                                         tot["done"])
    seeds = total * a.steps
    alg_bytes = events * bytes_per_event(n) + 12 * shipped
    # roofline of the dominant kernel (step_kernel): this rank's algorithmic
    # bytes over all timed launches / their summed HIP-event durations (events
    # recorded on the batch's own stream around every launch)
    r0_bytes = r0_events * bytes_per_event(n) + 12 * r0_shipped
    kern_s = kernel_ms / 1000.0
    achieved = r0_bytes / kern_s / 1e9 if kern_s > 0 else 0.0
    pmc = load_pmc(a.test, a.clusters)
    traffic = None
    if pmc:
        traffic = pmc.get("hbm_bytes_per_launch")
    out = {
        "metric": METRIC,
        "value": round(seeds / elapsed, 1),
        "unit": "seeds/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed * 1000 / a.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (device-generated Philox seeds; no dataset)",
        "config": {"workload": a.test, "nodes": n, "clusters_per_gpu": a.clusters,
                   "clusters_total": total, "parallelism": f"clusters sharded over {world} GPU(s)",
                   "loss": 0.1, "latency_ms": [1, 27], "safety_checks": not a.no_safety},
        "events_per_sec": round(events / elapsed, 1),
        "events_per_seed": round(events / seeds, 1),
        "pass_rate": round(passed / max(done, 1), 6),
        "coverage": {"leaders_elected_log2": (tot if world > 1 else last)["cov_leaders"]},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": traffic,
                     "kernel": "step_kernel",
                     "launches": launches,
                     "avg_launch_ms": round(kernel_ms / max(launches, 1), 4),
                     "alg_bytes_per_launch": round(r0_bytes / max(launches, 1)),
                     "bytes_per_event": bytes_per_event(n)},
        "alg_bytes_total": alg_bytes,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        procs = min(16, os.cpu_count() or 1)
        out["cpu_baseline"] = cpu_baseline(a.test, a.cpu_seeds, procs, safety=not a.no_safety)
        out["gpu_over_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 2)
    if rank == 0:
        print(json.dumps(out), flush=True)
    for x in bufs:
        x.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
