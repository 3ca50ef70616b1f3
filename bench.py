"""bench.py — seeds/sec & simulated Raft events/sec on 5-node figure_8_unreliable_2c.

BASELINE.json metric; config 3 = 1,048,576 clusters sharded across 8 MI355X,
i.e. 131,072 clusters (seeds) per GPU — weak scaling, per-GPU work fixed.
A step = reset every cluster of this rank's batch to RaftTester::new state with
fresh seeds (device-side), then run the whole test (src/raft/tests.rs:688-741)
for all of them to a verdict. Inputs (seeds) are generated on the device; all
state is resident in HBM before the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--clusters C]
For N > 1 the driver runs it under torch.distributed.run (one rank per GPU); run
directly with --gpus N > 1 it starts that launcher itself as a child process.
Rank 0 prints ONE JSON line. Besides the headline workload it times config 3's
crash-restart + persister variant (`figure_8_unreliable_crash`: tests.rs:612-660's
crash1/start1 in figure_8_unreliable's loop) on the same shard, reported under
"variants".
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


NODE_B = lambda n: 2 * (32 + 8 * n)  # noqa: E731  node state read + written per node event
TESTER_B = 2 * 72   # tester frame (pc, result, 8 locals, 5 helper words, u64 arg) read + written
MSG_B = 32          # one message record: written at enqueue, read at delivery
ENTRY_B = 16        # one log entry (term, command): LE record
APPLY_B = 48        # applier: log entry + checker entry read, checker entry written


def alg_bytes(c, n):
    """Algorithmic bytes of a run from its counters: what the simulation must
    move, counted where it moves. Node events read + write the node's state (SURVEY.md §8d:
    2 * (32 + 8N)); tester events their frame; every message enqueued is written once and
    every delivered one read once (clogged / lost sends move nothing); AppendEntries
    payloads are read by the receiver at delivery (entries_shipped) and every log write is
    16 B; the applier reads the entry and the checker record and writes the record."""
    enq = c["msgs_sent"] - c["drop_clog"] - c["drop_loss"] - c["drop_overflow"]
    return ((c["ev_msg"] + c["ev_timer"]) * NODE_B(n) + c["ev_tester"] * TESTER_B
            + MSG_B * (enq + c["ev_msg"])
            + ENTRY_B * (c["entries_shipped"] + c["log_writes"] + 2 * c["entries_materialized"])
            + APPLY_B * c["applies"])


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


def load_pmc(test, clusters, lib_sha):
    """HBM traffic per step-kernel launch from the committed rocprofv3 --pmc summary
    (profiles/pmc_*.json, tools/pmc_sum.py) of THIS library build on this workload: the record
    whose lib_sha16 equals the loaded library's, else None (the bench then reports traffic null
    rather than a figure measured on another build)."""
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if (d.get("test") == test and d.get("clusters") == clusters
                and d.get("lib_sha16") == lib_sha):
            d["file"] = os.path.relpath(p, ROOT)
            return d
    return None


def host_cores():
    """CPUs this process may run on (sched_getaffinity), and the cgroup CPU quota in cores
    if one is set (cpu.max / cfs_quota_us), else None."""
    n = len(os.sched_getaffinity(0))
    quota = None
    for qf, pf in (("/sys/fs/cgroup/cpu.max", None),
                   ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "/sys/fs/cgroup/cpu/cpu.cfs_period_us")):
        try:
            if pf is None:
                q, p = open(qf).read().split()[:2]
            else:
                q, p = open(qf).read().strip(), open(pf).read().strip()
            if q not in ("max", "-1"):
                quota = round(int(q) / int(p), 2)
            break
        except (OSError, ValueError):
            continue
    return n, quota


def relaunch(gpus):
    """`python bench.py --gpus N` (N > 1) outside torch.distributed.run: start the launcher as
    a child process (nothing here has touched the GPU) and exit with its code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", os.environ.get("MASTER_PORT", "29511"),
           os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def time_steps(bs, first_seed, total, warmup, steps, barrier):
    """warmup untimed steps, then `steps` timed ones (barrier + device sync on both sides);
    every step resets a batch to fresh seeds and runs it to its verdicts, and its verdict
    counters are read inside the timed region.

    `bs` is one batch or a list of them. With two (the default for the headline), consecutive
    steps alternate between them, each on its own HIP stream, and step j + 1 is submitted
    before step j is finished: a pool kernel's workgroup that has run all its clusters frees
    its CU while the slowest clusters of other pools still run (the drain),
    and the next step's workgroups take those CUs. Step j's counters are still read (finish)
    before step j + 2 reuses its batch, and all `steps` steps end inside the timed region."""
    bs = bs if isinstance(bs, (list, tuple)) else [bs]
    nb = len(bs)

    def run(j0, n):
        out, pend = [], []
        for j in range(n):
            if len(pend) == nb:  # this step's batch still holds step j - nb: finish it first
                out.append(pend.pop(0).finish())
            b = bs[j % nb]
            b.submit(first_seed + (j0 + j) * total)
            pend.append(b)
        out.extend(b.finish() for b in pend)
        return out

    run(0, warmup)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    acc = run(warmup, steps)
    torch.cuda.synchronize()
    barrier()
    return time.perf_counter() - t0, acc


def summed(acc):
    keys = ["events", "ev_msg", "ev_timer", "ev_tester", "msgs_sent", "drop_clog", "drop_loss",
            "drop_overflow", "entries_shipped", "log_writes", "entries_materialized", "applies",
            "passed", "done"]
    tot = {k: sum(int(c[k]) for _, c in acc) for k in keys}
    tot["kernel_ms"] = sum(st["kernel_ms"] for st, _ in acc)
    tot["launches"] = sum(st["launches"] for st, _ in acc)
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--clusters", type=int, default=131072, help="clusters (seeds) per GPU")
    ap.add_argument("--test", default="figure_8_unreliable_2c")
    ap.add_argument("--nodes", type=int, default=0,
                    help="servers per cluster (0: the test's default; BASELINE config 4 runs the 2D "
                         "tests at 7)")
    ap.add_argument("--variant", default="figure_8_unreliable_crash",
                    help="second workload timed on the same shard ('' = none)")
    ap.add_argument("--variant-steps", type=int, default=2)
    ap.add_argument("--million", type=int, default=1 << 20,
                    help="N = 1 only: config 3's whole job (this many clusters) of the headline test and "
                         "of its crash variant, each on this one GPU streaming through the resident pools "
                         "(0 = skip)")
    ap.add_argument("--cpu-seeds", type=int, default=320000,
                    help="cpu_baseline sample: seeds in total, split over one process per core")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-safety", action="store_true",
                    help="without the per-event Raft invariant checks (MR_F_SAFETY)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) or gloo (one-GPU rehearsal)")
    ap.add_argument("--pipeline", type=int, default=2, choices=(1, 2),
                    help="batches the timed steps alternate between, each on its own HIP stream "
                         "(2: step j + 1 takes the CUs step j's drained pools free; 1: one at a time)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", 1))
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        relaunch(a.gpus)
    if world != a.gpus and "WORLD_SIZE" in os.environ and a.gpus != 1:
        sys.exit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", 0))
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
    kw = {"nodes": a.nodes} if a.nodes else {}
    bs = [sim.Batch(a.test, count, _abi.README_SEED, cluster_base=base, device=local,
                    safety=not a.no_safety, **kw) for _ in range(a.pipeline)]
    n = int(bs[0].cfg.n_nodes)
    elapsed, acc = time_steps(bs, _abi.README_SEED, total, a.warmup, a.steps, barrier)
    kernel = bs[0].kernel  # mr_batch_kernel: the kernel the timed launches ran
    for b in bs:
        b.close()
    r0 = summed(acc)
    last = acc[-1][1]
    tot = dict(r0)
    if world > 1:
        elapsed = mdist.allreduce_max(elapsed, device=dev)
        red = mdist.allreduce_counters({**last, **{k: r0[k] for k in mdist.SUM_KEYS if k in r0}},
                                       device=dev)
        tot.update({k: red[k] for k in r0 if k in red})
        last = red
    seeds = total * a.steps
    # roofline of the dominant kernel (pool_kernel / step_kernel): this rank's algorithmic bytes over its
    # timed launches / their summed HIP-event durations (events recorded on the batch's own
    # stream around every launch; rocprofv3 --kernel-trace agrees, profiles/). With pipelined
    # steps the launches overlap (step j + 1's workgroups start on CUs step j's drained pools
    # free), so the summed launch durations exceed the timed region: the bytes are then taken
    # over the timed region's wall clock per step instead (the launches' own average is kept
    # beside it as avg_launch_ms)
    r0_bytes = alg_bytes(r0, n)
    kern_s = r0["kernel_ms"] / 1000.0
    overlap = a.pipeline > 1
    time_s = elapsed if overlap else kern_s
    achieved = r0_bytes / time_s / 1e9 if time_s > 0 else 0.0
    lib_sha = sim.lib_sha16()
    pmc = load_pmc(a.test, a.clusters, lib_sha)
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    per_launch = r0_bytes / max(r0["launches"], 1)
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
        "events_per_sec": round(tot["events"] / elapsed, 1),
        "events_per_seed": round(tot["events"] / seeds, 1),
        "pass_rate": round(tot["passed"] / max(tot["done"], 1), 6),
        "drop_overflow": tot["drop_overflow"],
        "coverage": {"leaders_elected_log2": last["cov_leaders"]},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": traffic,
                     "traffic_over_alg": round(traffic / per_launch, 3) if traffic else None,
                     # wavefront divergence and LDS bank conflicts of the same build (rocprofv3
                     # --pmc: SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU / 64, calibrated by
                     # tools/valu_calib.hip; SQ_LDS_BANK_CONFLICT per launch), or null
                     "valu_lane_util": round(pmc["valu_lane_util"], 4) if pmc and "valu_lane_util" in pmc else None,
                     "lds_bank_conflicts": pmc.get("lds_bank_conflicts_per_launch") if pmc else None,
                     "valu_insts_per_event": (round(pmc["sq_insts_valu_per_launch"] / (r0["events"] / max(r0["launches"], 1)), 2)
                                              if pmc and "sq_insts_valu_per_launch" in pmc else None),
                     "traffic_source": (f"{pmc['file']} (lib {lib_sha}): {pmc.get('method', '')}"
                                        if pmc else f"no PMC record of lib {lib_sha} on this workload"),
                     "kernel": kernel,
                     "launches": r0["launches"],
                     "avg_launch_ms": round(r0["kernel_ms"] / max(r0["launches"], 1), 4),
                     "time_base": ("wall clock per step (pipelined steps: launches overlap)" if overlap
                                   else "HIP-event launch durations"),
                     "alg_bytes_per_launch": round(per_launch),
                     "alg_bytes_per_event": round(r0_bytes / max(r0["events"], 1), 1),
                     "model": "DESIGN.md §6 (node events 2(32+8N), tester 144, 32 B per message "
                              "enqueued / delivered, 16 B per entry read at delivery / written, "
                              "48 B per apply)"},
        "alg_bytes_total": alg_bytes(tot, n),
        "lib_sha16": lib_sha,
    }
    if a.variant:
        bvs = [sim.Batch(a.variant, count, _abi.README_SEED, cluster_base=base, device=local,
                         safety=not a.no_safety) for _ in range(a.pipeline)]
        ev, accv = time_steps(bvs, _abi.README_SEED, total, 1, a.variant_steps, barrier)
        for bv in bvs:
            bv.close()
        sv = summed(accv)
        if world > 1:
            ev = mdist.allreduce_max(ev, device=dev)
            red = mdist.allreduce_counters({**accv[-1][1], **{k: sv[k] for k in mdist.SUM_KEYS
                                                              if k in sv}}, device=dev)
            sv.update({k: red[k] for k in sv if k in red})
        out["variants"] = {a.variant: {
            "value": round(total * a.variant_steps / ev, 1), "unit": "seeds/s",
            "steps": a.variant_steps, "ms_per_step": round(ev * 1000 / a.variant_steps, 3),
            "events_per_sec": round(sv["events"] / ev, 1),
            "events_per_seed": round(sv["events"] / (total * a.variant_steps), 1),
            "pass_rate": round(sv["passed"] / max(sv["done"], 1), 6),
            "note": "config 3 read literally: crash1/start1 + persister (tests.rs:612-660) in "
                    "figure_8_unreliable's loop"}}
    if world == 1 and a.million:
        # config 3 read at full size on ONE GPU (BASELINE.json configs[2]: 1M clusters, which the
        # driver's 8-GPU run shards 131,072 per GPU): the whole job as consecutive chunks of the
        # resident capacity, headline test and its crash-restart + persister variant. The on-hardware
        # stand-in for the 8-GPU total; one untimed warmup job, then one timed job each
        out.setdefault("variants", {})
        for t in (a.test, "figure_8_unreliable_crash"):
            bm = sim.Batch(t, a.million, _abi.README_SEED, device=local, safety=not a.no_safety)
            em, accm = time_steps(bm, _abi.README_SEED + 7 * a.million, a.million, 1, 1, barrier)
            bm.close()
            sm = summed(accm)
            out["variants"][f"{t}@{a.million}"] = {
                "value": round(a.million / em, 1), "unit": "seeds/s", "clusters": a.million,
                "ms_per_job": round(em * 1000, 3), "events_per_sec": round(sm["events"] / em, 1),
                "events_per_seed": round(sm["events"] / a.million, 1),
                "pass_rate": round(sm["passed"] / max(sm["done"], 1), 6), "launches": sm["launches"],
                "note": "config 3's whole job on one MI355X (streaming through the resident pools)"}
    if world == 1 and not a.no_cpu_baseline:  # N = 1 only: the N > 1 lines are scaling points
        # one process per host core this job may use (north_star): the CPUs it may run on, capped
        # by its cgroup CPU quota — on the GPU box 256 CPUs are visible but the quota is 16
        # cores, and 256 processes on 16 cores' time measured 38 % below 16 processes
        # (profiles/r03_cpu_cores.txt), so the cap gives the CPU its best showing
        ncpu, quota = host_cores()
        procs = max(1, min(ncpu, int(quota))) if quota else ncpu
        per = max(100, -(-a.cpu_seeds // procs))
        out["cpu_baseline"] = cpu_baseline(a.test, per, procs, safety=not a.no_safety)
        out["cpu_baseline"]["host_cpus_visible"] = ncpu
        if quota is not None:
            out["cpu_baseline"]["cgroup_cpu_quota_cores"] = quota
        out["gpu_over_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 2)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
