"""BASELINE.json configs 1-5 on one MI355X beside the CPU oracle (dev tool; profiles/r02_configs.txt).

usage: python tools/configs.py [cpu_seconds_per_config] [steps]
Each GPU line: 1 warmup + `steps` (default 4) timed steps of the config's per-GPU batch, stepped
as bench.py steps the headline (bench.time_steps: two batches on two streams, step j + 1
submitted before step j is finished; kernel ms = the launches' HIP-event average, which overlap;
seeds/s = wall clock); each CPU line: the oracle CLI with the same checks, 16 processes, a
bounded sample. Config 1 is the reference's single-seed CPU case (GPU column: one cluster).
"""
import json
import os
import subprocess
import sys
import time

import torch  # noqa: F401  (HIP runtime first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from madraft_amd import _abi, sim
from bench import time_steps  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_build", "mr_oracle")
CPU_S = float(sys.argv[1]) if len(sys.argv) > 1 else 6.0
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 4

CONFIGS = [  # (name, test, clusters per GPU, Batch kwargs, oracle CLI args)
    ("C1 initial_election_2a, 3 nodes, 1 seed", "initial_election_2a", 1, {}, []),
    ("C2 fail_agree_2b, 5 nodes, message drop", "fail_agree_2b", 65536,
     dict(nodes=5, unreliable=True), ["--nodes", "5", "--unreliable"]),
    ("C3 figure_8_unreliable_2c, 5 nodes (per-GPU shard of 1M)", "figure_8_unreliable_2c", 131072,
     dict(safety=True), ["--safety"]),
    ("C3' figure_8_unreliable_crash (crash-restart + persister)", "figure_8_unreliable_crash",
     131072, dict(safety=True), ["--safety"]),
    ("C4 snapshot_install_unreliable_2d, 7 nodes", "snapshot_install_unreliable_2d", 262144,
     dict(nodes=7), ["--nodes", "7"]),
    ("C5 unreliable_3a kvraft, 5 servers + 5 clerks", "unreliable_3a", 65536, {}, []),
    ("C5-lin persist_partition_unreliable_linearizable_3a, 7 servers + 15 clerks",
     "persist_partition_unreliable_linearizable_3a", 65536, {}, []),
    ("C5-lin snapshot_..._concurrent_partition_linearizable_3b, 7 servers + 15 clerks",
     "snapshot_unreliable_recover_concurrent_partition_linearizable_3b", 65536, {}, []),
]


def cpu_rate(test, args, seconds):
    """Seeds/s of the oracle CLI on 16 host processes, sample sized to ~`seconds`."""
    probe = subprocess.run([EXE, test] + args, env=dict(os.environ, MADSIM_TEST_NUM="20"),
                           capture_output=True, text=True)
    per = json.loads(probe.stdout.strip().splitlines()[-1])
    n = max(1, int(seconds * per["seeds_per_s"]))
    procs = 16
    t0 = time.perf_counter()
    ps = [subprocess.Popen([EXE, test] + args, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                           text=True, env=dict(os.environ, MADSIM_TEST_NUM=str(n),
                                               MADSIM_TEST_SEED=str(_abi.README_SEED + k * n)))
          for k in range(procs)]
    outs = [json.loads(p.communicate()[0].strip().splitlines()[-1]) for p in ps]
    wall = time.perf_counter() - t0
    return sum(o["seeds"] for o in outs) / wall, sum(o["events"] for o in outs) / wall, procs * n


for name, test, c, kw, args in CONFIGS:
    bs = [sim.Batch(test, c, **kw) for _ in range(2 if c > 1 else 1)]
    wall, acc = time_steps(bs, _abi.README_SEED, c, 1, STEPS, lambda: None)
    kern = bs[0].kernel
    for b in bs:
        b.close()
    ms = sum(st["kernel_ms"] for st, _ in acc) / STEPS
    ev = sum(cn["events"] for _, cn in acc)
    cnt = {k: sum(cn[k] for _, cn in acc) for k in ("passed", "done", "kv_lin_checked")}
    cs, ce, n = cpu_rate(test, args, CPU_S)
    print(f"{name}: GPU {STEPS * c / wall:,.0f} seeds/s, {ev / wall / 1e9:.3f} G events/s, "
          f"{wall * 1000 / STEPS:.1f} ms per step, {ms:.1f} kernel ms per {c} clusters ({kern}), "
          f"pass {cnt['passed']}/{cnt['done']}"
          + (f", lin-checked Gets {cnt['kv_lin_checked']:,}" if cnt["kv_lin_checked"] else "") + " | "
          f"CPU (oracle, 16 procs, {n} seeds) {cs:,.0f} seeds/s, {ce / 1e6:.1f} M events/s | "
          f"x{STEPS * c / wall / cs:.1f}", flush=True)
