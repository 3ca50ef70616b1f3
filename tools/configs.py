"""BASELINE.json configs 1-5 on one MI355X beside the CPU oracle (dev tool; profiles/r02_configs.txt).

usage: python tools/configs.py [cpu_seconds_per_config]
Each GPU line: 1 warmup + 2 timed steps of the config's per-GPU batch (kernel ms from HIP
events, wall seeds/s); each CPU line: the oracle CLI with the same checks, 16 processes, a
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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_build", "mr_oracle")
CPU_S = float(sys.argv[1]) if len(sys.argv) > 1 else 6.0

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
    with sim.Batch(test, c, **kw) as b:
        b.run()
        ms = ev = 0.0
        t0 = time.perf_counter()
        for k in range(2):
            b.reset(_abi.README_SEED + (k + 1) * c)
            st = b.run()
            ms += st["kernel_ms"]
            ev += st["events"]
        wall = time.perf_counter() - t0
        cnt = b.counters()
    cs, ce, n = cpu_rate(test, args, CPU_S)
    print(f"{name}: GPU {2 * c / wall:,.0f} seeds/s, {ev / wall / 1e9:.3f} G events/s, "
          f"{ms / 2:.1f} kernel ms per {c} clusters, pass {cnt['passed']}/{cnt['done']}"
          + (f", lin-checked Gets {cnt['kv_lin_checked']:,}" if cnt["kv_lin_checked"] else "") + " | "
          f"CPU (oracle, 16 procs, {n} seeds) {cs:,.0f} seeds/s, {ce / 1e6:.1f} M events/s | "
          f"x{2 * c / wall / cs:.1f}", flush=True)
