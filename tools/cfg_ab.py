"""Dev A/B: GPU-only throughput of the BASELINE configs 2-5 for one library variant.

usage: MADRAFT_HIP_LIB=<lib> python tools/cfg_ab.py <tag> [C2,C3,C3c,C4,C5]
One line per config: kernel ms per step and seeds/s (1 warmup + 2 steps, as tools/configs.py).
"""
import os
import sys
import time

import torch  # noqa: F401  (HIP runtime first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from madraft_amd import _abi, sim

CONFIGS = {
    "C2": ("fail_agree_2b", 65536, dict(nodes=5, unreliable=True)),
    "C3": ("figure_8_unreliable_2c", 131072, dict(safety=True)),
    "C3c": ("figure_8_unreliable_crash", 131072, dict(safety=True)),
    "C3M": ("figure_8_unreliable_2c", 1048576, dict(safety=True)),  # config 3's whole job
    "C3cM": ("figure_8_unreliable_crash", 1048576, dict(safety=True)),
    "C4": ("snapshot_install_unreliable_2d", 262144, dict(nodes=7)),
    "C5": ("unreliable_3a", 65536, {}),
    "C5L": ("persist_partition_unreliable_linearizable_3a", 65536, {}),
    "C5L3b": ("snapshot_unreliable_recover_concurrent_partition_linearizable_3b", 65536, {}),
}
tag = sys.argv[1]
names = sys.argv[2].split(",") if len(sys.argv) > 2 else list(CONFIGS)
for name in names:
    test, c, kw = CONFIGS[name]
    if os.environ.get("LPW"):  # lanes per wave (0 = auto)
        kw = dict(kw, lanes_per_wave=int(os.environ["LPW"]))
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
    print(f"{tag} {name} {test} C={c} kernel_ms/step={ms / 2:.1f} seeds/s={2 * c / wall:.0f} "
          f"Gev/s={ev / (ms / 1e3) / 1e9:.3f}", flush=True)
