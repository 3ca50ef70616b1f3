"""Dev A/B: step-kernel throughput vs lanes per wave (mr_cfg.lanes_per_wave) on BASELINE
configs. usage: MADRAFT_HIP_LIB=<lib> python tools/lpw_ab.py <tag> <config> <lpw,...>"""
import os
import sys
import time

import torch  # noqa: F401  (HIP runtime first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from madraft_amd import _abi, sim

CONFIGS = {
    "C2": ("fail_agree_2b", 65536, dict(nodes=5, unreliable=True)),
    "C3": ("figure_8_unreliable_2c", 131072, dict(safety=True)),
    "C5": ("unreliable_3a", 65536, {}),
}
tag, name = sys.argv[1], sys.argv[2]
test, c, kw = CONFIGS[name]
for lpw in [int(v) for v in sys.argv[3].split(",")]:
    with sim.Batch(test, c, lanes_per_wave=lpw, **kw) as b:
        b.run()
        ms = ev = 0.0
        t0 = time.perf_counter()
        for k in range(2):
            b.reset(_abi.README_SEED + (k + 1) * c)
            st = b.run()
            ms += st["kernel_ms"]
            ev += st["events"]
        wall = time.perf_counter() - t0
    print(f"{tag} {name} lpw={lpw} kernel_ms/step={ms / 2:.1f} seeds/s={2 * c / wall:.0f} "
          f"Gev/s={ev / (ms / 1e3) / 1e9:.3f} launches={st['launches']}", flush=True)
