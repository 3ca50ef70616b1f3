"""Dev experiment: step-kernel throughput vs clusters per launch for one library variant.

usage: MADRAFT_HIP_LIB=<lib> python tools/occ.py <tag> <msg_slots> <clusters,...> [test]
Prints one line per batch size: kernel ms per step, seeds/s, events/s (1 warmup + 2 steps).
"""
import os
import sys
import time

import torch  # noqa: F401  (HIP runtime first, as in bench.py)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from madraft_amd import _abi, sim

tag, m, sizes = sys.argv[1], int(sys.argv[2]), [int(s) for s in sys.argv[3].split(",")]
test = sys.argv[4] if len(sys.argv) > 4 else "figure_8_unreliable_2c"
for c in sizes:
    with sim.Batch(test, c, safety=True, msg_slots=m) as b:
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
    print(f"{tag} M={m} C={c} kernel_ms/step={ms / 2:.1f} seeds/s={2 * c / wall:.0f} "
          f"Gev/s={ev / (ms / 1e3) / 1e9:.3f} ev/seed={ev / 2 / c:.0f} overflow={cnt['drop_overflow']}",
          flush=True)
