"""Dev A/B: serial steps vs two batches with step i+1 queued while step i runs
(mr_batch_submit / mr_batch_finish on their own streams). usage: python tools/pipe.py [C] [steps]"""
import os
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from madraft_amd import _abi, sim

C = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
test = "figure_8_unreliable_2c"
bufs = [sim.Batch(test, C, safety=True), sim.Batch(test, C, safety=True)]
for mode in ("serial", "pipelined", "serial", "pipelined"):
    bufs[0].submit(_abi.README_SEED)
    bufs[0].finish()
    t0 = time.perf_counter()
    if mode == "serial":
        for j in range(K):
            bufs[0].submit(_abi.README_SEED + (j + 1) * C)
            bufs[0].finish()
    else:
        bufs[0].submit(_abi.README_SEED + C)
        for j in range(K):
            if j + 1 < K:
                bufs[(j + 1) % 2].submit(_abi.README_SEED + (j + 2) * C)
            bufs[j % 2].finish()
    dt = time.perf_counter() - t0
    print(f"{mode} C={C} steps={K} ms/step={dt * 1e3 / K:.1f} seeds/s={K * C / dt:.0f}", flush=True)
for b in bufs:
    b.close()
