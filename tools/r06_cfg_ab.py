"""Dev helper: one BASELINE config on the pool kernel and on the step kernel (MR_POOL=0), same
library, same box, each stepped as bench.py steps the headline (bench.time_steps, pipelined).

usage: python tools/r06_cfg_ab.py <test> <clusters> [nodes] [steps] [rounds]
(POOLS="1" runs the pool kernel only, e.g. to compare variant libraries via MADRAFT_HIP_LIB)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
import torch  # noqa: E402,F401  (HIP runtime first)

from bench import time_steps  # noqa: E402
from madraft_amd import _abi, sim  # noqa: E402

test, c = sys.argv[1], int(sys.argv[2])
nodes = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3] != "0" else None
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 2
kw = {"nodes": nodes} if nodes else {}
for r in range(rounds):
    for pool in os.environ.get("POOLS", "1 0").split():
        os.environ["MR_POOL"] = pool
        bs = [sim.Batch(test, c, **kw) for _ in range(2)]
        wall, acc = time_steps(bs, _abi.README_SEED, c, 1, steps, lambda: None)
        kern = bs[0].kernel
        for b in bs:
            b.close()
        ev = sum(cn["events"] for _, cn in acc)
        ok = sum(cn["passed"] for _, cn in acc)
        lib = os.path.basename(sim.LIB_PATH)
        print(f"{r} {test} n={nodes} {lib} {kern}: {steps * c / wall:,.0f} seeds/s, "
              f"{wall * 1000 / steps:.1f} ms per step, ev/seed {ev / (steps * c):.1f}, "
              f"pass {ok}/{steps * c}", flush=True)
