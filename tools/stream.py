"""Dev experiment: streaming lanes (cfg.lanes < clusters) vs one lane per cluster.

usage: MADRAFT_HIP_LIB=<lib> python tools/stream.py <clusters> <lanes,...> [test]
(lanes: 0 = automatic chunks; L = chunks of L clusters; sL = streaming over L lanes)
Prints kernel ms, seeds/s per lane setting (1 warmup + 2 runs) and checks that verdicts and
digests do not depend on the lane count.
"""
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (HIP runtime first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from madraft_amd import _abi, sim

c = int(sys.argv[1])
lanes = sys.argv[2].split(",")
test = sys.argv[3] if len(sys.argv) > 3 else "figure_8_unreliable_2c"
kw = dict(nodes=int(sys.argv[4])) if len(sys.argv) > 4 else dict(safety=True)
ref = None
for L in lanes:
    with sim.Batch(test, c, lanes=int(L.lstrip("s")), stream=L.startswith("s"), **kw) as b:
        b.run()
        ms = 0.0
        t0 = time.perf_counter()
        for k in range(2):
            b.reset(_abi.README_SEED + (k + 1) * c)
            st = b.run()
            ms += st["kernel_ms"]
        wall = time.perf_counter() - t0
        code, t, dig = b.verdicts()
        cnt = b.counters()
    same = "ref" if ref is None else ("same" if all(np.array_equal(a, b_) for a, b_ in zip(ref, (code, t, dig))) else "DIFFERENT")
    ref = ref or (code, t, dig)
    print(f"lanes={L} C={c} kernel_ms/run={ms / 2:.1f} seeds/s={2 * c / wall:.0f} "
          f"launches={st['launches']} pass={cnt['passed']}/{cnt['done']} events={cnt['events']} {same}",
          flush=True)
