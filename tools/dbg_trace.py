"""Dev helper: print a traced cluster's GPU records next to the oracle's around the first
difference. usage: MADRAFT_HIP_LIB=<lib> python tools/dbg_trace.py <test> <clusters> [k] [before]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from madraft_amd import sim  # noqa: E402
from tests.oracle_lib import Oracle  # noqa: E402

test, clusters = sys.argv[1], int(sys.argv[2])
k = int(sys.argv[3]) if len(sys.argv) > 3 else 0
before = int(sys.argv[4]) if len(sys.argv) > 4 else 40
with sim.Batch(test, clusters, trace_clusters=k + 1) as b:
    b.run()
    g = b.trace(k)
    cfg = b.cfg
    print("kernel", b.kernel)
_, o = Oracle().run_cluster(cfg, k, trace_cap=int(cfg.trace_cap))
n = min(len(g), len(o))
d = next((i for i in range(n) if g[i] != o[i]), n)
print(f"{test} cluster {k}: gpu {len(g)} records, oracle {len(o)}, first difference at {d}")
for i in range(max(0, d - before), min(n, d + 5)):
    mark = "  " if g[i] == o[i] else "!!"
    print(mark, i, "gpu", tuple(int(v) for v in g[i]), "oracle", tuple(int(v) for v in o[i]))
