import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import torch  # noqa
from madraft_amd import sim
from tests.oracle_lib import Oracle
o = Oracle()
for lib in sys.argv[1:]:
    sim.LIB_PATH = lib; sim._lib = None
    with sim.Batch("figure_8_unreliable_2c", 4096, safety=True) as b:
        b.run(); code, t, dig = b.verdicts(); cfg = b.cfg
    oc, ot, od, _ = o.run_batch(cfg, 0, 4096)
    print(os.path.basename(lib), "parity", np.array_equal(code, oc) and np.array_equal(t, ot) and np.array_equal(dig, od), flush=True)
