"""Regenerate tests/golden/verdict_hist.json: the oracle's verdict histogram of every supported
scenario over its first 256 seeds, with the configuration the GPU parity test builds
(madraft_amd.sim.make_cfg(test, 256): the reference defaults of mr_cfg_init), plus the BASELINE
config 2 shape (fail_agree_2b, 5 nodes, message drop) over 8 192 seeds (verdict r4 item 2).

test_scenario_bit_exact asserts the GPU's histogram equals this file (and the oracle's, through
bit-exact parity), so a change that costs liveness on both sides at once fails it; the CPU suite
checks the oracle against it. Run:
    python tests/golden/make_verdicts.py
"""
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from madraft_amd import _abi, sim  # noqa: E402
from tests.oracle_lib import Oracle  # noqa: E402

SUPPORTED = [n for n in _abi.SCENARIOS if n and n not in _abi.GPU_UNSUPPORTED]
# (name, test, clusters, make_cfg keywords)
CASES = [(t, t, 256, {}) for t in SUPPORTED] + [
    ("fail_agree_2b@5u", "fail_agree_2b", 8192, dict(nodes=5, unreliable=True)),
]


def histogram(o, test, clusters, kw):
    cfg = sim.make_cfg(test, clusters, **kw)
    code, _, _, _ = o.run_batch(cfg, 0, clusters)
    return {str(k): v for k, v in sorted(collections.Counter(code.tolist()).items())}


def main():
    o = Oracle()
    out = {"note": "oracle verdict histograms (code -> clusters) over seeds [0, clusters) of "
                   "sim.make_cfg(test, clusters, **kw); tests/golden/make_verdicts.py",
           "cases": [{"name": n, "test": t, "clusters": c, "kw": kw, "hist": histogram(o, t, c, kw)}
                     for n, t, c, kw in CASES]}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "verdict_hist.json")
    json.dump(out, open(path, "w"), indent=1)
    print(path, len(out["cases"]), "cases")


if __name__ == "__main__":
    main()
