"""The oracle against the committed verdict histograms (tests/golden/verdict_hist.json): every
supported scenario over its first 256 seeds and BASELINE config 2's shape over 8 192 seeds.
The GPU parity tests hold the HIP path to the same file (test_scenario_bit_exact,
test_config2_verdict_histogram), so a liveness regression common to both sides fails here."""
import json
import os

import numpy as np
import pytest

from madraft_amd import sim

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "verdict_hist.json")))


@pytest.mark.parametrize("case", GOLD["cases"], ids=[c["name"] for c in GOLD["cases"]])
def test_oracle_verdict_histogram(oracle, case):
    cfg = sim.make_cfg(case["test"], case["clusters"], **case["kw"])
    code, _, _, _ = oracle.run_batch(cfg, 0, case["clusters"])
    vals, cnt = np.unique(code, return_counts=True)
    assert {str(int(v)): int(n) for v, n in zip(vals, cnt)} == case["hist"]
