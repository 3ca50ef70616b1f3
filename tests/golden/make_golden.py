"""Regenerate tests/golden/oracle_golden.json from the CPU oracle.

The reference ships no golden vectors for this path, so
these fixtures are the oracle's own outputs for fixed seeds — regression pins
for the oracle and the expected values of the GPU parity tests. Run:
    python tests/golden/make_golden.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from madraft_amd import _abi  # noqa: E402
from tests.oracle_lib import Oracle  # noqa: E402

CASES = [dict(test=n, cfg={}, first=0, count=8)
         for n in _abi.SCENARIOS if n and n not in _abi.UNSUPPORTED]
CASES += [
    dict(test="initial_election_2a", cfg={"flags": _abi.MR_F_NULL_RAFT}, first=0, count=4),
    dict(test="basic_agree_2b", cfg={"flags": _abi.MR_F_NULL_RAFT}, first=0, count=2),
    dict(test="fail_agree_2b", cfg={"n_nodes": 5, "flags": _abi.MR_F_UNRELIABLE}, first=100,
         count=16),
    dict(test="snapshot_install_unreliable_2d", cfg={"n_nodes": 7}, first=0, count=8),
    dict(test="figure_8_unreliable_2c", cfg={}, first=1000, count=16),
    # Raft invariant checks and the buggy variants they catch (SEMANTICS §11)
    dict(test="figure_8_unreliable_2c", cfg={"flags": _abi.MR_F_SAFETY}, first=0, count=8),
    dict(test="many_election_2a", cfg={"flags": _abi.MR_F_SAFETY | _abi.MR_F_BUG_VOTE_TWICE},
         first=0, count=16),
    dict(test="figure_8_2c", cfg={"flags": _abi.MR_F_SAFETY | _abi.MR_F_BUG_VOTE_STALE},
         first=0, count=8),
    dict(test="rejoin_2b", cfg={"flags": _abi.MR_F_SAFETY | _abi.MR_F_BUG_NO_PREV_CHECK},
         first=0, count=8),
    # generic_test_linearizability's checker (SEMANTICS §9b) and the buggy servers it catches
    dict(test="persist_partition_unreliable_linearizable_3a", cfg={"flags": _abi.MR_F_BUG_NO_DEDUP},
         first=0, count=4),
    dict(test="persist_partition_unreliable_linearizable_3a",
         cfg={"flags": _abi.MR_F_BUG_STALE_READ}, first=0, count=8),
    dict(test="snapshot_unreliable_recover_concurrent_partition_linearizable_3b",
         cfg={"flags": _abi.MR_F_BUG_NO_DEDUP}, first=0, count=4),
]


def main():
    o = Oracle()
    out = {"generator": "tests/golden/make_golden.py", "seed_base": _abi.README_SEED,
           "cases": []}
    for case in CASES:
        cfg = o.cfg(case["test"], **case["cfg"])
        code, t, dig, s = o.run_batch(cfg, case["first"], case["count"])
        out["cases"].append(dict(case, code=code.tolist(), time_us=t.tolist(),
                                 digest=[format(int(d), "016x") for d in dig],
                                 events=s["events"]))
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, len(out["cases"]), "cases")


if __name__ == "__main__":
    main()
