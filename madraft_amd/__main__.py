"""CLI: `python -m madraft_amd <test> [--clusters N] [--seed S]` — the batched
analogue of `MADSIM_TEST_SEED=S MADSIM_TEST_NUM=N cargo test <test>`;
`--replay log.jsonl` plays one cluster driven by an event-level decision log
(madraft_amd/trace.py) and prints its verdict."""
import argparse
import json
import time

from . import _abi, sim, trace


# test bodies that switch the net back to reliable part-way (tests.rs:680 unreliable_agree_2c
# before join_all and the final one(); tests.rs:832 internal_churn before the final one()):
# their sends have no single mode, so a log of them must carry it per line (or be a raw log)
MIXED_MODE = {"unreliable_agree_2c", "unreliable_churn_2c"}


def net_mode(test, unreliable_flag):
    """The network mode a replayed log's sends were drawn under when a line does not say:
    `--unreliable` (MR_F_UNRELIABLE from the tester's start: every send unreliable), else the
    test body's own single mode — the tests named *unreliable* that stay unreliable to the end
    (figure_8_unreliable_2c tests.rs:692, snap_common's unreliable 2D tests :864) send every
    message unreliably, the others reliably. For the tests that switch modes (MIXED_MODE) there
    is no single answer: None, so trace.decisions_from_events rejects a send line without its
    own "unreliable" field instead of decoding it under the wrong latency range and loss draw."""
    if unreliable_flag:
        return True
    if test in MIXED_MODE:
        return None
    return "unreliable" in test


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("test")
    ap.add_argument("--clusters", type=int, default=None, help="seeds (MADSIM_TEST_NUM)")
    ap.add_argument("--seed", type=int, default=None, help="first seed (MADSIM_TEST_SEED)")
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--iters", type=int, default=0)
    ap.add_argument("--unreliable", action="store_true")
    ap.add_argument("--null", action="store_true", help="skeleton node (never campaigns)")
    ap.add_argument("--safety", action="store_true",
                    help="per-event Raft invariant checks (docs/SEMANTICS.md §11)")
    ap.add_argument("--bug", choices=["vote_twice", "vote_stale", "no_prev_check"],
                    help="run a known-buggy Raft variant")
    ap.add_argument("--replay", metavar="LOG", help="JSON-lines decision log (trace.py) to replay")
    a = ap.parse_args()
    flags = 0
    if a.bug:
        flags |= {"vote_twice": _abi.MR_F_BUG_VOTE_TWICE, "vote_stale": _abi.MR_F_BUG_VOTE_STALE,
                  "no_prev_check": _abi.MR_F_BUG_NO_PREV_CHECK}[a.bug]
    if a.replay:
        dec = trace.load_jsonl(a.replay, unreliable=net_mode(a.test, a.unreliable))
        tr, code, tm, misses = sim.replay(a.test, dec, seed=a.seed or _abi.README_SEED,
                                          nodes=a.nodes, iters=a.iters, unreliable=a.unreliable,
                                          null_raft=a.null, safety=a.safety, flags=flags)
        print(json.dumps({"code": code, "verdict": _abi.FAIL_NAMES.get(code, str(code)),
                          "time_us": tm, "events": int(tr.size), "misses": misses}))
        raise SystemExit(0 if code == _abi.MR_PASS else 1)
    t0 = time.time()
    code, _, _, cnt = sim.run_test(a.test, a.seed, a.clusters, nodes=a.nodes, iters=a.iters,
                                   unreliable=a.unreliable, null_raft=a.null, safety=a.safety,
                                   flags=flags)
    cnt["wall_s"] = time.time() - t0
    print(json.dumps(cnt))
    raise SystemExit(0 if cnt["failed"] == 0 else 1)


if __name__ == "__main__":
    main()
