"""Decision tapes and replay (docs/SEMANTICS.md §12; SURVEY.md §8b mr_replay, §8f rank 4).

A tape is a cluster's random draws in order (two words per draw). Recording a run and replaying
its tape reproduces the run; an edited tape (a forced drop, a different timeout) drives GPU and
oracle to the same new run, bit for bit — the path a recorder of another simulator's decisions
would take. CPU tests pin the oracle side; GPU tests compare the HIP path with it.
"""
import numpy as np
import pytest

from madraft_amd import _abi

W = 1 << 16  # words per cluster (figure_8_unreliable_2c draws ~2.4e4)


def _record(oracle, cfg, n):
    tape = np.zeros((n, W), np.uint32)
    with oracle.with_tape(tape, 2) as used:
        code, t, dig, _ = oracle.run_batch(cfg, 0, n)
    assert (used <= W).all()
    return tape, used, code, t, dig


def _edit(tape, used, seed=7):
    """Force every 97th draw's first word to 0 (a drop where it decides loss, the shortest
    timeout / latency where it decides those) — a different but valid decision stream."""
    rng = np.random.default_rng(seed)
    t = tape.copy()
    for k in range(t.shape[0]):
        idx = np.arange(int(rng.integers(0, 97)) * 2, int(used[k]), 97 * 2)
        t[k, idx] = 0
    return t


def test_oracle_record_replay_roundtrip(oracle):
    cfg = oracle.cfg("figure_8_unreliable_2c", iters=200)
    tape, used, code, t, dig = _record(oracle, cfg, 8)
    with oracle.with_tape(tape, 1) as used2:
        code2, t2, dig2, _ = oracle.run_batch(cfg, 0, 8)
    assert (code2 == code).all() and (t2 == t).all() and (dig2 == dig).all()
    assert (used2 == used).all()
    edited = _edit(tape, used)
    with oracle.with_tape(edited, 1):
        _, _, dig3, _ = oracle.run_batch(cfg, 0, 8)
    assert (dig3 != dig).all()
    # a tape does not depend on the seed: replay under another seed base is the same run
    cfg2 = oracle.cfg("figure_8_unreliable_2c", iters=200, seed_base=12345)
    with oracle.with_tape(tape, 1):
        _, _, dig4, _ = oracle.run_batch(cfg2, 0, 8)
    assert (dig4 == dig).all()


def test_oracle_tape_end_reads_zero(oracle):
    cfg = oracle.cfg("initial_election_2a")
    short = np.zeros((1, 2), np.uint32)  # one draw, then (0, 0) for ever
    with oracle.with_tape(short, 1) as used:
        c1, _, d1, _ = oracle.run_batch(cfg, 0, 1)
    empty = np.zeros((1, 64), np.uint32)
    with oracle.with_tape(empty, 1):
        c2, _, d2, _ = oracle.run_batch(cfg, 0, 1)
    assert used[0] > 2 and d1[0] == d2[0] and c1[0] == c2[0]


@pytest.mark.gpu
def test_gpu_records_the_oracle_tape(hip, oracle):
    cfg = oracle.cfg("figure_8_unreliable_2c", iters=200)
    tape, used, code, t, dig = _record(oracle, cfg, 64)
    with hip.Batch("figure_8_unreliable_2c", 64, iters=200, flags=_abi.MR_F_RECORD, tape_cap=W) as b:
        b.run()
        gc, gt, gd = b.verdicts()
        for k in range(64):
            n, words = b.tape(k, W)
            assert n == used[k]
            assert np.array_equal(words, tape[k, :n]), k
    assert (gc == code).all() and (gd == dig).all()


@pytest.mark.gpu
@pytest.mark.parametrize("test,kw", [("figure_8_unreliable_2c", dict(iters=200)),
                                     ("unreliable_3a", {}), ("snapshot_install_unreliable_2d", {})])
def test_gpu_replays_an_edited_tape(hip, oracle, test, kw):
    n = 32
    cfg = oracle.cfg(test, **kw)
    tape, used, _, _, dig = _record(oracle, cfg, n)
    edited = _edit(tape, used)
    with oracle.with_tape(edited, 1):
        code, t, odig, _ = oracle.run_batch(cfg, 0, n)
    with hip.Batch(test, n, trace_clusters=2, **kw) as b:
        b.set_tape(edited)
        st = b.run()
        assert st["remaining"] == 0
        gc, gt, gd = b.verdicts()
        tr = [b.trace(k) for k in range(2)]
    assert (gc == code).all() and (gt == t).all() and (gd == odig).all()
    assert (odig != dig).any()
    for k in range(2):  # per-node term / role / commit / applied after every event
        with oracle.with_tape(edited, 1):
            _, otr = oracle.run_cluster(cfg, k, trace_cap=int(cfg.trace_cap))
        assert np.array_equal(tr[k], otr), k


@pytest.mark.gpu
def test_mr_replay_single_cluster(hip, oracle):
    cfg = oracle.cfg("figure_8_unreliable_2c", iters=100)
    tape, used, _, _, _ = _record(oracle, cfg, 1)
    edited = _edit(tape, used, seed=3)[0, : int(used[0])]
    tr, code, tm = hip.replay("figure_8_unreliable_2c", edited, iters=100)
    row = np.zeros((1, W), np.uint32)
    row[0, : edited.size] = edited
    with oracle.with_tape(row, 1):
        r, otr = oracle.run_cluster(cfg, 0, trace_cap=1 << 16)
    assert code == r["code"] and tm == r["time_us"]
    assert np.array_equal(tr, otr)
