"""Keyed decision traces and replay (docs/SEMANTICS.md §12; SURVEY.md §8b mr_replay, §8f rank 4).

A trace is a SET of decisions keyed by who makes them — (stream, entity, seq): a host's n-th
send (dropped? latency), a server's n-th election timeout, a tester thread's n-th draw — not
by draw position, so a recorder of another simulator's run (a MadSim seed) can emit one. A
recorded trace replays the run exactly in any order; an edited trace (forced drops, other
timeouts and latencies, some records removed) is a different, well-defined run that GPU and
oracle play identically, bit for bit. CPU tests pin the oracle side; GPU tests compare the
HIP path with it.
"""
import numpy as np
import pytest

from madraft_amd import _abi

CAP = 1 << 15  # decisions per cluster (figure_8_unreliable_2c at 200 iterations draws ~5e3)


def _record(oracle, cfg, n):
    with oracle.recording(n, CAP) as (count, rec):
        code, t, dig, _ = oracle.run_batch(cfg, 0, n)
    assert (count <= CAP).all()
    return np.concatenate([rec[k, : int(count[k])] for k in range(n)]), count, code, t, dig


def _edit(d, seed=7):
    """Shuffle the records, force every 13th send to be dropped, every 11th election timeout
    to the shortest (150 ms), every 7th latency to 1 ms, and remove every 29th record (its
    draw falls back to the seed's own): a different but well-defined run."""
    rng = np.random.default_rng(seed)
    e = d.copy()
    net = np.nonzero(e["stream"] == _abi.MR_DS_NET)[0]
    e["w0"][net[::13]] = 0
    e["w1"][net[3::7]] = 0
    ele = np.nonzero(e["stream"] == _abi.MR_DS_ELECT)[0]
    e["w0"][ele[::11]] = _abi.decision_word(150_000, 150_000, 300_000)
    keep = np.ones(e.size, bool)
    keep[rng.integers(0, 29)::29] = False
    e = e[keep]
    return e[rng.permutation(e.size)]


def test_decision_word_inverts_the_range_map():
    for lo, hi in [(150_000, 300_000), (1000, 27000), (0, 1000), (0, 2)]:
        for v in [lo, lo + 1, (lo + hi) // 2, hi - 1]:
            w = _abi.decision_word(v, lo, hi)
            assert lo + ((w * (hi - lo)) >> 32) == v
            assert w == 0 or lo + (((w - 1) * (hi - lo)) >> 32) == v - 1


def test_oracle_record_replay_shuffled_roundtrip(oracle):
    cfg = oracle.cfg("figure_8_unreliable_2c", iters=200)
    d, count, code, t, dig = _record(oracle, cfg, 8)
    assert set(np.unique(d["stream"]).tolist()) == {1, 2, 3}
    shuf = d[np.random.default_rng(1).permutation(d.size)]
    with oracle.replaying(shuf, 8) as misses:
        code2, t2, dig2, _ = oracle.run_batch(cfg, 0, 8)
    assert (code2 == code).all() and (t2 == t).all() and (dig2 == dig).all()
    assert (misses == 0).all()
    # a complete trace does not depend on the seed: another seed base plays the same run
    cfg2 = oracle.cfg("figure_8_unreliable_2c", iters=200, seed_base=12345)
    with oracle.replaying(shuf, 8) as misses:
        _, _, dig4, _ = oracle.run_batch(cfg2, 0, 8)
    assert (dig4 == dig).all() and (misses == 0).all()
    with oracle.replaying(_edit(d), 8) as misses:
        _, _, dig3, _ = oracle.run_batch(cfg, 0, 8)
    assert (dig3 != dig).all() and (misses > 0).all()


def test_oracle_empty_trace_is_the_seed_run(oracle):
    cfg = oracle.cfg("initial_election_2a")
    code, t, dig, _ = oracle.run_batch(cfg, 0, 2)
    with oracle.replaying(np.zeros(0, _abi.DECISION_DTYPE), 2) as misses:
        c2, t2, d2, _ = oracle.run_batch(cfg, 0, 2)
    assert (c2 == code).all() and (d2 == dig).all() and (misses > 0).all()


def test_oracle_hand_written_decisions(oracle):
    """Hand-written decisions, as an external recorder would emit them: server 0's first
    election timeout forced to 150 ms, the others' to 299 ms, and every server's first sends
    delivered after exactly 1 ms: server 0 asks for votes at 150 ms, they arrive at 151 ms,
    the grants at 152 ms, and it leads from then on."""
    cfg = oracle.cfg("initial_election_2a")
    d = [(0, _abi.MR_DS_ELECT, 0, 0, _abi.decision_word(150_000, 150_000, 300_000), 0)]
    for i in (1, 2):  # the others time out late
        d.append((0, _abi.MR_DS_ELECT, i, 0, _abi.decision_word(299_000, 150_000, 300_000), 0))
    for src in range(3):
        for k in range(4):
            d.append((0, _abi.MR_DS_NET, src, k, *_abi.net_decision(False, 1000, unreliable=False)))
    dec = np.array(d, _abi.DECISION_DTYPE)
    with oracle.replaying(dec, 1):
        r, tr = oracle.run_cluster(cfg, 0, trace_cap=4096)
    assert r["code"] == 0
    first_leader = tr[tr["role"] == 2][0]
    assert first_leader["node"] == 0 and first_leader["time_us"] == 152_000


@pytest.mark.gpu
def test_gpu_records_the_oracle_decisions(hip, oracle):
    cfg = oracle.cfg("figure_8_unreliable_2c", iters=200)
    n = 64
    with oracle.recording(n, CAP) as (count, rec):
        code, t, dig, _ = oracle.run_batch(cfg, 0, n)
    with hip.Batch("figure_8_unreliable_2c", n, iters=200, flags=_abi.MR_F_RECORD,
                   tape_cap=CAP) as b:
        b.run()
        gc, gt, gd = b.verdicts()
        for k in range(n):
            m, got = b.decisions(k, CAP)
            assert m == count[k]
            assert np.array_equal(got, rec[k, :m]), k  # same decisions, same draw order
    assert (gc == code).all() and (gd == dig).all()


@pytest.mark.gpu
@pytest.mark.parametrize("test,kw", [("figure_8_unreliable_2c", dict(iters=200)),
                                     ("unreliable_3a", {}), ("snapshot_install_unreliable_2d", {})])
def test_gpu_replays_an_edited_shuffled_trace(hip, oracle, test, kw):
    n = 32
    cfg = oracle.cfg(test, **kw)
    d, _, _, _, dig = _record(oracle, cfg, n)
    edited = _edit(d)
    with oracle.replaying(edited, n) as omiss:
        code, t, odig, _ = oracle.run_batch(cfg, 0, n)
    with hip.Batch(test, n, trace_clusters=2, **kw) as b:
        b.set_decisions(edited)
        st = b.run()
        assert st["remaining"] == 0
        gc, gt, gd = b.verdicts()
        tr = [b.trace(k) for k in range(2)]
        gmiss = [b.decisions(k)[0] for k in range(n)]
    assert (gc == code).all() and (gt == t).all() and (gd == odig).all()
    assert gmiss == omiss.tolist()
    assert (odig != dig).any()
    for k in range(2):  # per-node term / role / commit / applied after every event
        with oracle.replaying(edited, n):
            _, otr = oracle.run_cluster(cfg, k, trace_cap=int(cfg.trace_cap))
        assert np.array_equal(tr[k], otr), k


@pytest.mark.gpu
def test_mr_replay_single_cluster(hip, oracle):
    cfg = oracle.cfg("figure_8_unreliable_2c", iters=100)
    d, _, _, _, _ = _record(oracle, cfg, 1)
    edited = _edit(d, seed=3)
    tr, code, tm, misses = hip.replay("figure_8_unreliable_2c", edited, iters=100)
    with oracle.replaying(edited, 1) as omiss:
        r, otr = oracle.run_cluster(cfg, 0, trace_cap=1 << 16)
    assert code == r["code"] and tm == r["time_us"] and misses == omiss[0]
    assert np.array_equal(tr, otr)
