"""GPU parity: the HIP step kernel (through the C ABI) against the CPU oracle.

Bar (integer simulation): bit-exact. Per cluster the verdict code, verdict
time and the FNV-1a digest of the full event trace must equal the oracle's;
for traced clusters every 32-byte trace record (per-node term / role /
commit / applied / last / snapshot index after every event) must be equal;
the batch counters must equal the oracle's sums. At BASELINE sizes the
oracle checks a seeded random subset of clusters, and size-independent
properties cover the rest (every cluster reaches a verdict, verdicts are in
the set the test can produce, counters are self-consistent).
"""
import numpy as np
import pytest

from madraft_amd import _abi

pytestmark = pytest.mark.gpu

SUPPORTED = [n for n in _abi.SCENARIOS if n and n not in _abi.GPU_UNSUPPORTED]
COUNTER_KEYS = ["events", "ev_msg", "ev_timer", "ev_tester", "msgs_sent", "drop_clog",
                "drop_loss", "drop_overflow", "drop_deliver", "drop_stale", "elections",
                "leaders_elected", "applies", "snapshots", "installs", "entries_shipped",
                "max_inflight", "max_log", "max_index", "kv_ops", "kv_checked", "log_writes",
                "kv_lin_checked"]


def first_diff(a, b):
    n = min(len(a), len(b))
    for i in range(n):
        if a[i] != b[i]:
            return i, a[i], b[i]
    return n, (a[n] if n < len(a) else None), (b[n] if n < len(b) else None)


def compare(hip, oracle, test, clusters, traced=4, first=0, oracle_codes=False, **kw):
    with hip.Batch(test, clusters, trace_clusters=traced, cluster_base=first, **kw) as b:
        st = b.run()
        assert st["remaining"] == 0
        code, t, dig = b.verdicts()
        cnt = b.counters()
        traces = [b.trace(k) for k in range(traced)]
        tdigs = [b.trace_digests(k) for k in range(traced)]
        cfg = b.cfg
    ocode, ot, odig, osum = oracle.run_batch(cfg, 0, clusters)
    for k in range(traced):
        _, otr, odg = oracle.run_cluster_dig(cfg, k, int(cfg.trace_cap))
        if not np.array_equal(traces[k], otr):
            i, g, o = first_diff(traces[k], otr)
            pytest.fail(f"{test} cluster {k}: trace differs at record {i}: gpu={g} oracle={o}")
        if not np.array_equal(tdigs[k], odg):
            i = int(np.nonzero(tdigs[k] != odg)[0][0])
            pytest.fail(f"{test} cluster {k}: apply digest differs at record {i}: {traces[k][i]}")
    bad = np.nonzero((code != ocode) | (t != ot) | (dig != odig))[0]
    assert bad.size == 0, (f"{test}: {bad.size} clusters differ, first {bad[0]}: "
                           f"gpu=({code[bad[0]]},{t[bad[0]]}) oracle=({ocode[bad[0]]},{ot[bad[0]]})")
    for k in COUNTER_KEYS:
        assert cnt[k] == osum[k], (test, k, cnt[k], osum[k])
    assert cnt["done"] == clusters
    return (code, cnt, ocode) if oracle_codes else (code, cnt)


def golden_hist(name):
    """tests/golden/verdict_hist.json (tests/golden/make_verdicts.py): the oracle's verdict
    histogram of a case when the file was written"""
    import json
    import os
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "verdict_hist.json")))
    return next(c for c in gold["cases"] if c["name"] == name)


def hist_of(code):
    vals, cnt = np.unique(code, return_counts=True)
    return {str(int(v)): int(n) for v, n in zip(vals, cnt)}


@pytest.mark.parametrize("test", SUPPORTED)
def test_scenario_bit_exact(hip, oracle, test):
    """Every scenario GPU == oracle (verdicts, times, digests, traces, counters) on 256 seeds,
    and the verdict histogram equal to the committed one: a change that costs liveness (or
    passes what used to fail) on both sides at once is visible (verdict r4 item 2)."""
    code, _ = compare(hip, oracle, test, 256)
    assert hist_of(code) == golden_hist(test)["hist"]


def test_config2_verdict_histogram(hip):
    """BASELINE config 2's shape over 8 192 seeds on the HIP path alone: 122 clusters end
    ONE_NO_AGREEMENT, every one explained from its trace in DESIGN.md §6.11 (a new leader that
    cannot commit the command's earlier-term entry, or a deposed leader that accepted it: the
    test calls one(.., retry = false) under message loss, tests.rs:146-150, tester.rs:254-255)."""
    g = golden_hist("fail_agree_2b@5u")
    with hip.Batch(g["test"], g["clusters"], **g["kw"]) as b:
        b.run()
        code, _, _ = b.verdicts()
    assert hist_of(code) == g["hist"]


def test_null_node_kat(hip, oracle):
    """Skeleton KAT on the GPU: README.md:44-48 verdict, same as the oracle."""
    code, cnt = compare(hip, oracle, "initial_election_2a", 64, null_raft=True)
    assert (code == 1).all() and cnt["msgs_sent"] == 0
    code, cnt = compare(hip, oracle, "basic_agree_2b", 64, null_raft=True)
    assert (code == 6).all()


@pytest.mark.parametrize("test", ["unreliable_3a", "unreliable_one_key_3a", "snapshot_rpc_3b",
                                  "multi_4a"])
def test_null_service_kat(hip, oracle, test):
    """Skeleton-service KAT on the GPU: kvraft/server.rs:69 / kvraft/client.rs:59 panics,
    same verdicts, times and traces as the oracle."""
    code, cnt = compare(hip, oracle, test, 128, null_raft=True)
    assert np.isin(code, [50, 51]).all() and (code == 50).mean() > 0.8 and cnt["kv_ops"] == 0


def test_fail_agree_5_unreliable(hip, oracle):
    """BASELINE config 2 shape (5 nodes, message drop) at oracle-checkable size."""
    compare(hip, oracle, "fail_agree_2b", 1024, nodes=5, unreliable=True)


def test_snapshot_7_nodes(hip, oracle):
    """BASELINE config 4 shape: 2D InstallSnapshot with partitions, 7 nodes."""
    code, cnt = compare(hip, oracle, "snapshot_install_unreliable_2d", 256, nodes=7)
    assert cnt["installs"] > 0 and cnt["snapshots"] > 0


@pytest.mark.parametrize("test", ["figure_8_unreliable_2c", "many_partitions_many_clients_3a",
                                  "snapshot_unreliable_3b", "unreliable_churn_2c"])
def test_eight_servers(hip, oracle, test):
    """MR_MAX_NODES = 8 servers (the NB = 8 kernel instances) on scenarios built for 5."""
    kw = {"iters": 200} if test == "figure_8_unreliable_2c" else {}
    # a few 8-server partition runs never settle: the event cap ends them alike on both sides
    compare(hip, oracle, test, 128, traced=2, nodes=8, max_events=200000, **kw)


@pytest.mark.parametrize("test", ["persist_partition_unreliable_linearizable_3a",
                                  "snapshot_unreliable_recover_concurrent_partition_linearizable_3b"])
def test_linearizable_kv_15_clients_7_servers(hip, oracle, test):
    """generic_test_linearizability (the reference's sketched kvraft/tests.rs:386-390,
    524-528; SEMANTICS §9b): 15 clients with random keys, Appends, Puts and Gets over 7
    unreliable, crashing, partitioned servers; every Get judged by the Put-epoch checker.
    Traced clusters record by record, counters (kv_lin_checked: BASELINE config 5's
    linearizability-check counter) equal to the oracle's."""
    code, cnt = compare(hip, oracle, test, 256, traced=4)
    assert (code == 0).all() and cnt["kv_lin_checked"] > 256 * 100 and cnt["kv_checked"] == 0


def test_kv_unreliable_traced(hip, oracle):
    """BASELINE config 5 shape: 5 servers + 5 clerk threads over the unreliable
    net; traced clusters compared record by record (clerk deliveries, client
    thread segments, server KV events)."""
    code, cnt = compare(hip, oracle, "unreliable_3a", 128, traced=8)
    assert cnt["drop_loss"] > 0 and cnt["applies"] > 0


def test_sharded_cluster_base(hip, oracle):
    """A shard (cluster_base != 0) computes the same seeds as the oracle's global ids."""
    compare(hip, oracle, "figure_8_unreliable_2c", 128, traced=2, first=5000)


def test_small_capacities_fail_identically(hip, oracle):
    """Capacity limits are part of the semantics: tiny rings / slots give the
    same SIM_CAPACITY / overflow verdicts on both sides."""
    compare(hip, oracle, "figure_8_unreliable_2c", 128, log_cap=64, msg_slots=6, ae_max=2)


@pytest.mark.parametrize("test,kw", [
    ("figure_8_unreliable_2c", dict(nodes=7, log_cap=32, msg_slots=12)),
    ("figure_8_unreliable_2c", dict(nodes=7, log_cap=64, flags=_abi.MR_F_SAFETY)),
    ("figure_8_unreliable_2c", dict(nodes=8, flags=_abi.MR_F_SAFETY | _abi.MR_F_BUG_NO_PREV_CHECK)),
    ("snapshot_install_unreliable_2d", dict(nodes=7))])
def test_cooperative_append_receive(hip, oracle, monkeypatch, test, kw):
    """The cooperative AppendEntries receive of the 7- / 8-server step kernels (a payload's
    entries after the first batch spread over the wave; the pool kernels and the 3- / 5-server
    step kernels receive sequentially): full 16-entry
    payloads hitting a tiny log ring (SIM_CAPACITY part-way through the spread entries,
    write-guard materializations), MR_F_SAFETY log matching, a Raft without the prev check
    (whose logs diverge) and snapshot compaction under the spread — all equal to the oracle's
    sequential walk, and the spread path taken (coop_entries, ABI 4). The step kernel is forced
    (MR_POOL=0): since round 6 the 2D bodies at 7 servers run on the Raft pool."""
    monkeypatch.setenv("MR_POOL", "0")
    code, cnt = compare(hip, oracle, test, 512, traced=3, **kw)
    assert cnt["log_writes"] > 0 and cnt["coop_entries"] > 0


def test_step_budget_independence(hip):
    """Results do not depend on how many events one launch processes."""
    with hip.Batch("figure_8_unreliable_2c", 512) as b:
        b.run()
        ref = b.verdicts()
        b.reset(b.cfg.seed_base)
        while b.run(max_events=97)["remaining"]:
            pass
        got = b.verdicts()
    for a, c in zip(ref, got):
        assert np.array_equal(a, c)


@pytest.mark.parametrize("lanes,stream", [(1000, False), (1000, True), (64, True)])
def test_lanes_chunks_and_streaming(hip, oracle, lanes, stream):
    """Results do not depend on how many clusters are in flight: chunks of `lanes` clusters
    one after another, or `lanes` streaming lanes that each take the next unstarted cluster
    when theirs ends (mr_cfg.lanes, MR_F_STREAM) equal one lane per cluster and the oracle,
    also when a launch's budget ends mid-way (max_events)."""
    code, cnt = compare(hip, oracle, "figure_8_unreliable_2c", 2500, traced=3, iters=200,
                        lanes=lanes, stream=stream)
    with hip.Batch("figure_8_unreliable_2c", 2500, iters=200) as b:
        b.run()
        ref = b.verdicts()
    with hip.Batch("figure_8_unreliable_2c", 2500, iters=200, lanes=lanes, stream=stream) as b:
        while b.run(max_events=3001)["remaining"]:
            pass
        got = b.verdicts()
        assert b.counters()["done"] == 2500
    for a_, c_ in zip(ref, got):
        assert np.array_equal(a_, c_)


def test_streaming_after_set_decisions(hip):
    """A streaming batch whose decision table is set and dropped keeps its held-cluster lists
    (they were freed with the decision table, then written by the next launch)."""
    with hip.Batch("figure_8_unreliable_2c", 700, iters=100) as b:
        b.run()
        ref = b.verdicts()
    with hip.Batch("figure_8_unreliable_2c", 700, iters=100, lanes=128, stream=True) as b:
        b.set_decisions(None)
        for _ in range(2):  # a launch, then another set + drop between launches of one run
            b.run(max_events=2001)
            b.set_decisions(None)
        while b.run(max_events=2001)["remaining"]:
            pass
        got = b.verdicts()
        assert b.counters()["done"] == 700
    for a_, c_ in zip(ref, got):
        assert np.array_equal(a_, c_)


@pytest.mark.parametrize("lpw", [64, 32, 16])
@pytest.mark.parametrize("test,kw", [("figure_8_unreliable_2c", dict(iters=200)),
                                     ("fail_agree_2b", dict(nodes=5, unreliable=True)),
                                     ("unreliable_3a", {})])
def test_lanes_per_wave(hip, oracle, test, kw, lpw):
    """Half- and quarter-full waves (mr_cfg.lanes_per_wave: a small batch spread over more
    waves) give the oracle's results; so does the automatic choice."""
    compare(hip, oracle, test, 700, traced=2, lanes_per_wave=lpw, **kw)
    with hip.Batch(test, 700, **kw) as b:  # auto: 700 clusters fill far less than half
        b.run()
        auto = b.verdicts()
    with hip.Batch(test, 700, lanes_per_wave=lpw, **kw) as b:
        b.run()
        got = b.verdicts()
    for a_, c_ in zip(auto, got):
        assert np.array_equal(a_, c_)


@pytest.mark.parametrize("test,clusters,kw", [
    ("fail_agree_2b", 65536, dict(nodes=5, unreliable=True)),     # BASELINE config 2
    ("figure_8_unreliable_2c", 131072, {}),                        # config 3, one GPU's shard
    ("figure_8_unreliable_2c", 131072, dict(safety=True)),         # ... as bench.py times it
    # config 3 read literally: crash1 / start1 + persister (tests.rs:612-660) in
    # figure_8_unreliable's loop (tests.rs:688-741), one GPU's shard
    ("figure_8_unreliable_crash", 131072, dict(safety=True)),
    ("snapshot_install_unreliable_2d", 262144, dict(nodes=7)),     # config 4: 256K 7-node / GPU
    ("unreliable_3a", 65536, {}),                                  # config 5: kvraft clerks
])
def test_baseline_sizes(hip, oracle, test, clusters, kw):
    with hip.Batch(test, clusters, **kw) as b:
        st = b.run()
        code, t, dig = b.verdicts()
        cnt = b.counters()
        cfg = b.cfg
    assert st["remaining"] == 0 and cnt["done"] == clusters
    assert (code != _abi.MR_RUNNING).all()
    assert cnt["events"] == cnt["ev_msg"] + cnt["ev_timer"] + cnt["ev_tester"]
    assert sum(cnt["fail_hist"].values()) == clusters
    assert cnt["drop_overflow"] == 0 and (code < 60).all()  # no simulator limits hit
    rng = np.random.default_rng(clusters)
    for k in rng.choice(clusters, 48, replace=False):
        oc, ot, od, _ = oracle.run_batch(cfg, int(k), 1)
        assert (oc[0], ot[0], od[0]) == (code[k], t[k], dig[k]), (test, int(k))


@pytest.mark.parametrize("test", ["figure_8_unreliable_2c", "figure_8_unreliable_crash"])
def test_config3_one_million_on_one_gpu(hip, oracle, test):
    """BASELINE config 3's whole job — 1,048,576 clusters of figure_8_unreliable_2c, which the
    driver shards over 8 GPUs (131,072 each), and config 3 read literally (crash1 / start1 +
    persister, tests.rs:612-660, in figure_8_unreliable's loop) — run on ONE MI355X, streaming
    through the resident pools: every cluster reaches a
    verdict, no simulator capacity is hit, and 64 sampled clusters equal the oracle (verdict,
    time, trace digest)."""
    n = 1 << 20
    with hip.Batch(test, n, safety=True) as b:
        st = b.run()
        code, t, dig = b.verdicts()
        cnt = b.counters()
        cfg = b.cfg
    assert st["remaining"] == 0 and cnt["done"] == n and (code != _abi.MR_RUNNING).all()
    assert cnt["drop_overflow"] == 0 and not (code >= 60).any()  # no simulator limit
    assert not np.isin(code, [42, 43, 49]).any()  # no Raft safety violation
    assert sum(cnt["fail_hist"].values()) == n
    rng = np.random.default_rng(n)
    for k in rng.choice(n, 64, replace=False):
        oc, ot, od, _ = oracle.run_batch(cfg, int(k), 1)
        assert (oc[0], ot[0], od[0]) == (code[k], t[k], dig[k]), int(k)


@pytest.mark.parametrize("test,flags", [
    ("figure_8_unreliable_2c", _abi.MR_F_SAFETY),
    ("unreliable_3a", _abi.MR_F_SAFETY),
    ("many_election_2a", _abi.MR_F_SAFETY | _abi.MR_F_BUG_VOTE_TWICE),
    ("figure_8_2c", _abi.MR_F_SAFETY | _abi.MR_F_BUG_VOTE_STALE),
    ("rejoin_2b", _abi.MR_F_SAFETY | _abi.MR_F_BUG_NO_PREV_CHECK),
])
def test_safety_checks_bit_exact(hip, oracle, test, flags):
    """MR_F_SAFETY checks (and the buggy-Raft variants they catch) on the GPU:
    same verdicts, times and traces as the oracle."""
    code, _ = compare(hip, oracle, test, 512, flags=flags)
    if flags & (_abi.MR_F_BUG_VOTE_TWICE | _abi.MR_F_BUG_VOTE_STALE | _abi.MR_F_BUG_NO_PREV_CHECK):
        assert (code != 0).sum() >= 10
    else:
        assert not np.isin(code, [42, 43, 49]).any()


# floor: the oracle's count on these 256 seeds when written (246 / 256 / 256 / 24 / 256 / 256),
# rounded down, so a checker weakened on both sides at once still fails the test
@pytest.mark.parametrize("test,kw,floor", [
    ("figure_8_unreliable_2c", dict(flags=_abi.MR_F_BUG_VOTE_STALE), 200),
    ("figure_8_unreliable_2c", dict(flags=_abi.MR_F_BUG_NO_PREV_CHECK), 200),
    ("snapshot_install_unreliable_2d", dict(flags=_abi.MR_F_BUG_VOTE_STALE), 200),
    ("snapshot_install_unreliable_2d", dict(flags=_abi.MR_F_BUG_VOTE_TWICE, nodes=7), 20),
    ("figure_8_unreliable_2c", dict(apply_cap=64), 200),
    ("snapshot_basic_2d", dict(apply_cap=40), 200),
])
def test_apply_checker_failures_bit_exact(hip, oracle, test, kw, floor):
    """The tester's apply checker (push_and_check, tester.rs:366-396) failing inside the
    cooperative applier (entries of one cluster spread over the wave's lanes): buggy Rafts
    without MR_F_SAFETY commit diverging entries (APPLY_MISMATCH), a tiny apply_cap trips
    the capacity check; verdict, time, trace digest, traced records and counters (applies,
    snapshots, max_index) equal the oracle's sequential walk."""
    code, _, ocode = compare(hip, oracle, test, 256, oracle_codes=True, **kw)
    # the bar is the oracle's own count on these seeds (compare() already made every verdict
    # equal): the checker must have caught something for the test to mean anything
    caught = int(np.isin(ocode, [8, 9, 60]).sum())
    assert caught >= floor and int(np.isin(code, [8, 9, 60]).sum()) == caught


# floor: the oracle's count on these 256 seeds when written (256 / 256 / 255 / 76 / 256 / 121)
@pytest.mark.parametrize("test,flags,floor", [
    ("unreliable_3a", _abi.MR_F_BUG_NO_DEDUP, 200),
    ("unreliable_one_key_3a", _abi.MR_F_BUG_NO_DEDUP, 200),
    ("persist_partition_unreliable_3a", _abi.MR_F_BUG_STALE_READ, 200),
    ("many_partitions_many_clients_3a", _abi.MR_F_BUG_STALE_READ, 60),
    ("persist_partition_unreliable_linearizable_3a", _abi.MR_F_BUG_NO_DEDUP, 200),
    ("persist_partition_unreliable_linearizable_3a", _abi.MR_F_BUG_STALE_READ, 100),
])
def test_linearizability_checker_bit_exact(hip, oracle, test, flags, floor):
    """SEMANTICS §9a on the GPU: the buggy kvraft servers are caught at the same Get, at the
    same virtual time, with the same traces and counters as the oracle."""
    code, cnt, ocode = compare(hip, oracle, test, 256, oracle_codes=True, flags=flags)
    caught = int((ocode == 52).sum())  # the oracle's own count on these seeds is the bar
    assert caught >= floor and int((code == 52).sum()) == caught and cnt["kv_lin_checked"] > 0


@pytest.mark.parametrize("test", ["figure_8_unreliable_2c", "unreliable_3a"])
def test_coverage_histograms(hip, oracle, test):
    """mr_counters.cov_*: per-cluster leaders elected / events in log2 buckets, equal to the
    histograms of the oracle's per-cluster results."""
    n = 128
    with hip.Batch(test, n) as b:
        b.run()
        cnt = b.counters()
        cfg = b.cfg
    lead, ev = [0] * 16, [0] * 16
    for c in range(n):
        r, _ = oracle.run_cluster(cfg, c)
        lead[_abi.cov_bucket(r["leaders_elected"])] += 1
        ev[_abi.cov_bucket(r["events"])] += 1
    assert cnt["cov_leaders"] == lead and cnt["cov_events"] == ev
    assert sum(lead) == n


def test_golden_fixtures_on_gpu(hip):
    """The committed fixtures (tests/golden/oracle_golden.json) reproduced by the HIP path
    directly — no oracle in the loop: verdicts, verdict times, trace digests, event counts."""
    import json
    import os
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.json")))
    for case in gold["cases"]:
        kw = dict(case["cfg"])  # the same overrides as the oracle's cfg (n_nodes set as is)
        with hip.Batch(case["test"], case["count"], cluster_base=case["first"], **kw) as b:
            b.run()
            code, t, dig = b.verdicts()
            ev = b.counters()["events"]
        assert code.tolist() == case["code"], case["test"]
        assert t.tolist() == case["time_us"], case["test"]
        assert [format(int(d), "016x") for d in dig] == case["digest"], case["test"]
        assert ev == case["events"], case["test"]


@pytest.mark.parametrize("test", ["unreliable_3a", "persist_partition_unreliable_linearizable_3a",
                                  "basic_4a", "figure_8_unreliable_2c"])
def test_pool_and_step_kernels_agree(hip, monkeypatch, test):
    """The pool kernel (Raft-only bodies and, round 5, the kvraft / shard_ctrler ones) and the
    per-lane step kernel (MR_POOL=0) give the same verdicts, times, digests and counters: only
    which lanes run together differs."""
    def run():
        with hip.Batch(test, 256) as b:
            b.run()
            return b.kernel, b.verdicts(), b.counters()
    kp, vp, cp = run()
    monkeypatch.setenv("MR_POOL", "0")
    ks, vs, cs = run()
    assert (kp, ks) == ("pool_kernel", "step_kernel")
    for a, c in zip(vp, vs):
        assert np.array_equal(a, c)
    for k in COUNTER_KEYS:
        assert cp[k] == cs[k], k


@pytest.mark.parametrize("test,kw", [("snapshot_install_unreliable_2d", dict(nodes=7)),
                                     ("snapshot_install_unreliable_crash_2d", dict(nodes=7))])
@pytest.mark.parametrize("rows", [32, 4])
def test_seven_server_pool_agrees_with_step_kernel(hip, monkeypatch, test, kw, rows):
    """Round 6: the 2D bodies at 7 servers (BASELINE config 4) run on the Raft pool, whose LDS
    holds the keys of message slots 0..31 and HBM those of slots 32..63; same verdicts, times,
    digests and counters as the step kernel (all 64 keys in LDS). Config 4 peaks at 28 messages in
    flight per 512 seeds, so the HBM keys are exercised with 4 LDS rows too (MR_KEY_ROWS)."""
    def run():
        with hip.Batch(test, 512, **kw) as b:
            b.run()
            return b.kernel, b.verdicts(), b.counters()
    monkeypatch.setenv("MR_KEY_ROWS", str(rows))
    kp, vp, cp = run()
    monkeypatch.setenv("MR_POOL", "0")
    ks, vs, cs = run()
    assert (kp, ks) == ("pool_kernel", "step_kernel")
    for a, c in zip(vp, vs):
        assert np.array_equal(a, c)
    for k in COUNTER_KEYS:
        assert cp[k] == cs[k], k
    if rows < 32:
        assert cp["max_inflight"] > rows  # slots past the LDS rows were used


def test_pool_workgroup_streaming_counters(hip, monkeypatch):
    """one pool workgroup streams a whole batch (lanes = 512); its 64-bit counter sums
    (D.pcnt, added by reduce_kernel) equal the step kernel's per-cluster counters."""
    def run(lanes):
        with hip.Batch("figure_8_unreliable_2c", 4096, lanes=lanes, iters=40) as b:
            st = b.run()
            return b.kernel, st["launches"], b.verdicts(), b.counters()
    kp, lp, vp, cp = run(512)
    monkeypatch.setenv("MR_POOL", "0")
    ks, _, vs, cs = run(0)
    assert (kp, ks) == ("pool_kernel", "step_kernel")
    for a, c in zip(vp, vs):
        assert np.array_equal(a, c)
    for k in COUNTER_KEYS:
        assert cp[k] == cs[k], k
