"""Raft properties read straight off the event traces — a check that does not go through the
oracle. Parity (tests/test_gpu_parity.py) shows the GPU and the oracle agree; both restate one
docs/SEMANTICS.md, so a misreading common to both would pass it. These properties come from the
Raft paper (Figure 3) and the trace format alone (SEMANTICS §7: after every node event, the
node's role / term / commit / applied / last / snapshot index), and hold for any correct Raft:

* times never go back; a node's term never decreases (it is persisted across crashes);
* election safety: at most one node is leader in a term;
* snapshot <= applied <= commit <= last on a live node;
* without crashes, a node's commit and applied indices never decrease, and its snapshot index
  never decreases either way;
* leader append-only: while a node leads in a term, its last index never decreases;
* leader completeness: a new leader's log reaches every index committed before its election;
* commit quorum: every committed index is within the logs of a majority (check_commit_quorum);
* state-machine safety by value (check_apply_digests): nodes that report the same applied index
  report the same apply digest — the sum of mr_apply_mix(i, command_i) over the entries they
  applied (ABI 4 mr_trace_digests), so two nodes that applied different commands at any index
  up to it disagree.

CPU: oracle traces of many seeds over the BASELINE shapes; GPU: the HIP path's own traces.
"""
import numpy as np
import pytest

from madraft_amd import _abi

R_L, R_DOWN = 2, 3
NO_CRASH = {"figure_8_unreliable_2c", "fail_agree_2b", "basic_agree_2b", "unreliable_3a",
            "snapshot_install_unreliable_2d", "many_partitions_many_clients_3a"}


def check_commit_quorum(tr, n):
    """Leader completeness and the commit quorum, from the traced indices alone (Raft paper
    Figure 3; tester.rs:366-428 checks the same entries by value):

    * a node that becomes leader at time t holds every entry committed before t: its last
      index is at least the largest commit index any node reported before t;
    * a committed entry is on a majority: at every event the largest commit index reported so
      far is at most the majority-th largest last index the nodes last reported.

    A node's traced last can lag its true one only by start() appends on a leader (tester
    events), which only add entries, so both checks hold for a correct Raft on traced values."""
    maj = n // 2 + 1
    last = np.zeros(n, np.int64)
    cmax, prev_t, cmax_before = 0, -1, 0
    lead_term = {}
    node = tr[(tr["cls"] <= 1) & (tr["node"] < n)]
    for ev in node:
        t = int(ev["time_us"])
        if t != prev_t:  # commits reported strictly before this time
            cmax_before, prev_t = cmax, t
        d, term = int(ev["node"]), int(ev["term"])
        last[d] = int(ev["last"])
        if ev["role"] == R_L and term not in lead_term:
            lead_term[term] = d
            assert last[d] >= cmax_before, \
                f"leader {d} of term {term} at t={t} lacks committed index {cmax_before} (last {last[d]})"
        if ev["role"] != R_DOWN:
            cmax = max(cmax, int(ev["commit"]))
        assert np.sort(last)[::-1][maj - 1] >= cmax, \
            f"t={t}: index {cmax} committed but on fewer than {maj} logs: {last.tolist()}"


def check_apply_digests(tr, dg):
    """State-machine safety by value (Raft paper Figure 3): every node that has applied up to
    index a has applied the same commands 1..a, so node records with equal `applied` carry equal
    apply digests (a node that installed a snapshot or restarted above 0 reports none). Returns
    the number of (applied index) groups with two or more records compared."""
    node = (tr["cls"] <= 1) & (tr["node"] < 8) & (dg != _abi.DIGEST_INVALID)
    seen, compared = {}, set()
    for ev, d in zip(tr[node], dg[node]):
        a = int(ev["applied"])
        if a in seen:
            assert seen[a] == int(d), f"t={int(ev['time_us'])}: node {int(ev['node'])} applied 1..{a} with other commands"
            compared.add(a)
        else:
            seen[a] = int(d)
    assert seen.get(0, 0) == 0, "an empty applied prefix has digest 0"
    return len(compared)


def check_trace(tr, test, n=None):
    assert (np.diff(tr["time_us"].astype(np.int64)) >= 0).all(), "time went back"
    node = tr[(tr["cls"] <= 1) & (tr["node"] < 8)]  # node events (messages, timers)
    leaders = {}
    for d in np.unique(node["node"]):
        r = node[node["node"] == d]
        assert (np.diff(r["term"].astype(np.int64)) >= 0).all(), f"node {d}: term decreased"
        live = r[r["role"] != R_DOWN]
        assert (live["snap"] <= live["applied"]).all(), f"node {d}: applied below the snapshot"
        assert (live["applied"] <= live["commit"]).all(), f"node {d}: applied beyond commit"
        assert (live["commit"] <= live["last"]).all(), f"node {d}: commit beyond the log"
        assert (np.diff(r["snap"].astype(np.int64)) >= 0).all(), f"node {d}: snapshot went back"
        if test in NO_CRASH:
            assert (np.diff(r["commit"].astype(np.int64)) >= 0).all(), f"node {d}: commit went back"
            assert (np.diff(r["applied"].astype(np.int64)) >= 0).all(), f"node {d}: applied went back"
        for t in np.unique(r["term"][r["role"] == R_L]):
            assert leaders.setdefault(int(t), int(d)) == int(d), f"two leaders in term {t}"
            led = r[(r["role"] == R_L) & (r["term"] == t)]
            assert (np.diff(led["last"].astype(np.int64)) >= 0).all(), \
                f"node {d}: leader of term {t} removed entries"
    if n:
        check_commit_quorum(tr, n)
    return len(leaders)


CASES = [("figure_8_unreliable_2c", {}), ("figure_8_unreliable_crash", {}),
         ("fail_agree_2b", dict(n_nodes=5, flags=_abi.MR_F_UNRELIABLE)),
         ("snapshot_install_unreliable_2d", dict(n_nodes=7)), ("unreliable_3a", {}),
         ("persist_partition_unreliable_linearizable_3a", {}), ("unreliable_churn_2c", {})]


@pytest.mark.parametrize("test,kw", CASES)
def test_oracle_traces_hold_raft_properties(oracle, test, kw):
    terms = groups = 0
    for c in range(24):
        cfg = oracle.cfg(test, **kw)
        r, tr, dg = oracle.run_cluster_dig(cfg, c, 1 << 17)
        assert tr[-1]["cls"] == 3 and tr[-1]["kind"] == r["code"], "trace truncated"
        terms += check_trace(tr, test, int(cfg.n_nodes))
        groups += check_apply_digests(tr, dg)
    assert terms > 24  # leaders were elected: the properties had something to hold for
    assert groups > 24  # applied prefixes were compared by value


@pytest.mark.gpu
@pytest.mark.parametrize("test,kw", CASES)
def test_gpu_traces_hold_raft_properties(hip, test, kw):
    kw = {("nodes" if k == "n_nodes" else k): v for k, v in kw.items()}
    if "flags" in kw and kw["flags"] & _abi.MR_F_UNRELIABLE:
        kw.pop("flags")
        kw["unreliable"] = True
    with hip.Batch(test, 64, trace_clusters=16, trace_cap=1 << 17, **kw) as b:
        b.run()
        traces = [b.trace(k) for k in range(16)]
        digests = [b.trace_digests(k) for k in range(16)]
        n = int(b.cfg.n_nodes)
    assert all(tr[-1]["cls"] == 3 for tr in traces)  # complete: each ends with its verdict
    assert sum(check_trace(tr, test, n) for tr in traces) > 16
    assert sum(check_apply_digests(tr, dg) for tr, dg in zip(traces, digests)) > 16


@pytest.mark.gpu
@pytest.mark.parametrize("test,clusters,kw", [
    ("figure_8_unreliable_2c", 131072, dict(safety=True)),     # config 3, one GPU's shard
    ("figure_8_unreliable_crash", 131072, dict(safety=True)),  # ... crash-restart + persister
    ("snapshot_install_unreliable_2d", 262144, dict(nodes=7)),  # config 4
    ("unreliable_3a", 65536, {}),                                # config 5: kvraft servers
])
def test_gpu_traces_at_baseline_size(hip, test, clusters, kw):
    """The same properties on traces taken from a BASELINE-size run: 48 clusters spread over
    the batch (cluster_base shards of the full job, each traced whole) keep every property."""
    terms = groups = 0
    for first in (0, clusters // 2, clusters - 16):
        with hip.Batch(test, 16 if first else clusters, cluster_base=first, trace_clusters=16,
                       trace_cap=1 << 17, **kw) as b:
            b.run()
            traces = [b.trace(k) for k in range(16)]
            digests = [b.trace_digests(k) for k in range(16)]
            n = int(b.cfg.n_nodes)
        assert all(tr[-1]["cls"] == 3 for tr in traces)
        terms += sum(check_trace(tr, test, n) for tr in traces)
        groups += sum(check_apply_digests(tr, dg) for tr, dg in zip(traces, digests))
    assert terms > 48 and groups > 48


@pytest.mark.parametrize("test,bug,check,floor", [
    ("many_election_2a", _abi.MR_F_BUG_VOTE_TWICE, "all", 20),
    ("figure_8_unreliable_2c", _abi.MR_F_BUG_VOTE_STALE, "all", 20),
    ("figure_8_unreliable_2c", _abi.MR_F_BUG_VOTE_STALE, "quorum", 10),
    ("figure_8_2c", _abi.MR_F_BUG_VOTE_STALE, "quorum", 20)])
def test_trace_properties_catch_buggy_raft(oracle, test, bug, check, floor):
    """The trace checks are not vacuous: a Raft that votes twice in a term (or for a stale
    log) elects two leaders in one term on some seeds, and one that votes for a stale log
    elects leaders that lack committed entries (leader completeness); the traces alone show it
    (counts over 64 seeds: 45 / 40 / 26 / 32 when written, floors below them)."""
    caught = 0
    for c in range(64):
        cfg = oracle.cfg(test, flags=bug)
        _, tr = oracle.run_cluster(cfg, c, trace_cap=1 << 17)
        try:
            if check == "quorum":
                check_commit_quorum(tr, int(cfg.n_nodes))
            else:
                check_trace(tr, test, int(cfg.n_nodes))
        except AssertionError:
            caught += 1
    assert caught >= floor


# floors: the counts over 64 seeds when written (64 / 61 / 64), rounded down
@pytest.mark.parametrize("test,bug,floor", [
    ("figure_8_unreliable_2c", _abi.MR_F_BUG_NO_PREV_CHECK, 50),
    ("figure_8_unreliable_2c", _abi.MR_F_BUG_VOTE_STALE, 45),
    ("rejoin_2b", _abi.MR_F_BUG_NO_PREV_CHECK, 40)])
def test_apply_digests_catch_diverging_state_machines(oracle, test, bug, floor):
    """check_apply_digests is not vacuous: with the tester's own value check off
    (MR_F_BUG_NO_APPLY_CHECK, so the run is not stopped at the first APPLY_MISMATCH), a Raft
    without the prevLogTerm check (or voting for stale logs) applies different commands at the
    same index on other nodes, and the digests in the trace alone show it."""
    caught = 0
    for c in range(64):
        cfg = oracle.cfg(test, flags=bug | _abi.MR_F_BUG_NO_APPLY_CHECK)
        _, tr, dg = oracle.run_cluster_dig(cfg, c, 1 << 17)
        try:
            check_apply_digests(tr, dg)
        except AssertionError:
            caught += 1
    assert caught >= floor


@pytest.mark.gpu
@pytest.mark.parametrize("test,bug,floor", [
    ("figure_8_unreliable_2c", _abi.MR_F_BUG_NO_PREV_CHECK, 50),
    ("rejoin_2b", _abi.MR_F_BUG_NO_PREV_CHECK, 40)])
def test_gpu_apply_digests_catch_diverging_state_machines(hip, test, bug, floor):
    """The same on the HIP path's own traces and digests (no oracle in the loop)."""
    with hip.Batch(test, 64, trace_clusters=64, trace_cap=1 << 17,
                   flags=bug | _abi.MR_F_BUG_NO_APPLY_CHECK) as b:
        b.run()
        caught = 0
        for k in range(64):
            try:
                check_apply_digests(b.trace(k), b.trace_digests(k))
            except AssertionError:
                caught += 1
    assert caught >= floor


def test_apply_digest_checker_units():
    """check_apply_digests on hand-made records: equal applied indices with equal digests pass,
    with different ones fail; invalid digests (a snapshot install / restart) are skipped."""
    tr = np.zeros(4, _abi.EVENT_DTYPE)
    tr["cls"] = 0
    tr["node"] = [0, 1, 2, 1]
    tr["applied"] = [3, 3, 5, 5]
    d = _abi.apply_mix(1, 11) + _abi.apply_mix(2, 12) + _abi.apply_mix(3, 13)
    dg = np.array([d & (2**64 - 1), d & (2**64 - 1), 7, _abi.DIGEST_INVALID], np.uint64)
    assert check_apply_digests(tr, dg) == 1
    dg[1] ^= 1
    with pytest.raises(AssertionError):
        check_apply_digests(tr, dg)
