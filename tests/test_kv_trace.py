"""kvraft append order and get == last, checked from the applied command log alone (verdict r4
item 3): no oracle in the loop on the GPU side, and no reuse of the simulator's value model.

mr_trace_applies (ABI 4) gives, per log index i of a traced cluster, the KV command the service
applied there and the hash of its key's value right after the first server to apply i applied it
(a Get: the hash it answered). check_kv_applies replays the commands with real strings — a Put
sets the value, an Append of "x {cli} {j} y" concatenates, a clerk's command is applied once
(kvraft/server.rs:76-87: a request with a sequence number the clerk already had applied is a
duplicate) — and asserts:

* the servers' state machine: the recorded hash is the hash of the replayed value (so a server
  that applies a retried Append twice, or drops one, is caught at that index);
* linearizability per clerk: a clerk's calls are sequential (ClerkCore::call,
  kvraft/client.rs:49-62), so when its call `seq` is in the log every call 1..seq-1 returned, and
  a call returns only after its command was applied: all of them are at lower indices;
* check_clnt_appends (kvraft/tests.rs:21-43) on every value a Get answered and on every final
  value: each appender's tokens once each, in order, `j = 0..count-1` (the generic_test
  clients); the 15-client linearizable tests draw j from a growing counter, so there only the
  order is checked;
* get == last (kvraft/tests.rs:113-128) where a clerk owns its key (generic_test: client cli
  puts "" to key cli, then appends and gets): the value a Get answers is the clerk's own
  appends with lower sequence numbers, in order.
"""
import numpy as np
import pytest

from madraft_amd import _abi

GET, PUT, APPEND = 0, 1, 2
PHI, HP = 0x9E3779B97F4A7C15, 0x100000001B3
M64 = (1 << 64) - 1
# generic_test bodies: every clerk that appends owns its key (kvraft/tests.rs:65-220, 344-384)
GENERIC = ["basic_3a", "concurrent_3a", "unreliable_3a", "many_partitions_one_client_3a",
           "many_partitions_many_clients_3a", "persist_one_client_3a", "persist_concurrent_3a",
           "persist_concurrent_unreliable_3a", "persist_partition_3a",
           "persist_partition_unreliable_3a", "snapshot_recover_3b",
           "snapshot_recover_many_clients_3b", "snapshot_unreliable_3b",
           "snapshot_unreliable_recover_3b", "snapshot_unreliable_recover_concurrent_partition_3b"]
OTHER = ["unreliable_one_key_3a", "one_partition_3a", "snapshot_rpc_3b", "snapshot_size_3b"]


def decode(v):
    """SEMANTICS §9 log command: bit 63, op at 61, key at 55, clerk at 48, seq at 24, elem."""
    return ((v >> 61) & 3, (v >> 55) & 63, (v >> 48) & 127, (v >> 24) & 0xFFFFFF, v & 0xFFFFFF)


def put_string(t):
    """a Put value token: 0 = "", t < 2^20 = the decimal string of t - 1, else one letter"""
    return "" if t == 0 else str(t - 1) if t < (1 << 20) else "abcdefghijklmnopqrstuvwxyz"[t % 26]


def app_string(e):
    return f"x {e >> 19} {e & 0x7FFFF} y"


class Value:
    """a key's value as the real string plus its token list; `h` is the value hash of
    docs/SEMANTICS.md §9 over those tokens (a Put token t, then h · HP + elem + 1 per Append)"""

    def __init__(self):
        self.s, self.apps, self.h = "", [], 0

    def put(self, t, lin15):
        if lin15:  # §9b: a Put of token "x cli j y": "" then the token
            self.s, self.apps, self.h = app_string(t), [t], t + 1
        else:
            self.s, self.apps = put_string(t), []
            self.h = (t + 1) * PHI & M64 if t else 0

    def append(self, e):
        self.s += app_string(e)
        self.apps.append(e)
        self.h = (self.h * HP + e + 1) & M64


def check_clnt_appends(cli, v, count):
    """kvraft/tests.rs:21-43 on the real string"""
    last = -1
    for j in range(count):
        wanted = f"x {cli} {j} y"
        off = v.find(wanted)
        assert off >= 0, f"{cli} missing element {wanted!r} in Append result {v!r}"
        assert v.rfind(wanted) == off, f"duplicate element {wanted!r} in Append result"
        assert off > last, f"wrong order for element {wanted!r} in Append result"
        last = off


def check_value(val, consecutive):
    by_cli = {}
    for e in val.apps:
        by_cli.setdefault(e >> 19, []).append(e & 0x7FFFF)
    for cli, js in by_cli.items():
        if consecutive:
            check_clnt_appends(cli, val.s, len(js))
            assert js == list(range(len(js))), f"appender {cli}: tokens {js[:8]}..."
        else:
            assert all(a < b for a, b in zip(js, js[1:])), f"appender {cli} out of order: {js}"


def check_kv_applies(ap, lin15=False, owned=False):
    """See the module docstring. ap: [n, 2] (command, key hash after it) by log index. Returns
    (Gets checked, commands replayed)."""
    vals, ded = {}, {}
    got, low = {}, {}  # clerk -> its sequence numbers in the log so far, the lowest one absent
    owner = {}  # key -> (clerk, [(seq, elem) of its Appends]) while one clerk owns the key
    gets = 0
    for i in range(1, len(ap)):
        v, h = int(ap[i, 0]), int(ap[i, 1])
        assert v >> 63, f"log index {i} was not applied by any server"
        op, key, clerk, seq, elem = decode(v)
        if lin15:
            key &= 15
        val = vals.setdefault(key, Value())
        assert low.get(clerk, 1) >= seq, (f"index {i}: clerk {clerk} call {seq} is in the log, its "
                                          f"call {low.get(clerk, 1)} is not")
        if op == GET:
            check_value(val, not lin15)
            own = owner.get(key)
            if owned and own and own[0] == clerk:  # get == last
                last = [e for q, e in sorted(own[1]) if q < seq]
                assert val.apps == last, f"index {i}: get != last for clerk {clerk}"
            gets += 1
        elif seq > ded.get(clerk, 0):
            if op == PUT:
                val.put(elem, lin15)
                owner[key] = (clerk, [])
            else:
                val.append(elem)
                if key in owner and owner[key][0] == clerk:
                    owner[key][1].append((seq, elem))
                else:
                    owner.pop(key, None)
            ded[clerk] = seq
        g = got.setdefault(clerk, set())
        g.add(seq)
        q = low.get(clerk, 1)
        while q in g:
            q += 1
        low[clerk] = q
        assert h == val.h, (f"index {i}: the servers' value hash {h:#x} is not the replayed "
                            f"value's {val.h:#x} ({['get', 'put', 'append'][op]} by clerk {clerk} seq {seq})")
    for val in vals.values():
        check_value(val, not lin15)
    return gets, len(ap) - 1


CASES = [(t, {}) for t in GENERIC + OTHER] + [(t, {}) for t in _abi.LIN_TESTS]


@pytest.mark.parametrize("test,kw", CASES[:6] + [c for c in CASES if c[0] in OTHER + _abi.LIN_TESTS])
def test_oracle_kv_applies_hold(oracle, test, kw):
    """The oracle's applied command logs pass the replay (the checker against the build's own
    restatement; the GPU test below holds the HIP path to it without the oracle)."""
    gets = cmds = 0
    for c in range(6):
        cfg = oracle.cfg(test, **kw)
        r, tr, ap = oracle.run_cluster_kv(cfg, c, 1 << 17)
        assert tr[-1]["cls"] == 3
        g, n = check_kv_applies(ap, test in _abi.LIN_TESTS, test in GENERIC)
        gets += g
        cmds += n
    assert cmds > 20 and (gets > 5 or test in ("snapshot_size_3b",))


# floors: the counts over 48 seeds when written (48, 48), rounded down
@pytest.mark.parametrize("test,floor", [("unreliable_3a", 40), ("persist_concurrent_unreliable_3a", 40)])
def test_kv_replay_catches_duplicate_appends(oracle, test, floor):
    """The replay is not vacuous: servers without the duplicate check (MR_F_BUG_NO_DEDUP) apply
    retried Appends twice under message loss, and the recorded hashes show it."""
    caught = 0
    for c in range(48):
        cfg = oracle.cfg(test, flags=_abi.MR_F_BUG_NO_DEDUP)
        _, _, ap = oracle.run_cluster_kv(cfg, c, 1 << 17)
        try:
            check_kv_applies(ap, False, True)
        except AssertionError:
            caught += 1
    assert caught >= floor


@pytest.mark.gpu
@pytest.mark.parametrize("test", GENERIC + OTHER + _abi.LIN_TESTS)
def test_gpu_kv_applies_hold(hip, oracle, test):
    """The HIP path's applied command logs pass the replay, and equal the oracle's."""
    with hip.Batch(test, 16, trace_clusters=8, trace_cap=1 << 17) as b:
        b.run()
        aps = [b.trace_applies(k) for k in range(8)]
        cfg = b.cfg
    cmds = 0
    for k, ap in enumerate(aps):
        cmds += check_kv_applies(ap, test in _abi.LIN_TESTS, test in GENERIC)[1]
        _, _, oap = oracle.run_cluster_kv(cfg, k, 1 << 17)
        assert np.array_equal(ap, oap), f"{test} cluster {k}: applied commands differ from the oracle's"
    assert cmds > 20


@pytest.mark.gpu
def test_gpu_kv_applies_at_baseline_size(hip):
    """BASELINE config 5 (unreliable_3a) at its bench batch: sampled clusters across the batch
    through the replay, HIP path only."""
    cmds = 0
    clusters = 32768
    for first in (0, clusters // 2, clusters - 8):
        with hip.Batch("unreliable_3a", 8 if first else clusters, cluster_base=first,
                       trace_clusters=8, trace_cap=1 << 17) as b:
            b.run()
            aps = [b.trace_applies(k) for k in range(8)]
        cmds += sum(check_kv_applies(ap, False, True)[1] for ap in aps)
    assert cmds > 24 * 20


@pytest.mark.gpu
def test_gpu_kv_replay_catches_duplicate_appends(hip):
    with hip.Batch("unreliable_3a", 48, trace_clusters=48, trace_cap=1 << 17,
                   flags=_abi.MR_F_BUG_NO_DEDUP) as b:
        b.run()
        caught = 0
        for k in range(48):
            try:
                check_kv_applies(b.trace_applies(k), False, True)
            except AssertionError:
                caught += 1
    assert caught >= 40


def _cmd(op, key, clerk, seq, elem):
    """a SEMANTICS §9 log command"""
    return (1 << 63) | (op << 61) | (key << 55) | (clerk << 48) | (seq << 24) | elem


def _log(cmds, bad_hash_at=None):
    """[n, 2] applies of `cmds` (indices 1..) with the hashes a correct server reports"""
    ap = np.zeros((len(cmds) + 1, 2), np.uint64)
    vals, ded = {}, {}
    for i, c in enumerate(cmds, 1):
        op, key, clerk, seq, elem = decode(c)
        v = vals.setdefault(key, Value())
        if op != GET and seq > ded.get(clerk, 0):
            v.put(elem, False) if op == PUT else v.append(elem)
            ded[clerk] = seq
        ap[i] = (c, v.h if i != bad_hash_at else v.h ^ 1)
    return ap


def test_kv_replay_checker_units():
    """The replay on hand-made logs: a generic_test client (clerk 3, key 0: Put "", Appends of
    "x 0 j y", Gets) passes; a dropped dedup, an append out of order, a call before its
    predecessor and a wrong server hash each fail."""
    ok = [_cmd(PUT, 0, 3, 1, 0), _cmd(APPEND, 0, 3, 2, 0), _cmd(APPEND, 0, 3, 3, 1),
          _cmd(APPEND, 0, 3, 3, 1),  # a retried Append: a duplicate the servers skip
          _cmd(GET, 0, 3, 4, 0), _cmd(APPEND, 0, 3, 5, 2), _cmd(GET, 0, 3, 6, 0)]
    assert check_kv_applies(_log(ok), False, True) == (2, 7)
    with pytest.raises(AssertionError):  # the server reports the retried Append applied twice
        ap = _log(ok)
        v = Value()
        v.put(0, False)
        for e in (0, 1, 1):
            v.append(e)
        ap[4, 1] = v.h
        check_kv_applies(ap, False, True)
    with pytest.raises(AssertionError):  # "x 0 1 y" before "x 0 0 y"
        check_kv_applies(_log([_cmd(PUT, 0, 3, 1, 0), _cmd(APPEND, 0, 3, 2, 1), _cmd(APPEND, 0, 3, 3, 0)]),
                         False, True)
    with pytest.raises(AssertionError):  # call 3 in the log before call 2
        check_kv_applies(_log([_cmd(PUT, 0, 3, 1, 0), _cmd(APPEND, 0, 3, 3, 0)]), False, True)
    with pytest.raises(AssertionError):  # a server hash that is not the replayed value's
        check_kv_applies(_log(ok, bad_hash_at=5), False, True)
