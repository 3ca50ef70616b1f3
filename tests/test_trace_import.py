"""Event-level decision logs (madraft_amd/trace.py, docs/SEMANTICS.md §12).

A recorded run written as JSON-lines events (sends with drop / latency, election timeouts,
tester draws, each keyed by host / node / thread and its own count) and read back replays the
same run; hand-written event logs drive a run the way a MadSim-side recorder's output would.
CPU tests use the oracle; the GPU test plays an imported log through mr_replay.
"""
import json

import numpy as np
import pytest

from madraft_amd import _abi, trace

CAP = 1 << 15


def _record(oracle, cfg, n):
    with oracle.recording(n, CAP) as (count, rec):
        code, t, dig, _ = oracle.run_batch(cfg, 0, n)
    return np.concatenate([rec[k, : int(count[k])] for k in range(n)]), code, t, dig


@pytest.mark.parametrize("test,unrel", [("figure_8_unreliable_2c", True), ("basic_agree_2b", False),
                                        ("unreliable_3a", True)])
def test_jsonl_roundtrip_replays_the_run(oracle, tmp_path, test, unrel):
    cfg = oracle.cfg(test, iters=100) if test.startswith("figure") else oracle.cfg(test)
    n = 4
    d, code, t, dig = _record(oracle, cfg, n)
    p = tmp_path / "run.jsonl"
    trace.dump_jsonl(p, d, unreliable=unrel)
    lines = p.read_text().splitlines()
    assert len(lines) == d.size
    kinds = {json.loads(s)["event"] for s in lines}
    assert kinds <= {"send", "election_timeout", "rng"} and "send" in kinds
    back = trace.load_jsonl(p)
    assert np.array_equal(back[["cluster", "stream", "entity", "seq"]], d[["cluster", "stream", "entity", "seq"]])
    # decoded values re-encode to other words with the same meaning: the same run, no misses
    with oracle.replaying(back[np.random.default_rng(0).permutation(back.size)], n) as misses:
        c2, t2, dig2, _ = oracle.run_batch(cfg, 0, n)
    assert (c2 == code).all() and (t2 == t).all() and (dig2 == dig).all()
    assert (misses == 0).all()


def test_raw_words_roundtrip_is_exact(oracle):
    cfg = oracle.cfg("figure_8_unreliable_2c", iters=50)
    d, _, _, _ = _record(oracle, cfg, 2)
    back = trace.decisions_from_events(trace.events_from_decisions(d, raw=True))
    assert np.array_equal(back, d)


def test_hand_written_event_log(oracle, tmp_path):
    """Server 0 times out first (150 ms), the others late; every first message takes 1 ms:
    server 0 leads from t = 152 ms (the same run as test_replay's hand-written decisions)."""
    lines = ["# a hand-written three-server run",
             json.dumps({"event": "election_timeout", "node": 0, "index": 0, "timeout_us": 150000})]
    lines += [json.dumps({"event": "election_timeout", "node": i, "index": 0, "timeout_us": 299000})
              for i in (1, 2)]
    lines += [json.dumps({"event": "send", "host": h, "index": k, "latency_us": 1000,
                          "unreliable": False}) for h in range(3) for k in range(4)]
    p = tmp_path / "hand.jsonl"
    p.write_text("\n".join(lines) + "\n")
    dec = trace.load_jsonl(p)
    cfg = oracle.cfg("initial_election_2a")
    with oracle.replaying(dec, 1):
        r, tr = oracle.run_cluster(cfg, 0, trace_cap=4096)
    assert r["code"] == 0
    first = tr[tr["role"] == 2][0]
    assert first["node"] == 0 and first["time_us"] == 152_000


def test_forced_drop_changes_the_run(oracle):
    cfg = oracle.cfg("figure_8_unreliable_2c", iters=100)
    d, _, _, dig = _record(oracle, cfg, 1)
    ev = trace.events_from_decisions(d, unreliable=True)
    sends = [e for e in ev if e["event"] == "send" and not e["dropped"]]
    for e in sends[:40]:
        e["dropped"] = True
    with oracle.replaying(trace.decisions_from_events(ev), 1) as misses:
        _, _, dig2, _ = oracle.run_batch(cfg, 0, 1)
    assert dig2[0] != dig[0]  # a different run (whose later draws may have no record: misses)


def test_bad_events_are_rejected():
    with pytest.raises(ValueError):
        trace.decisions_from_events([{"event": "crash", "node": 1, "index": 0}])
    with pytest.raises(ValueError):
        trace.decisions_from_events([{"event": "rng", "thread": 70000, "index": 0, "u64": 1}])
    # a decoded send needs its network mode (the line's or the caller's), never a guessed one
    with pytest.raises(ValueError):
        trace.decisions_from_events([{"event": "send", "host": 0, "index": 0, "latency_us": 2000}])
    with pytest.raises(ValueError):  # the reliable net loses nothing (tester.rs:127-137)
        trace.decisions_from_events([{"event": "send", "host": 0, "index": 0, "dropped": True,
                                      "unreliable": False}])
    with pytest.raises(ValueError):
        trace.decisions_from_events([{"event": "send", "host": 0, "index": 0, "unreliable": True}])


def test_send_mode_and_dropped_defaults():
    rel = trace.decisions_from_events([{"event": "send", "host": 1, "index": 2, "latency_us": 9000}],
                                      unreliable=False)
    unr = trace.decisions_from_events([{"event": "send", "host": 1, "index": 2, "latency_us": 9000}],
                                      unreliable=True)
    assert int(rel["w1"][0]) != int(unr["w1"][0])  # the latency word depends on the mode
    assert trace.events_from_decisions(rel, unreliable=False)[0]["latency_us"] == 9000
    dropped = trace.decisions_from_events([{"event": "send", "host": 1, "index": 2, "dropped": True,
                                            "unreliable": True}])
    assert int(dropped["w0"][0]) < _abi.LOSS_Q32


def test_cli_net_mode_defaults_to_the_tests_own():
    """A replayed log whose send lines carry no mode takes the run's: --unreliable, else the
    test body's (reliable for initial_election_2a, unreliable for figure_8_unreliable_2c)."""
    from madraft_amd.__main__ import net_mode
    assert net_mode("initial_election_2a", False) is False
    assert net_mode("initial_election_2a", True) is True
    assert net_mode("figure_8_unreliable_2c", False) is True
    line = {"event": "send", "host": 0, "index": 0, "latency_us": 9000}
    rel = trace.decisions_from_events([line], unreliable=net_mode("basic_agree_2b", False))
    assert trace.events_from_decisions(rel, unreliable=False)[0]["latency_us"] == 9000


@pytest.mark.parametrize("test", ["unreliable_agree_2c", "unreliable_churn_2c"])
def test_cli_net_mode_rejects_mixed_mode_logs(test):
    """tests that switch the net back to reliable part-way (tests.rs:680, :832) have
    no single mode, so a send line without its own "unreliable" field is rejected, not decoded
    under the unreliable latency range; lines that carry it, and --unreliable runs, still load."""
    from madraft_amd.__main__ import net_mode
    assert net_mode(test, False) is None
    assert net_mode(test, True) is True
    line = {"event": "send", "host": 0, "index": 0, "latency_us": 9000}
    with pytest.raises(ValueError):
        trace.decisions_from_events([line], unreliable=net_mode(test, False))
    d = trace.decisions_from_events([dict(line, unreliable=False)], unreliable=net_mode(test, False))
    assert trace.events_from_decisions(d, unreliable=False)[0]["latency_us"] == 9000


@pytest.mark.gpu
def test_gpu_replays_an_imported_event_log(hip, oracle, tmp_path):
    cfg = oracle.cfg("figure_8_unreliable_2c", iters=100)
    d, _, _, _ = _record(oracle, cfg, 1)
    ev = trace.events_from_decisions(d, unreliable=True)
    for e in ev[::17]:
        if e["event"] == "send":
            e["latency_us"] = 1000 + (e["latency_us"] * 7) % 26000
    p = tmp_path / "edited.jsonl"
    p.write_text("".join(json.dumps(e) + "\n" for e in ev))
    dec = trace.load_jsonl(p)
    tr, code, tm, misses = hip.replay("figure_8_unreliable_2c", dec, iters=100)
    with oracle.replaying(dec, 1) as om:
        r, otr = oracle.run_cluster(cfg, 0, trace_cap=1 << 16)
    assert code == r["code"] and tm == r["time_us"] and misses == om[0]
    assert np.array_equal(tr, otr)


@pytest.mark.gpu
def test_cli_replays_a_hand_written_log(hip, tmp_path):
    import subprocess
    import sys
    lines = [json.dumps({"event": "election_timeout", "node": i, "index": 0,
                         "timeout_us": 150000 if i == 0 else 299000}) for i in range(3)]
    lines += [json.dumps({"event": "send", "host": h, "index": k, "latency_us": 1000,
                          "unreliable": False}) for h in range(3) for k in range(4)]
    p = tmp_path / "hand.jsonl"
    p.write_text("\n".join(lines) + "\n")
    r = subprocess.run([sys.executable, "-m", "madraft_amd", "initial_election_2a", "--replay", str(p)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["code"] == 0 and out["events"] > 0 and out["misses"] > 0


@pytest.mark.gpu
def test_cli_replays_a_reliable_log_without_modes(hip, tmp_path):
    """The same hand-written run with no per-line "unreliable": the reliable test's own mode
    decodes the sends (the CLI used to reject such a log)."""
    import subprocess
    import sys
    lines = [json.dumps({"event": "election_timeout", "node": i, "index": 0,
                         "timeout_us": 150000 if i == 0 else 299000}) for i in range(3)]
    lines += [json.dumps({"event": "send", "host": h, "index": k, "latency_us": 1000})
              for h in range(3) for k in range(4)]
    p = tmp_path / "hand_rel.jsonl"
    p.write_text("\n".join(lines) + "\n")
    r = subprocess.run([sys.executable, "-m", "madraft_amd", "initial_election_2a", "--replay", str(p)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["code"] == 0 and out["events"] > 0
