"""Event-level decision logs: the keyed decisions of docs/SEMANTICS.md §12 as JSON lines.

A MadSim-side recorder (a patch to madsim's net send, the election-timeout call of a completed
raft.rs and the tests' `rand::rng()`) writes one line per random choice,
keyed by who made it — never by this simulator's event order:

    {"event": "send", "host": 0, "index": 3, "dropped": false, "latency_us": 2300, "unreliable": true}
    {"event": "election_timeout", "node": 2, "index": 0, "timeout_us": 180000}
    {"event": "rng", "thread": 0, "index": 5, "u64": 1234567}

`host` is a server id or `8 + k` for clerk k; `index` counts that host's sends (all
destinations, from 0), that node's election timeouts, or that tester thread's draws. A send's
`latency_us` is read with the network mode it was sent under (`unreliable`: U[1, 27) ms, else
U[1, 10) ms, tester.rs:127-137); `dropped` is its loss draw (unreliable mode only). Any line may
carry `"cluster"` (default 0) and, instead of the decoded value, the raw draw words
`"w0"` / `"w1"`. `decisions_from_events` builds the DECISION_DTYPE table `Batch.set_decisions`
and `replay` take; `events_from_decisions` writes a recorded table back as lines.
"""
import json

import numpy as np

from . import _abi

LAT_LO = 1000


def _lat_hi(unreliable):
    return 27000 if unreliable else 10000


def _range_value(w, lo, hi):
    return lo + ((int(w) * (hi - lo)) >> 32)


def decisions_from_events(events, elect_lo_us=150_000, elect_hi_us=300_000, unreliable=None):
    """DECISION_DTYPE records for an iterable of event dicts (see the module docstring).

    A decoded send needs its network mode: the line's `"unreliable"`, else the `unreliable`
    argument (the run's mode, e.g. the scenario's); with neither it is rejected, never guessed.
    A dropped send (unreliable mode only: the reliable net loses nothing) needs no latency."""
    rows = []
    for e in events:
        kind, c = e["event"], int(e.get("cluster", 0))
        raw = "w0" in e
        if kind == "send":
            stream, ent = _abi.MR_DS_NET, int(e["host"])
            if raw:
                w0, w1 = int(e["w0"]), int(e.get("w1", 0))
            else:
                mode = e.get("unreliable", unreliable)
                if mode is None:
                    raise ValueError(f"send event without its network mode ('unreliable'): {e}")
                dropped = bool(e.get("dropped", False))
                if dropped and not mode:
                    raise ValueError(f"dropped send in reliable mode (loss 0, tester.rs:127-137): {e}")
                if not dropped and "latency_us" not in e:
                    raise ValueError(f"delivered send without latency_us: {e}")
                w0, w1 = _abi.net_decision(dropped, int(e.get("latency_us", LAT_LO)), bool(mode))
        elif kind == "election_timeout":
            stream, ent = _abi.MR_DS_ELECT, int(e["node"])
            w0 = int(e["w0"]) if raw else _abi.decision_word(int(e["timeout_us"]), elect_lo_us,
                                                            elect_hi_us)
            w1 = int(e.get("w1", 0))
        elif kind == "rng":
            stream, ent = _abi.MR_DS_TESTER, int(e["thread"])
            if raw:
                w0, w1 = int(e["w0"]), int(e.get("w1", 0))
            else:
                v = int(e["u64"])
                w0, w1 = v & 0xFFFFFFFF, v >> 32
        else:
            raise ValueError(f"unknown decision event {kind!r}")
        if not (0 <= ent < 1 << 16 and 0 <= w0 < 1 << 32 and 0 <= w1 < 1 << 32):
            raise ValueError(f"decision event out of range: {e}")
        rows.append((c, stream, ent, int(e["index"]), w0, w1))
    return np.array(rows, _abi.DECISION_DTYPE)


def events_from_decisions(d, unreliable=True, elect_lo_us=150_000, elect_hi_us=300_000, raw=False):
    """Event dicts for DECISION_DTYPE records; sends are decoded under one network mode
    (`unreliable`), so a run that switches modes is written with `raw=True` (draw words)."""
    out = []
    for r in np.asarray(d, _abi.DECISION_DTYPE):
        c, s, ent, seq, w0, w1 = (int(r[f]) for f in ("cluster", "stream", "entity", "seq", "w0", "w1"))
        if s == _abi.MR_DS_NET:
            e = {"event": "send", "host": ent, "index": seq}
            if raw:
                e.update(w0=w0, w1=w1)
            else:
                e.update(dropped=bool(unreliable and w0 < _abi.LOSS_Q32),
                         latency_us=_range_value(w1, LAT_LO, _lat_hi(unreliable)),
                         unreliable=bool(unreliable))
        elif s == _abi.MR_DS_ELECT:
            e = {"event": "election_timeout", "node": ent, "index": seq}
            if raw:
                e.update(w0=w0, w1=w1)
            else:
                e["timeout_us"] = _range_value(w0, elect_lo_us, elect_hi_us)
        elif s == _abi.MR_DS_TESTER:
            e = {"event": "rng", "thread": ent, "index": seq}
            if raw:
                e.update(w0=w0, w1=w1)
            else:
                e["u64"] = (w1 << 32) | w0
        else:
            raise ValueError(f"unknown decision stream {s}")
        if c:
            e["cluster"] = c
        out.append(e)
    return out


def load_jsonl(path, **kw):  # kw: decisions_from_events' (elect_lo_us, elect_hi_us, unreliable)
    """decisions_from_events over a JSON-lines file (blank lines and # comments skipped)."""
    with open(path) as f:
        ev = [json.loads(line) for line in f if line.strip() and not line.lstrip().startswith("#")]
    return decisions_from_events(ev, **kw)


def dump_jsonl(path, d, **kw):
    with open(path, "w") as f:
        for e in events_from_decisions(d, **kw):
            f.write(json.dumps(e) + "\n")
