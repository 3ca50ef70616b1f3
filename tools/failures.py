"""Account for the clusters that do not pass at a BASELINE config (verdict r4 item 2): the
oracle's verdict histogram over a seed range, and for failing seeds the panic site, the fail
time and what their trace shows (dev tool; CPU only, the oracle).

usage: python tools/failures.py <test> <clusters> [nodes] [--unreliable] [--explain K]
Runs the oracle over clusters [0, clusters) in one process per CPU, prints the histogram and
the failing clusters, and with --explain K walks the first K failures' traces:
  * ONE_NO_AGREEMENT (tester.rs:254-255 with retry = false, :261 otherwise): the one() window
    [t_fail - 2 s, t_fail] (retry = false) — which leader accepted the command, whether a
    leader change happened inside the window, and each server's commit / applied at the end;
  * any other code: the last 30 trace records.
"""
import argparse
import collections
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from madraft_amd import _abi  # noqa: E402
from tests.oracle_lib import Oracle  # noqa: E402

KIND = {1: "RVreq", 2: "RVrep", 3: "AEreq", 4: "AErep", 5: "ISreq", 6: "ISrep"}
ROLE = {0: "F", 1: "C", 2: "L", 3: "D"}
ONE_NO_AGREEMENT = 6  # include/madraft_sim.h MR_FAIL_ONE_NO_AGREEMENT (tester.rs:255, :261)


def make_cfg(o, a):
    kw = {"flags": _abi.MR_F_UNRELIABLE} if a.unreliable else {}
    if a.seed_offset:  # tools/configs.py times seeds README_SEED + 2 * clusters + [0, clusters)
        kw["seed_base"] = _abi.README_SEED + a.seed_offset
    if a.nodes:
        kw["n_nodes"] = a.nodes
        if a.nodes > 5:  # as madraft_amd.sim.make_cfg: 7-node runs keep 64 message slots
            kw["msg_slots"] = 64
    return o.cfg(a.test, **kw)


def _chunk(args):
    a, lo, hi = args
    o = Oracle()
    code, t, _, _ = o.run_batch(make_cfg(o, a), lo, hi - lo)
    return lo, code, t


def scan(a):
    n = a.clusters
    step = max(1, -(-n // (4 * (os.cpu_count() or 1))))
    jobs = [(a, lo, min(n, lo + step)) for lo in range(0, n, step)]
    code = np.empty(n, np.uint16)
    t = np.empty(n, np.uint32)
    with mp.Pool(os.cpu_count()) as p:
        for lo, c, tt in p.imap_unordered(_chunk, jobs):
            code[lo:lo + len(c)] = c
            t[lo:lo + len(c)] = tt
    return code, t


def fmt(e):
    cls, k, n = int(e["cls"]), int(e["kind"]), int(e["node"])
    if cls == 2:
        return "tester"
    if cls == 3:
        return f"VERDICT {k}"
    s = f"timer {'hb' if k == 1 else 'elect'} n{n}" if cls == 1 else f"{KIND.get(k, 'drop')} n{n}"
    return (s + f" {ROLE[int(e['role'])]} term={int(e['term'])} commit={int(e['commit'])} "
            f"applied={int(e['applied'])} last={int(e['last'])} snap={int(e['snap'])}")


def explain_one(o, cfg, c, code, tf):
    _, tr = o.run_cluster(cfg, c, trace_cap=1 << 18)
    print(f"--- cluster {c}: code {code} at {tf / 1e6:.3f} s, {len(tr)} events")
    node = [r for r in tr if int(r["cls"]) in (0, 1)]
    if code != ONE_NO_AGREEMENT:
        for r in tr[-30:]:
            print(f"  {int(r['time_us']) / 1e3:10.3f} ms  {fmt(r)}")
        return "other"
    w0 = tf - 2_000_000
    # leaders: (term, node, first time seen as leader)
    lead = {}
    for r in node:
        if int(r["role"]) == 2:
            key = (int(r["term"]), int(r["node"]))
            lead.setdefault(key, int(r["time_us"]))
    before = [k for k, ts in lead.items() if ts < w0]
    inside = sorted((ts, k) for k, ts in lead.items() if w0 <= ts <= tf)
    last = {}
    for r in node:
        last[int(r["node"])] = r
    print(f"  one() window [{w0 / 1e6:.3f}, {tf / 1e6:.3f}] s; leader before it: "
          f"{max(before) if before else None} (term, node); elected inside it: "
          f"{[(k, round(ts / 1e3, 1)) for ts, k in inside]}")
    for n_, r in sorted(last.items()):
        print(f"  server {n_}: {fmt(r)}")
    term, ln = max(lead)  # the last leader (highest term)
    lr = last[ln]
    top = max(int(r["last"]) for r in last.values())
    if int(lr["commit"]) < int(lr["last"]):
        # Figure 8 / Raft section 5.4.2: a leader commits an entry of an earlier term only with
        # an entry of its own term above it; one(.., retry = false) starts no second command
        why = "uncommittable_earlier_term"
    elif top > int(lr["last"]):
        # the command went to a leader that had lost (or was losing) its term: the new
        # leader's log does not hold it, so it is never replicated to the expected servers
        why = "accepted_by_deposed_leader"
    else:
        why = "other"
    print(f"  -> {why}: last leader server {ln} (term {term}) last={int(lr['last'])} "
          f"commit={int(lr['commit'])}; longest log {top}; elected inside the window: {bool(inside)}")
    return why


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("test")
    ap.add_argument("clusters", type=int)
    ap.add_argument("nodes", type=int, nargs="?", default=0)
    ap.add_argument("--unreliable", action="store_true")
    ap.add_argument("--explain", type=int, default=0)
    ap.add_argument("--seed-offset", type=int, default=0,
                    help="seed_base = README_SEED + this (the configs table's range: 2 x clusters)")
    a = ap.parse_args()
    code, t = scan(a)
    h = collections.Counter(code.tolist())
    print(f"{a.test} nodes={a.nodes or 'default'} unreliable={a.unreliable} clusters={a.clusters} "
          f"seed_base=README_SEED+{a.seed_offset}: "
          f"verdicts {dict(sorted(h.items()))}")
    bad = np.nonzero(code != 0)[0]
    print(f"failing clusters (first 40): {bad[:40].tolist()}")
    print(f"their fail times (s): {[round(int(x) / 1e6, 3) for x in t[bad[:40]]]}")
    if a.explain:
        o = Oracle()
        cfg = make_cfg(o, a)
        kinds = collections.Counter()
        for c in bad[:a.explain]:
            kinds[explain_one(o, cfg, int(c), int(code[c]), int(t[c]))] += 1
        print(f"explained {sum(kinds.values())}: {dict(kinds)}")


if __name__ == "__main__":
    main()
