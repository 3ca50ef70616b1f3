"""Offline model of the step kernel's wave scheduling (dev tool).

Per-cluster event sequences come from oracle traces (each node event's class / kind / node and
whether its node applied entries); 64 clusters share a wave; every iteration the wave picks an
event class by the kernel's rule (mr_kernel.hip step loop) and the lanes whose next event is in
it run it. An iteration costs a base plus, per event kind present, that kind's section cost (wave
ticks per visit, profiles/r03d_section_profile.txt). Results do not depend on the policy, so
any policy can be scored here before it is built.

usage: python tools/sched_sim.py [clusters=256] [policy ...]
"""
import collections
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tests.oracle_lib import Oracle  # noqa: E402

# wave ticks (100 MHz) per visit, r03d section profile
C = dict(tail=57, sel=46, decode=104, load=20, drop=33, rv_req=157, rv_rep=133, ae_req=554,
         ae_probe=299, ae_rep=131, hb=39, elect=20, apply=561, send=32, store=23, tester=550,
         stepdown=77, s_trip=94 + 57 + 16)
KIND = {1: "rv_req", 2: "rv_rep", 3: "ae_req", 4: "ae_rep", 16: "drop", 17: "drop"}


def events(o, cfg, c):
    _, tr = o.run_cluster(cfg, c, trace_cap=1 << 17)
    out, applied = [], collections.defaultdict(int)
    for r in tr:
        cls, kind, node = int(r["cls"]), int(r["kind"]), int(r["node"])
        if cls == 2:
            out.append(("T", None, 0, 0))
        elif cls in (0, 1):
            k = KIND.get(kind, "drop") if cls == 0 else ("hb" if kind == 1 else "elect")
            ap = int(r["applied"]) > applied[node]
            applied[node] = int(r["applied"])
            sends = {"rv_req": 1, "ae_req": 1, "rv_rep": 0, "ae_rep": 1, "hb": 2, "elect": 2}.get(k, 0)
            out.append(("N", k, ap, sends))
    return out


def iter_cost(evs):
    cost = C["tail"] + C["sel"]
    if any(e[0] == "T" for e in evs):
        cost += C["tester"]
    node = [e for e in evs if e[0] == "N"]
    if node:
        cost += C["decode"] + C["load"] + C["store"] + C["stepdown"]
        for k in {e[1] for e in node}:
            cost += C[k] + (C["ae_probe"] if k == "ae_req" else 0)
        if any(e[2] for e in node):
            cost += C["apply"]
        cost += C["send"] + C["s_trip"] * max(e[3] for e in node)
    return cost


def greedy(groups):
    """each iteration: the candidate class (a set of kinds, 'T' = tester) with the most events
    per tick of its iteration's cost"""
    def pol(nxt, live, ns, nn):
        best, bsc = [], -1.0
        for g in groups:
            run = [i for i in live if (nxt[i][0] == "T" and "T" in g) or (nxt[i][0] == "N" and nxt[i][1] in g)]
            if not run:
                continue
            sc = len(run) / iter_cost([nxt[i] for i in run])
            if sc > bsc:
                best, bsc = run, sc
        return best
    return pol


NODE = {"rv_req", "rv_rep", "ae_req", "ae_rep", "hb", "elect", "drop"}


def run_wave(seqs, policy):
    pos = [0] * len(seqs)
    ticks, iters, nit, tit = 0, 0, 0, 0
    while True:
        live = [i for i in range(len(seqs)) if pos[i] < len(seqs[i])]
        if not live:
            break
        nxt = {i: seqs[i][pos[i]] for i in live}
        ns = sum(1 for i in live if nxt[i][0] == "T")
        nn = len(live) - ns
        run = policy(nxt, live, ns, nn)
        iters += 1
        cost = iter_cost([nxt[i] for i in run])
        if any(nxt[i][0] == "T" for i in run):
            tit += 1
        if any(nxt[i][0] == "N" for i in run):
            nit += 1
        ticks += cost
        for i in run:
            pos[i] += 1
    return ticks, iters, nit, tit


def kernel_policy(nxt, live, ns, nn, tnum=1, tden=3, ae_others=32):
    if tden * ns >= tnum * (ns + nn):
        return [i for i in live if nxt[i][0] == "T"]
    node = [i for i in live if nxt[i][0] == "N"]
    ae = [i for i in node if nxt[i][1] == "ae_req"]
    if len(ae) < len(node) and 2 * len(ae) < len(node) and len(node) - len(ae) >= ae_others:
        return [i for i in node if nxt[i][1] != "ae_req"]
    return node


POLICIES = {
    "kernel": kernel_policy,
    "no_ae_class": lambda n, l, s, m: kernel_policy(n, l, s, m, ae_others=10 ** 9),
    "all_in_one": lambda n, l, s, m: l,  # every lane its own event (union of paths)
    "greedy3": greedy([{"T"}, NODE, NODE - {"ae_req"}]),
    "greedy5": greedy([{"T"}, NODE, NODE - {"ae_req"}, {"ae_req"}, NODE - {"ae_req", "ae_rep"}]),
    "greedy_all": greedy([{"T"}, NODE, NODE - {"ae_req"}, {"ae_req"}, {"ae_req", "ae_rep"},
                          NODE - {"ae_req", "ae_rep"}, {"hb"}, {"hb", "elect", "drop"},
                          {"rv_req", "rv_rep"}, NODE | {"T"}]),
    "tester_quarter": lambda n, l, s, m: kernel_policy(n, l, s, m, tnum=1, tden=4),
    "tester_half": lambda n, l, s, m: kernel_policy(n, l, s, m, tnum=1, tden=2),
}


def main():
    clusters = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    names = sys.argv[2:] or list(POLICIES)
    o = Oracle()
    cfg = o.cfg("figure_8_unreliable_2c")
    seqs = [events(o, cfg, c) for c in range(clusters)]
    nev = sum(len(s) for s in seqs)
    for name in names:
        tot = it = ni = ti = 0
        for w in range(0, clusters, 64):
            t, a, b, c = run_wave(seqs[w:w + 64], POLICIES[name])
            tot += t; it += a; ni += b; ti += c
        waves = clusters // 64
        print(f"{name:14s} ticks/wave {tot / waves:10.0f}  iters/wave {it / waves:7.0f} "
              f"(node {ni / waves:6.0f}, tester {ti / waves:6.0f})  events/iter {nev / it:5.1f}")


if __name__ == "__main__":
    main()
