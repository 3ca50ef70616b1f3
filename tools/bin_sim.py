"""Offline model of cross-wave event-kind binning (dev tool; verdict r4 item 1).

A workgroup of K waves owns a pool of P clusters (the kernel today: K = 8 waves per CU, each
bound to its own 64 clusters, P = 512). In the binned form a wave that becomes free takes up to
64 ready clusters (not held by another wave) whose next event is of ONE kind — the kind its
policy picks — runs them, and releases them. An iteration costs what `sched_sim.iter_cost`
charges for that kind set (the r04 section profile's wave ticks per visit, which already hold
two waves per SIMD of contention), plus `move` ticks to bring a cluster's run state into the
lane and back (registers <-> LDS / HBM) and `bin` ticks for the binning itself.

Event sequences: oracle traces of figure_8_unreliable_2c (the headline), same as sched_sim.
Output: workgroup makespan (ticks of the slowest wave until the pool is drained) per policy,
compared with the kernel's own rule on the same clusters.

usage: python tools/bin_sim.py [clusters=512] [move=0] [bin=0]
"""
import heapq
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tests.oracle_lib import Oracle  # noqa: E402
from tools.sched_sim import C, events, iter_cost, kernel_policy  # noqa: E402

# section costs of the final round-4 library (profiles/r04_section_profile_headline.txt)
C.update(tail=64, sel=45, decode=74, load=21, drop=32, rv_req=124, rv_rep=97, ae_req=564,
         ae_probe=266, ae_rep=74, hb=41, elect=21, apply=575, send=31, store=22, tester=528,
         stepdown=75, s_trip=96 + 58 + 16)


def kind_of(e):
    return "T" if e[0] == "T" else e[1]


def per_wave_kernel(seqs, K):
    """today: wave w owns clusters [64w, 64w + 64) for the whole launch (sched_sim.run_wave)"""
    ends = []
    for w in range(K):
        part = seqs[64 * w: 64 * w + 64]
        pos = [0] * len(part)
        t = 0
        while True:
            live = [i for i in range(len(part)) if pos[i] < len(part[i])]
            if not live:
                break
            nxt = {i: part[i][pos[i]] for i in live}
            ns = sum(1 for i in live if nxt[i][0] == "T")
            run = kernel_policy(nxt, live, ns, len(live) - ns)
            t += iter_cost([nxt[i] for i in run])
            for i in run:
                pos[i] += 1
        ends.append(t)
    return max(ends), sum(ends) / len(ends)


def binned(seqs, K, move, binc, pick="most", width=64, merge=None, bank=0, per=1):
    """K waves share the pool; a free wave takes up to `width` ready clusters of one kind.
    merge: kinds folded together into one bin (e.g. the short node kinds).
    bank (round 6, verdict r5 item 1): a claim takes at most `per` clusters of each LDS bank
    class, cluster i's class being i % bank — bank=64: lane b claims a slot with slot % 64 == b;
    bank=32, per=2: lanes b and b + 32 (the two 32-lane halves of a ds_read_b32 / ds_write_b32,
    which never conflict with each other) share the slots with slot % 32 == b % 32"""
    merge = merge or {}
    P = len(seqs)
    pos = [0] * P
    busy = [False] * P
    free_at = [(0, w) for w in range(K)]  # (time the wave is free, wave)
    heapq.heapify(free_at)
    release = []  # (time, wave, clusters)
    now = 0
    iters = 0
    evs = 0
    done = 0
    wave_time = 0
    while done < P:
        t, w = heapq.heappop(free_at)
        now = max(now, t)
        # clusters released by waves that finished by `now`
        while release and release[0][0] <= now:
            _, _, cl = heapq.heappop(release)
            for i in cl:
                busy[i] = False
                if pos[i] == len(seqs[i]):
                    done += 1
        bins = {}
        for i in range(P):
            if not busy[i] and pos[i] < len(seqs[i]):
                k = kind_of(seqs[i][pos[i]])
                k = merge.get(k, k)
                bins.setdefault(k, []).append(i)
        if not bins:
            if not release:
                break
            heapq.heappush(free_at, (release[0][0], w))
            continue
        def take(lst):
            if not bank:
                return lst[:width]
            cnt, out = {}, []
            for i in lst:
                if cnt.get(i % bank, 0) < per and len(out) < width:
                    cnt[i % bank] = cnt.get(i % bank, 0) + 1
                    out.append(i)
            return out
        if pick == "most":
            k = max(bins, key=lambda k: len(take(bins[k])))
        else:  # most events per tick of the iteration's cost
            k = max(bins, key=lambda k: len(take(bins[k])) /
                    (iter_cost([seqs[i][pos[i]] for i in take(bins[k])]) + move + binc))
        cl = take(bins[k])
        cost = iter_cost([seqs[i][pos[i]] for i in cl]) + move + binc
        for i in cl:
            busy[i] = True
            pos[i] += 1
        iters += 1
        evs += len(cl)
        wave_time += cost
        heapq.heappush(release, (now + cost, w, cl))
        heapq.heappush(free_at, (now + cost, w))
    end = max(r[0] for r in release) if release else now
    return end, iters, evs, wave_time


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    move = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    binc = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    o = Oracle()
    cfg = o.cfg("figure_8_unreliable_2c")
    seqs = [events(o, cfg, c) for c in range(P)]
    nev = sum(len(s) for s in seqs)
    K = P // 64
    base, mean = per_wave_kernel(seqs, K)
    print(f"pool {P} clusters, {nev} events; kernel rule, wave-bound: makespan {base:.0f} ticks "
          f"(mean wave {mean:.0f})")
    short = {k: "short" for k in ("rv_req", "rv_rep", "ae_rep", "hb", "elect", "drop")}
    for name, kw in [(f"binned K={K} most", dict(K=K)),
                     (f"binned K={K} rate", dict(K=K, pick="rate")),
                     (f"binned K={K // 2} most", dict(K=K // 2)),
                     (f"binned K={K // 2} rate", dict(K=K // 2, pick="rate")),
                     (f"binned K={K} short", dict(K=K, merge=short)),
                     (f"binned K={K // 2} short", dict(K=K // 2, merge=short)),
                     (f"binned K={K} bank 64", dict(K=K, bank=64)),
                     (f"binned K={K} bank 32x2", dict(K=K, bank=32, per=2))]:
        end, it, ev, wt = binned(seqs, move=move, binc=binc, **kw)
        print(f"{name:26s} makespan {end:9.0f} ({base / end:5.2f}x)  iters {it:7d}  "
              f"events/iter {ev / it:5.1f}  ticks/event {wt / ev:6.1f}")


if __name__ == "__main__":
    main()
