// mr_kernel.hip — CDNA4 (gfx950) kernels of the batched Raft simulator.
//
// step_kernel: one lane owns one cluster (one seed of one reference test).
// Each lane keeps its next event — the minimum (time, class, tie) key over
// its node timers, its cached earliest in-flight message and its tester
// wake-up (docs/SEMANTICS.md §3) — in registers. Per iteration the wave picks
// ONE event class by ballot (message / node timer / tester) and only lanes
// whose next event has that class process it; the others wait with their
// event cached. Waiting never reorders a cluster's own events, so results
// are identical to processing every lane every iteration, but a wave now runs
// one handler path per iteration instead of the union of all three (the
// 64-lane divergence cost of SIMT), and the tester path — the longest — runs
// when at least half the live lanes want it.
//
// Replaces, for a whole batch at once: the madsim executor + net + fs + rand,
// the Raft node (src/raft/raft.rs), the tester (src/raft/tester.rs) and the
// test bodies (src/raft/tests.rs, here as native protothread coroutines).
//
// Fail handling mirrors a Rust panic: the first verdict stops the cluster;
// handlers return as soon as x.code leaves MR_RUNNING, before any further
// observable effect (sends, trace records).
#include <hip/hip_runtime.h>

#include "mr_dev.h"

namespace mr {

#define DI __device__ __forceinline__
constexpr uint32_t INF_T = 0xFFFFFFFFu;
constexpr uint32_t LOSS_Q32 = 429496729u;  // floor(0.1 * 2^32), tester.rs:130
constexpr uint64_t FNV_OFF = 0xCBF29CE484222325ull, FNV_P = 0x100000001B3ull;
constexpr uint32_t RUN = MR_RUNNING;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t ELECTION_US = 1000000;  // RAFT_ELECTION_TIMEOUT, tests.rs:18

// per-lane registers of one cluster during a launch
struct X {
  uint32_t c, now, events, msgs_sent, inflight, code, trace_n, mslot, netmode, t_ctr;
  uint32_t sleep_us, yield;
  uint64_t free_mask, digest, mmin;
  uint32_t cnt[CNT__N];
};

// field accessors (32-bit element offsets, checked at batch creation)
#define CS(f) D.cs32[(uint32_t)(f) * D.C + x.c]
#define C64(f) D.cs64[(uint32_t)(f) * D.C + x.c]
#define ND(f, d) D.nd32[((uint32_t)(f) * D.n + (d)) * D.C + x.c]
#define NSV(d) D.nsnapv[(uint32_t)(d) * D.C + x.c]
#define PR(f, d, p) D.pr32[(((uint32_t)(f) * D.n + (d)) * D.n + (p)) * D.C + x.c]
#define MS32(f, mi) D.ms32[(uint32_t)(f) * D.M * D.C + (mi)]
#define MS64(f, mi) D.ms64[(uint32_t)(f) * D.M * D.C + (mi)]

// ---------------------------------------------------------------- helpers
DI uint32_t f_role(uint32_t f) { return f & 3u; }
DI uint32_t f_alive(uint32_t f) { return (f >> 2) & 1u; }
DI uint32_t f_conn(uint32_t f) { return (f >> 3) & 1u; }
DI uint32_t f_voted(uint32_t f) { return (f >> 4) & 15u; }
DI uint32_t f_inc(uint32_t f) { return (f >> 8) & 255u; }
DI uint32_t f_votes(uint32_t f) { return (f >> 16) & 255u; }
DI uint32_t f_set(uint32_t f, uint32_t sh, uint32_t w, uint32_t v) {
  uint32_t m = ((1u << w) - 1u) << sh;
  return (f & ~m) | ((v << sh) & m);
}
DI uint32_t u_range(uint32_t w, uint32_t lo, uint32_t hi) {
  return lo + (uint32_t)(((uint64_t)w * (uint64_t)(hi - lo)) >> 32);
}

// Philox4x32-10, counter (c0, c1, c2, 0), key = the cluster's seed; returns w0, w1
DI void philox(const Dev& D, const X& x, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t& w0,
               uint32_t& w1) {
  uint64_t seed = D.seed0 + x.c;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32), c3 = 0;
#pragma unroll
  for (int r = 0; r < 10; r++) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  w0 = c0; w1 = c1;
}

DI size_t logi(const Dev& D, const X& x, uint32_t d, uint32_t i) {
  return ((size_t)x.c * D.n + d) * D.log_cap + (i & (D.log_cap - 1u));
}
DI uint32_t term_at(const Dev& D, const X& x, uint32_t d, uint32_t i, uint32_t snap,
                    uint32_t snapt) {
  if (i == 0) return 0;
  if (i == snap) return snapt;
  return D.lterm[logi(D, x, d, i)];
}

DI uint32_t net_loss(const X& x) { return (x.netmode & 1u) ? LOSS_Q32 : 0u; }  // tester.rs:127-137
DI uint32_t net_lat_hi(const X& x) { return (x.netmode & 1u) ? 27000u : 10000u; }

// ---------------------------------------------------------------- trace
DI void rec8(const Dev& D, X& x, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4,
             uint32_t w5, uint32_t w6, uint32_t w7) {
  uint64_t h = x.digest;
  h = (h ^ w0) * FNV_P; h = (h ^ w1) * FNV_P; h = (h ^ w2) * FNV_P; h = (h ^ w3) * FNV_P;
  h = (h ^ w4) * FNV_P; h = (h ^ w5) * FNV_P; h = (h ^ w6) * FNV_P; h = (h ^ w7) * FNV_P;
  x.digest = h;
  if (x.c < D.trace_clusters && x.trace_n < D.trace_cap) {
    uint32_t* p = reinterpret_cast<uint32_t*>(D.trace + (size_t)x.c * D.trace_cap + x.trace_n);
    p[0] = w0; p[1] = w1; p[2] = w2; p[3] = w3; p[4] = w4; p[5] = w5; p[6] = w6; p[7] = w7;
  }
  x.trace_n++;
}

DI void rec_node(const Dev& D, X& x, uint32_t cls, uint32_t kind, uint32_t d, uint32_t aux) {
  uint32_t f = ND(NF_FLAGS, d);
  uint32_t role = f_alive(f) ? f_role(f) : R_DOWN;
  rec8(D, x, x.now, cls | (kind << 8) | (d << 16) | (role << 24), aux, ND(NF_TERM, d),
       ND(NF_COMMIT, d), ND(NF_APPLIED, d), ND(NF_LAST, d), ND(NF_SNAP, d));
}

DI void rec_simple(const Dev& D, X& x, uint32_t cls, uint32_t kind) {
  rec8(D, x, x.now, cls | (kind << 8) | (0xFFu << 16), x.msgs_sent, 0, 0, 0, 0, 0);
}

DI void fail(const Dev& D, X& x, uint32_t code) {
  if (x.code != RUN) return;
  x.code = code;
  rec_simple(D, x, 3, code);
}

// ---------------------------------------------------------------- timers / net
DI void reset_timer(const Dev& D, X& x, uint32_t d) {  // raft.rs:260-263
  uint32_t ctr = ND(NF_ECTR, d);
  ND(NF_ECTR, d) = ctr + 1;
  uint32_t w0, w1;
  philox(D, x, ctr, d, ST_ELECT, w0, w1);
  ND(NF_TIMER, d) = x.now + u_range(w0, D.elo, D.ehi);
}

DI void rescan_min(const Dev& D, X& x) {
  uint64_t best = ~0ull;
  uint32_t bs = 0;
  uint64_t occ = ~x.free_mask;
  for (uint32_t s = 0; s < D.M; s++) {
    if (!((occ >> s) & 1ull)) continue;
    uint64_t k = MS64(M64_KEY, s * D.C + x.c);
    if (k < best) { best = k; bs = s; }
  }
  x.mmin = best;
  x.mslot = bs;
}

// madsim net send (tester.rs:127-137, :147-149). Returns the slot or -1.
DI int net_send(const Dev& D, X& x, uint32_t src, uint32_t dst, uint32_t type, uint32_t inc,
                uint32_t term, uint32_t a, uint32_t b, uint32_t c, uint64_t v, uint32_t k) {
  uint32_t seq = x.msgs_sent++;
  uint32_t ctr = ND(NF_NCTR, src);
  ND(NF_NCTR, src) = ctr + 1;
  if (!f_conn(ND(NF_FLAGS, src)) || !f_conn(ND(NF_FLAGS, dst))) { x.cnt[CNT_DROP_CLOG]++; return -1; }
  uint32_t w0, w1;
  philox(D, x, ctr, src, ST_NET, w0, w1);
  if (w0 < net_loss(x)) { x.cnt[CNT_DROP_LOSS]++; return -1; }
  if (x.inflight >= D.M) { x.cnt[CNT_DROP_OVERFLOW]++; return -1; }
  if (seq >= (1u << 30)) { fail(D, x, MR_FAIL_SIM_CAPACITY); return -1; }
  uint32_t t = x.now + u_range(w1, 1000u, net_lat_hi(x));
  uint32_t slot = (uint32_t)__builtin_ctzll(x.free_mask);
  x.free_mask &= ~(1ull << slot);
  uint64_t key = ((uint64_t)t << 32) | seq;
  uint32_t mi = slot * D.C + x.c;
  MS64(M64_KEY, mi) = key;
  MS32(MF_HDR, mi) = type | (src << 3) | (dst << 6) | (inc << 9) | (k << 17);
  MS32(MF_TERM, mi) = term; MS32(MF_A, mi) = a; MS32(MF_B, mi) = b; MS32(MF_C, mi) = c; MS64(M64_V, mi) = v;
  x.inflight++;
  if (x.inflight > x.cnt[CNT_MAX_INFLIGHT]) x.cnt[CNT_MAX_INFLIGHT] = x.inflight;
  if (key < x.mmin) { x.mmin = key; x.mslot = slot; }
  return (int)slot;
}

// ---------------------------------------------------------------- tester storage
DI void push_and_check(const Dev& D, X& x, uint32_t i, uint32_t idx, uint64_t v) {
  if (idx >= D.apply_cap) { fail(D, x, MR_FAIL_SIM_CAPACITY); return; }
  x.cnt[CNT_APPLIES]++;
  size_t si = (size_t)x.c * D.apply_cap + idx;
  uint32_t m = D.smask[si];
  if (m && D.sval[si] != v) { fail(D, x, MR_FAIL_APPLY_MISMATCH); return; }  // tester.rs:384
  uint32_t len = ND(NF_SLEN, i);
  if (idx > len) { fail(D, x, MR_FAIL_APPLY_OUT_OF_ORDER); return; }  // tester.rs:393
  if (idx == len) {
    D.sval[si] = v;
    D.smask[si] = (uint8_t)(m | (1u << i));
    ND(NF_SLEN, i) = len + 1;
    if (idx > x.cnt[CNT_MAX_INDEX]) x.cnt[CNT_MAX_INDEX] = idx;
  }
}

DI void storage_snapshot(const Dev& D, X& x, uint32_t i, uint32_t idx) {  // tester.rs:399-402
  if (idx >= D.apply_cap) { fail(D, x, MR_FAIL_SIM_CAPACITY); return; }
  uint32_t nl = idx + 1, len = ND(NF_SLEN, i);
  for (uint32_t j = nl; j < len; j++) {
    size_t si = (size_t)x.c * D.apply_cap + j;
    D.smask[si] = (uint8_t)(D.smask[si] & ~(1u << i));
  }
  ND(NF_SLEN, i) = nl;
}

DI uint32_t n_committed(const Dev& D, X& x, uint32_t idx, uint64_t& v) {  // tester.rs:405-422
  if (idx >= D.apply_cap) { v = 0; return 0; }
  size_t si = (size_t)x.c * D.apply_cap + idx;
  v = D.sval[si];
  return (uint32_t)__builtin_popcount((uint32_t)D.smask[si]);
}

// ---------------------------------------------------------------- Raft node
DI void node_apply(const Dev& D, X& x, uint32_t me) {  // tester.rs:302-325 applier
  uint32_t applied = ND(NF_APPLIED, me), commit = ND(NF_COMMIT, me);
  uint32_t snap = ND(NF_SNAP, me), snapt = ND(NF_SNAPT, me);
  bool snapmode = (x.netmode >> 1) & 1u;
  while (applied < commit) {
    applied++;
    uint64_t v = D.lval[logi(D, x, me, applied)];
    push_and_check(D, x, me, applied, v);
    if (x.code != RUN) return;
    if (snapmode && (applied + 1) % 10u == 0 && applied > snap) {
      snapt = term_at(D, x, me, applied, snap, snapt);
      snap = applied;
      ND(NF_SNAP, me) = snap; ND(NF_SNAPT, me) = snapt; NSV(me) = v;
      x.cnt[CNT_SNAPSHOTS]++;
    }
  }
  ND(NF_APPLIED, me) = applied;
}

DI void send_append(const Dev& D, X& x, uint32_t l, uint32_t p) {
  uint32_t nx = PR(PF_NEXT, l, p), snap = ND(NF_SNAP, l), snapt = ND(NF_SNAPT, l), term = ND(NF_TERM, l);
  uint32_t inc = f_inc(ND(NF_FLAGS, l));
  if (nx <= snap) {
    net_send(D, x, l, p, M_IS_REQ, inc, term, snap, snapt, 0, NSV(l), 0);
    return;
  }
  uint32_t prev = nx - 1, last = ND(NF_LAST, l);
  uint32_t k = last - prev;
  if (k > D.K) k = D.K;
  uint32_t pt = term_at(D, x, l, prev, snap, snapt);
  x.cnt[CNT_SHIPPED] += k;
  int slot = net_send(D, x, l, p, M_AE_REQ, inc, term, prev, pt, ND(NF_COMMIT, l), 0, k);
  if (slot >= 0) {
    size_t pb = ((size_t)x.c * D.M + (uint32_t)slot) * D.K;
    for (uint32_t j = 0; j < k; j++) {
      size_t li = logi(D, x, l, prev + 1 + j);
      D.pterm[pb + j] = D.lterm[li];
      D.pval[pb + j] = D.lval[li];
    }
  }
}

DI void become_leader(const Dev& D, X& x, uint32_t me) {
  ND(NF_FLAGS, me) = f_set(ND(NF_FLAGS, me), 0, 2, R_L);
  x.cnt[CNT_LEADERS]++;
  uint32_t last = ND(NF_LAST, me);
  for (uint32_t p = 0; p < D.n; p++) { PR(PF_NEXT, me, p) = last + 1; PR(PF_MATCH, me, p) = 0; }
  PR(PF_MATCH, me, me) = last;
  for (uint32_t p = 0; p < D.n; p++) {
    if (p == me) continue;
    send_append(D, x, me, p);
    if (x.code != RUN) return;
  }
  ND(NF_TIMER, me) = x.now + D.hb;
}

// commit = the majority-th largest match index, if it is from the current term
DI void advance_commit(const Dev& D, X& x, uint32_t me) {
  uint32_t last = ND(NF_LAST, me), maj = D.n / 2 + 1, N = 0;
  for (uint32_t i = 0; i < D.n; i++) {
    uint32_t mi = (i == me) ? last : PR(PF_MATCH, me, i);
    if (mi <= N) continue;
    uint32_t ge = 0;
    for (uint32_t j = 0; j < D.n; j++) {
      uint32_t mj = (j == me) ? last : PR(PF_MATCH, me, j);
      ge += (mj >= mi) ? 1u : 0u;
    }
    if (ge >= maj) N = mi;
  }
  if (N > ND(NF_COMMIT, me) &&
      term_at(D, x, me, N, ND(NF_SNAP, me), ND(NF_SNAPT, me)) == ND(NF_TERM, me)) {
    ND(NF_COMMIT, me) = N;
    node_apply(D, x, me);
  }
}

DI void on_ack(const Dev& D, X& x, uint32_t me, uint32_t p, uint32_t xv) {
  if (xv > PR(PF_MATCH, me, p)) PR(PF_MATCH, me, p) = xv;
  if (xv + 1 > PR(PF_NEXT, me, p)) PR(PF_NEXT, me, p) = xv + 1;
  advance_commit(D, x, me);
  if (x.code != RUN) return;
  if (PR(PF_NEXT, me, p) <= ND(NF_LAST, me)) send_append(D, x, me, p);
}

DI void deliver(const Dev& D, X& x, uint32_t slot, uint32_t seq) {
  uint32_t mi = slot * D.C + x.c;
  uint32_t hdr = MS32(MF_HDR, mi);
  uint32_t type = hdr & 7u, src = (hdr >> 3) & 7u, me = (hdr >> 6) & 7u, inc = (hdr >> 9) & 255u;
  uint32_t k = (hdr >> 17) & 63u;
  uint32_t mterm = MS32(MF_TERM, mi), ma = MS32(MF_A, mi), mb = MS32(MF_B, mi), mc = MS32(MF_C, mi);
  uint64_t mv = MS64(M64_V, mi);
  MS64(M64_KEY, mi) = ~0ull;
  x.free_mask |= 1ull << slot;
  x.inflight--;
  rescan_min(D, x);

  uint32_t f = ND(NF_FLAGS, me);
  if (!f_alive(f) || !f_conn(f) || !f_conn(ND(NF_FLAGS, src))) {
    x.cnt[CNT_DROP_DELIVER]++;
    rec_node(D, x, 0, 16, me, seq);
    return;
  }
  bool is_reply = (type == M_RV_REP || type == M_AE_REP || type == M_IS_REP);
  if (is_reply && inc != f_inc(f)) {
    x.cnt[CNT_DROP_STALE]++;
    rec_node(D, x, 0, 17, me, seq);
    return;
  }
  uint32_t term = ND(NF_TERM, me);
  if (mterm > term) {  // step down
    uint32_t was = f_role(f);
    term = mterm;
    ND(NF_TERM, me) = term;
    f = f_set(f_set(f_set(f, 4, 4, 15u), 16, 8, 0u), 0, 2, R_F);
    ND(NF_FLAGS, me) = f;
    if (was == R_L) reset_timer(D, x, me);
  }
  uint32_t role = f_role(f);
  switch (type) {
    case M_RV_REQ: {
      uint32_t last = ND(NF_LAST, me);
      uint32_t lt = term_at(D, x, me, last, ND(NF_SNAP, me), ND(NF_SNAPT, me));
      bool up = (mc > lt) || (mc == lt && mb >= last);
      uint32_t voted = f_voted(f);
      bool granted = (mterm == term) && (voted == 15u || voted == ma) && up;
      if (granted) {
        ND(NF_FLAGS, me) = f_set(f, 4, 4, ma);
        reset_timer(D, x, me);
      }
      net_send(D, x, me, src, M_RV_REP, inc, term, granted ? 1u : 0u, 0, 0, 0, 0);
    } break;
    case M_RV_REP:
      if (role == R_C && mterm == term && ma) {
        uint32_t votes = f_votes(f) | (1u << src);
        ND(NF_FLAGS, me) = f_set(f, 16, 8, votes);
        if ((uint32_t)__builtin_popcount(votes) > D.n / 2) become_leader(D, x, me);
      }
      break;
    case M_AE_REQ: {
      if (mterm < term) { net_send(D, x, me, src, M_AE_REP, inc, term, 0, 0, 0, 0, 0); break; }
      if (role == R_C) ND(NF_FLAGS, me) = f_set(f, 0, 2, R_F);
      reset_timer(D, x, me);
      uint32_t snap = ND(NF_SNAP, me), snapt = ND(NF_SNAPT, me), last = ND(NF_LAST, me);
      uint32_t prev = ma, pterm = mb, j0 = 0;
      if (prev < snap) {
        uint32_t skip = snap - prev;
        j0 = skip < k ? skip : k;
        prev = snap; pterm = snapt;
      }
      if (prev > last) {
        net_send(D, x, me, src, M_AE_REP, inc, term, 0, last + 1, 0, 0, 0);
        break;
      }
      uint32_t tp = term_at(D, x, me, prev, snap, snapt);
      if (tp != pterm) {
        uint32_t xx = prev;
        while (xx - 1 > snap && term_at(D, x, me, xx - 1, snap, snapt) == tp) xx--;
        net_send(D, x, me, src, M_AE_REP, inc, term, 0, xx, 0, 0, 0);
        break;
      }
      size_t pb = ((size_t)x.c * D.M + slot) * D.K;
      for (uint32_t j = j0; j < k; j++) {
        uint32_t i = ma + 1 + j, et = D.pterm[pb + j];
        if (i <= last && term_at(D, x, me, i, snap, snapt) == et) continue;
        if (i - snap > D.log_cap) { fail(D, x, MR_FAIL_SIM_CAPACITY); return; }
        size_t li = logi(D, x, me, i);
        D.lterm[li] = et;
        D.lval[li] = D.pval[pb + j];
        last = i;
        if (i - snap > x.cnt[CNT_MAX_LOG]) x.cnt[CNT_MAX_LOG] = i - snap;
      }
      ND(NF_LAST, me) = last;
      uint32_t lc = ma + k;
      if (mc < lc) lc = mc;
      if (lc > ND(NF_COMMIT, me)) {
        ND(NF_COMMIT, me) = lc;
        node_apply(D, x, me);
        if (x.code != RUN) return;
      }
      net_send(D, x, me, src, M_AE_REP, inc, term, 1, ma + k, 0, 0, 0);
    } break;
    case M_AE_REP:
      if (role != R_L || mterm != term) break;
      if (ma) {
        on_ack(D, x, me, src, mb);
      } else {
        uint32_t xx = mb, lo = PR(PF_MATCH, me, src) + 1, hi = ND(NF_LAST, me) + 1;
        if (xx < lo) xx = lo;
        if (xx > hi) xx = hi;
        PR(PF_NEXT, me, src) = xx;
        send_append(D, x, me, src);
      }
      break;
    case M_IS_REQ: {
      if (mterm < term) { net_send(D, x, me, src, M_IS_REP, inc, term, 0, 0, 0, 0, 0); break; }
      if (role == R_C) ND(NF_FLAGS, me) = f_set(f, 0, 2, R_F);
      reset_timer(D, x, me);
      uint32_t idx = ma;
      if (idx > ND(NF_COMMIT, me)) {
        uint32_t last = ND(NF_LAST, me);
        if (!(idx <= last && term_at(D, x, me, idx, ND(NF_SNAP, me), ND(NF_SNAPT, me)) == mb))
          ND(NF_LAST, me) = idx;
        ND(NF_SNAP, me) = idx; ND(NF_SNAPT, me) = mb; NSV(me) = mv;
        ND(NF_COMMIT, me) = idx; ND(NF_APPLIED, me) = idx;
        storage_snapshot(D, x, me, idx);
        if (x.code != RUN) return;
        x.cnt[CNT_INSTALLS]++;
      }
      net_send(D, x, me, src, M_IS_REP, inc, term, 0, idx, 0, 0, 0);
    } break;
    case M_IS_REP:
      if (role == R_L && mterm == term && mb > 0) on_ack(D, x, me, src, mb);
      break;
  }
  if (x.code != RUN) return;
  rec_node(D, x, 0, type, me, seq);
}

DI void on_timer(const Dev& D, X& x, uint32_t me) {
  uint32_t f = ND(NF_FLAGS, me);
  if (f_role(f) == R_L) {  // heartbeat / replication round
    for (uint32_t p = 0; p < D.n; p++) {
      if (p == me) continue;
      send_append(D, x, me, p);
      if (x.code != RUN) return;
    }
    ND(NF_TIMER, me) = x.now + D.hb;
    rec_node(D, x, 1, 1, me, 0);
    return;
  }
  uint32_t term = ND(NF_TERM, me) + 1;  // election timeout: become candidate
  ND(NF_TERM, me) = term;
  ND(NF_FLAGS, me) = f_set(f_set(f_set(f, 4, 4, me), 0, 2, R_C), 16, 8, 1u << me);
  x.cnt[CNT_ELECTIONS]++;
  reset_timer(D, x, me);
  uint32_t last = ND(NF_LAST, me);
  uint32_t lt = term_at(D, x, me, last, ND(NF_SNAP, me), ND(NF_SNAPT, me));
  for (uint32_t p = 0; p < D.n; p++) {
    if (p == me) continue;
    net_send(D, x, me, p, M_RV_REQ, f_inc(f), term, me, last, lt, 0, 0);
    if (x.code != RUN) return;
  }
  rec_node(D, x, 1, 0, me, 0);
}

// ---------------------------------------------------------------- tester API (tester.rs)
struct T {  // the tester coroutine frame, in registers during a tester event
  uint32_t pc, res, helper;
  uint32_t l[T_NL];
  uint32_t h[T_NH];
  uint64_t hv;
};

DI uint32_t t_draw(const Dev& D, X& x, uint32_t& w1) {
  uint32_t w0;
  philox(D, x, x.t_ctr++, 0, ST_TESTER, w0, w1);
  return w0;
}
DI uint32_t t_range(const Dev& D, X& x, uint32_t lo, uint32_t hi) {
  uint32_t w1, w0 = t_draw(D, x, w1);
  return u_range(w0, lo, hi);
}
DI bool t_bool(const Dev& D, X& x, uint32_t p_q32) {
  uint32_t w1;
  return t_draw(D, x, w1) < p_q32;
}
DI uint64_t t_entry(const Dev& D, X& x) {  // tests.rs:943-951 gen_entry
  uint32_t w1, w0 = t_draw(D, x, w1);
  return ((uint64_t)w1 << 32) | w0;
}
DI void t_set_unrel(X& x, bool u) { x.netmode = (x.netmode & ~1u) | (u ? 1u : 0u); }
DI bool t_started(const Dev& D, X& x, uint32_t i) { return f_alive(ND(NF_FLAGS, i)); }
DI bool t_connected(const Dev& D, X& x, uint32_t i) { return f_conn(ND(NF_FLAGS, i)); }
DI void t_conn(const Dev& D, X& x, uint32_t i, uint32_t v) {
  ND(NF_FLAGS, i) = f_set(ND(NF_FLAGS, i), 3, 1, v);
}
DI void t_crash1(const Dev& D, X& x, uint32_t i) {  // tester.rs:329-333
  ND(NF_FLAGS, i) = f_set(ND(NF_FLAGS, i), 2, 1, 0u);
  ND(NF_TIMER, i) = INF_T;
}
DI void t_start1(const Dev& D, X& x, uint32_t i) {  // tester.rs:293-327, raft.rs:108-122
  t_crash1(D, x, i);
  uint32_t f = ND(NF_FLAGS, i);
  f = f_set(f, 2, 1, 1u);
  f = f_set(f, 8, 8, f_inc(f) + 1u);
  f = f_set(f_set(f, 0, 2, R_F), 16, 8, 0u);
  ND(NF_FLAGS, i) = f;
  uint32_t snap = ND(NF_SNAP, i);
  ND(NF_COMMIT, i) = snap;
  ND(NF_APPLIED, i) = snap;
  if (!D.null_raft) reset_timer(D, x, i);
}
DI void t_new(const Dev& D, X& x, bool snapshot) {  // RaftTester::new, tester.rs:34-60
  x.netmode = (x.netmode & ~2u) | (snapshot ? 2u : 0u);
  for (uint32_t i = 0; i < D.n; i++) { t_start1(D, x, i); t_conn(D, x, i, 1); }
  if (D.unrel_flag) t_set_unrel(x, true);
}
// tester.rs:165-171 -> raft.rs:238-244; unwrap() on a crashed raft panics
DI bool t_start(const Dev& D, X& x, uint32_t i, uint64_t v, uint32_t& idx, uint32_t& term) {
  uint32_t f = ND(NF_FLAGS, i);
  if (!f_alive(f)) { fail(D, x, MR_FAIL_UNWRAP_NONE); return false; }
  if (D.null_raft || f_role(f) != R_L) return false;  // Err(NotLeader((me+1)%n))
  uint32_t snap = ND(NF_SNAP, i), last = ND(NF_LAST, i) + 1;
  if (last - snap > D.log_cap) { fail(D, x, MR_FAIL_SIM_CAPACITY); return false; }
  size_t li = logi(D, x, i, last);
  term = ND(NF_TERM, i);
  D.lterm[li] = term;
  D.lval[li] = v;
  ND(NF_LAST, i) = last;
  if (last - snap > x.cnt[CNT_MAX_LOG]) x.cnt[CNT_MAX_LOG] = last - snap;
  PR(PF_MATCH, i, i) = last;
  idx = last;
  return true;
}
DI bool t_start(const Dev& D, X& x, uint32_t i, uint64_t v) {
  uint32_t a, b;
  return t_start(D, x, i, v, a, b);
}
DI uint32_t t_term(const Dev& D, X& x, uint32_t i) {
  if (!f_alive(ND(NF_FLAGS, i))) { fail(D, x, MR_FAIL_UNWRAP_NONE); return 0; }
  return ND(NF_TERM, i);
}
DI uint32_t t_log_size(const Dev& D, X& x) {  // tester.rs:152-158 + SEMANTICS §5 size model
  uint32_t mx = 0;
  for (uint32_t i = 0; i < D.n; i++) {
    uint32_t sz = 32u + (f_voted(ND(NF_FLAGS, i)) != 15u ? 9u : 1u) +
                  24u * (ND(NF_LAST, i) - ND(NF_SNAP, i));
    if (sz > mx) mx = sz;
  }
  return mx;
}
DI uint32_t t_check_terms(const Dev& D, X& x) {  // tester.rs:95-109
  uint32_t term = 0;
  for (uint32_t i = 0; i < D.n; i++) {
    uint32_t f = ND(NF_FLAGS, i);
    if (!f_conn(f)) continue;
    if (!f_alive(f)) { fail(D, x, MR_FAIL_UNWRAP_NONE); return 0; }
    uint32_t xt = ND(NF_TERM, i);
    if (term == 0) term = xt;
    else if (term != xt) { fail(D, x, MR_FAIL_TERM_DISAGREE); return 0; }
  }
  return term;
}
DI void t_check_no_leader(const Dev& D, X& x) {  // tester.rs:112-122
  for (uint32_t i = 0; i < D.n; i++) {
    uint32_t f = ND(NF_FLAGS, i);
    if (!f_conn(f)) continue;
    if (!f_alive(f)) { fail(D, x, MR_FAIL_UNWRAP_NONE); return; }
    if (!D.null_raft && f_role(f) == R_L) { fail(D, x, MR_FAIL_UNEXPECTED_LEADER); return; }
  }
}
DI void t_sleep(X& x, uint32_t us) { x.sleep_us = us; x.yield = 1; }
DI void t_end(const Dev& D, X& x) {  // tester.rs:339-358
  if (x.now > 120000000u) { fail(D, x, MR_FAIL_TIMEOUT_120S); return; }
  x.code = MR_PASS;
  rec_simple(D, x, 3, MR_PASS);
}

// ---- multi-event tester calls: step() returns true when done, false after
// scheduling a sleep or failing. Frame: t.h[0..4], t.hv; result in t.res / t.hv.

// check_one_leader, tester.rs:64-92. h0 iteration, h4 phase
DI void col_init(T& t) { t.h[0] = 0; t.h[4] = 1; }
DI bool col_step(const Dev& D, X& x, T& t) {
  for (;;) {
    if (t.h[4] == 1) {
      if (t.h[0] >= 10) { fail(D, x, MR_FAIL_ONE_LEADER_NONE); return false; }
      t_sleep(x, t_range(D, x, 450000u, 550000u));
      t.h[4] = 2;
      return false;
    }
    uint32_t best_term = 0, best = NONE, terms_seen = 0;
    for (uint32_t i = 0; i < D.n; i++) {
      uint32_t f = ND(NF_FLAGS, i);
      if (!f_conn(f)) continue;
      if (!f_alive(f)) { fail(D, x, MR_FAIL_UNWRAP_NONE); return false; }
      if (D.null_raft || f_role(f) != R_L) continue;
      uint32_t ti = ND(NF_TERM, i);
      for (uint32_t j = 0; j < i; j++) {  // >1 leaders in one term?
        uint32_t g = ND(NF_FLAGS, j);
        if (f_conn(g) && f_role(g) == R_L && ND(NF_TERM, j) == ti) {
          fail(D, x, MR_FAIL_MULTI_LEADER_TERM);
          return false;
        }
      }
      terms_seen++;
      if (best == NONE || ti > best_term) { best_term = ti; best = i; }
    }
    if (terms_seen) { t.res = best; return true; }
    t.h[0]++;
    t.h[4] = 1;
  }
}

// one(cmd, expected, retry), tester.rs:216-262.
// h0 t0, h1 starts, h2 index, h3 t1, h4 phase | expected << 8 | retry << 16; hv cmd
DI void one_init(const Dev& D, X& x, T& t, uint64_t cmd, uint32_t expected, bool retry) {
  t.hv = cmd;
  t.h[0] = x.now;
  t.h[1] = 0;
  t.h[4] = 1u | (expected << 8) | (retry ? 1u << 16 : 0u);
}
DI bool one_step(const Dev& D, X& x, T& t) {
  uint32_t expected = (t.h[4] >> 8) & 255u;
  bool retry = (t.h[4] >> 16) & 1u;
  for (;;) {
    if ((t.h[4] & 255u) == 1) {
      if (!(x.now - t.h[0] < 10000000u)) { fail(D, x, MR_FAIL_ONE_NO_AGREEMENT); return false; }
      uint32_t starts = t.h[1], index = 0, term;
      bool have = false;
      for (uint32_t k = 0; k < D.n; k++) {
        starts = (starts + 1) % D.n;
        uint32_t f = ND(NF_FLAGS, starts);
        if (!f_conn(f) || !f_alive(f)) continue;
        if (t_start(D, x, starts, t.hv, index, term)) { have = true; break; }
        if (x.code != RUN) return false;
      }
      t.h[1] = starts;
      if (!have) { t_sleep(x, 50000); return false; }
      t.h[2] = index;
      t.h[3] = x.now;
      t.h[4] = (t.h[4] & ~255u) | 2u;
    }
    if (!(x.now - t.h[3] < 2000000u)) {
      if (!retry) { fail(D, x, MR_FAIL_ONE_NO_AGREEMENT); return false; }
      t.h[4] = (t.h[4] & ~255u) | 1u;
      continue;
    }
    uint64_t v;
    uint32_t cnt = n_committed(D, x, t.h[2], v);
    if (cnt > 0 && cnt >= expected && v == t.hv) { t.res = t.h[2]; return true; }
    t_sleep(x, 20000);
    return false;
  }
}

// wait(index, n, start_term), tester.rs:175-201.
// h0 to, h1 iteration, h2 index, h3 start term, h4 phase | n << 8 | has_st << 16
// result: t.res = Some?, t.hv = value
DI void wait_init(T& t, uint32_t index, uint32_t nn, bool has_st, uint32_t st) {
  t.h[0] = 10000; t.h[1] = 0; t.h[2] = index; t.h[3] = st;
  t.h[4] = 1u | (nn << 8) | (has_st ? 1u << 16 : 0u);
}
DI bool wait_step(const Dev& D, X& x, T& t) {
  uint32_t nn = (t.h[4] >> 8) & 255u;
  uint64_t v;
  if ((t.h[4] & 255u) == 2) {
    if ((t.h[4] >> 16) & 1u) {
      for (uint32_t i = 0; i < D.n; i++)
        if (f_alive(ND(NF_FLAGS, i)) && ND(NF_TERM, i) > t.h[3]) { t.res = 0; return true; }
    }
    t.h[1]++;
    t.h[4] = (t.h[4] & ~255u) | 1u;
  }
  uint32_t cnt = n_committed(D, x, t.h[2], v);
  if (t.h[1] < 30 && cnt < nn) {
    t_sleep(x, t.h[0]);
    if (t.h[0] < 1000000u) t.h[0] *= 2;
    t.h[4] = (t.h[4] & ~255u) | 2u;
    return false;
  }
  if (cnt < nn) { fail(D, x, MR_FAIL_WAIT_TOO_FEW); return false; }
  t.res = cnt > 0 ? 1u : 0u;
  t.hv = v;
  return true;
}

// ---- protothreads: the scenario's persistent locals live in t.l[]; a
// yield stores the frame (pc = the source line) and returns. SLEEP returns to
// the event loop; AWAIT starts a multi-event tester call and returns to the
// dispatcher in tester(), which owns the only copy of each call's state
// machine and resumes the scenario at the same line once the call is done.
enum : uint32_t { H_NONE = 0, H_ONE, H_COL, H_WAIT };
#define PT_BEGIN switch (t.pc) { case 0:;
#define PT_END } fail(D, x, MR_FAIL_SIM_BAD_PROGRAM);
#define CK() do { if (x.code != RUN) return; } while (0)
#define SLEEP(us) do { t_sleep(x, (us)); t.pc = __LINE__; return; case __LINE__:; } while (0)
#define AWAIT(init, kind) do { init; t.helper = (kind); t.pc = __LINE__; return; case __LINE__:; } while (0)
#define ONE(cmd, expected, retry) AWAIT(one_init(D, x, t, (cmd), (expected), (retry)), H_ONE)
#define CHECK_ONE_LEADER() AWAIT(col_init(t), H_COL)
#define WAIT(idx, nn, has, st) AWAIT(wait_init(t, (idx), (nn), (has), (st)), H_WAIT)
#define TV(k) C64(C64_TV + (k))

// ---------------------------------------------------------------- scenarios (tests.rs)
DI void scn_initial_election(const Dev& D, X& x, T& t) {  // tests.rs:20-46
  PT_BEGIN
  t_new(D, x, false);
  CHECK_ONE_LEADER();
  SLEEP(50000);
  t_check_terms(D, x); CK();
  SLEEP(2 * ELECTION_US);
  t_check_terms(D, x); CK();
  CHECK_ONE_LEADER();
  t_end(D, x);
  return;
  PT_END
}

DI void scn_reelection(const Dev& D, X& x, T& t) {  // tests.rs:48-78
  const uint32_t n = D.n;
  uint32_t& l1 = t.l[0];
  uint32_t& l2 = t.l[1];
  PT_BEGIN
  t_new(D, x, false);
  CHECK_ONE_LEADER(); l1 = t.res;
  t_conn(D, x, l1, 0);
  CHECK_ONE_LEADER();
  t_conn(D, x, l1, 1);
  CHECK_ONE_LEADER(); l2 = t.res;
  t_conn(D, x, l2, 0);
  t_conn(D, x, (l2 + 1) % n, 0);
  SLEEP(2 * ELECTION_US);
  t_check_no_leader(D, x); CK();
  t_conn(D, x, (l2 + 1) % n, 1);
  CHECK_ONE_LEADER();
  t_conn(D, x, l2, 1);
  CHECK_ONE_LEADER();
  t_end(D, x);
  return;
  PT_END
}

DI void scn_many_election(const Dev& D, X& x, T& t) {  // tests.rs:80-112
  const uint32_t n = D.n;
  uint32_t& it = t.l[0];
  uint32_t& i1 = t.l[1];
  uint32_t& i2 = t.l[2];
  uint32_t& i3 = t.l[3];
  PT_BEGIN
  t_new(D, x, false);
  CHECK_ONE_LEADER();
  for (it = 0; it < D.iters; it++) {
    i1 = t_range(D, x, 0, n); i2 = t_range(D, x, 0, n); i3 = t_range(D, x, 0, n);
    t_conn(D, x, i1, 0); t_conn(D, x, i2, 0); t_conn(D, x, i3, 0);
    CHECK_ONE_LEADER();
    t_conn(D, x, i1, 1); t_conn(D, x, i2, 1); t_conn(D, x, i3, 1);
  }
  CHECK_ONE_LEADER();
  t_end(D, x);
  return;
  PT_END
}

DI void scn_basic_agree(const Dev& D, X& x, T& t) {  // tests.rs:114-130
  uint32_t& index = t.l[0];
  PT_BEGIN
  t_new(D, x, false);
  for (index = 1; index <= 3; index++) {
    {
      uint64_t v;
      if (n_committed(D, x, index, v) != 0) { fail(D, x, MR_FAIL_BASIC_PRECOMMIT); return; }
    }
    ONE((uint64_t)index * 100, D.n, false);
    if (t.res != index) { fail(D, x, MR_FAIL_BASIC_INDEX); return; }
  }
  t_end(D, x);
  return;
  PT_END
}

DI void scn_fail_agree(const Dev& D, X& x, T& t) {  // tests.rs:132-161
  const uint32_t n = D.n;
  uint32_t& leader = t.l[0];
  PT_BEGIN
  t_new(D, x, false);
  ONE(101, n, false);
  CHECK_ONE_LEADER(); leader = t.res;
  t_conn(D, x, (leader + 1) % n, 0);
  ONE(102, n - 1, false);
  ONE(103, n - 1, false);
  SLEEP(ELECTION_US);
  ONE(104, n - 1, false);
  ONE(105, n - 1, false);
  t_conn(D, x, (leader + 1) % n, 1);
  ONE(106, n, true);
  SLEEP(ELECTION_US);
  ONE(107, n, true);
  t_end(D, x);
  return;
  PT_END
}

DI void scn_fail_no_agree(const Dev& D, X& x, T& t) {  // tests.rs:163-209
  const uint32_t n = D.n;
  uint32_t& leader = t.l[0];
  uint32_t& index = t.l[1];
  PT_BEGIN
  t_new(D, x, false);
  ONE(10, n, false);
  CHECK_ONE_LEADER(); leader = t.res;
  t_conn(D, x, (leader + 1) % n, 0);
  t_conn(D, x, (leader + 2) % n, 0);
  t_conn(D, x, (leader + 3) % n, 0);
  {
    uint32_t term;
    bool ok = t_start(D, x, leader, 20, index, term);
    CK();
    if (!ok) { fail(D, x, MR_FAIL_LEADER_REJECTED); return; }
  }
  if (index != 2) { fail(D, x, MR_FAIL_EXPECTED_INDEX2); return; }
  SLEEP(2 * ELECTION_US);
  {
    uint64_t v;
    if (n_committed(D, x, index, v) != 0) { fail(D, x, MR_FAIL_NO_MAJORITY_COMMIT); return; }
  }
  t_conn(D, x, (leader + 1) % n, 1);
  t_conn(D, x, (leader + 2) % n, 1);
  t_conn(D, x, (leader + 3) % n, 1);
  CHECK_ONE_LEADER();
  {
    uint32_t idx2, term;
    bool ok = t_start(D, x, t.res, 30, idx2, term);
    CK();
    if (!ok) { fail(D, x, MR_FAIL_LEADER_REJECTED); return; }
    if (idx2 < 2 || idx2 > 3) { fail(D, x, MR_FAIL_UNEXPECTED_INDEX); return; }
  }
  ONE(1000, n, true);
  t_end(D, x);
  return;
  PT_END
}

// (0..servers).any(|j| t.term(j) != term) with unwrap() semantics
DI bool any_term_changed(const Dev& D, X& x, uint32_t term) {
  for (uint32_t j = 0; j < D.n; j++) {
    uint32_t tj = t_term(D, x, j);
    if (x.code != RUN) return false;
    if (tj != term) return true;
  }
  return false;
}

DI void scn_concurrent_starts(const Dev& D, X& x, T& t) {  // tests.rs:211-275
  const uint32_t n = D.n;
  uint32_t& tried = t.l[0];
  uint32_t& term = t.l[1];
  uint32_t& ni = t.l[2];   // idxes in TV(0..5)
  uint32_t& q = t.l[3];
  uint32_t& nc = t.l[4];   // cmds in TV(8..13)
  PT_BEGIN
  t_new(D, x, false);
  for (tried = 0; tried < 5; tried++) {
    if (tried > 0) SLEEP(3000000);
    CHECK_ONE_LEADER();
    {
      uint32_t leader = t.res, idx, st;
      bool ok = t_start(D, x, leader, 1, idx, term);
      CK();
      if (!ok) continue;
      ni = 0;
      for (uint32_t ii = 0; ii < 5; ii++) {
        bool ok2 = t_start(D, x, leader, 100 + ii, idx, st);
        CK();
        if (ok2 && st == term) { TV(ni) = idx; ni++; }
      }
    }
    {
      bool ch = any_term_changed(D, x, term);
      CK();
      if (ch) continue;
    }
    nc = 0;
    for (q = 0; q < ni; q++) {
      WAIT((uint32_t)TV(q), n, true, term);
      if (t.res) { TV(8 + nc) = t.hv; nc++; }
    }
    for (uint32_t ii = 0; ii < 5; ii++) {
      bool ok = false;
      for (uint32_t k = 0; k < nc; k++)
        if (TV(8 + k) == 100 + ii) ok = true;
      if (!ok) { fail(D, x, MR_FAIL_CMD_MISSING); return; }
    }
    t_end(D, x);  // success -> break; assert!(success); t.end()
    return;
  }
  fail(D, x, MR_FAIL_TERM_CHANGED);
  return;
  PT_END
}

DI void scn_rejoin(const Dev& D, X& x, T& t) {  // tests.rs:277-313
  const uint32_t n = D.n;
  uint32_t& l1 = t.l[0];
  uint32_t& l2 = t.l[1];
  PT_BEGIN
  t_new(D, x, false);
  ONE(101, n, true);
  CHECK_ONE_LEADER(); l1 = t.res;
  t_conn(D, x, l1, 0);
  t_start(D, x, l1, 102); CK();
  t_start(D, x, l1, 103); CK();
  t_start(D, x, l1, 104); CK();
  ONE(103, 2, true);
  CHECK_ONE_LEADER(); l2 = t.res;
  t_conn(D, x, l2, 0);
  t_conn(D, x, l1, 1);
  ONE(104, 2, true);
  t_conn(D, x, l2, 1);
  ONE(105, n, true);
  t_end(D, x);
  return;
  PT_END
}

DI void scn_backup(const Dev& D, X& x, T& t) {  // tests.rs:315-386
  const uint32_t n = D.n;
  uint32_t& l1 = t.l[0];
  uint32_t& l2 = t.l[1];
  uint32_t& other = t.l[2];
  uint32_t& i = t.l[3];
  PT_BEGIN
  t_new(D, x, false);
  ONE(t_entry(D, x), n, true);
  CHECK_ONE_LEADER(); l1 = t.res;
  t_conn(D, x, (l1 + 2) % n, 0); t_conn(D, x, (l1 + 3) % n, 0); t_conn(D, x, (l1 + 4) % n, 0);
  for (uint32_t k = 0; k < 50; k++) {
    uint64_t e = t_entry(D, x);
    t_start(D, x, l1, e); CK();
  }
  SLEEP(ELECTION_US / 2);
  t_conn(D, x, (l1 + 0) % n, 0); t_conn(D, x, (l1 + 1) % n, 0);
  t_conn(D, x, (l1 + 2) % n, 1); t_conn(D, x, (l1 + 3) % n, 1); t_conn(D, x, (l1 + 4) % n, 1);
  for (i = 0; i < 50; i++) ONE(t_entry(D, x), 3, true);
  CHECK_ONE_LEADER(); l2 = t.res;
  other = (l1 + 2) % n;
  if (l2 == other) other = (l2 + 1) % n;
  t_conn(D, x, other, 0);
  for (uint32_t k = 0; k < 50; k++) {
    uint64_t e = t_entry(D, x);
    t_start(D, x, l2, e); CK();
  }
  SLEEP(ELECTION_US / 2);
  for (uint32_t k = 0; k < n; k++) t_conn(D, x, k, 0);
  t_conn(D, x, (l1 + 0) % n, 1); t_conn(D, x, (l1 + 1) % n, 1); t_conn(D, x, other, 1);
  for (i = 0; i < 50; i++) ONE(t_entry(D, x), 3, true);
  for (uint32_t k = 0; k < n; k++) t_conn(D, x, k, 1);
  ONE(t_entry(D, x), n, true);
  t_end(D, x);
  return;
  PT_END
}

DI void scn_count(const Dev& D, X& x, T& t) {  // tests.rs:388-479
  const uint32_t n = D.n;
  uint32_t& total1 = t.l[0];
  uint32_t& total2 = t.l[1];
  uint32_t& tried = t.l[2];
  uint32_t& starti = t.l[3];
  uint32_t& term = t.l[4];
  uint32_t& i = t.l[5];
  PT_BEGIN
  t_new(D, x, false);
  CHECK_ONE_LEADER();
  total1 = x.msgs_sent / 2;
  if (total1 < 1 || total1 > 30) { fail(D, x, MR_FAIL_RPC_INITIAL); return; }
  total2 = 0;
  for (tried = 0; tried < 5; tried++) {
    if (tried > 0) SLEEP(3000000);
    CHECK_ONE_LEADER();
    total1 = x.msgs_sent / 2;
    {
      uint32_t leader = t.res, idx, st;
      bool ok = t_start(D, x, leader, 1, starti, term);
      CK();
      if (!ok) continue;
      bool outer = false;
      for (uint32_t k = 1; k < 10 + 2; k++) {
        uint64_t xv = t_entry(D, x);  // random.gen::<u64>()
        TV(k - 1) = xv;
        bool ok2 = t_start(D, x, leader, xv, idx, st);
        CK();
        if (!ok2 || st != term) { outer = true; break; }
        if (starti + k != idx) { fail(D, x, MR_FAIL_START_FAILED); return; }
      }
      if (outer) continue;
    }
    for (i = 1; i <= 10; i++) {
      WAIT(starti + i, n, true, term);
      if (t.res && t.hv != TV(i - 1)) { fail(D, x, MR_FAIL_WRONG_VALUE); return; }
    }
    {
      bool ch = any_term_changed(D, x, term);
      CK();
      if (ch) continue;
    }
    total2 = x.msgs_sent / 2;
    if (total2 - total1 > (10 + 1 + 3) * 3) { fail(D, x, MR_FAIL_RPC_TOO_MANY); return; }
    break;
  }
  if (tried >= 5) { fail(D, x, MR_FAIL_TERM_CHANGED); return; }
  SLEEP(ELECTION_US);
  if (x.msgs_sent / 2 - total2 > 3 * 20) { fail(D, x, MR_FAIL_RPC_IDLE); return; }
  t_end(D, x);
  return;
  PT_END
}

DI void scn_persist1(const Dev& D, X& x, T& t) {  // tests.rs:481-526
  const uint32_t n = D.n;
  uint32_t& l = t.l[0];
  PT_BEGIN
  t_new(D, x, false);
  ONE(11, n, true);
  for (uint32_t i = 0; i < n; i++) t_start1(D, x, i);
  for (uint32_t i = 0; i < n; i++) { t_conn(D, x, i, 0); t_conn(D, x, i, 1); }
  ONE(12, n, true);
  CHECK_ONE_LEADER(); l = t.res;
  t_conn(D, x, l, 0); t_start1(D, x, l); t_conn(D, x, l, 1);
  ONE(13, n, true);
  CHECK_ONE_LEADER(); l = t.res;
  t_conn(D, x, l, 0);
  ONE(14, n - 1, true);
  t_start1(D, x, l); t_conn(D, x, l, 1);
  WAIT(4, n, false, 0);
  CHECK_ONE_LEADER(); l = (t.res + 1) % n;
  t_conn(D, x, l, 0);
  ONE(15, n - 1, true);
  t_start1(D, x, l); t_conn(D, x, l, 1);
  ONE(16, n, true);
  t_end(D, x);
  return;
  PT_END
}

DI void scn_persist2(const Dev& D, X& x, T& t) {  // tests.rs:528-572
  const uint32_t n = D.n;
  uint32_t& index = t.l[0];
  uint32_t& k = t.l[1];
  uint32_t& l1 = t.l[2];
  PT_BEGIN
  t_new(D, x, false);
  index = 1;
  for (k = 0; k < 5; k++) {
    ONE(10 + index, n, true); index++;
    CHECK_ONE_LEADER(); l1 = t.res;
    t_conn(D, x, (l1 + 1) % n, 0); t_conn(D, x, (l1 + 2) % n, 0);
    ONE(10 + index, n - 2, true); index++;
    t_conn(D, x, (l1 + 0) % n, 0); t_conn(D, x, (l1 + 3) % n, 0); t_conn(D, x, (l1 + 4) % n, 0);
    t_start1(D, x, (l1 + 1) % n); t_start1(D, x, (l1 + 2) % n);
    t_conn(D, x, (l1 + 1) % n, 1); t_conn(D, x, (l1 + 2) % n, 1);
    SLEEP(ELECTION_US);
    t_start1(D, x, (l1 + 3) % n); t_conn(D, x, (l1 + 3) % n, 1);
    ONE(10 + index, n - 2, true); index++;
    t_conn(D, x, (l1 + 4) % n, 1); t_conn(D, x, (l1 + 0) % n, 1);
  }
  ONE(1000, n, true);
  t_end(D, x);
  return;
  PT_END
}

DI void scn_persist3(const Dev& D, X& x, T& t) {  // tests.rs:574-602
  const uint32_t n = D.n;
  uint32_t& leader = t.l[0];
  PT_BEGIN
  t_new(D, x, false);
  ONE(101, 3, true);
  CHECK_ONE_LEADER(); leader = t.res;
  t_conn(D, x, (leader + 2) % n, 0);
  ONE(102, 2, true);
  t_crash1(D, x, (leader + 0) % n); t_crash1(D, x, (leader + 1) % n);
  t_conn(D, x, (leader + 2) % n, 1);
  t_start1(D, x, (leader + 0) % n); t_conn(D, x, (leader + 0) % n, 1);
  ONE(103, 2, true);
  t_start1(D, x, (leader + 1) % n); t_conn(D, x, (leader + 1) % n, 1);
  ONE(104, n, true);
  t_end(D, x);
  return;
  PT_END
}

DI uint32_t fig8_delay(const Dev& D, X& x) {  // tests.rs:631-635 / 711-715
  if (t_bool(D, x, LOSS_Q32)) return t_range(D, x, 0, ELECTION_US / 2);
  return t_range(D, x, 0, 13000);
}

// figure_8_2c (tests.rs:612-660); with `unreliable` the config-3 literal variant
DI void scn_figure_8(const Dev& D, X& x, T& t, bool unreliable) {
  const uint32_t n = D.n;
  uint32_t& nup = t.l[0];
  uint32_t& it = t.l[1];
  uint32_t& leader = t.l[2];
  PT_BEGIN
  t_new(D, x, false);
  if (unreliable) t_set_unrel(x, true);
  ONE(t_entry(D, x), 1, true);
  nup = n;
  for (it = 0; it < D.iters; it++) {
    leader = NONE;
    for (uint32_t i = 0; i < n; i++) {
      if (!t_started(D, x, i)) continue;
      uint64_t e = t_entry(D, x);
      bool ok = t_start(D, x, i, e);
      CK();
      if (ok) leader = i;
    }
    SLEEP(fig8_delay(D, x));
    if (leader != NONE) { t_crash1(D, x, leader); nup--; }
    if (nup < 3) {
      uint32_t s = t_range(D, x, 0, n);
      if (!t_started(D, x, s)) { t_start1(D, x, s); nup++; }
    }
  }
  for (uint32_t i = 0; i < n; i++)
    if (!t_started(D, x, i)) t_start1(D, x, i);
  ONE(t_entry(D, x), n, true);
  t_end(D, x);
  return;
  PT_END
}

DI void scn_figure_8_unreliable(const Dev& D, X& x, T& t) {  // tests.rs:688-741
  const uint32_t n = D.n;
  uint32_t& nup = t.l[0];
  uint32_t& it = t.l[1];
  uint32_t& leader = t.l[2];
  PT_BEGIN
  t_new(D, x, false);
  t_set_unrel(x, true);
  ONE(t_entry(D, x), 1, true);
  nup = n;
  for (it = 0; it < D.iters; it++) {
    leader = NONE;
    for (uint32_t i = 0; i < n; i++) {
      uint64_t e = t_entry(D, x);
      bool ok = t_start(D, x, i, e);
      CK();
      if (ok && t_connected(D, x, i)) leader = i;
    }
    SLEEP(fig8_delay(D, x));
    if (leader != NONE && t_range(D, x, 0, 1000) < ELECTION_US / 1000 / 2) {
      t_conn(D, x, leader, 0);
      nup--;
    }
    if (nup < 3) {
      uint32_t s = t_range(D, x, 0, n);
      if (!t_connected(D, x, s)) { t_conn(D, x, s, 1); nup++; }
    }
  }
  for (uint32_t i = 0; i < n; i++) t_conn(D, x, i, 1);
  ONE(t_entry(D, x), n, true);
  t_end(D, x);
  return;
  PT_END
}

DI void scn_snap_common(const Dev& D, X& x, T& t, bool disconnect, bool reliable, bool crash) {
  // tests.rs:858-911
  const uint32_t n = D.n;
  uint32_t& leader1 = t.l[0];
  uint32_t& i = t.l[1];
  uint32_t& victim = t.l[2];
  PT_BEGIN
  t_new(D, x, true);
  t_set_unrel(x, !reliable);
  ONE(t_entry(D, x), n, true);
  CHECK_ONE_LEADER(); leader1 = t.res;
  for (i = 0; i < D.iters; i++) {
    victim = (leader1 + 1) % n;
    if (i % 3 == 1) victim = leader1;
    if (disconnect) {
      t_conn(D, x, victim, 0);
      ONE(t_entry(D, x), n - 1, true);
    }
    if (crash) {
      t_crash1(D, x, victim);
      ONE(t_entry(D, x), n - 1, true);
    }
    {
      uint32_t sender = (i % 3 == 1) ? (leader1 + 1) % n : leader1;
      for (uint32_t k = 0; k <= 10; k++) {  // send enough to get a snapshot
        uint64_t e = t_entry(D, x);
        t_start(D, x, sender, e);
        CK();
      }
    }
    ONE(t_entry(D, x), n - 1, true);
    if (t_log_size(D, x) >= 2000) { fail(D, x, MR_FAIL_LOG_SIZE); return; }
    if (disconnect) {
      t_conn(D, x, victim, 1);
      ONE(t_entry(D, x), n, true);
      CHECK_ONE_LEADER(); leader1 = t.res;
    }
    if (crash) {
      t_start1(D, x, victim);
      t_conn(D, x, victim, 1);
      ONE(t_entry(D, x), n, true);
      CHECK_ONE_LEADER(); leader1 = t.res;
    }
  }
  t_end(D, x);
  return;
  PT_END
}

// one tester event: resume the cluster's coroutine until it sleeps or ends
DI void run_scenario(const Dev& D, X& x, T& t) {
  switch (D.scenario) {
    case MR_SCN_INITIAL_ELECTION_2A: scn_initial_election(D, x, t); break;
    case MR_SCN_REELECTION_2A: scn_reelection(D, x, t); break;
    case MR_SCN_MANY_ELECTION_2A: scn_many_election(D, x, t); break;
    case MR_SCN_BASIC_AGREE_2B: scn_basic_agree(D, x, t); break;
    case MR_SCN_FAIL_AGREE_2B: scn_fail_agree(D, x, t); break;
    case MR_SCN_FAIL_NO_AGREE_2B: scn_fail_no_agree(D, x, t); break;
    case MR_SCN_CONCURRENT_STARTS_2B: scn_concurrent_starts(D, x, t); break;
    case MR_SCN_REJOIN_2B: scn_rejoin(D, x, t); break;
    case MR_SCN_BACKUP_2B: scn_backup(D, x, t); break;
    case MR_SCN_COUNT_2B: scn_count(D, x, t); break;
    case MR_SCN_PERSIST1_2C: scn_persist1(D, x, t); break;
    case MR_SCN_PERSIST2_2C: scn_persist2(D, x, t); break;
    case MR_SCN_PERSIST3_2C: scn_persist3(D, x, t); break;
    case MR_SCN_FIGURE_8_2C: scn_figure_8(D, x, t, false); break;
    case MR_SCN_FIGURE_8_UNRELIABLE_CRASH: scn_figure_8(D, x, t, true); break;
    case MR_SCN_FIGURE_8_UNRELIABLE_2C: scn_figure_8_unreliable(D, x, t); break;
    case MR_SCN_SNAPSHOT_BASIC_2D: scn_snap_common(D, x, t, false, true, false); break;
    case MR_SCN_SNAPSHOT_INSTALL_2D: scn_snap_common(D, x, t, true, true, false); break;
    case MR_SCN_SNAPSHOT_INSTALL_UNRELIABLE_2D: scn_snap_common(D, x, t, true, false, false); break;
    case MR_SCN_SNAPSHOT_INSTALL_CRASH_2D: scn_snap_common(D, x, t, false, true, true); break;
    case MR_SCN_SNAPSHOT_INSTALL_UNRELIABLE_CRASH_2D:
      scn_snap_common(D, x, t, false, false, true);
      break;
    default: fail(D, x, MR_FAIL_SIM_BAD_PROGRAM); return;
  }
}

// one tester event: resume the cluster's coroutine until it sleeps or ends
DI void tester(const Dev& D, X& x) {
  T t;
  uint32_t pcw = CS(CS_TPC);
  t.pc = pcw & 0xFFFFFFu;
  t.helper = pcw >> 24;
  t.res = CS(CS_TRES);
#pragma unroll
  for (uint32_t k = 0; k < T_NL; k++) t.l[k] = CS(CS_TL + k);
#pragma unroll
  for (uint32_t k = 0; k < T_NH; k++) t.h[k] = CS(CS_TH + k);
  t.hv = C64(C64_THV);
  x.yield = 0;
  for (int guard = 0;; guard++) {
    if (guard > 4096) { fail(D, x, MR_FAIL_SIM_BAD_PROGRAM); return; }
    if (t.helper != H_NONE) {  // a multi-event tester call in progress
      bool done = t.helper == H_ONE   ? one_step(D, x, t)
                  : t.helper == H_COL ? col_step(D, x, t)
                                      : wait_step(D, x, t);
      if (x.code != RUN) return;
      if (!done) break;  // it slept
      t.helper = H_NONE;
    }
    run_scenario(D, x, t);
    if (x.code != RUN) return;
    if (x.yield) break;
    if (t.helper == H_NONE) { fail(D, x, MR_FAIL_SIM_BAD_PROGRAM); return; }
  }
  rec_simple(D, x, 2, 0);  // time::sleep closes this tester segment (SEMANTICS §7)
  uint64_t target = (uint64_t)x.now + x.sleep_us;
  if (target >= INF_T) { fail(D, x, MR_FAIL_SIM_CAPACITY); return; }
  CS(CS_TWAKE) = (uint32_t)target;
  CS(CS_TPC) = t.pc | (t.helper << 24);
  CS(CS_TRES) = t.res;
#pragma unroll
  for (uint32_t k = 0; k < T_NL; k++) CS(CS_TL + k) = t.l[k];
#pragma unroll
  for (uint32_t k = 0; k < T_NH; k++) CS(CS_TH + k) = t.h[k];
  C64(C64_THV) = t.hv;
}

// ---------------------------------------------------------------- kernels
constexpr uint32_t CLS_MSG = 0, CLS_TIMER = 1, CLS_TESTER = 2, CLS_NONE = 3;

#ifndef MR_WAVES_PER_EU
#define MR_WAVES_PER_EU 2
#endif
__global__ void __launch_bounds__(256, MR_WAVES_PER_EU) step_kernel(Dev D, uint32_t budget) {
  X x;
  x.c = blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = x.c < D.C;
  x.code = in ? CS(CS_CODE) : (uint32_t)MR_PASS;
  if (x.code == RUN) {
    x.now = CS(CS_NOW); x.events = CS(CS_EVENTS); x.msgs_sent = CS(CS_MSGS);
    x.inflight = CS(CS_INFLIGHT); x.trace_n = CS(CS_TRACEN); x.mslot = CS(CS_MSLOT);
    x.netmode = CS(CS_NETMODE); x.t_ctr = CS(CS_TCTR);
    x.free_mask = C64(C64_FREE); x.digest = C64(C64_DIGEST); x.mmin = C64(C64_MMIN);
#pragma unroll
    for (uint32_t k = 0; k < CNT__N; k++) x.cnt[k] = CS(CS_CNT + k);
  }
  const bool live = x.code == RUN;
  uint64_t key = 0;
  uint32_t cls = CLS_NONE, node = 0;
  bool need = true;
  for (uint32_t it = 0; it < budget; it++) {
    const bool run = x.code == RUN;
    if (__ballot(run) == 0) break;
    if (run && need) {  // next event: min over tester wake-up, node timers, earliest message
      key = ((uint64_t)CS(CS_TWAKE) << 32) | (2ull << 30);
      cls = CLS_TESTER;
      for (uint32_t d = 0; d < D.n; d++) {
        uint64_t kt = ((uint64_t)ND(NF_TIMER, d) << 32) | (1ull << 30) | d;
        if (kt < key) { key = kt; cls = CLS_TIMER; node = d; }
      }
      if (x.mmin < key) { key = x.mmin; cls = CLS_MSG; }
      need = false;
    }
    // wave-uniform choice of the event class processed this iteration
    const uint32_t nm = __popcll(__ballot(run && cls == CLS_MSG));
    const uint32_t nt = __popcll(__ballot(run && cls == CLS_TIMER));
    const uint32_t ns = __popcll(__ballot(run && cls == CLS_TESTER));
    const uint32_t pick = (2 * ns >= nm + nt + ns) ? CLS_TESTER : (nm >= nt ? CLS_MSG : CLS_TIMER);
    if (!run || cls != pick) continue;
    x.now = (uint32_t)(key >> 32);
    need = true;
    x.events++;
    if (x.events > D.max_events) { fail(D, x, MR_FAIL_SIM_EVENT_LIMIT); continue; }
    if (pick == CLS_MSG) {
      x.cnt[CNT_EV_MSG]++;
      deliver(D, x, x.mslot, (uint32_t)key & 0x3FFFFFFFu);
    } else if (pick == CLS_TIMER) {
      x.cnt[CNT_EV_TIMER]++;
      on_timer(D, x, node);
    } else {
      x.cnt[CNT_EV_TESTER]++;
      tester(D, x);
    }
  }
  if (!live) return;
  CS(CS_CODE) = x.code;
  if (x.code != RUN) CS(CS_VTIME) = x.now;
  CS(CS_NOW) = x.now; CS(CS_EVENTS) = x.events; CS(CS_MSGS) = x.msgs_sent;
  CS(CS_INFLIGHT) = x.inflight; CS(CS_TRACEN) = x.trace_n; CS(CS_MSLOT) = x.mslot;
  CS(CS_NETMODE) = x.netmode; CS(CS_TCTR) = x.t_ctr;
  C64(C64_FREE) = x.free_mask; C64(C64_DIGEST) = x.digest; C64(C64_MMIN) = x.mmin;
#pragma unroll
  for (uint32_t k = 0; k < CNT__N; k++) CS(CS_CNT + k) = x.cnt[k];
  if (x.code == RUN) atomicAdd(D.remaining, 1u);
}

// RaftTester state before the test body runs (SEMANTICS §3: tester wakes at t = 0)
__global__ void __launch_bounds__(256) reset_kernel(Dev D) {
  X x;
  x.c = blockIdx.x * blockDim.x + threadIdx.x;
  if (x.c >= D.C) return;
  for (uint32_t f = 0; f < CS__N; f++) CS(f) = 0;
  CS(CS_CODE) = RUN;
  for (uint32_t f = 0; f < C64__N; f++) C64(f) = 0;
  C64(C64_FREE) = D.M >= 64 ? ~0ull : ((1ull << D.M) - 1ull);
  C64(C64_DIGEST) = FNV_OFF;
  C64(C64_MMIN) = ~0ull;
  for (uint32_t d = 0; d < D.n; d++) {
    for (uint32_t f = 0; f < NF__N; f++) ND(f, d) = 0;
    ND(NF_FLAGS, d) = 15u << 4;  // follower, down, disconnected, voted none
    ND(NF_TIMER, d) = INF_T;
    ND(NF_SLEN, d) = 1;
    NSV(d) = 0;
    for (uint32_t p = 0; p < D.n; p++) { PR(PF_NEXT, d, p) = 0; PR(PF_MATCH, d, p) = 0; }
  }
  for (uint32_t s = 0; s < D.M; s++) MS64(M64_KEY, s * D.C + x.c) = ~0ull;
}

// counters_reduce: per-GPU sums / maxima / verdict histogram / first failing
// cluster; out[] layout documented in mr_host.cpp (RED_*)
__global__ void __launch_bounds__(256) reduce_kernel(Dev D, unsigned long long* out,
                                                    uint64_t cluster_base) {
  __shared__ unsigned long long acc[CNT__N + 8 + 64];
  for (uint32_t i = threadIdx.x; i < CNT__N + 8 + 64; i += blockDim.x) acc[i] = 0;
  __syncthreads();
  X x;
  x.c = blockIdx.x * blockDim.x + threadIdx.x;
  if (x.c < D.C) {
    for (uint32_t k = 0; k < CNT__N; k++) {
      unsigned long long v = CS(CS_CNT + k);
      if (k >= CNT_MAX_INFLIGHT) atomicMax(&acc[k], v);
      else atomicAdd(&acc[k], v);
    }
    uint32_t code = CS(CS_CODE);
    atomicAdd(&acc[CNT__N + 0], (unsigned long long)CS(CS_EVENTS));
    atomicAdd(&acc[CNT__N + 1], (unsigned long long)CS(CS_MSGS));
    atomicAdd(&acc[CNT__N + 2], (unsigned long long)CS(CS_VTIME));
    atomicAdd(&acc[CNT__N + 3], code != RUN ? 1ull : 0ull);
    atomicAdd(&acc[CNT__N + 4], code == MR_PASS ? 1ull : 0ull);
    if (code != RUN) atomicAdd(&acc[CNT__N + 8 + (code < 63 ? code : 63)], 1ull);
    if (code != RUN && code != MR_PASS)
      atomicMin(&out[CNT__N + 5], (unsigned long long)(cluster_base + x.c));
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < CNT__N + 8 + 64; i += blockDim.x) {
    if (i == CNT__N + 5 || i == CNT__N + 6 || i == CNT__N + 7) continue;
    if (acc[i] == 0) continue;
    if (i >= CNT_MAX_INFLIGHT && i < CNT__N) atomicMax(&out[i], acc[i]);
    else atomicAdd(&out[i], acc[i]);
  }
}

hipError_t launch_step(const Dev& D, uint32_t budget, hipStream_t s) {
  dim3 blk(256), grd((D.C + 255) / 256);
  hipLaunchKernelGGL(step_kernel, grd, blk, 0, s, D, budget);
  return hipGetLastError();
}
hipError_t launch_reset(const Dev& D, hipStream_t s) {
  dim3 blk(256), grd((D.C + 255) / 256);
  hipLaunchKernelGGL(reset_kernel, grd, blk, 0, s, D);
  return hipGetLastError();
}
hipError_t launch_reduce(const Dev& D, unsigned long long* out, uint64_t cluster_base,
                         hipStream_t s) {
  dim3 blk(256), grd((D.C + 255) / 256);
  hipLaunchKernelGGL(reduce_kernel, grd, blk, 0, s, D, out, cluster_base);
  return hipGetLastError();
}

}  // namespace mr
