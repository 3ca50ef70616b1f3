// mr_kernel.hip — CDNA4 (gfx950) kernels of the batched Raft simulator.
//
// step_kernel: one lane owns one cluster (one seed of one reference test) and
// advances it through up to `budget` events of the discrete-event schedule of
// docs/SEMANTICS.md §3: pick the minimum (time, class, tie) key over the
// cluster's node timers, its cached earliest in-flight message and its tester
// wake-up; process it (node handler, tester program segment); repeat. State
// lives in HBM in the cluster-minor SoA of mr_dev.h. This replaces, for a
// whole batch at once, the madsim executor + net + fs + rand, the Raft node
// (src/raft/raft.rs) and the tester (src/raft/tester.rs, src/raft/tests.rs).
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

// per-lane registers of one cluster during a launch
struct X {
  uint32_t c, now, events, msgs_sent, inflight, code, trace_n, mslot, netmode, t_ctr;
  uint32_t k0, k1, loss, lat_lo, lat_hi;
  uint64_t free_mask, digest, mmin;
  uint32_t cnt[CNT__N];
};

#define ND(arr, d) D.arr[(size_t)(d) * D.C + x.c]
#define PR(arr, d, p) D.arr[((size_t)(d) * D.n + (p)) * D.C + x.c]

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

// Philox4x32-10, counter (ctr, ent, stream, 0), key (k0, k1); returns w0, w1
DI void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t k0, uint32_t k1, uint32_t& w0,
               uint32_t& w1) {
  uint32_t c3 = 0;
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

DI void set_net(X& x) {  // tester.rs:127-137
  if (x.netmode & 1u) { x.loss = LOSS_Q32; x.lat_lo = 1000; x.lat_hi = 27000; }
  else { x.loss = 0; x.lat_lo = 1000; x.lat_hi = 10000; }
}

// ---------------------------------------------------------------- trace
DI void rec8(const Dev& D, X& x, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4,
             uint32_t w5, uint32_t w6, uint32_t w7) {
  uint64_t h = x.digest;
  h = (h ^ w0) * FNV_P; h = (h ^ w1) * FNV_P; h = (h ^ w2) * FNV_P; h = (h ^ w3) * FNV_P;
  h = (h ^ w4) * FNV_P; h = (h ^ w5) * FNV_P; h = (h ^ w6) * FNV_P; h = (h ^ w7) * FNV_P;
  x.digest = h;
  if (x.c < D.trace_clusters) {
    if (x.trace_n < D.trace_cap) {
      uint32_t* p = reinterpret_cast<uint32_t*>(D.trace + (size_t)x.c * D.trace_cap + x.trace_n);
      p[0] = w0; p[1] = w1; p[2] = w2; p[3] = w3; p[4] = w4; p[5] = w5; p[6] = w6; p[7] = w7;
    }
  }
  x.trace_n++;
}

DI void rec_node(const Dev& D, X& x, uint32_t cls, uint32_t kind, uint32_t d, uint32_t aux) {
  uint32_t f = ND(nflags, d);
  uint32_t role = f_alive(f) ? f_role(f) : R_DOWN;
  rec8(D, x, x.now, cls | (kind << 8) | (d << 16) | (role << 24), aux, ND(nterm, d),
       ND(ncommit, d), ND(napplied, d), ND(nlast, d), ND(nsnap, d));
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
  uint32_t ctr = ND(nectr, d);
  ND(nectr, d) = ctr + 1;
  uint32_t w0, w1;
  philox(ctr, d, ST_ELECT, x.k0, x.k1, w0, w1);
  ND(ntimer, d) = x.now + u_range(w0, D.elo, D.ehi);
}

DI void rescan_min(const Dev& D, X& x) {
  uint64_t best = ~0ull;
  uint32_t bs = 0;
  for (uint32_t s = 0; s < D.M; s++) {
    uint64_t k = D.mkey[(size_t)s * D.C + x.c];
    if (k < best) { best = k; bs = s; }
  }
  x.mmin = best;
  x.mslot = bs;
}

// madsim net send (tester.rs:127-137, :147-149). Returns the slot or -1.
DI int net_send(const Dev& D, X& x, uint32_t src, uint32_t dst, uint32_t type, uint32_t inc,
                uint32_t term, uint32_t a, uint32_t b, uint32_t c, uint64_t v, uint32_t k) {
  uint32_t seq = x.msgs_sent++;
  uint32_t ctr = ND(nnctr, src);
  ND(nnctr, src) = ctr + 1;
  if (!f_conn(ND(nflags, src)) || !f_conn(ND(nflags, dst))) { x.cnt[CNT_DROP_CLOG]++; return -1; }
  uint32_t w0, w1;
  philox(ctr, src, ST_NET, x.k0, x.k1, w0, w1);
  if (w0 < x.loss) { x.cnt[CNT_DROP_LOSS]++; return -1; }
  if (x.inflight >= D.M) { x.cnt[CNT_DROP_OVERFLOW]++; return -1; }
  if (seq >= (1u << 30)) { fail(D, x, MR_FAIL_SIM_CAPACITY); return -1; }
  uint32_t t = x.now + u_range(w1, x.lat_lo, x.lat_hi);
  uint32_t slot = (uint32_t)__builtin_ctzll(x.free_mask);
  x.free_mask &= ~(1ull << slot);
  uint64_t key = ((uint64_t)t << 32) | seq;
  size_t mi = (size_t)slot * D.C + x.c;
  D.mkey[mi] = key;
  D.mhdr[mi] = type | (src << 3) | (dst << 6) | (inc << 9) | (k << 17);
  D.mterm[mi] = term; D.ma[mi] = a; D.mb[mi] = b; D.mc[mi] = c; D.mv[mi] = v;
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
  uint32_t len = ND(slen, i);
  if (idx > len) { fail(D, x, MR_FAIL_APPLY_OUT_OF_ORDER); return; }  // tester.rs:393
  if (idx == len) {
    D.sval[si] = v;
    D.smask[si] = (uint8_t)(m | (1u << i));
    ND(slen, i) = len + 1;
    if (idx > x.cnt[CNT_MAX_INDEX]) x.cnt[CNT_MAX_INDEX] = idx;
  }
}

DI void storage_snapshot(const Dev& D, X& x, uint32_t i, uint32_t idx) {  // tester.rs:399-402
  if (idx >= D.apply_cap) { fail(D, x, MR_FAIL_SIM_CAPACITY); return; }
  uint32_t nl = idx + 1, len = ND(slen, i);
  for (uint32_t j = nl; j < len; j++) {
    size_t si = (size_t)x.c * D.apply_cap + j;
    D.smask[si] = (uint8_t)(D.smask[si] & ~(1u << i));
  }
  ND(slen, i) = nl;
}

DI void n_committed(const Dev& D, X& x, uint32_t idx, uint32_t& cnt, uint64_t& v) {
  if (idx >= D.apply_cap) { cnt = 0; v = 0; return; }
  size_t si = (size_t)x.c * D.apply_cap + idx;
  cnt = (uint32_t)__builtin_popcount((uint32_t)D.smask[si]);
  v = D.sval[si];
}

// ---------------------------------------------------------------- Raft node
DI void node_apply(const Dev& D, X& x, uint32_t me) {  // tester.rs:302-325 applier
  uint32_t applied = ND(napplied, me), commit = ND(ncommit, me);
  uint32_t snap = ND(nsnap, me), snapt = ND(nsnapt, me);
  bool snapmode = (x.netmode >> 1) & 1u;
  while (applied < commit) {
    applied++;
    uint64_t v = D.lval[logi(D, x, me, applied)];
    push_and_check(D, x, me, applied, v);
    if (x.code != RUN) return;
    if (snapmode && (applied + 1) % 10u == 0 && applied > snap) {
      snapt = term_at(D, x, me, applied, snap, snapt);
      snap = applied;
      ND(nsnap, me) = snap; ND(nsnapt, me) = snapt; ND(nsnapv, me) = v;
      x.cnt[CNT_SNAPSHOTS]++;
    }
  }
  ND(napplied, me) = applied;
}

DI void send_append(const Dev& D, X& x, uint32_t l, uint32_t p) {
  uint32_t nx = PR(nnext, l, p), snap = ND(nsnap, l), snapt = ND(nsnapt, l), term = ND(nterm, l);
  uint32_t inc = f_inc(ND(nflags, l));
  if (nx <= snap) {
    net_send(D, x, l, p, M_IS_REQ, inc, term, snap, snapt, 0, ND(nsnapv, l), 0);
    return;
  }
  uint32_t prev = nx - 1, last = ND(nlast, l);
  uint32_t k = last - prev;
  if (k > D.K) k = D.K;
  uint32_t pt = term_at(D, x, l, prev, snap, snapt);
  x.cnt[CNT_SHIPPED] += k;
  int slot = net_send(D, x, l, p, M_AE_REQ, inc, term, prev, pt, ND(ncommit, l), 0, k);
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
  ND(nflags, me) = f_set(ND(nflags, me), 0, 2, R_L);
  x.cnt[CNT_LEADERS]++;
  uint32_t last = ND(nlast, me);
  for (uint32_t p = 0; p < D.n; p++) { PR(nnext, me, p) = last + 1; PR(nmatch, me, p) = 0; }
  PR(nmatch, me, me) = last;
  for (uint32_t p = 0; p < D.n; p++) {
    if (p == me) continue;
    send_append(D, x, me, p);
    if (x.code != RUN) return;
  }
  ND(ntimer, me) = x.now + D.hb;
}

// commit = the majority-th largest match index, if it is from the current term
DI void advance_commit(const Dev& D, X& x, uint32_t me) {
  uint32_t last = ND(nlast, me);
  uint32_t mv[MR_MAX_NODES];
#pragma unroll
  for (uint32_t p = 0; p < MR_MAX_NODES; p++)
    mv[p] = (p < D.n) ? ((p == me) ? last : PR(nmatch, me, p)) : 0u;
  uint32_t maj = D.n / 2 + 1, N = 0;
#pragma unroll
  for (uint32_t i = 0; i < MR_MAX_NODES; i++) {
    uint32_t ge = 0;
#pragma unroll
    for (uint32_t j = 0; j < MR_MAX_NODES; j++) ge += (j < D.n && mv[j] >= mv[i]) ? 1u : 0u;
    if (i < D.n && ge >= maj && mv[i] > N) N = mv[i];
  }
  if (N > ND(ncommit, me) &&
      term_at(D, x, me, N, ND(nsnap, me), ND(nsnapt, me)) == ND(nterm, me)) {
    ND(ncommit, me) = N;
    node_apply(D, x, me);
  }
}

DI void on_ack(const Dev& D, X& x, uint32_t me, uint32_t p, uint32_t xv) {
  if (xv > PR(nmatch, me, p)) PR(nmatch, me, p) = xv;
  if (xv + 1 > PR(nnext, me, p)) PR(nnext, me, p) = xv + 1;
  advance_commit(D, x, me);
  if (x.code != RUN) return;
  if (PR(nnext, me, p) <= ND(nlast, me)) send_append(D, x, me, p);
}

DI void deliver(const Dev& D, X& x, uint32_t slot, uint32_t seq) {
  size_t mi = (size_t)slot * D.C + x.c;
  uint32_t hdr = D.mhdr[mi];
  uint32_t type = hdr & 7u, src = (hdr >> 3) & 7u, me = (hdr >> 6) & 7u, inc = (hdr >> 9) & 255u;
  uint32_t k = (hdr >> 17) & 63u;
  uint32_t mterm = D.mterm[mi], ma = D.ma[mi], mb = D.mb[mi], mc = D.mc[mi];
  uint64_t mv = D.mv[mi];
  D.mkey[mi] = ~0ull;
  x.free_mask |= 1ull << slot;
  x.inflight--;
  rescan_min(D, x);

  uint32_t f = ND(nflags, me);
  if (!f_alive(f) || !f_conn(f) || !f_conn(ND(nflags, src))) {
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
  uint32_t term = ND(nterm, me);
  if (mterm > term) {  // step down
    uint32_t was = f_role(f);
    term = mterm;
    ND(nterm, me) = term;
    f = f_set(f_set(f_set(f, 4, 4, 15u), 16, 8, 0u), 0, 2, R_F);
    ND(nflags, me) = f;
    if (was == R_L) reset_timer(D, x, me);
  }
  uint32_t role = f_role(f);
  switch (type) {
    case M_RV_REQ: {
      uint32_t last = ND(nlast, me);
      uint32_t lt = term_at(D, x, me, last, ND(nsnap, me), ND(nsnapt, me));
      bool up = (mc > lt) || (mc == lt && mb >= last);
      uint32_t voted = f_voted(f);
      bool granted = (mterm == term) && (voted == 15u || voted == ma) && up;
      if (granted) {
        ND(nflags, me) = f_set(f, 4, 4, ma);
        reset_timer(D, x, me);
      }
      net_send(D, x, me, src, M_RV_REP, inc, term, granted ? 1u : 0u, 0, 0, 0, 0);
    } break;
    case M_RV_REP:
      if (role == R_C && mterm == term && ma) {
        uint32_t votes = f_votes(f) | (1u << src);
        ND(nflags, me) = f_set(f, 16, 8, votes);
        if ((uint32_t)__builtin_popcount(votes) > D.n / 2) become_leader(D, x, me);
      }
      break;
    case M_AE_REQ: {
      if (mterm < term) { net_send(D, x, me, src, M_AE_REP, inc, term, 0, 0, 0, 0, 0); break; }
      if (role == R_C) ND(nflags, me) = f_set(f, 0, 2, R_F);
      reset_timer(D, x, me);
      uint32_t snap = ND(nsnap, me), snapt = ND(nsnapt, me), last = ND(nlast, me);
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
      ND(nlast, me) = last;
      uint32_t lc = ma + k;
      if (mc < lc) lc = mc;
      if (lc > ND(ncommit, me)) {
        ND(ncommit, me) = lc;
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
        uint32_t xx = mb, lo = PR(nmatch, me, src) + 1, hi = ND(nlast, me) + 1;
        if (xx < lo) xx = lo;
        if (xx > hi) xx = hi;
        PR(nnext, me, src) = xx;
        send_append(D, x, me, src);
      }
      break;
    case M_IS_REQ: {
      if (mterm < term) { net_send(D, x, me, src, M_IS_REP, inc, term, 0, 0, 0, 0, 0); break; }
      if (role == R_C) ND(nflags, me) = f_set(f, 0, 2, R_F);
      reset_timer(D, x, me);
      uint32_t idx = ma;
      if (idx > ND(ncommit, me)) {
        uint32_t last = ND(nlast, me);
        if (!(idx <= last && term_at(D, x, me, idx, ND(nsnap, me), ND(nsnapt, me)) == mb))
          ND(nlast, me) = idx;
        ND(nsnap, me) = idx; ND(nsnapt, me) = mb; ND(nsnapv, me) = mv;
        ND(ncommit, me) = idx; ND(napplied, me) = idx;
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
  uint32_t f = ND(nflags, me);
  if (f_role(f) == R_L) {  // heartbeat / replication round
    for (uint32_t p = 0; p < D.n; p++) {
      if (p == me) continue;
      send_append(D, x, me, p);
      if (x.code != RUN) return;
    }
    ND(ntimer, me) = x.now + D.hb;
    rec_node(D, x, 1, 1, me, 0);
    return;
  }
  uint32_t term = ND(nterm, me) + 1;  // election timeout: become candidate
  ND(nterm, me) = term;
  ND(nflags, me) = f_set(f_set(f_set(f, 4, 4, me), 0, 2, R_C), 16, 8, 1u << me);
  x.cnt[CNT_ELECTIONS]++;
  reset_timer(D, x, me);
  uint32_t last = ND(nlast, me);
  uint32_t lt = term_at(D, x, me, last, ND(nsnap, me), ND(nsnapt, me));
  for (uint32_t p = 0; p < D.n; p++) {
    if (p == me) continue;
    net_send(D, x, me, p, M_RV_REQ, f_inc(f), term, me, last, lt, 0, 0);
    if (x.code != RUN) return;
  }
  rec_node(D, x, 1, 0, me, 0);
}

// ---------------------------------------------------------------- tester actions
DI void t_crash1(const Dev& D, X& x, uint32_t i) {  // tester.rs:329-333
  ND(nflags, i) = f_set(ND(nflags, i), 2, 1, 0u);
  ND(ntimer, i) = INF_T;
}
DI void t_start1(const Dev& D, X& x, uint32_t i) {  // tester.rs:293-327, raft.rs:108-122
  t_crash1(D, x, i);
  uint32_t f = ND(nflags, i);
  f = f_set(f, 2, 1, 1u);
  f = f_set(f, 8, 8, f_inc(f) + 1u);
  f = f_set(f_set(f, 0, 2, R_F), 16, 8, 0u);
  ND(nflags, i) = f;
  uint32_t snap = ND(nsnap, i);
  ND(ncommit, i) = snap;
  ND(napplied, i) = snap;
  if (!D.null_raft) reset_timer(D, x, i);
}
DI void t_conn(const Dev& D, X& x, uint32_t i, uint32_t v) {
  ND(nflags, i) = f_set(ND(nflags, i), 3, 1, v);
}
// raft.rs:238-244 start(); returns ok. Caller checked unwrap.
DI bool t_start(const Dev& D, X& x, uint32_t i, uint64_t v, uint32_t& idx, uint32_t& term) {
  uint32_t f = ND(nflags, i);
  if (D.null_raft || f_role(f) != R_L) return false;
  uint32_t snap = ND(nsnap, i), last = ND(nlast, i) + 1;
  if (last - snap > D.log_cap) { fail(D, x, MR_FAIL_SIM_CAPACITY); return false; }
  size_t li = logi(D, x, i, last);
  term = ND(nterm, i);
  D.lterm[li] = term;
  D.lval[li] = v;
  ND(nlast, i) = last;
  if (last - snap > x.cnt[CNT_MAX_LOG]) x.cnt[CNT_MAX_LOG] = last - snap;
  PR(nmatch, i, i) = last;
  idx = last;
  return true;
}

DI uint32_t t_draw(const Dev& D, X& x, uint32_t& w1) {
  uint32_t w0;
  philox(x.t_ctr++, 0, ST_TESTER, x.k0, x.k1, w0, w1);
  return w0;
}
DI uint32_t t_range(const Dev& D, X& x, uint32_t lo, uint32_t hi) {
  uint32_t w1, w0 = t_draw(D, x, w1);
  return u_range(w0, lo, hi);
}

// ---------------------------------------------------------------- tester interpreter
#define TR(k) D.tr[(size_t)(k) * D.C + x.c]
#define TV(k) D.tv[(size_t)(k) * D.C + x.c]
#define TS(k) D.ts[(size_t)(k) * D.C + x.c]

// Runs the cluster's scenario program from its saved pc until the next sleep
// (SEMANTICS §6). Returns after a yield or a verdict.
DI void tester(const Dev& D, X& x) {
  uint32_t pc = D.tpc[x.c], phase = D.tphase[x.c];
  const uint32_t n = D.n;
  uint32_t sleep_us = 0;
  for (int budget = 0;; budget++) {
    if (budget > 100000 || pc >= D.prog_len) { fail(D, x, MR_FAIL_SIM_BAD_PROGRAM); return; }
    uint64_t ins = D.prog[pc];
    uint32_t op = (uint32_t)ins & 255u, a = (uint32_t)(ins >> 8) & 255u;
    uint32_t b = (uint32_t)(ins >> 16) & 255u, c = (uint32_t)(ins >> 24) & 255u;
    uint32_t imm = (uint32_t)(ins >> 32);
    bool yield = false;
    switch (op) {
      case OP_NOP: pc++; break;
      case OP_NEW:  // RaftTester::new / new_with_snapshot (tester.rs:34-60)
        x.netmode = (x.netmode & ~2u) | (a ? 2u : 0u);
        for (uint32_t i = 0; i < n; i++) { t_start1(D, x, i); t_conn(D, x, i, 1); }
        if (D.unrel_flag) { x.netmode |= 1u; set_net(x); }
        pc++;
        break;
      case OP_SET_UNREL:
        x.netmode = (x.netmode & ~1u) | (a ? 1u : 0u);
        set_net(x);
        pc++;
        break;
      case OP_END:  // tester.rs:339-358
        if (x.now > 120000000u) { fail(D, x, MR_FAIL_TIMEOUT_120S); return; }
        x.code = MR_PASS;
        rec_simple(D, x, 3, MR_PASS);
        return;
      case OP_FAIL: fail(D, x, imm); return;
      case OP_SLEEP: sleep_us = imm; pc++; yield = true; break;
      case OP_SLEEP_FIG8: {  // tests.rs:631-636
        uint32_t w1, w0 = t_draw(D, x, w1);
        sleep_us = (w0 < LOSS_Q32) ? t_range(D, x, 0, 500000u) : t_range(D, x, 0, 13000u);
        pc++;
        yield = true;
      } break;
      case OP_CHECK_ONE_LEADER: {  // tester.rs:64-92
        if (phase == 0) { TS(0) = 0; phase = 1; }
        if (phase == 1) {
          if (TS(0) >= 10) { fail(D, x, MR_FAIL_ONE_LEADER_NONE); return; }
          sleep_us = t_range(D, x, 450000u, 550000u);
          phase = 2;
          yield = true;
          break;
        }
        // phase 2: sample
        uint32_t lt[MR_MAX_NODES], ln[MR_MAX_NODES], nl = 0;
        for (uint32_t i = 0; i < n; i++) {
          uint32_t f = ND(nflags, i);
          if (!f_conn(f)) continue;
          if (!f_alive(f)) { fail(D, x, MR_FAIL_UNWRAP_NONE); return; }
          if (!D.null_raft && f_role(f) == R_L) { lt[nl] = ND(nterm, i); ln[nl] = i; nl++; }
        }
        for (uint32_t p = 0; p < nl; p++)
          for (uint32_t q = p + 1; q < nl; q++)
            if (lt[p] == lt[q]) { fail(D, x, MR_FAIL_MULTI_LEADER_TERM); return; }
        if (nl) {
          uint32_t best = 0;
          for (uint32_t p = 1; p < nl; p++)
            if (lt[p] > lt[best]) best = p;
          TR(a) = ln[best];
          phase = 0;
          pc++;
        } else {
          TS(0) = TS(0) + 1;
          phase = 1;
        }
      } break;
      case OP_CHECK_TERMS: {  // tester.rs:95-109
        uint32_t term = 0;
        for (uint32_t i = 0; i < n; i++) {
          uint32_t f = ND(nflags, i);
          if (!f_conn(f)) continue;
          if (!f_alive(f)) { fail(D, x, MR_FAIL_UNWRAP_NONE); return; }
          uint32_t xt = ND(nterm, i);
          if (term == 0) term = xt;
          else if (term != xt) { fail(D, x, MR_FAIL_TERM_DISAGREE); return; }
        }
        TR(a) = term;
        pc++;
      } break;
      case OP_CHECK_NO_LEADER:  // tester.rs:112-122
        for (uint32_t i = 0; i < n; i++) {
          uint32_t f = ND(nflags, i);
          if (!f_conn(f)) continue;
          if (!f_alive(f)) { fail(D, x, MR_FAIL_UNWRAP_NONE); return; }
          if (!D.null_raft && f_role(f) == R_L) { fail(D, x, MR_FAIL_UNEXPECTED_LEADER); return; }
        }
        pc++;
        break;
      case OP_ONE: {  // tester.rs:216-262; TS: 0 t0, 1 starts, 2 index, 3 t1
        uint64_t cmd = TV(b & 15u);
        bool retry = (b >> 7) & 1u;
        uint32_t expected = c < 128 ? c : n - (c - 128);
        if (phase == 0) { TS(0) = x.now; TS(1) = 0; phase = 1; }
        if (phase == 1) {
          if (!(x.now - TS(0) < 10000000u)) { fail(D, x, MR_FAIL_ONE_NO_AGREEMENT); return; }
          uint32_t starts = TS(1), index = 0, term;
          bool have = false;
          for (uint32_t k = 0; k < n; k++) {
            starts = (starts + 1) % n;
            uint32_t f = ND(nflags, starts);
            if (!f_conn(f) || !f_alive(f)) continue;
            if (t_start(D, x, starts, cmd, index, term)) { have = true; break; }
            if (x.code != RUN) return;
          }
          TS(1) = starts;
          if (!have) { sleep_us = 50000; yield = true; break; }
          TS(2) = index;
          TS(3) = x.now;
          phase = 2;
        }
        // phase 2: poll n_committed every 20 ms for < 2 s
        if (!(x.now - TS(3) < 2000000u)) {
          if (!retry) { fail(D, x, MR_FAIL_ONE_NO_AGREEMENT); return; }
          phase = 1;
          break;
        }
        uint32_t cnt;
        uint64_t v;
        n_committed(D, x, TS(2), cnt, v);
        if (cnt > 0 && cnt >= expected && v == cmd) {
          TR(a) = TS(2);
          phase = 0;
          pc++;
          break;
        }
        sleep_us = 20000;
        yield = true;
      } break;
      case OP_WAIT: {  // tester.rs:175-201; TS: 0 to, 1 iteration
        uint32_t index = TR(a), nn = c < 128 ? c : n - (c - 128);
        if (phase == 0) { TS(0) = 10000; TS(1) = 0; phase = 1; }
        if (phase == 2) {
          if (b != 0xFFu) {
            uint32_t st = TR(b);
            bool moved = false;
            for (uint32_t i = 0; i < n; i++)
              if (f_alive(ND(nflags, i)) && ND(nterm, i) > st) moved = true;
            if (moved) { TR(R_FLAG) = 0; phase = 0; pc++; break; }
          }
          TS(1) = TS(1) + 1;
          phase = 1;
        }
        if (phase == 1) {
          uint32_t cnt;
          uint64_t v;
          n_committed(D, x, index, cnt, v);
          if (TS(1) < 30 && cnt < nn) {
            uint32_t to = TS(0);
            sleep_us = to;
            if (to < 1000000u) TS(0) = to * 2;
            phase = 2;
            yield = true;
            break;
          }
        }
        uint32_t cnt;
        uint64_t v;
        n_committed(D, x, index, cnt, v);
        if (cnt < nn) { fail(D, x, MR_FAIL_WAIT_TOO_FEW); return; }
        TR(R_FLAG) = cnt > 0 ? 1u : 0u;
        TV(V_RES) = v;
        phase = 0;
        pc++;
      } break;
      case OP_NCOMMITTED: {
        uint32_t cnt;
        uint64_t v;
        n_committed(D, x, TR(a), cnt, v);
        TR(R_FLAG) = cnt;
        TV(V_RES) = v;
        pc++;
      } break;
      case OP_START: {
        uint32_t i = (TR(a) + b) % n, idx = 0, term = 0;
        if (!f_alive(ND(nflags, i))) { fail(D, x, MR_FAIL_UNWRAP_NONE); return; }
        bool ok = t_start(D, x, i, TV(c & 15u), idx, term);
        if (x.code != RUN) return;
        TR(R_FLAG) = ok ? 1u : 0u;
        if (ok) { TR(R_IDX) = idx; TR(R_TERM) = term; }
        pc++;
      } break;
      case OP_ENTRY: {  // tests.rs:943-951
        uint32_t w1, w0 = t_draw(D, x, w1);
        TV(a & 15u) = ((uint64_t)w1 << 32) | w0;
        pc++;
      } break;
      case OP_LDV: TV(a & 15u) = imm; pc++; break;
      case OP_VLDR: TV(a & 15u) = TR(b & 31u); pc++; break;
      case OP_RAND: TR(a) = t_range(D, x, 0, c ? n : imm); pc++; break;
      case OP_CONNECT: t_conn(D, x, (TR(a) + b) % n, 1); pc++; break;
      case OP_DISCONNECT: t_conn(D, x, (TR(a) + b) % n, 0); pc++; break;
      case OP_CRASH: t_crash1(D, x, (TR(a) + b) % n); pc++; break;
      case OP_START1: t_start1(D, x, (TR(a) + b) % n); pc++; break;
      case OP_CONNECT_ALL:
        for (uint32_t i = 0; i < n; i++) t_conn(D, x, i, 1);
        pc++;
        break;
      case OP_DISCONNECT_ALL:
        for (uint32_t i = 0; i < n; i++) t_conn(D, x, i, 0);
        pc++;
        break;
      case OP_IS_STARTED: TR(R_FLAG) = f_alive(ND(nflags, (TR(a) + b) % n)); pc++; break;
      case OP_IS_CONNECTED: TR(R_FLAG) = f_conn(ND(nflags, (TR(a) + b) % n)); pc++; break;
      case OP_TERM: {
        uint32_t i = (TR(b) + c) % n;
        if (!f_alive(ND(nflags, i))) { fail(D, x, MR_FAIL_UNWRAP_NONE); return; }
        TR(a) = ND(nterm, i);
        pc++;
      } break;
      case OP_LOG_SIZE: {  // tester.rs:152-158 + SEMANTICS §5 size model
        uint32_t mx = 0;
        for (uint32_t i = 0; i < n; i++) {
          uint32_t sz = 32u + (f_voted(ND(nflags, i)) != 15u ? 9u : 1u) +
                        24u * (ND(nlast, i) - ND(nsnap, i));
          if (sz > mx) mx = sz;
        }
        TR(a) = mx;
        pc++;
      } break;
      case OP_RPC_TOTAL: TR(a) = x.msgs_sent / 2; pc++; break;
      case OP_MOVI: TR(a) = imm; pc++; break;
      case OP_MOVN: TR(a) = n; pc++; break;
      case OP_MOV: TR(a) = TR(b); pc++; break;
      case OP_ADDI: TR(a) = TR(b) + imm; pc++; break;
      case OP_ADD: TR(a) = TR(b) + TR(c); pc++; break;
      case OP_SUB: TR(a) = TR(b) - TR(c); pc++; break;
      case OP_MODN: TR(a) = (TR(b) + imm) % n; pc++; break;
      case OP_LT: TR(a) = TR(b) < TR(c) ? 1u : 0u; pc++; break;
      case OP_LTI: TR(a) = TR(b) < imm ? 1u : 0u; pc++; break;
      case OP_LTN: TR(a) = TR(b) < n ? 1u : 0u; pc++; break;
      case OP_EQ: TR(a) = TR(b) == TR(c) ? 1u : 0u; pc++; break;
      case OP_EQI: TR(a) = TR(b) == imm ? 1u : 0u; pc++; break;
      case OP_VEQ: TR(a) = TV(b & 15u) == TV(c & 15u) ? 1u : 0u; pc++; break;
      case OP_RSETX: TR((TR(a) + b) & 31u) = TR(c); pc++; break;
      case OP_RGETX: TR(a) = TR((TR(b) + c) & 31u); pc++; break;
      case OP_VSETX: TV((TR(a) + b) & 15u) = TV(c & 15u); pc++; break;
      case OP_VGETX: TV(a & 15u) = TV((TR(b) + c) & 15u); pc++; break;
      case OP_JMP: pc = imm; break;
      case OP_BRZ: pc = TR(a) == 0 ? imm : pc + 1; break;
      case OP_BRNZ: pc = TR(a) != 0 ? imm : pc + 1; break;
      default: fail(D, x, MR_FAIL_SIM_BAD_PROGRAM); return;
    }
    if (x.code != RUN) return;
    if (yield) {  // time::sleep: close this tester segment (SEMANTICS §7)
      rec_simple(D, x, 2, 0);
      uint64_t target = (uint64_t)x.now + sleep_us;
      if (target >= INF_T) { fail(D, x, MR_FAIL_SIM_CAPACITY); return; }
      D.twake[x.c] = (uint32_t)target;
      D.tpc[x.c] = pc;
      D.tphase[x.c] = phase;
      return;
    }
  }
}

// ---------------------------------------------------------------- kernels
__global__ void __launch_bounds__(256) step_kernel(Dev D, uint32_t budget) {
  X x;
  x.c = blockIdx.x * blockDim.x + threadIdx.x;
  if (x.c >= D.C) return;
  x.code = D.code[x.c];
  if (x.code != RUN) return;
  x.now = D.now[x.c]; x.events = D.events[x.c]; x.msgs_sent = D.msgs_sent[x.c];
  x.inflight = D.inflight[x.c]; x.trace_n = D.trace_n[x.c]; x.mslot = D.mslot[x.c];
  x.netmode = D.netmode[x.c]; x.t_ctr = D.t_ctr[x.c];
  x.free_mask = D.free_mask[x.c]; x.digest = D.digest[x.c]; x.mmin = D.mmin[x.c];
#pragma unroll
  for (uint32_t k = 0; k < CNT__N; k++) x.cnt[k] = D.cnt[(size_t)k * D.C + x.c];
  uint64_t seed = D.seed0 + x.c;
  x.k0 = (uint32_t)seed; x.k1 = (uint32_t)(seed >> 32);
  set_net(x);

  for (uint32_t it = 0; it < budget; it++) {
    // next event: min over tester wake-up, node timers, earliest message
    uint64_t best = ((uint64_t)D.twake[x.c] << 32) | (2ull << 30);
    uint32_t kind = 2, node = 0;
    for (uint32_t d = 0; d < D.n; d++) {
      uint64_t kt = ((uint64_t)ND(ntimer, d) << 32) | (1ull << 30) | d;
      if (kt < best) { best = kt; kind = 1; node = d; }
    }
    if (x.mmin < best) { best = x.mmin; kind = 0; }
    x.now = (uint32_t)(best >> 32);
    x.events++;
    if (x.events > D.max_events) { fail(D, x, MR_FAIL_SIM_EVENT_LIMIT); break; }
    if (kind == 0) {
      x.cnt[CNT_EV_MSG]++;
      deliver(D, x, x.mslot, (uint32_t)best & 0x3FFFFFFFu);
    } else if (kind == 1) {
      x.cnt[CNT_EV_TIMER]++;
      on_timer(D, x, node);
    } else {
      x.cnt[CNT_EV_TESTER]++;
      tester(D, x);
    }
    if (x.code != RUN) break;
  }

  D.code[x.c] = (uint16_t)x.code;
  if (x.code != RUN) D.vtime[x.c] = x.now;
  D.now[x.c] = x.now; D.events[x.c] = x.events; D.msgs_sent[x.c] = x.msgs_sent;
  D.inflight[x.c] = x.inflight; D.trace_n[x.c] = x.trace_n; D.mslot[x.c] = x.mslot;
  D.netmode[x.c] = x.netmode; D.t_ctr[x.c] = x.t_ctr;
  D.free_mask[x.c] = x.free_mask; D.digest[x.c] = x.digest; D.mmin[x.c] = x.mmin;
#pragma unroll
  for (uint32_t k = 0; k < CNT__N; k++) D.cnt[(size_t)k * D.C + x.c] = x.cnt[k];
  if (x.code == RUN) atomicAdd(D.remaining, 1u);
}

// RaftTester state before the test body runs (SEMANTICS §3: tester wakes at t = 0)
__global__ void __launch_bounds__(256) reset_kernel(Dev D) {
  uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= D.C) return;
  D.code[c] = (uint16_t)RUN;
  D.vtime[c] = 0; D.now[c] = 0; D.events[c] = 0; D.msgs_sent[c] = 0; D.inflight[c] = 0;
  D.netmode[c] = 0; D.t_ctr[c] = 0; D.trace_n[c] = 0; D.mslot[c] = 0;
  D.free_mask[c] = D.M >= 64 ? ~0ull : ((1ull << D.M) - 1ull);
  D.digest[c] = FNV_OFF;
  D.mmin[c] = ~0ull;
  for (uint32_t k = 0; k < CNT__N; k++) D.cnt[(size_t)k * D.C + c] = 0;
  for (uint32_t d = 0; d < D.n; d++) {
    size_t i = (size_t)d * D.C + c;
    D.nflags[i] = 15u << 4;  // follower, down, disconnected, voted none
    D.nterm[i] = 0; D.ncommit[i] = 0; D.napplied[i] = 0; D.nlast[i] = 0;
    D.nsnap[i] = 0; D.nsnapt[i] = 0; D.nsnapv[i] = 0; D.ntimer[i] = INF_T;
    D.nectr[i] = 0; D.nnctr[i] = 0; D.slen[i] = 1;
    for (uint32_t p = 0; p < D.n; p++) {
      size_t j = ((size_t)d * D.n + p) * D.C + c;
      D.nnext[j] = 0; D.nmatch[j] = 0;
    }
  }
  for (uint32_t s = 0; s < D.M; s++) D.mkey[(size_t)s * D.C + c] = ~0ull;
  D.tpc[c] = 0; D.twake[c] = 0; D.tphase[c] = 0;
  for (uint32_t k = 0; k < N_S; k++) D.ts[(size_t)k * D.C + c] = 0;
  for (uint32_t k = 0; k < N_R; k++) D.tr[(size_t)k * D.C + c] = 0;
  for (uint32_t k = 0; k < N_V; k++) D.tv[(size_t)k * D.C + c] = 0;
}

// counters_reduce: out[] layout documented in mr_host.cpp (RED_*)
__global__ void __launch_bounds__(256) reduce_kernel(Dev D, unsigned long long* out,
                                                    uint64_t cluster_base) {
  __shared__ unsigned long long acc[CNT__N + 8 + 64];
  for (uint32_t i = threadIdx.x; i < CNT__N + 8 + 64; i += blockDim.x) acc[i] = 0;
  __syncthreads();
  uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < D.C) {
    for (uint32_t k = 0; k < CNT__N; k++) {
      unsigned long long v = D.cnt[(size_t)k * D.C + c];
      if (k >= CNT_MAX_INFLIGHT) atomicMax(&acc[k], v);
      else atomicAdd(&acc[k], v);
    }
    uint32_t code = D.code[c];
    atomicAdd(&acc[CNT__N + 0], (unsigned long long)D.events[c]);
    atomicAdd(&acc[CNT__N + 1], (unsigned long long)D.msgs_sent[c]);
    atomicAdd(&acc[CNT__N + 2], (unsigned long long)D.vtime[c]);
    atomicAdd(&acc[CNT__N + 3], code != RUN ? 1ull : 0ull);
    atomicAdd(&acc[CNT__N + 4], code == MR_PASS ? 1ull : 0ull);
    if (code != RUN) atomicAdd(&acc[CNT__N + 8 + (code < 63 ? code : 63)], 1ull);
    if (code != RUN && code != MR_PASS) {
      atomicMin(&out[CNT__N + 5], (unsigned long long)(cluster_base + c));
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < CNT__N + 8 + 64; i += blockDim.x) {
    if (i == CNT__N + 5 || i == CNT__N + 6 || i == CNT__N + 7) continue;
    if (acc[i] == 0) continue;
    if (i >= CNT_MAX_INFLIGHT && i < CNT__N) atomicMax(&out[i], acc[i]);
    else atomicAdd(&out[i], acc[i]);
  }
}

}  // namespace mr

// host-callable launchers (C++ linkage inside the library)
namespace mr {
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
