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

#include <atomic>

#include "mr_dev.h"

#ifndef MR_TAPE
#define MR_TAPE 0
#endif
#if MR_TAPE  // a decision-tape build of the same kernels (SEMANTICS §12): distinct symbols
#define step_kernel step_kernel_tape
#define launch_step_t launch_step_tape_t
#endif

namespace mr {

// internal linkage: this file is compiled several times with different MR_NB
#define DI static __device__ __forceinline__
// node-count bound of this translation unit's kernels: per-node register arrays
// and unrolled node loops are sized NB (the scenario's server count, or 8), so
// a 5-server test does not pay for 8 (memory layouts keep MR_MAX_NODES)
#ifndef MR_NB
#define MR_NB MR_MAX_NODES
#endif
constexpr uint32_t NB = MR_NB;
// message-slot bound of this translation unit: MR_MW 64-bit words of the free-slot mask
// (1: up to 64 slots; the 20-client snapshot_recover_many_clients_3b keeps up to 229
// messages in flight, so its unit is built with MR_MW = 4: 256 slots)
#ifndef MR_MW
#define MR_MW 1
#endif
constexpr uint32_t MW = MR_MW;
constexpr uint32_t INF_T = 0xFFFFFFFFu;
constexpr uint32_t LOSS_Q32 = 429496729u;  // floor(0.1 * 2^32), tester.rs:130
[[maybe_unused]] constexpr uint64_t FNV_OFF = 0xCBF29CE484222325ull;
constexpr uint64_t FNV_P = 0x100000001B3ull;
constexpr uint32_t RUN = MR_RUNNING;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t ELECTION_US = 1000000;  // RAFT_ELECTION_TIMEOUT, tests.rs:18

// entries per batch of independent loads in log walks (A/B round 2: 4 vs 8 +1.7 % figure_8 with
// 64-lane blocks, profiles/r02_ab_configs.txt r02_s2r; round 3: 2 / 3 / 5 / 6 / 8 -7.0 / -1.7 /
// -3.3 / -3.3 / -20 %; round 6, the pool: 6 / 8 ±0.3 %, profiles/r06_ab_ac.txt)
constexpr uint32_t AC = 4;

// per-lane registers of one cluster during a launch
struct X {
  uint32_t c, now, events, msgs_sent, inflight, code, trace_n, mslot, netmode, t_ctr;
  uint32_t sleep_us, yield, twake;  // twake: the tester's next wake-up (CS_TWAKE)
  uint32_t cwake, ctid, cslot;      // kvraft: earliest client thread (wake, tid, slot)
  uint32_t conn, alive;  // node bit masks: connected (net clog state), started (tester.rs:24-25)
  uint32_t lmask;        // servers whose stored role is leader (kept by store_node)
  uint64_t free_mask[MW], digest, mmin;
  uint32_t timer[NB];  // node timers (election / heartbeat deadline), INF_T = none
  uint32_t cnt[CNT__N];  // pool_kernel: the lane's sums over its events (per cluster: POOL_CNT)
  uint32_t ls;  // pool_kernel: the cluster's pool slot (its LDS column)
  uint64_t aem;  // pool_kernel (MR_POOL 2): the message slots that hold AppendEntries requests
  // pool_kernel (MR_POOL 2): a node event whose applier backlog continues in later iterations
  // (node_event, AP_CAP): bit 31 pending | node | send mode | reply type | is_msg | kind | inc |
  // answered pending slots; ra | src << 1; rb; seq
  uint32_t ap0, ap1, ap2, ap3;
};

// MR_GUARD (a debug build, build.build_guard; tests/test_guard.py): every computed index into a
// per-cluster global array is checked against its bound. A violation is recorded in D.guard
// {tag, cluster, index, bound} with plain vector stores and the index replaced by 0, so the run
// ends with an error from mr_batch_run instead of a memory fault. Product builds: GI(i) = i.
#ifndef MR_GUARD
#define MR_GUARD 0
#endif
enum : uint32_t { G_NODE = 1, G_MSG, G_LOG, G_KT_SLOT, G_KT_FIELD, G_KWK, G_KV, G_CFG_S, G_CFG_J,
                  G_OP, G_STOR, G_CHURN, G_LINJ, G_LKEY, G_PAY };
#if MR_GUARD
__device__ __noinline__ uint32_t guard_bad(uint32_t* g, uint32_t tag, uint32_t c, uint32_t i,
                                           uint32_t n) {
  if (atomicCAS(&g[0], 0u, ~0u) == 0u) {  // the first violation of the run is the one reported
    g[1] = c; g[2] = i; g[3] = n;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    atomicExch(&g[0], tag);
  }
  return 0u;
}
#define GI(i, n, tag) \
  ((uint32_t)(i) < (uint32_t)(n) ? (uint32_t)(i) : guard_bad(D.guard, (tag), x.c, (uint32_t)(i), (uint32_t)(n)))
#else
#define GI(i, n, tag) (i)
#endif

// field accessors (32-bit element offsets, checked at batch creation)
#define CS(f) D.cs32[CS_IDX(f, x.c, D.C)]
#define C64(f) D.cs64[C64_IDX(f, x.c, D.C)]
#define NDP(d) (D.nd32 + ((size_t)x.c * D.n + GI(d, D.n, G_NODE)) * NREC)  // node d's 128-B record
#define ND(f, d) NDP(d)[f]
#define NSV(d) (*reinterpret_cast<uint64_t*>(NDP(d) + NF_SNAPV))
#define PR(f, d, p) NDP(d)[NR_PEER + (f) * MR_MAX_NODES + (p)]
#define MSP(s) (D.ms32 + ((size_t)x.c * D.M + GI(s, D.M, G_MSG)) * MREC)  // message slot s's 32-B record
#define MS32(f, s) MSP(s)[f]
#define MSV(s) (*reinterpret_cast<uint64_t*>(MSP(s) + MF_V))
#define MKEY(s) D.mkey[(size_t)GI(s, D.M, G_MSG) * D.C + x.c]
#define TMR(d) D.tmr[(size_t)GI(d, D.n, G_NODE) * D.C + x.c]
// message keys of the lane's cluster live in LDS during a launch: [slot][lane],
// so a wave's 64 lanes read 64 consecutive u64 (conflict-free). Free slots hold
// ~0, so the earliest-message scan is a branch-free min over all M slots.
// lanes per block: 64 — one wave (A/B round 2 against 128: configs 2-4 +2.4-10 %, config 5 -1 %,
// r02_s2r; 256 message slots of keys need it to fit the 160 KiB of LDS). The step kernel maps
// lane l < lpw of block b to cluster b * lpw + l (lanes_per_wave), which the capacity math
// (cap * lpw / 64) assumes too
constexpr uint32_t STEP_BLOCK = 64;
// MR_KEY32: a 32-bit LDS key t << 5 | dst (t < 2^27 - 1, SEMANTICS §4); the (rare) tie of
// two messages at the same t is broken by their sequence numbers, kept in the message
// record (word MF_PAD). Otherwise a 64-bit key (t << 32 | seq << 6 | ae << 5 | dst).
#ifndef MR_KEY32
#define MR_KEY32 0
#endif
// AppendEntries deliveries as a sub-class of the node events (step_kernel): a scheduling policy
// (results do not depend on it) for the Raft-only kernels with 64-bit keys whose test body does
// not restart servers (restarts_servers, mr_dev.h). A/B (profiles/r03_ab_round3.txt):
// figure_8_unreliable_2c +6.5 %, fail_agree_2b 0; with restarts (figure_8_unreliable_crash) -9 %
// and in the kvraft kernels (unreliable_3a) -7 %, for every per-wave threshold tried. The
// deliveries wait while they are under 1/2 of the wave's node events (A/B: 1/2 135.4 ms, 1/3
// 136.1, 1/4 138.2, 2/3 139.3, off 144.7) and at least AE_OTHERS other node events run (A/B:
// 0 132.4, 32 131.65, 40 134.9, 48 139.75 ms on figure_8_unreliable_2c)
constexpr uint32_t AE_OTHERS = 32;
// MR_POOL: the cluster-pool kernel (pool_kernel below): a workgroup of
// POOL_WAVES waves shares a pool of POOL_SLOTS clusters whose run state lives in LDS; a wave
// takes up to 64 ready clusters whose next event is of one kind (the bins). Its translation
// units use 32-bit keys.
#ifndef MR_POOL
#define MR_POOL 0
#endif
static_assert(!MR_POOL || MR_KEY32, "the pool kernel keeps 32-bit message keys");
// MR_POOL 1: the Raft-only pool (8 waves, 512 clusters); 2: the kvraft / shard_ctrler pool (4 waves
// of 256 clusters: their 64 message slots' keys and one wave per SIMD of registers)
constexpr uint32_t POOL_WAVES = MR_POOL == 2 ? 4 : 8, POOL_SLOTS = 64 * POOL_WAVES;
using lkey_t = std::conditional_t<MR_KEY32 != 0, uint32_t, uint64_t>;
constexpr lkey_t LKEY_FREE = ~lkey_t(0);
constexpr uint32_t T_KEY_MAX = (1u << 27) - 1u;  // delivery times at or past it: SIM_CAPACITY
extern __shared__ uint64_t s_keys_raw[];
#define s_keys reinterpret_cast<lkey_t*>(s_keys_raw)
// key rows: one column per lane (step_kernel) or per pool slot (pool_kernel, x.ls)
constexpr uint32_t KSTR = MR_POOL ? POOL_SLOTS : STEP_BLOCK;
// the Raft pool's 7-server units (MR_POOL 1, NB 7: up to 64 messages in flight) lay out LDS rows
// for slots 0..KROWS-1 only, so a pool of 512 clusters fits the CU's LDS: a cluster's slots from
// D.krows on (KROWS, or fewer: MR_KEY_ROWS, a test knob that exercises the HBM keys) keep their
// keys in HBM (D.mkey, the key format between launches) — the slot allocator takes the lowest
// free slot, so those hold a key only while more than krows messages of the cluster are in
// flight (config 4's peak is 28 per 512 seeds). (The 3- / 5-server pools run M <= 32.)
constexpr bool KEYS_HBM = MR_POOL == 1 && NB > 5;
constexpr uint32_t KROWS = KEYS_HBM ? 32u : 0xFFFFFFFFu;
DI uint32_t key_rows(const Dev& D) { return D.M < KROWS ? D.M : KROWS; }  // LDS layout
DI uint32_t key_live(const Dev& D) {  // rows in use: slots below hold their key in LDS
  if constexpr (KEYS_HBM) return D.krows < key_rows(D) ? D.krows : key_rows(D);
  return key_rows(D);
}
#if MR_POOL
#define LK(s) s_keys[GI(s, key_rows(D), G_LKEY) * KSTR + x.ls]
#else
#define LK(s) s_keys[GI(s, D.M, G_LKEY) * KSTR + threadIdx.x]
#endif
// a message slot's key: its LDS row, or (KEYS_HBM, slots past KROWS) its HBM word
DI lkey_t lk_get(const Dev& D, const X& x, uint32_t s) {
  if constexpr (KEYS_HBM)
    if (s >= key_live(D)) return (lkey_t)MKEY(s);
  return LK(s);
}
DI void lk_set(const Dev& D, const X& x, uint32_t s, lkey_t v) {
  if constexpr (KEYS_HBM) {
    if (s >= key_live(D)) {
      MKEY(s) = v == LKEY_FREE ? ~0ull : (uint64_t)v;
      return;
    }
  }
  LK(s) = v;
}
// per-wave staging after the M key rows: 16 rows of 64 lanes (u32) for each wave of the block —
// the send loop's next[p] / term at next[p] - 1, the appliers' and the AppendEntries receive's
// exchange words
constexpr uint32_t WSTG_ROWS = 2 * MR_MAX_NODES;
DI uint32_t* wstg(const Dev& D) {
  return reinterpret_cast<uint32_t*>(s_keys + key_rows(D) * KSTR) + (threadIdx.x >> 6) * (WSTG_ROWS * 64u);
}
DI uint32_t lane64() { return threadIdx.x & 63u; }
#define LNX(p) wstg(D)[(p) * 64u + lane64()]
#define LPT(p) wstg(D)[(MR_MAX_NODES + (p)) * 64u + lane64()]

// Development profile (MR_PROF builds): the first active lane of a wave adds
// the wave cycles since the previous mark to section k, so the sections
// partition each wave's time; slot 32 + k counts the marks.
enum : uint32_t {
  P_TAIL, P_SEL, P_DECODE, P_LOAD, P_DROP, P_RVREQ, P_RVREP, P_AEREQ, P_AEREP, P_ISREQ, P_ISREP,
  P_HB, P_ELECT, P_APPLY, P_SEND, P_STORE, P_TESTER, P_STEPDOWN, P_PRO, P_EPI,
  P_S_SETUP, P_S_NET, P_S_PAY, P_AE_PROBE, P_AP_LOAD, P_AP_CHECK, P_AP_KV, P_AP_PEND, P__N
};
#ifdef MR_PROF
__shared__ unsigned long long s_prof[MR_POOL ? POOL_WAVES : 1][2 * P__N + 1];
#define PROF(k)                                                            \
  do {                                                                     \
    unsigned long long t_ = wall_clock64();                                \
    if (__lane_id() == (uint32_t)__builtin_ctzll(__ballot(1))) {           \
      uint32_t w_ = threadIdx.x >> 6;                                      \
      unsigned long long d_ = t_ - s_prof[w_][2 * P__N];                   \
      if ((long long)d_ > 0) s_prof[w_][k] += d_;                          \
      s_prof[w_][P__N + (k)] += 1;                                         \
      s_prof[w_][2 * P__N] = t_;                                           \
    }                                                                      \
  } while (0)
#else
#define PROF(k) do {} while (0)
#endif

// ---------------------------------------------------------------- helpers
// per-cluster statistics counters: in registers, or (MR_CNT_MEM) updated in
// place with fire-and-forget atomics so they hold no registers
#define CADD(k, v) (x.cnt[k] += (v))
#define CNT_GET(k) x.cnt[k]
#define CMAX(k, v) do { uint32_t v_ = (v); if (v_ > x.cnt[k]) x.cnt[k] = v_; } while (0)
// node flag word: role[0:2) voted[4:8) (15 = none) inc[8:16) votes[16:24)
DI uint32_t f_role(uint32_t f) { return f & 3u; }
DI uint32_t f_voted(uint32_t f) { return (f >> 4) & 15u; }
DI uint32_t f_inc(uint32_t f) { return (f >> 8) & 255u; }
DI uint32_t f_votes(uint32_t f) { return (f >> 16) & 255u; }
DI uint32_t f_set(uint32_t f, uint32_t sh, uint32_t w, uint32_t v) {
  uint32_t m = ((1u << w) - 1u) << sh;
  return (f & ~m) | ((v << sh) & m);
}
DI uint32_t bit(uint32_t m, uint32_t i) { return (m >> i) & 1u; }
DI uint32_t u_range(uint32_t w, uint32_t lo, uint32_t hi) {
  return lo + (uint32_t)(((uint64_t)w * (uint64_t)(hi - lo)) >> 32);
}
// timers live in registers; a node index is per-lane, so reads / writes are
// unrolled selects instead of dynamic register indexing
DI uint32_t get_timer(const X& x, uint32_t d) {
  uint32_t v = x.timer[0];
#pragma unroll
  for (uint32_t j = 1; j < NB; j++) v = (d == j) ? x.timer[j] : v;
  return v;
}
DI void set_timer(X& x, uint32_t d, uint32_t t) {
#pragma unroll
  for (uint32_t j = 0; j < NB; j++) x.timer[j] = (d == j) ? t : x.timer[j];
}

// Philox4x32-10 with counter (c0, c1, c2, 0) and key (k0, k1); returns (w0, w1).
// Out of line: one copy serves every draw site of the kernel.
__device__ __forceinline__ uint2 philox2(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t k0,
                                      uint32_t k1) {
  uint32_t c3 = 0;
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)c0 * 0xD2511F53u, p1 = (uint64_t)c2 * 0xCD9E8D57u;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return make_uint2(c0, c1);
}
// the cluster's draw: counter (c0, c1, c2) = (seq, entity, stream), key = its seed
// (SEMANTICS §2). In MR_TAPE builds with keyed decisions set (§12), replay looks the key up
// in the cluster's sorted table (a miss takes the Philox draw and is counted), and record
// appends {key, words} in draw order.
DI void philox(const Dev& D, X& x, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t& w0,
               uint32_t& w1) {
  if constexpr (MR_TAPE) {
    if (D.tape_mode) {
      const uint32_t khi = (c2 << 16) | c1;
      if (D.tape_mode == 1u) {  // lower bound over the cluster's CSR row (sorted by key)
        const uint4* tb = D.dtab + D.doff[x.c];
        uint32_t lo = 0, n = D.doff[x.c + 1] - D.doff[x.c];
        while (n) {  // first record with key >= (khi, c0)
          const uint32_t h = n >> 1;
          const uint4 r = tb[lo + h];
          if (r.x < khi || (r.x == khi && r.y < c0)) { lo += h + 1; n -= h + 1; }
          else n = h;
        }
        if (lo < D.doff[x.c + 1] - D.doff[x.c]) {
          const uint4 r = tb[lo];
          if (r.x == khi && r.y == c0) { w0 = r.z; w1 = r.w; return; }
        }
        CS(CS_TAPE) = CS(CS_TAPE) + 1u;  // no record: the seed's own draw
      } else {
        uint4* tb = D.dtab + (size_t)x.c * D.dcap;
        const uint64_t seed = D.seed0 + x.c;
        const uint2 w = philox2(c0, c1, c2, (uint32_t)seed, (uint32_t)(seed >> 32));
        w0 = w.x;
        w1 = w.y;
        const uint32_t p = CS(CS_TAPE);
        CS(CS_TAPE) = p + 1u;
        if (p < D.dcap) tb[p] = make_uint4(khi, c0, w0, w1);
        return;
      }
    }
  }
  const uint64_t seed = D.seed0 + x.c;
  const uint2 w = philox2(c0, c1, c2, (uint32_t)seed, (uint32_t)(seed >> 32));
  w0 = w.x;
  w1 = w.y;
}
DI size_t logi(const Dev& D, const X& x, uint32_t d, uint32_t i) {
  return ((size_t)x.c * D.n + GI(d, D.n, G_LOG)) * D.log_cap + (i & (D.log_cap - 1u));
}

// One node's scalar state, loaded into registers at the start of an event
// (one batch of independent loads) and stored back at its end.
struct NC {
  uint32_t f, term, commit, applied, last, snap, snapt, ectr, nctr, pexp, slen, lastt;
};
// words 0..11 of the node record as three 16-B accesses
DI NC load_node(const Dev& D, const X& x, uint32_t d) {
  const uint4* p = reinterpret_cast<const uint4*>(NDP(d));
  const uint4 a = p[0], b = p[1], c = p[2];
  return NC{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
}
// every role change of a record passes here, so x.lmask mirrors the stored roles and the
// tester's is_leader() sampling (t_leaders) reads no record
DI void store_node(const Dev& D, X& x, uint32_t d, const NC& n) {
  x.lmask = (x.lmask & ~(1u << d)) | (f_role(n.f) == R_L ? 1u << d : 0u);
  uint4* p = reinterpret_cast<uint4*>(NDP(d));
  p[0] = make_uint4(n.f, n.term, n.commit, n.applied);
  p[1] = make_uint4(n.last, n.snap, n.snapt, n.ectr);
  p[2] = make_uint4(n.nctr, n.pexp, n.slen, n.lastt);
}
// next[] / match[] of a node (words 16..31), loaded with its scalars at the start of
// every node event: a leader's sends and acknowledgements then wait on no further load
struct PV {
  uint32_t nx[NB], mt[NB];
};
DI void load_peers(const Dev& D, const X& x, uint32_t d, PV& pv) {
  const uint4* p = reinterpret_cast<const uint4*>(NDP(d) + NR_PEER);
#pragma unroll
  for (uint32_t q = 0; q < (NB + 3) / 4; q++) {
    const uint4 a = p[q], b = p[MR_MAX_NODES / 4 + q];
    const uint32_t an[4] = {a.x, a.y, a.z, a.w}, bm[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (uint32_t r = 0; r < 4; r++)
      if (4 * q + r < NB) { pv.nx[4 * q + r] = an[r]; pv.mt[4 * q + r] = bm[r]; }
  }
}
// v[i] for a per-lane index, as a select chain over constant indices (no scratch)
DI uint32_t sel_nb(const uint32_t (&v)[NB], uint32_t i) {
  uint32_t r = 0;
#pragma unroll
  for (uint32_t q = 0; q < NB; q++) r = q == i ? v[q] : r;
  return r;
}
DI void put_nb(uint32_t (&v)[NB], uint32_t i, uint32_t val) {
#pragma unroll
  for (uint32_t q = 0; q < NB; q++) v[q] = q == i ? val : v[q];
}

DI uint32_t term_at(const Dev& D, const X& x, uint32_t d, const NC& n, uint32_t i) {
  if (i == 0) return 0;
  if (i == n.snap) return n.snapt;
  if (i == n.last) return n.lastt;
  return D.log[logi(D, x, d, i)].term;
}

// Run starts (fast backup in O(1)): every log entry written on the device carries rs = the
// first index of the run of equal terms that ends at it (LE.rs), computed from the entry
// below it as it is written — rs(i) = rs(i - 1) if term(i) == term(i - 1), else i — and
// CS_LRS + d keeps rs(last) so an append needs no log read. Below or at the snapshot the
// entries are gone: the entry at the snapshot index counts with rs = snap, so a stored rs is
// either the run's true start or <= snap, and the fast-backup walk of a conflicting term
// (raft.rs AppendEntries handler; the oracle walks entry by entry)
//   xx = prev; while (xx - 1 > snap && term(xx - 1) == term(prev)) xx--;
// is xx = max(rs(prev), snap + 1) for prev > snap — one load instead of one round trip per
// entry of the run (figure_8_unreliable: 16-127 entries per walk, ≈ 40 walks per seed).
// (term, rs) of entry i of node d: the snapshot, cached last entry, or the ring
DI void le_at(const Dev& D, const X& x, uint32_t d, const NC& n, uint32_t lrs, uint32_t i,
              uint32_t& t, uint32_t& rs) {
  if (i == 0) { t = 0; rs = 0; return; }
  if (i == n.snap) { t = n.snapt; rs = n.snap; return; }
  if (i == n.last) { t = n.lastt; rs = lrs; return; }
  const LE e = D.log[logi(D, x, d, i)];
  t = e.term;
  rs = e.rs;
}
#define LRS(d) CS(CS_LRS + (d))

// message header word: type[0:4) src[4:9) dst[9:14) inc/tag[14:22) k[22:28) MAT[28]
// (hosts: servers 0..7, clerks 8..31)
DI uint32_t hdr_make(uint32_t type, uint32_t src, uint32_t dst, uint32_t inc, uint32_t k) {
  return type | (src << 4) | (dst << 9) | ((inc & 255u) << 14) | (k << 22);
}
DI uint32_t hdr_type(uint32_t h) { return h & 15u; }
DI uint32_t hdr_src(uint32_t h) { return (h >> 4) & 31u; }
DI uint32_t hdr_inc(uint32_t h) { return (h >> 14) & 255u; }
DI uint32_t hdr_k(uint32_t h) { return (h >> 22) & 63u; }

DI uint32_t net_loss(const X& x) { return (x.netmode & 1u) ? LOSS_Q32 : 0u; }  // tester.rs:127-137
DI uint32_t net_lat_hi(const X& x) { return (x.netmode & 1u) ? 27000u : 10000u; }

// ---------------------------------------------------------------- trace
// FNV-1a-64 over the 8 words of one trace record (out of line: one copy)
__device__ __forceinline__ uint64_t fnv8(uint64_t h, uint32_t w0, uint32_t w1, uint32_t w2,
                                      uint32_t w3, uint32_t w4, uint32_t w5, uint32_t w6,
                                      uint32_t w7) {
  h = (h ^ w0) * FNV_P; h = (h ^ w1) * FNV_P; h = (h ^ w2) * FNV_P; h = (h ^ w3) * FNV_P;
  h = (h ^ w4) * FNV_P; h = (h ^ w5) * FNV_P; h = (h ^ w6) * FNV_P; h = (h ^ w7) * FNV_P;
  return h;
}
DI void rec8(const Dev& D, X& x, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4,
             uint32_t w5, uint32_t w6, uint32_t w7) {
  x.digest = fnv8(x.digest, w0, w1, w2, w3, w4, w5, w6, w7);
  if (x.c < D.trace_clusters && x.trace_n < D.trace_cap) {
    uint32_t* p = reinterpret_cast<uint32_t*>(D.trace + (size_t)x.c * D.trace_cap + x.trace_n);
    p[0] = w0; p[1] = w1; p[2] = w2; p[3] = w3; p[4] = w4; p[5] = w5; p[6] = w6; p[7] = w7;
  }
  x.trace_n++;
}

DI void rec_node(const Dev& D, X& x, uint32_t cls, uint32_t kind, uint32_t d, uint32_t aux,
                 const NC& n) {
  uint32_t role = bit(x.alive, d) ? f_role(n.f) : R_DOWN;
  const uint32_t idx = x.trace_n;
  rec8(D, x, x.now, cls | (kind << 8) | (d << 16) | (role << 24), aux, n.term, n.commit,
       n.applied, n.last, n.snap);
  if (x.c < D.trace_clusters && idx < D.trace_cap) {  // the node's apply digest beside the record
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");  // after this event's (helpers') adds
    uint64_t* p = D.adig + ((size_t)x.c * MR_MAX_NODES + d) * 2u;
    const uint64_t s = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t inv = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    D.tdig[(size_t)x.c * D.trace_cap + idx] = inv ? ~0ull : s;
  }
}

// ---- apply digests of traced clusters (ABI 4: mr_trace_digests, docs/SEMANTICS.md §7): per
// node the sum of mr_apply_mix(i, value) over the entries it applied one by one, an invalid flag
// once it installed a snapshot or restarted above index 0; trace builds only (c < trace_clusters)
DI uint64_t amix(uint32_t i, uint64_t v) {  // include/madraft_sim.h mr_apply_mix
  uint64_t z = v ^ ((uint64_t)i * 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
DI void adig_add(const Dev& D, uint32_t c, uint32_t node, uint32_t i, uint64_t v) {
  if (c < D.trace_clusters)  // (a helper lane of the cooperative applier adds for its owner)
    __hip_atomic_fetch_add(D.adig + ((size_t)c * MR_MAX_NODES + node) * 2u, amix(i, v),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DI void adig_set(const Dev& D, uint32_t c, uint32_t node, bool invalid) {  // restart / install
  if (c < D.trace_clusters) {
    uint64_t* p = D.adig + ((size_t)c * MR_MAX_NODES + node) * 2u;
    __hip_atomic_exchange(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_exchange(p + 1, invalid ? 1ull : 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

DI void rec_simple(const Dev& D, X& x, uint32_t cls, uint32_t kind) {
  rec8(D, x, x.now, cls | (kind << 8) | (0xFFu << 16), x.msgs_sent, 0, 0, 0, 0, 0);
}

// A verdict stops the cluster (a Rust panic): its trace record (class 3) is the event's last.
// Handlers return as soon as x.code leaves MR_RUNNING, before any further observable effect.
DI void fail(const Dev& D, X& x, uint32_t code) {
  if (x.code != RUN) return;
  x.code = code;
  rec_simple(D, x, 3, code);
}

// ---------------------------------------------------------------- timers / net
DI void reset_timer(const Dev& D, X& x, uint32_t d, NC& n) {  // raft.rs:260-263
  uint32_t w0, w1;
  philox(D, x, n.ectr++, d, ST_ELECT, w0, w1);
  set_timer(x, d, x.now + u_range(w0, D.elo, D.ehi));
}

// the earliest-message rescan four occupied slots per trip, their LDS reads issued together:
// after the argument laundering (ab20) figure_8_unreliable_2c +1.2 %, crash +0.6 %, C5 +1 %
// (ab11), the 3-server 2D kernel −1.3 % (ab20): on for 64-bit keys (the 3- / 5-server kernels)
// (round 6, the pool kernels' 32-bit keys: four slots per trip -0.5 % on config 4, +-0 on the
// headline, profiles/r06_ab_rx4.txt — off)
constexpr bool RESCAN_X4 = !MR_KEY32;
DI void rescan_min(const Dev& D, X& x) {
  if constexpr (MR_KEY32) {
    uint32_t bt = ~0u, bk = ~0u, bs = 0;
    bool tie = false;
#pragma unroll
    for (uint32_t w = 0; w < MW; w++) {
      const uint32_t mw = D.M > 64u * w ? D.M - 64u * w : 0u;
      uint64_t occ = ~x.free_mask[w] & (mw >= 64 ? ~0ull : ((1ull << mw) - 1ull));
      if constexpr (RESCAN_X4) {  // four occupied slots per trip, their LDS reads issued together
        while (occ) {
          uint32_t s4[4];
          bool v4[4];
#pragma unroll
          for (uint32_t q = 0; q < 4; q++) {
            v4[q] = occ != 0ull;
            s4[q] = v4[q] ? 64u * w + (uint32_t)__builtin_ctzll(occ) : 64u * w;
            occ &= occ - 1ull;
          }
          uint32_t k4[4];
#pragma unroll
          for (uint32_t q = 0; q < 4; q++) k4[q] = (uint32_t)lk_get(D, x, s4[q]);
#pragma unroll
          for (uint32_t q = 0; q < 4; q++) {
            if (!v4[q]) continue;
            const uint32_t t = k4[q] >> 5;
            tie = t == bt || (tie && t > bt);
            if (t < bt) { bt = t; bk = k4[q]; bs = s4[q]; }
          }
        }
      }
      while (occ) {
        const uint32_t s = 64u * w + (uint32_t)__builtin_ctzll(occ);
        occ &= occ - 1ull;
        const uint32_t k = (uint32_t)lk_get(D, x, s), t = k >> 5;
        tie = t == bt || (tie && t > bt);
        if (t < bt) { bt = t; bk = k; bs = s; }
      }
    }
    if (tie) {  // two or more messages at time bt: the smaller sequence number first
      // (round 6: the tied slots found in LDS first and their sequence numbers loaded four per
      // trip: headline +0.5 %, config 4 -0.3 %, config 5 -0.7 / -3.1 %, profiles/r06_ab_tb.txt —
      // not kept)
      uint32_t bq = ~0u;
      for (uint32_t w = 0; w < MW; w++) {
        const uint32_t mw = D.M > 64u * w ? D.M - 64u * w : 0u;
        uint64_t occ = ~x.free_mask[w] & (mw >= 64 ? ~0ull : ((1ull << mw) - 1ull));
        while (occ) {
          const uint32_t s = 64u * w + (uint32_t)__builtin_ctzll(occ);
          occ &= occ - 1ull;
          const uint32_t k = (uint32_t)lk_get(D, x, s);
          if ((k >> 5) != bt) continue;
          const uint32_t q = MS32(MF_PAD, s);
          if (q < bq) { bq = q; bk = k; bs = s; }
        }
      }
    }
    x.mmin = bk == ~0u ? ~0ull : (((uint64_t)(bk >> 5) << 32) | (bk & 31u));
    x.mslot = bs;
    return;
  }
  uint64_t best = ~0ull;
  uint32_t bs = 0;
  if constexpr (RESCAN_X4 && MW == 1) {
    uint64_t occ = ~x.free_mask[0] & (D.M >= 64 ? ~0ull : ((1ull << D.M) - 1ull));
    while (occ) {
      uint32_t s4[4];
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {  // a slot past the last occupied one repeats s4[0]
        s4[q] = occ ? (uint32_t)__builtin_ctzll(occ) : s4[0];
        occ &= occ - 1ull;
      }
      uint64_t k4[4];
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) k4[q] = LK(s4[q]);
#pragma unroll
      for (uint32_t q = 0; q < 4; q++)
        if (k4[q] < best) { best = k4[q]; bs = s4[q]; }
    }
  } else if constexpr (MW == 1) {
    uint64_t occ = ~x.free_mask[0] & (D.M >= 64 ? ~0ull : ((1ull << D.M) - 1ull));
    while (occ) {
      const uint32_t s = (uint32_t)__builtin_ctzll(occ);
      occ &= occ - 1ull;
      const uint64_t k = LK(s);
      if (k < best) { best = k; bs = s; }
    }
  } else {
#pragma unroll 8
    for (uint32_t s = 0; s < D.M; s++) {
      uint64_t k = LK(s);
      if (k < best) { best = k; bs = s; }
    }
  }
  x.mmin = best;
  x.mslot = bs;
}

// link a~b cut by disconnect2 (kvraft partitions, connect_client)
DI bool link_cut(const Dev& D, X& x, uint32_t a, uint32_t b) {
  if (!D.links || (a >= CLERK_HOST && b >= CLERK_HOST)) return false;
  if (a >= CLERK_HOST || b >= CLERK_HOST) {  // clerk host 8 + k and server j
    const uint32_t k = (a >= CLERK_HOST ? a : b) - CLERK_HOST, j = a >= CLERK_HOST ? b : a;
    return (CS(CS_CCUT + (k >> 2)) >> (8u * (k & 3u) + j)) & 1u;
  }
  return (CS(CS_CUT + (a >> 2)) >> (8u * (a & 3u) + b)) & 1u;
}

// madsim net send from node `src` (whose state is `s`) (tester.rs:127-137,
// :147-149). Returns the slot or -1 if the message is dropped.
// `lean` (the node event's send loop, MR_SEND_LEAN): the caller has already dropped the sends
// that clog (its `reach` mask folds in the connect state and the cut links), and records a
// capacity verdict itself where the loop exits, so the loop body carries no clog test and no
// inlined copy of the verdict record
DI int net_send(const Dev& D, X& x, uint32_t src, uint32_t& nctr, uint32_t dst, uint32_t type,
                uint32_t inc, uint32_t term, uint32_t a, uint32_t b, uint32_t c, uint64_t v,
                uint32_t k, uint32_t ent = NONE, bool lean = false) {
  // the sender in its NET draws: server src, or a clerk's 8 + clerk id (ent; SEMANTICS §12)
  const uint32_t who = ent == NONE ? src : ent;
  uint32_t seq = x.msgs_sent++;
  uint32_t ctr = nctr++;
  uint32_t w0, w1;
  if (!lean && (!bit(x.conn, src) || !bit(x.conn, dst) || link_cut(D, x, src, dst))) {
    if (MR_TAPE && D.tape_mode) philox(D, x, ctr, who, ST_NET, w0, w1);  // recorded too (as the oracle)
    CADD(CNT_DROP_CLOG, 1u);
    return -1;
  }
  philox(D, x, ctr, who, ST_NET, w0, w1);
  if (w0 < net_loss(x)) { CADD(CNT_DROP_LOSS, 1u); return -1; }
  // madsim's net has no cap: a full slot table (SEMANTICS §9), a sequence number past 2^24
  // (§3) or a delivery time past the key range (§4) is a simulator limit, one verdict
  const bool full = x.inflight >= D.M;
  if (full) CADD(CNT_DROP_OVERFLOW, 1u);
  uint32_t t = x.now + u_range(w1, 1000u, net_lat_hi(x));
  if (full || seq >= (1u << 24) || t >= T_KEY_MAX) {
    if (lean) {
      if (x.code == RUN) x.code = MR_FAIL_SIM_CAPACITY;  // recorded by the caller
    } else {
      fail(D, x, MR_FAIL_SIM_CAPACITY);
    }
    return -1;
  }
  uint32_t slot = 0;
  if constexpr (MW == 1) {
    slot = (uint32_t)__builtin_ctzll(x.free_mask[0]);
    x.free_mask[0] &= ~(1ull << slot);
  } else {
    bool got = false;
#pragma unroll
    for (uint32_t w = 0; w < MW; w++) {
      if (!got && x.free_mask[w]) {
        slot = 64u * w + (uint32_t)__builtin_ctzll(x.free_mask[w]);
        x.free_mask[w] &= x.free_mask[w] - 1ull;
        got = true;
      }
    }
  }
  // key = (time, seq, dst): ordered as (time, seq) since seq is unique; dst (5
  // bits) in the low bits lets a delivery load the node's state before the message body
  uint4* mp = reinterpret_cast<uint4*>(MSP(slot));
  mp[0] = make_uint4(hdr_make(type, src, dst, inc, k), term, a, b);
  mp[1] = make_uint4(c, seq, (uint32_t)v, (uint32_t)(v >> 32));
  x.inflight++;
  CMAX(CNT_MAX_INFLIGHT, x.inflight);
  if constexpr (MR_KEY32) {
    // Raft-only pool kernels (dst < 8): bit 3 marks an AppendEntries request, bit 4 a
    // RequestVote, the event kinds the pool bins by (pool_kind); dst is key & 7 there. The
    // service pool keeps dst (clerk hosts up to 8 + 16) and marks AppendEntries slots in x.aem
    const uint32_t lo = MR_POOL != 1 ? dst
                        : type == M_AE_REQ ? dst | 8u
                        : type == M_RV_REQ || type == M_RV_REP ? dst | 16u
                                                               : dst;
    if constexpr (MR_POOL == 2) {
      if (type == M_AE_REQ) x.aem |= 1ull << slot;
    }
    lk_set(D, x, slot, (t << 5) | lo);
    // every message in flight has a smaller seq: a new one is earliest only by time
    if (t < (uint32_t)(x.mmin >> 32)) { x.mmin = ((uint64_t)t << 32) | lo; x.mslot = slot; }
  } else {
    // bit 5: AppendEntries request (the step loop's AE sub-class, MR_AE_CLASS); below the
    // unique seq, so it never decides the order
    const uint64_t key = ((uint64_t)t << 32) | (seq << 6) |
                         (type == M_AE_REQ ? 32u : 0u) | dst;
    LK(slot) = key;
    if (key < x.mmin) { x.mmin = key; x.mslot = slot; }
  }
  return (int)slot;
}

// ---------------------------------------------------------------- zero-copy payloads
// An AppendEntries message does not copy its entries at send time: the
// receiver reads them from the sender's log ring at delivery. That is exact as
// long as the sender does not overwrite a ring slot an in-flight message still
// references, so each node keeps the index range [PLO, PHI] its unmaterialized
// messages reference and a deadline PEXP by which all of them are delivered
// (send time + the 27 ms latency bound). A log write that would overwrite a
// referenced slot first materializes (copies) those messages' payloads into
// their slots — rare: it takes a deposed leader whose entries are replaced, or
// a ring that wraps under in-flight messages.
constexpr uint32_t HDR_MAT = 1u << 28;  // message header: payload copied into D.pay
constexpr uint32_t LAT_BOUND_US = 27000u;

// a node event's pending payload range (NF_PLO, NF_PHI) loaded with its record (before round 3's
// second half this switch was tested before its definition and so was always off: pend_note and
// the AppendEntries write guard reloaded the range after the sends, waiting on their stores)
DI void pend_note(const Dev& D, X& x, uint32_t me, NC& d, uint32_t lo, uint32_t hi,
                  uint32_t olo_early = 0, uint32_t ohi_early = 0) {
  uint32_t plo = lo, phi = hi;
  if (x.now <= d.pexp) {
    uint32_t olo = olo_early, ohi = ohi_early;
    if (olo <= ohi) { plo = olo < lo ? olo : lo; phi = ohi > hi ? ohi : hi; }
  }
  ND(NF_PLO, me) = plo;
  ND(NF_PHI, me) = phi;
  d.pexp = x.now + LAT_BOUND_US;
}

// copy the payload of every unmaterialized AppendEntries from node L still in flight; L's
// pending range becomes empty and its deadline pexp 0, so no copy of the old range (a
// node event's early PLO/PHI load, MR_PLO_EARLY) is used again: pend_note merges the old
// range only while x.now <= pexp
DI void materialize(const Dev& D, X& x, uint32_t L, uint32_t& pexp) {
#pragma unroll
  for (uint32_t w = 0; w < MW; w++) {
  const uint32_t mw = D.M > 64u * w ? D.M - 64u * w : 0u;  // slots of word w
  uint64_t occ = ~x.free_mask[w] & (mw >= 64 ? ~0ull : ((1ull << mw) - 1ull));
  while (occ) {
    const uint32_t s = 64u * w + (uint32_t)__builtin_ctzll(occ);
    occ &= occ - 1ull;
    const uint32_t hdr = MS32(MF_HDR, s), k = hdr_k(hdr);
    if (hdr_type(hdr) != M_AE_REQ || hdr_src(hdr) != L || (hdr & HDR_MAT) || k == 0) continue;
    const uint32_t prev = MS32(MF_A, s);
    LE* pp = D.pay + ((size_t)x.c * D.M + GI(s, D.M, G_PAY)) * D.K;
    for (uint32_t j = 0; j < k; j++) pp[j] = D.log[logi(D, x, L, prev + 1 + j)];
    MS32(MF_HDR, s) = hdr | HDR_MAT;
    CADD(CNT_MATERIALIZED, k);
  }
  }
  ND(NF_PLO, L) = 1u;  // empty range
  ND(NF_PHI, L) = 0u;
  pexp = 0;
}

// before node L (pending deadline pexp) overwrites log index i
DI void guard_log_write(const Dev& D, X& x, uint32_t L, uint32_t& pexp, uint32_t i, uint32_t plo,
                        uint32_t phi) {  // plo / phi: L's pending payload range (NF_PLO, NF_PHI)
  if (x.now > pexp) return;  // every message L sent has been delivered
  if (plo > phi) return;
  const uint32_t span = phi - plo;  // referenced j in [plo, phi] shares i's slot iff j = i mod cap
  if (span < D.log_cap - 1u && ((i - plo) & (D.log_cap - 1u)) > span) return;
  materialize(D, x, L, pexp);
}
DI void guard_log_write(const Dev& D, X& x, uint32_t L, uint32_t& pexp, uint32_t i) {
  if (x.now > pexp) return;
  guard_log_write(D, x, L, pexp, i, ND(NF_PLO, L), ND(NF_PHI, L));
}

// ---------------------------------------------------------------- tester storage
constexpr uint32_t AC_APPLY = 5;  // entries per batch in the applier
DI void storage_snapshot(const Dev& D, X& x, uint32_t i, uint32_t& slen, uint32_t idx) {  // tester.rs:399-402
  if (idx >= D.apply_cap) { fail(D, x, MR_FAIL_SIM_CAPACITY); return; }
  uint32_t nl = idx + 1;
  for (uint32_t j = nl; j < slen; j++) {
    SE* e = D.stor + (size_t)x.c * D.apply_cap + GI(j, D.apply_cap, G_STOR);
    e->mask &= ~(1u << i);
  }
  slen = nl;
}

DI uint32_t n_committed(const Dev& D, X& x, uint32_t idx, uint64_t& v) {  // tester.rs:405-422
  if (idx >= D.apply_cap) { v = 0; return 0; }
  const SE e = D.stor[(size_t)x.c * D.apply_cap + GI(idx, D.apply_cap, G_STOR)];
  v = e.val;
  return (uint32_t)__builtin_popcount(e.mask);
}

// ---------------------------------------------------------------- Raft node
// One node event (a message delivery or a timer firing) runs in four phases
// so that the kernel holds exactly one copy of the send path:
//   decode + load the node's state into registers -> handler (state changes
//   only; it names the messages to send) -> apply newly committed entries
//   (the tester's applier) -> send loop over the named peers, ascending ->
//   store the node, append the trace record.
// The order of observable effects is the same as calling send() inline in the
// handlers (SEMANTICS §5): every send of an event happens after its state
// changes and its applies, in ascending peer order.
enum : uint32_t { SEND_NONE = 0, SEND_REPLY, SEND_APPEND, SEND_VOTE };

#include "mr_kv.inc"

// the tester's applier (tester.rs:302-325) with push_and_check
// (tester.rs:366-396) inlined: committed entries are walked in batches of AC
// whose loads (log entry, storage mask / value) are all issued before any is
// used — entries have distinct indices, so a batch never reads what it writes.
// A copy of the kernel arguments whose fields are each their own scalar value (an opaque `asm`
// per field, pointers cast back to the global address space so loads stay global_load): the
// kernel-argument words otherwise live as 16-register tuples (s_load_dwordx16) that, spilled to
// VGPR lanes, are reloaded whole (16 v_readlane) wherever one of their fields is used. On it:
// the node event (MR_NE_LAUNDER, headline kernel 1 662 -> 988 v_readlane, VALU -9 %) or, as an
// A/B, only the applier (MR_AP_LAUNDER). Fields the scenario fixes at compile time are left alone.
template <class T>
DI T* glp(T* p) {
  uint64_t v = (uint64_t)(uintptr_t)p;
  asm volatile("" : "+s"(v));
  return (T*)((__attribute__((address_space(1))) T*)(uintptr_t)v);
}
DI uint32_t glu(uint32_t v) {
  asm volatile("" : "+s"(v));
  return v;
}
template <uint32_t S>
DI Dev dev_launder(const Dev& D0) {
  Dev D = D0;
  D.log = glp(D0.log); D.stor = glp(D0.stor); D.cs32 = glp(D0.cs32); D.nd32 = glp(D0.nd32);
  if (is_svc(S)) D.kv32 = glp(D0.kv32);
  if (kv_gen(S).maxraft > 0) { D.kvs32 = glp(D0.kvs32); D.kring = glp(D0.kring); }
  D.trace = glp(D0.trace);
  D.apply_cap = glu(D0.apply_cap); D.log_cap = glu(D0.log_cap); D.bugs = glu(D0.bugs);
  D.trace_clusters = glu(D0.trace_clusters); D.trace_cap = glu(D0.trace_cap);
  D.ms32 = glp(D0.ms32); D.pay = glp(D0.pay); D.tmr = glp(D0.tmr);
  if (D0.led) D.led = glp(D0.led);
  if (is_kv(S)) D.lin32 = glp(D0.lin32);
  if (nthr(S) > 0) { D.kt32 = glp(D0.kt32); D.kwk = glp(D0.kwk); }
  D.seed0 = ((uint64_t)glu((uint32_t)(D0.seed0 >> 32)) << 32) | glu((uint32_t)D0.seed0);
  D.M = glu(D0.M); D.K = glu(D0.K); D.hb = glu(D0.hb); D.elo = glu(D0.elo); D.ehi = glu(D0.ehi);
  D.safety = glu(D0.safety); D.max_events = glu(D0.max_events);
  return D;
}

template <uint32_t S>
DI void node_apply(const Dev& D, X& x, uint32_t me, NC& d, uint32_t& kvready, uint32_t lim = ~0u) {
  const uint32_t end = d.commit < lim ? d.commit : lim;  // entries applied now: up to end
  constexpr bool KV = is_svc(S);
  const bool snapmode = (x.netmode >> 1) & 1u;
  SE* const sb = D.stor + (size_t)x.c * D.apply_cap;
  uint32_t len = d.slen;
  uint32_t pm = 0;  // KV: the server's occupied pending-request slots (kv_apply)
  if constexpr (KV) pm = KVP(me)[KVR_PMASK];
  // software-pipelined: batch b + 1's loads are issued before batch b's checker stores, so
  // they do not wait behind them on vmcnt (disjoint indices: a batch never reads what an
  // earlier one wrote; the log is not written here)
  LE e[AC_APPLY];
  uint32_t m[AC_APPLY];
  uint64_t sv[AC_APPLY];
  auto load_batch = [&](uint32_t i0) {
#pragma unroll
    for (uint32_t j = 0; j < AC_APPLY; j++) {
      const uint32_t i = i0 + j;
      const bool ok = i <= end && i < D.apply_cap;
      e[j] = ok ? D.log[logi(D, x, me, i)] : LE{};
      const SE s = ok ? sb[i] : SE{};
      m[j] = s.mask;
      sv[j] = s.val;
    }
  };
  if (d.applied < end) load_batch(d.applied + 1);
  while (d.applied < end) {
    const uint32_t i0 = d.applied + 1;
    LE ce[AC_APPLY];
    uint32_t cm[AC_APPLY];
    uint64_t csv[AC_APPLY];
#pragma unroll
    for (uint32_t j = 0; j < AC_APPLY; j++) { ce[j] = e[j]; cm[j] = m[j]; csv[j] = sv[j]; }
    if (i0 + AC_APPLY <= end) load_batch(i0 + AC_APPLY);
    PROF(P_AP_LOAD);
#pragma unroll
    for (uint32_t j = 0; j < AC_APPLY; j++) {
      const uint32_t i = i0 + j;
      if (i > end) break;
      d.applied = i;
      if (i >= D.apply_cap) { fail(D, x, MR_FAIL_SIM_CAPACITY); return; }
      CADD(CNT_APPLIES, 1u);
      if (cm[j] && csv[j] != ce[j].val && !(D.bugs & MR_F_BUG_NO_APPLY_CHECK)) {  // tester.rs:384
        fail(D, x, MR_FAIL_APPLY_MISMATCH);
        return;
      }
      if (i > len) { fail(D, x, MR_FAIL_APPLY_OUT_OF_ORDER); return; }  // tester.rs:393
      adig_add(D, x.c, me, i, ce[j].val);
      if (i == len) {
        sb[i] = SE{ce[j].val, cm[j] | (1u << me), ce[j].term};
        len++;
        CMAX(CNT_MAX_INDEX, i);
      }
      if (snapmode && (i + 1) % 10u == 0 && i > d.snap) {  // 2D: service snapshots every 10
        d.snapt = ce[j].term;
        d.snap = i;
        NSV(me) = ce[j].val;
        CADD(CNT_SNAPSHOTS, 1u);
      }
      if constexpr (KV) {
        kv_apply<is_ctrl(S)>(D, x, me, i, ce[j].val, kvready, pm);
        if (x.code != RUN) return;
      }
      if constexpr (kv_gen(S).maxraft > 0) {  // the KV service snapshots (SEMANTICS §9)
        const uint32_t sz = 32u + (f_voted(d.f) != 15u ? 9u : 1u) + 24u * (d.last - d.snap);
        if (i % KV_SNAP_EVERY == 0 && i > d.snap && sz >= kv_gen(S).maxraft / 2) {
          d.snapt = ce[j].term;
          d.snap = i;
          NSV(me) = ce[j].val;
          CADD(CNT_SNAPSHOTS, 1u);
          kv_snapshot<kv_chunk(S)>(D, x, me, i);
          if (x.code != RUN) return;
        }
      }
    }
    PROF(P_AP_CHECK);
  }
  d.slen = len;
}

// Cooperative applier (Raft-only scenarios; the KV services apply through a sequential state
// machine and keep node_apply). The committed entries of every lane that reached the applier
// in this wave iteration are spread over ALL those lanes, one entry per lane per round: a
// lane with a backlog of hundreds of entries (a reconnected follower) costs the wave
// ceil(total / lanes) round trips instead of one per batch of AC_APPLY of its own entries.
// Exactly node_apply's result: the applier of tester.rs:302-325 with push_and_check
// (tester.rs:366-396) is order-dependent only through the storage length `len` and the first
// failure, both computed in closed form —
//   * entries base..end (base = applied + 1, end = commit) have distinct indices, so their
//     loads (log entry, checker record) and checks are independent;
//   * the out-of-order failure can only hit the first entry (base > len); from index len on
//     every entry is appended (len follows i), below it only checked;
//   * the first failing entry f (lowest index, per cluster: an LDS atomic min over
//     index << 2 | code) stops the cluster: entries below f are applied, f is counted unless
//     it failed the capacity check (which precedes the count), nothing above f is written;
//   * 2D service snapshots (every index with (i + 1) % 10 == 0 above the last) keep only the
//     last: its term reaches the owner through LDS, its value goes straight to the record.
// Helper work is found by a wave-uniform loop over the owning lanes (readlane), so lanes
// that are not in this call never contribute a value.
template <uint32_t S>
DI void node_apply_coop(const Dev& D, X& x, uint32_t me, NC& d) {
  // snap_common (the 2D tests, uses_service_snapshots) runs with service snapshots:
  // t_new(snapshot = true) precedes every node event of such a batch, so the mode is the same
  // for every lane here. A scenario whose runtime mode (x.netmode bit 1, what node_apply
  // reads) disagrees would skip or invent snapshots: it fails loudly instead.
  constexpr bool snapmode = uses_service_snapshots(S);
  if (((x.netmode >> 1) & 1u) != (snapmode ? 1u : 0u)) { fail(D, x, MR_FAIL_SIM_BAD_PROGRAM); return; }
  const uint32_t cnt = d.commit > d.applied ? d.commit - d.applied : 0u;
  const uint32_t base = d.applied + 1u, len0 = d.slen;
  // per-owner LDS words (the send-loop staging, unused until the send loop): first failure
  // key, last snapshot's term
  uint32_t* const fkw = wstg(D);
  uint32_t* const stw = fkw + 64u;
  const uint32_t lane = lane64();
  if (cnt) fkw[lane] = ~0u;
  const uint64_t act = __ballot(1);
  const uint64_t own = __ballot(cnt != 0u);
  const uint32_t nh = (uint32_t)__popcll(act);
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
  uint32_t total = 0;
  bool anyfail = false;
  for (uint64_t m = own; m; m &= m - 1ull)
    total += (uint32_t)__builtin_amdgcn_readlane((int)cnt, (int)__builtin_ctzll(m));
  for (uint32_t w0 = 0; w0 < total; w0 += nh) {
    // this lane's item w0 + rank: its owner lane o, index i, and o's cluster / node / length
    const uint32_t w = w0 + rank;
    uint32_t o = 64u, i = 0, oc = 0, ome = 0, olen = 0, obase = 0, oend = 0;
    uint32_t pre = 0;
    for (uint64_t m = own; m; m &= m - 1ull) {
      const int ol = __builtin_ctzll(m);
      const uint32_t oc_n = (uint32_t)__builtin_amdgcn_readlane((int)cnt, ol);
      if (pre < w0 + nh && pre + oc_n > w0) {  // owner's range meets this round (uniform)
        const uint32_t ob = (uint32_t)__builtin_amdgcn_readlane((int)base, ol);
        if (w >= pre && w < pre + oc_n) {
          o = (uint32_t)ol;
          i = ob + (w - pre);
          obase = ob;
          oend = ob + oc_n - 1u;
          oc = (uint32_t)__builtin_amdgcn_readlane((int)x.c, ol);
          ome = (uint32_t)__builtin_amdgcn_readlane((int)me, ol);
          olen = (uint32_t)__builtin_amdgcn_readlane((int)len0, ol);
        }
      }
      pre += oc_n;
      if (pre >= w0 + nh) break;
    }
    const bool mine = o < 64u;
    // phase 1: loads and checks (node_apply's order: capacity, count, mismatch, out of order)
    LE e = LE{};
    SE s = SE{};
    const bool inb = mine && i < D.apply_cap;
    if (inb) {
      e = D.log[((size_t)oc * D.n + ome) * D.log_cap + (i & (D.log_cap - 1u))];
      s = D.stor[(size_t)oc * D.apply_cap + GI(i, D.apply_cap, G_STOR)];
    }
    // the entry is consumed here on every path (not only where it is stored): a load left pending
    // past the applier makes the step loop's next write to that register wait on vmcnt(0)
    asm volatile("" ::"v"(e.term), "v"(e.val));
    uint32_t key = ~0u;
    if (mine) {
      if (!inb) key = (i << 2) | 0u;                                    // SIM_CAPACITY
      else if (s.mask && s.val != e.val && !(D.bugs & MR_F_BUG_NO_APPLY_CHECK))
        key = (i << 2) | 1u;                                            // APPLY_MISMATCH
      else if (i == obase && obase > olen) key = (i << 2) | 2u;         // APPLY_OUT_OF_ORDER
    }
    // the LDS exchange only once some entry of the wave has failed (wave-uniform flag)
    if (__ballot(key != ~0u)) anyfail = true;
    if (anyfail) {
      if (key != ~0u)
        __hip_atomic_fetch_min(&fkw[o], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    // phase 2: entries below the owner's first failure are applied
    if (mine) {
      const uint32_t fk = anyfail ? fkw[o] : ~0u;
      const uint32_t f = fk == ~0u ? ~0u : fk >> 2;
      if (i < f) adig_add(D, oc, ome, i, e.val);
      if (i < f && i >= olen)  // i == len in node_apply's walk: appended
        D.stor[(size_t)oc * D.apply_cap + GI(i, D.apply_cap, G_STOR)] = SE{e.val, s.mask | (1u << ome), e.term};
      if (snapmode && i < f && (i + 1u) % 10u == 0u) {
        // the last snapshot index of the applied range [obase, min(oend, f - 1)]
        const uint32_t hi = f <= oend ? f - 1u : oend;
        if (hi - i < 10u) {  // no later one in range: this entry is the snapshot kept
          stw[o] = e.term;
          *reinterpret_cast<uint64_t*>(D.nd32 + ((size_t)oc * D.n + ome) * NREC + NF_SNAPV) = e.val;
        }
      }
    }
    if (snapmode || anyfail) {  // LDS writes (snapshot term) / reads done before the next round
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (!cnt) return;
  // the owner: counters and node state as node_apply leaves them
  const uint32_t fk = anyfail ? fkw[lane] : ~0u;
  const uint32_t end = fk == ~0u ? d.commit : (fk >> 2) - 1u;  // last entry applied in full
  const uint32_t napplied = end + 1u - base;                    // may be 0 (f == base)
  CADD(CNT_APPLIES, napplied + (fk != ~0u && (fk & 3u) != 0u ? 1u : 0u));
  if (end + 1u > len0 && napplied) {  // entries len0..end appended
    CMAX(CNT_MAX_INDEX, end);
    d.slen = end + 1u;
  }
  if (snapmode && napplied) {
    const uint32_t lo = base > d.snap + 1u ? base : d.snap + 1u;
    const uint32_t first = lo + (19u - lo % 10u) % 10u;  // smallest index >= lo with i % 10 == 9
    if (first <= end) {
      const uint32_t k = (end - first) / 10u + 1u;
      d.snap = first + 10u * (k - 1u);
      d.snapt = stw[lane];
      CADD(CNT_SNAPSHOTS, k);
    }
  }
  d.applied = end;
  if (fk != ~0u) {
    const uint32_t code = fk & 3u;
    fail(D, x, code == 0u ? MR_FAIL_SIM_CAPACITY : code == 1u ? MR_FAIL_APPLY_MISMATCH
                                                              : MR_FAIL_APPLY_OUT_OF_ORDER);
  }
}

// commit = the majority-th largest of the match indices mv[] (mv[me] = last),
// if that entry is from the current term: for a leader, exactly the entries
// above its base lbase (mr_dev.h NF record note), so no log access
DI void advance_commit(const Dev& D, X& x, uint32_t me, NC& d, const uint32_t (&mv)[NB],
                       uint32_t lbase) {
  uint32_t maj = D.n / 2 + 1, N = 0;
#pragma unroll
  for (uint32_t i = 0; i < NB; i++) {
    uint32_t ge = 0;
#pragma unroll
    for (uint32_t j = 0; j < NB; j++) ge += (j < D.n && mv[j] >= mv[i]) ? 1u : 0u;
    if (i < D.n && ge >= maj && mv[i] > N) N = mv[i];
  }
  if (N > d.commit && N > lbase) d.commit = N;  // term_at(N) == term
}

// MR_F_SAFETY (SEMANTICS §11) when `me` wins term d.term:
//  * election safety, exact: one bit per term that has had a leader (a second win in a
//    term is the violation; a node never wins one term twice, its term only grows);
//  * leader completeness: the committed entry at the highest index any server applied —
//    its index, term and command as the apply checker recorded them — is in the new
//    leader's log (or under its snapshot). By log matching (checked at every
//    AppendEntries) the same index and term imply every earlier committed entry too.
DI void safety_on_leader(const Dev& D, X& x, uint32_t me, const NC& d) {
  const uint32_t t = d.term;
  if (t >= LED_TERMS) { fail(D, x, MR_FAIL_SIM_CAPACITY); return; }
  uint32_t* lw = D.led + (size_t)x.c * LED_W + (t >> 5);
  const uint32_t j = CNT_GET(CNT_MAX_INDEX);
  const uint32_t w = *lw;
  const LE le = D.log[logi(D, x, me, j)];
  const SE se = D.stor[(size_t)x.c * D.apply_cap + GI(j, D.apply_cap, G_STOR)];
  if ((w >> (t & 31u)) & 1u) { fail(D, x, MR_FAIL_SAFETY_ELECTION); return; }
  *lw = w | (1u << (t & 31u));
  if (j > d.snap && (j > d.last || le.val != se.val || le.term != se.term))
    fail(D, x, MR_FAIL_SAFETY_COMPLETENESS);
}

// AppendEntries / InstallSnapshot acknowledgement up to xv; returns the peer
// mask to send a follow-up append to. The match indices of every peer and
// next[p] are loaded as one batch of independent loads.
DI uint32_t on_ack(const Dev& D, X& x, uint32_t me, NC& d, uint32_t p, uint32_t xv, PV& pv) {
  // constant indices only: a select chain over a per-lane index is turned
  // back into a dynamically indexed scratch array by the compiler
  uint32_t mv[NB], mp = 0, lbase = 0, nx = 0;
#pragma unroll
  for (uint32_t q = 0; q < NB; q++) {
    const uint32_t v = q < D.n ? pv.mt[q] : 0u;  // match[me] = the leader base
    mp = (q == p) ? v : mp;
    nx = (q == p) ? pv.nx[q] : nx;
    lbase = (q == me) ? v : lbase;
    mv[q] = (q == me) ? d.last : ((q == p && xv > v) ? xv : v);
  }
  if (xv > mp) { PR(PF_MATCH, me, p) = xv; put_nb(pv.mt, p, xv); }
  if (xv + 1 > nx) { nx = xv + 1; PR(PF_NEXT, me, p) = nx; put_nb(pv.nx, p, nx); }
  advance_commit(D, x, me, d, mv, lbase);
  return nx <= d.last ? (1u << p) : 0u;  // still behind: pipeline the next batch
}

// AC entries j.. of an AppendEntries payload (the sender's ring, or the
// materialized copy) and the receiver's entries at their indices: their terms, and (MR_F_SAFETY
// log matching) their commands, from one 16-B load per entry
// MR_AE_OWN: 5-server kernels: yes (+0.7 %); 7 / 8: no (118 -> 4 spilled VGPRs at NB = 7)
#define MR_AE_OWN (MR_NB <= 5)
DI void ae_load_batch(const Dev& D, const X& x, uint32_t me, const NC& d, uint32_t src, bool mat,
                      const LE* pp, uint32_t ma, uint32_t k, uint32_t j, LE (&pe)[AC],
                      uint32_t (&lt)[AC], uint64_t (&ov)[AC], uint32_t (&ors)[AC]) {
#pragma unroll
  for (uint32_t q = 0; q < AC; q++) {
    const uint32_t jx = j + q, i = ma + 1 + jx;
    pe[q] = jx < k ? (mat ? pp[jx] : D.log[logi(D, x, src, i)]) : LE{};
#if MR_AE_OWN
    // i > snap here (the caller skips a payload's prefix at or below the snapshot). Only
    // entries we hold are loaded: the log-matching check reads a command only where i <= last
    // (loading every slot under MR_F_SAFETY measured -2.0 %, profiles/r03b_ab.txt e17)
    const bool own = jx < k && i <= d.last;
    const LE o = own ? D.log[logi(D, x, me, i)] : LE{};
    lt[q] = (jx < k && i <= d.last) ? (i == d.last ? d.lastt : o.term) : 0u;
    ov[q] = o.val;
    ors[q] = o.rs;
#else
    // (term, rs) of our entry at i as one 8-B load (i > snap, see above); the MR_F_SAFETY
    // log-matching check loads the commands separately
    const bool own = jx < k && i <= d.last;
    const uint2 tr = (own && i != d.last) ? *reinterpret_cast<const uint2*>(&D.log[logi(D, x, me, i)])
                                          : make_uint2(0u, 0u);
    lt[q] = own ? (i == d.last ? d.lastt : tr.x) : 0u;
    ov[q] = 0;
    ors[q] = tr.y;
#endif
  }
}

// Cooperative AppendEntries receive (AE_COOP). A catch-up payload carries up to K entries;
// its receiver used to walk them in batches of AC, one dependent round trip per batch, while the
// wave's other lanes waited. The first batch is still walked by its receiver (the common
// heartbeat or short append ends there); the entries after it, of every lane of the wave that
// reached this point, are spread over all those lanes, one entry per lane per round, exactly as
// node_apply_coop spreads applies. The order-dependent parts of the walk have closed forms:
//   * skips form a prefix: the first entry written, f, is the first entry that is past our log
//     or whose term differs from ours (an LDS atomic min per owner); every entry from f on is
//     written, so d.last = the last entry written;
//   * MR_F_SAFETY log matching fails iff a skipped entry (below f) differs in its command: no
//     entry is written then, as in the walk (it fails at that entry's batch, before any write);
//   * the capacity check fails at the first index past snap + log_cap: the entries below it are
//     written, then the cluster stops;
//   * run starts (le_at): entry i >= f written from the sender's entry whose run starts at rs_s
//     gets rs_s if rs_s >= index(f) (the run starts within what is written), else the run reaches
//     below f, where our entry f - 1 matched the sender's, so it continues our run: rs(f - 1);
//   * the write guard (materialize) runs once, before the writes, if any index written shares a
//     ring slot with the pending payload range — the walk's first guarded write copies the same
//     messages (no earlier write of this event touched a referenced slot).
// The kernel's LDS send staging (free until the send loop) holds the exchange words.
// Measured (round 4, same box, profiles/r04_ab_ae_coop.txt): figure_8_unreliable_2c 124.4 -> 125.8 ms,
// its crash variant -1 %, the 15-clerk linearizable kvraft config +1.4 %; ae_req ticks per visit
// 570 -> 675 in the section profile (the owner walk's readlanes and the LDS exchange cost more
// than the batches they replace). Re-measured after the argument laundering (ab20): 5-server
// kernels −0.2 / −0.8 %, the 3-server 2D kernel +2.2 %; the 15-clerk kvraft kernels +1.5 / +0.3 %
// (ab21): on where keys are 32-bit (the 7- / 8-server kernels).
// the 7- / 8-server kernels; not the pool kernels (A/B r05ab1: figure_8_unreliable_2c +2.8 %,
// its crash variant +3.3 % without it; round 6, config 4 on the 7-server pool: +0.9 % with it,
// profiles/r06_ab_c4.txt — within a box's noise, so off)
constexpr bool AE_COOP = MR_KEY32 && !MR_POOL;
constexpr uint32_t AE_COOP_REM = 12;  // entries after the first batch an owner may hand out (LDS rows)
DI void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
DI uint32_t rl(uint32_t v, uint32_t lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}
// returns false if the cluster failed (its verdict is set)
DI bool ae_recv_coop(const Dev& D, X& x, uint32_t me, NC& d, uint32_t src, bool mat, uint32_t slot,
                     uint32_t ma, uint32_t k, uint32_t jr, uint32_t lrs, uint32_t& tprev,
                     uint32_t& rsprev, bool& wrote, uint32_t plo, uint32_t phi) {
  uint32_t* const stg = wstg(D);
  uint32_t* const fw = stg;                    // row 0: first entry written (j), per owner
  uint32_t* const bw = stg + 64u;              // row 1: first skipped entry with another command
  uint32_t* const mw = stg + 4u * 64u;         // rows 4..15: our rs at jr + r (matched entries);
                                               // pass 2: rows 4 / 5 = rs / term of the last written
  const uint32_t lane = lane64();
  const uint32_t cnt = k > jr ? k - jr : 0u;
  if (cnt) CADD(CNT_COOP, cnt);  // entries handed to the wave (mr_counters.coop_entries)
  // entries from jp on are past our log (index ma + 1 + j > last): never a match
  const uint32_t jp = d.last - ma;  // prev <= last and ma <= prev (a snapshot skip raises prev)
  const uint32_t f0 = wrote ? jr : (jp > jr ? (jp < k ? jp : k) : jr);
  const uint32_t c1 = (cnt && !wrote) ? f0 - jr : 0u;  // entries to compare
  if (cnt) { fw[lane] = f0; bw[lane] = ~0u; }
  wave_sync_lds();  // the owners' words are set before any helper's atomic min on them
  const uint64_t act = __ballot(1);
  const uint32_t nh = (uint32_t)__popcll(act);
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
  // the owner's constant fields, packed for the helpers' readlanes
  const uint32_t oc_ = x.c, pk_ = (mat ? 1u : 0u) | (slot << 1) | (src << 9) | (me << 14) | (jr << 20);
  const uint32_t la_ = d.last, lt_ = d.lastt;
  // pass 1: compare our entries with the payload's where both exist
  const uint64_t own1 = __ballot(c1 != 0u);
  if (own1) {
    uint32_t total = 0;
    for (uint64_t m = own1; m; m &= m - 1ull) total += rl(c1, (uint32_t)__builtin_ctzll(m));
    for (uint32_t w0 = 0; w0 < total; w0 += nh) {
      const uint32_t w = w0 + rank;
      uint32_t o = 64u, jx = 0, oc = 0, opk = 0, oma = 0, olast = 0, olastt = 0, olrs = 0, pre = 0;
      for (uint64_t m = own1; m; m &= m - 1ull) {
        const uint32_t ol = (uint32_t)__builtin_ctzll(m);
        const uint32_t c = rl(c1, ol);
        if (pre < w0 + nh && pre + c > w0) {  // uniform: this owner has items in the round
          const uint32_t v0 = rl(oc_, ol), v1 = rl(pk_, ol), v2 = rl(ma, ol), v3 = rl(la_, ol),
                         v4 = rl(lt_, ol), v5 = rl(lrs, ol);
          if (w >= pre && w < pre + c) {
            o = ol; jx = w - pre; oc = v0; opk = v1; oma = v2; olast = v3; olastt = v4; olrs = v5;
          }
        }
        pre += c;
        if (pre >= w0 + nh) break;
      }
      if (o < 64u) {
        // the owner's jr (a helper's own first-batch end differs when its payload is shorter)
        const uint32_t ojr = opk >> 20, j = ojr + jx, i = oma + 1u + j, ri = i & (D.log_cap - 1u);
        const uint32_t ome = (opk >> 14) & 7u, osrc = (opk >> 9) & 31u, oslot = (opk >> 1) & 255u;
        const LE pe = (opk & 1u) ? D.pay[((size_t)oc * D.M + GI(oslot, D.M, G_PAY)) * D.K + GI(j, D.K, G_PAY)]
                                 : D.log[((size_t)oc * D.n + osrc) * D.log_cap + ri];
        const LE ow = D.log[((size_t)oc * D.n + ome) * D.log_cap + ri];
        const uint32_t ot = i == olast ? olastt : ow.term, ors = i == olast ? olrs : ow.rs;
        if (ot != pe.term) {
          __hip_atomic_fetch_min(&fw[o], j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        } else {
          mw[jx * 64u + o] = ors;
          if (D.safety && ow.val != pe.val)
            __hip_atomic_fetch_min(&bw[o], j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
      }
    }
    wave_sync_lds();
  }
  // owners: the first write, the end of the writes, rs(f - 1), the write guard
  uint32_t f = k, jend = k, fcode = 0, rsf = 0;
  if (cnt) {
    f = fw[lane];
    if (D.safety && bw[lane] < f) { fcode = MR_FAIL_SAFETY_LOG_MATCHING; f = k; }
    const uint32_t jcap = d.snap + D.log_cap - ma;  // index ma + 1 + jcap fails the capacity check
    if (!fcode) {
      jend = k < jcap ? k : jcap;
      if (jend < f) jend = f;
      if (k > jcap && f < k) fcode = MR_FAIL_SIM_CAPACITY;  // after the entries below it
    } else {
      jend = f;
    }
    rsf = f == jr ? rsprev : mw[(f - 1u - jr) * 64u + lane];
    if (jend > f && x.now <= d.pexp && plo <= phi) {  // guard_log_write over [index(f), index(jend - 1)]
      const uint32_t a = ma + 1u + f, len = jend - 1u - f, span = phi - plo;
      const uint32_t u = (a - plo) & (D.log_cap - 1u);
      if (span >= D.log_cap - 1u || u <= span || u + len >= D.log_cap) materialize(D, x, me, d.pexp);
    }
  }
  // pass 2: the writes (materialize's copies are done: program order within the wave)
  const uint32_t c2 = jend > f ? jend - f : 0u;
  const uint64_t own2 = __ballot(c2 != 0u);
  if (own2) {
    wave_sync_lds();  // pass 1's LDS words are read: rows 4 / 5 take the last entries written
    uint32_t total = 0;
    for (uint64_t m = own2; m; m &= m - 1ull) total += rl(c2, (uint32_t)__builtin_ctzll(m));
    const uint32_t fe_ = f | (jend << 8);
    for (uint32_t w0 = 0; w0 < total; w0 += nh) {
      const uint32_t w = w0 + rank;
      uint32_t o = 64u, jx = 0, oc = 0, opk = 0, oma = 0, ofe = 0, orsf = 0, pre = 0;
      for (uint64_t m = own2; m; m &= m - 1ull) {
        const uint32_t ol = (uint32_t)__builtin_ctzll(m);
        const uint32_t c = rl(c2, ol);
        if (pre < w0 + nh && pre + c > w0) {
          const uint32_t v0 = rl(oc_, ol), v1 = rl(pk_, ol), v2 = rl(ma, ol), v3 = rl(fe_, ol),
                         v4 = rl(rsf, ol);
          if (w >= pre && w < pre + c) { o = ol; jx = w - pre; oc = v0; opk = v1; oma = v2; ofe = v3; orsf = v4; }
        }
        pre += c;
        if (pre >= w0 + nh) break;
      }
      if (o < 64u) {
        const uint32_t of = ofe & 255u, j = of + jx, i = oma + 1u + j, ri = i & (D.log_cap - 1u);
        const uint32_t ome = (opk >> 14) & 7u, osrc = (opk >> 9) & 31u, oslot = (opk >> 1) & 255u;
        const LE pe = (opk & 1u) ? D.pay[((size_t)oc * D.M + GI(oslot, D.M, G_PAY)) * D.K + GI(j, D.K, G_PAY)]
                                 : D.log[((size_t)oc * D.n + osrc) * D.log_cap + ri];
        const uint32_t rs = pe.rs >= oma + 1u + of ? pe.rs : orsf;
        D.log[((size_t)oc * D.n + ome) * D.log_cap + ri] = LE{pe.term, rs, pe.val};
        if (j + 1u == (ofe >> 8)) { mw[o] = rs; mw[64u + o] = pe.term; }
      }
    }
    wave_sync_lds();
  }
  if (c2) {
    wrote = true;
    d.last = ma + jend;
    rsprev = mw[lane];
    tprev = d.lastt = mw[64u + lane];
    CADD(CNT_LOG_WRITES, c2);
    CMAX(CNT_MAX_LOG, d.last - d.snap);
  }
  if (fcode) { fail(D, x, fcode); return false; }
  return true;
}

// the whole node event on the laundered argument copy (dev_launder). Same-box A/B, round 4
// (profiles/r04_ab_round4.txt ab15): figure_8_unreliable_2c 125.6 -> 121.8 ms, its crash variant
// 67.2 -> 63.6, C5 183 -> 176, C5-lin 561 -> 528 / 690 -> 675; the tester on it too: worse
// The service pool (MR_POOL 2) caps the applier of an event that does not append at AP_CAP
// entries: a server catching up on a backlog (a reconnected follower applies hundreds of entries)
// leaves the rest — and the event's sends, answers, record store and trace record, in their
// order — to continuation iterations of a kind of their own (x.ap*, mr_pool.inc PK_APPLY), where
// every lane is such an applier, instead of holding its wave while the other lanes wait. The
// cluster runs nothing else in between (it is held in that queue), so every effect is the one
// the uncapped event has.
// (cap 5 / 10 / 20, C5-lin 3A: 103.8 / 102.2 / 99.5 K seeds/s, profiles/r06_ab_kvap.txt; 5 = one
// batch of the applier's loads, AC_APPLY)
constexpr uint32_t AP_CAP = 5;
template <uint32_t S>
DI void node_event(const Dev& Darg, X& x, bool is_msg, uint32_t tnode, uint32_t slot,
                   uint32_t seq) {
  const Dev D = dev_launder<S>(Darg);
  constexpr bool KV = is_svc(S);  // kvraft / shard_ctrler request path
  constexpr bool APC = MR_POOL == 2 && ap_cont(S);
  const bool apc = APC && (x.ap0 >> 31);  // an applier continuation (see AP_CAP)
  if (apc) { tnode = x.ap0 & 7u; is_msg = false; }
  uint32_t me = tnode, src = 0, type = 0, inc = 0, k = 0, mterm = 0, ma = 0, mb = 0, mc = 0;
  uint32_t kvready = 0;  // KV: the pending-request slots answered in this event (kv_flush)
  uint32_t hdr_bits = 0;
  // the server is known from the event key, so its record, next[] / match[] and pending
  // payload range are loaded together with the message (a clerk host has no record)
  const bool has_rec = !KV || me < CLERK_HOST;
  NC d = has_rec ? load_node(D, x, me) : NC{};
  PV pv;
  // only a leader reads them (appends, acknowledgements); x.lmask mirrors the stored roles
  // (store_node), so the record's role is known without waiting for it
  if (has_rec && bit(x.lmask, me)) {
    load_peers(D, x, me, pv);
  } else {
#pragma unroll
    for (uint32_t q = 0; q < NB; q++) { pv.nx[q] = 0u; pv.mt[q] = 0u; }
  }
  const uint2 prange = has_rec ? reinterpret_cast<const uint2*>(NDP(me))[NF_PLO / 2] : make_uint2(0u, 0u);
  if (is_msg) {
#if MR_GUARD
    if (D.gprobe && x.c == 0) {  // positive control of the guard (tests/test_guard.py): a read of
      const uint32_t v = MS32(MF_HDR, D.M);  // the message slot past the table (GI substitutes 0)
      asm volatile("" ::"v"(v));
    }
#endif
    const uint4 m0 = reinterpret_cast<const uint4*>(MSP(slot))[0];
    const uint32_t hdr = m0.x;
    const uint2 m1 = reinterpret_cast<const uint2*>(MSP(slot))[MF_C / 2];
    mterm = m0.y; ma = m0.z; mb = m0.w; mc = m1.x;
    if constexpr (MR_KEY32) seq = m1.y;  // the key carries no sequence number
    type = hdr_type(hdr); src = hdr_src(hdr); inc = hdr_inc(hdr);  // dst = tnode (key)
    k = hdr_k(hdr);
    hdr_bits = hdr;
    lk_set(D, x, slot, LKEY_FREE);
    if constexpr (MW == 1) {
      x.free_mask[0] |= 1ull << slot;
      if constexpr (MR_POOL == 2) x.aem &= ~(1ull << slot);
    } else {
#pragma unroll
      for (uint32_t w = 0; w < MW; w++) x.free_mask[w] |= (slot >> 6) == w ? 1ull << (slot & 63u) : 0ull;
    }
    x.inflight--;
    rescan_min(D, x);
    PROF(P_DECODE);
    if constexpr (KV) {
      if (me >= CLERK_HOST) {  // KV_REP at a clerk host
        const uint64_t mv = ((uint64_t)MS32(MF_V + 1, slot) << 32) | MS32(MF_V, slot);
        clerk_deliver(D, x, me, src, inc, mterm, ma, mb, mc, mv, seq);
        return;
      }
    }
  }
  PROF(P_LOAD);
  uint2 prange_r = prange;
  asm volatile("" : "+v"(prange_r.x), "+v"(prange_r.y));
  // election-timer resets (raft.rs:260-263) are counted where the handlers call them and
  // drawn once, after the handler: the timer keeps only the last draw, each draw is keyed by
  // its own ectr (SEMANTICS §2), and nothing between reads the timer, so one Philox site
  // serves every handler of the wave (MR_TAPE builds record every draw: immediate there)
  uint32_t nrst = 0;
#if !MR_TAPE
#define RESET_ME() (nrst++)
#else
#define RESET_ME() reset_timer(D, x, me, d)
#endif
  uint32_t mode = SEND_NONE, peers = 0, rtype = 0, ra = 0, rb = 0, kind;
  const uint32_t others = ((1u << D.n) - 1u) & ~(1u << me);
  if (apc) {  // the deferred event's tail state
    mode = (x.ap0 >> 3) & 3u; rtype = (x.ap0 >> 5) & 15u; is_msg = (x.ap0 >> 9) & 1u;
    kind = (x.ap0 >> 10) & 31u; inc = (x.ap0 >> 15) & 255u; kvready = (x.ap0 >> 23) & 255u;
    ra = x.ap1 & 1u; src = x.ap1 >> 1; rb = x.ap2; seq = x.ap3;
    if (mode == SEND_VOTE) peers = others;
  } else if (is_msg) {
    kind = type;
    if (!bit(x.alive, me) || !bit(x.conn, me) || !bit(x.conn, src) || link_cut(D, x, src, me)) {
      CADD(CNT_DROP_DELIVER, 1u);
      rec_node(D, x, 0, 16, me, seq, d);
      PROF(P_DROP);
      return;
    }
    bool is_reply = (type == M_RV_REP || type == M_AE_REP || type == M_IS_REP);
    if (is_reply && inc != f_inc(d.f)) {
      CADD(CNT_DROP_STALE, 1u);
      rec_node(D, x, 0, 17, me, seq, d);
      PROF(P_DROP);
      return;
    }
    if constexpr (KV) {
      if (type == M_KV_REQ) {  // no Raft term: handled before the step-down rule
        kv_request(D, x, me, d, src, inc, mterm, ma, mb, mc, prange_r);
        if (x.code != RUN) return;
        store_node(D, x, me, d);
        rec_node(D, x, 0, type, me, seq, d);
        return;
      }
    }
    if (mterm > d.term) {  // step down
      uint32_t was = f_role(d.f);
      d.term = mterm;
      d.f = f_set(f_set(f_set(d.f, 4, 4, 15u), 16, 8, 0u), 0, 2, R_F);
      if (was == R_L) RESET_ME();
      PROF(P_STEPDOWN);
    }
    const uint32_t role = f_role(d.f), term = d.term;
    switch (type) {
      case M_RV_REQ: {
        const uint32_t lt = d.lastt;  // term_at(last)
        bool up = (mc > lt) || (mc == lt && mb >= d.last);
        uint32_t voted = f_voted(d.f);
        if (D.bugs & MR_F_BUG_VOTE_STALE) up = true;
        const bool free_vote = voted == 15u || voted == ma || (D.bugs & MR_F_BUG_VOTE_TWICE);
        bool granted = (mterm == term) && free_vote && up;
        if (granted) {
          d.f = f_set(d.f, 4, 4, ma);
          RESET_ME();
        }
        mode = SEND_REPLY; rtype = M_RV_REP; ra = granted ? 1u : 0u;
        PROF(P_RVREQ);
      } break;
      case M_RV_REP:
        if (role == R_C && mterm == term && ma) {
          uint32_t votes = f_votes(d.f) | (1u << src);
          d.f = f_set(d.f, 16, 8, votes);
          if ((uint32_t)__builtin_popcount(votes) > D.n / 2) {  // become leader
            if (D.safety) {
              safety_on_leader(D, x, me, d);
              if (x.code != RUN) return;
            }
            d.f = f_set(d.f, 0, 2, R_L);
            CADD(CNT_LEADERS, 1u);
#pragma unroll
            for (uint32_t p = 0; p < NB; p++) {
              if (p >= D.n) break;
              pv.nx[p] = d.last + 1;
              pv.mt[p] = (p == me) ? d.last : 0u;
              PR(PF_NEXT, me, p) = pv.nx[p];
              PR(PF_MATCH, me, p) = pv.mt[p];
            }
            set_timer(x, me, x.now + D.hb);
            mode = SEND_APPEND; peers = others;
          }
        }
        PROF(P_RVREP);
        break;
      case M_AE_REQ: {
        mode = SEND_REPLY; rtype = M_AE_REP;
        if (mterm < term) break;  // reply {term, false, 0}
        if (role == R_C) d.f = f_set(d.f, 0, 2, R_F);
        RESET_ME();
        uint32_t prev = ma, pterm = mb, j0 = 0;
        if (prev < d.snap) {
          uint32_t skip = d.snap - prev;
          j0 = skip < k ? skip : k;
          prev = d.snap; pterm = d.snapt;
        }
        if (prev > d.last) { rb = d.last + 1; break; }
        const LE* pp = D.pay + ((size_t)x.c * D.M + GI(slot, D.M, G_PAY)) * D.K;
        const bool mat = (hdr_bits & HDR_MAT) != 0u;
        // one batch of independent loads: prev's term, then AC payload entries
        // (sender's ring or materialized copy) and our terms at their indices
        LE pe[AC];
        uint32_t lt[AC], ors[AC];
        uint64_t ov[AC];
        const uint32_t lrs = LRS(me);
        uint32_t tp, rsp;  // term and run start of our entry at prev
        le_at(D, x, me, d, lrs, prev, tp, rsp);
        ae_load_batch(D, x, me, d, src, mat, pp, ma, k, j0, pe, lt, ov, ors);
        PROF(P_AE_PROBE);
        if (!(D.bugs & MR_F_BUG_NO_PREV_CHECK) && tp != pterm) {
          rb = prev <= d.snap ? prev : (rsp > d.snap + 1u ? rsp : d.snap + 1u);
          break;
        }
        uint32_t tprev = tp, rsprev = rsp;  // the entry below the next one written
        bool wrote = false;
        CADD(CNT_SHIPPED, k - j0);  // the payload entries this receiver reads (zero-copy until here)
        // AE_COOP: the receiver walks the first batch; the entries after it go to the wave
        const bool coop = AE_COOP && !MR_TAPE && D.K <= AC + AE_COOP_REM;
        const uint32_t jw = coop ? (k < j0 + AC ? k : j0 + AC) : k;
        for (uint32_t j = j0; j < jw; j += AC) {
          if (j != j0) ae_load_batch(D, x, me, d, src, mat, pp, ma, k, j, pe, lt, ov, ors);
          if (D.safety) {  // MR_F_SAFETY log matching: same index and term => same entry
#if !MR_AE_OWN
#pragma unroll
            for (uint32_t q = 0; q < AC; q++) ov[q] = D.log[logi(D, x, me, ma + 1 + j + q)].val;
#endif
            bool bad = false, skipping = true;  // skips form a prefix: the first write appends the rest
#pragma unroll
            for (uint32_t q = 0; q < AC; q++) {
              const uint32_t i = ma + 1 + j + q;
              const bool sk = j + q < k && i <= d.last && lt[q] == pe[q].term;
              skipping = skipping && sk;
              bad |= skipping && ov[q] != pe[q].val;
            }
            if (bad) { fail(D, x, MR_FAIL_SAFETY_LOG_MATCHING); return; }
          }
#pragma unroll
          for (uint32_t q = 0; q < AC; q++) {
            const uint32_t jx = j + q, i = ma + 1 + jx;
            if (jx >= k) break;
            if (i <= d.last && lt[q] == pe[q].term) {  // d.last only drops below i here
              tprev = lt[q];
              rsprev = i == d.last ? lrs : ors[q];
              continue;
            }
            if (i - d.snap > D.log_cap) { fail(D, x, MR_FAIL_SIM_CAPACITY); return; }
            guard_log_write(D, x, me, d.pexp, i, prange_r.x, prange_r.y);
            rsprev = pe[q].term == tprev ? rsprev : i;
            tprev = pe[q].term;
            D.log[logi(D, x, me, i)] = LE{pe[q].term, rsprev, pe[q].val};
            wrote = true;
            CADD(CNT_LOG_WRITES, 1u);
            d.last = i;
            d.lastt = pe[q].term;
            CMAX(CNT_MAX_LOG, i - d.snap);
          }
        }
        if (coop && !ae_recv_coop(D, x, me, d, src, mat, slot, ma, k, jw, lrs, tprev, rsprev, wrote,
                                  prange_r.x, prange_r.y))
          return;
        if (wrote) LRS(me) = rsprev;
        uint32_t lc = ma + k;
        if (mc < lc) lc = mc;
        if (lc > d.commit) d.commit = lc;
        ra = 1; rb = ma + k;
        PROF(P_AEREQ);
      } break;
      case M_AE_REP:
        if (role != R_L || mterm != term) break;
        mode = SEND_APPEND;
        if (ma) {
          peers = on_ack(D, x, me, d, src, mb, pv);
        } else {
          uint32_t xx = mb, lo = sel_nb(pv.mt, src) + 1, hi = d.last + 1;
          if (xx < lo) xx = lo;
          if (xx > hi) xx = hi;
          PR(PF_NEXT, me, src) = xx;
          put_nb(pv.nx, src, xx);
          peers = 1u << src;
        }
        PROF(P_AEREP);
        break;
      case M_IS_REQ: {
        mode = SEND_REPLY; rtype = M_IS_REP;
        if (mterm < term) break;  // reply {term, 0}
        if (role == R_C) d.f = f_set(d.f, 0, 2, R_F);
        RESET_ME();
        uint32_t idx = ma;
        if (idx > d.commit) {
          if (!(idx <= d.last && term_at(D, x, me, d, idx) == mb)) {
            d.last = idx; d.lastt = mb;
            LRS(me) = idx;  // the snapshot entry (rs <= snap)
          }
          d.snap = idx; d.snapt = mb; NSV(me) = MSV(slot);
          d.commit = idx; d.applied = idx;
          adig_set(D, x.c, me, true);
          storage_snapshot(D, x, me, d.slen, idx);
          if (x.code != RUN) return;
          if constexpr (kv_gen(S).maxraft > 0) {
            kv_install(D, x, me, idx, kvready);
            if (x.code != RUN) return;
          }
          CADD(CNT_INSTALLS, 1u);
        }
        rb = idx;
        PROF(P_ISREQ);
      } break;
      case M_IS_REP:
        if (role == R_L && mterm == term && mb > 0) {
          mode = SEND_APPEND;
          peers = on_ack(D, x, me, d, src, mb, pv);
        }
        PROF(P_ISREP);
        break;
    }
  } else if (f_role(d.f) == R_L) {  // heartbeat / replication round
    kind = 1;
    set_timer(x, me, x.now + D.hb);
    mode = SEND_APPEND; peers = others;
    PROF(P_HB);
  } else {  // election timeout: become candidate
    kind = 0;
    d.term++;
    d.f = f_set(f_set(f_set(d.f, 4, 4, me), 0, 2, R_C), 16, 8, 1u << me);
    CADD(CNT_ELECTIONS, 1u);
    RESET_ME();
    mode = SEND_VOTE; peers = others;
    PROF(P_ELECT);
  }
  if (nrst) {  // the last of this event's nrst draws (ectr advances by nrst, as drawn inline)
    d.ectr += nrst - 1u;
    reset_timer(D, x, me, d);
  }
#undef RESET_ME
  // peers a send can reach: one from a disconnected sender or to a disconnected destination
  // clogs (net_send, SEMANTICS §4), so it needs only its accounting — a sequence number, a
  // send index, drop_clog — and none of the send path's loads (MR_TAPE builds record its
  // draw, so they send it the long way)
  uint32_t reach = MR_TAPE ? ~0u : (bit(x.conn, me) ? x.conn : 0u);
  constexpr bool lean = !MR_TAPE;
  if (lean && D.links)  // links cut by disconnect2 / partition (link_cut): word me / 4, byte me % 4
    reach &= ~((CS(CS_CUT + (me >> 2)) >> (8u * (me & 3u))) & 0xFFu);
  // a leader's appends read our terms at next[p] - 1: issue those loads before the applier's
  // checker stores (the ring slot is valid whatever the applier does; gated after it)
  uint32_t rawt[NB];
  const uint32_t lbase0 = sel_nb(pv.mt, me);
#pragma unroll
  for (uint32_t p = 0; p < NB; p++) {
    const uint32_t ix = pv.nx[p] - 1u;
    // the append reads the ring only for an index below the leader's base that is neither the
    // snapshot nor the last entry (LPT below); the applier may raise the snapshot index, which
    // only turns a load into an InstallSnapshot or a snapshot-term read, never the other way
    const bool need = ix != d.snap && ix != d.last && ix <= lbase0;
    rawt[p] = (mode == SEND_APPEND && bit(peers & reach, p) && p < D.n && ix != 0u && need)
                  ? D.log[logi(D, x, me, ix)].term : 0u;
  }
  if (!KV && kv_gen(S).maxraft == 0) {
    if (__ballot(d.applied < d.commit)) {  // committed entries reach the tester's applier
      node_apply_coop<S>(D, x, me, d);
      if (x.code != RUN) return;
      PROF(P_APPLY);
    }
  } else if (d.applied < d.commit) {
    const bool cap = APC && mode != SEND_APPEND;
    node_apply<S>(D, x, me, d, kvready, cap ? d.applied + AP_CAP : ~0u);
    if (x.code != RUN) return;
    if constexpr (APC) {
      if (cap && d.applied < d.commit) {  // the rest of the backlog, then the tail: later
        x.ap0 = (1u << 31) | me | (mode << 3) | (rtype << 5) | ((is_msg ? 1u : 0u) << 9) | (kind << 10) |
                ((inc & 255u) << 15) | (kvready << 23);
        x.ap1 = (ra & 1u) | (src << 1);
        x.ap2 = rb;
        x.ap3 = seq;
        store_node(D, x, me, d);
        return;
      }
      x.ap0 = 0u;
    }
    PROF(P_APPLY);
  }
  if (mode == SEND_REPLY) peers = 1u << src;
  const uint32_t lt = mode == SEND_VOTE ? d.lastt : 0u;  // term_at(last)
  // appends: next[p] of every peer, then the terms at next[p] - 1, as two
  // batches of independent loads, staged in LDS for the send loop
  const uint32_t all = peers, seq0 = x.msgs_sent, ctr0 = d.nctr;
  peers &= reach;
  if (mode == SEND_APPEND) {  // only a leader appends
    uint32_t nxa[NB];
    const uint32_t lbase = sel_nb(pv.mt, me);
#pragma unroll
    for (uint32_t p = 0; p < NB; p++) {
      nxa[p] = bit(peers, p) ? pv.nx[p] : 0u;
    }
#pragma unroll
    for (uint32_t p = 0; p < NB; p++) {  // term_at(next[p] - 1)
      const uint32_t pv = nxa[p] - 1u;
      const bool ld = bit(peers, p) && nxa[p] > d.snap && pv != 0u && pv != d.snap &&
                      pv != d.last && pv <= lbase;
      const uint32_t t = ld ? rawt[p] : 0u;
      LNX(p) = nxa[p];
      LPT(p) = pv == 0u ? 0u : pv == d.snap ? d.snapt : pv == d.last ? d.lastt : pv > lbase ? d.term : t;
    }
  }
  uint32_t plo_acc = ~0u, phi_acc = 0u;  // index range referenced by this event's payloads
  // a reply or a vote request carries the same fields to every peer; an append's come from
  // the peer's next[] (LDS staging) inside the loop
  const bool rep = mode == SEND_REPLY;
  const uint32_t st0 = rep ? rtype : M_RV_REQ, sa0 = rep ? ra : me, sb0 = rep ? rb : d.last,
                 sc0 = rep ? 0u : lt, sinc = rep ? inc : f_inc(d.f);
  bool sfail = false;  // a send hit a simulator limit (lean sends: recorded after the loop)
  uint32_t sclog = 0;  // ... and the clogged sends before it
  while (peers) {  // the single send path: ascending peer order over the reachable peers
    uint32_t p = (uint32_t)__builtin_ctz(peers);
    peers &= peers - 1u;
    const uint32_t below = all & ((1u << p) - 1u);  // earlier sends of this event, clogged ones too
    x.msgs_sent = seq0 + (uint32_t)__builtin_popcount(below);
    d.nctr = ctr0 + (uint32_t)__builtin_popcount(below);
    uint32_t st = st0, sa = sa0, sb = sb0, sc = sc0, sk = 0, prev = 0;
    uint64_t sv = 0;
    if (mode == SEND_APPEND) {
      const uint32_t nx = LNX(p);
      if (has_snaps(S) && nx <= d.snap) {
        st = M_IS_REQ; sa = d.snap; sb = d.snapt; sc = 0; sv = NSV(me);
      } else {
        prev = nx - 1;
        sk = d.last - prev;
        if (sk > D.K) sk = D.K;
        st = M_AE_REQ; sa = prev; sb = LPT(p); sc = d.commit;
      }
    }
    PROF(P_S_SETUP);
    int s = net_send(D, x, me, d.nctr, p, st, sinc, d.term, sa, sb, sc, sv, sk, NONE, lean);
    if (x.code != RUN) {  // the clogged sends before this one are counted as they happened
      sfail = true;
      sclog = (uint32_t)__builtin_popcount(below & ~reach);
      break;
    }
    PROF(P_S_NET);
    if (s >= 0 && sk) {  // zero-copy payload: entries prev+1 .. prev+sk stay in this log
      plo_acc = prev + 1 < plo_acc ? prev + 1 : plo_acc;
      phi_acc = prev + sk > phi_acc ? prev + sk : phi_acc;
      PROF(P_S_PAY);
    }
  }
  if (sfail) {
    if (lean) rec_simple(D, x, 3, x.code);  // the verdict net_send left unrecorded
    CADD(CNT_DROP_CLOG, sclog);
    return;
  }
  x.msgs_sent = seq0 + (uint32_t)__builtin_popcount(all);  // every send of the event, clogged too
  d.nctr = ctr0 + (uint32_t)__builtin_popcount(all);
  CADD(CNT_DROP_CLOG, (uint32_t)__builtin_popcount(all & ~reach));
  if (plo_acc <= phi_acc) pend_note(D, x, me, d, plo_acc, phi_acc, prange_r.x, prange_r.y);
  if constexpr (KV) {
    if (kvready) {
      kv_flush(D, x, me, d, kvready);
      if (x.code != RUN) return;
    }
  }
  PROF(P_SEND);
  store_node(D, x, me, d);
  rec_node(D, x, is_msg ? 0u : 1u, kind, me, is_msg ? seq : 0u, d);
  PROF(P_STORE);
}

// ---------------------------------------------------------------- tester API (tester.rs)
DI void t_set_unrel(X& x, bool u) { x.netmode = (x.netmode & ~1u) | (u ? 1u : 0u); }
DI bool t_started(const Dev& D, X& x, uint32_t i) { return bit(x.alive, i); }
DI bool t_connected(const Dev& D, X& x, uint32_t i) { return bit(x.conn, i); }
DI void t_conn(const Dev& D, X& x, uint32_t i, uint32_t v) {
  x.conn = v ? (x.conn | (1u << i)) : (x.conn & ~(1u << i));
}
DI void t_crash1(const Dev& D, X& x, uint32_t i) {  // tester.rs:329-333
  x.alive &= ~(1u << i);
  set_timer(x, i, INF_T);
  if (D.kv32) {  // its RPC handler tasks die with it: pending requests are dropped
    uint4* pp = reinterpret_cast<uint4*>(D.kv32 + ((size_t)x.c * D.n + i) * KVREC + KVR_PEND);
    for (uint32_t p = 0; p < 2 * KV_PEND; p++) pp[p] = make_uint4(0u, 0u, 0u, 0u);
    D.kv32[((size_t)x.c * D.n + i) * KVREC + KVR_PMASK] = 0u;
  }
}
DI void t_start1(const Dev& D, X& x, uint32_t i) {  // tester.rs:293-327, raft.rs:108-122
  t_crash1(D, x, i);
  x.alive |= 1u << i;
  NC n = load_node(D, x, i);
  n.f = f_set(n.f, 8, 8, f_inc(n.f) + 1u);
  n.f = f_set(f_set(n.f, 0, 2, R_F), 16, 8, 0u);
  n.commit = n.snap;
  n.applied = n.snap;
  adig_set(D, x.c, i, n.snap != 0u);
  if (!D.null_raft) reset_timer(D, x, i, n);
  store_node(D, x, i, n);
}
DI void t_new(const Dev& D, X& x, bool snapshot) {  // RaftTester::new, tester.rs:34-60
  x.netmode = (x.netmode & ~2u) | (snapshot ? 2u : 0u);
  for (uint32_t i = 0; i < D.n; i++) { t_start1(D, x, i); t_conn(D, x, i, 1); }
  if (D.unrel_flag) t_set_unrel(x, true);
}
// bit mask of the servers whose role is leader: x.lmask, kept by store_node (every role change
// of a record passes there), so is_leader() sampling reads no record
DI uint32_t t_leaders(const Dev& D, X& x) { return x.lmask; }
// tester.rs:165-171 -> raft.rs:238-244; unwrap() on a crashed raft panics.
// `lead` = whether server i is leader (t_leaders), read before the call.
DI bool t_start(const Dev& D, X& x, uint32_t i, uint64_t v, uint32_t& idx, uint32_t& term,
                bool lead) {
  if (!bit(x.alive, i)) { fail(D, x, MR_FAIL_UNWRAP_NONE); return false; }
  if (D.null_raft || !lead) return false;  // Err(NotLeader((me+1)%n))
  // words 0..15 of the record (scalars, pending payload range) and rs(last) as one batch of
  // independent loads: the write guard below needs no further round trip
  const uint4* rp = reinterpret_cast<const uint4*>(NDP(i));
  const uint4 r0 = rp[0], r1 = rp[1], r2 = rp[2];
  const uint2 pr = reinterpret_cast<const uint2*>(NDP(i))[NF_PLO / 2];
  const uint32_t lrs = LRS(i);
  const uint32_t snap = r1.y, last = r1.x + 1;
  if (last - snap > D.log_cap) { fail(D, x, MR_FAIL_SIM_CAPACITY); return false; }
  size_t li = logi(D, x, i, last);
  term = r0.y;
  uint32_t pexp = r2.y;
  const uint32_t rs = term == r2.w ? lrs : last;  // run start (le_at)
  guard_log_write(D, x, i, pexp, last, pr.x, pr.y);
  ND(NF_PEXP, i) = pexp;
  D.log[li] = LE{term, rs, v};
  LRS(i) = rs;
  CADD(CNT_LOG_WRITES, 1u);
  ND(NF_LAST, i) = last;
  ND(NF_LASTT, i) = term;
  CMAX(CNT_MAX_LOG, last - snap);
  idx = last;
  return true;
}
// `count` start(gen_entry()) calls on server i in a row with nothing between them (snap_common's
// burst, tests.rs:889-892): the record is loaded once and stored once, the appends in between
// are the same as `count` t_start calls (each draw precedes its start; a failure stops there)
DI uint64_t t_entry_for_start(const Dev& D, X& x, uint32_t i, uint32_t lm);
DI void t_start_burst(const Dev& D, X& x, uint32_t i, uint32_t count) {
  const uint32_t lm = t_leaders(D, x);
  const bool go = bit(x.alive, i) && !D.null_raft && bit(lm, i);
  uint4 r0 = make_uint4(0u, 0u, 0u, 0u), r1 = r0, r2 = r0;
  uint2 pr = make_uint2(0u, 0u);
  uint32_t lrs = 0;
  if (go) {
    const uint4* rp = reinterpret_cast<const uint4*>(NDP(i));
    r0 = rp[0]; r1 = rp[1]; r2 = rp[2];
    pr = reinterpret_cast<const uint2*>(NDP(i))[NF_PLO / 2];
    lrs = LRS(i);
  }
  const uint32_t term = r0.y, snap = r1.y;
  uint32_t last = r1.x, lastt = r2.w, pexp = r2.y;
  for (uint32_t k = 0; k < count; k++) {
    const uint64_t v = t_entry_for_start(D, x, i, lm);
    if (!bit(x.alive, i)) { fail(D, x, MR_FAIL_UNWRAP_NONE); return; }
    if (!go) continue;  // Err(NotLeader)
    const uint32_t idx = last + 1;
    if (idx - snap > D.log_cap) { fail(D, x, MR_FAIL_SIM_CAPACITY); return; }
    guard_log_write(D, x, i, pexp, idx, pr.x, pr.y);  // pexp = 0 after a materialize
    const uint32_t rs = term == lastt ? lrs : idx;
    D.log[logi(D, x, i, idx)] = LE{term, rs, v};
    CADD(CNT_LOG_WRITES, 1u);
    CMAX(CNT_MAX_LOG, idx - snap);
    last = idx;
    lastt = term;
    lrs = rs;
  }
  if (!go) return;
  ND(NF_PEXP, i) = pexp;
  ND(NF_LAST, i) = last;
  ND(NF_LASTT, i) = lastt;
  LRS(i) = lrs;
}
DI bool t_start(const Dev& D, X& x, uint32_t i, uint64_t v, uint32_t& idx, uint32_t& term) {
  return t_start(D, x, i, v, idx, term, bit(t_leaders(D, x), i) != 0u);
}
DI bool t_start(const Dev& D, X& x, uint32_t i, uint64_t v) {
  uint32_t a, b;
  return t_start(D, x, i, v, a, b);
}
DI uint32_t t_term(const Dev& D, X& x, uint32_t i) {
  if (!bit(x.alive, i)) { fail(D, x, MR_FAIL_UNWRAP_NONE); return 0; }
  return ND(NF_TERM, i);
}
// The tester's checks over every server read each record's words as one batch of loads
// (unrolled over the node bound): a loop that loads server by server is one round trip per
// server, and one per server index some lane needs (A/B in DESIGN.md §6.8)
// the terms of every server (words NF_TERM), 0 past D.n
DI void t_terms(const Dev& D, X& x, uint32_t (&tm)[NB]) {
#pragma unroll
  for (uint32_t q = 0; q < NB; q++) tm[q] = q < D.n ? ND(NF_TERM, q) : 0u;
}
DI uint32_t t_log_size(const Dev& D, X& x) {  // tester.rs:152-158 + SEMANTICS §5 size model
  uint32_t mx = 0;
  uint32_t fl[NB], la[NB], sn[NB];
#pragma unroll
  for (uint32_t q = 0; q < NB; q++) {
    const bool in = q < D.n;
    fl[q] = in ? ND(NF_FLAGS, q) : 0u;
    la[q] = in ? ND(NF_LAST, q) : 0u;
    sn[q] = in ? ND(NF_SNAP, q) : 0u;
  }
#pragma unroll
  for (uint32_t q = 0; q < NB; q++) {
    const uint32_t sz = 32u + (f_voted(fl[q]) != 15u ? 9u : 1u) + 24u * (la[q] - sn[q]);
    if (q < D.n && sz > mx) mx = sz;
  }
  return mx;
}
DI uint32_t t_check_terms(const Dev& D, X& x) {  // tester.rs:95-109
  uint32_t term = 0;
  uint32_t tm[NB];
  t_terms(D, x, tm);
  for (uint32_t i = 0; i < D.n; i++) {
    if (!bit(x.conn, i)) continue;
    if (!bit(x.alive, i)) { fail(D, x, MR_FAIL_UNWRAP_NONE); return 0; }
    uint32_t xt = sel_nb(tm, i);
    if (term == 0) term = xt;
    else if (term != xt) { fail(D, x, MR_FAIL_TERM_DISAGREE); return 0; }
  }
  return term;
}
DI void t_check_no_leader(const Dev& D, X& x) {  // tester.rs:112-122
  for (uint32_t i = 0; i < D.n; i++) {
    if (!bit(x.conn, i)) continue;
    if (!bit(x.alive, i)) { fail(D, x, MR_FAIL_UNWRAP_NONE); return; }
    if (!D.null_raft && bit(t_leaders(D, x), i)) {
      fail(D, x, MR_FAIL_UNEXPECTED_LEADER);
      return;
    }
  }
}
DI void t_sleep(X& x, uint32_t us) { x.sleep_us = us; x.yield = 1; }
DI void t_end(const Dev& D, X& x) {  // tester.rs:339-358
  if (x.now > 120000000u) { fail(D, x, MR_FAIL_TIMEOUT_120S); return; }
  x.code = MR_PASS;
  rec_simple(D, x, 3, MR_PASS);
}

DI uint32_t nd_role(const Dev& D, X& x, uint32_t i) { return f_role(ND(NF_FLAGS, i)); }
DI uint32_t nd_term(const Dev& D, X& x, uint32_t i) { return ND(NF_TERM, i); }
#define TV(k) C64(C64_TV + (k))
#include "mr_tester.inc"

// one tester event: resume the cluster's coroutine until it sleeps or ends
template <uint32_t S>
DI void tester(const Dev& Darg, X& x) {
  const Dev& D = Darg;
  T t;
  // the frame: one cluster-major 80-B record (mr_dev.h TF_Q), five 16-B loads from one address
  // instead of 17 cluster-minor words with 17 field bases (which the compiler keeps live in
  // scalar registers across the step loop)
  const uint4* fr = D.tfr + (size_t)x.c * TF_Q;
  const uint4 q0 = fr[0], q1 = fr[1], q2 = fr[2], q3 = fr[3], q4 = fr[4];
  t.pc = q0.x & 0xFFFFFFu;
  t.helper = q0.x >> 24;
  t.res = q0.y;
  t.l[0] = q0.z; t.l[1] = q0.w; t.l[2] = q1.x; t.l[3] = q1.y;
  t.l[4] = q1.z; t.l[5] = q1.w; t.l[6] = q2.x; t.l[7] = q2.y;
  t.h[0] = q2.z; t.h[1] = q2.w; t.h[2] = q3.x; t.h[3] = q3.y; t.h[4] = q3.z;
  t.hv = ((uint64_t)q4.x << 32) | q3.w;
  static_assert(T_NL == 8 && T_NH == 5, "tester frame record layout");
  x.yield = 0;
  for (int guard = 0;; guard++) {
    if (guard > 4096) { fail(D, x, MR_FAIL_SIM_BAD_PROGRAM); return; }
    if (t.helper != H_NONE) {  // a multi-event tester call in progress
      bool done;
      if constexpr (is_svc(S)) {
        done = t.helper == H_CALL ? call_step(D, x, t) : join_step(D, x, t);
      } else if constexpr (nthr(S) > 0) {
        done = t.helper == H_ONE    ? one_step(D, x, t)
               : t.helper == H_WAIT ? wait_step(D, x, t)
                                    : join_step(D, x, t);  // H_JOIN: join_all
      } else {
        done = t.helper == H_ONE   ? one_step(D, x, t)
               : t.helper == H_COL ? col_step(D, x, t)
                                   : wait_step(D, x, t);
      }
      if (x.code != RUN) return;
      if (!done) break;  // it slept
      t.helper = H_NONE;
    }
    run_scenario<S>(D, x, t);
    if (x.code != RUN) return;
    if (x.yield) break;
    if (t.helper == H_NONE) { fail(D, x, MR_FAIL_SIM_BAD_PROGRAM); return; }
  }
  rec_simple(D, x, 2, 0);  // the test body blocks: this tester segment ends (SEMANTICS §7)
  if (x.yield != 2) {  // time::sleep; 2 = clerk call / join (x.twake already set)
    uint64_t target = (uint64_t)x.now + x.sleep_us;
    if (target >= INF_T) { fail(D, x, MR_FAIL_SIM_CAPACITY); return; }
    x.twake = (uint32_t)target;
  }
  uint4* fw = D.tfr + (size_t)x.c * TF_Q;
  fw[0] = make_uint4(t.pc | (t.helper << 24), t.res, t.l[0], t.l[1]);
  fw[1] = make_uint4(t.l[2], t.l[3], t.l[4], t.l[5]);
  fw[2] = make_uint4(t.l[6], t.l[7], t.h[0], t.h[1]);
  fw[3] = make_uint4(t.h[2], t.h[3], t.h[4], (uint32_t)t.hv);
  fw[4].x = (uint32_t)(t.hv >> 32);
}

// ---------------------------------------------------------------- kernels
constexpr uint32_t CLS_MSG = 0, CLS_TIMER = 1, CLS_TESTER = 2, CLS_NONE = 3;

// a cluster's run state into the lane (registers, LDS message keys) and back: at the start and
// end of a launch, and when a lane that finished its cluster takes the next one (D.stream)
template <uint32_t S>
DI void lane_load(const Dev& D, X& x) {
  x.code = CS(CS_CODE);
  if (x.code != RUN) return;
  x.now = CS(CS_NOW); x.events = CS(CS_EVENTS); x.msgs_sent = CS(CS_MSGS);
  x.inflight = CS(CS_INFLIGHT); x.trace_n = CS(CS_TRACEN); x.mslot = CS(CS_MSLOT);
  x.netmode = CS(CS_NETMODE); x.t_ctr = CS(CS_TCTR);
  x.conn = CS(CS_CONN); x.alive = CS(CS_ALIVE); x.twake = CS(CS_TWAKE); x.lmask = CS(CS_LMASK);
  if constexpr (nthr(S) > 0) { x.cwake = CS(CS_CWAKE); x.ctid = CS(CS_CTID); x.cslot = CS(CS_CSLOT); }
#pragma unroll
  for (uint32_t d = 0; d < NB; d++) x.timer[d] = d < D.n ? TMR(d) : INF_T;
#pragma unroll
  for (uint32_t w = 0; w < MW; w++) x.free_mask[w] = C64(w ? C64_FREE1 + w - 1 : C64_FREE);
  x.digest = C64(C64_DIGEST); x.mmin = C64(C64_MMIN);
#pragma unroll
  for (uint32_t k = 0; k < CNT__N; k++) x.cnt[k] = CS(CS_CNT + k);
  for (uint32_t s = 0; s < D.M; s++) LK(s) = (lkey_t)MKEY(s);
  // every load above completes here (each loaded register is read by an empty asm): a lane that
  // takes a new cluster inside the step loop (streaming) then leaves no load pending into the
  // loop, where the compiler would otherwise place a conservative vmcnt(0) — one that also
  // waits for every store in flight — at the first later use of these registers on EVERY
  // iteration's path
  asm volatile("" ::"v"(x.now), "v"(x.events), "v"(x.msgs_sent), "v"(x.inflight), "v"(x.trace_n),
               "v"(x.mslot), "v"(x.netmode), "v"(x.t_ctr), "v"(x.conn), "v"(x.alive), "v"(x.twake),
               "v"(x.lmask), "v"(x.digest), "v"(x.mmin));
  if constexpr (nthr(S) > 0) asm volatile("" ::"v"(x.cwake), "v"(x.ctid), "v"(x.cslot));
#pragma unroll
  for (uint32_t d = 0; d < NB; d++) asm volatile("" ::"v"(x.timer[d]));
#pragma unroll
  for (uint32_t w = 0; w < MW; w++) asm volatile("" ::"v"(x.free_mask[w]));
#pragma unroll
  for (uint32_t k = 0; k < CNT__N; k++) asm volatile("" ::"v"(x.cnt[k]));
}
template <uint32_t S>
DI void lane_store(const Dev& D, X& x) {
  CS(CS_CODE) = x.code;
  if (x.code != RUN) CS(CS_VTIME) = x.now;
  CS(CS_NOW) = x.now; CS(CS_EVENTS) = x.events; CS(CS_MSGS) = x.msgs_sent;
  CS(CS_INFLIGHT) = x.inflight; CS(CS_TRACEN) = x.trace_n; CS(CS_MSLOT) = x.mslot;
  CS(CS_NETMODE) = x.netmode; CS(CS_TCTR) = x.t_ctr;
  CS(CS_CONN) = x.conn; CS(CS_ALIVE) = x.alive; CS(CS_TWAKE) = x.twake; CS(CS_LMASK) = x.lmask;
  if constexpr (nthr(S) > 0) { CS(CS_CWAKE) = x.cwake; CS(CS_CTID) = x.ctid; CS(CS_CSLOT) = x.cslot; }
#pragma unroll
  for (uint32_t d = 0; d < NB; d++)
    if (d < D.n) TMR(d) = x.timer[d];
#pragma unroll
  for (uint32_t w = 0; w < MW; w++) C64(w ? C64_FREE1 + w - 1 : C64_FREE) = x.free_mask[w];
  C64(C64_DIGEST) = x.digest; C64(C64_MMIN) = x.mmin;
#pragma unroll
  for (uint32_t k = 0; k < CNT__N; k++) CS(CS_CNT + k) = x.cnt[k];
  if (x.code != RUN) return;  // a finished cluster's messages are never read again
  for (uint32_t s = 0; s < D.M; s++) MKEY(s) = LK(s) == LKEY_FREE ? ~0ull : (uint64_t)LK(s);
}
// lanes that want a cluster (`want`) take the next unclaimed ones, one atomic per wave per
// round; a taken cluster that already has its verdict (a later launch of a long run) is
// skipped. Returns whether this lane now holds a running cluster.
template <uint32_t S>
DI bool lane_claim(const Dev& D, X& x, bool want) {
  bool held = false;
  for (uint64_t wm = __ballot(want); wm; wm = __ballot(want)) {
    const uint32_t first = (uint32_t)__builtin_ctzll(wm);
    uint32_t base = 0;
    if (__lane_id() == first) base = atomicAdd(&D.remaining[1], (uint32_t)__popcll(wm));
    base = __shfl(base, (int)first);
    if (want) {
      x.c = base + (uint32_t)__popcll(wm & ((1ull << __lane_id()) - 1ull));
      if (x.c >= D.C) {
        want = false;
        x.code = MR_PASS;  // nothing left: the lane idles
      } else {
        lane_load<S>(D, x);
        if (x.code == RUN) { held = true; want = false; }
      }
    }
  }
  return held;
}

// waves per SIMD the register allocation targets: the kvraft / shard_ctrler kernels keep 64
// message slots (LDS for one wave per SIMD), so they take the whole register file and keep
// their overflow in AGPRs instead of scratch (config 5: 299 -> 265 ms)
// (and the generic 8-server instances, which serve only node counts without an exact one: one
// wave per SIMD, no scratch); the other kernels two waves per SIMD
template <uint32_t S>
constexpr uint32_t step_waves() {
  return NB >= 8 || is_svc(S) ? 1u : 2u;
}
// exact-size instances (NB < 8, mr_dev.h has_exact): the node count is NB at compile time
constexpr bool EXACT_N = MR_NB < MR_MAX_NODES;
template <uint32_t S, uint32_t NBT>
__global__ void __launch_bounds__(STEP_BLOCK, step_waves<S>()) step_kernel(Dev Din, uint32_t budget) {
  static_assert(NBT == NB, "one node bound per translation unit");
  Dev D = Din;
  if constexpr (EXACT_N) D.n = NB;  // the host launches this instance for D.n == NB only
  // configuration the scenario fixes (mr_host.cpp sets the same values): compile-time here, so no
  // loop-invariant predicate on them is kept in scalar registers across the step loop
  D.nthr = nthr(S);
  D.links = kv_gen(S).part ? 1u : 0u;
  D.lin15 = kv_gen(S).lin ? 1u : 0u;
  if constexpr (!is_svc(S)) D.kv32 = nullptr;
  if constexpr (kv_gen(S).maxraft == 0) D.kvs32 = nullptr;
  if constexpr (is_svc(S)) __builtin_assume(D.kv32 != nullptr);
  if constexpr (kv_gen(S).maxraft > 0) __builtin_assume(D.kvs32 != nullptr);
  X x;
  // lanes 0 .. lpw - 1 of each 64-lane block hold clusters (D.lpw < 64: a batch smaller than the
  // resident lanes still spreads over two waves per SIMD; the other lanes idle)
  x.c = blockIdx.x * D.lpw + threadIdx.x;  // this launch's lane
#ifdef MR_PROF
  if ((threadIdx.x & 63) == 0) {
    for (uint32_t k = 0; k < 2 * P__N; k++) s_prof[threadIdx.x >> 6][k] = 0;
    s_prof[threadIdx.x >> 6][2 * P__N] = wall_clock64();
  }
#endif
  const bool lane_ok = threadIdx.x < D.lpw && x.c < D.L;
  bool in;
  if (D.stream && D.resume) {  // a later launch of a streaming batch: the clusters the previous
    in = lane_ok && x.c < D.nheld;  // launch's lanes still held first, then the claim pointer
    if (in) x.c = D.held_in[x.c];
  } else {
    x.c += D.c0;  // lane l starts with cluster c0 + l of this launch's chunk
    in = lane_ok && x.c < D.C;
  }
  x.code = MR_PASS;
  if (in) lane_load<S>(D, x);
  bool held = x.code == RUN;  // this lane runs cluster x.c (its state is in registers / LDS)
  if (D.stream) held = held || lane_claim<S>(D, x, (D.resume ? lane_ok : in) && !held);
  PROF(P_PRO);
  uint64_t key = 0;
  uint32_t cls = CLS_NONE, node = 0;
  bool need = true, tcli = false;
  for (uint32_t it = 0; it < budget; it++) {
    asm volatile("" : "+v"(x.c));  // no LICM of per-lane addresses: recompute, do not keep live
    PROF(P_TAIL);
    if (D.stream) {  // streaming lanes: the last iteration's finished clusters make way
      const bool fin = held && x.code != RUN;
      if (__ballot(fin)) {
        if (fin) lane_store<S>(D, x);
        const bool got = lane_claim<S>(D, x, fin);
        if (fin) { held = got; need = true; }
      }
    }
    const bool run = x.code == RUN;
    if (__ballot(run) == 0) break;
    if (run && need) {  // next event: min over tester wake-up, node timers, earliest message
      key = ((uint64_t)x.twake << 32) | (2ull << 30);
      cls = CLS_TESTER;
      if constexpr (nthr(S) > 0) {  // the earliest spawned thread (tie = tid)
        const uint64_t kc = ((uint64_t)x.cwake << 32) | (2ull << 30) | x.ctid;
        tcli = kc < key;
        if (tcli) key = kc;
      }
#pragma unroll
      for (uint32_t d = 0; d < NB; d++) {  // timers of absent nodes are INF_T
        uint64_t kt = ((uint64_t)x.timer[d] << 32) | (1ull << 30) | d;
        if (kt < key) { key = kt; cls = CLS_TIMER; node = d; }
      }
      if (x.mmin < key) { key = x.mmin; cls = CLS_MSG; node = (uint32_t)key & 31u; }
      need = false;
    }
    // wave-uniform choice of the event class processed this iteration
    const uint32_t nm = __popcll(__ballot(run && cls == CLS_MSG));
    const uint32_t nt = __popcll(__ballot(run && cls == CLS_TIMER));
    const uint32_t ns = __popcll(__ballot(run && cls == CLS_TESTER));
    // tester events run when >= 1/3 of the live lanes want them (A/B: 1/4, 2/5, 1/2 lose
    // 0.3-2.6 %), node events (messages and timers, one node_event pass) otherwise
    const bool tpick = 3u * ns >= nm + nt + ns;
    bool mine = tpick ? cls == CLS_TESTER : cls != CLS_TESTER;
    // AppendEntries deliveries (the longest node path: probe, payload batches, log writes) wait
    // until they are >= AE_NUM / AE_DEN of the wave's node events, so the other node events run
    // without their round trips; like any lane that waits, a cluster's own order is unchanged
    if constexpr (!MR_KEY32 && !is_svc(S) && !restarts_servers(S)) {
      if (!tpick) {
        const bool ae = run && cls == CLS_MSG && ((key >> 5) & 1u);
        const uint32_t nae = __popcll(__ballot(ae));
        if (nae < nm + nt && 2u * nae < nm + nt && nm + nt - nae >= AE_OTHERS) mine = mine && !ae;
      }
    }
    PROF(P_SEL);
    if (!run || !mine) continue;
    if (nthr(S) > 0 && (uint32_t)(key >> 32) == INF_T) {  // nothing can wake the test body
      fail(D, x, MR_FAIL_SIM_BAD_PROGRAM);
      continue;
    }
    x.now = (uint32_t)(key >> 32);
    need = true;
    x.events++;
    if (x.events > D.max_events) { fail(D, x, MR_FAIL_SIM_EVENT_LIMIT); continue; }
    if (cls != CLS_TESTER) {
      CADD(cls == CLS_MSG ? CNT_EV_MSG : CNT_EV_TIMER, 1u);
      node_event<S>(D, x, cls == CLS_MSG, node, x.mslot, ((uint32_t)key & 0x3FFFFFFFu) >> 6);
    } else {
      CADD(CNT_EV_TESTER, 1u);
      if constexpr (nthr(S) > 0) {
        if (tcli) thr_step<S>(D, x, x.cslot);
        else tester<S>(D, x);
      } else {
        tester<S>(D, x);
      }
      PROF(P_TESTER);
    }
  }
#ifdef MR_PROF
  PROF(P_TAIL);
  if ((threadIdx.x & 63) == 0)
    for (uint32_t k = 0; k < P__N; k++) {
      atomicAdd(&D.prof[k], s_prof[threadIdx.x >> 6][k]);
      atomicAdd(&D.prof[32 + k], s_prof[threadIdx.x >> 6][P__N + k]);
    }
#endif
  if (!held) return;
  lane_store<S>(D, x);
  if (x.code == RUN) {  // still running: counted, and (streaming) resumed first by the next launch
    const uint32_t k = atomicAdd(D.remaining, 1u);
    if (D.stream) D.held_out[k] = x.c;
  }
}

#if MR_POOL
#include "mr_pool.inc"
#endif

#ifndef MR_COMMON
#define MR_COMMON 1
#endif
#if MR_COMMON
// RaftTester state before the test body runs (SEMANTICS §3: tester wakes at t = 0)
__global__ void __launch_bounds__(256) reset_kernel(Dev D) {
  X x;
  x.c = blockIdx.x * blockDim.x + threadIdx.x;
  if (x.c >= D.C) return;
  for (uint32_t f = 0; f < CS__N; f++) CS(f) = 0;
  CS(CS_CODE) = RUN;
  for (uint32_t f = 0; f < C64__N; f++) C64(f) = 0;
  for (uint32_t w = 0; w < 4; w++) {  // the first M slots are free
    const uint32_t mw = D.M > 64u * w ? D.M - 64u * w : 0u;
    C64(w ? C64_FREE1 + w - 1 : C64_FREE) = mw >= 64 ? ~0ull : ((1ull << mw) - 1ull);
  }
  C64(C64_DIGEST) = FNV_OFF;
  C64(C64_MMIN) = ~0ull;
  for (uint32_t d = 0; d < D.n; d++) {
    for (uint32_t f = 0; f < NF__N; f++) ND(f, d) = 0;
    ND(NF_FLAGS, d) = 15u << 4;  // follower, voted none (down, disconnected: CS_ALIVE/CS_CONN = 0)
    TMR(d) = INF_T;
    ND(NF_SLEN, d) = 1;
    ND(NF_PLO, d) = 1;  // no pending payload range
    NSV(d) = 0;
    for (uint32_t p = 0; p < D.n; p++) { PR(PF_NEXT, d, p) = 0; PR(PF_MATCH, d, p) = 0; }
  }
  for (uint32_t s = 0; s < D.M; s++) MKEY(s) = ~0ull;
  CS(CS_MJOIN) = 0xFFFFFFFFu;
  CS(CS_CWAKE) = INF_T;
  for (uint32_t q = 0; q < TF_Q; q++) D.tfr[(size_t)x.c * TF_Q + q] = make_uint4(0u, 0u, 0u, 0u);
  if (D.kt32) {  // spawned threads: slot 0 = the test body (+ ck, clerk 0); others empty
    for (uint32_t s = 0; s < D.nthr; s++)
      for (uint32_t f = 0; f < KT__N; f++) KT(f, s) = 0u;
    KT(KT_LIVE, 0) = 1u;
    // the scheduler keys: empty slots (INF_T, tid 0); slot 0 (the test body: x.twake) and the
    // pad slot ~0, below no key
    uint32_t* kw = D.kwk + (size_t)x.c * kws(D.nthr) * 2u;
    for (uint32_t s = 0; s < kws(D.nthr); s++) {
      const bool none = s == 0 || s >= D.nthr;
      kw[2 * s] = none ? ~0u : 0u;
      kw[2 * s + 1] = none ? ~0u : INF_T;
    }
  }
  if (D.cfg32)  // shard_ctrler: every server starts with config 0 (num 0, no groups)
    for (uint32_t d = 0; d < D.n; d++) {
      D.kv32[((size_t)x.c * D.n + d) * KVREC + KVR_NCFG] = 1u;
      uint32_t* c0 = D.cfg32 + (((size_t)x.c * D.n + d) * CFG_CAP) * CFGW;
      for (uint32_t w = 0; w < CF_GID; w++) c0[w] = 0u;
    }
}

// counters_reduce: per-GPU sums / maxima / verdict histogram / first failing
// cluster; out[] layout documented in mr_host.cpp (RED_*)
__global__ void __launch_bounds__(256) reduce_kernel(Dev D, unsigned long long* out,
                                                    uint64_t cluster_base) {
  constexpr uint32_t RN = CNT__N + 8 + 64 + 32 + 3;  // counters, scalars, verdicts, coverage, kv
  __shared__ unsigned long long acc[RN];
  for (uint32_t i = threadIdx.x; i < RN; i += blockDim.x) acc[i] = 0;
  __syncthreads();
  X x;
  x.c = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < CNT__N) {  // the pool kernels' workgroup sums
    const unsigned long long v = D.pcnt[threadIdx.x];
    if (v) {
      if (threadIdx.x >= CNT_MAX_INFLIGHT) atomicMax(&acc[threadIdx.x], v);
      else atomicAdd(&acc[threadIdx.x], v);
    }
  }
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
    auto bucket = [](uint32_t v) { return v == 0 ? 0u : min(15u, 32u - (uint32_t)__builtin_clz(v)); };
    atomicAdd(&acc[CNT__N + 72 + bucket(CS(CS_CNT + CNT_LEADERS))], 1ull);
    atomicAdd(&acc[CNT__N + 88 + bucket(CS(CS_EVENTS))], 1ull);
    atomicAdd(&acc[CNT__N + 104], (unsigned long long)CS(CS_KV_OPS));
    atomicAdd(&acc[CNT__N + 105], (unsigned long long)CS(CS_KV_CHECKED));
    atomicAdd(&acc[CNT__N + 106], (unsigned long long)CS(CS_KV_LIN));
    if (code != RUN && code != MR_PASS)
      atomicMin(&out[CNT__N + 5], (unsigned long long)(cluster_base + x.c));
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < RN; i += blockDim.x) {
    if (i == CNT__N + 5 || i == CNT__N + 6 || i == CNT__N + 7) continue;
    if (acc[i] == 0) continue;
    if (i >= CNT_MAX_INFLIGHT && i < CNT__N) atomicMax(&out[i], acc[i]);
    else atomicAdd(&out[i], acc[i]);
  }
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
#endif  // MR_COMMON

template <uint32_t S, uint32_t NBT>
hipError_t launch_step_t(const Dev& D, uint32_t budget, hipStream_t s) {
  dim3 blk(STEP_BLOCK), grd((D.L + D.lpw - 1) / D.lpw);
  const size_t lds = (size_t)D.M * STEP_BLOCK * sizeof(lkey_t) +  // message keys
                    2 * MR_MAX_NODES * STEP_BLOCK * sizeof(uint32_t);  // send-loop staging
  hipLaunchKernelGGL((step_kernel<S, NBT>), grd, blk, lds, s, D, budget);
  return hipGetLastError();
}
// clusters the step kernel keeps resident: blocks per CU (registers, LDS for M message slots)
// x CUs x lanes per block
template <uint32_t S, uint32_t NBT>
uint32_t step_capacity_t(int device, uint32_t M) {
  const size_t lds = (size_t)M * STEP_BLOCK * sizeof(lkey_t) + 2 * MR_MAX_NODES * STEP_BLOCK * sizeof(uint32_t);
  int blocks = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, (const void*)step_kernel<S, NBT>, STEP_BLOCK,
                                                   lds) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return 0;
  return (uint32_t)blocks * (uint32_t)cus * STEP_BLOCK;
}
// Step-kernel instances built by this translation unit: build.py compiles
// this file once per scenario group (-DMR_SCN_LIST=...) in parallel, and once
// with MR_COMMON=1 for the reset / reduce kernels.
#ifndef MR_SCN_LIST
#define MR_SCN_LIST MR_ALL_SCNS
#endif
#if MR_TAPE  // replay / record batches run one launch of all their clusters
#define MR_INST(S) template hipError_t launch_step_t<S, MR_NB>(const Dev&, uint32_t, hipStream_t);
#elif MR_POOL
#define MR_INST(S)                                                                     \
  template hipError_t launch_pool_t<S, MR_NB>(const Dev&, uint32_t, hipStream_t);      \
  template uint32_t pool_capacity_t<S, MR_NB>(int, uint32_t);
#else
#define MR_INST(S)                                                                     \
  template hipError_t launch_step_t<S, MR_NB>(const Dev&, uint32_t, hipStream_t);      \
  template uint32_t step_capacity_t<S, MR_NB>(int, uint32_t);
#endif
MR_SCN_LIST
#undef MR_INST

}  // namespace mr
