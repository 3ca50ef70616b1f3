/*
 * mr_oracle.c — CPU oracle (TEST INFRASTRUCTURE ONLY; see mr_oracle.h).
 *
 * One cluster at a time, madsim-shaped: a binary heap of (time, class, tie)
 * keys holds in-flight messages and node timers (timers are lazily
 * invalidated by a generation number, as an executor's cancelled timers
 * would be); the tester script is ordinary sequential C whose sleep() drains
 * the heap up to its wake time, and whose panics longjmp to the seed loop.
 * Semantics: docs/SEMANTICS.md. Reference lines are cited per function.
 */
#include "mr_oracle.h"

#include <setjmp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon, Moraes, Dror, Shaw SC'11; Random123 constants) */
/* ------------------------------------------------------------------ */
void mro_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; r++) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

enum { ST_TESTER = 1, ST_ELECT = 2, ST_NET = 3 };
enum { R_F = 0, R_C = 1, R_L = 2, R_DOWN = 3 };
enum { M_RV_REQ = 1, M_RV_REP, M_AE_REQ, M_AE_REP, M_IS_REQ, M_IS_REP, M_KV_REQ, M_KV_REP };
enum { KV_GET = 0, KV_PUT = 1, KV_APPEND = 2 };
enum { KV_OK = 0, KV_WRONG_LEADER = 1, KV_FAILED = 2 };
#define CLERK_HOST 8u   /* the clerk of thread slot k is host 8 + k (SEMANTICS §9) */
#define MAX_CLERKS 128u /* clerk ids (make_client order) */
#define KV_KEYS 64u     /* keys a KV server may hold */
#define KV_APP 5u       /* distinct appenders tracked per key */
#define LIN_CLI 15u     /* generic_test_linearizability: clients, keys, appender states per key (§9b) */
#define KV_ALL 0xFFFFFFu /* Get elem: the states of appenders 0..4, packed */
#define KV_HP 0x100000001B3ull /* value hash multiplier (SEMANTICS §9) */
#define KV_SLOTS 6u     /* thread / clerk slots: 0 = main + ck, 1 + cli = client cli */
#define KV_PEND 8u
#define CK_SLOTS 24u    /* clerk slots (thread slot k owns clerk k, host 8 + k) */
#define MAX_THR 64u     /* tester thread slots (unreliable_agree_2c: concurrent one() tasks) */
#define JOIN_ALL 0xFFFFFFFEu
#define JOIN_ANY 0xFFFFFFFDu /* select! over spawned tasks: the first finish wakes the body */
#define CHURN_VCAP 512u /* values a churn client may record (tests.rs:763-797) */
/* shard_ctrler (SEMANTICS §10) */
#define N_SHARDS 10u    /* shard_ctrler/mod.rs:9 */
#define CFG_CAP 128u    /* configs a controller server may hold */
#define CFG_G 32u       /* groups in one config */
#define OP_CAP 256u     /* clerk operations per cluster */
enum { CT_QUERY = 0, CT_JOIN = 1, CT_LEAVE = 2, CT_MOVE = 3 };
#define INF_T 0xFFFFFFFFu
#define LOSS_Q32 429496729u /* floor(0.1 * 2^32), tester.rs:130 */

/* keyed decisions (SEMANTICS §12): mode 1 replays (a sorted copy, rows by batch-relative
 * cluster), mode 2 records in draw order; set by mro_set_decisions */
static mr_decision* g_dec;       /* mode 1: sorted by (cluster, stream, entity, seq) */
static uint64_t* g_dec_off;      /* mode 1: row r = g_dec[g_dec_off[r] .. g_dec_off[r + 1]) */
static uint64_t g_dec_rows;
static mr_decision* g_rec;       /* mode 2: [rows][g_rec_cap] */
static uint64_t g_rec_cap, *g_dec_count;
static int g_tape_mode;

static inline uint32_t u_range(uint32_t w, uint32_t lo, uint32_t hi) {
  return lo + (uint32_t)(((uint64_t)w * (uint64_t)(hi - lo)) >> 32);
}

/* ------------------------------------------------------------------ */
/* cluster state                                                        */
/* ------------------------------------------------------------------ */
typedef struct {
  uint32_t time, seq;
  uint8_t type, src, dst, inc;
  uint32_t term, a, b, c, k;
  uint64_t v;
  uint32_t et[MR_MAX_AE];
  uint64_t ev[MR_MAX_AE];
} OMsg;

typedef struct {
  uint32_t term; int32_t voted; uint32_t role; int alive, conn; uint32_t inc;
  uint32_t commit, applied, last, snap_idx, snap_term; uint64_t snap_val;
  uint32_t timer_gen, votes;
  uint32_t next[MR_MAX_NODES], match[MR_MAX_NODES];
  uint32_t e_ctr, n_ctr;
  uint32_t* lterm; uint64_t* lval; /* ring of log_cap */
} ONode;

typedef struct { uint64_t key; uint32_t ref; uint32_t gen; } HEnt;

/* kvraft clerk (kvraft/client.rs ClerkCore) and the tester thread that owns it */
typedef struct {
  uint32_t id, lh, seq, tag, nctr, waiting, got, rstat, rhint, rval; uint64_t rvh;
  uint32_t owner, mcl; /* the thread its calls wake (0 = the test body); mcl: a test-body clerk */
  uint32_t op, key, elem;
  uint32_t llo; /* a Get's lower bound at its call (SEMANTICS §9a) */
  uint32_t lepoch, lnopend; /* §9b: the key's Put epoch at the call; no Put pending at the call */
} OClerk;
typedef struct {
  uint32_t tid, live, pc, j, cli, tctr, gen;
  uint32_t kind, perm;
  uint64_t hlast; /* generic_test client: hash of its predicted value `last` */ /* kind 1 = generic_test partitioner (perm: its shuffled `all`, 4 bits/server) */
  /* churn client (tests.rs:763-797) */
  uint64_t xv; uint32_t idx, has, toi, nval;
  /* one() task (tester.rs:216-262) */
  uint64_t cmd; uint32_t t0, starts, index, t1, ph, expected, retry;
} OThr;
typedef struct { uint32_t used, idx, clerk, seq, tag, ready, status, value, host; uint64_t vh; } OPend;
/* a key's value (SEMANTICS §9): the hash of its token sequence, its byte length, and
 * per appender (cli + 1 | count << 8 | bad << 31) for the append-order checks */
/* (generic_test_linearizability, SEMANTICS §9b: app[cli] = count | last j << 12 | bad << 31) */
typedef struct { uint64_t h; uint32_t len; uint32_t app[LIN_CLI]; } OKey;
/* a KV server's state machine as its snapshot holds it (SEMANTICS §9) */
typedef struct { uint32_t dedup[MAX_CLERKS]; OKey keys[KV_KEYS]; } OKvState;
#define KV_SNAP_EVERY 16u /* the service snapshots at applied indices that are multiples of 16 */
#define KV_RING 16u       /* recent snapshots by index / 16 mod 16, read by InstallSnapshot */
/* Config (shard_ctrler/msg.rs:11-18): groups sorted by gid; a server list is
 * packed as len | a0 << 8 | a1 << 16 | a2 << 24 (addrs! takes `as u8`) */
typedef struct { uint32_t num, shards[N_SHARDS], ng, gid[CFG_G], addr[CFG_G]; } OCfg;
/* Op (shard_ctrler/msg.rs:21-37): a = num (Query) / shard (Move), b = gid (Move) */
typedef struct { uint32_t type, a, b, ng, gid[5], addr[5]; } OOp;

typedef struct {
  mr_cfg cfg;
  uint32_t n, key[2], now, scenario, snapshot_mode, null_raft;
  uint32_t lat_lo, lat_hi, loss;
  ONode nd[MR_MAX_NODES];
  /* network */
  OMsg pool[MR_MAX_MSG_SLOTS]; uint32_t free_stack[MR_MAX_MSG_SLOTS]; uint32_t n_free;
  uint32_t inflight;
  HEnt* heap; uint32_t heap_n, heap_cap;
  /* tester */
  uint32_t t_ctr;
  uint8_t* mask; uint64_t* sval; uint32_t* sterm; uint32_t slen[MR_MAX_NODES];
  /* kvraft (SEMANTICS §8-9) */
  uint32_t kv_mode, kv_done, next_tid, mwake, main_join;
  OKey kv[MR_MAX_NODES][KV_KEYS]; uint32_t kv_dedup[MR_MAX_NODES][MAX_CLERKS];
  uint32_t kv_maxraft;                /* maxraftstate (0 = None) */
  OKvState* kvs;                      /* [MR_MAX_NODES] persisted KV snapshots */
  OKvState* kring; uint32_t* kring_idx; /* [KV_RING] */
  OPend pend[MR_MAX_NODES][KV_PEND];
  OClerk ck[CK_SLOTS]; OThr th[MAX_THR];
  uint64_t* cval; uint32_t* cidx; /* churn values [3][CHURN_VCAP] + their indices */
  uint32_t ctrl_mode, nops, ncfg[MR_MAX_NODES];
  uint32_t led[64];   /* MR_F_SAFETY: bit t = a leader was elected in term t (t < 2048) */
  uint32_t lin[KV_KEYS][KV_APP][5]; /* linearizability: per (key, appender) tag, called, acked,
                                     * seen, and a pending all-appenders Get's lower bound */
  uint32_t lin15; /* generic_test_linearizability (SEMANTICS §9b): keys of 15 client states */
  uint32_t l15_called[16][LIN_CLI], l15_acked[16][LIN_CLI], l15_epoch[16], l15_pend[16];
  uint32_t l15_j[LIN_CLI]; /* client cli's next token j, carried over iterations (tokens unique) */
  uint8_t link[MR_MAX_NODES]; /* server links (connect2/disconnect2): bit j of link[i] = i~j */
  uint64_t tape_row; int tape_on; uint64_t tape_pos; /* keyed decisions: row, count (§12) */
  /* apply digests (ABI 4 mr_trace_digests): per node the sum of mr_apply_mix over the entries it
   * applied one by one, invalid once it installed a snapshot or restarted above index 0 */
  uint64_t adig[MR_MAX_NODES]; uint8_t ainv[MR_MAX_NODES];
  uint8_t ccut[CK_SLOTS];     /* clerk links cut: bit j of ccut[k] = clerk host 8 + k !~ server j */
  OCfg* cfgs; /* [MR_MAX_NODES][CFG_CAP] */
  OOp* ops;   /* [OP_CAP] */
  uint32_t churn_stop;
  /* results */
  mro_result r;
  mr_event* trace; size_t trace_cap, n_trace;
  uint64_t* tdig; /* [trace_cap] the apply digest beside each record (0: not a node event) */
  uint64_t* tapp; /* [trace_cap][2] KV command, key hash after its first application */
  jmp_buf jb;
} OSim;

/* ------------------------------------------------------------------ */
/* trace / verdict                                                      */
/* ------------------------------------------------------------------ */
static void rec_push(OSim* s, const mr_event* e) {
  const uint32_t* w = (const uint32_t*)e;
  uint64_t h = s->r.digest;
  for (int i = 0; i < 8; i++) { h ^= w[i]; h *= 0x100000001B3ull; }
  s->r.digest = h;
  if (s->trace && s->n_trace < s->trace_cap) s->trace[s->n_trace] = *e;
  if (s->tdig && s->n_trace < s->trace_cap) s->tdig[s->n_trace] = 0;
  s->n_trace++;
}

static void rec_node(OSim* s, uint32_t cls, uint32_t kind, uint32_t node, uint32_t aux) {
  const ONode* d = &s->nd[node];
  mr_event e;
  e.time_us = s->now; e.cls = (uint8_t)cls; e.kind = (uint8_t)kind; e.node = (uint8_t)node;
  e.role = (uint8_t)(d->alive ? d->role : R_DOWN);
  e.aux = aux; e.term = d->term; e.commit = d->commit; e.applied = d->applied;
  e.last = d->last; e.snap = d->snap_idx;
  const size_t idx = s->n_trace;
  rec_push(s, &e);
  if (s->tdig && idx < s->trace_cap) s->tdig[idx] = s->ainv[node] ? ~0ull : s->adig[node];
}

static void rec_simple(OSim* s, uint32_t cls, uint32_t kind) {
  mr_event e;
  memset(&e, 0, sizeof e);
  e.time_us = s->now; e.cls = (uint8_t)cls; e.kind = (uint8_t)kind; e.node = 0xFF;
  e.aux = (uint32_t)s->r.msgs_sent;
  rec_push(s, &e);
}

/* panic!(..): the verdict record, then unwind to the seed loop (README.md:44-48) */
static void t_fail(OSim* s, uint32_t code) {
  s->r.code = code; s->r.time_us = s->now;
  rec_simple(s, 3, code);
  longjmp(s->jb, 1);
}

static void count_event(OSim* s) {
  s->r.events++;
  if (s->r.events > s->cfg.max_events) t_fail(s, MR_FAIL_SIM_EVENT_LIMIT);
}

/* ------------------------------------------------------------------ */
/* executor: binary heap                                                */
/* ------------------------------------------------------------------ */
static void heap_push(OSim* s, uint64_t key, uint32_t ref, uint32_t gen) {
  if (s->heap_n == s->heap_cap) {
    s->heap_cap = s->heap_cap ? 2 * s->heap_cap : 256;
    s->heap = (HEnt*)realloc(s->heap, s->heap_cap * sizeof(HEnt));
  }
  uint32_t i = s->heap_n++;
  while (i) {
    uint32_t p = (i - 1) >> 1;
    if (s->heap[p].key <= key) break;
    s->heap[i] = s->heap[p];
    i = p;
  }
  s->heap[i].key = key; s->heap[i].ref = ref; s->heap[i].gen = gen;
}

static HEnt heap_pop(OSim* s) {
  HEnt top = s->heap[0];
  HEnt last = s->heap[--s->heap_n];
  uint32_t i = 0, n = s->heap_n;
  for (;;) {
    uint32_t l = 2 * i + 1;
    if (l >= n) break;
    uint32_t m = (l + 1 < n && s->heap[l + 1].key < s->heap[l].key) ? l + 1 : l;
    if (s->heap[m].key >= last.key) break;
    s->heap[i] = s->heap[m];
    i = m;
  }
  if (n) s->heap[i] = last;
  return top;
}

static void set_timer(OSim* s, uint32_t d, uint32_t t) {
  ONode* x = &s->nd[d];
  x->timer_gen++;
  heap_push(s, ((uint64_t)t << 32) | (1ull << 30) | d, d, x->timer_gen);
}

static int dec_cmp(const mr_decision* a, uint32_t stream, uint32_t entity, uint32_t seq) {
  if (a->stream != stream) return a->stream < stream ? -1 : 1;
  if (a->entity != entity) return a->entity < entity ? -1 : 1;
  if (a->seq != seq) return a->seq < seq ? -1 : 1;
  return 0;
}

/* every random draw of the simulation: Philox4x32-10 with counter (seq, entity, stream)
 * keyed by the seed (§2), or the keyed decision recorded for (stream, entity, seq) (§12) */
static void draw(OSim* s, const uint32_t ctr[4], uint32_t w[4]) {
  if (s->tape_on && g_tape_mode == 1) {
    const mr_decision* row = g_dec + g_dec_off[s->tape_row];
    uint64_t lo = 0, hi = g_dec_off[s->tape_row + 1] - g_dec_off[s->tape_row];
    while (lo < hi) { /* binary search of the row */
      uint64_t mid = (lo + hi) / 2;
      int c = dec_cmp(&row[mid], ctr[2], ctr[1], ctr[0]);
      if (c == 0) { w[0] = row[mid].w0; w[1] = row[mid].w1; w[2] = w[3] = 0; return; }
      if (c < 0) lo = mid + 1; else hi = mid;
    }
    s->tape_pos++; /* no record: the seed's own draw */
  }
  mro_philox4x32_10(ctr, s->key, w);
  if (s->tape_on && g_tape_mode == 2) {
    uint64_t p = s->tape_pos++;
    if (p < g_rec_cap) {
      mr_decision* r = &g_rec[s->tape_row * g_rec_cap + p];
      r->cluster = (uint32_t)s->tape_row; r->stream = (uint16_t)ctr[2];
      r->entity = (uint16_t)ctr[1]; r->seq = ctr[0]; r->w0 = w[0]; r->w1 = w[1];
    }
  }
}

/* raft.rs:260-263 generate_election_timeout: U[150,300) ms */
static void reset_timer(OSim* s, uint32_t d) {
  ONode* x = &s->nd[d];
  uint32_t ctr[4] = {x->e_ctr++, d, ST_ELECT, 0}, w[4];
  draw(s, ctr, w);
  set_timer(s, d, s->now + u_range(w[0], s->cfg.elect_lo_us, s->cfg.elect_hi_us));
}

/* ------------------------------------------------------------------ */
/* network (madsim net: tester.rs:127-137 config, :147-149 stat)        */
/* ------------------------------------------------------------------ */
static int host_conn(OSim* s, uint32_t h) { return h < CLERK_HOST ? s->nd[h].conn : 1; }
/* the link between two hosts (madsim connect2/disconnect2, kvraft/tester.rs:88-124):
 * server-server links are symmetric bits; clerk links are always up here */
static int link_up(OSim* s, uint32_t a, uint32_t b) {
  if (a >= CLERK_HOST && b >= CLERK_HOST) return 1;
  if (a >= CLERK_HOST) return !((s->ccut[a - CLERK_HOST] >> b) & 1u);
  if (b >= CLERK_HOST) return !((s->ccut[b - CLERK_HOST] >> a) & 1u);
  return (s->link[a] >> b) & 1u;
}
static uint32_t* host_nctr(OSim* s, uint32_t h) {
  if (h < CLERK_HOST) return &s->nd[h].n_ctr;
  return &s->ck[h - CLERK_HOST].nctr;
}
/* the sender's identity in its NET draws (§2, §12): server i, or clerk id k as 8 + k (a
 * clerk's host slot is reused by later clerks; its id, like madsim's 0.0.2.id address, is not) */
static uint32_t host_entity(OSim* s, uint32_t h) {
  return h < CLERK_HOST ? h : CLERK_HOST + s->ck[h - CLERK_HOST].id;
}

static void net_send(OSim* s, uint32_t src, uint32_t dst, OMsg* m) {
  uint32_t seq = (uint32_t)s->r.msgs_sent;
  s->r.msgs_sent++;
  uint32_t ctr[4] = {(*host_nctr(s, src))++, host_entity(s, src), ST_NET, 0}, w[4];
  draw(s, ctr, w);
  if (!host_conn(s, src) || !host_conn(s, dst) || !link_up(s, src, dst)) { s->r.drop_clog++; return; }
  if (w[0] < s->loss) { s->r.drop_loss++; return; }
  /* madsim's net has no in-flight cap: a full slot table is a simulator limit, not loss */
  if (s->inflight >= s->cfg.msg_slots) { s->r.drop_overflow++; t_fail(s, MR_FAIL_SIM_CAPACITY); }
  if (seq >= (1u << 24)) t_fail(s, MR_FAIL_SIM_CAPACITY); /* SEMANTICS §3, §9 */
  m->time = s->now + u_range(w[1], s->lat_lo, s->lat_hi);
  if (m->time >= (1u << 27) - 1u) t_fail(s, MR_FAIL_SIM_CAPACITY); /* SEMANTICS §4: t < 2^27 - 1 */
  m->seq = seq; m->src = (uint8_t)src; m->dst = (uint8_t)dst;
  uint32_t slot = s->free_stack[--s->n_free];
  s->pool[slot] = *m;
  s->inflight++;
  if (s->inflight > s->r.max_inflight) s->r.max_inflight = s->inflight;
  heap_push(s, ((uint64_t)m->time << 32) | seq, slot, 0);
}

/* ------------------------------------------------------------------ */
/* tester storage (tester.rs:366-428)                                   */
/* ------------------------------------------------------------------ */
static void push_and_check(OSim* s, uint32_t i, uint32_t idx, uint64_t v, uint32_t term) {
  if (idx >= s->cfg.apply_cap) t_fail(s, MR_FAIL_SIM_CAPACITY);
  s->r.applies++;
  if (s->mask[idx] && s->sval[idx] != v && !(s->cfg.flags & MR_F_BUG_NO_APPLY_CHECK))
    t_fail(s, MR_FAIL_APPLY_MISMATCH); /* :384 */
  if (idx > s->slen[i]) t_fail(s, MR_FAIL_APPLY_OUT_OF_ORDER);              /* :393 */
  if (idx == s->slen[i]) {
    s->sval[idx] = v;
    s->sterm[idx] = term;
    s->mask[idx] |= (uint8_t)(1u << i);
    s->slen[i]++;
    if (idx > s->r.max_index) s->r.max_index = idx;
  }
}

static void storage_snapshot(OSim* s, uint32_t i, uint32_t idx) { /* :399-402 resize(idx+1) */
  if (idx >= s->cfg.apply_cap) t_fail(s, MR_FAIL_SIM_CAPACITY);
  uint32_t nl = idx + 1;
  for (uint32_t j = nl; j < s->slen[i]; j++) s->mask[j] &= (uint8_t)~(1u << i);
  s->slen[i] = nl;
}

static void n_committed(OSim* s, uint32_t idx, uint32_t* cnt, uint64_t* v) { /* :405-422 */
  if (idx >= s->cfg.apply_cap) { *cnt = 0; *v = 0; return; }
  *cnt = (uint32_t)__builtin_popcount(s->mask[idx]);
  *v = s->sval[idx];
}

/* ------------------------------------------------------------------ */
/* Raft node (SEMANTICS.md §5; API raft.rs:107-168)                     */
/* ------------------------------------------------------------------ */
static inline uint32_t lpos(OSim* s, uint32_t i) { return i & (s->cfg.log_cap - 1); }

static uint32_t term_at(OSim* s, ONode* d, uint32_t i) {
  if (i == 0) return 0;
  if (i == d->snap_idx) return d->snap_term;
  return d->lterm[lpos(s, i)];
}

static void log_put(OSim* s, ONode* d, uint32_t i, uint32_t t, uint64_t v) {
  if (i - d->snap_idx > s->cfg.log_cap) t_fail(s, MR_FAIL_SIM_CAPACITY);
  d->lterm[lpos(s, i)] = t;
  d->lval[lpos(s, i)] = v;
  s->r.log_writes++;
  d->last = i;
  if (i - d->snap_idx > s->r.max_log) s->r.max_log = i - d->snap_idx;
}

/* kvraft Server::apply + Kv::apply (the build's completion of kvraft/server.rs:68-87,
 * SEMANTICS §9): dedup by (clerk, seq), value model (n, ok), answer pending requests */
/* the build's rebalance (SEMANTICS §10): every shard assigned, group loads
 * differ by <= 1, and a shard only moves off a removed or over-target group */
static void ctl_rebalance(OCfg* c) {
  if (c->ng == 0) { for (uint32_t j = 0; j < N_SHARDS; j++) c->shards[j] = 0; return; }
  uint32_t cnt[CFG_G], tgt[CFG_G], pool[N_SHARDS], np = 0, rank[CFG_G];
  for (uint32_t g = 0; g < c->ng; g++) cnt[g] = 0;
  for (uint32_t j = 0; j < N_SHARDS; j++) {
    uint32_t g = 0;
    while (g < c->ng && c->gid[g] != c->shards[j]) g++;
    if (g < c->ng) cnt[g]++;
    else c->shards[j] = 0;
  }
  /* targets: base + 1 for the `extra` groups with the most shards (ties: smaller gid) */
  uint32_t base = N_SHARDS / c->ng, extra = N_SHARDS % c->ng;
  for (uint32_t g = 0; g < c->ng; g++) {
    rank[g] = 0;
    for (uint32_t h = 0; h < c->ng; h++)
      if (cnt[h] > cnt[g] || (cnt[h] == cnt[g] && h < g)) rank[g]++;
    tgt[g] = base + (rank[g] < extra ? 1u : 0u);
  }
  for (uint32_t g = 0; g < c->ng; g++) /* release over-target shards, highest shard first */
    for (int j = N_SHARDS - 1; j >= 0 && cnt[g] > tgt[g]; j--)
      if (c->shards[j] == c->gid[g]) { c->shards[j] = 0; cnt[g]--; }
  for (uint32_t j = 0; j < N_SHARDS; j++)
    if (c->shards[j] == 0) pool[np++] = j;
  for (uint32_t k = 0; k < np; k++) { /* unassigned shards, ascending, to the first group below target */
    uint32_t g = 0;
    while (cnt[g] >= tgt[g]) g++;
    c->shards[pool[k]] = c->gid[g];
    cnt[g]++;
  }
}

/* ShardInfo::apply (the build's completion of shard_ctrler/server.rs:8-19) at server me;
 * returns the output: for a Query the index of the answered config in me's store */
static uint32_t ctl_apply(OSim* s, uint32_t me, uint32_t clerk, uint32_t seq, uint32_t op_id) {
  const OOp* op = &s->ops[op_id];
  OCfg* store = &s->cfgs[me * CFG_CAP];
  uint32_t nc = s->ncfg[me];
  if (op->type == CT_QUERY) return op->a >= nc ? nc - 1 : op->a;
  if (seq <= s->kv_dedup[me][clerk]) return 0; /* duplicate */
  s->kv_dedup[me][clerk] = seq;
  if (nc >= CFG_CAP) t_fail(s, MR_FAIL_SIM_CAPACITY);
  OCfg* c = &store[nc];
  *c = store[nc - 1];
  c->num = nc;
  if (op->type == CT_JOIN) {
    for (uint32_t k = 0; k < op->ng; k++) {
      uint32_t g = 0;
      while (g < c->ng && c->gid[g] < op->gid[k]) g++;
      if (g < c->ng && c->gid[g] == op->gid[k]) { c->addr[g] = op->addr[k]; continue; }
      if (c->ng >= CFG_G) t_fail(s, MR_FAIL_SIM_CAPACITY);
      for (uint32_t h = c->ng; h > g; h--) { c->gid[h] = c->gid[h - 1]; c->addr[h] = c->addr[h - 1]; }
      c->gid[g] = op->gid[k]; c->addr[g] = op->addr[k]; c->ng++;
    }
    ctl_rebalance(c);
  } else if (op->type == CT_LEAVE) {
    for (uint32_t k = 0; k < op->ng; k++) {
      uint32_t g = 0;
      while (g < c->ng && c->gid[g] != op->gid[k]) g++;
      if (g == c->ng) continue;
      for (uint32_t h = g; h + 1 < c->ng; h++) { c->gid[h] = c->gid[h + 1]; c->addr[h] = c->addr[h + 1]; }
      c->ng--;
    }
    ctl_rebalance(c);
  } else {
    if (op->a < N_SHARDS) c->shards[op->a] = op->b;
  }
  s->ncfg[me] = nc + 1;
  return 0;
}

static uint32_t ndig(uint32_t v) { uint32_t d = 1; while (v >= 10) { v /= 10; d++; } return d; }
/* a Put value token: 0 = "", t < 2^20 = the decimal string of t - 1, else one letter */
static uint32_t put_len(uint32_t t) { return t == 0 ? 0 : t < (1u << 20) ? ndig(t - 1) : 1; }

/* the state of appender `cli` of a key: count | ok << 31 (ok: its tokens arrived in order, once) */
static uint32_t kv_app_state(const OKey* k, uint32_t cli, int lin15) {
  if (lin15) return cli < LIN_CLI ? (k->app[cli] & 0xFFFu) | ((~k->app[cli] >> 31) << 31) : 1u << 31;
  for (uint32_t a = 0; a < KV_APP; a++)
    if ((k->app[a] & 0xFFu) == cli + 1) return ((k->app[a] >> 8) & 0x7FFFFFu) | ((~k->app[a] >> 31) << 31);
  return 1u << 31;
}

/* a Get's reply value: the state of appender elem, or (KV_ALL) of appenders 0..4 packed as
 * count (5 bits, saturating at 31) | ok << 5 each */
static uint32_t kv_get_value(const OKey* k, uint32_t elem, int lin15) {
  if (elem != KV_ALL || lin15) return kv_app_state(k, elem, lin15);
  uint32_t out = 0;
  for (uint32_t c = 0; c < KV_APP; c++) {
    uint32_t st = kv_app_state(k, c, 0), n = st & 0xFFFFFFu;
    out |= ((n > 31 ? 31 : n) | ((st >> 31) ? 32u : 0u)) << (6 * c);
  }
  return out;
}

/* Kv::apply (kvraft/server.rs:74-87, the build's completion; SEMANTICS §9) of log entry i
 * (command v) at server me: values are token sequences kept as (hash, length, appenders) */
static void kv_apply(OSim* s, uint32_t me, uint32_t i, uint64_t v) {
  uint32_t op = (uint32_t)(v >> 61) & 3u, key = (uint32_t)(v >> 55) & 63u;
  uint32_t clerk = (uint32_t)(v >> 48) & 127u, seq = (uint32_t)(v >> 24) & 0xFFFFFFu;
  uint32_t elem = (uint32_t)v & 0xFFFFFFu, out = 0;
  uint64_t outh = 0;
  OKey* k = &s->kv[me][key];
  int query = op == KV_GET;
  if (s->ctrl_mode) { /* shard_ctrler: elem = the operation's id */
    out = ctl_apply(s, me, clerk, seq, elem);
    query = s->ops[elem].type == CT_QUERY;
  } else if (op == KV_GET) {
    outh = k->h;
    out = kv_get_value(k, elem, s->lin15);
  } else if (seq > s->kv_dedup[me][clerk] || (s->cfg.flags & MR_F_BUG_NO_DEDUP)) {
    if (s->lin15) { /* SEMANTICS §9b: a Put / Append of token "x {cli} {j} y", elem = cli << 19 | j */
      uint32_t cli = elem >> 19, j = elem & 0x7FFFFu;
      if (cli >= LIN_CLI) t_fail(s, MR_FAIL_SIM_CAPACITY);
      if (op == KV_PUT) {
        memset(k, 0, sizeof *k);
        k->h = elem + 1ull; /* the hash of "" then the token */
        k->len = 5 + ndig(cli) + ndig(j);
        k->app[cli] = 1u | (j << 12);
      } else {
        uint32_t w = k->app[cli], n = w & 0xFFFu;
        if (!(w >> 31) && (n == 0 || j > ((w >> 12) & 0x7FFFFu))) {
          if (n + 1 > 0xFFFu) t_fail(s, MR_FAIL_SIM_CAPACITY);
          w = (n + 1) | (j << 12);
        } else {
          w |= 1u << 31;
        }
        k->app[cli] = w;
        k->h = k->h * KV_HP + elem + 1;
        k->len += 5 + ndig(cli) + ndig(j);
      }
    } else if (op == KV_PUT) { /* elem = the value's token (0 = "") */
      memset(k, 0, sizeof *k);
      if (elem) { k->h = (elem + 1ull) * 0x9E3779B97F4A7C15ull; k->len = put_len(elem); }
    } else { /* Append of token "x {cli} {j} y": elem = cli << 19 | j */
      uint32_t cli = elem >> 19, j = elem & 0x7FFFFu, a = 0;
      while (a < KV_APP && (k->app[a] & 0xFFu) != cli + 1 && (k->app[a] & 0xFFu) != 0) a++;
      if (a == KV_APP) t_fail(s, MR_FAIL_SIM_CAPACITY);
      uint32_t w = k->app[a], n = (w >> 8) & 0xFFFFFFu;
      if (!(w >> 31) && n == j) w = (cli + 1) | ((n + 1) << 8);
      else w = (cli + 1) | (n << 8) | (1u << 31);
      k->app[a] = w;
      k->h = k->h * KV_HP + elem + 1;
      k->len += 5 + ndig(cli) + ndig(j);
    }
    s->kv_dedup[me][clerk] = seq;
  }
  if (!s->ctrl_mode && s->tapp && i < s->trace_cap && !s->tapp[2 * i]) { /* mr_trace_applies */
    s->tapp[2 * i] = v; s->tapp[2 * i + 1] = k->h;
  }
  for (uint32_t p = 0; p < KV_PEND; p++) { /* answered at the end of the event (kv_flush) */
    OPend* q = &s->pend[me][p];
    if (!q->used || q->ready || q->idx != i) continue;
    int ok = q->clerk == clerk && q->seq == seq;
    q->ready = 1; q->status = ok ? KV_OK : KV_FAILED;
    q->value = (ok && query) ? out : 0; q->vh = (ok && query) ? outh : 0;
  }
}

static void kv_send_rep(OSim* s, uint32_t src, uint32_t dst, uint32_t clerk, uint32_t tag,
                        uint32_t status, uint32_t hint, uint32_t value, uint64_t vh) {
  OMsg m;
  m.type = M_KV_REP; m.inc = (uint8_t)clerk; m.term = tag; m.a = status; m.b = hint; m.c = value;
  m.k = 0; m.v = vh;
  net_send(s, src, dst, &m);
}

/* the event's answered requests at server me, after its Raft sends, in slot order (SEMANTICS §9) */
static void kv_flush(OSim* s, uint32_t me) {
  for (uint32_t p = 0; p < KV_PEND; p++) {
    OPend* q = &s->pend[me][p];
    if (!q->used || !q->ready) continue;
    q->used = 0; q->ready = 0;
    kv_send_rep(s, me, q->host, q->clerk, q->tag, q->status, me, q->value, q->vh); /* hint = server */
  }
}

/* the persisted "state" size (SEMANTICS §5 size model) */
static uint32_t raft_state_size(const ONode* d) {
  return 32 + (d->voted >= 0 ? 9 : 1) + 24 * (d->last - d->snap_idx);
}

static void kv_state_get(OSim* s, uint32_t me, OKvState* st) {
  memcpy(st->dedup, s->kv_dedup[me], sizeof st->dedup);
  memcpy(st->keys, s->kv[me], sizeof st->keys);
}
static void kv_state_put(OSim* s, uint32_t me, const OKvState* st) {
  memcpy(s->kv_dedup[me], st->dedup, sizeof st->dedup);
  memcpy(s->kv[me], st->keys, sizeof st->keys);
}

/* the KV service snapshots its state at applied index i (kvraft/server.rs:12-16 with
 * maxraftstate; SEMANTICS §9): Raft's snapshot(i), the persisted KV snapshot, and the
 * cluster's ring of recent snapshots (equal states at equal indices, or APPLY_MISMATCH) */
static void kv_snapshot(OSim* s, uint32_t me, uint32_t i) {
  ONode* d = &s->nd[me];
  d->snap_term = term_at(s, d, i);
  d->snap_val = d->lval[lpos(s, i)];
  d->snap_idx = i;
  s->r.snapshots++;
  kv_state_get(s, me, &s->kvs[me]);
  uint32_t r = (i / KV_SNAP_EVERY) % KV_RING;
  if (s->kring_idx[r] == i) {
    if (memcmp(&s->kring[r], &s->kvs[me], sizeof(OKvState))) t_fail(s, MR_FAIL_APPLY_MISMATCH);
  } else {
    s->kring[r] = s->kvs[me];
    s->kring_idx[r] = i;
  }
}

/* InstallSnapshot(idx) at server me: the KV state of index idx from the ring; requests
 * pending at or below idx are answered FAILED (their entries are never applied here) */
static void kv_install(OSim* s, uint32_t me, uint32_t idx) {
  uint32_t r = (idx / KV_SNAP_EVERY) % KV_RING;
  if (s->kring_idx[r] != idx) t_fail(s, MR_FAIL_SIM_CAPACITY);
  s->kvs[me] = s->kring[r];
  kv_state_put(s, me, &s->kring[r]);
  for (uint32_t p = 0; p < KV_PEND; p++) {
    OPend* q = &s->pend[me][p];
    if (q->used && !q->ready && q->idx <= idx) { q->ready = 1; q->status = KV_FAILED; q->value = 0; q->vh = 0; }
  }
}

/* the persisted KV snapshot's size (snapshot_size(), kvraft/tester.rs:69-76; SEMANTICS §9):
 * 8 + per non-empty key (16 + name + value bytes) + 8 + 16 per clerk with a dedup entry */
static uint32_t kv_snap_size(const OKvState* st) {
  uint32_t sz = 16;
  for (uint32_t k = 0; k < KV_KEYS; k++)
    if (st->keys[k].h || st->keys[k].len) sz += 16 + (k < 50 ? ndig(k) : 1) + st->keys[k].len;
  for (uint32_t c = 0; c < MAX_CLERKS; c++) sz += st->dedup[c] ? 16 : 0;
  return sz;
}

/* tester.rs:303-325 applier: push_and_check, snapshot every SNAPSHOT_INTERVAL */
static void node_apply(OSim* s, uint32_t me) {
  ONode* d = &s->nd[me];
  while (d->applied < d->commit) {
    uint32_t i = ++d->applied;
    uint64_t v = d->lval[lpos(s, i)];
    push_and_check(s, me, i, v, d->lterm[lpos(s, i)]);
    s->adig[me] += mr_apply_mix(i, v);
    if (s->kv_mode) kv_apply(s, me, i, v);
    if (s->kv_maxraft && i % KV_SNAP_EVERY == 0 && i > d->snap_idx &&
        raft_state_size(d) >= s->kv_maxraft / 2) kv_snapshot(s, me, i);
    if (s->snapshot_mode && (i + 1) % 10 == 0 && i > d->snap_idx) {
      d->snap_term = term_at(s, d, i);
      d->snap_val = v;
      d->snap_idx = i;
      s->r.snapshots++;
    }
  }
}

static void send_append(OSim* s, uint32_t me, uint32_t p) {
  ONode* d = &s->nd[me];
  OMsg m;
  m.term = d->term; m.inc = (uint8_t)d->inc;
  if (d->next[p] <= d->snap_idx) {
    m.type = M_IS_REQ; m.a = d->snap_idx; m.b = d->snap_term; m.v = d->snap_val;
    m.c = 0; m.k = 0;
  } else {
    uint32_t prev = d->next[p] - 1;
    uint32_t k = d->last - prev;
    if (k > s->cfg.ae_max) k = s->cfg.ae_max;
    m.type = M_AE_REQ; m.a = prev; m.b = term_at(s, d, prev); m.c = d->commit; m.k = k; m.v = 0;
    for (uint32_t j = 0; j < k; j++) {
      m.et[j] = d->lterm[lpos(s, prev + 1 + j)];
      m.ev[j] = d->lval[lpos(s, prev + 1 + j)];
    }
  }
  net_send(s, me, p, &m);
}

/* MR_F_SAFETY (SEMANTICS §11) when `me` wins its term: election safety, exact (one bit
 * per term that had a leader), and leader completeness for the committed entry at the
 * highest index any server applied (index, term and command; log matching, checked at
 * every AppendEntries, extends it to every earlier committed entry) */
static void safety_on_leader(OSim* s, uint32_t me) {
  ONode* d = &s->nd[me];
  uint32_t t = d->term;
  if (t >= 64u * 32u) t_fail(s, MR_FAIL_SIM_CAPACITY);
  if ((s->led[t >> 5] >> (t & 31u)) & 1u) t_fail(s, MR_FAIL_SAFETY_ELECTION);
  s->led[t >> 5] |= 1u << (t & 31u);
  uint32_t j = (uint32_t)s->r.max_index;
  if (j > d->snap_idx && (j > d->last || d->lval[lpos(s, j)] != s->sval[j] ||
                          d->lterm[lpos(s, j)] != s->sterm[j]))
    t_fail(s, MR_FAIL_SAFETY_COMPLETENESS);
}

static void become_leader(OSim* s, uint32_t me) {
  ONode* d = &s->nd[me];
  if (s->cfg.flags & MR_F_SAFETY) safety_on_leader(s, me);
  d->role = R_L;
  s->r.leaders_elected++;
  for (uint32_t p = 0; p < s->n; p++) { d->next[p] = d->last + 1; d->match[p] = 0; }
  d->match[me] = d->last;
  for (uint32_t p = 0; p < s->n; p++)
    if (p != me) send_append(s, me, p);
  set_timer(s, me, s->now + s->cfg.hb_us);
}

static void advance_commit(OSim* s, uint32_t me) {
  ONode* d = &s->nd[me];
  uint32_t mv[MR_MAX_NODES];
  for (uint32_t p = 0; p < s->n; p++) mv[p] = (p == me) ? d->last : d->match[p];
  /* insertion sort, descending */
  for (uint32_t i = 1; i < s->n; i++) {
    uint32_t x = mv[i], j = i;
    while (j > 0 && mv[j - 1] < x) { mv[j] = mv[j - 1]; j--; }
    mv[j] = x;
  }
  uint32_t N = mv[s->n / 2];
  if (N > d->commit && term_at(s, d, N) == d->term) {
    d->commit = N;
    node_apply(s, me);
  }
}

static void on_ack(OSim* s, uint32_t me, uint32_t p, uint32_t x) {
  ONode* d = &s->nd[me];
  if (x > d->match[p]) d->match[p] = x;
  if (x + 1 > d->next[p]) d->next[p] = x + 1;
  advance_commit(s, me);
  if (d->next[p] <= d->last) send_append(s, me, p);
}

static void reply(OSim* s, uint32_t me, const OMsg* req, uint32_t type, uint32_t a, uint32_t b) {
  OMsg m;
  m.type = (uint8_t)type; m.inc = req->inc; m.term = s->nd[me].term;
  m.a = a; m.b = b; m.c = 0; m.k = 0; m.v = 0;
  net_send(s, me, req->src, &m);
}

static void rec_host(OSim* s, uint32_t kind, uint32_t host, uint32_t aux) {
  mr_event e;
  memset(&e, 0, sizeof e);
  e.time_us = s->now; e.cls = 0; e.kind = (uint8_t)kind; e.node = (uint8_t)host; e.aux = aux;
  rec_push(s, &e);
}

static void thr_wake(OSim* s, uint32_t slot, uint32_t t);

/* KV_REP at a clerk host: wake the clerk's thread if it waits for this tag */
static void clerk_deliver(OSim* s, OMsg* m) {
  uint32_t slot = m->dst - CLERK_HOST;
  OClerk* c = &s->ck[slot];
  if (!host_conn(s, m->src) || !link_up(s, m->src, m->dst)) {
    s->r.drop_deliver++;
    rec_host(s, 16, m->dst, m->seq);
    return;
  }
  if (!(s->th[slot].live || c->mcl) || c->id != m->inc || !c->waiting || c->got || m->term != c->tag) {
    s->r.drop_stale++;
    rec_host(s, 17, m->dst, m->seq);
    return;
  }
  c->got = 1; c->rstat = m->a; c->rhint = m->b; c->rval = m->c; c->rvh = m->v;
  thr_wake(s, c->owner, s->now);
  rec_host(s, M_KV_REP, m->dst, m->seq);
}

/* KV_REQ at server `me` (kvraft/server.rs:48-56 handler + :68-70 apply, SEMANTICS §9) */
static void kv_request(OSim* s, uint32_t me, OMsg* m) {
  ONode* d = &s->nd[me];
  uint32_t clerk = m->inc; /* the request names its clerk; the reply goes to the sending host */
  /* the as-shipped skeleton: the RPC handler's Server::apply is todo!() (kvraft/server.rs:69) */
  if (s->null_raft) t_fail(s, MR_FAIL_TODO_APPLY);
  if (d->role != R_L) {
    kv_send_rep(s, me, m->src, clerk, m->term, KV_WRONG_LEADER, (me + 1) % s->n, 0, 0);
    return;
  }
  if ((s->cfg.flags & MR_F_BUG_STALE_READ) && (m->a & 3u) == KV_GET && !s->ctrl_mode) {
    /* the buggy leader answers from its own state at once: no log entry, no quorum */
    OKey* k = &s->kv[me][(m->a >> 2) & 63u];
    uint32_t elem = m->c & 0xFFFFFFu;
    kv_send_rep(s, me, m->src, clerk, m->term, KV_OK, me, kv_get_value(k, elem, s->lin15), k->h);
    return;
  }
  uint32_t p = 0;
  while (p < KV_PEND && s->pend[me][p].used) p++;
  if (p == KV_PEND) { kv_send_rep(s, me, m->src, clerk, m->term, KV_FAILED, 0, 0, 0); return; }
  /* command: 1 | op << 61 | key << 55 | clerk << 48 | seq24 << 24 | elem24 */
  uint64_t cmd = (1ull << 63) | ((uint64_t)(m->a & 3u) << 61) | ((uint64_t)((m->a >> 2) & 63u) << 55) |
                 ((uint64_t)clerk << 48) | ((uint64_t)(m->b & 0xFFFFFFu) << 24) | (m->c & 0xFFFFFFu);
  log_put(s, d, d->last + 1, d->term, cmd); /* start(), raft.rs:238-244 */
  d->match[me] = d->last;
  OPend* q = &s->pend[me][p];
  q->used = 1; q->idx = d->last; q->clerk = clerk; q->seq = m->b & 0xFFFFFFu; q->tag = m->term;
  q->host = m->src;
}

static void deliver(OSim* s, OMsg* m) {
  uint32_t me = m->dst;
  if (me >= CLERK_HOST) { clerk_deliver(s, m); return; }
  ONode* d = &s->nd[me];
  if (!d->alive || !d->conn || !host_conn(s, m->src) || !link_up(s, m->src, me)) {
    s->r.drop_deliver++;
    rec_node(s, 0, 16, me, m->seq);
    return;
  }
  int is_reply = (m->type == M_RV_REP || m->type == M_AE_REP || m->type == M_IS_REP);
  if (is_reply && m->inc != (uint8_t)d->inc) {
    s->r.drop_stale++;
    rec_node(s, 0, 17, me, m->seq);
    return;
  }
  if (m->type == M_KV_REQ) {
    kv_request(s, me, m);
    rec_node(s, 0, m->type, me, m->seq);
    return;
  }
  if (m->term > d->term) { /* step down */
    d->term = m->term; d->voted = -1; d->votes = 0;
    if (d->role == R_L) reset_timer(s, me);
    d->role = R_F;
  }
  switch (m->type) {
    case M_RV_REQ: {
      uint32_t lt = term_at(s, d, d->last);
      int up = (m->c > lt) || (m->c == lt && m->b >= d->last);
      if (s->cfg.flags & MR_F_BUG_VOTE_STALE) up = 1;
      int free_vote = (d->voted < 0 || d->voted == (int32_t)m->a) || (s->cfg.flags & MR_F_BUG_VOTE_TWICE);
      int granted = (m->term == d->term) && free_vote && up;
      if (granted) { d->voted = (int32_t)m->a; reset_timer(s, me); }
      reply(s, me, m, M_RV_REP, (uint32_t)granted, 0);
    } break;
    case M_RV_REP:
      if (d->role == R_C && m->term == d->term && m->a) {
        d->votes |= 1u << m->src;
        if ((uint32_t)__builtin_popcount(d->votes) > s->n / 2) become_leader(s, me);
      }
      break;
    case M_AE_REQ: {
      if (m->term < d->term) { reply(s, me, m, M_AE_REP, 0, 0); break; }
      if (d->role == R_C) d->role = R_F;
      reset_timer(s, me);
      uint32_t prev = m->a, pterm = m->b, j0 = 0;
      if (prev < d->snap_idx) {
        uint32_t skip = d->snap_idx - prev;
        j0 = skip < m->k ? skip : m->k;
        prev = d->snap_idx; pterm = d->snap_term;
      }
      if (prev > d->last) { reply(s, me, m, M_AE_REP, 0, d->last + 1); break; }
      if (!(s->cfg.flags & MR_F_BUG_NO_PREV_CHECK) && term_at(s, d, prev) != pterm) {
        uint32_t ct = term_at(s, d, prev), x = prev;
        while (x - 1 > d->snap_idx && term_at(s, d, x - 1) == ct) x--;
        reply(s, me, m, M_AE_REP, 0, x);
        break;
      }
      s->r.entries_shipped += m->k - j0; /* the payload entries this receiver reads */
      for (uint32_t j = j0; j < m->k; j++) {
        uint32_t i = m->a + 1 + j;
        if (i <= d->last && term_at(s, d, i) == m->et[j]) {
          /* MR_F_SAFETY log matching: an entry with the same index and term is the same entry */
          if ((s->cfg.flags & MR_F_SAFETY) && d->lval[lpos(s, i)] != m->ev[j])
            t_fail(s, MR_FAIL_SAFETY_LOG_MATCHING);
          continue;
        }
        log_put(s, d, i, m->et[j], m->ev[j]); /* truncates to i-1, appends */
      }
      uint32_t lc = m->a + m->k;
      if (m->c < lc) lc = m->c;
      if (lc > d->commit) { d->commit = lc; node_apply(s, me); }
      reply(s, me, m, M_AE_REP, 1, m->a + m->k);
    } break;
    case M_AE_REP:
      if (d->role != R_L || m->term != d->term) break;
      if (m->a) {
        on_ack(s, me, m->src, m->b);
      } else {
        uint32_t x = m->b, lo = d->match[m->src] + 1, hi = d->last + 1;
        if (x < lo) x = lo;
        if (x > hi) x = hi;
        d->next[m->src] = x;
        send_append(s, me, m->src);
      }
      break;
    case M_IS_REQ: {
      if (m->term < d->term) { reply(s, me, m, M_IS_REP, 0, 0); break; }
      if (d->role == R_C) d->role = R_F;
      reset_timer(s, me);
      uint32_t idx = m->a;
      if (idx > d->commit) {
        if (!(idx <= d->last && term_at(s, d, idx) == m->b)) d->last = idx;
        d->snap_idx = idx; d->snap_term = m->b; d->snap_val = m->v;
        d->commit = idx; d->applied = idx;
        s->ainv[me] = 1;
        storage_snapshot(s, me, idx);
        if (s->kv_maxraft) kv_install(s, me, idx);
        s->r.installs++;
      }
      reply(s, me, m, M_IS_REP, 0, idx);
    } break;
    case M_IS_REP:
      if (d->role == R_L && m->term == d->term && m->b > 0) on_ack(s, me, m->src, m->b);
      break;
  }
  if (s->kv_mode) kv_flush(s, me);
  rec_node(s, 0, m->type, me, m->seq);
}

static void on_timer(OSim* s, uint32_t me) {
  ONode* d = &s->nd[me];
  if (d->role == R_L) {
    for (uint32_t p = 0; p < s->n; p++)
      if (p != me) send_append(s, me, p);
    set_timer(s, me, s->now + s->cfg.hb_us);
    rec_node(s, 1, 1, me, 0);
    return;
  }
  d->term++; d->voted = (int32_t)me; d->role = R_C; d->votes = 1u << me;
  s->r.elections++;
  reset_timer(s, me);
  OMsg m;
  m.type = M_RV_REQ; m.inc = (uint8_t)d->inc; m.term = d->term;
  m.a = me; m.b = d->last; m.c = term_at(s, d, d->last); m.k = 0; m.v = 0;
  for (uint32_t p = 0; p < s->n; p++)
    if (p != me) net_send(s, me, p, &m);
  rec_node(s, 1, 0, me, 0);
}

static void client_step(OSim* s, uint32_t slot);
static void kv_task_step(OSim* s, uint32_t slot);

/* a thread becomes runnable at (t, 2, tid) (SEMANTICS §8); slot 0 is the test body */
static void thr_wake(OSim* s, uint32_t slot, uint32_t t) {
  if (slot == 0) { s->mwake = t; return; }
  OThr* th = &s->th[slot];
  th->gen++;
  heap_push(s, ((uint64_t)t << 32) | (2ull << 30) | th->tid, slot, th->gen);
}

/* drain the executor until the test body's wake-up key (mwake, 2, 0): every
 * message / timer / other thread ordered before it (SEMANTICS §3, §8) */
static void main_wait(OSim* s) {
  for (;;) {
    uint64_t mk = s->mwake == INF_T ? ~0ull : (((uint64_t)s->mwake << 32) | (2ull << 30));
    if (!s->heap_n || s->heap[0].key >= mk) break;
    HEnt e = heap_pop(s);
    uint32_t cls = (uint32_t)(e.key >> 30) & 3u;
    if (cls == 1) {
      ONode* d = &s->nd[e.ref];
      if (!d->alive || e.gen != d->timer_gen) continue; /* cancelled timer */
      s->now = (uint32_t)(e.key >> 32);
      count_event(s);
      s->r.ev_timer++;
      on_timer(s, e.ref);
    } else if (cls == 2) {
      OThr* th = &s->th[e.ref];
      if (!th->live || e.gen != th->gen) continue; /* superseded wake-up */
      s->now = (uint32_t)(e.key >> 32);
      count_event(s);
      s->r.ev_tester++;
      client_step(s, e.ref);
    } else {
      OMsg m = s->pool[e.ref];
      s->free_stack[s->n_free++] = e.ref;
      s->inflight--;
      s->now = m.time;
      count_event(s);
      s->r.ev_msg++;
      deliver(s, &m);
    }
  }
  if (s->mwake == INF_T) t_fail(s, MR_FAIL_SIM_BAD_PROGRAM); /* deadlock: nothing wakes main */
  s->now = s->mwake;
}

/* ------------------------------------------------------------------ */
/* tester API (src/raft/tester.rs)                                      */
/* ------------------------------------------------------------------ */
/* the test body blocks (its segment ends) until mwake; then one tester event */
static void main_block(OSim* s) {
  rec_simple(s, 2, 0); /* the tester segment that ends here */
  main_wait(s);
  count_event(s);
  s->r.ev_tester++;
}

static void t_sleep(OSim* s, uint32_t us) { /* time::sleep */
  uint64_t target = (uint64_t)s->now + us;
  if (target >= INF_T) { rec_simple(s, 2, 0); t_fail(s, MR_FAIL_SIM_CAPACITY); }
  s->mwake = (uint32_t)target;
  main_block(s);
}

static void t_draw(OSim* s, uint32_t w[4]) {
  uint32_t ctr[4] = {s->t_ctr++, 0, ST_TESTER, 0};
  draw(s, ctr, w);
}
static uint32_t t_range(OSim* s, uint32_t lo, uint32_t hi) {
  uint32_t w[4]; t_draw(s, w); return u_range(w[0], lo, hi);
}
static int t_bool(OSim* s, uint32_t p_q32) { uint32_t w[4]; t_draw(s, w); return w[0] < p_q32; }
static uint64_t t_entry(OSim* s) { /* tests.rs:943-951 gen_entry */
  uint32_t w[4]; t_draw(s, w); return ((uint64_t)w[1] << 32) | w[0];
}

static void t_set_unreliable(OSim* s, int u) { /* tester.rs:127-137 */
  if (u) { s->loss = LOSS_Q32; s->lat_lo = 1000; s->lat_hi = 27000; }
  else { s->loss = 0; s->lat_lo = 1000; s->lat_hi = 10000; }
}

static ONode* t_raft(OSim* s, uint32_t i) { /* rafts[i].as_ref().unwrap() */
  if (!s->nd[i].alive) t_fail(s, MR_FAIL_UNWRAP_NONE);
  return &s->nd[i];
}
static int t_is_started(OSim* s, uint32_t i) { return s->nd[i].alive; }
static int t_is_connected(OSim* s, uint32_t i) { return s->nd[i].conn; }
static uint32_t t_term(OSim* s, uint32_t i) { return t_raft(s, i)->term; }
static uint32_t t_rpc_total(OSim* s) { return (uint32_t)(s->r.msgs_sent / 2); }

/* tester.rs:165-171 -> raft.rs:238-244 */
static int t_start(OSim* s, uint32_t i, uint64_t v, uint32_t* idx, uint32_t* term) {
  ONode* d = t_raft(s, i);
  if (s->null_raft || d->role != R_L) return 0; /* Err(NotLeader((me+1)%n)) */
  log_put(s, d, d->last + 1, d->term, v);
  d->match[i] = d->last;
  *idx = d->last; *term = d->term;
  return 1;
}

static void t_connect(OSim* s, uint32_t i) { s->nd[i].conn = 1; }
static void t_disconnect(OSim* s, uint32_t i) { s->nd[i].conn = 0; }

static void t_crash1(OSim* s, uint32_t i) { /* tester.rs:329-333 */
  ONode* d = &s->nd[i];
  memset(s->pend[i], 0, sizeof s->pend[i]); /* its RPC handler tasks die with it */
  d->alive = 0;
  d->timer_gen++;
}

static void t_start1(OSim* s, uint32_t i) { /* tester.rs:293-327 + raft.rs:108-122 restore */
  t_crash1(s, i);
  ONode* d = &s->nd[i];
  d->alive = 1; d->inc++; d->role = R_F; d->votes = 0;
  d->commit = d->snap_idx; d->applied = d->snap_idx;
  s->adig[i] = 0; s->ainv[i] = d->snap_idx != 0;
  if (!s->null_raft) reset_timer(s, i);
}

static uint32_t t_log_size(OSim* s) { /* tester.rs:152-158 + SEMANTICS §5 size model */
  uint32_t mx = 0;
  for (uint32_t i = 0; i < s->n; i++) {
    ONode* d = &s->nd[i];
    uint32_t sz = 32 + (d->voted >= 0 ? 9 : 1) + 24 * (d->last - d->snap_idx);
    if (sz > mx) mx = sz;
  }
  return mx;
}

/* tester.rs:64-92 */
static uint32_t t_check_one_leader(OSim* s) {
  for (int it = 0; it < 10; it++) {
    t_sleep(s, t_range(s, 450000, 550000));
    uint32_t lt[MR_MAX_NODES], ln[MR_MAX_NODES], nl = 0;
    for (uint32_t i = 0; i < s->n; i++) {
      if (!s->nd[i].conn) continue;
      ONode* d = t_raft(s, i);
      if (!s->null_raft && d->role == R_L) { lt[nl] = d->term; ln[nl] = i; nl++; }
    }
    for (uint32_t a = 0; a < nl; a++)
      for (uint32_t b = a + 1; b < nl; b++)
        if (lt[a] == lt[b]) t_fail(s, MR_FAIL_MULTI_LEADER_TERM);
    if (nl) {
      uint32_t best = 0;
      for (uint32_t a = 1; a < nl; a++)
        if (lt[a] > lt[best]) best = a;
      return ln[best];
    }
  }
  t_fail(s, MR_FAIL_ONE_LEADER_NONE);
  return 0;
}

/* tester.rs:95-109 */
static uint32_t t_check_terms(OSim* s) {
  uint32_t term = 0;
  for (uint32_t i = 0; i < s->n; i++) {
    if (!s->nd[i].conn) continue;
    uint32_t x = t_term(s, i);
    if (term == 0) term = x;
    else if (term != x) t_fail(s, MR_FAIL_TERM_DISAGREE);
  }
  return term;
}

/* tester.rs:112-122 */
static void t_check_no_leader(OSim* s) {
  for (uint32_t i = 0; i < s->n; i++) {
    if (!s->nd[i].conn) continue;
    ONode* d = t_raft(s, i);
    if (!s->null_raft && d->role == R_L) t_fail(s, MR_FAIL_UNEXPECTED_LEADER);
  }
}

/* tester.rs:175-201; returns 1 and *v on Some */
static int t_wait(OSim* s, uint32_t index, uint32_t n, int has_st, uint32_t start_term, uint64_t* v) {
  uint32_t to = 10000, cnt;
  uint64_t val;
  for (int it = 0; it < 30; it++) {
    n_committed(s, index, &cnt, &val);
    if (cnt >= n) break;
    t_sleep(s, to);
    if (to < 1000000) to *= 2;
    if (has_st)
      for (uint32_t i = 0; i < s->n; i++)
        if (s->nd[i].alive && s->nd[i].term > start_term) return 0;
  }
  n_committed(s, index, &cnt, &val);
  if (cnt < n) t_fail(s, MR_FAIL_WAIT_TOO_FEW);
  *v = val;
  return cnt > 0;
}

/* tester.rs:216-262 */
static uint32_t t_one(OSim* s, uint64_t cmd, uint32_t expected, int retry) {
  uint32_t t0 = s->now, starts = 0;
  while (s->now - t0 < 10000000u) {
    int have = 0;
    uint32_t index = 0, term;
    for (uint32_t k = 0; k < s->n; k++) {
      starts = (starts + 1) % s->n;
      if (!t_is_connected(s, starts) || !t_is_started(s, starts)) continue;
      if (t_start(s, starts, cmd, &index, &term)) { have = 1; break; }
    }
    if (have) {
      uint32_t t1 = s->now;
      while (s->now - t1 < 2000000u) {
        uint32_t cnt; uint64_t v;
        n_committed(s, index, &cnt, &v);
        if (cnt > 0 && cnt >= expected && v == cmd) return index;
        t_sleep(s, 20000);
      }
      if (!retry) t_fail(s, MR_FAIL_ONE_NO_AGREEMENT);
    } else {
      t_sleep(s, 50000);
    }
  }
  t_fail(s, MR_FAIL_ONE_NO_AGREEMENT);
  return 0;
}

static void t_end(OSim* s) { /* tester.rs:339-358 */
  if (s->now > 120000000u) t_fail(s, MR_FAIL_TIMEOUT_120S);
  s->r.code = MR_PASS; s->r.time_us = s->now;
  rec_simple(s, 3, MR_PASS);
}

/* RaftTester::new / new_with_snapshot (tester.rs:34-60) */
static void t_new(OSim* s, int snapshot) {
  s->snapshot_mode = (uint32_t)snapshot;
  for (uint32_t i = 0; i < s->n; i++) { t_start1(s, i); t_connect(s, i); }
  if (s->cfg.flags & MR_F_UNRELIABLE) t_set_unreliable(s, 1);
}

/* ------------------------------------------------------------------ */
/* scenarios (src/raft/tests.rs), straight-line                          */
/* ------------------------------------------------------------------ */
#define ELECTION_US 1000000u /* RAFT_ELECTION_TIMEOUT tests.rs:18 */
static uint32_t iters_or(OSim* s, uint32_t d) { return s->cfg.iters ? s->cfg.iters : d; }

static void scn_initial_election(OSim* s) { /* tests.rs:20-46 */
  t_new(s, 0);
  t_check_one_leader(s);
  t_sleep(s, 50000);
  uint32_t term1 = t_check_terms(s);
  t_sleep(s, 2 * ELECTION_US);
  uint32_t term2 = t_check_terms(s);
  (void)term1; (void)term2; /* warn! only */
  t_check_one_leader(s);
  t_end(s);
}

static void scn_reelection(OSim* s) { /* tests.rs:48-78 */
  uint32_t n = s->n;
  t_new(s, 0);
  uint32_t l1 = t_check_one_leader(s);
  t_disconnect(s, l1);
  t_check_one_leader(s);
  t_connect(s, l1);
  uint32_t l2 = t_check_one_leader(s);
  t_disconnect(s, l2);
  t_disconnect(s, (l2 + 1) % n);
  t_sleep(s, 2 * ELECTION_US);
  t_check_no_leader(s);
  t_connect(s, (l2 + 1) % n);
  t_check_one_leader(s);
  t_connect(s, l2);
  t_check_one_leader(s);
  t_end(s);
}

static void scn_many_election(OSim* s) { /* tests.rs:80-112 */
  uint32_t n = s->n, iters = iters_or(s, 10);
  t_new(s, 0);
  t_check_one_leader(s);
  for (uint32_t it = 0; it < iters; it++) {
    uint32_t i1 = t_range(s, 0, n), i2 = t_range(s, 0, n), i3 = t_range(s, 0, n);
    t_disconnect(s, i1); t_disconnect(s, i2); t_disconnect(s, i3);
    t_check_one_leader(s);
    t_connect(s, i1); t_connect(s, i2); t_connect(s, i3);
  }
  t_check_one_leader(s);
  t_end(s);
}

static void scn_basic_agree(OSim* s) { /* tests.rs:114-130 */
  t_new(s, 0);
  for (uint32_t index = 1; index <= 3; index++) {
    uint32_t nd; uint64_t v;
    n_committed(s, index, &nd, &v);
    if (nd != 0) t_fail(s, MR_FAIL_BASIC_PRECOMMIT);
    uint32_t x = t_one(s, (uint64_t)index * 100, s->n, 0);
    if (x != index) t_fail(s, MR_FAIL_BASIC_INDEX);
  }
  t_end(s);
}

static void scn_fail_agree(OSim* s) { /* tests.rs:132-161 */
  uint32_t n = s->n;
  t_new(s, 0);
  t_one(s, 101, n, 0);
  uint32_t leader = t_check_one_leader(s);
  t_disconnect(s, (leader + 1) % n);
  t_one(s, 102, n - 1, 0);
  t_one(s, 103, n - 1, 0);
  t_sleep(s, ELECTION_US);
  t_one(s, 104, n - 1, 0);
  t_one(s, 105, n - 1, 0);
  t_connect(s, (leader + 1) % n);
  t_one(s, 106, n, 1);
  t_sleep(s, ELECTION_US);
  t_one(s, 107, n, 1);
  t_end(s);
}

static void scn_fail_no_agree(OSim* s) { /* tests.rs:163-209 */
  uint32_t n = s->n, idx, term;
  t_new(s, 0);
  t_one(s, 10, n, 0);
  uint32_t leader = t_check_one_leader(s);
  t_disconnect(s, (leader + 1) % n);
  t_disconnect(s, (leader + 2) % n);
  t_disconnect(s, (leader + 3) % n);
  if (!t_start(s, leader, 20, &idx, &term)) t_fail(s, MR_FAIL_LEADER_REJECTED);
  if (idx != 2) t_fail(s, MR_FAIL_EXPECTED_INDEX2);
  t_sleep(s, 2 * ELECTION_US);
  uint32_t nc; uint64_t v;
  n_committed(s, idx, &nc, &v);
  if (nc != 0) t_fail(s, MR_FAIL_NO_MAJORITY_COMMIT);
  t_connect(s, (leader + 1) % n);
  t_connect(s, (leader + 2) % n);
  t_connect(s, (leader + 3) % n);
  uint32_t leader2 = t_check_one_leader(s);
  uint32_t idx2;
  if (!t_start(s, leader2, 30, &idx2, &term)) t_fail(s, MR_FAIL_LEADER_REJECTED);
  if (idx2 < 2 || idx2 > 3) t_fail(s, MR_FAIL_UNEXPECTED_INDEX);
  t_one(s, 1000, n, 1);
  t_end(s);
}

static void scn_concurrent_starts(OSim* s) { /* tests.rs:211-275 */
  uint32_t n = s->n;
  t_new(s, 0);
  int success = 0;
  for (int tried = 0; tried < 5; tried++) {
    if (tried > 0) t_sleep(s, 3000000);
    uint32_t leader = t_check_one_leader(s), idx, term, st;
    if (!t_start(s, leader, 1, &idx, &term)) continue;
    uint32_t idxes[5], ni = 0;
    for (uint32_t ii = 0; ii < 5; ii++) {
      uint32_t i2;
      if (t_start(s, leader, 100 + ii, &i2, &st) && st == term) idxes[ni++] = i2;
    }
    int changed = 0;
    for (uint32_t j = 0; j < n; j++)
      if (t_term(s, j) != term) { changed = 1; break; }
    if (changed) continue;
    uint64_t cmds[5]; uint32_t nc = 0;
    for (uint32_t q = 0; q < ni; q++) {
      uint64_t v;
      if (t_wait(s, idxes[q], n, 1, term, &v)) cmds[nc++] = v;
    }
    for (uint32_t ii = 0; ii < 5; ii++) {
      int ok = 0;
      for (uint32_t q = 0; q < nc; q++) if (cmds[q] == 100 + ii) ok = 1;
      if (!ok) t_fail(s, MR_FAIL_CMD_MISSING);
    }
    success = 1;
    break;
  }
  if (!success) t_fail(s, MR_FAIL_TERM_CHANGED);
  t_end(s);
}

static void scn_rejoin(OSim* s) { /* tests.rs:277-313 */
  uint32_t n = s->n, idx, term;
  t_new(s, 0);
  t_one(s, 101, n, 1);
  uint32_t l1 = t_check_one_leader(s);
  t_disconnect(s, l1);
  t_start(s, l1, 102, &idx, &term);
  t_start(s, l1, 103, &idx, &term);
  t_start(s, l1, 104, &idx, &term);
  t_one(s, 103, 2, 1);
  uint32_t l2 = t_check_one_leader(s);
  t_disconnect(s, l2);
  t_connect(s, l1);
  t_one(s, 104, 2, 1);
  t_connect(s, l2);
  t_one(s, 105, n, 1);
  t_end(s);
}

static void scn_backup(OSim* s) { /* tests.rs:315-386 */
  uint32_t n = s->n, idx, term;
  t_new(s, 0);
  t_one(s, t_entry(s), n, 1);
  uint32_t l1 = t_check_one_leader(s);
  t_disconnect(s, (l1 + 2) % n); t_disconnect(s, (l1 + 3) % n); t_disconnect(s, (l1 + 4) % n);
  for (int i = 0; i < 50; i++) { uint64_t e = t_entry(s); t_start(s, l1, e, &idx, &term); }
  t_sleep(s, ELECTION_US / 2);
  t_disconnect(s, (l1 + 0) % n); t_disconnect(s, (l1 + 1) % n);
  t_connect(s, (l1 + 2) % n); t_connect(s, (l1 + 3) % n); t_connect(s, (l1 + 4) % n);
  for (int i = 0; i < 50; i++) t_one(s, t_entry(s), 3, 1);
  uint32_t l2 = t_check_one_leader(s);
  uint32_t other = (l1 + 2) % n;
  if (l2 == other) other = (l2 + 1) % n;
  t_disconnect(s, other);
  for (int i = 0; i < 50; i++) { uint64_t e = t_entry(s); t_start(s, l2, e, &idx, &term); }
  t_sleep(s, ELECTION_US / 2);
  for (uint32_t i = 0; i < n; i++) t_disconnect(s, i);
  t_connect(s, (l1 + 0) % n); t_connect(s, (l1 + 1) % n); t_connect(s, other);
  for (int i = 0; i < 50; i++) t_one(s, t_entry(s), 3, 1);
  for (uint32_t i = 0; i < n; i++) t_connect(s, i);
  t_one(s, t_entry(s), n, 1);
  t_end(s);
}

static void scn_count(OSim* s) { /* tests.rs:388-479 */
  uint32_t n = s->n;
  t_new(s, 0);
  t_check_one_leader(s);
  uint32_t total1 = t_rpc_total(s);
  if (total1 < 1 || total1 > 30) t_fail(s, MR_FAIL_RPC_INITIAL);
  uint32_t total2 = 0;
  int success = 0;
  for (int tried = 0; tried < 5 && !success; tried++) {
    if (tried > 0) t_sleep(s, 3000000);
    uint32_t leader = t_check_one_leader(s);
    total1 = t_rpc_total(s);
    const uint32_t iters = 10;
    uint32_t starti, term, idx, st;
    if (!t_start(s, leader, 1, &starti, &term)) continue;
    uint64_t cmds[12];
    int outer = 0;
    for (uint32_t i = 1; i < iters + 2; i++) {
      uint64_t x = t_entry(s); /* random.gen::<u64>() */
      cmds[i - 1] = x;
      if (t_start(s, leader, x, &idx, &st)) {
        if (st != term) { outer = 1; break; }
        if (starti + i != idx) t_fail(s, MR_FAIL_START_FAILED);
      } else { outer = 1; break; }
    }
    if (outer) continue;
    for (uint32_t i = 1; i <= iters; i++) {
      uint64_t v;
      if (t_wait(s, starti + i, n, 1, term, &v) && v != cmds[i - 1]) t_fail(s, MR_FAIL_WRONG_VALUE);
    }
    int changed = 0;
    for (uint32_t i = 0; i < n; i++)
      if (t_term(s, i) != term) { changed = 1; break; }
    if (changed) continue;
    total2 = t_rpc_total(s);
    if (total2 - total1 > (iters + 1 + 3) * 3) t_fail(s, MR_FAIL_RPC_TOO_MANY);
    success = 1;
  }
  if (!success) t_fail(s, MR_FAIL_TERM_CHANGED);
  t_sleep(s, ELECTION_US);
  uint32_t total3 = t_rpc_total(s);
  if (total3 - total2 > 3 * 20) t_fail(s, MR_FAIL_RPC_IDLE);
  t_end(s);
}

static void scn_persist1(OSim* s) { /* tests.rs:481-526 */
  uint32_t n = s->n;
  uint64_t v;
  t_new(s, 0);
  t_one(s, 11, n, 1);
  for (uint32_t i = 0; i < n; i++) t_start1(s, i);
  for (uint32_t i = 0; i < n; i++) { t_disconnect(s, i); t_connect(s, i); }
  t_one(s, 12, n, 1);
  uint32_t l1 = t_check_one_leader(s);
  t_disconnect(s, l1); t_start1(s, l1); t_connect(s, l1);
  t_one(s, 13, n, 1);
  uint32_t l2 = t_check_one_leader(s);
  t_disconnect(s, l2);
  t_one(s, 14, n - 1, 1);
  t_start1(s, l2); t_connect(s, l2);
  t_wait(s, 4, n, 0, 0, &v);
  uint32_t i3 = (t_check_one_leader(s) + 1) % n;
  t_disconnect(s, i3);
  t_one(s, 15, n - 1, 1);
  t_start1(s, i3); t_connect(s, i3);
  t_one(s, 16, n, 1);
  t_end(s);
}

static void scn_persist2(OSim* s) { /* tests.rs:528-572 */
  uint32_t n = s->n;
  uint64_t index = 1;
  t_new(s, 0);
  for (int k = 0; k < 5; k++) {
    t_one(s, 10 + index, n, 1); index++;
    uint32_t l1 = t_check_one_leader(s);
    t_disconnect(s, (l1 + 1) % n); t_disconnect(s, (l1 + 2) % n);
    t_one(s, 10 + index, n - 2, 1); index++;
    t_disconnect(s, (l1 + 0) % n); t_disconnect(s, (l1 + 3) % n); t_disconnect(s, (l1 + 4) % n);
    t_start1(s, (l1 + 1) % n); t_start1(s, (l1 + 2) % n);
    t_connect(s, (l1 + 1) % n); t_connect(s, (l1 + 2) % n);
    t_sleep(s, ELECTION_US);
    t_start1(s, (l1 + 3) % n); t_connect(s, (l1 + 3) % n);
    t_one(s, 10 + index, n - 2, 1); index++;
    t_connect(s, (l1 + 4) % n); t_connect(s, (l1 + 0) % n);
  }
  t_one(s, 1000, n, 1);
  t_end(s);
}

static void scn_persist3(OSim* s) { /* tests.rs:574-602 */
  uint32_t n = s->n;
  t_new(s, 0);
  t_one(s, 101, 3, 1);
  uint32_t leader = t_check_one_leader(s);
  t_disconnect(s, (leader + 2) % n);
  t_one(s, 102, 2, 1);
  t_crash1(s, (leader + 0) % n); t_crash1(s, (leader + 1) % n);
  t_connect(s, (leader + 2) % n);
  t_start1(s, (leader + 0) % n); t_connect(s, (leader + 0) % n);
  t_one(s, 103, 2, 1);
  t_start1(s, (leader + 1) % n); t_connect(s, (leader + 1) % n);
  t_one(s, 104, n, 1);
  t_end(s);
}

static uint32_t fig8_delay(OSim* s) { /* tests.rs:631-635 / 711-715 */
  if (t_bool(s, LOSS_Q32)) return t_range(s, 0, ELECTION_US / 2);
  return t_range(s, 0, 13000);
}

static void scn_figure_8(OSim* s) { /* tests.rs:612-660 (+ unreliable variant, config 3) */
  uint32_t n = s->n, iters = iters_or(s, 1000), idx, term;
  t_new(s, 0);
  if (s->scenario == MR_SCN_FIGURE_8_UNRELIABLE_CRASH) t_set_unreliable(s, 1);
  t_one(s, t_entry(s), 1, 1);
  uint32_t nup = n;
  for (uint32_t it = 0; it < iters; it++) {
    int leader = -1;
    for (uint32_t i = 0; i < n; i++)
      if (t_is_started(s, i)) {
        uint64_t e = t_entry(s);
        if (t_start(s, i, e, &idx, &term)) leader = (int)i;
      }
    t_sleep(s, fig8_delay(s));
    if (leader >= 0) { t_crash1(s, (uint32_t)leader); nup--; }
    if (nup < 3) {
      uint32_t x = t_range(s, 0, n);
      if (!t_is_started(s, x)) { t_start1(s, x); nup++; }
    }
  }
  for (uint32_t i = 0; i < n; i++)
    if (!t_is_started(s, i)) t_start1(s, i);
  t_one(s, t_entry(s), n, 1);
  t_end(s);
}

static void scn_figure_8_unreliable(OSim* s) { /* tests.rs:688-741 */
  uint32_t n = s->n, iters = iters_or(s, 1000), idx, term;
  t_new(s, 0);
  t_set_unreliable(s, 1);
  t_one(s, t_entry(s), 1, 1);
  uint32_t nup = n;
  for (uint32_t it = 0; it < iters; it++) {
    int leader = -1;
    for (uint32_t i = 0; i < n; i++) {
      uint64_t e = t_entry(s);
      if (t_start(s, i, e, &idx, &term) && t_is_connected(s, i)) leader = (int)i;
    }
    t_sleep(s, fig8_delay(s));
    if (leader >= 0 && t_range(s, 0, 1000) < 500) { t_disconnect(s, (uint32_t)leader); nup--; }
    if (nup < 3) {
      uint32_t x = t_range(s, 0, n);
      if (!t_is_connected(s, x)) { t_connect(s, x); nup++; }
    }
  }
  for (uint32_t i = 0; i < n; i++) t_connect(s, i);
  t_one(s, t_entry(s), n, 1);
  t_end(s);
}

static void scn_snap_common(OSim* s, int disconnect, int reliable, int crash) { /* tests.rs:858-911 */
  const uint32_t MAX_LOG_SIZE = 2000;
  uint32_t n = s->n, iters = iters_or(s, 30), idx, term;
  t_new(s, 1);
  t_set_unreliable(s, !reliable);
  t_one(s, t_entry(s), n, 1);
  uint32_t leader1 = t_check_one_leader(s);
  for (uint32_t i = 0; i < iters; i++) {
    uint32_t victim = (leader1 + 1) % n, sender = leader1;
    if (i % 3 == 1) { sender = (leader1 + 1) % n; victim = leader1; }
    if (disconnect) { t_disconnect(s, victim); t_one(s, t_entry(s), n - 1, 1); }
    if (crash) { t_crash1(s, victim); t_one(s, t_entry(s), n - 1, 1); }
    for (int k = 0; k <= 10; k++) { uint64_t e = t_entry(s); t_start(s, sender, e, &idx, &term); }
    t_one(s, t_entry(s), n - 1, 1);
    if (t_log_size(s) >= MAX_LOG_SIZE) t_fail(s, MR_FAIL_LOG_SIZE);
    if (disconnect) {
      t_connect(s, victim);
      t_one(s, t_entry(s), n, 1);
      leader1 = t_check_one_leader(s);
    }
    if (crash) {
      t_start1(s, victim);
      t_connect(s, victim);
      t_one(s, t_entry(s), n, 1);
      leader1 = t_check_one_leader(s);
    }
  }
  t_end(s);
}

/* ------------------------------------------------------------------ */
/* kvraft: clerks, client threads, generic_test (SEMANTICS §8-9)        */
/* ------------------------------------------------------------------ */
static void clerk_send(OSim* s, uint32_t slot) { /* one call_timeout attempt, client.rs:52-57 */
  OClerk* c = &s->ck[slot];
  c->tag++;
  OMsg m;
  m.type = M_KV_REQ; m.inc = (uint8_t)c->id; m.term = c->tag; m.a = c->op | (c->key << 2);
  m.b = c->seq; m.c = c->elem; m.k = 0; m.v = 0;
  net_send(s, CLERK_HOST + slot, c->lh, &m);
  c->waiting = 1; c->got = 0;
  thr_wake(s, c->owner, s->now + 500000u); /* Duration::from_millis(500) */
}

/* ---- the linearizability checker (SEMANTICS §9a): each key is an append / get register;
 * per (key, appender) the tester counts the appends called and acknowledged and the largest
 * count a returned Get observed, and bounds every Get's observed count by the call / return
 * order: at least the appends acknowledged (and the count seen by Gets that returned) before
 * it was called, at most the appends called before it returned, and the appender's tokens in
 * order, once each. */
static uint32_t* lin_ent(OSim* s, uint32_t key, uint32_t cli) {
  key &= KV_KEYS - 1; /* the key as the command carries it (6 bits, kv_request) */
  for (uint32_t a = 0; a < KV_APP; a++) {
    uint32_t* e = s->lin[key][a];
    if (e[0] == cli + 1) return e;
    if (e[0] == 0) { e[0] = cli + 1; e[1] = e[2] = e[3] = e[4] = 0; return e; }
  }
  t_fail(s, MR_FAIL_SIM_CAPACITY);
  return NULL;
}
/* SEMANTICS §9b: the Put-epoch checker of generic_test_linearizability (keys 0..14) */
static void lin15_call(OSim* s, OClerk* c) {
  uint32_t k = c->key & 15u;
  if (c->op == KV_PUT) {
    s->l15_epoch[k]++;
    s->l15_pend[k]++;
    s->l15_called[k][(c->elem >> 19) % LIN_CLI]++;
    memset(s->l15_acked[k], 0, sizeof s->l15_acked[k]);
  } else if (c->op == KV_APPEND) {
    s->l15_called[k][(c->elem >> 19) % LIN_CLI]++;
    c->lepoch = s->l15_epoch[k];
    c->lnopend = s->l15_pend[k] == 0;
  } else {
    c->llo = s->l15_acked[k][c->elem % LIN_CLI];
    c->lepoch = s->l15_epoch[k];
  }
}
static void lin15_return(OSim* s, OClerk* c) {
  uint32_t k = c->key & 15u;
  if (c->op == KV_PUT) { s->l15_pend[k]--; return; }
  if (c->op == KV_APPEND) {
    if (c->lnopend && s->l15_epoch[k] == c->lepoch) s->l15_acked[k][(c->elem >> 19) % LIN_CLI]++;
    return;
  }
  uint32_t lo = s->l15_epoch[k] == c->lepoch ? c->llo : 0, n = c->rval & 0xFFFFFFu;
  s->r.kv_lin_checked++;
  if (!(c->rval >> 31) || n < lo || n > s->l15_called[k][c->elem % LIN_CLI])
    t_fail(s, MR_FAIL_KV_NOT_LINEARIZABLE);
}
static void lin_call(OSim* s, OClerk* c) {
  if (s->ctrl_mode) return;
  if (s->lin15) { lin15_call(s, c); return; }
  if (c->op == KV_PUT) { /* a new value */
    memset(s->lin[c->key & (KV_KEYS - 1)], 0, sizeof s->lin[0]);
    return;
  }
  if (c->op == KV_APPEND) { lin_ent(s, c->key, c->elem >> 19)[1]++; return; }
  if (c->elem == KV_ALL) { /* appenders 0..4: each one's bound, kept in its entry */
    for (uint32_t cli = 0; cli < KV_APP; cli++) {
      uint32_t* e = lin_ent(s, c->key, cli);
      e[4] = e[2] > e[3] ? e[2] : e[3];
    }
    return;
  }
  uint32_t* e = lin_ent(s, c->key, c->elem);
  c->llo = e[2] > e[3] ? e[2] : e[3];
}
static void lin_return(OSim* s, OClerk* c) {
  if (s->ctrl_mode) return;
  if (s->lin15) { lin15_return(s, c); return; }
  if (c->op == KV_APPEND) { lin_ent(s, c->key, c->elem >> 19)[2]++; return; }
  if (c->op != KV_GET) return;
  if (c->elem == KV_ALL) { /* count (5 bits, 31 = saturated) | ok << 5 per appender */
    s->r.kv_lin_checked++;
    for (uint32_t cli = 0; cli < KV_APP; cli++) {
      uint32_t* e = lin_ent(s, c->key, cli), st = (c->rval >> (6 * cli)) & 63u, n = st & 31u;
      if (!(st >> 5) || (n < 31u && (n < e[4] || n > e[1]))) t_fail(s, MR_FAIL_KV_NOT_LINEARIZABLE);
      if (n > e[3]) e[3] = n;
    }
    return;
  }
  uint32_t* e = lin_ent(s, c->key, c->elem);
  uint32_t n = c->rval & 0xFFFFFFu;
  s->r.kv_lin_checked++;
  if (!(c->rval >> 31) || n < c->llo || n > e[1]) t_fail(s, MR_FAIL_KV_NOT_LINEARIZABLE);
  if (n > e[3]) e[3] = n;
}

static void clerk_begin(OSim* s, uint32_t slot, uint32_t op, uint32_t key, uint32_t elem) {
  OClerk* c = &s->ck[slot];
  c->seq++; c->op = op; c->key = key; c->elem = elem;
  lin_call(s, c);
  clerk_send(s, slot);
}

/* the clerk's thread woke (reply or timeout): 1 = call done (value in rval) */
static int clerk_resume(OSim* s, uint32_t slot) {
  OClerk* c = &s->ck[slot];
  c->waiting = 0;
  /* the as-shipped ClerkCore::call: todo!() once call_timeout returns (kvraft/client.rs:59) */
  if (s->null_raft) t_fail(s, MR_FAIL_TODO_RPC_RESULTS);
  if (c->got) {
    if (c->rstat == KV_OK) { s->r.kv_ops++; lin_return(s, c); return 1; }
    c->lh = c->rstat == KV_WRONG_LEADER ? c->rhint : (c->lh + 1) % s->n;
  } else {
    c->lh = (c->lh + 1) % s->n;
  }
  clerk_send(s, slot);
  return 0;
}

static int thr_bool(OSim* s, OThr* t, uint32_t p_q32) { /* rng.gen_bool on the thread's stream */
  uint32_t ctr[4] = {t->tctr++, t->tid, ST_TESTER, 0}, w[4];
  draw(s, ctr, w);
  return w[0] < p_q32;
}

/* a tester thread finished (its segment record is written): wake a joining test body */
static void thr_finish(OSim* s, uint32_t slot) {
  s->th[slot].live = 0;
  if (s->main_join == slot || s->main_join == JOIN_ANY) s->mwake = s->now;
  if (s->main_join == JOIN_ALL) {
    uint32_t live = 0;
    for (uint32_t k = 1; k < MAX_THR; k++) live += s->th[k].live;
    if (!live) s->mwake = s->now;
  }
}

/* client task of generic_test, kvraft/tests.rs:109-131 */
static void kv_client_step(OSim* s, uint32_t slot) {
  OThr* t = &s->th[slot];
  OClerk* c = &s->ck[slot];
  for (;;) {
    switch (t->pc) {
      case 0: clerk_begin(s, slot, KV_PUT, t->cli, 0); t->hlast = 0; t->pc = 1; goto block; /* ck.put(&key, "") */
      case 1: if (!clerk_resume(s, slot)) goto block; t->pc = 2; break;
      case 2:
        if (s->kv_done) goto finish;
        if (thr_bool(s, t, 0x80000000u)) {
          uint32_t e = (t->cli << 19) | t->j; /* "x {cli} {j} y"; last += &nv */
          t->hlast = t->hlast * KV_HP + e + 1;
          clerk_begin(s, slot, KV_APPEND, t->cli, e);
          t->pc = 3;
        } else {
          clerk_begin(s, slot, KV_GET, t->cli, t->cli);
          t->pc = 4;
        }
        goto block;
      case 3: if (!clerk_resume(s, slot)) goto block; t->j++; t->pc = 2; break;
      case 4:
        if (!clerk_resume(s, slot)) goto block;
        s->r.kv_checked++;
        if (c->rvh != t->hlast) t_fail(s, MR_FAIL_KV_GET_WRONG); /* kvraft/tests.rs:127 */
        t->pc = 2;
        break;
      default: t_fail(s, MR_FAIL_SIM_BAD_PROGRAM);
    }
  }
block:
  rec_simple(s, 2, t->tid & 0xFFu);
  return;
finish:
  rec_simple(s, 2, t->tid & 0xFFu);
  thr_finish(s, slot);
}

/* client task of generic_test_linearizability (SEMANTICS §9b): random keys and operations */
static uint32_t thr_range(OSim* s, OThr* t, uint32_t lo, uint32_t hi);
static void lin_client_step(OSim* s, uint32_t slot) {
  OThr* t = &s->th[slot];
  for (;;) {
    switch (t->pc) {
      case 0: {
        if (s->kv_done) goto finish;
        uint32_t key = thr_range(s, t, 0, LIN_CLI), e = (t->cli << 19) | t->j;
        if (thr_range(s, t, 0, 1000) < 500) {
          clerk_begin(s, slot, KV_APPEND, key, e);
          t->pc = 1;
        } else if (thr_range(s, t, 0, 1000) < 100) {
          clerk_begin(s, slot, KV_PUT, key, e);
          t->pc = 1;
        } else {
          clerk_begin(s, slot, KV_GET, key, thr_range(s, t, 0, LIN_CLI));
          t->pc = 2;
        }
        goto block;
      }
      case 1: if (!clerk_resume(s, slot)) goto block; t->j++; t->pc = 0; break;
      case 2: if (!clerk_resume(s, slot)) goto block; t->pc = 0; break;
      default: t_fail(s, MR_FAIL_SIM_BAD_PROGRAM);
    }
  }
block:
  rec_simple(s, 2, t->tid & 0xFFu);
  return;
finish:
  rec_simple(s, 2, t->tid & 0xFFu);
  thr_finish(s, slot);
}

/* kvraft/tester.rs:88-124: connect2 / disconnect2 of every (i in p1, j in p2), both ways */
static void set_link(OSim* s, uint32_t i, uint32_t j, int up) {
  if (up) { s->link[i] |= (uint8_t)(1u << j); s->link[j] |= (uint8_t)(1u << i); }
  else { s->link[i] &= (uint8_t)~(1u << j); s->link[j] &= (uint8_t)~(1u << i); }
}
static void t_partition(OSim* s, uint32_t p1, uint32_t p2) { /* masks of servers; tester.rs:112-122 */
  for (uint32_t i = 0; i < s->n; i++) {
    if (!((p1 >> i) & 1u)) continue;
    for (uint32_t j = 0; j < s->n; j++) if ((p2 >> j) & 1u) set_link(s, i, j, 0);
    for (uint32_t j = 0; j < s->n; j++) if ((p1 >> j) & 1u) set_link(s, i, j, 1);
  }
  for (uint32_t i = 0; i < s->n; i++) {
    if (!((p2 >> i) & 1u)) continue;
    for (uint32_t j = 0; j < s->n; j++) if ((p1 >> j) & 1u) set_link(s, i, j, 0);
    for (uint32_t j = 0; j < s->n; j++) if ((p2 >> j) & 1u) set_link(s, i, j, 1);
  }
}
static void t_connect_all(OSim* s) { memset(s->link, 0xFF, sizeof s->link); } /* tester.rs:106-110 */

static uint32_t thr_range(OSim* s, OThr* t, uint32_t lo, uint32_t hi) { /* rng.gen_range(lo..hi) */
  uint32_t ctr[4] = {t->tctr++, t->tid, ST_TESTER, 0}, w[4];
  draw(s, ctr, w);
  return u_range(w[0], lo, hi);
}

/* the partitioner task of generic_test (kvraft/tests.rs:135-157): while !done,
 * shuffle `all` (rand 0.8 SliceRandom::shuffle: i = n-1..1, swap(i, gen_range(0..i+1))),
 * split at gen_range(0..n), partition, sleep RAFT_ELECTION_TIMEOUT + gen_range(0..200) ms */
static void part_step(OSim* s, uint32_t slot) {
  OThr* t = &s->th[slot];
  if (s->kv_done) {
    rec_simple(s, 2, t->tid & 0xFFu);
    thr_finish(s, slot);
    return;
  }
  uint32_t n = s->n, a[MR_MAX_NODES];
  for (uint32_t i = 0; i < n; i++) a[i] = (t->perm >> (4 * i)) & 15u;
  for (uint32_t i = n - 1; i >= 1; i--) {
    uint32_t j = thr_range(s, t, 0, i + 1), x = a[i];
    a[i] = a[j]; a[j] = x;
  }
  uint32_t k = thr_range(s, t, 0, n), left = 0, right = 0;
  t->perm = 0;
  for (uint32_t i = 0; i < n; i++) {
    t->perm |= a[i] << (4 * i);
    if (i < k) left |= 1u << a[i]; else right |= 1u << a[i];
  }
  t_partition(s, left, right);
  uint32_t ms = thr_range(s, t, 0, 200);
  rec_simple(s, 2, t->tid & 0xFFu);
  thr_wake(s, slot, s->now + 1000000u + 1000u * ms);
}

/* ---- raft tests with spawn_local (tests.rs:662-686, 743-856) ---- */
static uint64_t thr_entry(OSim* s, OThr* t) { /* random.gen_entry() on the thread's stream */
  uint32_t ctr[4] = {t->tctr++, t->tid, ST_TESTER, 0}, w[4];
  draw(s, ctr, w);
  return ((uint64_t)w[1] << 32) | w[0];
}

/* cfn, the churn client (tests.rs:763-797); slot 1 + me */
static void churn_step(OSim* s, uint32_t slot) {
  static const uint32_t TO_MS[5] = {10, 20, 50, 100, 200};
  OThr* t = &s->th[slot];
  uint32_t me = slot - 1, idx, term;
  for (int guard = 0;; guard++) {
    if (guard > 4096) t_fail(s, MR_FAIL_SIM_BAD_PROGRAM); /* a segment must end (SEMANTICS §8) */
    if (t->pc == 0) {
      if (s->churn_stop) { rec_simple(s, 2, t->tid & 0xFFu); thr_finish(s, slot); return; }
      t->xv = thr_entry(s, t);
      t->has = 0;
      for (uint32_t i = 0; i < s->n; i++) { /* try them all, maybe one of them is a leader */
        if (!t_is_started(s, i)) continue;
        if (t_start(s, i, t->xv, &idx, &term)) { t->idx = idx; t->has = 1; }
      }
      if (!t->has) { s->th[slot].j = 79 + me * 17; goto sleep_ms; }
      t->toi = 0;
      t->pc = 1;
    }
    /* pc 1: for to in [10, 20, 50, 100, 200] { n_committed(index) ...; sleep(to) } */
    uint32_t cnt; uint64_t v;
    n_committed(s, t->idx, &cnt, &v);
    if (cnt > 0) {
      if (v == t->xv) {
        if (t->nval >= CHURN_VCAP) t_fail(s, MR_FAIL_SIM_CAPACITY);
        s->cval[me * CHURN_VCAP + t->nval] = v;
        s->cidx[me * CHURN_VCAP + t->nval] = t->idx;
        t->nval++;
      }
      t->pc = 0;
      continue;
    }
    s->th[slot].j = TO_MS[t->toi++];
    if (t->toi == 5) t->pc = 0;
    goto sleep_ms;
  }
sleep_ms:
  rec_simple(s, 2, t->tid & 0xFFu);
  thr_wake(s, slot, s->now + s->th[slot].j * 1000u);
}

/* one(cmd, expected, retry) as a spawned task (tester.rs:216-262), unreliable_agree_2c */
static void one_thr_step(OSim* s, uint32_t slot) {
  OThr* t = &s->th[slot];
  uint32_t term;
  for (;;) {
    if (t->ph == 1) {
      if (!(s->now - t->t0 < 10000000u)) t_fail(s, MR_FAIL_ONE_NO_AGREEMENT);
      int have = 0;
      for (uint32_t k = 0; k < s->n; k++) {
        t->starts = (t->starts + 1) % s->n;
        if (!t_is_connected(s, t->starts) || !t_is_started(s, t->starts)) continue;
        if (t_start(s, t->starts, t->cmd, &t->index, &term)) { have = 1; break; }
      }
      if (!have) { rec_simple(s, 2, t->tid & 0xFFu); thr_wake(s, slot, s->now + 50000u); return; }
      t->t1 = s->now;
      t->ph = 2;
    }
    if (s->now - t->t1 < 2000000u) {
      uint32_t cnt; uint64_t v;
      n_committed(s, t->index, &cnt, &v);
      if (cnt > 0 && cnt >= t->expected && v == t->cmd) {
        rec_simple(s, 2, t->tid & 0xFFu);
        thr_finish(s, slot);
        return;
      }
      rec_simple(s, 2, t->tid & 0xFFu);
      thr_wake(s, slot, s->now + 20000u);
      return;
    }
    if (!t->retry) t_fail(s, MR_FAIL_ONE_NO_AGREEMENT);
    t->ph = 1;
  }
}

static void ctl_client_step(OSim* s, uint32_t slot);

static void client_step(OSim* s, uint32_t slot) {
  switch (s->scenario) {
    case MR_SCN_RELIABLE_CHURN_2C:
    case MR_SCN_UNRELIABLE_CHURN_2C: churn_step(s, slot); break;
    case MR_SCN_UNRELIABLE_AGREE_2C: one_thr_step(s, slot); break;
    case MR_SCN_CTRL_BASIC_4A:
    case MR_SCN_CTRL_MULTI_4A: ctl_client_step(s, slot); break;
    default:
      if (s->th[slot].kind == 1) part_step(s, slot);
      else if (s->th[slot].kind == 4) lin_client_step(s, slot);
      else if (s->th[slot].kind >= 2) kv_task_step(s, slot);
      else kv_client_step(s, slot);
      break;
  }
}

static void t_join_all(OSim* s) { /* future::join_all(handles).await: wakes when the last ends */
  uint32_t live = 0;
  for (uint32_t k = 1; k < MAX_THR; k++) live += s->th[k].live;
  if (!live) return;
  s->main_join = JOIN_ALL;
  s->mwake = INF_T;
  main_block(s);
  s->main_join = ~0u;
}

static void thr_spawn(OSim* s, uint32_t slot, uint32_t tid) { /* task::spawn_local */
  OThr* t = &s->th[slot];
  uint32_t gen = t->gen;
  memset(t, 0, sizeof *t);
  t->tid = tid; t->live = 1; t->gen = gen;
  thr_wake(s, slot, s->now);
}

static void scn_churn(OSim* s, int unreliable) { /* internal_churn, tests.rs:755-856 */
  uint32_t n = s->n;
  t_new(s, 0);
  t_set_unreliable(s, unreliable);
  s->churn_stop = 0;
  s->th[0].live = 1;
  for (uint32_t i = 0; i < 3; i++) thr_spawn(s, 1 + i, 1 + i); /* ncli = 3 */
  for (int it = 0; it < 20; it++) {
    if (t_bool(s, 858993459u)) { uint32_t i = t_range(s, 0, n); t_disconnect(s, i); } /* 0.2 */
    if (t_bool(s, 0x80000000u)) {
      uint32_t i = t_range(s, 0, n);
      if (!t_is_started(s, i)) t_start1(s, i);
      t_connect(s, i);
    }
    if (t_bool(s, 858993459u)) {
      uint32_t i = t_range(s, 0, n);
      if (t_is_started(s, i)) t_crash1(s, i);
    }
    t_sleep(s, ELECTION_US * 7 / 10);
  }
  t_sleep(s, ELECTION_US);
  t_set_unreliable(s, 0);
  for (uint32_t i = 0; i < n; i++) {
    if (!t_is_started(s, i)) t_start1(s, i);
    t_connect(s, i);
  }
  s->churn_stop = 1;
  t_sleep(s, ELECTION_US);
  uint32_t last = t_one(s, t_entry(s), n, 1);
  uint64_t v;
  for (uint32_t index = 1; index <= last; index++) t_wait(s, index, n, 0, 0, &v);
  t_join_all(s);
  for (uint32_t c = 0; c < 3; c++)
    for (uint32_t k = 0; k < s->th[1 + c].nval; k++) {
      uint64_t v1 = s->cval[c * CHURN_VCAP + k];
      int found = 0;
      for (uint32_t index = 1; index <= last && !found; index++) {
        uint32_t cnt; uint64_t w;
        n_committed(s, index, &cnt, &w);
        found = cnt > 0 && w == v1;
      }
      if (!found) t_fail(s, MR_FAIL_CHURN_VALUE); /* tests.rs:852 */
    }
  t_end(s);
}

static void scn_unreliable_agree(OSim* s) { /* tests.rs:662-686 */
  uint32_t n = s->n, tid = 1;
  t_new(s, 0);
  t_set_unreliable(s, 1);
  s->th[0].live = 1;
  for (uint32_t iters = 1; iters < 50; iters++) {
    for (uint32_t j = 0; j < 4; j++) {
      uint32_t slot = 1;
      while (slot < MAX_THR && s->th[slot].live) slot++;
      if (slot == MAX_THR) t_fail(s, MR_FAIL_SIM_CAPACITY);
      thr_spawn(s, slot, tid++);
      OThr* t = &s->th[slot];
      t->cmd = 100 * iters + j; t->expected = 1; t->retry = 1;
      t->t0 = s->now; t->starts = 0; t->ph = 1;
    }
    t_one(s, iters, 1, 1);
  }
  t_set_unreliable(s, 0);
  t_join_all(s);
  t_one(s, 100, n, 1);
  t_end(s);
}

static void kv_spawn(OSim* s, uint32_t slot, uint32_t tid, uint32_t cli) { /* task::spawn_local */
  OThr* t = &s->th[slot];
  uint32_t gen = t->gen;
  memset(t, 0, sizeof *t);
  t->tid = tid; t->live = 1; t->cli = cli; t->gen = gen;
  memset(&s->ck[slot], 0, sizeof s->ck[slot]);
  s->ck[slot].id = tid; /* make_client order: ck = 0, then one clerk per client task */
  s->ck[slot].owner = slot;
  thr_wake(s, slot, s->now);
}

static void t_join(OSim* s, uint32_t slot) { /* JoinHandle.await */
  if (!s->th[slot].live) return;
  s->main_join = slot;
  s->mwake = INF_T;
  main_block(s);
  s->main_join = ~0u;
}

/* a call by the test body through the clerk of slot k (ck = slot 0) */
static uint32_t main_callk(OSim* s, uint32_t k, uint32_t op, uint32_t key, uint32_t elem) {
  clerk_begin(s, k, op, key, elem);
  for (;;) {
    main_block(s);
    if (clerk_resume(s, k)) return s->ck[k].rval;
  }
}
static uint32_t main_call(OSim* s, uint32_t op, uint32_t key, uint32_t elem) { /* ck.get etc. */
  return main_callk(s, 0, op, key, elem);
}

/* ---- kvraft tests with their own bodies (kvraft/tests.rs:240-342, 396-492) ---- */
#define KEY_LETTER(c) (50u + (uint32_t)((c) - 'a')) /* keys "a".."n" (SEMANTICS §9) */
#define TOK_NUM(v) ((v) + 1u)                         /* the Put token of decimal string v */
#define TOK_LETTER(c) ((1u << 20) + (uint32_t)((c) - 'A'))
static uint64_t put_hash(uint32_t tok) { return tok ? (tok + 1ull) * 0x9E3779B97F4A7C15ull : 0; }

/* make_client(to) owned by the test body in slot k (kvraft/tester.rs:127-150) */
static void main_clerk(OSim* s, uint32_t k, uint32_t id, uint32_t to) {
  memset(&s->ck[k], 0, sizeof s->ck[k]);
  s->ck[k].id = id; s->ck[k].mcl = k != 0; s->ck[k].owner = 0;
  s->ccut[k] = (uint8_t)~to;
}
static void t_connect_client(OSim* s, uint32_t k, uint32_t to) { s->ccut[k] = (uint8_t)~to; }
static void t_check(OSim* s, uint32_t k, uint32_t key, uint32_t tok) { /* Clerk::check */
  main_callk(s, k, KV_GET, key, 0);
  s->r.kv_checked++;
  if (s->ck[k].rvh != put_hash(tok)) t_fail(s, MR_FAIL_KV_CHECK);
}
static uint32_t kv_leader(OSim* s) { /* Tester::leader (kvraft/tester.rs:171-182) */
  for (uint32_t i = 0; i < s->n; i++) if (s->nd[i].alive && s->nd[i].role == R_L) return i;
  return ~0u;
}
/* a one-key appender (kvraft/tests.rs:255-262) or a single-call task (:309-314) */
static void kv_task_step(OSim* s, uint32_t slot) {
  OThr* t = &s->th[slot];
  if (t->pc == 1) {
    if (!clerk_resume(s, slot)) { rec_simple(s, 2, t->tid & 0xFFu); return; }
    t->j++;
    t->pc = 0;
  }
  if (t->j < t->expected) {
    uint32_t elem = t->kind == 2 ? (t->cli << 19) | t->j : (uint32_t)t->cmd;
    clerk_begin(s, slot, (uint32_t)t->retry, t->index, elem);
    t->pc = 1;
    rec_simple(s, 2, t->tid & 0xFFu);
    return;
  }
  rec_simple(s, 2, t->tid & 0xFFu);
  thr_finish(s, slot);
}
/* make_client(to) whose calls a spawned task in slot k will make */
static void task_clerk(OSim* s, uint32_t k, uint32_t id, uint32_t to) {
  memset(&s->ck[k], 0, sizeof s->ck[k]);
  s->ck[k].id = id; s->ck[k].owner = k;
  s->ccut[k] = (uint8_t)~to;
}
/* task::spawn_local of a task over the clerk of its slot: `count` calls of op on key */
static void kv_task_spawn(OSim* s, uint32_t slot, uint32_t tid, uint32_t kind, uint32_t cli,
                          uint32_t op, uint32_t key, uint32_t elem, uint32_t count) {
  thr_spawn(s, slot, tid);
  OThr* t = &s->th[slot];
  t->kind = kind; t->cli = cli; t->retry = op; t->index = key; t->cmd = elem; t->expected = count;
}

static void scn_kv_one_key(OSim* s) { /* unreliable_one_key_3a, kvraft/tests.rs:240-274 */
  t_new(s, 0);
  t_set_unreliable(s, 1);
  s->kv_mode = 1;
  s->th[0].live = 1;
  main_clerk(s, 0, 0, 0xFFu);
  const uint32_t K = KEY_LETTER('k');
  main_call(s, KV_PUT, K, 0);
  for (uint32_t i = 0; i < 5; i++) { /* make_client(&t.all()), then spawn its appender */
    task_clerk(s, 1 + i, 1 + i, 0xFFu);
    kv_task_spawn(s, 1 + i, 1 + i, 2, i, KV_APPEND, K, 0, 10);
  }
  t_join_all(s);
  uint32_t v = main_call(s, KV_GET, K, KV_ALL);
  s->r.kv_checked++;
  for (uint32_t i = 0; i < 5; i++) { /* check_concurrent_appends(&vx, &counts) */
    uint32_t f = (v >> (6 * i)) & 63u;
    if (!(f >> 5)) t_fail(s, MR_FAIL_KV_APPEND_BAD);
    if ((f & 31u) < 10) t_fail(s, MR_FAIL_KV_MISSING);
  }
  t_end(s);
}

static void scn_kv_one_partition(OSim* s) { /* one_partition_3a, kvraft/tests.rs:276-342 */
  uint32_t n = s->n, all = (1u << n) - 1;
  t_new(s, 0);
  s->kv_mode = 1;
  s->th[0].live = 1;
  main_clerk(s, 0, 0, all);
  main_call(s, KV_PUT, 1, TOK_NUM(13));
  uint32_t leader = kv_leader(s), a[MR_MAX_NODES], m = n; /* make_partition (tester.rs:184-192) */
  if (leader == ~0u) leader = 0;
  for (uint32_t i = 0; i < n; i++) a[i] = i;
  a[leader] = a[m - 1]; m--; /* swap_remove(leader) */
  uint32_t p1 = 0, p2 = 1u << leader;
  for (uint32_t i = 0; i < m; i++) { if (i < n / 2 + 1) p1 |= 1u << a[i]; else p2 |= 1u << a[i]; }
  t_partition(s, p1, p2);
  main_clerk(s, 1, 1, p1); /* ckp1 */
  task_clerk(s, 2, 2, p2);  /* ckp2a */
  task_clerk(s, 3, 3, p2);  /* ckp2b */
  main_callk(s, 1, KV_PUT, 1, TOK_NUM(14));
  t_check(s, 1, 1, TOK_NUM(14));
  kv_task_spawn(s, 2, 1, 3, 0, KV_PUT, 1, TOK_NUM(15), 1); /* ckp2a.put("1", "15") */
  kv_task_spawn(s, 3, 2, 3, 0, KV_GET, 1, 0, 1);           /* ckp2b.get("1") */
  s->main_join = JOIN_ANY; s->mwake = s->now + 1000000u; /* select! { put, get, sleep(1 s) } */
  main_block(s);
  s->main_join = ~0u;
  if (!s->th[2].live || !s->th[3].live) t_fail(s, MR_FAIL_KV_MINORITY_PROGRESS);
  t_check(s, 1, 1, TOK_NUM(14));
  main_callk(s, 1, KV_PUT, 1, TOK_NUM(16));
  t_check(s, 1, 1, TOK_NUM(16));
  t_connect_all(s);
  t_connect_client(s, 2, all);
  t_connect_client(s, 3, all);
  t_sleep(s, ELECTION_US);
  if (s->th[2].live && s->th[3].live) { /* select! { sleep(3 s), put, get } */
    s->main_join = JOIN_ANY; s->mwake = s->now + 3000000u;
    main_block(s);
    s->main_join = ~0u;
    if (s->th[2].live && s->th[3].live) t_fail(s, MR_FAIL_KV_NO_COMPLETION);
  }
  t_check(s, 0, 1, TOK_NUM(15));
  t_end(s);
}

static void scn_kv_snapshot_rpc(OSim* s) { /* snapshot_rpc_3b, kvraft/tests.rs:396-454 */
  s->kv_maxraft = 1000;
  t_new(s, 0);
  s->kv_mode = 1;
  s->th[0].live = 1;
  main_clerk(s, 0, 0, 7u);
  main_call(s, KV_PUT, KEY_LETTER('a'), TOK_LETTER('A'));
  t_check(s, 0, KEY_LETTER('a'), TOK_LETTER('A'));
  t_partition(s, 3u, 4u); /* [0, 1] | [2] */
  main_clerk(s, 1, 1, 3u);
  for (uint32_t i = 0; i < 50; i++) main_callk(s, 1, KV_PUT, i, TOK_NUM(i));
  t_sleep(s, ELECTION_US);
  main_callk(s, 1, KV_PUT, KEY_LETTER('b'), TOK_LETTER('B'));
  if (t_log_size(s) > 2 * s->kv_maxraft) t_fail(s, MR_FAIL_KV_LOG_SIZE);
  t_partition(s, 5u, 2u); /* [0, 2] | [1] */
  main_clerk(s, 2, 2, 5u);
  main_callk(s, 2, KV_PUT, KEY_LETTER('c'), TOK_LETTER('C'));
  main_callk(s, 2, KV_PUT, KEY_LETTER('d'), TOK_LETTER('D'));
  t_check(s, 2, KEY_LETTER('a'), TOK_LETTER('A'));
  t_check(s, 2, KEY_LETTER('b'), TOK_LETTER('B'));
  t_check(s, 2, 1, TOK_NUM(1));
  t_check(s, 2, 49, TOK_NUM(49));
  t_partition(s, 7u, 0u);
  main_call(s, KV_PUT, KEY_LETTER('e'), TOK_LETTER('E'));
  t_check(s, 0, KEY_LETTER('c'), TOK_LETTER('C'));
  t_check(s, 0, KEY_LETTER('e'), TOK_LETTER('E'));
  t_check(s, 0, 1, TOK_NUM(1));
  t_end(s);
}

static void scn_kv_snapshot_size(OSim* s) { /* snapshot_size_3b, kvraft/tests.rs:456-492 */
  s->kv_maxraft = 1000;
  t_new(s, 0);
  s->kv_mode = 1;
  s->th[0].live = 1;
  main_clerk(s, 0, 0, 7u);
  const uint32_t X = KEY_LETTER('x');
  for (int i = 0; i < 200; i++) {
    main_call(s, KV_PUT, X, TOK_NUM(0));
    t_check(s, 0, X, TOK_NUM(0));
    main_call(s, KV_PUT, X, TOK_NUM(1));
    t_check(s, 0, X, TOK_NUM(1));
  }
  if (t_log_size(s) > 2 * s->kv_maxraft) t_fail(s, MR_FAIL_KV_LOG_SIZE);
  uint32_t mx = 0;
  for (uint32_t i = 0; i < s->n; i++) { uint32_t z = kv_snap_size(&s->kvs[i]); if (z > mx) mx = z; }
  if (mx > 500) t_fail(s, MR_FAIL_KV_SNAPSHOT_SIZE);
  t_end(s);
}

/* kvraft/tester.rs:153-169: the KV server's state machine is volatile (rebuilt by
 * re-applying the log from the snapshot); its Raft state persists (SEMANTICS §9) */
static void t_shutdown_server(OSim* s, uint32_t i) { t_crash1(s, i); }
static void t_start_server(OSim* s, uint32_t i) {
  t_start1(s, i);
  if (s->kv_maxraft) { kv_state_put(s, i, &s->kvs[i]); return; } /* restore from the snapshot */
  memset(s->kv[i], 0, sizeof s->kv[i]);
  memset(s->kv_dedup[i], 0, sizeof s->kv_dedup[i]);
}

/* kvraft/tests.rs:65-220; with `lin`, generic_test_linearizability (SEMANTICS §9b, the
 * reference's sketched kvraft/tests.rs:386-390, 524-528) */
static void scn_kv_generic(OSim* s, uint32_t nclients, int unreliable, int crash, int partitions,
                           uint32_t maxraftstate, int lin) {
  s->kv_maxraft = maxraftstate;
  s->lin15 = lin;
  t_new(s, 0); /* Tester::new (kvraft/tester.rs:27-56): start_server for every server */
  if (unreliable) t_set_unreliable(s, 1);
  s->kv_mode = 1;
  s->th[0].live = 1;
  memset(&s->ck[0], 0, sizeof s->ck[0]); /* ck = make_client(&t.all()): clerk 0 */
  uint32_t ps = 1 + nclients; /* the partitioner's slot */
  for (uint32_t i = 0; i < 3; i++) {
    s->kv_done = 0;
    for (uint32_t cli = 0; cli < nclients; cli++) {
      kv_spawn(s, 1 + cli, 1 + nclients * i + cli, cli);
      if (lin) { s->th[1 + cli].kind = 4; s->th[1 + cli].j = s->l15_j[cli]; }
    }
    if (partitions) {
      t_sleep(s, 1000000u);
      thr_spawn(s, ps, 1 + 3 * nclients + i);
      s->th[ps].kind = 1;
      s->ck[ps].id = 0xFFFFu; /* no clerk */
      for (uint32_t k = 0; k < s->n; k++) s->th[ps].perm |= k << (4 * k); /* t.all() */
    }
    t_sleep(s, 5000000u);
    s->kv_done = 1;
    if (partitions) {
      t_join(s, ps);
      t_connect_all(s);
      t_sleep(s, ELECTION_US);
    }
    if (crash) {
      for (uint32_t k = 0; k < s->n; k++) t_shutdown_server(s, k);
      t_sleep(s, ELECTION_US);
      for (uint32_t k = 0; k < s->n; k++) t_start_server(s, k);
      t_connect_all(s);
    }
    for (uint32_t cli = 0; cli < nclients; cli++) {
      t_join(s, 1 + cli);
      if (lin) { /* no predicted values: the checker judged every Get (SEMANTICS §9b) */
        s->l15_j[cli] = s->th[1 + cli].j;
        continue;
      }
      uint32_t j = s->th[1 + cli].j;
      uint32_t v = main_call(s, KV_GET, cli, cli); /* check_clnt_appends(cli, &v, j) */
      s->r.kv_checked++;
      if (!(v >> 31)) t_fail(s, MR_FAIL_KV_APPEND_BAD);         /* kvraft/tests.rs:31-39 */
      if ((v & 0x7FFFFFFFu) < j) t_fail(s, MR_FAIL_KV_MISSING); /* kvraft/tests.rs:25-30 */
    }
    if (maxraftstate && t_log_size(s) > 2 * maxraftstate) t_fail(s, MR_FAIL_KV_LOG_SIZE); /* :208-215 */
  }
  t_end(s);
}

/* ---- shard_ctrler tests (src/shard_ctrler/tests.rs, tester.rs; SEMANTICS §10) ---- */
static uint32_t ct_op(OSim* s, uint32_t type, uint32_t a, uint32_t b) {
  if (s->nops >= OP_CAP) t_fail(s, MR_FAIL_SIM_CAPACITY);
  OOp* op = &s->ops[s->nops];
  memset(op, 0, sizeof *op);
  op->type = type; op->a = a; op->b = b;
  return s->nops++;
}
static void ct_grp(OSim* s, uint32_t id, uint32_t gid, uint32_t addr) { /* groups! / gids entry */
  OOp* op = &s->ops[id];
  op->gid[op->ng] = gid; op->addr[op->ng] = addr; op->ng++;
}
static uint32_t addrs(uint32_t n, uint32_t a0, uint32_t a1, uint32_t a2) { /* addrs![..], `as u8` */
  return n | (a0 & 255u) << 8 | (n > 1 ? (a1 & 255u) << 16 : 0) | (n > 2 ? (a2 & 255u) << 24 : 0);
}
/* ck.<op>() by the test body: the reply's config (Query) as (server, index) */
static const OCfg* ct_call(OSim* s, uint32_t id) {
  uint32_t idx = main_call(s, 0, 0, id);
  return &s->cfgs[s->ck[0].rhint * CFG_CAP + idx];
}
static const OCfg* ct_query(OSim* s, uint32_t num) { return ct_call(s, ct_op(s, CT_QUERY, num, 0)); }
static int cfg_has(const OCfg* c, uint32_t gid) {
  for (uint32_t g = 0; g < c->ng; g++) if (c->gid[g] == gid) return 1;
  return 0;
}
static int cfg_eq(const OCfg* a, const OCfg* b) {
  if (a->num != b->num || a->ng != b->ng) return 0;
  for (uint32_t j = 0; j < N_SHARDS; j++) if (a->shards[j] != b->shards[j]) return 0;
  for (uint32_t g = 0; g < a->ng; g++)
    if (a->gid[g] != b->gid[g] || a->addr[g] != b->addr[g]) return 0;
  return 1;
}
static void ct_servers(OSim* s, const OCfg* c, uint32_t gid, uint32_t addr) { /* cfx.groups[&gid] == addr */
  for (uint32_t g = 0; g < c->ng; g++)
    if (c->gid[g] == gid) { if (c->addr[g] != addr) t_fail(s, MR_FAIL_CTRL_SERVERS); return; }
  t_fail(s, MR_FAIL_CTRL_SERVERS); /* HashMap index panics */
}
static void ct_check(OSim* s, uint32_t ng, const uint32_t* gids) { /* Clerk::check, tester.rs:113-150 */
  const OCfg* c = ct_query(s, 0xFFFFFFFFu);
  if (c->ng != ng) t_fail(s, MR_FAIL_CTRL_NGROUPS);
  for (uint32_t k = 0; k < ng; k++) if (!cfg_has(c, gids[k])) t_fail(s, MR_FAIL_CTRL_MISSING);
  if (ng == 0)
    for (uint32_t j = 0; j < N_SHARDS; j++)
      if (c->shards[j] != 0 && !cfg_has(c, c->shards[j])) t_fail(s, MR_FAIL_CTRL_INVALID);
  if (c->ng) {
    uint32_t mn = ~0u, mx = 0;
    for (uint32_t g = 0; g < c->ng; g++) {
      uint32_t k = 0;
      for (uint32_t j = 0; j < N_SHARDS; j++) k += c->shards[j] == c->gid[g];
      if (k < mn) mn = k;
      if (k > mx) mx = k;
    }
    if (mx > mn + 1) t_fail(s, MR_FAIL_CTRL_IMBALANCED);
  }
}
static void ct_minimal(OSim* s, const OCfg* a, const OCfg* b, uint32_t npara, uint32_t code) {
  for (uint32_t i = 1; i <= npara; i++) /* tests.rs:133-140 / 152-159 */
    for (uint32_t j = 0; j < N_SHARDS; j++)
      if (b->shards[j] == i && a->shards[j] != i) t_fail(s, code);
}
static int ct_leader(OSim* s) { /* Tester::leader, shard_ctrler/tester.rs:76-87 */
  for (uint32_t i = 0; i < s->n; i++) if (s->nd[i].alive && s->nd[i].role == R_L) return (int)i;
  return -1;
}

/* a concurrent client task (tests.rs:110-117 / 224-233): one clerk call per segment chain */
static void ctl_client_step(OSim* s, uint32_t slot) {
  OThr* t = &s->th[slot];
  const uint32_t gid = t->cli, multi = s->scenario == MR_SCN_CTRL_MULTI_4A;
  const uint32_t nops = multi ? 2 : 3;
  if (t->pc > 0 && !clerk_resume(s, slot)) goto block; /* the call in flight */
  if (t->pc == nops) { rec_simple(s, 2, t->tid & 0xFFu); thr_finish(s, slot); return; }
  {
    uint32_t id;
    if (!multi) {
      if (t->pc == 0) { id = ct_op(s, CT_JOIN, 0, 0); ct_grp(s, id, gid + 1000, addrs(1, gid + 1, 0, 0)); }
      else if (t->pc == 1) { id = ct_op(s, CT_JOIN, 0, 0); ct_grp(s, id, gid, addrs(1, gid + 2, 0, 0)); }
      else { id = ct_op(s, CT_LEAVE, 0, 0); ct_grp(s, id, gid + 1000, 0); }
    } else if (t->pc == 0) {
      id = ct_op(s, CT_JOIN, 0, 0);
      ct_grp(s, id, gid, addrs(3, gid + 1, gid + 2, gid + 3));
      ct_grp(s, id, gid + 1000, addrs(1, gid + 1000 + 1, 0, 0));
      ct_grp(s, id, gid + 2000, addrs(1, gid + 2000 + 1, 0, 0));
    } else {
      id = ct_op(s, CT_LEAVE, 0, 0);
      ct_grp(s, id, gid + 1000, 0); ct_grp(s, id, gid + 2000, 0);
    }
    t->pc++;
    clerk_begin(s, slot, 0, 0, id);
  }
block:
  rec_simple(s, 2, t->tid & 0xFFu);
}

static void ct_spawn(OSim* s, uint32_t slot, uint32_t tid, uint32_t gid) {
  thr_spawn(s, slot, tid);
  s->th[slot].cli = gid;
  memset(&s->ck[slot], 0, sizeof s->ck[slot]);
  s->ck[slot].id = tid; /* cka = t.make_client() */
  s->ck[slot].owner = slot;
}

static void scn_ctrl_basic(OSim* s) { /* basic_4a, shard_ctrler/tests.rs:24-166 */
  const uint32_t npara = 10;
  const OCfg* cfa[8];
  uint32_t ncfa = 0, id, g[10];
  t_new(s, 0);
  s->kv_mode = 1; s->ctrl_mode = 1; s->th[0].live = 1;
  cfa[ncfa++] = ct_query(s, 0xFFFFFFFFu);
  ct_check(s, 0, g);
  id = ct_op(s, CT_JOIN, 0, 0); ct_grp(s, id, 1, addrs(3, 11, 12, 13)); ct_call(s, id);
  g[0] = 1; ct_check(s, 1, g);
  cfa[ncfa++] = ct_query(s, 0xFFFFFFFFu);
  id = ct_op(s, CT_JOIN, 0, 0); ct_grp(s, id, 2, addrs(3, 21, 22, 23)); ct_call(s, id);
  g[1] = 2; ct_check(s, 2, g);
  cfa[ncfa++] = ct_query(s, 0xFFFFFFFFu);
  const OCfg* cfx = ct_query(s, 0xFFFFFFFFu);
  ct_servers(s, cfx, 1, addrs(3, 11, 12, 13));
  ct_servers(s, cfx, 2, addrs(3, 21, 22, 23));
  id = ct_op(s, CT_LEAVE, 0, 0); ct_grp(s, id, 1, 0); ct_call(s, id);
  g[0] = 2; ct_check(s, 1, g);
  cfa[ncfa++] = ct_query(s, 0xFFFFFFFFu);
  id = ct_op(s, CT_LEAVE, 0, 0); ct_grp(s, id, 2, 0); ct_call(s, id);
  cfa[ncfa++] = ct_query(s, 0xFFFFFFFFu);
  for (uint32_t sv = 0; sv < s->n; sv++) { /* Historical queries */
    t_crash1(s, sv);
    for (uint32_t k = 0; k < ncfa; k++)
      if (!cfg_eq(ct_query(s, cfa[k]->num), cfa[k])) t_fail(s, MR_FAIL_CTRL_HISTORY);
    t_start1(s, sv);
  }
  id = ct_op(s, CT_JOIN, 0, 0); ct_grp(s, id, 503, addrs(3, 31, 32, 33)); ct_call(s, id);
  id = ct_op(s, CT_JOIN, 0, 0); ct_grp(s, id, 504, addrs(3, 41, 42, 43)); ct_call(s, id);
  for (uint32_t i = 0; i < N_SHARDS; i++) { /* Move */
    const OCfg* cf = ct_query(s, 0xFFFFFFFFu);
    uint32_t shard = i < N_SHARDS / 2 ? 503 : 504;
    ct_call(s, ct_op(s, CT_MOVE, i, shard));
    if (cf->shards[i] != shard) {
      const OCfg* cf1 = ct_query(s, 0xFFFFFFFFu);
      if (!(cf1->num > cf->num)) t_fail(s, MR_FAIL_CTRL_MOVE_NUM);
    }
  }
  const OCfg* cf2 = ct_query(s, 0xFFFFFFFFu);
  for (uint32_t i = 0; i < N_SHARDS; i++)
    if (cf2->shards[i] != (i < N_SHARDS / 2 ? 503u : 504u)) t_fail(s, MR_FAIL_CTRL_MOVE_WRONG);
  id = ct_op(s, CT_LEAVE, 0, 0); ct_grp(s, id, 503, 0); ct_call(s, id);
  id = ct_op(s, CT_LEAVE, 0, 0); ct_grp(s, id, 504, 0); ct_call(s, id);
  for (uint32_t i = 0; i < npara; i++) ct_spawn(s, 1 + i, 1 + i, i * 10 + 100); /* Concurrent leave/join */
  t_join_all(s);
  for (uint32_t i = 0; i < npara; i++) g[i] = i * 10 + 100;
  ct_check(s, npara, g);
  const OCfg* c1 = ct_query(s, 0xFFFFFFFFu); /* Minimal transfers after joins */
  for (uint32_t i = 0; i < 5; i++) {
    uint32_t gid = npara + 1 + i;
    id = ct_op(s, CT_JOIN, 0, 0); ct_grp(s, id, gid, addrs(3, gid + 1, gid + 2, gid + 2)); ct_call(s, id);
  }
  const OCfg* c2 = ct_query(s, 0xFFFFFFFFu);
  ct_minimal(s, c1, c2, npara, MR_FAIL_CTRL_MINIMAL_JOIN);
  for (uint32_t i = 0; i < 5; i++) { /* Minimal transfers after leaves */
    id = ct_op(s, CT_LEAVE, 0, 0); ct_grp(s, id, npara + 1 + i, 0); ct_call(s, id);
  }
  const OCfg* c3 = ct_query(s, 0xFFFFFFFFu);
  ct_minimal(s, c3, c2, npara, MR_FAIL_CTRL_MINIMAL_LEAVE); /* !(c2 == i && c3 != i) */
  t_end(s);
}

static void scn_ctrl_multi(OSim* s) { /* multi_4a, shard_ctrler/tests.rs:168-299 */
  const uint32_t npara = 10;
  uint32_t id, g[10];
  t_new(s, 0);
  s->kv_mode = 1; s->ctrl_mode = 1; s->th[0].live = 1;
  ct_query(s, 0xFFFFFFFFu); /* cfa.push */
  ct_check(s, 0, g);
  id = ct_op(s, CT_JOIN, 0, 0);
  ct_grp(s, id, 1, addrs(3, 11, 12, 13)); ct_grp(s, id, 2, addrs(3, 21, 22, 23)); ct_call(s, id);
  g[0] = 1; g[1] = 2; ct_check(s, 2, g);
  ct_query(s, 0xFFFFFFFFu);
  id = ct_op(s, CT_JOIN, 0, 0); ct_grp(s, id, 3, addrs(3, 31, 32, 33)); ct_call(s, id);
  g[2] = 3; ct_check(s, 3, g);
  ct_query(s, 0xFFFFFFFFu);
  const OCfg* cfx = ct_query(s, 0xFFFFFFFFu);
  ct_servers(s, cfx, 1, addrs(3, 11, 12, 13));
  ct_servers(s, cfx, 2, addrs(3, 21, 22, 23));
  ct_servers(s, cfx, 3, addrs(3, 31, 32, 33));
  id = ct_op(s, CT_LEAVE, 0, 0); ct_grp(s, id, 1, 0); ct_grp(s, id, 3, 0); ct_call(s, id);
  g[0] = 2; ct_check(s, 1, g);
  ct_query(s, 0xFFFFFFFFu);
  cfx = ct_query(s, 0xFFFFFFFFu);
  ct_servers(s, cfx, 2, addrs(3, 21, 22, 23));
  id = ct_op(s, CT_LEAVE, 0, 0); ct_grp(s, id, 2, 0); ct_call(s, id);
  for (uint32_t i = 0; i < npara; i++) ct_spawn(s, 1 + i, 1 + i, i + 1000); /* Concurrent multi leave/join */
  t_join_all(s);
  for (uint32_t i = 0; i < npara; i++) g[i] = i + 1000;
  ct_check(s, npara, g);
  const OCfg* c1 = ct_query(s, 0xFFFFFFFFu); /* Minimal transfers after multijoins */
  id = ct_op(s, CT_JOIN, 0, 0);
  for (uint32_t i = 0; i < 5; i++) {
    uint32_t gid = npara + 1 + i;
    ct_grp(s, id, gid, addrs(2, gid + 1, gid + 2, 0));
  }
  ct_call(s, id);
  const OCfg* c2 = ct_query(s, 0xFFFFFFFFu);
  ct_minimal(s, c1, c2, npara, MR_FAIL_CTRL_MINIMAL_JOIN);
  id = ct_op(s, CT_LEAVE, 0, 0); /* Minimal transfers after multileaves */
  for (uint32_t i = 0; i < 5; i++) ct_grp(s, id, npara + 1 + i, 0);
  ct_call(s, id);
  const OCfg* c3 = ct_query(s, 0xFFFFFFFFu);
  ct_minimal(s, c3, c2, npara, MR_FAIL_CTRL_MINIMAL_LEAVE);
  int leader = ct_leader(s); /* Check Same config on servers */
  if (leader < 0) t_fail(s, MR_FAIL_CTRL_NO_LEADER);
  const OCfg* c = ct_query(s, 0xFFFFFFFFu);
  t_crash1(s, (uint32_t)leader);
  uint32_t attempts = 0;
  while (ct_leader(s) >= 0) {
    attempts++;
    if (!(attempts < 3)) t_fail(s, MR_FAIL_CTRL_NO_LEADER);
    t_sleep(s, 1000000u);
  }
  const OCfg* c1b = ct_query(s, 0xFFFFFFFFu);
  if (!cfg_eq(c, c1b)) t_fail(s, MR_FAIL_CTRL_SAME_CONFIG);
  t_end(s);
}

static int run_scenario(OSim* s) {
  switch (s->scenario) {
    case MR_SCN_INITIAL_ELECTION_2A: scn_initial_election(s); break;
    case MR_SCN_REELECTION_2A: scn_reelection(s); break;
    case MR_SCN_MANY_ELECTION_2A: scn_many_election(s); break;
    case MR_SCN_BASIC_AGREE_2B: scn_basic_agree(s); break;
    case MR_SCN_FAIL_AGREE_2B: scn_fail_agree(s); break;
    case MR_SCN_FAIL_NO_AGREE_2B: scn_fail_no_agree(s); break;
    case MR_SCN_CONCURRENT_STARTS_2B: scn_concurrent_starts(s); break;
    case MR_SCN_REJOIN_2B: scn_rejoin(s); break;
    case MR_SCN_BACKUP_2B: scn_backup(s); break;
    case MR_SCN_COUNT_2B: scn_count(s); break;
    case MR_SCN_PERSIST1_2C: scn_persist1(s); break;
    case MR_SCN_PERSIST2_2C: scn_persist2(s); break;
    case MR_SCN_PERSIST3_2C: scn_persist3(s); break;
    case MR_SCN_FIGURE_8_2C:
    case MR_SCN_FIGURE_8_UNRELIABLE_CRASH: scn_figure_8(s); break;
    case MR_SCN_FIGURE_8_UNRELIABLE_2C: scn_figure_8_unreliable(s); break;
    case MR_SCN_SNAPSHOT_BASIC_2D: scn_snap_common(s, 0, 1, 0); break;
    case MR_SCN_SNAPSHOT_INSTALL_2D: scn_snap_common(s, 1, 1, 0); break;
    case MR_SCN_SNAPSHOT_INSTALL_UNRELIABLE_2D: scn_snap_common(s, 1, 0, 0); break;
    case MR_SCN_SNAPSHOT_INSTALL_CRASH_2D: scn_snap_common(s, 0, 1, 1); break;
    case MR_SCN_SNAPSHOT_INSTALL_UNRELIABLE_CRASH_2D: scn_snap_common(s, 0, 0, 1); break;
    case MR_SCN_UNRELIABLE_AGREE_2C: scn_unreliable_agree(s); break;
    case MR_SCN_RELIABLE_CHURN_2C: scn_churn(s, 0); break;
    case MR_SCN_UNRELIABLE_CHURN_2C: scn_churn(s, 1); break;
    case MR_SCN_CTRL_BASIC_4A: scn_ctrl_basic(s); break;
    case MR_SCN_CTRL_MULTI_4A: scn_ctrl_multi(s); break;
    case MR_SCN_KV_BASIC_3A: scn_kv_generic(s, 1, 0, 0, 0, 0, 0); break;
    case MR_SCN_KV_CONCURRENT_3A: scn_kv_generic(s, 5, 0, 0, 0, 0, 0); break;
    case MR_SCN_KV_UNRELIABLE_3A: scn_kv_generic(s, 5, 1, 0, 0, 0, 0); break;
    case MR_SCN_KV_MANY_PARTITIONS_ONE_CLIENT_3A: scn_kv_generic(s, 1, 0, 0, 1, 0, 0); break;
    case MR_SCN_KV_MANY_PARTITIONS_MANY_CLIENTS_3A: scn_kv_generic(s, 5, 0, 0, 1, 0, 0); break;
    case MR_SCN_KV_PERSIST_ONE_CLIENT_3A: scn_kv_generic(s, 1, 0, 1, 0, 0, 0); break;
    case MR_SCN_KV_PERSIST_CONCURRENT_3A: scn_kv_generic(s, 5, 0, 1, 0, 0, 0); break;
    case MR_SCN_KV_PERSIST_CONCURRENT_UNRELIABLE_3A: scn_kv_generic(s, 5, 1, 1, 0, 0, 0); break;
    case MR_SCN_KV_PERSIST_PARTITION_3A: scn_kv_generic(s, 5, 0, 1, 1, 0, 0); break;
    case MR_SCN_KV_PERSIST_PARTITION_UNRELIABLE_3A: scn_kv_generic(s, 5, 1, 1, 1, 0, 0); break;
    case MR_SCN_KV_UNRELIABLE_ONE_KEY_3A: scn_kv_one_key(s); break;
    case MR_SCN_KV_ONE_PARTITION_3A: scn_kv_one_partition(s); break;
    case MR_SCN_KV_SNAPSHOT_RPC_3B: scn_kv_snapshot_rpc(s); break;
    case MR_SCN_KV_SNAPSHOT_SIZE_3B: scn_kv_snapshot_size(s); break;
    case MR_SCN_KV_SNAPSHOT_RECOVER_3B: scn_kv_generic(s, 1, 0, 1, 0, 1000, 0); break;
    case MR_SCN_KV_SNAPSHOT_RECOVER_MANY_CLIENTS_3B: scn_kv_generic(s, 20, 0, 1, 0, 1000, 0); break;
    case MR_SCN_KV_SNAPSHOT_UNRELIABLE_3B: scn_kv_generic(s, 5, 1, 0, 0, 1000, 0); break;
    case MR_SCN_KV_SNAPSHOT_UNRELIABLE_RECOVER_3B: scn_kv_generic(s, 5, 1, 1, 0, 1000, 0); break;
    case MR_SCN_KV_PERSIST_PARTITION_UNRELIABLE_LINEARIZABLE_3A:
      scn_kv_generic(s, LIN_CLI, 1, 1, 1, 0, 1);
      break;
    case MR_SCN_KV_SNAPSHOT_UNRELIABLE_RECOVER_CONCURRENT_PARTITION_LINEARIZABLE_3B:
      scn_kv_generic(s, LIN_CLI, 1, 1, 1, 1000, 1);
      break;
    case MR_SCN_KV_SNAPSHOT_UNRELIABLE_RECOVER_CONCURRENT_PARTITION_3B:
      scn_kv_generic(s, 5, 1, 1, 1, 1000, 0);
      break;
    default: return -1;
  }
  return 0;
}

/* ------------------------------------------------------------------ */
/* seed loop                                                            */
/* ------------------------------------------------------------------ */
static int sim_alloc(OSim* s, const mr_cfg* cfg) {
  memset(s, 0, sizeof *s);
  s->cfg = *cfg;
  if (cfg->n_nodes < 3 || cfg->n_nodes > MR_MAX_NODES) return -1;
  if (cfg->log_cap < 16 || (cfg->log_cap & (cfg->log_cap - 1))) return -1;
  if (cfg->msg_slots < 1 || cfg->msg_slots > MR_MAX_MSG_SLOTS) return -1;
  if (cfg->msg_slots > 64 && !mr_scn_wide_slots(cfg->scenario)) return -1;
  if (cfg->ae_max < 1 || cfg->ae_max > MR_MAX_AE) return -1;
  if (cfg->apply_cap < 16) return -1;
  for (uint32_t i = 0; i < cfg->n_nodes; i++) {
    s->nd[i].lterm = (uint32_t*)malloc(cfg->log_cap * sizeof(uint32_t));
    s->nd[i].lval = (uint64_t*)malloc(cfg->log_cap * sizeof(uint64_t));
  }
  s->cfgs = (OCfg*)malloc(MR_MAX_NODES * CFG_CAP * sizeof(OCfg));
  s->ops = (OOp*)malloc(OP_CAP * sizeof(OOp));
  s->cval = (uint64_t*)malloc(3 * CHURN_VCAP * sizeof(uint64_t));
  s->cidx = (uint32_t*)malloc(3 * CHURN_VCAP * sizeof(uint32_t));
  s->kvs = (OKvState*)malloc(MR_MAX_NODES * sizeof(OKvState));
  s->kring = (OKvState*)malloc(KV_RING * sizeof(OKvState));
  s->kring_idx = (uint32_t*)malloc(KV_RING * sizeof(uint32_t));
  s->mask = (uint8_t*)malloc(cfg->apply_cap);
  s->sval = (uint64_t*)malloc(cfg->apply_cap * sizeof(uint64_t));
  s->sterm = (uint32_t*)malloc(cfg->apply_cap * sizeof(uint32_t));
  return 0;
}

static void sim_free(OSim* s) {
  for (uint32_t i = 0; i < MR_MAX_NODES; i++) { free(s->nd[i].lterm); free(s->nd[i].lval); }
  free(s->mask); free(s->sval); free(s->sterm); free(s->heap); free(s->cval); free(s->cidx);
  free(s->cfgs); free(s->ops); free(s->kvs); free(s->kring); free(s->kring_idx);
}

static void sim_reset(OSim* s, uint64_t cluster) {
  uint64_t seed = s->cfg.seed_base + cluster;
  s->key[0] = (uint32_t)seed; s->key[1] = (uint32_t)(seed >> 32);
  s->n = s->cfg.n_nodes; s->now = 0; s->scenario = s->cfg.scenario;
  s->null_raft = (s->cfg.flags & MR_F_NULL_RAFT) ? 1 : 0;
  s->snapshot_mode = 0;
  t_set_unreliable(s, 0);
  for (uint32_t i = 0; i < MR_MAX_NODES; i++) {
    ONode* d = &s->nd[i];
    uint32_t* lt = d->lterm; uint64_t* lv = d->lval;
    memset(d, 0, sizeof *d);
    d->lterm = lt; d->lval = lv;
    d->voted = -1;
  }
  s->n_free = s->cfg.msg_slots;
  for (uint32_t i = 0; i < s->n_free; i++) s->free_stack[i] = s->n_free - 1 - i;
  s->inflight = 0; s->heap_n = 0; s->t_ctr = 0;
  s->kv_mode = 0; s->kv_done = 0; s->mwake = 0; s->main_join = ~0u;
  memset(s->kv, 0, sizeof s->kv);
  memset(s->kv_dedup, 0, sizeof s->kv_dedup); memset(s->pend, 0, sizeof s->pend);
  memset(s->ck, 0, sizeof s->ck); memset(s->th, 0, sizeof s->th); s->churn_stop = 0;
  s->ctrl_mode = 0; s->nops = 0;
  memset(s->led, 0, sizeof s->led);
  memset(s->lin, 0, sizeof s->lin);
  s->lin15 = 0;
  memset(s->l15_called, 0, sizeof s->l15_called); memset(s->l15_acked, 0, sizeof s->l15_acked);
  memset(s->l15_epoch, 0, sizeof s->l15_epoch); memset(s->l15_pend, 0, sizeof s->l15_pend);
  memset(s->l15_j, 0, sizeof s->l15_j);
  s->kv_maxraft = 0;
  memset(s->kvs, 0, MR_MAX_NODES * sizeof(OKvState));
  memset(s->kring_idx, 0, KV_RING * sizeof(uint32_t));
  memset(s->link, 0xFF, sizeof s->link);
  memset(s->ccut, 0, sizeof s->ccut);
  for (uint32_t i = 0; i < MR_MAX_NODES; i++) { /* the initial config, num 0 */
    s->ncfg[i] = 1;
    memset(&s->cfgs[i * CFG_CAP], 0, sizeof(OCfg));
  }
  memset(s->mask, 0, s->cfg.apply_cap);
  for (uint32_t i = 0; i < MR_MAX_NODES; i++) s->slen[i] = 1;
  memset(&s->r, 0, sizeof s->r);
  s->r.digest = 0xCBF29CE484222325ull;
  s->n_trace = 0;
  memset(s->adig, 0, sizeof s->adig); memset(s->ainv, 0, sizeof s->ainv);
  uint64_t row = cluster - s->cfg.cluster_base;
  s->tape_row = row;
  s->tape_on = g_tape_mode == 2 || (g_tape_mode == 1 && row < g_dec_rows);
  s->tape_pos = 0;
}

static void sim_run(OSim* s, uint64_t cluster) {
  sim_reset(s, cluster);
  if (setjmp(s->jb) == 0) {
    count_event(s); /* the tester's first wake-up at t = 0 */
    s->r.ev_tester++;
    if (run_scenario(s) != 0) t_fail(s, MR_FAIL_SIM_BAD_PROGRAM);
  }
  if (s->tape_on && g_dec_count) g_dec_count[cluster - s->cfg.cluster_base] = s->tape_pos;
}

static int dec_sort(const void* a, const void* b) {
  const mr_decision* x = (const mr_decision*)a;
  const mr_decision* y = (const mr_decision*)b;
  if (x->cluster != y->cluster) return x->cluster < y->cluster ? -1 : 1;
  return dec_cmp(x, y->stream, y->entity, y->seq);
}

int mro_set_decisions(int mode, const mr_decision* d, uint64_t n, uint64_t rows,
                      mr_decision* rec, uint64_t rec_cap, uint64_t* count) {
  free(g_dec); free(g_dec_off);
  g_dec = NULL; g_dec_off = NULL; g_dec_rows = 0; g_rec = NULL; g_rec_cap = 0;
  g_dec_count = count; g_tape_mode = 0;
  if (mode == 1) {
    g_dec = (mr_decision*)malloc((n ? n : 1) * sizeof(mr_decision));
    g_dec_off = (uint64_t*)calloc(rows + 1, sizeof(uint64_t));
    if (n) memcpy(g_dec, d, n * sizeof(mr_decision));
    qsort(g_dec, n, sizeof(mr_decision), dec_sort);
    for (uint64_t i = 0; i < n; i++) {
      if (g_dec[i].cluster >= rows) return -1;
      if (i && g_dec[i].cluster == g_dec[i - 1].cluster &&
          dec_cmp(&g_dec[i], g_dec[i - 1].stream, g_dec[i - 1].entity, g_dec[i - 1].seq) == 0)
        return -2; /* duplicate key */
      g_dec_off[g_dec[i].cluster + 1]++;
    }
    for (uint64_t r = 0; r < rows; r++) g_dec_off[r + 1] += g_dec_off[r];
    g_dec_rows = rows;
  } else if (mode == 2) {
    g_rec = rec; g_rec_cap = rec_cap;
  }
  g_tape_mode = mode;
  return 0;
}

int mro_run_cluster(const mr_cfg* cfg, uint64_t cluster, mro_result* out, mr_event* trace,
                    size_t trace_cap, size_t* n_trace) {
  return mro_run_cluster_dig(cfg, cluster, out, trace, NULL, trace_cap, n_trace);
}

int mro_run_cluster_dig(const mr_cfg* cfg, uint64_t cluster, mro_result* out, mr_event* trace,
                        uint64_t* tdig, size_t trace_cap, size_t* n_trace) {
  return mro_run_cluster_kv(cfg, cluster, out, trace, tdig, NULL, trace_cap, n_trace);
}

int mro_run_cluster_kv(const mr_cfg* cfg, uint64_t cluster, mro_result* out, mr_event* trace,
                       uint64_t* tdig, uint64_t* tapp, size_t trace_cap, size_t* n_trace) {
  OSim* s = (OSim*)malloc(sizeof(OSim));
  if (!s || sim_alloc(s, cfg) != 0) { free(s); return -1; }
  s->trace = trace; s->trace_cap = trace_cap; s->tdig = tdig; s->tapp = tapp;
  if (tapp) memset(tapp, 0, trace_cap * 2 * sizeof(uint64_t));
  sim_run(s, cfg->cluster_base + cluster);
  if (out) *out = s->r;
  if (n_trace) *n_trace = s->n_trace;
  sim_free(s);
  free(s);
  return 0;
}

static void acc(mro_result* a, const mro_result* b) {
  a->events += b->events; a->ev_msg += b->ev_msg; a->ev_timer += b->ev_timer;
  a->ev_tester += b->ev_tester; a->msgs_sent += b->msgs_sent; a->drop_clog += b->drop_clog;
  a->drop_loss += b->drop_loss; a->drop_overflow += b->drop_overflow;
  a->drop_deliver += b->drop_deliver; a->drop_stale += b->drop_stale;
  a->elections += b->elections; a->leaders_elected += b->leaders_elected;
  a->applies += b->applies; a->snapshots += b->snapshots; a->installs += b->installs;
  a->entries_shipped += b->entries_shipped; a->log_writes += b->log_writes;
  if (b->max_inflight > a->max_inflight) a->max_inflight = b->max_inflight;
  if (b->max_log > a->max_log) a->max_log = b->max_log;
  if (b->max_index > a->max_index) a->max_index = b->max_index;
  a->kv_ops += b->kv_ops; a->kv_checked += b->kv_checked; a->kv_lin_checked += b->kv_lin_checked;
}

int mro_run_batch(const mr_cfg* cfg, uint64_t first, uint64_t count, uint16_t* code,
                  uint32_t* time_us, uint64_t* digest, mro_result* sum) {
  OSim* s = (OSim*)malloc(sizeof(OSim));
  if (!s || sim_alloc(s, cfg) != 0) { free(s); return -1; }
  if (sum) memset(sum, 0, sizeof *sum);
  for (uint64_t c = 0; c < count; c++) {
    sim_run(s, cfg->cluster_base + first + c);
    if (code) code[c] = (uint16_t)s->r.code;
    if (time_us) time_us[c] = s->r.time_us;
    if (digest) digest[c] = s->r.digest;
    if (sum) acc(sum, &s->r);
  }
  sim_free(s);
  free(s);
  return 0;
}

/* ------------------------------------------------------------------ */
/* names / defaults (mirrors mr_cfg_init of the product ABI)           */
/* ------------------------------------------------------------------ */
static const char* k_names[MR_SCN_COUNT_] = {
    "", "initial_election_2a", "reelection_2a", "many_election_2a", "basic_agree_2b",
    "fail_agree_2b", "fail_no_agree_2b", "concurrent_starts_2b", "rejoin_2b", "backup_2b",
    "count_2b", "persist1_2c", "persist2_2c", "persist3_2c", "figure_8_2c",
    "unreliable_agree_2c", "figure_8_unreliable_2c", "reliable_churn_2c",
    "unreliable_churn_2c", "snapshot_basic_2d", "snapshot_install_2d",
    "snapshot_install_unreliable_2d", "snapshot_install_crash_2d",
    "snapshot_install_unreliable_crash_2d", "figure_8_unreliable_crash", "basic_3a",
    "concurrent_3a", "unreliable_3a", "basic_4a", "multi_4a",
    "many_partitions_one_client_3a", "many_partitions_many_clients_3a", "persist_one_client_3a",
    "persist_concurrent_3a", "persist_concurrent_unreliable_3a", "persist_partition_3a",
    "persist_partition_unreliable_3a", "unreliable_one_key_3a", "one_partition_3a",
    "snapshot_rpc_3b", "snapshot_size_3b", "snapshot_recover_3b", "snapshot_recover_many_clients_3b",
    "snapshot_unreliable_3b", "snapshot_unreliable_recover_3b",
    "snapshot_unreliable_recover_concurrent_partition_3b",
    "persist_partition_unreliable_linearizable_3a",
    "snapshot_unreliable_recover_concurrent_partition_linearizable_3b"};

uint32_t mro_scenario_from_name(const char* name) {
  for (uint32_t i = 1; i < MR_SCN_COUNT_; i++)
    if (strcmp(name, k_names[i]) == 0) return i;
  return 0;
}

int mro_cfg_init(mr_cfg* c, uint32_t scn) {
  static const uint8_t k_n[MR_SCN_COUNT_] = {0, 3, 3, 7, 5, 3, 5, 3, 3, 5, 3, 3, 5, 3,
                                             5, 5, 5, 5, 5, 3, 3, 3, 3, 3, 5, 5, 5, 5, 3, 3,
                                             5, 5, 5, 5, 5, 5, 5, 3, 5, 3, 3, 5, 5, 5, 5, 5, 7, 7};
  if (scn == 0 || scn >= MR_SCN_COUNT_) return -1;
  memset(c, 0, sizeof *c);
  c->abi_version = MR_ABI_VERSION;
  c->scenario = scn;
  c->n_nodes = k_n[scn];
  c->seed_base = 1629626496ull; /* README.md:48 */
  c->n_clusters = 1;
  /* capacities sized from the oracle's maxima over 2000 seeds */
  int fig8 = scn == MR_SCN_FIGURE_8_2C || scn == MR_SCN_FIGURE_8_UNRELIABLE_2C ||
             scn == MR_SCN_FIGURE_8_UNRELIABLE_CRASH;
  int snap = scn >= MR_SCN_SNAPSHOT_BASIC_2D && scn <= MR_SCN_SNAPSHOT_INSTALL_UNRELIABLE_CRASH_2D;
  int kv = mr_scn_is_kv(scn);
  int churn = scn == MR_SCN_RELIABLE_CHURN_2C || scn == MR_SCN_UNRELIABLE_CHURN_2C;
  uint32_t cap = fig8 ? 2048 : kv ? mr_kv_log_cap(scn)
               : churn ? 4096 : scn == MR_SCN_UNRELIABLE_AGREE_2C ? 1024 : 0;
  c->log_cap = cap ? cap : 256;
  c->apply_cap = cap ? cap : (snap ? 1024 : 512);
  c->msg_slots = mr_scn_wide_slots(scn) ? 256 : kv ? 64 : 32;
  c->ae_max = 16;
  c->hb_us = 50000;
  c->elect_lo_us = 150000;
  c->elect_hi_us = 300000;
  c->max_events = 4u << 20;
  c->trace_cap = 1u << 16;
  return 0;
}

const char* mro_fail_message(uint32_t code) {
  switch (code) {
    case MR_PASS: return "ok";
    case MR_FAIL_ONE_LEADER_NONE: return "expected one leader, got none";
    case MR_FAIL_MULTI_LEADER_TERM: return "term has (>1) leaders";
    case MR_FAIL_TERM_DISAGREE: return "servers disagree on term";
    case MR_FAIL_UNEXPECTED_LEADER: return "expected no leader, but claims to be leader";
    case MR_FAIL_WAIT_TOO_FEW: return "only decided for index; wanted more";
    case MR_FAIL_ONE_NO_AGREEMENT: return "one() failed to reach agreement";
    case MR_FAIL_TIMEOUT_120S: return "test took longer than 120 seconds";
    case MR_FAIL_APPLY_MISMATCH: return "commit index mismatch between servers";
    case MR_FAIL_APPLY_OUT_OF_ORDER: return "server apply out of order";
    case MR_FAIL_UNWRAP_NONE: return "called `Option::unwrap()` on a `None` value";
    case MR_FAIL_LOG_SIZE: return "log size too large";
    case MR_FAIL_KV_GET_WRONG: return "get wrong value";
    case MR_FAIL_KV_MISSING: return "missing element in Append result";
    case MR_FAIL_KV_APPEND_BAD: return "duplicate or wrong order element in Append result";
    case MR_FAIL_SAFETY_ELECTION: return "election safety: two leaders in one term";
    case MR_FAIL_SAFETY_COMPLETENESS: return "leader completeness: new leader lacks a committed entry";
    case MR_FAIL_KV_LOG_SIZE: return "logs were not trimmed";
    case MR_FAIL_KV_SNAPSHOT_SIZE: return "snapshot too large";
    case MR_FAIL_KV_MINORITY_PROGRESS: return "put/get in minority completed";
    case MR_FAIL_KV_NO_COMPLETION: return "put/get did not complete";
    case MR_FAIL_KV_CHECK: return "get(key) check failed";
    case MR_FAIL_SAFETY_LOG_MATCHING: return "log matching: same index and term, different entries";
    case MR_FAIL_TODO_APPLY: return "not yet implemented: apply command";
    case MR_FAIL_TODO_RPC_RESULTS: return "not yet implemented: handle RPC results";
    case MR_FAIL_KV_NOT_LINEARIZABLE: return "history is not linearizable";
    case MR_FAIL_SIM_CAPACITY: return "simulator capacity exceeded";
    case MR_FAIL_SIM_EVENT_LIMIT: return "simulator event limit exceeded";
    default: return "scenario assertion failed";
  }
}
