// mr_dev.h — device state layout shared by the HIP kernels (mr_kernel.hip)
// and the C++ batch driver (mr_host.cpp).
//
// Layout: one lane simulates one cluster. Two kinds of arrays:
//  * cluster-minor matrices [field][...][C] for what every lane of a wave
//    touches at the same field index (cluster scalars, tester frame, message
//    keys in the launch prologue / epilogue): 64 lanes read 64 consecutive
//    words;
//  * cluster-major records for what a lane touches at a per-lane index — a
//    node (the event's destination differs per lane), a message slot, log
//    entries, apply-checker indices: one node's whole state is one 128-B
//    record (scalars + next[] + match[]), one message one 32-B record, so an
//    event touches one or two lines per object instead of one line per field
//    (a [field][node][C] layout costs a line per field per lane once the
//    lanes' node indices differ).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/madraft_sim.h"

namespace mr {

// ---- node flag word (one u32 per node): role[0:2) voted[4:8) (15 = none)
//      inc[8:16) votes[16:24); started / connected are cluster bit masks (CS_ALIVE, CS_CONN)
enum : uint32_t { R_F = 0, R_C = 1, R_L = 2, R_DOWN = 3 };
enum : uint32_t { M_RV_REQ = 1, M_RV_REP, M_AE_REQ, M_AE_REP, M_IS_REQ, M_IS_REP, M_KV_REQ, M_KV_REP };
enum : uint32_t { ST_TESTER = 1, ST_ELECT = 2, ST_NET = 3 };

// per-cluster u32 counters (part of cs32); the last three are maxima
enum : uint32_t {
  CNT_EV_MSG, CNT_EV_TIMER, CNT_EV_TESTER, CNT_DROP_CLOG, CNT_DROP_LOSS, CNT_DROP_OVERFLOW,
  CNT_DROP_DELIVER, CNT_DROP_STALE, CNT_ELECTIONS, CNT_LEADERS, CNT_APPLIES, CNT_SNAPSHOTS,
  CNT_INSTALLS, CNT_SHIPPED, CNT_LOG_WRITES, CNT_MATERIALIZED, CNT_COOP,
  CNT_MAX_INFLIGHT, CNT_MAX_LOG, CNT_MAX_INDEX, CNT__N
};

// tester coroutine frame (per cluster): program counter, script locals,
// helper frame of the multi-event tester calls (one / wait / check_one_leader)
constexpr uint32_t T_NL = 8;   // u32 script locals
constexpr uint32_t T_NH = 5;   // u32 helper frame
constexpr uint32_t T_NV = 16;  // u64 script arrays (count_2b / concurrent_starts)

// cs32 [CS__N][C]: per-cluster u32 scalars
enum : uint32_t {
  CS_CODE, CS_VTIME, CS_NOW, CS_EVENTS, CS_MSGS, CS_INFLIGHT, CS_NETMODE, CS_TCTR, CS_TRACEN,
  CS_MSLOT, CS_CONN, CS_ALIVE, CS_TWAKE, CS_CNT,  // (the tester frame is the tfr record)
  CS_KVDONE = CS_CNT + CNT__N, CS_MJOIN, CS_CWAKE, CS_CTID, CS_CSLOT,  // tester threads (SEMANTICS §8-9)
  CS_NLIVE,  // live spawned threads
  CS_NOPS,   // shard_ctrler: clerk operations so far
  CS_CUT,    // server links cut (disconnect2): bit 8 (i mod 4) + j of word CS_CUT + i / 4
  CS_CUT_END = CS_CUT + 2,
  CS_CCUT,   // clerk links cut: bit 8 (k mod 4) + j of word CS_CCUT + k / 4 = clerk host 8 + k !~ server j
  CS_CCUT_END = CS_CCUT + 6,
  CS_TAPE,   // keyed decisions: recorded so far (record) / draws without a record (replay)
  CS_KV_OPS, CS_KV_CHECKED,  // service clerk calls completed / Get results verified
  CS_KV_LIN,                 // Get results the linearizability checker verified
  CS_LMASK,                  // servers whose record holds role leader (x.lmask, store_node)
  CS_LRS,                    // per node: run start of its last log entry (mr_kernel.hip le_at)
  CS_LRS_END = CS_LRS + 8,
  CS__N
};
// cs64 [C64__N][C]: per-cluster u64 scalars
// C64_FREE1..3: free-slot mask words 1..3 (slots 64..255, MR_MW = 4 units)
enum : uint32_t { C64_FREE, C64_DIGEST, C64_MMIN, C64_TV, C64_FREE1 = C64_TV + T_NV,
                  C64__N = C64_FREE1 + 3 };
// Cluster scalars: cluster-minor matrices [field][C] (a wave's lanes read 64 consecutive words
// of one field; cluster-major records measured -5 % in round 4). The strides pad the field
// counts; the host reads rows through these index macros.
constexpr uint32_t CS_STRIDE = (CS__N + 3u) & ~3u, C64_STRIDE = (C64__N + 1u) & ~1u;
#define CS_IDX(f, c, C) ((size_t)(f) * (C) + (c))
#define C64_IDX(f, c, C) ((size_t)(f) * (C) + (c))
// nd32 [C][n][NREC]: one 128-B record per node. Words 0..11 are the scalars
// an event loads / stores as a block (load_node), 12..13 the pending payload
// range, 14..15 the snapshot value (u64), 16..23 next[p], 24..31 match[p]
// (leader -> peer p). match[me] holds the leader's base: its last index when it
// won its term (every entry above it, and none at or below, has the current
// term). LASTT caches term_at(last). Node timers live in tmr [n][C].
enum : uint32_t {
  NF_FLAGS, NF_TERM, NF_COMMIT, NF_APPLIED, NF_LAST, NF_SNAP, NF_SNAPT, NF_ECTR, NF_NCTR,
  NF_PEXP, NF_SLEN, NF_LASTT, NF_PLO, NF_PHI, NF_SNAPV, NF__N = 16
};
enum : uint32_t { PF_NEXT, PF_MATCH, PF__N };
constexpr uint32_t NR_PEER = 16;  // next[] at 16, match[] at 16 + MR_MAX_NODES
constexpr uint32_t NREC = 32;
// ms32 [C][M][MREC]: one 32-B record per in-flight message (value at 6..7);
// mkey [M][C]: message keys (time, seq, dst), cluster-minor
enum : uint32_t { MF_HDR, MF_TERM, MF_A, MF_B, MF_C, MF_PAD, MF_V, MREC = 8 };

// one Raft log entry (raft.rs Log: term + command), 16 B so an entry moves as
// one 128-bit access; message payloads (AppendEntries entries) use the same form
struct alignas(16) LE {
  uint32_t term, rs;  // rs: first index of the run of entries of this term that ends here
  uint64_t val;       // (device log only; <= the snapshot index when the run reaches it)
};

// ---- kvraft (SEMANTICS §8-9); arrays allocated for the kvraft scenarios only
enum : uint32_t { KV_GET = 0, KV_PUT = 1, KV_APPEND = 2 };
enum : uint32_t { KV_OK = 0, KV_WRONG_LEADER = 1, KV_FAILED = 2 };
constexpr uint32_t CLERK_HOST = 8;  // clerk c is host 8 + c
constexpr uint32_t KV_PEND = 8;     // pending requests per server
// kt32 [C][nthr(S)][KT_STRIDE]: a spawned tester thread (+ its clerk, kvraft) per slot.
// Words KT_W.. are the thread's own frame: kvraft clerk fields, churn client
// (x lo/hi, index, timeout step, values), or a one() task (helper frame h[0..4], cmd).
enum : uint32_t {
  KT_TID, KT_LIVE, KT_PC, KT_J, KT_CLI, KT_TCTR, KT_ID, KT_LH, KT_SEQ, KT_TAG, KT_NCTR,  // (wake: kwk)
  KT_WAITING, KT_GOT, KT_RSTAT, KT_RHINT, KT_RVAL, KT_OP, KT_KEY, KT_ELEM,
  KT_KIND,  // 1 = generic_test partitioner (KT_PERM: its shuffled `all`, 4 bits per server)
  KT_PERM,
  KT_RVH0, KT_RVH1,  // the reply's value hash
  KT_HL0, KT_HL1,    // generic_test client: hash of its predicted value `last`
  KT_OWN,            // the thread the clerk's calls wake (0 = the test body)
  KT_MCL,            // 1 = a clerk of the test body in a slot that is not a thread
  KT_LLO,            // a Get's linearizability lower bound at its call (SEMANTICS §9a)
  KT_TOP, KT_TKEY, KT_TELEM, KT_TCNT,  // a task's call: op, key, elem (or appender), calls
  KT_LEP, KT_LNP,    // generic_test_linearizability (§9b): the key's Put epoch at the call, no
                     // Put pending at the call
  KT__N
};
constexpr uint32_t KT_W = KT_ID;
constexpr uint32_t KT_STRIDE = (KT__N + 3u) & ~3u;  // words per thread-slot record (16-B multiple)
constexpr uint32_t JOIN_ALL = 0xFFFFFFFEu;
constexpr uint32_t JOIN_ANY = 0xFFFFFFFDu;  // select! over spawned tasks: the first finish wakes
// kvraft key ids / Put value tokens of the test bodies (SEMANTICS §9)
constexpr uint32_t key_letter(char c) { return 50u + (uint32_t)(c - 'a'); }
constexpr uint32_t tok_num(uint32_t v) { return v + 1u; }
constexpr uint32_t tok_letter(char c) { return (1u << 20) + (uint32_t)(c - 'A'); }
constexpr uint32_t CHURN_VCAP = 512;  // values one churn client may record (tests.rs:763-797)
// kv32 [C][n][KVREC]: per-server KV state (SEMANTICS §9): dedup[clerk] at 0..127, pending
// request p at 128 + 8p: {index (0 = free), clerk | ready << 8 | status << 9 | host << 16,
// seq, tag, value, hash lo, hash hi, -}, the shard_ctrler config count at 192, the mask of
// occupied pending slots at 193, and key k at 256 + 8k: {hash lo, hash hi, byte length,
// appender 0..4 (cli + 1 | count << 8 | bad << 31)}
constexpr uint32_t KVR_DEDUP = 0, KVR_PEND = 128, KVR_NCFG = 192, KVR_PMASK = 193, KVR_KEYS = 256,
                   KVREC = 768;
constexpr uint32_t KV_KEYS = 64, KV_KW = 8, KV_APP = 5, MAX_CLERKS = 128;
constexpr uint32_t KV_ALL = 0xFFFFFFu;  // Get elem: appenders 0..4, packed
constexpr uint64_t KV_HP = 0x100000001B3ull;  // value hash multiplier
// a KV snapshot (SEMANTICS §9): dedup[128] then the 64 key records; the ring entry for
// index i (slot i / 16 mod 16) holds i at word 0 and the snapshot from word 4
constexpr uint32_t KVS_W = MAX_CLERKS + KV_KEYS * KV_KW, KV_RING = 16, KRW = 4 + KVS_W;
constexpr uint32_t KV_SNAP_EVERY = 16;
// linearizability bookkeeping per (key, appender): tag (cli + 1), appends called, appends
// acknowledged, largest count a returned Get observed, an all-appenders Get's lower bound
constexpr uint32_t LINW = 8;
// generic_test_linearizability (SEMANTICS §9b): 15 clients share keys 0..14, each key record
// is 32 words (hash lo, hi, length, the states of clients 0..14 by id: count | last j << 12 |
// bad << 31), and the tester keeps per key 32 words of lin32: called[15], acked[15], the Put
// epoch and the Puts pending; word 512 + cli of the cluster's lin32: client cli's next j
constexpr uint32_t LIN_CLI = 15, KV_KW15 = 32, LIN15_J = 512;
// ---- shard_ctrler (SEMANTICS §10): per-server append-only config store and a
// per-cluster table of clerk operations (the log command names an operation)
constexpr uint32_t N_SHARDS = 10;  // shard_ctrler/mod.rs:9
constexpr uint32_t CFG_CAP = 128, CFG_G = 32, OP_CAP = 256;
// cfg32 [C][n][CFG_CAP][CFGW]: num, shards[10], ng, gid[32], addr[32]
enum : uint32_t { CF_NUM = 0, CF_SHARDS = 1, CF_NG = 11, CF_GID = 12, CF_ADDR = 44, CFGW = 80 };
// op32 [C][OP_CAP][OPW]: type, a (num / shard), b (gid), ng, gid[5], addr[5]
enum : uint32_t { OP_TYPE = 0, OP_A, OP_B, OP_NG, OP_GID, OP_ADDR = 9, OPW = 16 };
enum : uint32_t { CT_QUERY = 0, CT_JOIN = 1, CT_LEAVE = 2, CT_MOVE = 3 };

// one tester apply-checker index (StorageHandle, tester.rs:366-428): the value
// the first applier stored, the mask of servers whose log holds it, and the
// entry's term (for the MR_F_SAFETY leader-completeness check)
struct alignas(16) SE {
  uint64_t val;
  uint32_t mask, term;
};

// ---- everything the kernels see (passed by value as a kernel argument)
struct Dev {
  // config
  uint32_t C, n, log_cap, apply_cap, M, K, hb, elo, ehi, max_events;
  uint32_t null_raft, unrel_flag, trace_clusters, trace_cap, scenario, iters, safety, bugs, links;
  uint64_t seed0;  // seed of cluster 0 = seed_base + cluster_base
  uint32_t* cs32;
  uint64_t* cs64;
  uint32_t* nd32;   // [C][n][NREC]
  uint32_t* tmr;    // [n][C] node timers (registers during a launch)
  uint32_t* ms32;   // [C][M][MREC]
  uint64_t* mkey;   // [M][C]
  LE* log;  // [C][n][log_cap] ring per node
  LE* pay;  // [C][M][K] AppendEntries payload per message slot
  SE* stor;         // [C][apply_cap]   tester storage (tester.rs:366-428)
  uint32_t* kt32;   // [C][nthr][KT_STRIDE] (spawning scenarios)
  uint32_t* kv32;   // [C][n][KVREC]        (kvraft only)
  uint32_t* kvs32;  // [C][n][KVS_W]        persisted KV snapshots (maxraftstate)
  uint32_t* kring;  // [C][KV_RING][KRW]    recent KV snapshots by index (maxraftstate)
  uint4* dtab;      // keyed decisions {stream << 16 | entity, seq, w0, w1}, else null:
                    // replay: CSR rows, cluster c's sorted by key at [doff[c], doff[c + 1]);
                    // record: [C][dcap], appended in draw order
  uint32_t* doff;   // replay: [C + 1] row offsets into dtab
  uint32_t dcap;       // record: decisions kept per cluster
  uint32_t tape_mode;  // 0 Philox, 1 replay keyed decisions, 2 Philox and record them
  uint64_t* cval;   // [C][3][CHURN_VCAP]   churn clients' committed values (churn only)
  uint32_t* cidx;   // [C][3][CHURN_VCAP]   ... and the index each was seen at
  uint32_t* cfg32;  // [C][n][CFG_CAP][CFGW] shard_ctrler config stores
  uint32_t* op32;   // [C][OP_CAP][OPW]       shard_ctrler operations
  uint32_t nthr;    // thread slots of kt32 (0 = none)
  mr_event* trace;  // [trace_clusters][trace_cap]
  uint64_t* tdig;   // [trace_clusters][trace_cap] apply digest of each record (ABI 4)
  uint64_t* tapp;   // [trace_clusters][trace_cap][2] KV command, key hash after it (ABI 4)
  uint64_t* adig;   // [trace_clusters][MR_MAX_NODES][2] per node: digest sum, invalid flag
  uint32_t* led;    // [C][LED_W] MR_F_SAFETY: bit t = a leader was elected in term t
  uint32_t* lin32;  // [C][KV_KEYS][KV_APP][LINW] kvraft linearizability bookkeeping (§9a, §9b)
  uint32_t lin15;   // generic_test_linearizability layout (§9b): key records / bookkeeping
  uint32_t* remaining;  // [2]: clusters without verdict after a step launch; next unclaimed cluster
  uint32_t L;           // clusters per launch: lane l starts with cluster c0 + l (chunk [c0, c0 + L))
  uint32_t lpw;         // lanes of each 64-lane block that hold a cluster (64, 32, 16; the rest idle)
  uint32_t c0;          // first cluster of this launch's chunk
  uint32_t stream;      // MR_F_STREAM: a lane that finishes takes the next unclaimed cluster
  uint32_t resume;      // streaming, not the chunk's first launch: lanes first take held_in[]
  uint32_t nheld;       // ... the clusters the previous launch's lanes still held
  uint32_t* held_in;    // [L] those clusters (streaming)
  uint32_t* held_out;   // [L] this launch's (index = its remaining[0] count)
  unsigned long long* prof;  // [PROF_SLOTS] wave-cycle profile (MR_PROF builds only)
  uint4* tfr;       // [C][TF_Q] the tester coroutine frame, one cluster-major 80-B record
  uint32_t* kwk;    // [C][kws(nthr)][2] thread slots' {tid, wake}: the scheduler's keys, packed
  uint32_t pool;    // the batch runs on pool_kernel (has_pool): 32-bit keys with the AE bit
  uint32_t* guard;  // [4] MR_GUARD builds: an out-of-range index {tag, cluster, index, bound}
  uint32_t gprobe;  // MR_GUARD builds, MR_GUARD_PROBE set: cluster 0's first delivery reads slot M
  unsigned long long* pcnt;  // [CNT__N] pool_kernel: the workgroups' counter sums (64-bit; reduce adds them)
  uint32_t krows;   // the 7-server Raft pool: message slots whose keys live in LDS (the rest in HBM)
};
// words-pairs per cluster of kwk: the thread slots rounded up to whole 16-B quads (two slots each;
// slot 0 = the test body and the pad slot hold ~0, so they never win a rescan)
constexpr uint32_t kws(uint32_t nthr) { return (nthr + 1u) & ~1u; }
// tester frame record (tester() in mr_kernel.hip): pc | helper << 24, result, locals l[0..7],
// helper frame h[0..4], u64 argument hv — 17 words in five 16-B quads, loaded and stored whole
constexpr uint32_t TF_Q = 5;
constexpr uint32_t PROF_SLOTS = 96;  // 64..94: pool_kernel statistics (MR_PROF, tools/prof.py)
// election-safety term bitmap (MR_F_SAFETY): terms 0..LED_TERMS-1; a leader elected in a
// later term is a simulator limit (MR_FAIL_SIM_CAPACITY); figure_8 peaks at term 177
constexpr uint32_t LED_W = 64, LED_TERMS = 32 * LED_W;

constexpr bool is_kv(uint32_t s) {
  return (s >= MR_SCN_KV_BASIC_3A && s <= MR_SCN_KV_UNRELIABLE_3A) ||
         (s >= MR_SCN_KV_MANY_PARTITIONS_ONE_CLIENT_3A &&
          s <= MR_SCN_KV_SNAPSHOT_UNRELIABLE_RECOVER_CONCURRENT_PARTITION_LINEARIZABLE_3B);
}
// generic_test(nclients, unreliable, crash, partitions, maxraftstate) of a kvraft scenario
// (kvraft/tests.rs:222-384, 494-522); snapshot_rpc / snapshot_size use maxraftstate too
struct KvGen { uint32_t nc; bool unrel, crash, part; uint32_t maxraft; bool lin; };
constexpr KvGen kv_gen(uint32_t s) {
  switch (s) {
    case MR_SCN_KV_BASIC_3A: return {1, false, false, false};
    case MR_SCN_KV_CONCURRENT_3A: return {5, false, false, false};
    case MR_SCN_KV_UNRELIABLE_3A: return {5, true, false, false};
    case MR_SCN_KV_MANY_PARTITIONS_ONE_CLIENT_3A: return {1, false, false, true};
    case MR_SCN_KV_MANY_PARTITIONS_MANY_CLIENTS_3A: return {5, false, false, true};
    case MR_SCN_KV_PERSIST_ONE_CLIENT_3A: return {1, false, true, false};
    case MR_SCN_KV_PERSIST_CONCURRENT_3A: return {5, false, true, false};
    case MR_SCN_KV_PERSIST_CONCURRENT_UNRELIABLE_3A: return {5, true, true, false};
    case MR_SCN_KV_PERSIST_PARTITION_3A: return {5, false, true, true};
    case MR_SCN_KV_PERSIST_PARTITION_UNRELIABLE_3A: return {5, true, true, true};
    case MR_SCN_KV_UNRELIABLE_ONE_KEY_3A: return {5, true, false, false};
    case MR_SCN_KV_ONE_PARTITION_3A: return {0, false, false, true};
    case MR_SCN_KV_SNAPSHOT_RPC_3B: return {0, false, false, true, 1000};
    case MR_SCN_KV_SNAPSHOT_SIZE_3B: return {0, false, false, false, 1000};
    case MR_SCN_KV_SNAPSHOT_RECOVER_3B: return {1, false, true, false, 1000};
    case MR_SCN_KV_SNAPSHOT_RECOVER_MANY_CLIENTS_3B: return {20, false, true, false, 1000};
    case MR_SCN_KV_SNAPSHOT_UNRELIABLE_3B: return {5, true, false, false, 1000};
    case MR_SCN_KV_SNAPSHOT_UNRELIABLE_RECOVER_3B: return {5, true, true, false, 1000};
    case MR_SCN_KV_SNAPSHOT_UNRELIABLE_RECOVER_CONCURRENT_PARTITION_3B: return {5, true, true, true, 1000};
    // generic_test_linearizability (15 clients, 7 servers; SEMANTICS §9b)
    case MR_SCN_KV_PERSIST_PARTITION_UNRELIABLE_LINEARIZABLE_3A: return {15, true, true, true, 0, true};
    case MR_SCN_KV_SNAPSHOT_UNRELIABLE_RECOVER_CONCURRENT_PARTITION_LINEARIZABLE_3B:
      return {15, true, true, true, 1000, true};
    default: return {0, false, false, false, 0, false};
  }
}
// the service pool's applier continuation (mr_kernel.hip AP_CAP) is built for the 15-client
// linearizable body without service snapshots, whose reconnected followers apply long backlogs:
// same box (profiles/r06_ab_kvap.txt) C5-lin 3A 76.4 K -> 103.8 K seeds/s (+36 %), while built for
// every service body config 5 (unreliable_3a) lost 21 % and the snapshotting 3B body 2 % (short
// backlogs: the extra kind and the registers cost more than the balance gains)
// (the snapshotting linearizable 3B body with it, cap 5: 89.8 K -> 88.5 K seeds/s, -1.4 %,
// profiles/r06_ab_kv47.txt)
constexpr bool ap_cont(uint32_t s) { return kv_gen(s).lin && kv_gen(s).maxraft == 0; }
// the KV snapshot copy's chunk (quads whose loads issue together, kv_snapshot): 8 for
// the 15-client linearizable body, 4 for the others. Same box (profiles/r06_ab_kc.txt): the
// snapshotting linearizable 3B body 89.7 K -> 93.6 K seeds/s with 8 (+4.4 %; 16: -5 %), the 5-client
// 3B body 238 K -> 220 K (-7.5 %: its kernel spills the larger chunk)
constexpr uint32_t kv_chunk(uint32_t s) { return kv_gen(s).lin ? 8u : 4u; }
constexpr bool is_ctrl(uint32_t s) { return s == MR_SCN_CTRL_BASIC_4A || s == MR_SCN_CTRL_MULTI_4A; }
// scenarios served by the clerk / server request path (kvraft + shard_ctrler)
constexpr bool is_svc(uint32_t s) { return is_kv(s) || is_ctrl(s); }
constexpr bool is_churn(uint32_t s) {
  return s == MR_SCN_RELIABLE_CHURN_2C || s == MR_SCN_UNRELIABLE_CHURN_2C;
}
// tester thread slots (slot 0 = the test body): kvraft 1 + 5 clients, churn 1 + 3
// clients, unreliable_agree_2c up to 63 concurrent one() tasks
constexpr uint32_t nthr(uint32_t s) {
  return is_kv(s) ? (kv_gen(s).nc + 2u > 6u ? kv_gen(s).nc + 2u : 6u)  // + test body, partitioner
         : is_ctrl(s) ? 11u : is_churn(s) ? 4u
         : s == MR_SCN_UNRELIABLE_AGREE_2C ? 64u : 0u;
}

// step-kernel instances (mr_kernel.hip launch_step_t<S, NB>): per scenario, one
// sized for its default server count (nb_of) and one for up to 8 servers
template <uint32_t S, uint32_t NB>
hipError_t launch_step_t(const Dev& D, uint32_t budget, hipStream_t s);
// the pool kernel of scenario S (has_pool(S, NB); mr_kernel.hip MR_POOL units)
template <uint32_t S, uint32_t NB>
hipError_t launch_pool_t(const Dev& D, uint32_t budget, hipStream_t s);
template <uint32_t S, uint32_t NB>
uint32_t pool_capacity_t(int device, uint32_t M);
// lanes the step kernel of scenario S keeps resident on the device (occupancy x CUs x block)
template <uint32_t S, uint32_t NB>
uint32_t step_capacity_t(int device, uint32_t M);
// the same kernels built with decision-tape draws (MR_TAPE=1 translation units, NB = 8):
// replay and record runs only, so the common draw path carries no tape branch
template <uint32_t S, uint32_t NB>
hipError_t launch_step_tape_t(const Dev& D, uint32_t budget, hipStream_t s);
constexpr uint8_t k_default_n[] = {0, 3, 3, 7, 5, 3, 5, 3, 3, 5, 3, 3, 5, 3, 5,
                                   5, 5, 5, 5, 3, 3, 3, 3, 3, 5, 5, 5, 5, 3, 3,
                                   5, 5, 5, 5, 5, 5, 5, 3, 5, 3, 3, 5, 5, 5, 5, 5, 7, 7};
constexpr uint32_t nb_of(uint32_t s) { return k_default_n[s] <= 5 ? k_default_n[s] : 8u; }
// scenarios with a 7-server instance as well (BASELINE config 4 runs the 2D tests with 7
// servers; arrays sized for 7 keep fewer registers live than the 8-server instance)
constexpr bool has_nb7(uint32_t s) {
  return s >= MR_SCN_SNAPSHOT_BASIC_2D && s <= MR_SCN_SNAPSHOT_INSTALL_UNRELIABLE_CRASH_2D;
}
// exact-size step-kernel instances (NB = n < 8): the node count is a compile-time constant there
// (every `q < n` over the unrolled node loops folds away, and with it the loop-invariant lane
// masks the compiler otherwise keeps in scalar registers); any other n runs the generic 8-server
// instance. Built: each scenario at its default n, BASELINE config 2 (fail_agree_2b at 5
// servers) and config 4 (the 2D tests at 7)
constexpr bool has_exact(uint32_t s, uint32_t n) {
  return n < 8u && (n == k_default_n[s] || (s == MR_SCN_FAIL_AGREE_2B && n == 5u) ||
                    (has_nb7(s) && n == 7u));
}
// pool-kernel instances (mr_kernel.hip pool_kernel): Raft-only test bodies
// without spawned threads at an exact server count of 3, 5 or 7 (512-cluster pools, up to 64
// message slots: the 32-bit keys of slots 0..31 take 64 KiB of LDS, slots 32..63 — 7-server
// bodies, BASELINE config 4 — keep theirs in HBM), and the kvraft / shard_ctrler test bodies at
// their exact server count (256-cluster pools, up to 64 message slots, all keys in LDS; not the
// 20-clerk snapshot_recover_many_clients_3b, whose 256 slots and clerk hosts do not fit)
constexpr bool has_pool(uint32_t s, uint32_t n) {
  return has_exact(s, n) &&
         ((n <= 7u && !is_svc(s) && nthr(s) == 0) ||
          (is_svc(s) && s != MR_SCN_KV_SNAPSHOT_RECOVER_MANY_CLIENTS_3B));
}
constexpr uint32_t pool_max_slots(uint32_t s, uint32_t n) { return is_svc(s) || n > 5u ? 64u : 32u; }
// scenarios whose test body starts the tester with service snapshots (t_new(snapshot = true),
// tester.rs:303-325 SNAPSHOT_INTERVAL): snap_common's five 2D tests. node_apply_coop specializes
// on it at compile time and checks it against the runtime mode (x.netmode bit 1).
constexpr bool uses_service_snapshots(uint32_t s) {
  return s >= MR_SCN_SNAPSHOT_BASIC_2D && s <= MR_SCN_SNAPSHOT_INSTALL_UNRELIABLE_CRASH_2D;
}
// scenarios in which a log can be compacted: the service snapshots of snap_common or a kvraft
// maxraftstate. Everywhere else snap stays 0, so no InstallSnapshot is ever sent (the node
// event compiles that path out of its send loop)
constexpr bool has_snaps(uint32_t s) {
  return uses_service_snapshots(s) || kv_gen(s).maxraft > 0;
}
// test bodies that crash and restart servers (crash1 / start1, tester.rs:293-333): persist1-3,
// figure_8 and its unreliable crash variant, the 2D crash variants, the churn tests
constexpr bool restarts_servers(uint32_t s) {
  return (s >= MR_SCN_PERSIST1_2C && s <= MR_SCN_FIGURE_8_2C) || s == MR_SCN_RELIABLE_CHURN_2C ||
         s == MR_SCN_UNRELIABLE_CHURN_2C || s == MR_SCN_SNAPSHOT_INSTALL_CRASH_2D ||
         s == MR_SCN_SNAPSHOT_INSTALL_UNRELIABLE_CRASH_2D || s == MR_SCN_FIGURE_8_UNRELIABLE_CRASH;
}
#define MR_ALL_SCNS                                                                       \
  MR_INST(1) MR_INST(2) MR_INST(3) MR_INST(4) MR_INST(5) MR_INST(6) MR_INST(7) MR_INST(8) \
  MR_INST(9) MR_INST(10) MR_INST(11) MR_INST(12) MR_INST(13) MR_INST(14) MR_INST(16)      \
  MR_INST(19) MR_INST(20) MR_INST(21) MR_INST(22) MR_INST(23) MR_INST(24) MR_INST(25)     \
  MR_INST(26) MR_INST(27) MR_INST(15) MR_INST(17) MR_INST(18) MR_INST(28) MR_INST(29)     \
  MR_INST(30) MR_INST(31) MR_INST(32) MR_INST(33) MR_INST(34) MR_INST(35) MR_INST(36)     \
  MR_INST(37) MR_INST(38) MR_INST(39) MR_INST(40) MR_INST(41) MR_INST(42) MR_INST(43)     \
  MR_INST(44) MR_INST(45) MR_INST(46) MR_INST(47)

}  // namespace mr
