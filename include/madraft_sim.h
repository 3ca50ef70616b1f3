/*
 * madraft_sim.h — C ABI of the MI355X batched deterministic Raft simulator.
 *
 * This is the drop-in boundary for the reference's hot path: the single-seed
 * MadSim executor + simulated network + Raft node + persister + tester that
 * `MADSIM_TEST_NUM=N cargo test <name>` runs once per seed
 * (/root/reference/README.md:44-66). One `mr_batch` runs `n_clusters`
 * independent seeds of one reference test in lockstep on one GPU.
 *
 * Interfaces replaced (reference file:line):
 *   - `#[madsim::test]` seed loop + MADSIM_TEST_SEED/NUM  (README.md:44-66)
 *       -> mr_batch_create / mr_batch_run / mr_batch_verdicts
 *   - RaftTester::new/one/wait/check_* / end                (src/raft/tester.rs:34-358)
 *       -> scenario programs executed inside mr_batch_run
 *   - RaftHandle::{new,start,term,is_leader,snapshot,cond_install_snapshot}
 *                                                            (src/raft/raft.rs:107-168)
 *       -> device Raft node state machine inside mr_batch_run
 *   - madsim net stat().msg_count, fs get_file_size          (src/raft/tester.rs:147-158)
 *       -> mr_counters, persisted-size model
 *   - panic!(...) + "MADSIM_TEST_SEED=" report               (README.md:44-48)
 *       -> per-cluster fail code (MR_FAIL_*) + fail time; mr_fail_message()
 *
 * Conventions: plain C types, caller-owned buffers, int status (0 = ok,
 * <0 = error, message in mr_last_error()). One mr_batch per device; a batch is
 * not thread-safe. The exact simulation semantics are in docs/SEMANTICS.md.
 */
#ifndef MADRAFT_SIM_H
#define MADRAFT_SIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MR_ABI_VERSION 4u
#define MR_MAX_NODES 8u
#define MR_MAX_MSG_SLOTS 256u
#define MR_MAX_AE 32u

/* ---- scenarios: one id per reference #[madsim::test] (src/raft/tests.rs) ---- */
enum mr_scenario {
  MR_SCN_NONE = 0,
  MR_SCN_INITIAL_ELECTION_2A = 1,        /* tests.rs:20-46   */
  MR_SCN_REELECTION_2A = 2,              /* tests.rs:48-78   */
  MR_SCN_MANY_ELECTION_2A = 3,           /* tests.rs:80-112  */
  MR_SCN_BASIC_AGREE_2B = 4,             /* tests.rs:114-130 */
  MR_SCN_FAIL_AGREE_2B = 5,              /* tests.rs:132-161 */
  MR_SCN_FAIL_NO_AGREE_2B = 6,           /* tests.rs:163-209 */
  MR_SCN_CONCURRENT_STARTS_2B = 7,       /* tests.rs:211-275 */
  MR_SCN_REJOIN_2B = 8,                  /* tests.rs:277-313 */
  MR_SCN_BACKUP_2B = 9,                  /* tests.rs:315-386 */
  MR_SCN_COUNT_2B = 10,                  /* tests.rs:388-479 */
  MR_SCN_PERSIST1_2C = 11,               /* tests.rs:481-526 */
  MR_SCN_PERSIST2_2C = 12,               /* tests.rs:528-572 */
  MR_SCN_PERSIST3_2C = 13,               /* tests.rs:574-602 */
  MR_SCN_FIGURE_8_2C = 14,               /* tests.rs:612-660 */
  MR_SCN_UNRELIABLE_AGREE_2C = 15,       /* tests.rs:662-686 */
  MR_SCN_FIGURE_8_UNRELIABLE_2C = 16,    /* tests.rs:688-741 */
  MR_SCN_RELIABLE_CHURN_2C = 17,         /* tests.rs:743-747 */
  MR_SCN_UNRELIABLE_CHURN_2C = 18,       /* tests.rs:749-753 */
  MR_SCN_SNAPSHOT_BASIC_2D = 19,         /* tests.rs:913-917 */
  MR_SCN_SNAPSHOT_INSTALL_2D = 20,       /* tests.rs:919-923 */
  MR_SCN_SNAPSHOT_INSTALL_UNRELIABLE_2D = 21,       /* tests.rs:925-929 */
  MR_SCN_SNAPSHOT_INSTALL_CRASH_2D = 22,            /* tests.rs:931-935 */
  MR_SCN_SNAPSHOT_INSTALL_UNRELIABLE_CRASH_2D = 23, /* tests.rs:937-941 */
  /* BASELINE.json config 3 read literally: figure_8_unreliable_2c's loop with
   * crash1/start1 (figure_8_2c, tests.rs:638-649) in place of disconnect. */
  MR_SCN_FIGURE_8_UNRELIABLE_CRASH = 24,
  /* kvraft generic_test (src/kvraft/tests.rs:65-220) over 5 servers; BASELINE config 5 */
  MR_SCN_KV_BASIC_3A = 25,               /* kvraft/tests.rs:222-226: 1 client        */
  MR_SCN_KV_CONCURRENT_3A = 26,          /* kvraft/tests.rs:228-232: 5 clients       */
  MR_SCN_KV_UNRELIABLE_3A = 27,          /* kvraft/tests.rs:234-238: 5, unreliable   */
  /* shard_ctrler (src/shard_ctrler/tests.rs) over 3 servers */
  MR_SCN_CTRL_BASIC_4A = 28,             /* shard_ctrler/tests.rs:24-166  */
  MR_SCN_CTRL_MULTI_4A = 29,             /* shard_ctrler/tests.rs:168-299 */
  /* kvraft generic_test with partitions / restarts (src/kvraft/tests.rs:344-385) */
  MR_SCN_KV_MANY_PARTITIONS_ONE_CLIENT_3A = 30,    /* kvraft/tests.rs:344-348 */
  MR_SCN_KV_MANY_PARTITIONS_MANY_CLIENTS_3A = 31,  /* kvraft/tests.rs:350-354 */
  MR_SCN_KV_PERSIST_ONE_CLIENT_3A = 32,            /* kvraft/tests.rs:356-360 */
  MR_SCN_KV_PERSIST_CONCURRENT_3A = 33,            /* kvraft/tests.rs:362-366 */
  MR_SCN_KV_PERSIST_CONCURRENT_UNRELIABLE_3A = 34, /* kvraft/tests.rs:368-372 */
  MR_SCN_KV_PERSIST_PARTITION_3A = 35,             /* kvraft/tests.rs:374-378 */
  MR_SCN_KV_PERSIST_PARTITION_UNRELIABLE_3A = 36,  /* kvraft/tests.rs:380-384 */
  MR_SCN_KV_UNRELIABLE_ONE_KEY_3A = 37,            /* kvraft/tests.rs:240-274 */
  MR_SCN_KV_ONE_PARTITION_3A = 38,                 /* kvraft/tests.rs:276-342 */
  /* kvraft 3B: services snapshot under maxraftstate = 1000 */
  MR_SCN_KV_SNAPSHOT_RPC_3B = 39,                  /* kvraft/tests.rs:396-454 */
  MR_SCN_KV_SNAPSHOT_SIZE_3B = 40,                 /* kvraft/tests.rs:456-492 */
  MR_SCN_KV_SNAPSHOT_RECOVER_3B = 41,              /* kvraft/tests.rs:494-498 */
  MR_SCN_KV_SNAPSHOT_RECOVER_MANY_CLIENTS_3B = 42, /* kvraft/tests.rs:500-504 */
  MR_SCN_KV_SNAPSHOT_UNRELIABLE_3B = 43,           /* kvraft/tests.rs:506-510 */
  MR_SCN_KV_SNAPSHOT_UNRELIABLE_RECOVER_3B = 44,   /* kvraft/tests.rs:512-516 */
  MR_SCN_KV_SNAPSHOT_UNRELIABLE_RECOVER_CONCURRENT_PARTITION_3B = 45, /* kvraft/tests.rs:518-522 */
  /* generic_test_linearizability (15 clients, 7 servers): the reference's commented-out
   * kvraft/tests.rs:386-390 and 524-528, defined by the build (docs/SEMANTICS.md §9b) */
  MR_SCN_KV_PERSIST_PARTITION_UNRELIABLE_LINEARIZABLE_3A = 46,
  MR_SCN_KV_SNAPSHOT_UNRELIABLE_RECOVER_CONCURRENT_PARTITION_LINEARIZABLE_3B = 47,
  MR_SCN_COUNT_
};

/* kvraft scenarios (generic_test and its variants) */
static inline int mr_scn_is_kv(uint32_t s) {
  return (s >= MR_SCN_KV_BASIC_3A && s <= MR_SCN_KV_UNRELIABLE_3A) ||
         (s >= MR_SCN_KV_MANY_PARTITIONS_ONE_CLIENT_3A &&
          s <= MR_SCN_KV_SNAPSHOT_UNRELIABLE_RECOVER_CONCURRENT_PARTITION_LINEARIZABLE_3B);
}
/* default log / apply capacity of a kvraft scenario (no snapshots: every op stays in the log) */
/* generic_test_linearizability scenarios (SEMANTICS §9b) */
static inline int mr_scn_is_lin15(uint32_t s) {
  return s == MR_SCN_KV_PERSIST_PARTITION_UNRELIABLE_LINEARIZABLE_3A ||
         s == MR_SCN_KV_SNAPSHOT_UNRELIABLE_RECOVER_CONCURRENT_PARTITION_LINEARIZABLE_3B;
}
/* scenarios whose clerks keep more than 64 messages in flight: 256 message slots */
static inline int mr_scn_wide_slots(uint32_t s) { return s == MR_SCN_KV_SNAPSHOT_RECOVER_MANY_CLIENTS_3B; }
static inline uint32_t mr_kv_log_cap(uint32_t s) {
  if (s == MR_SCN_KV_SNAPSHOT_RECOVER_MANY_CLIENTS_3B) return 16384u;
  return (s == MR_SCN_KV_BASIC_3A || s == MR_SCN_KV_UNRELIABLE_3A || s >= MR_SCN_KV_UNRELIABLE_ONE_KEY_3A ||
          s == MR_SCN_KV_PERSIST_CONCURRENT_UNRELIABLE_3A || s == MR_SCN_KV_PERSIST_PARTITION_UNRELIABLE_3A ||
          s == MR_SCN_KV_MANY_PARTITIONS_ONE_CLIENT_3A || s == MR_SCN_KV_PERSIST_ONE_CLIENT_3A) ? 2048u : 8192u;
}

/* ---- flags ---- */
#define MR_F_UNRELIABLE 0x1u /* set_unreliable(true) right after RaftTester::new (C2) */
#define MR_F_NULL_RAFT 0x2u  /* skeleton node: never campaigns (as-shipped raft.rs) */
#define MR_F_TRACE 0x4u      /* capture per-event trace for the first trace_clusters */
#define MR_F_SAFETY 0x8u     /* Raft invariant checks at every election (SEMANTICS §11) */
/* Known-buggy Raft variants (SEMANTICS §11), so the checkers can be shown to catch bugs the
 * way the reference tester grades a student's raft.rs */
#define MR_F_BUG_VOTE_TWICE 0x10u /* voters ignore votedFor: two leaders per term possible */
#define MR_F_BUG_VOTE_STALE 0x20u /* voters skip the up-to-date check (Raft §5.4.1) */
#define MR_F_BUG_NO_PREV_CHECK 0x40u /* followers skip AppendEntries' prevLogTerm check (§5.3) */
#define MR_F_RECORD 0x80u    /* record every random decision of each cluster (mr_batch_get_decisions) */
/* Known-buggy kvraft servers (SEMANTICS §9): the linearizability checker must catch them */
#define MR_F_BUG_NO_DEDUP 0x100u   /* servers re-apply a retried Put / Append (no per-clerk dedup) */
#define MR_F_BUG_STALE_READ 0x200u /* a leader answers Get from its local state, not via the log */
#define MR_F_STREAM 0x400u   /* with lanes < n_clusters: a lane whose cluster has its verdict takes
                              * the next unstarted cluster (default: chunks of `lanes` clusters) */
/* Test-only (ABI 4): the tester's apply checker records values but does not compare them
 * (tester.rs:384-388 disabled), so a diverging Raft runs on and the traces' apply digests
 * (mr_trace_digests) are what must catch it */
#define MR_F_BUG_NO_APPLY_CHECK 0x800u

/* ---- verdicts: one code per tester panic site ---- */
enum mr_fail {
  MR_PASS = 0,
  MR_FAIL_ONE_LEADER_NONE = 1,    /* tester.rs:91  "expected one leader, got none" */
  MR_FAIL_MULTI_LEADER_TERM = 2,  /* tester.rs:83  "term {} has {:?} (>1) leaders" */
  MR_FAIL_TERM_DISAGREE = 3,      /* tester.rs:105 "servers disagree on term" */
  MR_FAIL_UNEXPECTED_LEADER = 4,  /* tester.rs:119 "expected no leader, but {} claims..." */
  MR_FAIL_WAIT_TOO_FEW = 5,       /* tester.rs:198 "only {} decided for index {}; wanted {}" */
  MR_FAIL_ONE_NO_AGREEMENT = 6,   /* tester.rs:255,261 "one({:?}) failed to reach agreement" */
  MR_FAIL_TIMEOUT_120S = 7,       /* tester.rs:356 "test took longer than 120 seconds" */
  MR_FAIL_APPLY_MISMATCH = 8,     /* tester.rs:384-388 "commit index=.. server=.. != .." */
  MR_FAIL_APPLY_OUT_OF_ORDER = 9, /* tester.rs:393 "server {} apply out of order {}" */
  MR_FAIL_COMMIT_MISMATCH = 10,   /* tester.rs:411-415 "committed values do not match" */
  MR_FAIL_UNWRAP_NONE = 11,       /* tester.rs:76,101,118,144,166 unwrap() on a crashed raft */
  MR_FAIL_LOG_SIZE = 12,          /* tests.rs:894 "log size too large" */
  MR_FAIL_BASIC_PRECOMMIT = 13,   /* tests.rs:123 "some have committed before start()" */
  MR_FAIL_BASIC_INDEX = 14,       /* tests.rs:126 "got index {} but expected {}" */
  MR_FAIL_LEADER_REJECTED = 15,   /* tests.rs:180,202 "leader rejected start" (expect) */
  MR_FAIL_EXPECTED_INDEX2 = 16,   /* tests.rs:183 "expected index 2, got {}" */
  MR_FAIL_NO_MAJORITY_COMMIT = 17,/* tests.rs:189 "{} committed but no majority" */
  MR_FAIL_UNEXPECTED_INDEX = 18,  /* tests.rs:204 "unexpected index {}" */
  MR_FAIL_CMD_MISSING = 19,       /* tests.rs:266 "cmd {} missing in {:?}" */
  MR_FAIL_TERM_CHANGED = 20,      /* tests.rs:272,468 "term changed too often" */
  MR_FAIL_RPC_INITIAL = 21,       /* tests.rs:397-401 "too many or few RPCs..." */
  MR_FAIL_START_FAILED = 22,      /* tests.rs:434 "start failed" */
  MR_FAIL_WRONG_VALUE = 23,       /* tests.rs:445-452 "wrong value {:?} committed..." */
  MR_FAIL_RPC_TOO_MANY = 24,      /* tests.rs:462 "too many RPCs ({}) for {} entries" */
  MR_FAIL_RPC_IDLE = 25,          /* tests.rs:472-476 "too many RPCs for 1 second of idleness" */
  MR_FAIL_CHURN_VALUE = 26,       /* tests.rs:852 "didn't find a value" */
  MR_FAIL_KV_GET_WRONG = 27,      /* kvraft/tests.rs:127 "get wrong value, key {:?}" */
  MR_FAIL_KV_MISSING = 28,        /* kvraft/tests.rs:25-30 "missing element {:?} in Append result" */
  MR_FAIL_KV_APPEND_BAD = 29,     /* kvraft/tests.rs:31-39 duplicate / wrong order element */
  MR_FAIL_CTRL_NGROUPS = 30,      /* shard_ctrler/tester.rs:117 assert_eq!(c.groups.len(), ..) */
  MR_FAIL_CTRL_MISSING = 31,      /* shard_ctrler/tester.rs:120 "missing group {}" */
  MR_FAIL_CTRL_INVALID = 32,      /* shard_ctrler/tester.rs:125-130 "shard {} -> invalid group {}" */
  MR_FAIL_CTRL_IMBALANCED = 33,   /* shard_ctrler/tester.rs:142-148 "imbalanced sharding" */
  MR_FAIL_CTRL_SERVERS = 34,      /* shard_ctrler/tests.rs:51,53,198-202,210 "wrong servers for gid" */
  MR_FAIL_CTRL_HISTORY = 35,      /* shard_ctrler/tests.rs:70 historical query != config */
  MR_FAIL_CTRL_MOVE_NUM = 36,     /* shard_ctrler/tests.rs:91 "Move should increase Tester.Num" */
  MR_FAIL_CTRL_MOVE_WRONG = 37,   /* shard_ctrler/tests.rs:97 "shard {} wrong group" */
  MR_FAIL_CTRL_MINIMAL_JOIN = 38, /* shard_ctrler/tests.rs:135,251 "non-minimal transfer after Join()s" */
  MR_FAIL_CTRL_MINIMAL_LEAVE = 39,/* shard_ctrler/tests.rs:154,269 "non-minimal transfer after Leave()s" */
  MR_FAIL_CTRL_NO_LEADER = 40,    /* shard_ctrler/tests.rs:282,289 "Leader not found" */
  MR_FAIL_CTRL_SAME_CONFIG = 41,  /* shard_ctrler/tests.rs:294 assert_eq!(c, c1) */
  /* Raft invariants (MR_F_SAFETY; Raft paper Fig. 3), not reference panic sites */
  MR_FAIL_SAFETY_ELECTION = 42,   /* two leaders elected in one term */
  MR_FAIL_SAFETY_COMPLETENESS = 43, /* a new leader lacks a committed (applied) entry */
  MR_FAIL_KV_LOG_SIZE = 44,          /* kvraft/tests.rs:208-215, :422-428, :475-481 */
  MR_FAIL_KV_SNAPSHOT_SIZE = 45,     /* kvraft/tests.rs:483-489 */
  MR_FAIL_KV_MINORITY_PROGRESS = 46, /* kvraft/tests.rs:315-319 */
  MR_FAIL_KV_NO_COMPLETION = 47,     /* kvraft/tests.rs:333-337 */
  MR_FAIL_KV_CHECK = 48,             /* kvraft/tester.rs:266-271 Clerk::check */
  MR_FAIL_SAFETY_LOG_MATCHING = 49,  /* MR_F_SAFETY: same index and term, different command */
  /* the as-shipped service skeleton (MR_F_NULL_RAFT on kvraft / shard_ctrler tests) */
  MR_FAIL_TODO_APPLY = 50,           /* kvraft/server.rs:69 "not yet implemented: apply command" */
  MR_FAIL_TODO_RPC_RESULTS = 51,     /* kvraft/client.rs:59 "not yet implemented: handle RPC results" */
  /* the build's linearizability checker (SEMANTICS §9a; the reference's are commented out,
   * kvraft/tests.rs:386-390,524-528) */
  MR_FAIL_KV_NOT_LINEARIZABLE = 52,  /* a Get's result fits no linearization of the key's history */
  /* simulator limits (not reference panics): a cluster that hits one is reported, never passed */
  MR_FAIL_SIM_CAPACITY = 60,      /* a log / apply / sequence capacity of the config was exceeded */
  MR_FAIL_SIM_EVENT_LIMIT = 61,   /* cfg.max_events processed without a verdict */
  MR_FAIL_SIM_BAD_PROGRAM = 62,   /* scenario program error (interpreter budget, bad op) */
  MR_RUNNING = 0xFFFF             /* verdict not reached yet */
};

typedef struct mr_cfg {
  uint32_t abi_version;   /* = MR_ABI_VERSION */
  uint32_t scenario;      /* enum mr_scenario */
  uint32_t n_nodes;       /* servers, 3..8 (reference default per test if 0) */
  uint32_t flags;         /* MR_F_* */
  uint64_t seed_base;     /* cluster c runs seed  seed_base + cluster_base + c */
  uint64_t cluster_base;  /* global id of this batch's first cluster (multi-GPU shard) */
  uint64_t n_clusters;    /* clusters in this batch */
  uint32_t iters;         /* scenario loop count override (0 = the reference's) */
  uint32_t log_cap;       /* Raft log ring capacity per node, power of two */
  uint32_t apply_cap;     /* apply-checker index capacity per cluster */
  uint32_t msg_slots;     /* max in-flight messages per cluster (<= 64; <= 256 for
                           * snapshot_recover_many_clients_3b); more in flight = MR_FAIL_SIM_CAPACITY */
  uint32_t ae_max;        /* max entries per AppendEntries (<= 32) */
  uint32_t hb_us;         /* leader heartbeat period */
  uint32_t elect_lo_us;   /* election timeout U[lo, hi) (raft.rs:262: 150..300 ms) */
  uint32_t elect_hi_us;
  uint32_t max_events;    /* per-cluster event cap -> MR_FAIL_SIM_EVENT_LIMIT */
  uint32_t trace_clusters;/* with MR_F_TRACE: the first K clusters keep a trace */
  uint32_t trace_cap;     /* trace records per traced cluster */
  int32_t device;         /* HIP device ordinal */
  uint32_t tape_cap;      /* with MR_F_RECORD: decisions kept per cluster */
  uint32_t lanes;         /* clusters in flight per launch (0 = what the GPU keeps resident:
                           * waves / SIMD x SIMDs x 64). A bigger batch runs as consecutive
                           * chunks of `lanes` clusters (or streams them, MR_F_STREAM) instead of
                           * queueing waves behind the resident ones. Results do not depend on it. */
  uint32_t lanes_per_wave;/* lanes of each 64-lane wave that hold a cluster: 64, 32 or 16 (0 = auto:
                           * 32 when the batch fills at most half the resident lanes, so a small
                           * batch still runs two waves per SIMD; else 64). Results do not depend
                           * on it. */
  uint32_t reserved[3];
} mr_cfg;

/* Whole-batch counters (sums over clusters unless named max/first). */
typedef struct mr_counters {
  uint64_t clusters, done, passed, failed;
  uint64_t events, ev_msg, ev_timer, ev_tester;
  uint64_t msgs_sent;      /* every send: madsim stat().msg_count (tester.rs:147-149) */
  uint64_t drop_clog;      /* endpoint disconnected at send */
  uint64_t drop_loss;      /* Bernoulli(packet_loss_rate) */
  uint64_t drop_overflow;  /* a send found msg_slots in flight: the cluster fails MR_FAIL_SIM_CAPACITY */
  uint64_t drop_deliver;   /* endpoint disconnected / crashed at delivery */
  uint64_t drop_stale;     /* RPC reply to a killed incarnation */
  uint64_t elections, leaders_elected, applies, snapshots, installs;
  uint64_t entries_shipped;/* AppendEntries entries read by their receiver (counted at delivery,
                            * past the prevLogIndex/prevLogTerm check; clogged, lost and rejected
                            * appends carry none: payloads are zero-copy until delivery) */
  uint64_t virt_time_us;   /* sum of per-cluster virtual end time */
  uint64_t max_inflight, max_log, max_index;
  uint64_t first_fail_cluster; /* global cluster id (UINT64_MAX if none) */
  uint64_t first_fail_code;
  uint64_t fail_hist[64];  /* verdict histogram by code (index 63 = >= 63) */
  /* coverage histograms over clusters, bucket b = 0 for 0, else min(15, 1 + floor(log2 v)) */
  uint64_t cov_leaders[16]; /* leaders elected per cluster */
  uint64_t cov_events[16];  /* events per cluster */
  /* services (kvraft / shard_ctrler; BASELINE config 5 "linearizability-check counters") */
  uint64_t kv_ops;          /* clerk calls completed */
  uint64_t kv_checked;      /* Get results the tester verified against their linearizable value */
  /* ABI 3 */
  uint64_t log_writes;      /* log entries written (leader start() appends + follower appends) */
  uint64_t entries_materialized; /* zero-copy payload entries copied before their log slot was
                                  * overwritten (HIP path only; the oracle copies at send) */
  uint64_t kv_lin_checked;  /* Get results the linearizability checker verified (SEMANTICS §9a) */
  /* ABI 4 */
  uint64_t coop_entries;    /* HIP path only: AppendEntries entries a receiver's wave wrote for it
                             * (the cooperative receive of the 7- / 8-server step kernels) */
} mr_counters;

typedef struct mr_run_stats {
  uint64_t launches;       /* step-kernel launches */
  double kernel_ms;        /* summed step-kernel time (HIP events, batch stream) */
  double wall_ms;          /* host wall time of mr_batch_run */
  uint64_t events;         /* events processed in this call */
  uint64_t remaining;      /* clusters without verdict after the call */
} mr_run_stats;

/* One trace record per processed event (32 B); docs/SEMANTICS.md §Trace. */
typedef struct mr_event {
  uint32_t time_us;
  uint8_t cls;     /* 0 message, 1 node timer, 2 tester, 3 verdict */
  uint8_t kind;    /* message type / drop reason / fail code */
  uint8_t node;    /* destination or timer node (0xFF for tester) */
  uint8_t role;    /* node role after the event (0 F, 1 C, 2 L, 3 down) */
  uint32_t aux;    /* message seq / msgs_sent for tester events */
  uint32_t term, commit, applied, last, snap;
} mr_event;

typedef struct mr_batch mr_batch;

const char* mr_last_error(void);
const char* mr_fail_message(uint32_t code);
const char* mr_scenario_name(uint32_t scenario);
/* Name as in tests.rs (e.g. "figure_8_unreliable_2c") -> id; 0 if unknown. */
uint32_t mr_scenario_from_name(const char* name);
/* Fill cfg with the reference's defaults for `scenario`. */
int mr_cfg_init(mr_cfg* cfg, uint32_t scenario);

int mr_batch_create(const mr_cfg* cfg, mr_batch** out);
/* Re-seed and reset every cluster to RaftTester::new state (device-side). */
int mr_batch_reset(mr_batch* b, uint64_t seed_base);
/* Run until every cluster has a verdict or max_events_per_call events per
 * cluster were processed in this call (0 = no per-call bound). */
int mr_batch_run(mr_batch* b, uint64_t max_events_per_call, mr_run_stats* st);
/* Pipelined steps (the benchmark's double-buffered batches): mr_batch_submit enqueues
 * mr_batch_reset(seed_base) and the first step-kernel launch on the batch's own stream and
 * returns at once; mr_batch_finish waits for them, runs any clusters left past the per-launch
 * budget to their verdict, and returns the run stats and (cnt != NULL) the counters.
 * A second batch's step submitted meanwhile fills the CUs this batch's finished waves free.
 * Results are those of mr_batch_reset + mr_batch_run. */
int mr_batch_submit(mr_batch* b, uint64_t seed_base);
int mr_batch_finish(mr_batch* b, mr_run_stats* st, mr_counters* cnt);
/* Per-cluster verdict code, fail/end time (virtual us) and trace digest. */
int mr_batch_verdicts(mr_batch* b, uint16_t* code, uint32_t* time_us, uint64_t* digest);
int mr_batch_counters(mr_batch* b, mr_counters* out);
/* Trace of traced cluster `k` (k < trace_clusters). *n = records written. */
int mr_trace_get(mr_batch* b, uint32_t k, mr_event* out, size_t cap, size_t* n);
/* ABI 4: the apply-digest term of log entry i with command value v (splitmix64's finalizer of
 * v ^ i * golden ratio); the kernels compute the same in device code */
static inline uint64_t mr_apply_mix(uint32_t i, uint64_t v) {
  uint64_t z = v ^ ((uint64_t)i * 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
/* ABI 4: the apply digest of each of those records (docs/SEMANTICS.md §7): for a node event,
 * the sum mod 2^64 of mr_apply_mix(i, value_i) over the entries i = 1..applied the node applied
 * one by one; UINT64_MAX once it installed a snapshot or restarted above index 0; 0 for other
 * records. Equal applied indices with different digests = state-machine safety broken by
 * value, checkable from the trace alone (tests/test_trace_properties.py). */
int mr_trace_digests(mr_batch* b, uint32_t k, uint64_t* out, size_t cap, size_t* n);
/* ABI 4: the key-value commands of traced cluster k as the service applied them (kvraft
 * scenarios; zero rows elsewhere): out[2 i] = log entry i's command (SEMANTICS §9 layout), out[2 i
 * + 1] = the hash of its key's value right after the first server to apply entry i applied it
 * (a Get: the hash it answers). Rows i < min(cap, trace_cap); *n = 1 + the highest index
 * recorded. The log by value and the servers' state machine, checkable against a replay of
 * the real strings (tests/test_kv_trace.py). */
int mr_trace_applies(mr_batch* b, uint32_t k, uint64_t* out, size_t cap, size_t* n);
/* ABI 4: the kernel the batch's launches run: "pool_kernel", "step_kernel" or
 * "step_kernel_tape" (keyed decisions set or recorded) */
const char* mr_batch_kernel(const mr_batch* b);
void mr_batch_destroy(mr_batch* b);

/* ---- keyed decision traces and replay (docs/SEMANTICS.md §12) ----
 * Every random choice of a cluster is one decision, keyed by WHO makes it, not by when:
 *   stream MR_DS_NET    entity = sending host (server i, clerk 8 + k), seq = that host's
 *                       send index -> w0 < loss_q32 drops the message, w1 picks its latency
 *                       (madsim net send: drop + latency, tester.rs:127-137);
 *   stream MR_DS_ELECT  entity = server, seq = its timeout index -> w0 picks the election
 *                       timeout (raft.rs:260-263, U[150, 300) ms);
 *   stream MR_DS_TESTER entity = tester thread (0 = the test body), seq = its draw index ->
 *                       (w0, w1) is the rand::rng() value (tests.rs gen_range / gen_bool /
 *                       gen_entry as SEMANTICS §2 maps it).
 * A range choice v in [lo, hi) is the word mr_decision_word(v, lo, hi). A trace is a set:
 * any order, any subset; a draw whose key is absent takes the seed's own Philox draw and
 * counts as a miss. A recorder of another simulator's run (a MadSim seed) emits these
 * records and mr_replay plays them. */
enum mr_decision_stream { MR_DS_TESTER = 1, MR_DS_ELECT = 2, MR_DS_NET = 3 };
typedef struct mr_decision {
  uint32_t cluster; /* batch-relative cluster (mr_replay: ignored) */
  uint16_t stream;  /* enum mr_decision_stream */
  uint16_t entity;
  uint32_t seq;
  uint32_t w0, w1;
} mr_decision;
/* The smallest draw word w with lo + floor(w * (hi - lo) / 2^32) == v (lo <= v < hi). */
uint32_t mr_decision_word(uint32_t v, uint32_t lo, uint32_t hi);
/* Drive the batch's clusters by `d` (n records, any order; duplicate keys are an error);
 * n = 0 = Philox again. Call after create / reset and before run. */
int mr_batch_set_decisions(mr_batch* b, const mr_decision* d, size_t n);
/* Cluster k: with MR_F_RECORD its decisions so far in draw order (*n = decisions drawn, up to
 * cap copied); with decisions set, *n = its draws that found no record (misses). */
int mr_batch_get_decisions(mr_batch* b, uint32_t k, mr_decision* out, size_t cap, size_t* n);
/* One cluster of cfg (cluster_base selects the seed for misses) driven by the n decisions:
 * its per-event trace (per-node term / role / commit / applied / last / snapshot after every
 * event), its verdict and verdict time, and (misses != NULL) its draws not in `d`. */
int mr_replay(const mr_cfg* cfg, const mr_decision* d, size_t n, mr_event* out, size_t cap,
              size_t* n_out, uint16_t* code, uint32_t* time_us, uint64_t* misses);

#ifdef __cplusplus
}
#endif
#endif /* MADRAFT_SIM_H */
