/*
 * mr_oracle.h — CPU oracle for the batched Raft simulator.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product
 * (madraft_amd/, libmadraft_hip.so) never links or calls it.
 *
 * A scalar, one-cluster-at-a-time discrete-event restatement of the
 * reference's hot path, shaped like a madsim run: a binary heap of timers
 * and in-flight messages (madsim executor + net), the
 * Raft node of docs/SEMANTICS.md §5, and the tester/scenario code of
 * src/raft/tester.rs + src/raft/tests.rs restated as straight-line C whose
 * panics longjmp out (the #[madsim::test] seed loop, README.md:44-66).
 *
 * Parity status: MadSim RNG-stream / scheduler parity is UNPINNED (madsim
 * is not vendored, the reference Raft is todo!()). What pins
 * this oracle: Philox4x32-10 known-answer vectors, the skeleton-verdict KATs
 * (null node -> tester.rs:91 / tester.rs:261 panics) and the reference
 * tests' own assertions (tests/test_oracle_kat.py).
 */
#ifndef MR_ORACLE_H
#define MR_ORACLE_H
#include "../include/madraft_sim.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mro_result {
  uint32_t code;     /* enum mr_fail */
  uint32_t time_us;  /* virtual time of the verdict */
  uint64_t digest;   /* FNV-1a-64 over the trace records */
  uint64_t events, ev_msg, ev_timer, ev_tester;
  uint64_t msgs_sent, drop_clog, drop_loss, drop_overflow, drop_deliver, drop_stale;
  uint64_t elections, leaders_elected, applies, snapshots, installs, entries_shipped;
  uint64_t max_inflight, max_log, max_index;
  uint64_t kv_ops;      /* service clerk calls completed (kvraft / shard_ctrler) */
  uint64_t kv_checked;  /* Get results the tester verified against their linearizable value */
  uint64_t log_writes;  /* log entries written (leader appends + follower appends) */
  uint64_t kv_lin_checked; /* Gets the linearizability checker verified (SEMANTICS §9a) */
} mro_result;

/* Run cluster `cluster` (global id) of cfg; trace (optional) receives up to
 * trace_cap records, *n_trace the number written. Returns 0 or <0 on a bad cfg. */
int mro_run_cluster(const mr_cfg* cfg, uint64_t cluster, mro_result* out,
                    mr_event* trace, size_t trace_cap, size_t* n_trace);
/* The same, with tdig[trace_cap] (optional) receiving each record's apply digest (ABI 4
 * mr_trace_digests). */
int mro_run_cluster_dig(const mr_cfg* cfg, uint64_t cluster, mro_result* out, mr_event* trace,
                        uint64_t* tdig, size_t trace_cap, size_t* n_trace);
/* ... and tapp[trace_cap][2] (optional) receiving the KV commands as applied (ABI 4
 * mr_trace_applies). */
int mro_run_cluster_kv(const mr_cfg* cfg, uint64_t cluster, mro_result* out, mr_event* trace,
                       uint64_t* tdig, uint64_t* tapp, size_t trace_cap, size_t* n_trace);

/* Run clusters [first, first+count) and fill per-cluster arrays (any may be NULL). */
int mro_run_batch(const mr_cfg* cfg, uint64_t first, uint64_t count,
                  uint16_t* code, uint32_t* time_us, uint64_t* digest,
                  mro_result* sum);

/* Keyed decisions (SEMANTICS §12) for the following runs, rows = cluster - cfg.cluster_base:
 * mode 1 replays the n decisions `d` (any order; rows >= every d.cluster + 1), count[row] =
 * draws without a record; mode 2 records every draw into rec[row * rec_cap ..] in draw order,
 * count[row] = draws; mode 0 = off. Returns <0 on a bad / duplicate record. Not thread-safe. */
int mro_set_decisions(int mode, const mr_decision* d, uint64_t n, uint64_t rows,
                      mr_decision* rec, uint64_t rec_cap, uint64_t* count);

/* Philox4x32-10 block (exported for the known-answer test). */
void mro_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

int mro_cfg_init(mr_cfg* cfg, uint32_t scenario);
uint32_t mro_scenario_from_name(const char* name);
const char* mro_fail_message(uint32_t code);

#ifdef __cplusplus
}
#endif
#endif
