// mr_host.cpp — C ABI of include/madraft_sim.h on one MI355X: allocates the
// cluster-minor SoA of mr_dev.h in HBM (sized for the config, hundreds of
// GB fit on a 288 GB part), and drives the step kernel in bounded launches
// on the batch's own HIP stream, timing each launch with HIP events on that
// stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mr_dev.h"

namespace mr {
// the step-kernel instance of scenario S for D.n servers: the exact-size one where it is built
// (mr_dev.h has_exact), else the generic 8-server one
template <uint32_t S>
static hipError_t launch_any(const Dev& D, uint32_t budget, hipStream_t s) {
#if MR_NO_TAPE  // a debug library without decision-tape kernels (build.build_guard)
  if (D.tape_mode) return hipErrorInvalidValue;
#else
  if (D.tape_mode) return launch_step_tape_t<S, MR_MAX_NODES>(D, budget, s);
#endif
  if (D.pool) {  // the pool kernel (mr_dev.h has_pool; the host sets D.pool only where it exists)
    if constexpr (has_pool(S, 3)) if (D.n == 3) return launch_pool_t<S, 3>(D, budget, s);
    if constexpr (has_pool(S, 5)) if (D.n == 5) return launch_pool_t<S, 5>(D, budget, s);
    if constexpr (has_pool(S, 7)) if (D.n == 7) return launch_pool_t<S, 7>(D, budget, s);
    return hipErrorInvalidValue;
  }
  if constexpr (has_exact(S, 3)) if (D.n == 3) return launch_step_t<S, 3>(D, budget, s);
  if constexpr (has_exact(S, 5)) if (D.n == 5) return launch_step_t<S, 5>(D, budget, s);
  if constexpr (has_exact(S, 7)) if (D.n == 7) return launch_step_t<S, 7>(D, budget, s);
  return launch_step_t<S, MR_MAX_NODES>(D, budget, s);
}
template <uint32_t S>
static uint32_t capacity_any(const Dev& D, int device) {
  if (D.pool) {
    if constexpr (has_pool(S, 3)) if (D.n == 3) return pool_capacity_t<S, 3>(device, D.M);
    if constexpr (has_pool(S, 5)) if (D.n == 5) return pool_capacity_t<S, 5>(device, D.M);
    if constexpr (has_pool(S, 7)) if (D.n == 7) return pool_capacity_t<S, 7>(device, D.M);
    return 0;
  }
  if constexpr (has_exact(S, 3)) if (D.n == 3) return step_capacity_t<S, 3>(device, D.M);
  if constexpr (has_exact(S, 5)) if (D.n == 5) return step_capacity_t<S, 5>(device, D.M);
  if constexpr (has_exact(S, 7)) if (D.n == 7) return step_capacity_t<S, 7>(device, D.M);
  return step_capacity_t<S, MR_MAX_NODES>(device, D.M);
}
// the step-kernel instance of scenario `scn` (instances: MR_ALL_SCNS)
hipError_t launch_step(const Dev& D, uint32_t scn, uint32_t budget, hipStream_t s) {
  switch (scn) {
#define MR_INST(S) \
  case S: return launch_any<S>(D, budget, s);
#ifdef MR_DEV_SCNS  // dev variants built for a few scenarios (build.py scns=)
    MR_DEV_SCNS
#else
    MR_ALL_SCNS
#endif
#undef MR_INST
    default: return hipErrorInvalidValue;
  }
}
// clusters the scenario's step kernel keeps resident (0: unknown)
static uint32_t step_capacity(const Dev& D, uint32_t scn, int device) {
  switch (scn) {
#define MR_INST(S) \
  case S: return capacity_any<S>(D, device);
#ifdef MR_DEV_SCNS
    MR_DEV_SCNS
#else
    MR_ALL_SCNS
#endif
#undef MR_INST
    default: return 0;
  }
}
// the pool kernel serves this batch: an instance exists, the key rows fit (pool_max_slots), and the
// environment does not turn it off (MR_POOL=0: the per-lane step kernel, for A/B runs)
static bool use_pool(uint32_t scn, uint32_t n, uint32_t M) {
  if (const char* e = std::getenv("MR_POOL")) if (e[0] == '0') return false;
  switch (scn) {
#define MR_INST(S) \
  case S: return has_pool(S, n) && M <= pool_max_slots(S, n);
#ifdef MR_DEV_SCNS
    MR_DEV_SCNS
#else
    MR_ALL_SCNS
#endif
#undef MR_INST
    default: return false;
  }
}
hipError_t launch_reset(const Dev& D, hipStream_t s);
hipError_t launch_reduce(const Dev& D, unsigned long long* out, uint64_t cluster_base,
                         hipStream_t s);
}  // namespace mr

using namespace mr;

namespace {
thread_local std::string g_err;

int set_err(const std::string& s) {
  g_err = s;
  return -1;
}
#define HIPCHK(expr)                                                                  \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return set_err(std::string(#expr) + ": " + hipGetErrorString(e_));              \
  } while (0)

const char* k_names[MR_SCN_COUNT_] = {
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
// servers per test (tests.rs `let servers = ..`)
const uint8_t k_nodes[MR_SCN_COUNT_] = {0, 3, 3, 7, 5, 3, 5, 3, 3, 5, 3, 3, 5, 3,
                                        5, 5, 5, 5, 5, 3, 3, 3, 3, 3, 5, 5, 5, 5, 3, 3,
                                        5, 5, 5, 5, 5, 5, 5, 3, 5, 3, 3, 5, 5, 5, 5, 5, 7, 7};

constexpr size_t RED_N = CNT__N + 8 + 64 + 32 + 3;  // reduce_kernel output slots
constexpr uint32_t STEP_LANES = 64;  // lanes per step-kernel block (one wave)
}  // namespace

struct mr_batch {
  mr_cfg cfg;
  Dev D;
  void* base = nullptr;
  size_t bytes = 0;
  unsigned long long* red = nullptr;
  uint32_t* h_remaining = nullptr;  // [2]: remaining, next unclaimed cluster (D.remaining)
  uint32_t* h_ctl0 = nullptr;       // [2]: {0, L}, copied to D.remaining before each launch
  uint32_t c_open = 0;              // first cluster of the first chunk not yet finished
  uint32_t* held[2] = {nullptr, nullptr};  // streaming: clusters held at a launch's end (ping-pong)
  uint32_t hsel = 0;                // held[hsel] = the next launch's held_in
  bool resume = false;              // streaming: the next launch continues the current chunk
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  uint32_t budget = 16384;  // events per cluster per launch (MR_STEP_BUDGET)
  uint4* tape = nullptr;     // keyed decisions (own allocation: set_decisions / MR_F_RECORD)
  uint32_t* doff = nullptr;  // replay: CSR row offsets of `tape` (set_decisions)
  bool submitted = false;    // mr_batch_submit enqueued a step not yet finished
  uint32_t kern = 0;         // kernel family of the launches since the reset: 1 pool, 2 step / tape
  std::chrono::steady_clock::time_point t_submit;
};

extern "C" {

const char* mr_last_error(void) { return g_err.c_str(); }

const char* mr_scenario_name(uint32_t s) { return (s > 0 && s < MR_SCN_COUNT_) ? k_names[s] : ""; }

uint32_t mr_scenario_from_name(const char* name) {
  if (!name) return 0;
  for (uint32_t i = 1; i < MR_SCN_COUNT_; i++)
    if (std::strcmp(name, k_names[i]) == 0) return i;
  return 0;
}

const char* mr_fail_message(uint32_t code) {
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
    case MR_FAIL_COMMIT_MISMATCH: return "committed values do not match";
    case MR_FAIL_UNWRAP_NONE: return "called `Option::unwrap()` on a `None` value";
    case MR_FAIL_LOG_SIZE: return "log size too large";
    case MR_FAIL_BASIC_PRECOMMIT: return "some have committed before start()";
    case MR_FAIL_BASIC_INDEX: return "got index but expected another";
    case MR_FAIL_LEADER_REJECTED: return "leader rejected start";
    case MR_FAIL_EXPECTED_INDEX2: return "expected index 2";
    case MR_FAIL_NO_MAJORITY_COMMIT: return "committed but no majority";
    case MR_FAIL_UNEXPECTED_INDEX: return "unexpected index";
    case MR_FAIL_CMD_MISSING: return "cmd missing";
    case MR_FAIL_TERM_CHANGED: return "term changed too often";
    case MR_FAIL_RPC_INITIAL: return "too many or few RPCs to elect initial leader";
    case MR_FAIL_START_FAILED: return "start failed";
    case MR_FAIL_WRONG_VALUE: return "wrong value committed";
    case MR_FAIL_RPC_TOO_MANY: return "too many RPCs for entries";
    case MR_FAIL_RPC_IDLE: return "too many RPCs for 1 second of idleness";
    case MR_FAIL_CHURN_VALUE: return "didn't find a value";
    case MR_FAIL_KV_GET_WRONG: return "get wrong value";
    case MR_FAIL_KV_MISSING: return "missing element in Append result";
    case MR_FAIL_KV_APPEND_BAD: return "duplicate or wrong order element in Append result";
    case MR_FAIL_CTRL_NGROUPS: return "assertion failed: c.groups.len() == groups.len()";
    case MR_FAIL_CTRL_MISSING: return "missing group";
    case MR_FAIL_CTRL_INVALID: return "shard -> invalid group";
    case MR_FAIL_CTRL_IMBALANCED: return "imbalanced sharding";
    case MR_FAIL_CTRL_SERVERS: return "wrong servers for gid";
    case MR_FAIL_CTRL_HISTORY: return "historical query differs";
    case MR_FAIL_CTRL_MOVE_NUM: return "Move should increase Tester.Num";
    case MR_FAIL_CTRL_MOVE_WRONG: return "shard wrong group";
    case MR_FAIL_CTRL_MINIMAL_JOIN: return "non-minimal transfer after Join()s";
    case MR_FAIL_CTRL_MINIMAL_LEAVE: return "non-minimal transfer after Leave()s";
    case MR_FAIL_CTRL_NO_LEADER: return "Leader not found";
    case MR_FAIL_CTRL_SAME_CONFIG: return "config differs after leader shutdown";
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
    case MR_FAIL_SIM_BAD_PROGRAM: return "scenario program error";
    case MR_RUNNING: return "running";
    default: return "unknown";
  }
}

int mr_cfg_init(mr_cfg* c, uint32_t scn) {
  if (!c) return set_err("null cfg");
  if (scn == 0 || scn >= MR_SCN_COUNT_) return set_err("unknown scenario");
  std::memset(c, 0, sizeof *c);
  c->abi_version = MR_ABI_VERSION;
  c->scenario = scn;
  c->n_nodes = k_nodes[scn];
  c->seed_base = 1629626496ull;  // README.md:48
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
  /* in-flight maxima over 64K / 1K seeds: 20 (figure_8), <= 45 (7 / 8 servers,
   * kvraft), 229 (20 clerks); a send past msg_slots fails the cluster (MR_FAIL_SIM_CAPACITY) */
  c->msg_slots = mr_scn_wide_slots(scn) ? 256 : kv ? 64 : 32;
  c->ae_max = 16;
  c->hb_us = 50000;
  c->elect_lo_us = 150000;  // raft.rs:262
  c->elect_hi_us = 300000;
  c->max_events = 4u << 20;
  c->trace_cap = 1u << 16;
  return 0;
}

static int validate(const mr_cfg* c) {
  if (!c) return set_err("null cfg");
  if (c->abi_version != MR_ABI_VERSION) return set_err("abi_version mismatch");
  if (c->scenario == 0 || c->scenario >= MR_SCN_COUNT_) return set_err("unknown scenario");
  if (c->n_nodes < 3 || c->n_nodes > MR_MAX_NODES) return set_err("n_nodes must be 3..8");
  if (c->n_clusters == 0 || c->n_clusters > (1ull << 31)) return set_err("bad n_clusters");
  if (c->log_cap < 16 || (c->log_cap & (c->log_cap - 1))) return set_err("log_cap: power of 2 >= 16");
  if (c->apply_cap < 16) return set_err("apply_cap too small");
  if (c->msg_slots < 1 || c->msg_slots > MR_MAX_MSG_SLOTS ||
      (c->msg_slots > 64 && !mr_scn_wide_slots(c->scenario)))
    return set_err("msg_slots must be 1..64 (1..256 for snapshot_recover_many_clients_3b)");
  if (c->ae_max < 1 || c->ae_max > MR_MAX_AE) return set_err("ae_max must be 1..32");
  if (c->elect_hi_us <= c->elect_lo_us || c->hb_us == 0) return set_err("bad timers");
  if (c->max_events == 0) return set_err("max_events must be > 0");
  if ((c->flags & MR_F_TRACE) && (c->trace_cap == 0 || c->trace_clusters > c->n_clusters))
    return set_err("bad trace config");
  if (c->lanes_per_wave != 0 && c->lanes_per_wave != 16 && c->lanes_per_wave != 32 &&
      c->lanes_per_wave != 64)
    return set_err("lanes_per_wave must be 0 (auto), 16, 32 or 64");
  if ((c->flags & MR_F_RECORD) && c->tape_cap < 1)
    return set_err("MR_F_RECORD needs tape_cap >= 1 (decisions kept per cluster)");
  return 0;
}

static int mr_batch_create_impl(const mr_cfg* cfg, mr_batch** out) {
  if (!out) return set_err("null out");
  *out = nullptr;
  if (validate(cfg) != 0) return -1;
  const uint32_t scn = cfg->scenario;

  mr_batch* b = new mr_batch();
  b->cfg = *cfg;
  Dev& D = b->D;
  std::memset(&D, 0, sizeof D);
  const uint64_t C = cfg->n_clusters, n = cfg->n_nodes, M = cfg->msg_slots, K = cfg->ae_max;
  D.C = (uint32_t)C;
  D.L = cfg->lanes && cfg->lanes < C ? cfg->lanes : (uint32_t)C;  // no tape: capacity (below)
  D.stream = (cfg->flags & MR_F_STREAM) ? 1u : 0u;
  D.n = (uint32_t)n; D.log_cap = cfg->log_cap; D.apply_cap = cfg->apply_cap;
  D.M = (uint32_t)M; D.K = (uint32_t)K; D.hb = cfg->hb_us; D.elo = cfg->elect_lo_us;
  D.ehi = cfg->elect_hi_us; D.max_events = cfg->max_events;
  D.null_raft = (cfg->flags & MR_F_NULL_RAFT) ? 1u : 0u;
  D.unrel_flag = (cfg->flags & MR_F_UNRELIABLE) ? 1u : 0u;
  D.safety = (cfg->flags & MR_F_SAFETY) ? 1u : 0u;
  D.bugs = cfg->flags & (MR_F_BUG_VOTE_TWICE | MR_F_BUG_VOTE_STALE | MR_F_BUG_NO_PREV_CHECK |
                         MR_F_BUG_NO_DEDUP | MR_F_BUG_STALE_READ | MR_F_BUG_NO_APPLY_CHECK);
  D.links = kv_gen(cfg->scenario).part ? 1u : 0u;  // server-link cuts (CS_CUT) can exist
  D.lin15 = mr_scn_is_lin15(scn) ? 1u : 0u;  // generic_test_linearizability layout (SEMANTICS §9b)
  D.trace_clusters = (cfg->flags & MR_F_TRACE) ? cfg->trace_clusters : 0u;
  D.trace_cap = cfg->trace_cap;
  D.scenario = scn;
  // loop counts of the test bodies (tests.rs): many_election 10, figure_8 1000, snap_common 30
  uint32_t def_iters = scn == MR_SCN_MANY_ELECTION_2A ? 10 : (scn >= MR_SCN_SNAPSHOT_BASIC_2D &&
                       scn <= MR_SCN_SNAPSHOT_INSTALL_UNRELIABLE_CRASH_2D) ? 30 : 1000;
  D.iters = cfg->iters ? cfg->iters : def_iters;
  D.seed0 = cfg->seed_base + cfg->cluster_base;
  D.pool = !(cfg->flags & MR_F_RECORD) && use_pool(scn, (uint32_t)n, (uint32_t)M) ? 1u : 0u;

  // carve one allocation; every array 256-B aligned
  struct Item { void** p; size_t bytes; };
  std::vector<Item> items;
  auto add = [&](auto** p, size_t count) {
    items.push_back({reinterpret_cast<void**>(p), count * sizeof(**p)});
  };
  // field matrices use 32-bit element offsets in the kernels
  const uint64_t lim = 1ull << 32;
  if ((uint64_t)CS_STRIDE * C >= lim || (uint64_t)C64_STRIDE * C >= lim || M * C >= lim) {
    delete b;
    return set_err("n_clusters too large for one batch (32-bit field offsets)");
  }
  add(&D.cs32, (size_t)CS_STRIDE * C);
  add(&D.cs64, (size_t)C64_STRIDE * C);
  add(&D.nd32, (size_t)NREC * n * C);
  add(&D.tmr, n * C);
  add(&D.ms32, (size_t)MREC * M * C);
  add(&D.mkey, (size_t)M * C);
  add(&D.log, C * n * cfg->log_cap);
  add(&D.pay, C * M * K);
  add(&D.stor, C * cfg->apply_cap);
  // scenario-only arrays: spawned tester threads, kvraft servers, churn values
  D.nthr = nthr(scn);
  if (D.nthr) add(&D.kt32, (size_t)KT_STRIDE * D.nthr * C);
  if (D.nthr) add(&D.kwk, (size_t)2 * kws(D.nthr) * C);
  if (is_svc(scn)) add(&D.kv32, (size_t)KVREC * n * C);
  if (is_kv(scn)) add(&D.lin32, (size_t)KV_KEYS * KV_APP * LINW * C);
  if (kv_gen(scn).maxraft) {
    add(&D.kvs32, (size_t)KVS_W * n * C);
    add(&D.kring, (size_t)KRW * KV_RING * C);
  }
  if (is_ctrl(scn)) {
    add(&D.cfg32, (size_t)CFG_CAP * CFGW * n * C);
    add(&D.op32, (size_t)OP_CAP * OPW * C);
  }
  if (is_churn(scn)) {
    add(&D.cval, (size_t)3 * CHURN_VCAP * C);
    add(&D.cidx, (size_t)3 * CHURN_VCAP * C);
  }
  if (D.safety) add(&D.led, (size_t)LED_W * C);
  add(&D.trace, (size_t)D.trace_clusters * D.trace_cap);
  add(&D.tdig, (size_t)D.trace_clusters * D.trace_cap);       // apply digests (ABI 4)
  add(&D.tapp, (size_t)D.trace_clusters * D.trace_cap * 2u);  // KV applies (ABI 4)
  add(&D.adig, (size_t)D.trace_clusters * MR_MAX_NODES * 2u);
  add(&D.remaining, 2);
  add(&D.prof, PROF_SLOTS);
  add(&D.guard, 4);
  add(&D.pcnt, CNT__N);
  add(&D.tfr, (size_t)TF_Q * C);
  size_t total = 0;
  for (auto& it : items) total += (it.bytes + 255) & ~size_t(255);

  hipError_t e = hipSetDevice(cfg->device);
  if (e == hipSuccess) e = hipMalloc(&b->base, total);
  if (e == hipSuccess) e = hipMalloc(&b->red, RED_N * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipHostMalloc(&b->h_remaining, 2 * sizeof(uint32_t));
  if (e == hipSuccess) e = hipHostMalloc(&b->h_ctl0, 2 * sizeof(uint32_t));
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&b->ev0);
  if (e == hipSuccess) e = hipEventCreate(&b->ev1);
  if (e != hipSuccess) {
    std::string msg = std::string("allocation of ") + std::to_string(total) + " B failed: " +
                      hipGetErrorString(e);
    mr_batch_destroy(b);
    return set_err(msg);
  }
  b->bytes = total;
  char* p = static_cast<char*>(b->base);
  for (auto& it : items) {
    *it.p = it.bytes ? p : nullptr;
    p += (it.bytes + 255) & ~size_t(255);
  }
  if (cfg->flags & MR_F_RECORD) {
    e = hipMalloc(&b->tape, (size_t)C * cfg->tape_cap * sizeof(uint4));
    if (e != hipSuccess) {
      mr_batch_destroy(b);
      return set_err(std::string("tape allocation failed: ") + hipGetErrorString(e));
    }
    b->D.dtab = b->tape;
    b->D.dcap = cfg->tape_cap;
    b->D.tape_mode = 2;
  }
  if (hipMemset(b->D.prof, 0, PROF_SLOTS * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(b->D.guard, 0, 4 * sizeof(uint32_t)) != hipSuccess) {
    mr_batch_destroy(b);
    return set_err("hipMemset failed");
  }
  // lanes per wave: as configured, else 32 when the batch (or its chunk) fills at most half of
  // the resident lanes — two half-full waves per SIMD hide the latency chains better than one
  // full one — else 64
  const uint32_t cap = step_capacity(b->D, scn, cfg->device);  // resident lanes (64 per wave)
  b->D.lpw = cfg->lanes_per_wave ? cfg->lanes_per_wave
             : (cap && (uint64_t)(cfg->lanes && cfg->lanes < C ? cfg->lanes : C) * 2u <= cap) ? 32u : 64u;
  if (!cfg->lanes) {  // a batch bigger than the resident waves runs as chunks of that size
    const uint32_t capc = (uint32_t)((uint64_t)cap * b->D.lpw / STEP_LANES);
    if (capc && capc < b->D.C) {
      b->D.L = capc;
      // a pool kernel refills its slots from the rest of the batch (streaming) instead of
      // draining once per chunk (config 3's whole job on one GPU +10 %)
      if (b->D.pool && !b->D.tape_mode) b->D.stream = 1u;
    }
  }
  if (b->D.stream) {  // held-cluster lists, L entries each (L <= C)
    e = hipMalloc(&b->held[0], (size_t)b->D.C * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&b->held[1], (size_t)b->D.C * sizeof(uint32_t));
    if (e != hipSuccess) {
      mr_batch_destroy(b);
      return set_err(std::string("held-list allocation failed: ") + hipGetErrorString(e));
    }
  }
  // the 7-server Raft pool's LDS key rows (32); MR_KEY_ROWS (tests) puts more slots' keys in HBM
  b->D.krows = 32u;
  if (const char* s = std::getenv("MR_KEY_ROWS")) {
    const int r = std::atoi(s);
    if (r >= 1 && r <= 32) b->D.krows = (uint32_t)r;
  }
  if (const char* s = std::getenv("MR_STEP_BUDGET")) b->budget = (uint32_t)std::atoi(s);
  if (b->budget == 0) b->budget = 16384;
  if (mr_batch_reset(b, cfg->seed_base) != 0) {
    std::string msg = g_err;
    mr_batch_destroy(b);
    return set_err(msg);
  }
  *out = b;
  return 0;
}

static int enqueue_reset(mr_batch* b, uint64_t seed_base) {
  b->cfg.seed_base = seed_base;
  b->kern = 0;
  b->c_open = 0;
  b->resume = false;
  b->D.seed0 = seed_base + b->cfg.cluster_base;
  HIPCHK(hipSetDevice(b->cfg.device));
  HIPCHK(hipMemsetAsync(b->D.pcnt, 0, CNT__N * sizeof(unsigned long long), b->stream));
#if MR_GUARD  // a violation belongs to the run it happened in
  HIPCHK(hipMemsetAsync(b->D.guard, 0, 4 * sizeof(uint32_t), b->stream));
  b->D.gprobe = std::getenv("MR_GUARD_PROBE") ? 1u : 0u;
#endif
  HIPCHK(hipMemsetAsync(b->D.stor, 0, (size_t)b->D.C * b->D.apply_cap * sizeof(SE), b->stream));
  if (b->D.led)
    HIPCHK(hipMemsetAsync(b->D.led, 0, (size_t)b->D.C * LED_W * sizeof(uint32_t), b->stream));
  if (b->D.trace_clusters) {  // apply digests: every node starts at 0 (valid), no record yet
    HIPCHK(hipMemsetAsync(b->D.tdig, 0, (size_t)b->D.trace_clusters * b->D.trace_cap * 8u, b->stream));
    HIPCHK(hipMemsetAsync(b->D.tapp, 0, (size_t)b->D.trace_clusters * b->D.trace_cap * 16u, b->stream));
    HIPCHK(hipMemsetAsync(b->D.adig, 0, (size_t)b->D.trace_clusters * MR_MAX_NODES * 16u, b->stream));
  }
  if (b->D.kv32)
    HIPCHK(hipMemsetAsync(b->D.kv32, 0, (size_t)b->D.C * b->D.n * KVREC * sizeof(uint32_t), b->stream));
  if (b->D.lin32)
    HIPCHK(hipMemsetAsync(b->D.lin32, 0, (size_t)b->D.C * KV_KEYS * KV_APP * LINW * sizeof(uint32_t),
                          b->stream));
  if (b->D.kvs32) {
    HIPCHK(hipMemsetAsync(b->D.kvs32, 0, (size_t)b->D.C * b->D.n * KVS_W * sizeof(uint32_t), b->stream));
    HIPCHK(hipMemsetAsync(b->D.kring, 0, (size_t)b->D.C * KV_RING * KRW * sizeof(uint32_t), b->stream));
  }
  HIPCHK(launch_reset(b->D, b->stream));
  return 0;
}

// one step-kernel launch on the batch stream, bracketed by the timing events;
// the remaining-cluster count is copied back asynchronously
static int enqueue_step(mr_batch* b, uint32_t budget) {
  // the pool kernel's message keys (32-bit, AppendEntries bit) and the step / tape kernels' are
  // different HBM formats: a run does not switch family between its launches
  const uint32_t kern = b->D.pool && !b->D.tape_mode ? 1u : 2u;
  if (b->kern && b->kern != kern)
    return set_err("decisions set or dropped in the middle of a pool-kernel run: mr_batch_reset first");
  b->kern = kern;
  b->h_ctl0[0] = 0;
  if (b->D.stream && b->resume) {  // continue: the held clusters first, the claim pointer kept
    b->h_ctl0[1] = b->h_remaining[1];
    b->D.nheld = b->h_remaining[0];
    b->D.resume = 1;
  } else {
    b->h_ctl0[1] = b->D.c0 + b->D.L;  // lanes start with clusters c0 .. c0+L-1 (streaming: claim on)
    b->D.nheld = 0;
    b->D.resume = 0;
  }
  b->D.held_in = b->held[b->hsel];
  b->D.held_out = b->held[b->hsel ^ 1u];
  b->hsel ^= 1u;
  b->resume = b->D.stream != 0;
  HIPCHK(hipMemcpyAsync(b->D.remaining, b->h_ctl0, 2 * sizeof(uint32_t), hipMemcpyHostToDevice,
                        b->stream));
  HIPCHK(hipEventRecord(b->ev0, b->stream));
  HIPCHK(launch_step(b->D, b->D.scenario, budget, b->stream));
  HIPCHK(hipEventRecord(b->ev1, b->stream));
  HIPCHK(hipMemcpyAsync(b->h_remaining, b->D.remaining, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost,
                        b->stream));
  return 0;
}

// clusters of the launched chunk without a verdict: those the lanes held, plus (streaming)
// those never claimed
static uint64_t remaining_after(const mr_batch* b) {
  const uint32_t next = b->h_remaining[1];
  return (uint64_t)b->h_remaining[0] + (b->D.stream && next < b->D.C ? b->D.C - next : 0u);
}

// MR_GUARD builds: the run fails with the first out-of-range index its launches recorded
static int guard_check(mr_batch* b) {
#if MR_GUARD
  uint32_t g[4];
  HIPCHK(hipMemcpy(g, b->D.guard, sizeof g, hipMemcpyDeviceToHost));
  if (g[0])
    return set_err("MR_GUARD: index " + std::to_string(g[2]) + " out of range " + std::to_string(g[3]) +
                   " (tag " + std::to_string(g[0]) + ", cluster " + std::to_string(g[1]) + ")");
#else
  (void)b;
#endif
  return 0;
}

int mr_batch_reset(mr_batch* b, uint64_t seed_base) {
  if (!b) return set_err("null batch");
  if (b->submitted) return set_err("batch has a submitted step: mr_batch_finish it first");
  if (enqueue_reset(b, seed_base) != 0) return -1;
  HIPCHK(hipStreamSynchronize(b->stream));
  return 0;
}

int mr_batch_run(mr_batch* b, uint64_t max_events_per_call, mr_run_stats* st) {
  if (!b) return set_err("null batch");
  if (b->submitted) return set_err("batch has a submitted step: mr_batch_finish it first");
  HIPCHK(hipSetDevice(b->cfg.device));
  auto t0 = std::chrono::steady_clock::now();
  mr_run_stats s;
  std::memset(&s, 0, sizeof s);
  uint64_t done_events = 0;
  bool stop = false;
  // chunks of D.L clusters, one after another (a streaming batch is one chunk of all clusters);
  // a call cut short by max_events_per_call resumes with the chunk it stopped in
  const uint32_t chunk = b->D.stream ? b->D.C : b->D.L;
  for (uint32_t c0 = b->c_open; c0 < b->D.C && !stop; c0 += chunk) {
    b->D.c0 = c0;
    for (;;) {
      uint32_t budget = b->budget;
      if (max_events_per_call) {
        if (done_events >= max_events_per_call) { stop = true; break; }
        uint64_t left = max_events_per_call - done_events;
        if (left < budget) budget = (uint32_t)left;
      }
      if (enqueue_step(b, budget) != 0) { b->D.c0 = 0; return -1; }
      HIPCHK(hipStreamSynchronize(b->stream));
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, b->ev0, b->ev1));
      s.kernel_ms += ms;
      s.launches++;
      done_events += budget;
      if (remaining_after(b) == 0) {
        b->c_open = c0 + chunk;
        break;
      }
    }
  }
  b->D.c0 = 0;
  if (guard_check(b) != 0) return -1;
  s.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  // events processed and clusters left: sums over the per-cluster counters (cheap reduce)
  mr_counters c;
  if (mr_batch_counters(b, &c) != 0) return -1;
  s.events = c.events;
  s.remaining = c.clusters - c.done;
  if (st) *st = s;
  return 0;
}

// Pipelined steps (bench.py): reset + the first step-kernel launch are only
// enqueued, so the host can queue the next batch's step on its own stream and
// that batch's waves take the CUs this batch's early-finishing waves free.
int mr_batch_submit(mr_batch* b, uint64_t seed_base) {
  if (!b) return set_err("null batch");
  if (b->submitted) return set_err("batch already has a submitted step");
  b->t_submit = std::chrono::steady_clock::now();
  if (enqueue_reset(b, seed_base) != 0) return -1;
  if (enqueue_step(b, b->budget) != 0) return -1;
  b->submitted = true;
  return 0;
}

int mr_batch_finish(mr_batch* b, mr_run_stats* st, mr_counters* cnt) {
  if (!b) return set_err("null batch");
  if (!b->submitted) return set_err("no submitted step");
  HIPCHK(hipSetDevice(b->cfg.device));
  HIPCHK(hipStreamSynchronize(b->stream));
  b->submitted = false;
  mr_run_stats s;
  std::memset(&s, 0, sizeof s);
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, b->ev0, b->ev1));
  s.kernel_ms = ms;
  s.launches = 1;
  s.remaining = remaining_after(b);
  if (s.remaining == 0) b->c_open = b->D.stream ? b->D.C : b->D.L;  // the submitted chunk is done
  if (b->c_open < b->D.C) s.remaining = 1;  // later chunks: run them below
  if (s.remaining != 0) {  // clusters past the per-launch budget: finish them synchronously
    mr_run_stats more;
    if (mr_batch_run(b, 0, &more) != 0) return -1;
    s.kernel_ms += more.kernel_ms;
    s.launches += more.launches;
    s.remaining = more.remaining;
  }
  if (guard_check(b) != 0) return -1;  // (mr_batch_run above checked its own launches)
  mr_counters c;
  if (mr_batch_counters(b, &c) != 0) return -1;
  s.events = c.events;
  s.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() -
                                                        b->t_submit).count();
  if (st) *st = s;
  if (cnt) *cnt = c;
  return 0;
}

static int mr_batch_verdicts_impl(mr_batch* b, uint16_t* code, uint32_t* time_us, uint64_t* digest) {
  if (!b) return set_err("null batch");
  HIPCHK(hipSetDevice(b->cfg.device));
  size_t C = b->D.C;
  std::vector<uint32_t> c32;
  // one field of every cluster: a strided row (cluster-major records) or a contiguous one
  auto row = [&](void* dst, const void* base, size_t f, size_t width, bool wide) -> hipError_t {
    const char* p = static_cast<const char*>(base) + (wide ? C64_IDX(f, 0, C) : CS_IDX(f, 0, C)) * width;
    const size_t pitch = (wide ? C64_IDX(f, 1, C) - C64_IDX(f, 0, C) : CS_IDX(f, 1, C) - CS_IDX(f, 0, C)) * width;
    return hipMemcpy2DAsync(dst, width, p, pitch, width, C, hipMemcpyDeviceToHost, b->stream);
  };
  if (code) {
    c32.resize(C);
    HIPCHK(row(c32.data(), b->D.cs32, CS_CODE, 4, false));
  }
  if (time_us) HIPCHK(row(time_us, b->D.cs32, CS_VTIME, 4, false));
  if (digest) HIPCHK(row(digest, b->D.cs64, C64_DIGEST, 8, true));
  HIPCHK(hipStreamSynchronize(b->stream));
  for (size_t i = 0; i < c32.size(); i++) code[i] = (uint16_t)c32[i];
  return 0;
}

int mr_batch_counters(mr_batch* b, mr_counters* out) {
  if (!b || !out) return set_err("null argument");
  HIPCHK(hipSetDevice(b->cfg.device));
  std::vector<unsigned long long> h(RED_N, 0);
  h[CNT__N + 5] = ~0ull;
  HIPCHK(hipMemcpyAsync(b->red, h.data(), RED_N * 8, hipMemcpyHostToDevice, b->stream));
  HIPCHK(launch_reduce(b->D, b->red, b->cfg.cluster_base, b->stream));
  HIPCHK(hipMemcpyAsync(h.data(), b->red, RED_N * 8, hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  std::memset(out, 0, sizeof *out);
  out->clusters = b->D.C;
  out->ev_msg = h[CNT_EV_MSG]; out->ev_timer = h[CNT_EV_TIMER]; out->ev_tester = h[CNT_EV_TESTER];
  out->drop_clog = h[CNT_DROP_CLOG]; out->drop_loss = h[CNT_DROP_LOSS];
  out->drop_overflow = h[CNT_DROP_OVERFLOW]; out->drop_deliver = h[CNT_DROP_DELIVER];
  out->drop_stale = h[CNT_DROP_STALE]; out->elections = h[CNT_ELECTIONS];
  out->leaders_elected = h[CNT_LEADERS]; out->applies = h[CNT_APPLIES];
  out->snapshots = h[CNT_SNAPSHOTS]; out->installs = h[CNT_INSTALLS];
  out->entries_shipped = h[CNT_SHIPPED]; out->max_inflight = h[CNT_MAX_INFLIGHT];
  out->max_log = h[CNT_MAX_LOG]; out->max_index = h[CNT_MAX_INDEX];
  out->events = h[CNT__N + 0]; out->msgs_sent = h[CNT__N + 1]; out->virt_time_us = h[CNT__N + 2];
  out->done = h[CNT__N + 3]; out->passed = h[CNT__N + 4]; out->failed = out->done - out->passed;
  out->first_fail_cluster = h[CNT__N + 5];
  for (int i = 0; i < 64; i++) out->fail_hist[i] = h[CNT__N + 8 + i];
  for (int i = 0; i < 16; i++) {
    out->cov_leaders[i] = h[CNT__N + 72 + i];
    out->cov_events[i] = h[CNT__N + 88 + i];
  }
  out->kv_ops = h[CNT__N + 104];
  out->kv_checked = h[CNT__N + 105];
  out->kv_lin_checked = h[CNT__N + 106];
  out->log_writes = h[CNT_LOG_WRITES];
  out->entries_materialized = h[CNT_MATERIALIZED];
  out->coop_entries = h[CNT_COOP];
  out->first_fail_code = 0;
  if (out->first_fail_cluster != ~0ull) {
    uint32_t code = 0;
    size_t idx = out->first_fail_cluster - b->cfg.cluster_base;
    HIPCHK(hipMemcpy(&code, b->D.cs32 + CS_IDX(CS_CODE, idx, b->D.C), 4, hipMemcpyDeviceToHost));
    out->first_fail_code = code;
  }
  return 0;
}

int mr_trace_get(mr_batch* b, uint32_t k, mr_event* out, size_t cap, size_t* n) {
  if (!b || !out || !n) return set_err("null argument");
  if (k >= b->D.trace_clusters) return set_err("cluster not traced");
  HIPCHK(hipSetDevice(b->cfg.device));
  uint32_t tn = 0;
  HIPCHK(hipMemcpy(&tn, b->D.cs32 + CS_IDX(CS_TRACEN, k, b->D.C), 4, hipMemcpyDeviceToHost));
  size_t m = tn < b->D.trace_cap ? tn : b->D.trace_cap;
  if (m > cap) m = cap;
  HIPCHK(hipMemcpy(out, b->D.trace + (size_t)k * b->D.trace_cap, m * sizeof(mr_event),
                   hipMemcpyDeviceToHost));
  *n = m;
  return 0;
}

int mr_trace_digests(mr_batch* b, uint32_t k, uint64_t* out, size_t cap, size_t* n) {
  if (!b || !out || !n) return set_err("null argument");
  if (k >= b->D.trace_clusters) return set_err("cluster not traced");
  HIPCHK(hipSetDevice(b->cfg.device));
  HIPCHK(hipStreamSynchronize(b->stream));
  uint32_t tn = 0;
  HIPCHK(hipMemcpy(&tn, b->D.cs32 + CS_IDX(CS_TRACEN, k, b->D.C), 4, hipMemcpyDeviceToHost));
  size_t m = tn < b->D.trace_cap ? tn : b->D.trace_cap;
  if (m > cap) m = cap;
  HIPCHK(hipMemcpy(out, b->D.tdig + (size_t)k * b->D.trace_cap, m * sizeof(uint64_t),
                   hipMemcpyDeviceToHost));
  *n = m;
  return 0;
}

int mr_trace_applies(mr_batch* b, uint32_t k, uint64_t* out, size_t cap, size_t* n) {
  if (!b || !out || !n) return set_err("null argument");
  if (k >= b->D.trace_clusters) return set_err("cluster not traced");
  HIPCHK(hipSetDevice(b->cfg.device));
  HIPCHK(hipStreamSynchronize(b->stream));
  size_t m = cap < b->D.trace_cap ? cap : b->D.trace_cap;
  HIPCHK(hipMemcpy(out, b->D.tapp + (size_t)k * b->D.trace_cap * 2u, m * 2u * sizeof(uint64_t),
                   hipMemcpyDeviceToHost));
  while (m && !out[2 * (m - 1)]) m--;
  *n = m;
  return 0;
}

const char* mr_batch_kernel(const mr_batch* b) {
  if (!b) return "";
  return b->D.tape_mode ? "step_kernel_tape" : b->D.pool ? "pool_kernel" : "step_kernel";
}

uint32_t mr_decision_word(uint32_t v, uint32_t lo, uint32_t hi) {
  if (hi <= lo || v < lo || v >= hi) return 0;
  // ceil((v - lo) * 2^32 / (hi - lo)): the first w whose range image is v
  const uint64_t span = hi - lo, num = (uint64_t)(v - lo) << 32;
  return (uint32_t)((num + span - 1) / span);
}

// the batch's decision tables (replay rows + offsets, or the record tape) freed; Philox draws
static void drop_decisions(mr_batch* b) {
  if (b->tape) (void)hipFree(b->tape);
  if (b->doff) (void)hipFree(b->doff);
  b->tape = nullptr;
  b->doff = nullptr;
  b->D.dtab = nullptr; b->D.doff = nullptr; b->D.dcap = 0; b->D.tape_mode = 0;
}

// Keyed decisions as CSR rows: every decision once (16 B each) plus C + 1 offsets, so the
// table is O(n + C) whatever the longest row. Everything is validated and staged before the
// previous table is dropped, so a rejected call leaves the batch as it was.
static int set_decisions_impl(mr_batch* b, const mr_decision* d, size_t n) {
  const size_t C = b->D.C;
  if (n >= (1ull << 32)) return set_err("too many decisions for one batch (2^32 - 1 at most)");
  std::vector<uint32_t> off(C + 1, 0);
  for (size_t i = 0; i < n; i++) {
    if (d[i].cluster >= C) return set_err("decision for a cluster outside the batch");
    if (d[i].stream < MR_DS_TESTER || d[i].stream > MR_DS_NET) return set_err("bad decision stream");
    off[d[i].cluster + 1]++;
  }
  for (size_t c = 0; c < C; c++) off[c + 1] += off[c];
  std::vector<uint4> tab(n);
  std::vector<uint32_t> fill(off.begin(), off.end() - 1);
  for (size_t i = 0; i < n; i++) {
    const mr_decision& r = d[i];
    tab[fill[r.cluster]++] = make_uint4(((uint32_t)r.stream << 16) | r.entity, r.seq, r.w0, r.w1);
  }
  auto lt = [](const uint4& a, const uint4& c) { return a.x < c.x || (a.x == c.x && a.y < c.y); };
  for (size_t c = 0; c < C; c++) {
    uint4* row = tab.data() + off[c];
    const uint32_t cnt = off[c + 1] - off[c];
    std::sort(row, row + cnt, lt);
    for (uint32_t k = 1; k < cnt; k++)
      if (row[k].x == row[k - 1].x && row[k].y == row[k - 1].y)
        return set_err("duplicate decision key (cluster " + std::to_string(c) + ")");
  }
  uint4* dtab = nullptr;
  uint32_t* doff = nullptr;
  hipError_t e = hipMalloc(&dtab, (n ? n : 1) * sizeof(uint4));
  if (e == hipSuccess) e = hipMalloc(&doff, off.size() * sizeof(uint32_t));
  if (e == hipSuccess && n)
    e = hipMemcpy(dtab, tab.data(), n * sizeof(uint4), hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(doff, off.data(), off.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (dtab) (void)hipFree(dtab);
    if (doff) (void)hipFree(doff);
    return set_err(std::string("decision table: ") + hipGetErrorString(e));
  }
  drop_decisions(b);
  b->tape = dtab;
  b->doff = doff;
  b->D.dtab = dtab;
  b->D.doff = doff;
  b->D.tape_mode = 1;
  return 0;
}

int mr_batch_set_decisions(mr_batch* b, const mr_decision* d, size_t n) {
  if (!b) return set_err("null batch");
  if (n && !d) return set_err("null decisions");
  HIPCHK(hipSetDevice(b->cfg.device));
  HIPCHK(hipStreamSynchronize(b->stream));
  if (!n) { drop_decisions(b); return 0; }
  try {  // host staging may not fit: an error code across the C ABI, never an exception
    return set_decisions_impl(b, d, n);
  } catch (const std::bad_alloc&) {
    return set_err("decision table: host allocation failed");
  }
}

static int mr_batch_get_decisions_impl(mr_batch* b, uint32_t k, mr_decision* out, size_t cap, size_t* n) {
  if (!b || !n) return set_err("null argument");
  if (k >= b->D.C) return set_err("cluster out of range");
  HIPCHK(hipSetDevice(b->cfg.device));
  HIPCHK(hipStreamSynchronize(b->stream));
  uint32_t used = 0;
  HIPCHK(hipMemcpy(&used, b->D.cs32 + CS_IDX(CS_TAPE, k, b->D.C), 4, hipMemcpyDeviceToHost));
  *n = used;
  if (b->D.tape_mode != 2 || !out) return 0;
  size_t m = used < b->D.dcap ? used : b->D.dcap;
  if (m > cap) m = cap;
  std::vector<uint4> rows(m);
  if (m)
    HIPCHK(hipMemcpy(rows.data(), b->tape + (size_t)k * b->D.dcap, m * sizeof(uint4),
                     hipMemcpyDeviceToHost));
  for (size_t i = 0; i < m; i++)
    out[i] = mr_decision{k, (uint16_t)(rows[i].x >> 16), (uint16_t)(rows[i].x & 0xFFFFu), rows[i].y,
                         rows[i].z, rows[i].w};
  return 0;
}

static int mr_replay_impl(const mr_cfg* cfg, const mr_decision* d, size_t n, mr_event* out, size_t cap,
              size_t* n_out, uint16_t* code, uint32_t* time_us, uint64_t* misses) {
  if (!cfg || !n_out) return set_err("null argument");
  if (n && !d) return set_err("null decisions");
  mr_cfg c = *cfg;
  c.n_clusters = 1;
  c.flags = (c.flags | MR_F_TRACE) & ~MR_F_RECORD;
  c.trace_clusters = 1;
  c.trace_cap = cap ? (uint32_t)cap : 1u;
  mr_batch* b = nullptr;
  int rc = mr_batch_create(&c, &b);
  if (rc) return rc;
  std::vector<mr_decision> one(d, d + n);
  for (auto& r : one) r.cluster = 0;
  // keyed replay runs the MR_TAPE kernels even for an empty trace (every draw then misses)
  const mr_decision none{0, MR_DS_TESTER, 0xFFFFu, 0xFFFFFFFFu, 0u, 0u};
  if (one.empty()) one.push_back(none);
  rc = mr_batch_set_decisions(b, one.data(), one.size());
  mr_run_stats st;
  if (!rc) rc = mr_batch_run(b, 0, &st);
  uint16_t cd = 0;
  uint32_t t = 0;
  if (!rc) rc = mr_batch_verdicts(b, &cd, &t, nullptr);
  if (!rc && out && cap) rc = mr_trace_get(b, 0, out, cap, n_out);
  else if (!rc) *n_out = 0;
  size_t ms = 0;
  if (!rc && misses) rc = mr_batch_get_decisions(b, 0, nullptr, 0, &ms);
  if (!rc && misses) *misses = ms;
  if (!rc && code) *code = cd;
  if (!rc && time_us) *time_us = t;
  mr_batch_destroy(b);
  return rc;
}

void mr_batch_destroy(mr_batch* b) {
  if (!b) return;
  (void)hipSetDevice(b->cfg.device);
  if (b->stream) (void)hipStreamSynchronize(b->stream);
#ifdef MR_PROF
  if (b->base) {  // development profile: wave cycles per kernel section (mr_kernel.hip PROF_*)
    unsigned long long h[PROF_SLOTS];
    if (hipMemcpy(h, b->D.prof, sizeof h, hipMemcpyDeviceToHost) == hipSuccess) {
      std::fprintf(stderr, "MRPROF");
      for (uint32_t k = 0; k < PROF_SLOTS; k++) std::fprintf(stderr, " %llu", h[k]);
      std::fprintf(stderr, "\n");
    }
  }
#endif
  if (b->base) (void)hipFree(b->base);
  if (b->tape) (void)hipFree(b->tape);
  if (b->doff) (void)hipFree(b->doff);
  // the streaming held-cluster lists belong to the batch, not to its decision tables
  for (uint32_t h = 0; h < 2; h++)
    if (b->held[h]) { (void)hipFree(b->held[h]); b->held[h] = nullptr; }
  if (b->red) (void)hipFree(b->red);
  if (b->h_remaining) (void)hipHostFree(b->h_remaining);
  if (b->h_ctl0) (void)hipHostFree(b->h_ctl0);
  if (b->ev0) (void)hipEventDestroy(b->ev0);
  if (b->ev1) (void)hipEventDestroy(b->ev1);
  if (b->stream) (void)hipStreamDestroy(b->stream);
  delete b;
}

int mr_batch_create(const mr_cfg* cfg, mr_batch** out) {
  try {  // host allocations: an error code across the C ABI, never an exception
    return mr_batch_create_impl(cfg, out);
  } catch (const std::exception& e) {
    return set_err(std::string("mr_batch_create: ") + e.what());
  }
}

int mr_batch_verdicts(mr_batch* b, uint16_t* code, uint32_t* time_us, uint64_t* digest) {
  try {  // host allocations: an error code across the C ABI, never an exception
    return mr_batch_verdicts_impl(b, code, time_us, digest);
  } catch (const std::exception& e) {
    return set_err(std::string("mr_batch_verdicts: ") + e.what());
  }
}

int mr_batch_get_decisions(mr_batch* b, uint32_t k, mr_decision* out, size_t cap, size_t* n) {
  try {  // host allocations: an error code across the C ABI, never an exception
    return mr_batch_get_decisions_impl(b, k, out, cap, n);
  } catch (const std::exception& e) {
    return set_err(std::string("mr_batch_get_decisions: ") + e.what());
  }
}

int mr_replay(const mr_cfg* cfg, const mr_decision* d, size_t n, mr_event* out, size_t cap,
              size_t* n_out, uint16_t* code, uint32_t* time_us, uint64_t* misses) {
  try {  // host allocations: an error code across the C ABI, never an exception
    return mr_replay_impl(cfg, d, n, out, cap, n_out, code, time_us, misses);
  } catch (const std::exception& e) {
    return set_err(std::string("mr_replay: ") + e.what());
  }
}

}  // extern "C"
