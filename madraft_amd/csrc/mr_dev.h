// mr_dev.h — device state layout and tester ISA shared by the HIP kernels
// (mr_kernel.hip) and the C++ batch driver (mr_host.cpp).
//
// Layout: one thread simulates one cluster. Every per-cluster scalar is an
// array indexed [field][cluster] (cluster-minor), so the 64 lanes of a wave,
// which hold 64 consecutive clusters, touch 64 consecutive words of a field:
// one or two 256-B segments per wave instruction. Per-node fields are
// [node][cluster]; next/match are [(leader*n + peer)][cluster]. Data a lane
// walks through by index (Raft log rings, message payloads, the tester's
// apply checker) is cluster-major so each lane's walk stays in its own
// cache lines.
#pragma once
#include <stdint.h>

#include "../../include/madraft_sim.h"

namespace mr {

// ---- node flag word (one u32 per node): role[0:2) alive[2] conn[3]
//      voted[4:8) (15 = none) inc[8:16) votes[16:24)
enum : uint32_t { R_F = 0, R_C = 1, R_L = 2, R_DOWN = 3 };
enum : uint32_t { M_RV_REQ = 1, M_RV_REP, M_AE_REQ, M_AE_REP, M_IS_REQ, M_IS_REP };
enum : uint32_t { ST_TESTER = 1, ST_ELECT = 2, ST_NET = 3 };

// per-cluster u32 counters, [CNT_*][cluster]
enum : uint32_t {
  CNT_EV_MSG, CNT_EV_TIMER, CNT_EV_TESTER, CNT_DROP_CLOG, CNT_DROP_LOSS, CNT_DROP_OVERFLOW,
  CNT_DROP_DELIVER, CNT_DROP_STALE, CNT_ELECTIONS, CNT_LEADERS, CNT_APPLIES, CNT_SNAPSHOTS,
  CNT_INSTALLS, CNT_SHIPPED, CNT_MAX_INFLIGHT, CNT_MAX_LOG, CNT_MAX_INDEX, CNT__N
};

// ---- tester ISA: 64-bit instructions  op[0:8) a[8:16) b[16:24) c[24:32) imm[32:64)
enum : uint32_t {
  OP_NOP = 0,
  OP_NEW,            // a = snapshot mode: RaftTester::new / new_with_snapshot
  OP_SET_UNREL,      // a = flag: set_unreliable
  OP_END,            // end(): check_timeout, pass
  OP_FAIL,           // imm = fail code
  OP_SLEEP,          // imm = us
  OP_SLEEP_FIG8,     // tests.rs:631-636: gen_bool(0.1) ? U[0,500ms) : U[0,13ms)
  OP_CHECK_ONE_LEADER,  // r[a] = leader                       (multi-event)
  OP_CHECK_TERMS,    // r[a] = term
  OP_CHECK_NO_LEADER,
  OP_ONE,            // r[a] = one(v[b&15], expected(c), retry = b>>7)  (multi-event)
  OP_WAIT,           // wait(r[a], n(c), start_term = b==0xFF ? None : r[b]) -> r31 some, v15
  OP_NCOMMITTED,     // n_committed(r[a]) -> r31 count, v15 value
  OP_START,          // start((r[a]+b)%n, v[c]) -> r31 ok, r30 index, r29 term
  OP_ENTRY,          // v[a] = gen_entry
  OP_LDV,            // v[a] = imm
  OP_VLDR,           // v[a] = r[b]
  OP_RAND,           // r[a] = U[0, c ? n : imm)
  OP_CONNECT,        // node (r[a]+b)%n
  OP_DISCONNECT,
  OP_CRASH,
  OP_START1,
  OP_CONNECT_ALL,
  OP_DISCONNECT_ALL,
  OP_IS_STARTED,     // r31 = is_started((r[a]+b)%n)
  OP_IS_CONNECTED,   // r31 = is_connected((r[a]+b)%n)
  OP_TERM,           // r[a] = term((r[b]+c)%n)   (unwrap)
  OP_LOG_SIZE,       // r[a]
  OP_RPC_TOTAL,      // r[a]
  OP_MOVI,           // r[a] = imm
  OP_MOVN,           // r[a] = n
  OP_MOV,            // r[a] = r[b]
  OP_ADDI,           // r[a] = r[b] + imm
  OP_ADD,            // r[a] = r[b] + r[c]
  OP_SUB,            // r[a] = r[b] - r[c]
  OP_MODN,           // r[a] = (r[b] + imm) % n
  OP_LT,             // r[a] = r[b] < r[c]
  OP_LTI,            // r[a] = r[b] < imm
  OP_LTN,            // r[a] = r[b] < n
  OP_EQ,             // r[a] = r[b] == r[c]
  OP_EQI,            // r[a] = r[b] == imm
  OP_VEQ,            // r[a] = v[b] == v[c]
  OP_RSETX,          // r[(r[a]+b)&31] = r[c]
  OP_RGETX,          // r[a] = r[(r[b]+c)&31]
  OP_VSETX,          // v[(r[a]+b)&15] = v[c]
  OP_VGETX,          // v[a] = v[(r[b]+c)&15]
  OP_JMP,            // pc = imm
  OP_BRZ,            // if r[a] == 0: pc = imm
  OP_BRNZ,           // if r[a] != 0: pc = imm
  OP__N
};
// expected-server operand: c < 128 -> c ; c >= 128 -> n - (c - 128)
constexpr uint32_t EXP_N(uint32_t minus) { return 128u + minus; }
constexpr uint32_t R_FLAG = 31, R_IDX = 30, R_TERM = 29;  // fixed result registers
constexpr uint32_t V_RES = 15;
constexpr uint32_t N_R = 32, N_V = 16, N_S = 6;  // tester registers / multi-event op scratch

// ---- everything the kernels see (passed by value as a kernel argument)
struct Dev {
  // config
  uint32_t C, n, log_cap, apply_cap, M, K, hb, elo, ehi, max_events;
  uint32_t null_raft, unrel_flag, trace_clusters, trace_cap, prog_len, pad;
  uint64_t seed0;  // seed of cluster 0 = seed_base + cluster_base
  const uint64_t* prog;
  // cluster scalars [C]
  uint16_t* code;
  uint32_t *vtime, *now, *events, *msgs_sent, *inflight, *netmode, *t_ctr, *trace_n, *mslot;
  uint64_t *free_mask, *digest, *mmin;
  uint32_t* cnt;  // [CNT__N][C]
  // nodes [n][C]
  uint32_t *nflags, *nterm, *ncommit, *napplied, *nlast, *nsnap, *nsnapt, *ntimer, *nectr, *nnctr;
  uint64_t* nsnapv;
  uint32_t *nnext, *nmatch;  // [(d*n+p)][C]
  uint32_t* lterm;           // [C][n][log_cap]
  uint64_t* lval;
  // messages [M][C]
  uint64_t* mkey;
  uint32_t *mhdr, *mterm, *ma, *mb, *mc;
  uint64_t* mv;
  uint32_t* pterm;  // [C][M][K]
  uint64_t* pval;
  // tester storage (tester.rs:366-428)
  uint8_t* smask;  // [C][apply_cap]
  uint64_t* sval;
  uint32_t* slen;  // [n][C]
  // tester interpreter
  uint32_t *tpc, *twake, *tphase;
  uint32_t* ts;  // [N_S][C]
  uint32_t* tr;  // [N_R][C]
  uint64_t* tv;  // [N_V][C]
  mr_event* trace;  // [trace_clusters][trace_cap]
  uint32_t* remaining;  // clusters without verdict after a step launch
};

}  // namespace mr
