// mr_programs.cpp — the reference's raft test bodies (src/raft/tests.rs)
// compiled, by hand, to the tester ISA of mr_dev.h. The device interpreter
// (mr_kernel.hip: tester()) runs one program per cluster; multi-event tester
// helpers (one, wait, check_one_leader) are single ops. Each program follows
// its test line by line, including which RNG draws happen (SEMANTICS §6).
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "mr_dev.h"

namespace mr {

namespace {

struct Asm {
  std::vector<uint64_t> code;
  std::unordered_map<std::string, uint32_t> labels;
  std::vector<std::pair<size_t, std::string>> fix;
  uint32_t n;
  int uniq = 0;

  void op(uint32_t o, uint32_t a = 0, uint32_t b = 0, uint32_t c = 0, uint32_t imm = 0) {
    code.push_back((uint64_t)o | ((uint64_t)(a & 255) << 8) | ((uint64_t)(b & 255) << 16) |
                   ((uint64_t)(c & 255) << 24) | ((uint64_t)imm << 32));
  }
  std::string fresh(const char* p) { return std::string(p) + "#" + std::to_string(uniq++); }
  void L(const std::string& s) { labels[s] = (uint32_t)code.size(); }
  void jmp(const std::string& t) { fix.push_back({code.size(), t}); op(OP_JMP); }
  void brz(uint32_t r, const std::string& t) { fix.push_back({code.size(), t}); op(OP_BRZ, r); }
  void brnz(uint32_t r, const std::string& t) { fix.push_back({code.size(), t}); op(OP_BRNZ, r); }
  std::vector<uint64_t> finish() {
    for (auto& f : fix) {
      auto it = labels.find(f.second);
      if (it == labels.end()) throw std::runtime_error("undefined label " + f.second);
      code[f.first] |= (uint64_t)it->second << 32;
    }
    return code;
  }
  // ---- tester helpers (tester.rs)
  void one_imm(uint64_t value, uint32_t expected, bool retry, uint32_t dst = 9) {
    op(OP_LDV, 0, 0, 0, (uint32_t)value);
    op(OP_ONE, dst, 0 | (retry ? 128u : 0u), expected);
  }
  void one_rand(uint32_t expected, bool retry, uint32_t dst = 9) {
    op(OP_ENTRY, 0);
    op(OP_ONE, dst, 0 | (retry ? 128u : 0u), expected);
  }
  void col(uint32_t dst) { op(OP_CHECK_ONE_LEADER, dst); }
  void sleep(uint32_t us) { op(OP_SLEEP, 0, 0, 0, us); }
  void node(uint32_t o, uint32_t r, uint32_t off = 0) { op(o, r, off); }
  // for r = 0; r < limit(n if limit==0); r++ { body }
  template <class F>
  void loop(uint32_t r, uint32_t limit, F body) {
    std::string top = fresh("loop"), done = fresh("done");
    op(OP_MOVI, r, 0, 0, 0);
    L(top);
    if (limit == 0) op(OP_LTN, 28, r);
    else op(OP_LTI, 28, r, 0, limit);
    brz(28, done);
    body();
    op(OP_ADDI, r, r, 0, 1);
    jmp(top);
    L(done);
  }
};

constexpr uint32_t ELECTION_US = 1000000;  // RAFT_ELECTION_TIMEOUT, tests.rs:18
constexpr uint32_t NEG1 = 0xFFFFFFFFu;

void initial_election(Asm& a) {  // tests.rs:20-46
  a.op(OP_NEW, 0);
  a.col(0);
  a.sleep(50000);
  a.op(OP_CHECK_TERMS, 1);
  a.sleep(2 * ELECTION_US);
  a.op(OP_CHECK_TERMS, 2);
  a.col(0);
  a.op(OP_END);
}

void reelection(Asm& a) {  // tests.rs:48-78
  a.op(OP_NEW, 0);
  a.col(0);
  a.node(OP_DISCONNECT, 0);
  a.col(3);
  a.node(OP_CONNECT, 0);
  a.col(1);
  a.node(OP_DISCONNECT, 1);
  a.node(OP_DISCONNECT, 1, 1);
  a.sleep(2 * ELECTION_US);
  a.op(OP_CHECK_NO_LEADER);
  a.node(OP_CONNECT, 1, 1);
  a.col(3);
  a.node(OP_CONNECT, 1);
  a.col(3);
  a.op(OP_END);
}

void many_election(Asm& a, uint32_t iters) {  // tests.rs:80-112
  a.op(OP_NEW, 0);
  a.col(9);
  a.loop(0, iters, [&] {
    a.op(OP_RAND, 1, 0, 1);
    a.op(OP_RAND, 2, 0, 1);
    a.op(OP_RAND, 3, 0, 1);
    a.node(OP_DISCONNECT, 1); a.node(OP_DISCONNECT, 2); a.node(OP_DISCONNECT, 3);
    a.col(9);
    a.node(OP_CONNECT, 1); a.node(OP_CONNECT, 2); a.node(OP_CONNECT, 3);
  });
  a.col(9);
  a.op(OP_END);
}

void basic_agree(Asm& a) {  // tests.rs:114-130
  a.op(OP_NEW, 0);
  for (uint32_t index = 1; index <= 3; index++) {
    a.op(OP_MOVI, 0, 0, 0, index);
    a.op(OP_NCOMMITTED, 0);
    a.brnz(R_FLAG, "fail_pre");
    a.one_imm(index * 100ull, EXP_N(0), false, 1);
    a.op(OP_EQI, 28, 1, 0, index);
    a.brz(28, "fail_idx");
  }
  a.op(OP_END);
  a.L("fail_pre"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_BASIC_PRECOMMIT);
  a.L("fail_idx"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_BASIC_INDEX);
}

void fail_agree(Asm& a) {  // tests.rs:132-161
  a.op(OP_NEW, 0);
  a.one_imm(101, EXP_N(0), false);
  a.col(0);
  a.node(OP_DISCONNECT, 0, 1);
  a.one_imm(102, EXP_N(1), false);
  a.one_imm(103, EXP_N(1), false);
  a.sleep(ELECTION_US);
  a.one_imm(104, EXP_N(1), false);
  a.one_imm(105, EXP_N(1), false);
  a.node(OP_CONNECT, 0, 1);
  a.one_imm(106, EXP_N(0), true);
  a.sleep(ELECTION_US);
  a.one_imm(107, EXP_N(0), true);
  a.op(OP_END);
}

void fail_no_agree(Asm& a) {  // tests.rs:163-209
  a.op(OP_NEW, 0);
  a.one_imm(10, EXP_N(0), false);
  a.col(0);
  a.node(OP_DISCONNECT, 0, 1); a.node(OP_DISCONNECT, 0, 2); a.node(OP_DISCONNECT, 0, 3);
  a.op(OP_LDV, 0, 0, 0, 20);
  a.op(OP_START, 0, 0, 0);
  a.brz(R_FLAG, "fail_rej");
  a.op(OP_MOV, 1, R_IDX);
  a.op(OP_EQI, 28, 1, 0, 2);
  a.brz(28, "fail_idx2");
  a.sleep(2 * ELECTION_US);
  a.op(OP_NCOMMITTED, 1);
  a.brnz(R_FLAG, "fail_nomaj");
  a.node(OP_CONNECT, 0, 1); a.node(OP_CONNECT, 0, 2); a.node(OP_CONNECT, 0, 3);
  a.col(2);
  a.op(OP_LDV, 0, 0, 0, 30);
  a.op(OP_START, 2, 0, 0);
  a.brz(R_FLAG, "fail_rej");
  a.op(OP_MOV, 3, R_IDX);
  a.op(OP_LTI, 28, 3, 0, 2);
  a.brnz(28, "fail_unexp");
  a.op(OP_LTI, 28, 3, 0, 4);
  a.brz(28, "fail_unexp");
  a.one_imm(1000, EXP_N(0), true);
  a.op(OP_END);
  a.L("fail_rej"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_LEADER_REJECTED);
  a.L("fail_idx2"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_EXPECTED_INDEX2);
  a.L("fail_nomaj"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_NO_MAJORITY_COMMIT);
  a.L("fail_unexp"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_UNEXPECTED_INDEX);
}

// "if (0..servers).any(|j| t.term(j) != term) -> goto target", term in r[term_r]
void any_term_changed(Asm& a, uint32_t term_r, const std::string& target) {
  std::string top = a.fresh("tj"), done = a.fresh("tjd");
  a.op(OP_MOVI, 27, 0, 0, 0);
  a.L(top);
  a.op(OP_LTN, 28, 27);
  a.brz(28, done);
  a.op(OP_TERM, 26, 27, 0);
  a.op(OP_EQ, 28, 26, term_r);
  a.brz(28, target);
  a.op(OP_ADDI, 27, 27, 0, 1);
  a.jmp(top);
  a.L(done);
}

void concurrent_starts(Asm& a) {  // tests.rs:211-275
  a.op(OP_NEW, 0);
  a.op(OP_MOVI, 20, 0, 0, 0);  // success
  a.op(OP_MOVI, 0, 0, 0, 0);   // tried
  a.L("try");
  a.op(OP_LTI, 28, 0, 0, 5);
  a.brz(28, "after");
  a.brz(0, "nosleep");
  a.sleep(3000000);
  a.L("nosleep");
  a.col(1);
  a.op(OP_LDV, 0, 0, 0, 1);
  a.op(OP_START, 1, 0, 0);
  a.brz(R_FLAG, "cont");
  a.op(OP_MOV, 2, R_TERM);  // term
  a.op(OP_MOVI, 3, 0, 0, 0);  // number of idxes (kept in r10..r14)
  a.loop(4, 5, [&] {
    std::string nx = a.fresh("ii");
    a.op(OP_ADDI, 5, 4, 0, 100);
    a.op(OP_VLDR, 0, 5);
    a.op(OP_START, 1, 0, 0);
    a.brz(R_FLAG, nx);
    a.op(OP_EQ, 28, R_TERM, 2);
    a.brz(28, nx);
    a.op(OP_RSETX, 3, 10, R_IDX);
    a.op(OP_ADDI, 3, 3, 0, 1);
    a.L(nx);
  });
  any_term_changed(a, 2, "cont");
  a.op(OP_MOVI, 6, 0, 0, 0);  // number of cmds (kept in v1..v5)
  a.op(OP_MOVI, 4, 0, 0, 0);
  a.L("q");
  a.op(OP_LT, 28, 4, 3);
  a.brz(28, "qd");
  a.op(OP_RGETX, 7, 4, 10);
  a.op(OP_WAIT, 7, 2, EXP_N(0));
  a.brz(R_FLAG, "qn");
  a.op(OP_VSETX, 6, 1, V_RES);
  a.op(OP_ADDI, 6, 6, 0, 1);
  a.L("qn");
  a.op(OP_ADDI, 4, 4, 0, 1);
  a.jmp("q");
  a.L("qd");
  a.loop(4, 5, [&] {
    std::string inner = a.fresh("ck"), idone = a.fresh("ckd"), nx = a.fresh("ckn");
    a.op(OP_ADDI, 5, 4, 0, 100);
    a.op(OP_VLDR, 0, 5);
    a.op(OP_MOVI, 7, 0, 0, 0);
    a.op(OP_MOVI, 15, 0, 0, 0);
    a.L(inner);
    a.op(OP_LT, 28, 7, 6);
    a.brz(28, idone);
    a.op(OP_VGETX, 14, 7, 1);
    a.op(OP_VEQ, 28, 14, 0);
    a.brz(28, nx);
    a.op(OP_MOVI, 15, 0, 0, 1);
    a.L(nx);
    a.op(OP_ADDI, 7, 7, 0, 1);
    a.jmp(inner);
    a.L(idone);
    a.brz(15, "fail_missing");
  });
  a.op(OP_MOVI, 20, 0, 0, 1);
  a.jmp("after");
  a.L("cont");
  a.op(OP_ADDI, 0, 0, 0, 1);
  a.jmp("try");
  a.L("after");
  a.brz(20, "fail_tc");
  a.op(OP_END);
  a.L("fail_missing"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_CMD_MISSING);
  a.L("fail_tc"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_TERM_CHANGED);
}

void rejoin(Asm& a) {  // tests.rs:277-313
  a.op(OP_NEW, 0);
  a.one_imm(101, EXP_N(0), true);
  a.col(0);
  a.node(OP_DISCONNECT, 0);
  for (uint32_t v : {102u, 103u, 104u}) {
    a.op(OP_LDV, 0, 0, 0, v);
    a.op(OP_START, 0, 0, 0);
  }
  a.one_imm(103, 2, true);
  a.col(1);
  a.node(OP_DISCONNECT, 1);
  a.node(OP_CONNECT, 0);
  a.one_imm(104, 2, true);
  a.node(OP_CONNECT, 1);
  a.one_imm(105, EXP_N(0), true);
  a.op(OP_END);
}

void backup(Asm& a) {  // tests.rs:315-386
  a.op(OP_NEW, 0);
  a.one_rand(EXP_N(0), true);
  a.col(0);
  a.node(OP_DISCONNECT, 0, 2); a.node(OP_DISCONNECT, 0, 3); a.node(OP_DISCONNECT, 0, 4);
  a.loop(1, 50, [&] { a.op(OP_ENTRY, 0); a.op(OP_START, 0, 0, 0); });
  a.sleep(ELECTION_US / 2);
  a.node(OP_DISCONNECT, 0, 0); a.node(OP_DISCONNECT, 0, 1);
  a.node(OP_CONNECT, 0, 2); a.node(OP_CONNECT, 0, 3); a.node(OP_CONNECT, 0, 4);
  a.loop(1, 50, [&] { a.one_rand(3, true); });
  a.col(2);
  a.op(OP_MODN, 3, 0, 0, 2);  // other = (leader1 + 2) % servers
  a.op(OP_EQ, 28, 2, 3);
  a.brz(28, "o");
  a.op(OP_MODN, 3, 2, 0, 1);
  a.L("o");
  a.node(OP_DISCONNECT, 3);
  a.loop(1, 50, [&] { a.op(OP_ENTRY, 0); a.op(OP_START, 2, 0, 0); });
  a.sleep(ELECTION_US / 2);
  a.op(OP_DISCONNECT_ALL);
  a.node(OP_CONNECT, 0, 0); a.node(OP_CONNECT, 0, 1); a.node(OP_CONNECT, 3);
  a.loop(1, 50, [&] { a.one_rand(3, true); });
  a.op(OP_CONNECT_ALL);
  a.one_rand(EXP_N(0), true);
  a.op(OP_END);
}

void count(Asm& a) {  // tests.rs:388-479
  a.op(OP_NEW, 0);
  a.col(9);
  a.op(OP_RPC_TOTAL, 1);
  a.op(OP_LTI, 28, 1, 0, 1);
  a.brnz(28, "fail_init");
  a.op(OP_LTI, 28, 1, 0, 31);
  a.brz(28, "fail_init");
  a.op(OP_MOVI, 2, 0, 0, 0);   // total2
  a.op(OP_MOVI, 20, 0, 0, 0);  // success
  a.op(OP_MOVI, 0, 0, 0, 0);   // tried
  a.L("try");
  a.op(OP_LTI, 28, 0, 0, 5);
  a.brz(28, "after");
  a.brz(0, "ns");
  a.sleep(3000000);
  a.L("ns");
  a.col(3);
  a.op(OP_RPC_TOTAL, 1);
  a.op(OP_LDV, 0, 0, 0, 1);
  a.op(OP_START, 3, 0, 0);
  a.brz(R_FLAG, "cont");
  a.op(OP_MOV, 4, R_IDX);   // starti
  a.op(OP_MOV, 5, R_TERM);  // term
  a.op(OP_MOVI, 6, 0, 0, 1);
  a.L("i");  // for i in 1..iters+2; cmds[i-1] kept in v[i]
  a.op(OP_LTI, 28, 6, 0, 12);
  a.brz(28, "id");
  a.op(OP_ENTRY, 0);
  a.op(OP_VSETX, 6, 0, 0);
  a.op(OP_START, 3, 0, 0);
  a.brz(R_FLAG, "cont");
  a.op(OP_EQ, 28, R_TERM, 5);
  a.brz(28, "cont");
  a.op(OP_SUB, 7, R_IDX, 4);
  a.op(OP_EQ, 28, 7, 6);
  a.brz(28, "fail_start");
  a.op(OP_ADDI, 6, 6, 0, 1);
  a.jmp("i");
  a.L("id");
  a.op(OP_MOVI, 6, 0, 0, 1);
  a.L("w");
  a.op(OP_LTI, 28, 6, 0, 11);
  a.brz(28, "wd");
  a.op(OP_ADD, 7, 4, 6);  // starti + i
  a.op(OP_WAIT, 7, 5, EXP_N(0));
  a.brz(R_FLAG, "wn");
  a.op(OP_VGETX, 14, 6, 0);
  a.op(OP_VEQ, 28, V_RES, 14);
  a.brz(28, "fail_wrong");
  a.L("wn");
  a.op(OP_ADDI, 6, 6, 0, 1);
  a.jmp("w");
  a.L("wd");
  any_term_changed(a, 5, "cont");
  a.op(OP_RPC_TOTAL, 2);
  a.op(OP_SUB, 7, 2, 1);
  a.op(OP_LTI, 28, 7, 0, (10 + 1 + 3) * 3 + 1);
  a.brz(28, "fail_many");
  a.op(OP_MOVI, 20, 0, 0, 1);
  a.jmp("after");
  a.L("cont");
  a.op(OP_ADDI, 0, 0, 0, 1);
  a.jmp("try");
  a.L("after");
  a.brz(20, "fail_tc");
  a.sleep(ELECTION_US);
  a.op(OP_RPC_TOTAL, 7);
  a.op(OP_SUB, 7, 7, 2);
  a.op(OP_LTI, 28, 7, 0, 3 * 20 + 1);
  a.brz(28, "fail_idle");
  a.op(OP_END);
  a.L("fail_init"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_RPC_INITIAL);
  a.L("fail_start"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_START_FAILED);
  a.L("fail_wrong"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_WRONG_VALUE);
  a.L("fail_many"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_RPC_TOO_MANY);
  a.L("fail_tc"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_TERM_CHANGED);
  a.L("fail_idle"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_RPC_IDLE);
}

void persist1(Asm& a) {  // tests.rs:481-526
  a.op(OP_NEW, 0);
  a.one_imm(11, EXP_N(0), true);
  a.loop(1, 0, [&] { a.node(OP_START1, 1); });
  a.loop(1, 0, [&] { a.node(OP_DISCONNECT, 1); a.node(OP_CONNECT, 1); });
  a.one_imm(12, EXP_N(0), true);
  a.col(0);
  a.node(OP_DISCONNECT, 0); a.node(OP_START1, 0); a.node(OP_CONNECT, 0);
  a.one_imm(13, EXP_N(0), true);
  a.col(2);
  a.node(OP_DISCONNECT, 2);
  a.one_imm(14, EXP_N(1), true);
  a.node(OP_START1, 2); a.node(OP_CONNECT, 2);
  a.op(OP_MOVI, 3, 0, 0, 4);
  a.op(OP_WAIT, 3, 0xFF, EXP_N(0));
  a.col(4);
  a.op(OP_MODN, 5, 4, 0, 1);
  a.node(OP_DISCONNECT, 5);
  a.one_imm(15, EXP_N(1), true);
  a.node(OP_START1, 5); a.node(OP_CONNECT, 5);
  a.one_imm(16, EXP_N(0), true);
  a.op(OP_END);
}

void persist2(Asm& a) {  // tests.rs:528-572
  a.op(OP_NEW, 0);
  uint64_t index = 1;
  for (int k = 0; k < 5; k++) {
    a.one_imm(10 + index, EXP_N(0), true); index++;
    a.col(0);
    a.node(OP_DISCONNECT, 0, 1); a.node(OP_DISCONNECT, 0, 2);
    a.one_imm(10 + index, EXP_N(2), true); index++;
    a.node(OP_DISCONNECT, 0, 0); a.node(OP_DISCONNECT, 0, 3); a.node(OP_DISCONNECT, 0, 4);
    a.node(OP_START1, 0, 1); a.node(OP_START1, 0, 2);
    a.node(OP_CONNECT, 0, 1); a.node(OP_CONNECT, 0, 2);
    a.sleep(ELECTION_US);
    a.node(OP_START1, 0, 3); a.node(OP_CONNECT, 0, 3);
    a.one_imm(10 + index, EXP_N(2), true); index++;
    a.node(OP_CONNECT, 0, 4); a.node(OP_CONNECT, 0, 0);
  }
  a.one_imm(1000, EXP_N(0), true);
  a.op(OP_END);
}

void persist3(Asm& a) {  // tests.rs:574-602
  a.op(OP_NEW, 0);
  a.one_imm(101, 3, true);
  a.col(0);
  a.node(OP_DISCONNECT, 0, 2);
  a.one_imm(102, 2, true);
  a.node(OP_CRASH, 0, 0); a.node(OP_CRASH, 0, 1);
  a.node(OP_CONNECT, 0, 2);
  a.node(OP_START1, 0, 0); a.node(OP_CONNECT, 0, 0);
  a.one_imm(103, 2, true);
  a.node(OP_START1, 0, 1); a.node(OP_CONNECT, 0, 1);
  a.one_imm(104, EXP_N(0), true);
  a.op(OP_END);
}

void figure_8(Asm& a, uint32_t iters, bool unreliable) {  // tests.rs:612-660
  a.op(OP_NEW, 0);
  if (unreliable) a.op(OP_SET_UNREL, 1);
  a.one_rand(1, true);
  a.op(OP_MOVN, 1);  // nup
  a.loop(2, iters, [&] {
    a.op(OP_MOVI, 4, 0, 0, NEG1);  // leader = None
    a.loop(5, 0, [&] {
      std::string nx = a.fresh("f8n");
      a.op(OP_IS_STARTED, 5);
      a.brz(R_FLAG, nx);
      a.op(OP_ENTRY, 0);
      a.op(OP_START, 5, 0, 0);
      a.brz(R_FLAG, nx);
      a.op(OP_MOV, 4, 5);
      a.L(nx);
    });
    a.op(OP_SLEEP_FIG8);
    std::string nl = a.fresh("nl"), cont = a.fresh("cont");
    a.op(OP_EQI, 28, 4, 0, NEG1);
    a.brnz(28, nl);
    a.node(OP_CRASH, 4);
    a.op(OP_ADDI, 1, 1, 0, NEG1);
    a.L(nl);
    a.op(OP_LTI, 28, 1, 0, 3);
    a.brz(28, cont);
    a.op(OP_RAND, 6, 0, 1);
    a.op(OP_IS_STARTED, 6);
    a.brnz(R_FLAG, cont);
    a.node(OP_START1, 6);
    a.op(OP_ADDI, 1, 1, 0, 1);
    a.L(cont);
  });
  a.loop(5, 0, [&] {
    std::string nx = a.fresh("rs");
    a.op(OP_IS_STARTED, 5);
    a.brnz(R_FLAG, nx);
    a.node(OP_START1, 5);
    a.L(nx);
  });
  a.one_rand(EXP_N(0), true);
  a.op(OP_END);
}

void figure_8_unreliable(Asm& a, uint32_t iters) {  // tests.rs:688-741
  a.op(OP_NEW, 0);
  a.op(OP_SET_UNREL, 1);
  a.one_rand(1, true);
  a.op(OP_MOVN, 1);  // nup
  a.loop(2, iters, [&] {
    a.op(OP_MOVI, 4, 0, 0, NEG1);
    a.loop(5, 0, [&] {
      std::string nx = a.fresh("f8n");
      a.op(OP_ENTRY, 0);
      a.op(OP_START, 5, 0, 0);
      a.brz(R_FLAG, nx);
      a.op(OP_IS_CONNECTED, 5);
      a.brz(R_FLAG, nx);
      a.op(OP_MOV, 4, 5);
      a.L(nx);
    });
    a.op(OP_SLEEP_FIG8);
    std::string nl = a.fresh("nl"), cont = a.fresh("cont");
    a.op(OP_EQI, 28, 4, 0, NEG1);
    a.brnz(28, nl);
    a.op(OP_RAND, 6, 0, 0, 1000);
    a.op(OP_LTI, 28, 6, 0, ELECTION_US / 1000 / 2);
    a.brz(28, nl);
    a.node(OP_DISCONNECT, 4);
    a.op(OP_ADDI, 1, 1, 0, NEG1);
    a.L(nl);
    a.op(OP_LTI, 28, 1, 0, 3);
    a.brz(28, cont);
    a.op(OP_RAND, 6, 0, 1);
    a.op(OP_IS_CONNECTED, 6);
    a.brnz(R_FLAG, cont);
    a.node(OP_CONNECT, 6);
    a.op(OP_ADDI, 1, 1, 0, 1);
    a.L(cont);
  });
  a.op(OP_CONNECT_ALL);
  a.one_rand(EXP_N(0), true);
  a.op(OP_END);
}

void snap_common(Asm& a, uint32_t iters, bool disconnect, bool reliable, bool crash) {
  // tests.rs:858-911
  a.op(OP_NEW, 1);
  a.op(OP_SET_UNREL, reliable ? 0 : 1);
  a.one_rand(EXP_N(0), true);
  a.col(0);  // leader1
  a.op(OP_MOVI, 4, 0, 0, 0);  // i % 3
  a.loop(1, iters, [&] {
    std::string nsw = a.fresh("nsw"), tail = a.fresh("tail");
    a.op(OP_MODN, 2, 0, 0, 1);  // victim
    a.op(OP_MOV, 3, 0);         // sender
    a.op(OP_EQI, 28, 4, 0, 1);
    a.brz(28, nsw);
    a.op(OP_MODN, 3, 0, 0, 1);
    a.op(OP_MOV, 2, 0);
    a.L(nsw);
    if (disconnect) { a.node(OP_DISCONNECT, 2); a.one_rand(EXP_N(1), true); }
    if (crash) { a.node(OP_CRASH, 2); a.one_rand(EXP_N(1), true); }
    a.loop(5, 11, [&] { a.op(OP_ENTRY, 0); a.op(OP_START, 3, 0, 0); });
    a.one_rand(EXP_N(1), true);
    a.op(OP_LOG_SIZE, 6);
    a.op(OP_LTI, 28, 6, 0, 2000);
    a.brz(28, "fail_log");
    if (disconnect) {
      a.node(OP_CONNECT, 2);
      a.one_rand(EXP_N(0), true);
      a.col(0);
    }
    if (crash) {
      a.node(OP_START1, 2);
      a.node(OP_CONNECT, 2);
      a.one_rand(EXP_N(0), true);
      a.col(0);
    }
    a.op(OP_ADDI, 4, 4, 0, 1);
    a.op(OP_EQI, 28, 4, 0, 3);
    a.brz(28, tail);
    a.op(OP_MOVI, 4, 0, 0, 0);
    a.L(tail);
  });
  a.op(OP_END);
  a.L("fail_log"); a.op(OP_FAIL, 0, 0, 0, MR_FAIL_LOG_SIZE);
}

}  // namespace

// Returns false if the scenario has no GPU program yet.
bool build_program(const mr_cfg& cfg, std::vector<uint64_t>& out) {
  Asm a;
  a.n = cfg.n_nodes;
  auto it = [&](uint32_t d) { return cfg.iters ? cfg.iters : d; };
  switch (cfg.scenario) {
    case MR_SCN_INITIAL_ELECTION_2A: initial_election(a); break;
    case MR_SCN_REELECTION_2A: reelection(a); break;
    case MR_SCN_MANY_ELECTION_2A: many_election(a, it(10)); break;
    case MR_SCN_BASIC_AGREE_2B: basic_agree(a); break;
    case MR_SCN_FAIL_AGREE_2B: fail_agree(a); break;
    case MR_SCN_FAIL_NO_AGREE_2B: fail_no_agree(a); break;
    case MR_SCN_CONCURRENT_STARTS_2B: concurrent_starts(a); break;
    case MR_SCN_REJOIN_2B: rejoin(a); break;
    case MR_SCN_BACKUP_2B: backup(a); break;
    case MR_SCN_COUNT_2B: count(a); break;
    case MR_SCN_PERSIST1_2C: persist1(a); break;
    case MR_SCN_PERSIST2_2C: persist2(a); break;
    case MR_SCN_PERSIST3_2C: persist3(a); break;
    case MR_SCN_FIGURE_8_2C: figure_8(a, it(1000), false); break;
    case MR_SCN_FIGURE_8_UNRELIABLE_CRASH: figure_8(a, it(1000), true); break;
    case MR_SCN_FIGURE_8_UNRELIABLE_2C: figure_8_unreliable(a, it(1000)); break;
    case MR_SCN_SNAPSHOT_BASIC_2D: snap_common(a, it(30), false, true, false); break;
    case MR_SCN_SNAPSHOT_INSTALL_2D: snap_common(a, it(30), true, true, false); break;
    case MR_SCN_SNAPSHOT_INSTALL_UNRELIABLE_2D: snap_common(a, it(30), true, false, false); break;
    case MR_SCN_SNAPSHOT_INSTALL_CRASH_2D: snap_common(a, it(30), false, true, true); break;
    case MR_SCN_SNAPSHOT_INSTALL_UNRELIABLE_CRASH_2D:
      snap_common(a, it(30), false, false, true);
      break;
    default: return false;
  }
  out = a.finish();
  return true;
}

}  // namespace mr
