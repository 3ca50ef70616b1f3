/*
 * mr_oracle_main.c — CLI for the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * Mirrors the reference's CPU path `MADSIM_TEST_SEED=s MADSIM_TEST_NUM=N
 * cargo test <name>` (README.md:44-66): runs seeds s..s+N-1 of one test
 * sequentially in this process, prints the panic message and the failing
 * seed like the #[madsim::test] harness, and a one-line JSON summary that
 * bench.py's cpu_baseline leg parses.
 *
 * usage: mr_oracle <test_name> [--nodes N] [--iters K] [--unreliable] [--null]
 */
#define _POSIX_C_SOURCE 199309L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mr_oracle.h"

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <test_name> [--nodes N] [--iters K] [--unreliable] [--null]\n",
            argv[0]);
    return 2;
  }
  uint32_t scn = mro_scenario_from_name(argv[1]);
  mr_cfg cfg;
  if (!scn || mro_cfg_init(&cfg, scn) != 0) {
    fprintf(stderr, "unknown test %s\n", argv[1]);
    return 2;
  }
  for (int i = 2; i < argc; i++) {
    if (!strcmp(argv[i], "--nodes") && i + 1 < argc) cfg.n_nodes = (uint32_t)atoi(argv[++i]);
    else if (!strcmp(argv[i], "--iters") && i + 1 < argc) cfg.iters = (uint32_t)atoi(argv[++i]);
    else if (!strcmp(argv[i], "--unreliable")) cfg.flags |= MR_F_UNRELIABLE;
    else if (!strcmp(argv[i], "--null")) cfg.flags |= MR_F_NULL_RAFT;
    else if (!strcmp(argv[i], "--safety")) cfg.flags |= MR_F_SAFETY;
  }
  const char* es = getenv("MADSIM_TEST_SEED");
  const char* en = getenv("MADSIM_TEST_NUM");
  uint64_t seed = es ? strtoull(es, NULL, 10) : cfg.seed_base;
  uint64_t num = en ? strtoull(en, NULL, 10) : 1;
  cfg.seed_base = seed;
  cfg.cluster_base = 0;

  mro_result sum;
  memset(&sum, 0, sizeof sum);
  uint64_t passed = 0, failed = 0;
  double t0 = now_s();
  for (uint64_t k = 0; k < num; k++) {
    mro_result r;
    if (mro_run_cluster(&cfg, k, &r, NULL, 0, NULL) != 0) {
      fprintf(stderr, "bad config\n");
      return 2;
    }
    sum.events += r.events;
    sum.msgs_sent += r.msgs_sent;
    if (r.code == MR_PASS) {
      passed++;
    } else {
      failed++;
      if (failed <= 3)
        fprintf(stderr, "panicked at '%s' (code %u, t=%.3fs)\nMADSIM_TEST_SEED=%llu\n",
                mro_fail_message(r.code), r.code, r.time_us * 1e-6,
                (unsigned long long)(seed + k));
    }
  }
  double dt = now_s() - t0;
  printf("{\"test\": \"%s\", \"seeds\": %llu, \"passed\": %llu, \"failed\": %llu, "
         "\"events\": %llu, \"msgs\": %llu, \"wall_s\": %.6f, \"seeds_per_s\": %.3f, "
         "\"events_per_s\": %.1f}\n",
         argv[1], (unsigned long long)num, (unsigned long long)passed,
         (unsigned long long)failed, (unsigned long long)sum.events,
         (unsigned long long)sum.msgs_sent, dt, num / dt, sum.events / dt);
  return failed ? 1 : 0;
}
