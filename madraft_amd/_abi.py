"""ctypes mirror of include/madraft_sim.h (structs, enums, numpy trace dtype).

Plain data definitions only; loading a library is done by madraft_amd.sim
(the HIP product) or by the tests (the CPU oracle).
"""
import ctypes as C

import numpy as np

MR_ABI_VERSION = 4
MR_MAX_NODES = 8
MR_RUNNING = 0xFFFF
MR_PASS = 0

MR_F_UNRELIABLE = 0x1
MR_F_NULL_RAFT = 0x2
MR_F_TRACE = 0x4
MR_F_SAFETY = 0x8
MR_F_BUG_VOTE_TWICE = 0x10
MR_F_BUG_VOTE_STALE = 0x20
MR_F_BUG_NO_PREV_CHECK = 0x40
MR_F_RECORD = 0x80
MR_F_BUG_NO_DEDUP = 0x100
MR_F_BUG_STALE_READ = 0x200
MR_F_STREAM = 0x400  # lanes < clusters: finished lanes take the next cluster (mr_cfg.lanes)
MR_F_BUG_NO_APPLY_CHECK = 0x800  # test-only: apply checker compares no values (ABI 4)
DIGEST_INVALID = (1 << 64) - 1  # mr_trace_digests: the node's prefix was not applied entry by entry


def apply_mix(i, v):
    """include/madraft_sim.h mr_apply_mix: the apply-digest term of entry i with value v."""
    m = (1 << 64) - 1
    z = (v ^ (i * 0x9E3779B97F4A7C15)) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)

README_SEED = 1629626496  # /root/reference/README.md:48

# enum mr_scenario, in header order (tests.rs names)
SCENARIOS = [
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
    # generic_test_linearizability (15 clients, 7 servers; SEMANTICS §9b)
    "persist_partition_unreliable_linearizable_3a",
    "snapshot_unreliable_recover_concurrent_partition_linearizable_3b",
]
SCENARIO_ID = {n: i for i, n in enumerate(SCENARIOS) if n}
# tests that still need multi-threaded tester programs (spawn_local); not built yet
UNSUPPORTED = set()
# kvraft generic_test (src/kvraft/tests.rs:65-238), BASELINE config 5
KV_TESTS = ["basic_3a", "concurrent_3a", "unreliable_3a", "many_partitions_one_client_3a",
            "many_partitions_many_clients_3a", "persist_one_client_3a", "persist_concurrent_3a",
            "persist_concurrent_unreliable_3a", "persist_partition_3a",
            "persist_partition_unreliable_3a", "unreliable_one_key_3a", "one_partition_3a",
            "snapshot_rpc_3b", "snapshot_size_3b", "snapshot_recover_3b",
            "snapshot_recover_many_clients_3b", "snapshot_unreliable_3b",
            "snapshot_unreliable_recover_3b", "snapshot_unreliable_recover_concurrent_partition_3b",
            "persist_partition_unreliable_linearizable_3a",
            "snapshot_unreliable_recover_concurrent_partition_linearizable_3b"]
LIN_TESTS = KV_TESTS[-2:]  # generic_test_linearizability (SEMANTICS §9b)
GPU_UNSUPPORTED = set(UNSUPPORTED)

FAIL_NAMES = {
    0: "PASS", 1: "ONE_LEADER_NONE", 2: "MULTI_LEADER_TERM", 3: "TERM_DISAGREE",
    4: "UNEXPECTED_LEADER", 5: "WAIT_TOO_FEW", 6: "ONE_NO_AGREEMENT", 7: "TIMEOUT_120S",
    8: "APPLY_MISMATCH", 9: "APPLY_OUT_OF_ORDER", 10: "COMMIT_MISMATCH", 11: "UNWRAP_NONE",
    12: "LOG_SIZE", 13: "BASIC_PRECOMMIT", 14: "BASIC_INDEX", 15: "LEADER_REJECTED",
    16: "EXPECTED_INDEX2", 17: "NO_MAJORITY_COMMIT", 18: "UNEXPECTED_INDEX", 19: "CMD_MISSING",
    20: "TERM_CHANGED", 21: "RPC_INITIAL", 22: "START_FAILED", 23: "WRONG_VALUE",
    24: "RPC_TOO_MANY", 25: "RPC_IDLE", 26: "CHURN_VALUE", 27: "KV_GET_WRONG", 28: "KV_MISSING",
    29: "KV_APPEND_BAD", 30: "CTRL_NGROUPS", 31: "CTRL_MISSING", 32: "CTRL_INVALID",
    33: "CTRL_IMBALANCED", 34: "CTRL_SERVERS", 35: "CTRL_HISTORY", 36: "CTRL_MOVE_NUM",
    37: "CTRL_MOVE_WRONG", 38: "CTRL_MINIMAL_JOIN", 39: "CTRL_MINIMAL_LEAVE", 40: "CTRL_NO_LEADER",
    41: "CTRL_SAME_CONFIG", 42: "SAFETY_ELECTION", 43: "SAFETY_COMPLETENESS",
    44: "KV_LOG_SIZE", 45: "KV_SNAPSHOT_SIZE", 46: "KV_MINORITY_PROGRESS", 47: "KV_NO_COMPLETION",
    48: "KV_CHECK", 49: "SAFETY_LOG_MATCHING", 50: "TODO_APPLY", 51: "TODO_RPC_RESULTS",
    52: "KV_NOT_LINEARIZABLE",
    60: "SIM_CAPACITY",
    61: "SIM_EVENT_LIMIT", 62: "SIM_BAD_PROGRAM", 0xFFFF: "RUNNING",
}


class MrCfg(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32), ("scenario", C.c_uint32), ("n_nodes", C.c_uint32),
        ("flags", C.c_uint32), ("seed_base", C.c_uint64), ("cluster_base", C.c_uint64),
        ("n_clusters", C.c_uint64), ("iters", C.c_uint32), ("log_cap", C.c_uint32),
        ("apply_cap", C.c_uint32), ("msg_slots", C.c_uint32), ("ae_max", C.c_uint32),
        ("hb_us", C.c_uint32), ("elect_lo_us", C.c_uint32), ("elect_hi_us", C.c_uint32),
        ("max_events", C.c_uint32), ("trace_clusters", C.c_uint32), ("trace_cap", C.c_uint32),
        ("device", C.c_int32), ("tape_cap", C.c_uint32), ("lanes", C.c_uint32),
        ("lanes_per_wave", C.c_uint32), ("reserved", C.c_uint32 * 3),
    ]


class MrCounters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "clusters", "done", "passed", "failed", "events", "ev_msg", "ev_timer", "ev_tester",
        "msgs_sent", "drop_clog", "drop_loss", "drop_overflow", "drop_deliver", "drop_stale",
        "elections", "leaders_elected", "applies", "snapshots", "installs", "entries_shipped",
        "virt_time_us", "max_inflight", "max_log", "max_index", "first_fail_cluster",
        "first_fail_code")] + [("fail_hist", C.c_uint64 * 64), ("cov_leaders", C.c_uint64 * 16),
                               ("cov_events", C.c_uint64 * 16), ("kv_ops", C.c_uint64),
                               ("kv_checked", C.c_uint64), ("log_writes", C.c_uint64),
                               ("entries_materialized", C.c_uint64),
                               ("kv_lin_checked", C.c_uint64),
                               ("coop_entries", C.c_uint64)]  # ABI 4

    def to_dict(self):
        d = {n: getattr(self, n) for n, _ in self._fields_
             if n not in ("fail_hist", "cov_leaders", "cov_events")}
        d["fail_hist"] = {FAIL_NAMES.get(i, str(i)): int(v)
                          for i, v in enumerate(self.fail_hist) if v}
        d["cov_leaders"] = [int(v) for v in self.cov_leaders]
        d["cov_events"] = [int(v) for v in self.cov_events]
        return d


def cov_bucket(v):
    """Coverage-histogram bucket of a per-cluster count (mr_counters.cov_*)."""
    return 0 if v == 0 else min(15, int(v).bit_length())


class MrRunStats(C.Structure):
    _fields_ = [("launches", C.c_uint64), ("kernel_ms", C.c_double), ("wall_ms", C.c_double),
                ("events", C.c_uint64), ("remaining", C.c_uint64)]


EVENT_DTYPE = np.dtype([
    ("time_us", "<u4"), ("cls", "u1"), ("kind", "u1"), ("node", "u1"), ("role", "u1"),
    ("aux", "<u4"), ("term", "<u4"), ("commit", "<u4"), ("applied", "<u4"), ("last", "<u4"),
    ("snap", "<u4"),
])
assert EVENT_DTYPE.itemsize == 32

# keyed decisions (mr_decision, docs/SEMANTICS.md §12)
MR_DS_TESTER, MR_DS_ELECT, MR_DS_NET = 1, 2, 3
DECISION_DTYPE = np.dtype([("cluster", "<u4"), ("stream", "<u2"), ("entity", "<u2"), ("seq", "<u4"),
                           ("w0", "<u4"), ("w1", "<u4")])
assert DECISION_DTYPE.itemsize == 20
LOSS_Q32 = 429496729  # floor(0.1 * 2^32), tester.rs:130


def decision_word(v, lo, hi):
    """The smallest draw word w with lo + floor(w * (hi - lo) / 2^32) == v (mr_decision_word)."""
    assert lo <= v < hi
    return ((v - lo) << 32) // (hi - lo) + (1 if ((v - lo) << 32) % (hi - lo) else 0)


def net_decision(dropped, latency_us=1000, unreliable=True):
    """(w0, w1) of a send: dropped (by loss) or delivered after latency_us (tester.rs:127-137)."""
    hi = 27000 if unreliable else 10000
    return (0 if dropped else 0xFFFFFFFF), decision_word(latency_us, 1000, hi)

# symbols the product library exports (include/madraft_sim.h)
EXPORTS = [
    "mr_last_error", "mr_fail_message", "mr_scenario_name", "mr_scenario_from_name",
    "mr_cfg_init", "mr_batch_create", "mr_batch_reset", "mr_batch_run", "mr_batch_verdicts",
    "mr_batch_counters", "mr_trace_get", "mr_batch_destroy", "mr_batch_set_decisions",
    "mr_batch_get_decisions", "mr_decision_word", "mr_replay", "mr_batch_submit", "mr_batch_finish",
    "mr_trace_digests", "mr_trace_applies", "mr_batch_kernel",  # ABI 4
]
