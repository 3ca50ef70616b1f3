"""Host API of the MI355X batched Raft simulator (binds libmadraft_hip.so).

Mirrors the reference's test-harness interface for the hot path: a test is
named as in src/raft/tests.rs, seeds are chosen like MADSIM_TEST_SEED /
MADSIM_TEST_NUM (README.md:44-66), and a failing seed is reported with the
tester's panic message (src/raft/tester.rs) and "MADSIM_TEST_SEED=<seed>".
One `Batch` = many independent seeds of one test, run in lockstep on one GPU.

There is no CPU fallback: if the HIP library is missing this module raises.
"""
import ctypes as C
import os

import numpy as np

from . import _abi
from ._abi import DECISION_DTYPE, EVENT_DTYPE, FAIL_NAMES, MrCfg, MrCounters, MrRunStats

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MADRAFT_HIP_LIB") or os.path.join(_HERE, "lib", "libmadraft_hip.so")
_lib = None


def lib():
    """Load libmadraft_hip.so (built in-tree by __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"HIP library {LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; "
            "g.build()'` (there is no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    L.mr_last_error.restype = C.c_char_p
    L.mr_fail_message.restype = C.c_char_p
    L.mr_fail_message.argtypes = [C.c_uint32]
    L.mr_scenario_name.restype = C.c_char_p
    L.mr_scenario_name.argtypes = [C.c_uint32]
    L.mr_scenario_from_name.restype = C.c_uint32
    L.mr_scenario_from_name.argtypes = [C.c_char_p]
    L.mr_cfg_init.argtypes = [C.POINTER(MrCfg), C.c_uint32]
    L.mr_batch_create.argtypes = [C.POINTER(MrCfg), C.POINTER(C.c_void_p)]
    L.mr_batch_reset.argtypes = [C.c_void_p, C.c_uint64]
    L.mr_batch_run.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(MrRunStats)]
    L.mr_batch_submit.argtypes = [C.c_void_p, C.c_uint64]
    L.mr_batch_finish.argtypes = [C.c_void_p, C.POINTER(MrRunStats), C.POINTER(MrCounters)]
    L.mr_batch_verdicts.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.mr_batch_counters.argtypes = [C.c_void_p, C.POINTER(MrCounters)]
    L.mr_trace_get.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t,
                               C.POINTER(C.c_size_t)]
    L.mr_trace_digests.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t,
                                   C.POINTER(C.c_size_t)]
    L.mr_trace_applies.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t,
                                   C.POINTER(C.c_size_t)]
    L.mr_batch_kernel.argtypes = [C.c_void_p]
    L.mr_batch_kernel.restype = C.c_char_p
    L.mr_batch_set_decisions.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    L.mr_batch_get_decisions.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t,
                                         C.POINTER(C.c_size_t)]
    L.mr_decision_word.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
    L.mr_decision_word.restype = C.c_uint32
    L.mr_replay.argtypes = [C.POINTER(MrCfg), C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                            C.POINTER(C.c_size_t), C.POINTER(C.c_uint16), C.POINTER(C.c_uint32),
                            C.POINTER(C.c_uint64)]
    L.mr_batch_destroy.argtypes = [C.c_void_p]
    L.mr_batch_destroy.restype = None
    _lib = L
    return L


def lib_sha16(path=None):
    """First 16 hex digits of the SHA-256 of the product library file (the build a
    measurement was taken with: bench.py's JSON line and profiles/pmc_*.json carry it)."""
    import hashlib
    h = hashlib.sha256()
    with open(path or LIB_PATH, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()[:16]


class SimError(RuntimeError):
    pass


def _check(rc):
    if rc != 0:
        raise SimError(lib().mr_last_error().decode())


def fail_message(code):
    return lib().mr_fail_message(int(code)).decode()


def make_cfg(test, clusters=1, seed=_abi.README_SEED, *, nodes=None, iters=0, unreliable=False,
             null_raft=False, trace_clusters=0, trace_cap=None, cluster_base=0, device=0,
             safety=False, stream=False, **overrides):
    """mr_cfg for `test` with the reference's defaults (mr_cfg_init) plus overrides."""
    scn = _abi.SCENARIO_ID.get(test)
    if scn is None:
        raise SimError(f"unknown test {test!r}")
    cfg = MrCfg()
    _check(lib().mr_cfg_init(C.byref(cfg), scn))
    cfg.n_clusters = int(clusters)
    cfg.seed_base = int(seed)
    cfg.cluster_base = int(cluster_base)
    cfg.iters = int(iters)
    cfg.device = int(device)
    if nodes:
        cfg.n_nodes = int(nodes)
        if nodes > 5 and "msg_slots" not in overrides:
            cfg.msg_slots = 64  # 7-node elections peak at ~30 in flight
    if unreliable:
        cfg.flags |= _abi.MR_F_UNRELIABLE
    if null_raft:
        cfg.flags |= _abi.MR_F_NULL_RAFT
    if safety:
        cfg.flags |= _abi.MR_F_SAFETY
    if stream:
        cfg.flags |= _abi.MR_F_STREAM
    if trace_clusters:
        cfg.flags |= _abi.MR_F_TRACE
        cfg.trace_clusters = int(trace_clusters)
        if trace_cap:
            cfg.trace_cap = int(trace_cap)
    cfg.flags |= int(overrides.pop("flags", 0))  # extra MR_F_* bits (SAFETY, BUG_*)
    for k, v in overrides.items():
        setattr(cfg, k, int(v))
    return cfg


class Batch:
    """`clusters` seeds of one reference test, resident on one GPU."""

    def __init__(self, test=None, clusters=1, seed=_abi.README_SEED, *, cfg=None, **kw):
        self.cfg = cfg if cfg is not None else make_cfg(test, clusters, seed, **kw)
        self._b = C.c_void_p()
        _check(lib().mr_batch_create(C.byref(self.cfg), C.byref(self._b)))

    @property
    def clusters(self):
        return int(self.cfg.n_clusters)

    def close(self):
        if self._b:
            lib().mr_batch_destroy(self._b)
            self._b = C.c_void_p()

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def reset(self, seed_base):
        self.cfg.seed_base = int(seed_base)
        _check(lib().mr_batch_reset(self._b, int(seed_base)))

    def run(self, max_events=0):
        st = MrRunStats()
        _check(lib().mr_batch_run(self._b, int(max_events), C.byref(st)))
        return {n: getattr(st, n) for n, _ in MrRunStats._fields_}

    def submit(self, seed_base):
        """reset(seed_base) + run()'s first launch, enqueued without waiting (mr_batch_submit);
        finish() completes it. Another batch's step can be submitted in between."""
        self.cfg.seed_base = int(seed_base)
        _check(lib().mr_batch_submit(self._b, int(seed_base)))

    def finish(self):
        """(run stats, counters) of the submitted step (mr_batch_finish)."""
        st, c = MrRunStats(), MrCounters()
        _check(lib().mr_batch_finish(self._b, C.byref(st), C.byref(c)))
        return {n: getattr(st, n) for n, _ in MrRunStats._fields_}, c.to_dict()

    def verdicts(self):
        n = self.clusters
        code = np.empty(n, np.uint16)
        t = np.empty(n, np.uint32)
        dig = np.empty(n, np.uint64)
        _check(lib().mr_batch_verdicts(self._b, code.ctypes.data, t.ctypes.data,
                                       dig.ctypes.data))
        return code, t, dig

    def counters(self):
        c = MrCounters()
        _check(lib().mr_batch_counters(self._b, C.byref(c)))
        return c.to_dict()

    def set_decisions(self, d):
        """Drive the clusters by keyed decisions (DECISION_DTYPE records, any order;
        SEMANTICS §12); None = Philox again. Call before run()."""
        if d is None or len(d) == 0:
            _check(lib().mr_batch_set_decisions(self._b, None, 0))
            return
        a = np.ascontiguousarray(d, dtype=DECISION_DTYPE)
        _check(lib().mr_batch_set_decisions(self._b, a.ctypes.data, a.size))

    def decisions(self, k, cap=1 << 20):
        """(n, records): with MR_F_RECORD cluster k's decisions in draw order (n drawn);
        with decisions set, n = its draws that found no record."""
        out = np.empty(cap, DECISION_DTYPE)
        n = C.c_size_t()
        _check(lib().mr_batch_get_decisions(self._b, int(k), out.ctypes.data, cap, C.byref(n)))
        return int(n.value), out[: min(n.value, cap)]

    def trace(self, k, cap=None):
        cap = cap or int(self.cfg.trace_cap)
        out = np.empty(cap, EVENT_DTYPE)
        n = C.c_size_t()
        _check(lib().mr_trace_get(self._b, int(k), out.ctypes.data, cap, C.byref(n)))
        return out[: n.value]

    def trace_digests(self, k, cap=None):
        """mr_trace_digests: per record of trace(k), its node's apply digest (ABI 4)."""
        cap = cap or int(self.cfg.trace_cap)
        out = np.empty(cap, np.uint64)
        n = C.c_size_t()
        _check(lib().mr_trace_digests(self._b, int(k), out.ctypes.data, cap, C.byref(n)))
        return out[: n.value]

    def trace_applies(self, k, cap=None):
        """mr_trace_applies: [n, 2] (command, key hash after it) per log index (ABI 4)."""
        cap = cap or int(self.cfg.trace_cap)
        out = np.zeros((cap, 2), np.uint64)
        n = C.c_size_t()
        _check(lib().mr_trace_applies(self._b, int(k), out.ctypes.data, cap, C.byref(n)))
        return out[: n.value]

    @property
    def kernel(self):
        """mr_batch_kernel: "pool_kernel", "step_kernel" or "step_kernel_tape"."""
        return lib().mr_batch_kernel(self._b).decode()


def replay(test, decisions, trace_cap=1 << 16, cluster_base=0, **kw):
    """mr_replay: one cluster of `test` driven by keyed decisions (DECISION_DTYPE records,
    any order): (per-event trace, verdict code, verdict time, draws without a record)."""
    cfg = make_cfg(test, 1, cluster_base=cluster_base, **kw)
    d = np.ascontiguousarray(decisions, dtype=DECISION_DTYPE)
    out = np.empty(trace_cap, EVENT_DTYPE)
    n, code, tm, ms = C.c_size_t(), C.c_uint16(), C.c_uint32(), C.c_uint64()
    _check(lib().mr_replay(C.byref(cfg), d.ctypes.data if d.size else None, d.size,
                           out.ctypes.data, trace_cap, C.byref(n), C.byref(code), C.byref(tm),
                           C.byref(ms)))
    return out[: n.value], int(code.value), int(tm.value), int(ms.value)


def run_test(test, seed=None, num=None, **kw):
    """`MADSIM_TEST_SEED=seed MADSIM_TEST_NUM=num cargo test <test>` on the GPU.

    Returns (codes, times_us, digests, counters); failures are also printed
    like the #[madsim::test] harness (README.md:44-48).
    """
    seed = int(os.environ.get("MADSIM_TEST_SEED", _abi.README_SEED)) if seed is None else seed
    num = int(os.environ.get("MADSIM_TEST_NUM", 1)) if num is None else num
    with Batch(test, num, seed, **kw) as b:
        b.run()
        code, t, dig = b.verdicts()
        cnt = b.counters()
    bad = np.nonzero(code != _abi.MR_PASS)[0]
    for k in bad[:3]:
        print(f"---- {test} ----\npanicked at '{fail_message(code[k])}' "
              f"({FAIL_NAMES.get(int(code[k]), code[k])}, t={t[k] * 1e-6:.3f}s)\n"
              f"MADSIM_TEST_SEED={seed + int(b.cfg.cluster_base) + int(k)}")
    return code, t, dig, cnt
