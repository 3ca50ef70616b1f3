"""ctypes bindings of the CPU oracle (oracle/_build/libmr_oracle.so).

Test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg load it, as the checker — never as the product.
"""
import ctypes as C
import os

import numpy as np

from madraft_amd._abi import DECISION_DTYPE, EVENT_DTYPE, MrCfg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_build", "libmr_oracle.so")


class MroResult(C.Structure):
    _fields_ = [("code", C.c_uint32), ("time_us", C.c_uint32), ("digest", C.c_uint64)] + [
        (n, C.c_uint64) for n in (
            "events", "ev_msg", "ev_timer", "ev_tester", "msgs_sent", "drop_clog", "drop_loss",
            "drop_overflow", "drop_deliver", "drop_stale", "elections", "leaders_elected",
            "applies", "snapshots", "installs", "entries_shipped", "max_inflight", "max_log",
            "max_index", "kv_ops", "kv_checked", "log_writes", "kv_lin_checked")]

    def to_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class Oracle:
    def __init__(self, path=LIB):
        if not os.path.exists(path):
            from madraft_amd import build
            build.build_oracle()
        L = C.CDLL(path)
        L.mro_run_cluster.argtypes = [C.POINTER(MrCfg), C.c_uint64, C.POINTER(MroResult),
                                      C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
        L.mro_run_cluster_dig.argtypes = [C.POINTER(MrCfg), C.c_uint64, C.POINTER(MroResult),
                                          C.c_void_p, C.c_void_p, C.c_size_t,
                                          C.POINTER(C.c_size_t)]
        L.mro_run_cluster_kv.argtypes = [C.POINTER(MrCfg), C.c_uint64, C.POINTER(MroResult),
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                         C.POINTER(C.c_size_t)]
        L.mro_run_batch.argtypes = [C.POINTER(MrCfg), C.c_uint64, C.c_uint64, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.POINTER(MroResult)]
        L.mro_philox4x32_10.argtypes = [C.POINTER(C.c_uint32 * 4), C.POINTER(C.c_uint32 * 2),
                                        C.POINTER(C.c_uint32 * 4)]
        L.mro_philox4x32_10.restype = None
        L.mro_cfg_init.argtypes = [C.POINTER(MrCfg), C.c_uint32]
        L.mro_set_decisions.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p,
                                        C.c_uint64, C.c_void_p]
        L.mro_scenario_from_name.argtypes = [C.c_char_p]
        L.mro_scenario_from_name.restype = C.c_uint32
        self.L = L

    def philox(self, ctr, key):
        c = (C.c_uint32 * 4)(*ctr)
        k = (C.c_uint32 * 2)(*key)
        o = (C.c_uint32 * 4)()
        self.L.mro_philox4x32_10(C.byref(c), C.byref(k), C.byref(o))
        return list(o)

    def cfg(self, test, **kw):
        """Oracle-side defaults (mirror of mr_cfg_init) + overrides, for CPU-only tests."""
        cfg = MrCfg()
        scn = self.L.mro_scenario_from_name(test.encode())
        assert scn, test
        assert self.L.mro_cfg_init(C.byref(cfg), scn) == 0
        flags = kw.pop("flags", 0)
        cfg.flags |= flags
        for k, v in kw.items():
            setattr(cfg, k, v)
        return cfg

    def run_cluster(self, cfg, cluster, trace_cap=0):
        r = MroResult()
        n = C.c_size_t()
        tr = np.empty(max(trace_cap, 1), EVENT_DTYPE)
        rc = self.L.mro_run_cluster(C.byref(cfg), int(cluster), C.byref(r),
                                    tr.ctypes.data if trace_cap else None, int(trace_cap),
                                    C.byref(n))
        assert rc == 0, "bad config"
        return r.to_dict(), tr[: min(n.value, trace_cap)] if trace_cap else None

    def run_cluster_dig(self, cfg, cluster, trace_cap):
        """run_cluster with each trace record's apply digest (ABI 4 mr_trace_digests)."""
        r = MroResult()
        n = C.c_size_t()
        tr = np.empty(max(trace_cap, 1), EVENT_DTYPE)
        dg = np.empty(max(trace_cap, 1), np.uint64)
        rc = self.L.mro_run_cluster_dig(C.byref(cfg), int(cluster), C.byref(r), tr.ctypes.data,
                                        dg.ctypes.data, int(trace_cap), C.byref(n))
        assert rc == 0, "bad config"
        m = min(n.value, trace_cap)
        return r.to_dict(), tr[:m], dg[:m]

    def run_cluster_kv(self, cfg, cluster, trace_cap):
        """run_cluster with the KV commands as applied (ABI 4 mr_trace_applies): (result,
        trace, applies[n, 2])."""
        r = MroResult()
        n = C.c_size_t()
        tr = np.empty(max(trace_cap, 1), EVENT_DTYPE)
        ap = np.zeros((max(trace_cap, 1), 2), np.uint64)
        rc = self.L.mro_run_cluster_kv(C.byref(cfg), int(cluster), C.byref(r), tr.ctypes.data,
                                       None, ap.ctypes.data, int(trace_cap), C.byref(n))
        assert rc == 0, "bad config"
        m = len(ap)
        while m and not ap[m - 1, 0]:
            m -= 1
        return r.to_dict(), tr[: min(n.value, trace_cap)], ap[:m]

    def recording(self, rows, cap):
        """Context: the following runs record every draw as a keyed decision (SEMANTICS §12);
        yields (count[rows], rec[rows, cap]) with row = cluster - cfg.cluster_base."""
        import contextlib

        @contextlib.contextmanager
        def ctx():
            count = np.zeros(rows, np.uint64)
            rec = np.zeros((rows, cap), DECISION_DTYPE)
            assert self.L.mro_set_decisions(2, None, 0, rows, rec.ctypes.data, cap,
                                            count.ctypes.data) == 0
            try:
                yield count, rec
            finally:
                self.L.mro_set_decisions(0, None, 0, 0, None, 0, None)
        return ctx()

    def replaying(self, decisions, rows):
        """Context: the following runs take their draws from `decisions` (DECISION_DTYPE,
        any order, cluster = row); yields misses[rows] (draws without a record)."""
        import contextlib

        @contextlib.contextmanager
        def ctx():
            d = np.ascontiguousarray(decisions, dtype=DECISION_DTYPE)
            misses = np.zeros(rows, np.uint64)
            rc = self.L.mro_set_decisions(1, d.ctypes.data if d.size else None, d.size, rows,
                                          None, 0, misses.ctypes.data)
            assert rc == 0, rc
            try:
                yield misses
            finally:
                self.L.mro_set_decisions(0, None, 0, 0, None, 0, None)
        return ctx()

    def run_batch(self, cfg, first, count):
        code = np.empty(count, np.uint16)
        t = np.empty(count, np.uint32)
        dig = np.empty(count, np.uint64)
        s = MroResult()
        rc = self.L.mro_run_batch(C.byref(cfg), int(first), int(count), code.ctypes.data,
                                  t.ctypes.data, dig.ctypes.data, C.byref(s))
        assert rc == 0, "bad config"
        return code, t, dig, s.to_dict()
