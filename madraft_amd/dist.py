"""Multi-GPU: clusters shard across ranks; one collective at the end.

Clusters (seeds) are independent — there is no inter-cluster traffic in any
in-scope test — so rank r of W owns the contiguous global
cluster range shard(total, W, r) and runs the identical kernel on it. Seeds
derive from global cluster ids, so results do not depend on W. The only
collective is one all-gather of each rank's counter vector at the end (about 1 KB per rank),
reduced on every rank: sum for counts, verdict and coverage histograms, max for maxima, min for
the first failing global cluster id — one latency-bound collective instead of one per reduction
op. With backend "nccl" it is RCCL over xGMI. Tests run the same code with gloo on CPU.
"""
import torch
import torch.distributed as dist

from ._abi import FAIL_NAMES

SUM_KEYS = ["clusters", "done", "passed", "failed", "events", "ev_msg", "ev_timer", "ev_tester",
            "msgs_sent", "drop_clog", "drop_loss", "drop_overflow", "drop_deliver", "drop_stale",
            "elections", "leaders_elected", "applies", "snapshots", "installs",
            "entries_shipped", "virt_time_us", "kv_ops", "kv_checked", "log_writes",
            "entries_materialized", "kv_lin_checked", "coop_entries"]
MAX_KEYS = ["max_inflight", "max_log", "max_index"]
COV_KEYS = ["cov_leaders", "cov_events"]
NO_FAIL = (1 << 63) - 1


def shard(total, world, rank):
    """(cluster_base, count) of `rank`'s contiguous share of `total` clusters."""
    q, r = divmod(int(total), int(world))
    base = rank * q + min(rank, r)
    return base, q + (1 if rank < r else 0)


def allreduce_counters(c, device=None, group=None):
    """All-reduce a counters dict (madraft_amd.sim.Batch.counters()) across ranks."""
    dev = device if device is not None else torch.device("cpu")
    s = torch.tensor([int(c[k]) for k in SUM_KEYS], dtype=torch.int64, device=dev)
    m = torch.tensor([int(c[k]) for k in MAX_KEYS], dtype=torch.int64, device=dev)
    # the first failing global cluster and ITS code, reduced as one key (cluster << 16 | code)
    # so the pair always comes from the same rank
    ff = c.get("first_fail_cluster", None)
    ff = NO_FAIL if ff is None or int(ff) >= (NO_FAIL >> 16) else \
        (int(ff) << 16) | (int(c.get("first_fail_code", 0)) & 0xFFFF)
    f = torch.tensor([ff], dtype=torch.int64, device=dev)
    names = sorted(FAIL_NAMES.items())
    code_of = {v: k for k, v in names}
    h = torch.zeros(len(names), dtype=torch.int64, device=dev)
    for name, v in c.get("fail_hist", {}).items():
        h[[k for k, _ in names].index(code_of[name])] = int(v)
    cov = torch.tensor([int(v) for k in COV_KEYS for v in c.get(k, [0] * 16)], dtype=torch.int64,
                       device=dev)
    s = torch.cat([s, h, cov])
    # one collective: every rank's [sums | maxima | first failure], reduced locally
    v = torch.cat([s, m, f])
    parts = [torch.empty_like(v) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, v, group=group)
    g = torch.stack(parts)
    ns, nm = s.numel(), m.numel()
    s = g[:, :ns].sum(dim=0)
    m = g[:, ns:ns + nm].max(dim=0).values
    f = g[:, ns + nm:].min(dim=0).values
    out = dict(c)
    sl = s.tolist()
    out["fail_hist"] = {name: int(v) for (_, name), v in zip(names, sl[len(SUM_KEYS):]) if v}
    base = len(SUM_KEYS) + len(names)
    for j, k in enumerate(COV_KEYS):  # coverage histograms
        out[k] = [int(v) for v in sl[base + 16 * j: base + 16 * (j + 1)]]
    out.update({k: int(v) for k, v in zip(SUM_KEYS, sl)})
    out.update({k: int(v) for k, v in zip(MAX_KEYS, m.tolist())})
    fv = int(f.item())
    out["first_fail_cluster"] = None if fv == NO_FAIL else fv >> 16
    out["first_fail_code"] = 0 if fv == NO_FAIL else fv & 0xFFFF
    return out


def allreduce_max(x, device=None, group=None):
    t = torch.tensor([float(x)], dtype=torch.float64,
                     device=device if device is not None else torch.device("cpu"))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
