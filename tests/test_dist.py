"""CPU: the N>1 path with world_size-2 gloo process groups.

Clusters shard across ranks with no data-path collective; the
only collective is the all-reduce of the batch counters at the end
(madraft_amd/dist.py). On CPU the oracle stands in for each rank's GPU batch
(the GPU tests show GPU == oracle per cluster); the all-reduced result of a
2-rank sharded run must equal the single-process run over all clusters, i.e.
results do not depend on the number of GPUs.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from madraft_amd import dist as mdist
from madraft_amd._abi import FAIL_NAMES

KEYS_SUM = ["events", "msgs_sent", "drop_loss", "applies", "elections"]
KEYS_MAX = ["max_inflight", "max_log", "max_index"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_partitions_exactly():
    for total in (1, 7, 131072, 1048576, 1000003):
        for world in (1, 2, 3, 8):
            parts = [mdist.shard(total, world, r) for r in range(world)]
            assert parts[0][0] == 0
            for (b0, n0), (b1, _) in zip(parts, parts[1:]):
                assert b0 + n0 == b1
            assert sum(n for _, n in parts) == total
            assert max(n for _, n in parts) - min(n for _, n in parts) <= 1


def _counters_of(oracle, cfg, first, count):
    code, _, _, s = oracle.run_batch(cfg, first, count)
    fails = np.nonzero(code != 0)[0]
    hist = {}
    for c in code.tolist():
        name = FAIL_NAMES[int(c)]
        hist[name] = hist.get(name, 0) + 1
    out = {k: 0 for k in mdist.SUM_KEYS + mdist.MAX_KEYS}
    out.update({k: int(s[k]) for k in KEYS_SUM + KEYS_MAX})
    out.update(clusters=count, done=count, passed=int((code == 0).sum()),
               failed=int((code != 0).sum()),
               first_fail_cluster=(first + int(fails[0])) if fails.size else mdist.NO_FAIL,
               first_fail_code=int(code[fails[0]]) if fails.size else 0,
               fail_hist=hist)
    return out


def _worker(rank, world, port, test, total, kw, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests.oracle_lib import Oracle
    o = Oracle()
    base, count = mdist.shard(total, world, rank)
    c = _counters_of(o, o.cfg(test, **kw), base, count)
    tot = mdist.allreduce_counters(c)
    t = mdist.allreduce_max(float(rank + 1))
    if rank == 0:
        q.put((tot, t))
    dist.destroy_process_group()


@pytest.mark.parametrize("test,total,kw", [
    ("figure_8_unreliable_2c", 24, dict(iters=200)),
    ("fail_agree_2b", 40, dict(n_nodes=5, flags=1)),  # config 2 shape, some seeds fail
])
def test_gloo_sharded_run_equals_single_process(oracle, test, total, kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, test, total, kw, q)) for r in range(2)]
    for p in ps:
        p.start()
    tot, tmax = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _counters_of(oracle, oracle.cfg(test, **kw), 0, total)
    for k in KEYS_SUM + ["clusters", "done", "passed", "failed"]:
        assert tot[k] == ref[k], k
    for k in KEYS_MAX:
        assert tot[k] == ref[k], k
    ff = ref["first_fail_cluster"]
    assert tot["first_fail_cluster"] == (None if ff == mdist.NO_FAIL else ff)
    assert tot["first_fail_code"] == ref["first_fail_code"]
    assert sum(tot["fail_hist"].values()) == total
    assert tmax == 2.0  # max over ranks of the per-rank time (bench.py)



def _pair_worker(rank, world, port, q):
    """Rank 0 fails first at a higher cluster id with code 6, rank 1 at a lower one with
    code 1: the reduced pair must be rank 1's (cluster, code), never mixed across ranks."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = {k: 0 for k in mdist.SUM_KEYS + mdist.MAX_KEYS}
    c.update(first_fail_cluster=[10, 3][rank], first_fail_code=[6, 1][rank], fail_hist={})
    c.update({k: 3 + rank for k in mdist.SUM_KEYS})  # every count: summed over the ranks
    tot = mdist.allreduce_counters(c)
    if rank == 0:
        q.put((tot["first_fail_cluster"], tot["first_fail_code"],
               {k: tot[k] for k in mdist.SUM_KEYS}))
    dist.destroy_process_group()


def test_first_fail_pair_reduced_together():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_pair_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[:2] == (3, 1)
    assert got[2] == {k: 7 for k in mdist.SUM_KEYS}


def test_every_count_of_the_abi_is_reduced():
    """every mr_counters field is summed (SUM_KEYS), taken as a maximum (MAX_KEYS),
    reduced as the first failure, or a histogram — none reaches the reduced dict as rank 0's
    local value (coop_entries, ABI 4, was)."""
    from madraft_amd._abi import MrCounters
    hist = {"fail_hist", "cov_leaders", "cov_events"}
    first = {"first_fail_cluster", "first_fail_code"}
    for name, _ in MrCounters._fields_:
        assert name in hist or name in first or name in mdist.SUM_KEYS or name in mdist.MAX_KEYS, name
