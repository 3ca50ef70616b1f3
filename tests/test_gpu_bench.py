"""GPU: bench.py's contract on one MI355X — the single-rank JSON line, and the
N>1 path (two ranks sharing the card, counters all-reduced over gloo) giving
the same whole-job totals as one rank over the same clusters."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    r = subprocess.run(args, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def test_bench_single_rank_json():
    d = _run([sys.executable, "bench.py", "--steps", "1", "--warmup", "0", "--clusters", "4096",
              "--variant-steps", "1", "--no-cpu-baseline"])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["config"]["clusters_total"] == 4096
    assert d["value"] > 0 and d["pass_rate"] > 0.99 and d["drop_overflow"] == 0
    assert d["roofline"]["bound"] == "hbm" and 0 < d["roofline"]["frac"] < 1
    v = d["variants"]["figure_8_unreliable_crash"]
    assert v["value"] > 0 and v["pass_rate"] > 0.99


def test_bench_pipelined_steps_equal_sequential():
    """bench.py's pipelined steps (--pipeline 2, the default: two batches on two streams, step
    j + 1 submitted before step j is finished) run the same seeds to the same events and
    verdicts as one batch at a time (--pipeline 1); with overlapping launches the roofline is
    taken over the wall clock per step (roofline.time_base)."""
    args = [sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--clusters", "4096",
            "--variant", "", "--million", "0", "--no-cpu-baseline"]
    two, one = _run(args + ["--pipeline", "2"]), _run(args + ["--pipeline", "1"])
    for k in ("events_per_seed", "pass_rate"):
        assert two[k] == one[k], k
    assert two["roofline"]["alg_bytes_per_launch"] == one["roofline"]["alg_bytes_per_launch"]
    assert two["roofline"]["time_base"].startswith("wall clock")
    assert one["roofline"]["time_base"].startswith("HIP-event")


def test_bench_two_ranks_one_gpu():
    """`bench.py --gpus 2` starts torch.distributed.run itself; both ranks share
    the card, counters are all-reduced over gloo; cpu_baseline is an N = 1 figure only."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_PORT=str(port))
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--clusters", "2048", "--variant", "",
                        "--dist-backend", "gloo"], cwd=ROOT, capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["config"]["clusters_total"] == 4096
    assert d["scaling"] == "weak" and d["value"] > 0 and d["pass_rate"] > 0.99
    assert "cpu_baseline" not in d
    one = _run([sys.executable, "bench.py", "--steps", "1", "--warmup", "0", "--clusters", "4096",
                "--variant", "", "--no-cpu-baseline"])
    # same seeds (global cluster ids), so the same events whatever the rank count
    assert d["events_per_seed"] == one["events_per_seed"]


@pytest.mark.parametrize("budget", [None, "700"])
def test_submit_finish_pipeline_equals_run(budget, monkeypatch):
    """Two batches stepped as bench.py does (mr_batch_submit of step i+1 before
    mr_batch_finish of step i, each on its own stream) give every cluster's verdict,
    verdict time and trace digest, and the counters, of reset + run on one batch —
    also when clusters outlive the first launch (small MR_STEP_BUDGET)."""
    import numpy as np

    from madraft_amd import _abi, sim
    if budget:
        monkeypatch.setenv("MR_STEP_BUDGET", budget)
    test, n, seeds = "figure_8_unreliable_2c", 2048, [_abi.README_SEED + k * 7919 for k in range(3)]
    kw = dict(iters=200, safety=True)
    want = []
    with sim.Batch(test, n, **kw) as ref:
        for s in seeds:
            ref.reset(s)
            st = ref.run()
            assert st["remaining"] == 0
            want.append((ref.verdicts(), ref.counters()))
    bufs = [sim.Batch(test, n, **kw), sim.Batch(test, n, **kw)]
    try:
        got = []
        bufs[0].submit(seeds[0])
        for j in range(len(seeds)):
            if j + 1 < len(seeds):
                bufs[(j + 1) % 2].submit(seeds[j + 1])
            st, c = bufs[j % 2].finish()
            assert st["remaining"] == 0 and st["launches"] >= (2 if budget else 1)
            got.append((bufs[j % 2].verdicts(), c))
        with pytest.raises(sim.SimError):
            bufs[0].finish()  # nothing submitted
    finally:
        for b in bufs:
            b.close()
    for (wv, wc), (gv, gc) in zip(want, got):
        for x, y in zip(wv, gv):
            assert np.array_equal(x, y)
        assert wc == gc


def _nccl_worker(port, q):
    import torch
    import torch.distributed as dist

    from madraft_amd import dist as mdist
    from madraft_amd import sim
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)  # RCCL
    with sim.Batch("figure_8_unreliable_2c", 256, iters=50) as b:
        b.run()
        c = b.counters()
    tot = mdist.allreduce_counters(c, device=dev)
    t = mdist.allreduce_max(1.5, device=dev)
    dist.destroy_process_group()
    q.put(({k: tot[k] for k in ("events", "passed", "done", "max_inflight")},
           {k: c[k] for k in ("events", "passed", "done", "max_inflight")}, t))


def test_rccl_counter_allreduce_runs():
    """The multi-GPU collective path (bench.py with --dist-backend nccl) executed on the GPU
    box: RCCL all-reduce of a batch's counters on device tensors (world size 1 — one card),
    equal to the counters themselves."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(port, q))
    p.start()
    tot, c, t = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert tot == c and t == 1.5 and c["done"] == 256
