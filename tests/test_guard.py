"""The MR_GUARD debug library (verdict r4 item 6): every computed index into a per-cluster global
array — node records, message slots and payloads, log rings, tester storage, thread slots and
their scheduler keys, KV server records and snapshots, shard_ctrler configs / operations, the
churn clients' value slots, the linearizability counters and the LDS key rows — checked in the
kernel against its bound (mr_kernel.hip GI). A violation is recorded and mr_batch_run fails with
"MR_GUARD: index ... out of range" instead of the access faulting.

The GPU test runs the instances that use scratch or faulted before (count_2b, the churn tests at
5 and 8 servers — round 3's fault was step_kernel<18, 8> — every kvraft / shard_ctrler test) and
the headline on the guard library in a child process, and requires no violation and results
equal to the product library's (verdicts, times and trace digests).

Positive control (verdict r5 weak item 8): with MR_GUARD_PROBE set, the guard library reads one
message slot past the table (index M) at every message delivery of cluster 0; the run must fail
with that index, its bound, the message-slot tag and cluster 0 — through mr_batch_run and through
mr_batch_submit / mr_batch_finish (the bench's path) — and a reset clears the record: the same
batch then runs clean once the probe is off.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from madraft_amd import _abi, build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [(_abi.SCENARIOS[i], {}) for i in build.GUARD_SCNS] + [
    (_abi.SCENARIOS[i], {"nodes": 8}) for i in (16, 17, 18)]
CLUSTERS = 256

CHILD = r"""
import json, sys
import numpy as np
from madraft_amd import sim
out = []
for test, kw in json.loads(sys.argv[1]):
    with sim.Batch(test, %d, **kw) as b:
        b.run()
        code, t, dig = b.verdicts()
    out.append([test, kw, code.tolist(), t.tolist(), [int(d) for d in dig]])
    print("guard ok", test, kw, flush=True, file=sys.stderr)
print(json.dumps(out))
""" % CLUSTERS


PROBE_CHILD = r"""
import os, sys
from madraft_amd import sim
out = []
b = sim.Batch("figure_8_unreliable_2c", 64, iters=60)
for path in ("run", "submit"):
    os.environ["MR_GUARD_PROBE"] = "1"
    try:
        if path == "run":
            b.reset(7)
            b.run()
        else:
            b.submit(7)
            b.finish()
        out.append(path + ": no error")
    except sim.SimError as e:
        out.append(path + ": " + str(e))
os.environ.pop("MR_GUARD_PROBE")
b.reset(7)  # the probe is off and the reset clears the previous run's record
b.run()
code, _, _ = b.verdicts()
out.append("clean: %d of %d passed" % (int((code == 0).sum()), len(code)))
b.close()
print("\n".join(out))
"""


def test_guard_cases_have_instances():
    """every case names a scenario the guard library builds (an unbuilt one would fail the GPU
    test with 'no instance', not with a guard report)"""
    ids = {_abi.SCENARIOS.index(t) for t, _ in CASES}
    assert ids <= set(build.GUARD_SCNS)


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_guard_build_runs_clean(hip):
    assert os.path.exists(build.GUARD_LIB), "the MR_GUARD library is not built (build.build_guard)"
    env = dict(os.environ, MADRAFT_HIP_LIB=build.GUARD_LIB)
    p = subprocess.run([sys.executable, "-c", CHILD, json.dumps(CASES)], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=840)
    assert p.returncode == 0, p.stderr[-3000:]
    got = json.loads(p.stdout.strip().splitlines()[-1])
    for (test, kw, code, t, dig) in got:
        with hip.Batch(test, CLUSTERS, **kw) as b:
            b.run()
            rc, rt, rd = b.verdicts()
        assert np.array_equal(rc, code) and np.array_equal(rt, t), (test, kw)
        assert np.array_equal(rd, np.array(dig, np.uint64)), (test, kw)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_guard_reports_a_planted_violation(hip):
    """The guard is not vacuous: a planted out-of-range index is reported exactly (index M = 32
    message slots of figure_8_unreliable_2c, bound 32, tag G_MSG = 2, cluster 0) on both host
    paths, and a reset clears it."""
    assert os.path.exists(build.GUARD_LIB), "the MR_GUARD library is not built (build.build_guard)"
    env = dict(os.environ, MADRAFT_HIP_LIB=build.GUARD_LIB)
    env.pop("MR_GUARD_PROBE", None)
    p = subprocess.run([sys.executable, "-c", PROBE_CHILD], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    run, sub, clean = p.stdout.strip().splitlines()[-3:]
    want = "MR_GUARD: index 32 out of range 32 (tag 2, cluster 0)"
    assert run == "run: " + want, run
    assert sub == "submit: " + want, sub
    assert clean == "clean: 64 of 64 passed", clean
