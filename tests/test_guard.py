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
