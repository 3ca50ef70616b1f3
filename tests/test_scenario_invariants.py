"""Compile-time specialisations of the step kernel, checked against the oracle on CPU.

The step kernel compiles the InstallSnapshot branch of its send loop out of every scenario for
which `has_snaps(S)` is false (madraft_amd/csrc/mr_dev.h, mr_kernel.hip node_send_ae): there a
log is never compacted, so `nx <= snap` cannot hold. That is a claim about the scenarios, not
about the kernel, so it is checked here on the oracle: outside snap_common's five 2D tests
(raft/tests.rs:874-1010) and the kvraft tests with a maxraftstate (kvraft/tests.rs:494-522),
no node ever takes a snapshot or sends InstallSnapshot. The snapshot scenarios are checked for
the converse, so the counters are known to count.
"""
import pytest

from madraft_amd import _abi

SNAP_2D = {n for n in _abi.SCENARIOS if n.endswith("_2d")}
SNAP_KV = {"snapshot_rpc_3b", "snapshot_size_3b", "snapshot_recover_3b",
           "snapshot_recover_many_clients_3b", "snapshot_unreliable_3b",
           "snapshot_unreliable_recover_3b",
           "snapshot_unreliable_recover_concurrent_partition_3b",
           "snapshot_unreliable_recover_concurrent_partition_linearizable_3b"}
HAS_SNAPS = SNAP_2D | SNAP_KV
NO_SNAPS = [n for n in _abi.SCENARIOS if n and n not in HAS_SNAPS]


def _totals(oracle, test, clusters):
    _, _, _, s = oracle.run_batch(oracle.cfg(test), 0, clusters)
    return s


@pytest.mark.parametrize("test", NO_SNAPS)
def test_no_snapshot_outside_snapshot_scenarios(oracle, test):
    s = _totals(oracle, test, 64)
    assert s["events"] > 0
    assert s["snapshots"] == 0 and s["installs"] == 0, s


@pytest.mark.parametrize("test", sorted(HAS_SNAPS))
def test_snapshot_scenarios_take_snapshots(oracle, test):
    assert _totals(oracle, test, 4)["snapshots"] > 0
