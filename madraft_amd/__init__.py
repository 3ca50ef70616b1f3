"""madraft_amd — MI355X-native batched deterministic simulator for MadRaft's lab tests.

Runs tens of thousands to millions of independent seeds of a reference test
(src/raft/tests.rs) in lockstep on CDNA4 through the C ABI of
include/madraft_sim.h (libmadraft_hip.so). See DESIGN.md.
"""
from ._abi import MR_PASS, MR_RUNNING, README_SEED, SCENARIOS, FAIL_NAMES  # noqa: F401
from .sim import Batch, make_cfg, run_test, fail_message, SimError  # noqa: F401

__all__ = ["Batch", "make_cfg", "run_test", "fail_message", "SimError", "SCENARIOS"]
