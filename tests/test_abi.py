"""CPU: the C-ABI library loads and exports every symbol include/madraft_sim.h
declares; the ctypes mirror matches the C struct layout; host-only entry
points (no GPU needed) behave."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

from madraft_amd import _abi, build, sim

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "madraft_sim.h")


@pytest.fixture(scope="module")
def L():
    build.build_hip()
    return sim.lib()


def header_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(mr_\w+)\s*\(", txt, re.M)))


def test_exports_every_header_symbol(L):
    names = header_functions()
    assert set(names) == set(_abi.EXPORTS), names
    out = subprocess.run(["nm", "-D", "--defined-only", sim.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (mr_\w+)$", out, re.M))
    for n in names:
        assert n in exported, n
        assert hasattr(L, n)


def test_struct_layout_matches_c():
    src = f"""
#include <stdio.h>
#include <stddef.h>
#include "{HEADER}"
int main(void) {{
  printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(mr_cfg), sizeof(mr_counters), sizeof(mr_run_stats),
         sizeof(mr_event), offsetof(mr_cfg, device), offsetof(mr_counters, fail_hist));
  return 0;
}}"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-o", exe, c], check=True)
        got = list(map(int, subprocess.run([exe], capture_output=True, text=True,
                                           check=True).stdout.split()))
    assert got == [C.sizeof(_abi.MrCfg), C.sizeof(_abi.MrCounters), C.sizeof(_abi.MrRunStats),
                   _abi.EVENT_DTYPE.itemsize, _abi.MrCfg.device.offset,
                   _abi.MrCounters.fail_hist.offset]


def test_scenario_names_roundtrip(L):
    for i, n in enumerate(_abi.SCENARIOS):
        if not n:
            continue
        assert L.mr_scenario_from_name(n.encode()) == i
        assert L.mr_scenario_name(i).decode() == n
    assert L.mr_scenario_from_name(b"no_such_test") == 0


def test_cfg_init_defaults_match_oracle(L, oracle):
    for n in _abi.SCENARIOS:
        if not n:
            continue
        cfg = sim.make_cfg(n)
        ocfg = oracle.cfg(n)
        for f, _ in _abi.MrCfg._fields_:
            if f == "reserved":
                continue
            assert getattr(cfg, f) == getattr(ocfg, f), (n, f)
    assert sim.make_cfg("initial_election_2a").n_nodes == 3   # tests.rs:22
    assert sim.make_cfg("many_election_2a").n_nodes == 7      # tests.rs:82
    assert sim.make_cfg("figure_8_unreliable_2c").n_nodes == 5  # tests.rs:690


def test_fail_messages(L):
    assert sim.fail_message(1) == "expected one leader, got none"      # tester.rs:91
    assert sim.fail_message(7) == "test took longer than 120 seconds"  # tester.rs:356
    assert sim.fail_message(0) == "ok"


def test_bad_config_is_an_error_not_a_crash(L):
    cfg = sim.make_cfg("initial_election_2a")
    cfg.n_nodes = 9
    with pytest.raises(sim.SimError, match="n_nodes"):
        sim.Batch(cfg=cfg)
    cfg = sim.make_cfg("initial_election_2a")
    cfg.log_cap = 1000
    with pytest.raises(sim.SimError, match="log_cap"):
        sim.Batch(cfg=cfg)


def test_build_instance_tables_match_the_kernels():
    """build.py compiles the exact-size step-kernel instances mr_dev.h's has_exact() names (the
    host dispatches to them): the scenarios' default server counts and the 7-server set agree."""
    dev = open(os.path.join(ROOT, "madraft_amd", "csrc", "mr_dev.h")).read()
    body = re.search(r"k_default_n\[\]\s*=\s*\{([^}]*)\}", dev).group(1)
    assert [int(v) for v in body.replace("\n", " ").split(",")] == build.DEFAULT_N
    lo, hi = re.search(r"has_nb7\(uint32_t s\) \{\s*return s >= (\w+) && s <= (\w+);", dev).groups()
    hdr = open(HEADER).read()
    ids = {m.group(1): int(m.group(2)) for m in re.finditer(r"(MR_SCN_\w+) = (\d+)", hdr)}
    assert set(range(ids[lo], ids[hi] + 1)) == build.NB7_SCNS
    assert ids["MR_SCN_FAIL_AGREE_2B"] == 5 and build.has_exact(5, 5)  # BASELINE config 2
    for i in build.SCN_IDS:
        assert build.has_exact(i, build.DEFAULT_N[i]) == (build.DEFAULT_N[i] < 8)
        assert not build.has_exact(i, 8)
