"""In-tree builds: the HIP product library (gfx950) and the CPU oracle.

`build_hip()` compiles madraft_amd/csrc/*.{hip,cpp} with hipcc into
madraft_amd/lib/libmadraft_hip.so (git-ignored, travels to the GPU box).
`build_oracle()` runs oracle/Makefile (test infrastructure only).
Both are incremental: they rebuild only when a source is newer than the output.
"""
import glob
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "lib", "libmadraft_hip.so")
# the MR_GUARD debug library (mr_kernel.hip GI: every computed per-cluster index checked): the
# instances that use scratch or faulted once — count_2b, the churn tests (round 3's 8-server
# fault was step_kernel<18, 8>), every kvraft / shard_ctrler test — and the headline
GUARD_LIB = os.path.join(HERE, "lib", "libmadraft_guard.so")
GUARD_SCNS = [10, 16, 17, 18] + list(range(25, 48))
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _stale(out, srcs, key=""):
    """`out` is missing, older than a source, or was built with other options than `key`
    (kept in `out`.flags: a library built with other -D flags is never taken for this one)."""
    if not os.path.exists(out):
        return True
    try:
        with open(out + ".flags") as f:
            if f.read() != key:
                return True
    except OSError:
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


# step-kernel instances (one per scenario id, mr_dev.h MR_ALL_SCNS) are split
# over several translation units of mr_kernel.hip compiled in parallel
SCN_IDS = list(range(1, 48))
N_GROUPS = 8
# scenarios whose kernels carry 256 message slots (snapshot_recover_many_clients_3b: up to
# 229 messages in flight with 20 clerks)
WIDE_SLOTS = {42}


# scenarios with a 7-server instance too (mr_dev.h has_nb7: the 2D tests, BASELINE config 4)
NB7_SCNS = {19, 20, 21, 22, 23}
# the scenarios' default server counts (mr_dev.h k_default_n): each scenario
# gets an instance sized for it (NB = 3 or 5) and one for up to 8 servers
DEFAULT_N = [0, 3, 3, 7, 5, 3, 5, 3, 3, 5, 3, 3, 5, 3, 5, 5, 5, 5, 5, 3, 3, 3, 3, 3, 5, 5, 5, 5, 3, 3, 5, 5, 5, 5, 5, 5, 5, 3, 5, 3, 3, 5, 5, 5, 5, 5, 7, 7]


def has_exact(i, nb):
    """mr_dev.h has_exact: an exact-size instance (NB = n < 8) of scenario i is built."""
    return nb < 8 and (DEFAULT_N[i] == nb or (i == 5 and nb == 5) or (i in NB7_SCNS and nb == 7))


# Raft-only test bodies without spawned threads (mr_dev.h has_pool): the pool-kernel instances
POOL_SCNS = set(range(1, 15)) | {16} | set(range(19, 25))
# the kvraft / shard_ctrler test bodies (mr_dev.h is_svc): the service pool (MR_POOL=2), all but
# the 20-clerk snapshot_recover_many_clients_3b (256 message slots)
SVC_SCNS = set(range(25, 48))
SVC_POOL_SCNS = SVC_SCNS - WIDE_SLOTS


def has_pool(i, nb):
    """mr_dev.h has_pool: a pool-kernel instance of scenario i at nb servers is built."""
    return has_exact(i, nb) and ((nb <= 7 and i in POOL_SCNS) or i in SVC_POOL_SCNS)


def _units(csrc, scns=None, tape=True):
    kern = os.path.join(csrc, "mr_kernel.hip")
    units = [(kern, "common", ["-DMR_COMMON=1", "-DMR_SCN_LIST=", "-DMR_NB=8"])]
    for nb in (3, 5, 7, 8):
        ids = [i for i in (scns or SCN_IDS) if nb == 8 or has_exact(i, nb)]
        if not ids:
            continue
        wide = [i for i in ids if i in WIDE_SLOTS]
        ids = [i for i in ids if i not in WIDE_SLOTS]
        ng = max(1, min(N_GROUPS, (len(ids) + 2) // 3)) if ids else 0
        # 7- and 8-server runs keep up to 64 messages in flight: 32-bit LDS keys halve the
        # key table so two waves per SIMD fit (config 4: +80 %)
        key = ["-DMR_KEY32=1"] if nb >= 7 else []
        for g in range(ng):
            lst = " ".join(f"MR_INST({i})" for i in ids[g::ng])
            units.append((kern, f"nb{nb}_{g}", ["-DMR_COMMON=0", f"-DMR_SCN_LIST={lst}",
                                                f"-DMR_NB={nb}", *key]))
        for i in wide:  # 256 message slots (mr_kernel.hip MR_MW)
            units.append((kern, f"nb{nb}_w{i}", ["-DMR_COMMON=0", f"-DMR_SCN_LIST=MR_INST({i})",
                                                 f"-DMR_NB={nb}", "-DMR_MW=4", *key]))
    for nb in (3, 5, 7):  # pool kernels: 32-bit keys; Raft-only / service
        for kind, pool in (("pool", 1), ("svcpool", 2)):
            ids = [i for i in (scns or SCN_IDS)
                   if has_pool(i, nb) and (i in SVC_POOL_SCNS) == (pool == 2)]
            ng = max(1, min(N_GROUPS, (len(ids) + 2) // 3)) if ids else 0
            for g in range(ng):
                lst = " ".join(f"MR_INST({i})" for i in ids[g::ng])
                units.append((kern, f"{kind}{nb}_{g}", ["-DMR_COMMON=0", f"-DMR_SCN_LIST={lst}",
                                                        f"-DMR_NB={nb}", "-DMR_KEY32=1",
                                                        f"-DMR_POOL={pool}"]))
    ids = list(scns or SCN_IDS) if tape else []  # decision-tape builds (SEMANTICS §12), NB = 8
    wide = [i for i in ids if i in WIDE_SLOTS]
    ids = [i for i in ids if i not in WIDE_SLOTS]
    ng = max(1, min(N_GROUPS, (len(ids) + 3) // 4)) if ids else 0
    for g in range(ng):
        lst = " ".join(f"MR_INST({i})" for i in ids[g::ng])
        units.append((kern, f"tape_{g}", ["-DMR_COMMON=0", "-DMR_TAPE=1", f"-DMR_SCN_LIST={lst}",
                                          "-DMR_NB=8"]))
    for i in wide:
        units.append((kern, f"tape_w{i}", ["-DMR_COMMON=0", "-DMR_TAPE=1",
                                           f"-DMR_SCN_LIST=MR_INST({i})", "-DMR_NB=8",
                                           "-DMR_MW=4"]))
    host = ["-DMR_DEV_SCNS=" + " ".join(f"MR_INST({i})" for i in scns)] if scns else []
    if not tape:
        host.append("-DMR_NO_TAPE=1")
    for src in sorted(glob.glob(os.path.join(csrc, "*.cpp"))):
        units.append((src, os.path.splitext(os.path.basename(src))[0], host))
    return units


def build_hip(force=False, verbose=False, extra=(), out=None, scns=None, csrc=None, tape=True):
    """Compile the product library; `extra` flags / `out` path / only scenario ids `scns` /
    another source tree `csrc` (a snapshot laid out as madraft_amd/csrc + include/) / no
    decision-tape kernels (`tape`) for dev variants."""
    out = out or LIB
    csrc = csrc or os.path.join(HERE, "csrc")
    srcs = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.cpp")))
    deps = srcs + glob.glob(os.path.join(csrc, "*.h")) + glob.glob(os.path.join(csrc, "*.inc")) + \
        [os.path.join(ROOT, "include", "madraft_sim.h"), os.path.abspath(__file__)]
    key = repr((list(extra), sorted(scns) if scns else None, bool(tape), os.path.abspath(csrc), ARCH))
    if not force and not _stale(out, deps, key):
        return out
    objdir = os.path.join(HERE, "lib", "obj" + ("_" + os.path.basename(out) if out != LIB else ""))
    os.makedirs(objdir, exist_ok=True)
    base = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall",
            "-Wno-unused-function", *extra]
    jobs, objs, running = [], [], []
    njobs = max(1, min(16, os.cpu_count() or 1))
    for src, name, flags in _units(csrc, scns, tape):
        obj = os.path.join(objdir, name + ".o")
        objs.append(obj)
        cmd = base + flags + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        while len(running) >= njobs:
            running = [p for p in running if p.poll() is None]
            if len(running) >= njobs:
                running[0].wait()
        p = subprocess.Popen(cmd)
        running.append(p)
        jobs.append((cmd, p))
    bad = [c for c, p in jobs if p.wait() != 0]
    if bad:
        raise RuntimeError("hipcc failed: " + " ".join(bad[0]))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    with open(out + ".flags", "w") as f:
        f.write(key)
    return out


def build_guard(force=False, verbose=False):
    """The MR_GUARD library (tests/test_guard.py), without decision-tape kernels."""
    return build_hip(force=force, verbose=verbose, extra=["-DMR_GUARD=1"], out=GUARD_LIB,
                     scns=GUARD_SCNS, tape=False)


def build_oracle(verbose=False):
    d = os.path.join(ROOT, "oracle")
    subprocess.run(["make", "-s", "-C", d], check=True,
                   stdout=None if verbose else subprocess.DEVNULL)
    return os.path.join(d, "_build", "libmr_oracle.so")


if __name__ == "__main__":
    print(build_hip(verbose=True))
    print(build_oracle(verbose=True))
