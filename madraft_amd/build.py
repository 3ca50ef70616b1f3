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
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _stale(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def build_hip(force=False, verbose=False):
    srcs = sorted(glob.glob(os.path.join(HERE, "csrc", "*.hip")) +
                  glob.glob(os.path.join(HERE, "csrc", "*.cpp")))
    deps = srcs + glob.glob(os.path.join(HERE, "csrc", "*.h")) + \
        glob.glob(os.path.join(HERE, "csrc", "*.inc")) + \
        [os.path.join(ROOT, "include", "madraft_sim.h")]
    if not force and not _stale(LIB, deps):
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-fPIC", "-shared", "-std=c++17",
           "-Wall", "-Wno-unused-function", *srcs, "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


def build_oracle(verbose=False):
    d = os.path.join(ROOT, "oracle")
    subprocess.run(["make", "-s", "-C", d], check=True,
                   stdout=None if verbose else subprocess.DEVNULL)
    return os.path.join(d, "_build", "libmr_oracle.so")


if __name__ == "__main__":
    print(build_hip(verbose=True))
    print(build_oracle(verbose=True))
