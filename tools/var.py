"""Dev helper: build variant libraries of the step kernel for on-GPU A/B runs.

usage: python tools/var.py name:-DFLAG=1,-DOTHER=0 [name2:...] [--scns 16,19] [--rev GITREV]
(--rev: build from that commit's sources, snapshotted under build/src_<rev>/)
Writes madraft_amd/lib/var/<name>.so (only the listed scenario instances; default 16 =
figure_8_unreliable_2c). Variants build in parallel processes.
"""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from madraft_amd import build


def snapshot(rev):
    """madraft_amd/csrc + include/ of commit `rev` under build/src_<rev>/ (for A/B against it)."""
    import subprocess
    root = os.path.dirname(build.HERE)
    dst = os.path.join(root, "build", f"src_{rev}")
    if not os.path.exists(dst):
        os.makedirs(dst)
        tar = subprocess.run(["git", "-C", root, "archive", rev, "madraft_amd/csrc", "include"],
                             check=True, capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", dst], input=tar, check=True)
    return os.path.join(dst, "madraft_amd", "csrc")


def one(spec, scns, csrc=None):
    name, _, flags = spec.partition(":")
    extra = [f for f in flags.split(",") if f]
    out = os.path.join(build.HERE, "lib", "var", name + ".so")
    build.build_hip(force=True, extra=extra, out=out, scns=scns, csrc=csrc)
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    scns = [16]
    if "--scns" in args:
        i = args.index("--scns")
        scns = [int(s) for s in args[i + 1].split(",")]
        del args[i:i + 2]
    csrc = None
    if "--rev" in args:
        i = args.index("--rev")
        csrc = snapshot(args[i + 1])
        del args[i:i + 2]
    with ProcessPoolExecutor(max_workers=min(4, len(args))) as ex:
        for out in ex.map(one, args, [scns] * len(args), [csrc] * len(args)):
            print(out, flush=True)
