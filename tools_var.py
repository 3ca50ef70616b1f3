"""Dev helper: build variant libraries of the step kernel for on-GPU A/B runs.

usage: python tools_var.py name:-DFLAG=1,-DOTHER=0 [name2:...] [--scns 16,19]
Writes madraft_amd/lib/var/<name>.so (only the listed scenario instances; default 16 =
figure_8_unreliable_2c). Variants build in parallel processes.
"""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

from madraft_amd import build


def one(spec, scns):
    name, _, flags = spec.partition(":")
    extra = [f for f in flags.split(",") if f]
    out = os.path.join(build.HERE, "lib", "var", name + ".so")
    build.build_hip(extra=extra, out=out, scns=scns)
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    scns = [16]
    if "--scns" in args:
        i = args.index("--scns")
        scns = [int(s) for s in args[i + 1].split(",")]
        del args[i:i + 2]
    with ProcessPoolExecutor(max_workers=min(4, len(args))) as ex:
        for out in ex.map(one, args, [scns] * len(args)):
            print(out, flush=True)
