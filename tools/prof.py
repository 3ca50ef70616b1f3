"""Section profile of step_kernel (dev tool): needs a library built with -DMR_PROF.

usage: MADRAFT_HIP_LIB=.../libmr_prof.so python tools/prof.py [test] [clusters] [nodes]
Runs one batch in a child process (the library prints MRPROF at batch destroy)
and prints wave cycles per kernel section (mr_kernel.hip P_*).
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root

NAMES = ["tail", "sel", "decode", "load", "drop", "rv_req", "rv_rep", "ae_req", "ae_rep",
         "is_req", "is_rep", "hb", "elect", "apply", "send", "store", "tester", "stepdown",
         "prologue", "epilogue", "s_setup", "s_net", "s_pay", "ae_probe", "ap_load", "ap_check", "ap_kv", "ap_pend"]

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    import torch  # noqa: F401  (HIP runtime first, as in bench.py)
    from madraft_amd.sim import Batch
    test, n = sys.argv[2], int(sys.argv[3])
    b = Batch(test, n, **({"nodes": int(sys.argv[4])} if len(sys.argv) > 4 else {}))
    st = b.run()
    code, _, _ = b.verdicts()
    print("run", st, "pass", int((code == 0).sum()), flush=True)
    b.close()
    sys.exit(0)

test = sys.argv[1] if len(sys.argv) > 1 else "figure_8_unreliable_2c"
n = sys.argv[2] if len(sys.argv) > 2 else "131072"
r = subprocess.run([sys.executable, __file__, "--child", test, n] + sys.argv[3:4], capture_output=True,
                   text=True)
print(r.stdout.strip())
line = [l for l in r.stderr.splitlines() if l.startswith("MRPROF")]
if r.returncode or not line:
    print(r.stderr[-2000:])
    sys.exit(1)
v = [int(t) for t in line[-1].split()[1:]]
tot = sum(v[:len(NAMES)])
print(f"total wave-time {tot / 1e8:.4g} s (100 MHz wall clock)")
for k, name in enumerate(NAMES):
    if v[k] or v[32 + k]:
        print(f"{name:10s} {v[k] / tot * 100:6.2f}%  marks {v[32 + k]:12d}  cyc/mark {v[k] / max(1, v[32 + k]):10.0f}")
if len(v) >= 95 and any(v[64:95]):  # pool_kernel: per kind (mr_pool.inc PK_*)
    for k in range(8):
        it, cl, cy = v[64 + k], v[72 + k], v[80 + k]
        if it:
            print(f"pool bin {k} iterations {it:10d}  clusters/iter {cl / it:5.1f}  "
                  f"cyc/iter {cy / it:7.0f}  cyc/event {cy / max(1, cl):6.1f}")
    print(f"pool idle spins {v[88]}  lost claims {v[89]}")
    if v[94]:  # sums over blocks: crossing times / block lifetimes
        print("pool tail: live < 384 / 256 / 64 / 8 at " +
              " / ".join(f"{v[90 + q] / v[94]:.3f}" for q in range(4)) + " of the block lifetime")
