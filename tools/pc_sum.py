"""Dev tool: summarise a rocprofv3 PC-sampling CSV (host_trap / stochastic) by source line
and by instruction class. usage: python tools/pc_sum.py <csv> [top]"""
import collections
import csv
import re
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 80
rows = csv.DictReader(open(path, newline=""))
cols = rows.fieldnames
print("columns:", cols)
by_line, by_op, by_inst = collections.Counter(), collections.Counter(), collections.Counter()
n = 0
for r in rows:
    n += 1
    if n <= 3:
        print("row", n, r)
    inst = r.get("Instruction") or r.get("instruction") or ""
    com = r.get("Instruction_Comment") or r.get("Instruction_comment") or ""
    m = re.search(r"([\w.]+):(\d+)", com)
    src = f"{m.group(1)}:{m.group(2)}" if m else (com[-60:] or "?")
    op = inst.split()[0] if inst else "?"
    cls = ("VALU" if op.startswith("v_") else "SALU" if op.startswith("s_waitcnt") and False else
           "WAIT" if op.startswith("s_waitcnt") else "SALU" if op.startswith("s_") else
           "VMEM" if op.startswith(("global_", "buffer_", "flat_")) else
           "LDS" if op.startswith("ds_") else op)
    by_line[src] += 1
    by_op[cls] += 1
    by_inst[op] += 1
print("samples", n)
for k, v in by_op.most_common():
    print(f"  {k:10s} {v:9d} {100 * v / max(n, 1):6.2f}%")
print("top instructions")
for k, v in by_inst.most_common(30):
    print(f"  {k:28s} {v:9d} {100 * v / max(n, 1):6.2f}%")
print("top source lines")
for k, v in by_line.most_common(top):
    print(f"  {k:40s} {v:9d} {100 * v / max(n, 1):6.2f}%")
