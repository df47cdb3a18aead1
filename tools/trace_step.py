"""Per-kernel time of the last profiled steps of a rocprofv3 kernel trace (steps end at
adam_kernel): python tools/trace_step.py TRACE.csv [TRACE_B.csv]"""
import csv
import sys
from collections import defaultdict


def steps(path, n=5):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    per = defaultdict(float)
    span = 0.0
    for a, b in zip(idx[-n - 1:-1], idx[-n:]):
        seg = rows[a + 1:b + 1]
        span += (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
        for k, r in enumerate(seg):
            name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            per[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return {k: v / n for k, v in per.items()}, span / n


a, sa = steps(sys.argv[1])
b, sb = (steps(sys.argv[2]) if len(sys.argv) > 2 else ({}, 0.0))
for k in sorted(set(a) | set(b), key=lambda k: -max(a.get(k, 0), b.get(k, 0))):
    print(f"{a.get(k, 0):9.1f} {b.get(k, 0):9.1f} us  {k[:90]}")
print(f"step span {sa:.1f} {sb:.1f} us")
