"""Timeline of the last profiled step of a rocprofv3 kernel trace (steps end at adam_kernel):
start offset, duration and the gap before each kernel, then busy / gap / span totals.
python tools/step_timeline.py TRACE.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
seg = rows[idx[-2] + 1:idx[-1] + 1]
t0 = int(seg[0]["Start_Timestamp"])
busy = gaps = 0.0
prev = None
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = (s - prev) / 1e3 if prev else 0.0
    gaps += max(g, 0.0)
    busy += (e - s) / 1e3
    name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} gap {g:6.1f}  {name[:70]}")
    prev = e
print(f"kernels {len(seg)} busy {busy:.1f} us gaps {gaps:.1f} us span {(prev - t0) / 1e3:.1f} us")
