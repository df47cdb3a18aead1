"""Per-launch duration of bench.py's dominant kernel (student layer-2 forward
GEMM = the 2nd NT GEMM dispatch after each step's sampling kernel)
from a rocprofv3 --kernel-trace CSV, to check against bench.py's event timing.

    python tools/dominant_from_trace.py gpurun_out/prof_r02/bench_kernel_trace.csv [out.json] [kernel name prefix]
"""
import csv
import json
import sys

KERNEL = sys.argv[3] if len(sys.argv) > 3 else "gemm_nt_bf16_pp8"


def main():
    path = sys.argv[1]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    durs = []
    k = None
    for s, e, name in rows:
        if "context_walk_kernel" in name or "minibatch_sample_kernel" in name:
            k = 0
            continue
        if k is not None and KERNEL in name:
            k += 1
            if k == 2:
                durs.append(e - s)
    out = {"kernel": KERNEL + " (student layer-2 forward, 2nd NT launch of each step)",
           "launches": len(durs), "avg_ms": sum(durs) / len(durs) / 1e6 if durs else None,
           "median_ms": sorted(durs)[len(durs) // 2] / 1e6 if durs else None,
           "min_ms": min(durs) / 1e6 if durs else None, "max_ms": max(durs) / 1e6 if durs else None,
           "source": path}
    print(json.dumps(out))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
