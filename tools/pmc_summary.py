"""Summarise rocprofv3 --pmc passes of ``bench.py --dominant-only N`` into
profiles/<round>_pmc_dominant.json, which bench.py reads for roofline.traffic.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md, HBM
section: on gfx950 FETCH_SIZE reports half the bytes of a wide streaming
read; WRITE_SIZE is exact for 16-B stores), averaged over the last N
dispatches of the dominant kernel (the first dispatches belong to the warm-up
step that fills the activations).

    python tools/pmc_summary.py --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write \
        --kernel gemm_nt_bf16_256p --last 10 --rows 747214 --H 1024 --dtype bf16 \
        --out profiles/r01_pmc_dominant.json
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def per_dispatch(root, counter, kernel):
    files = glob.glob(os.path.join(root, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {root}")
    vals = defaultdict(float)
    names = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter or kernel not in row.get("Kernel_Name", ""):
                    continue
                d = int(row["Dispatch_Id"])
                vals[d] += float(row["Counter_Value"])
                names[d] = row["Kernel_Name"]
    return [vals[d] for d in sorted(vals)], [names[d] for d in sorted(vals)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="gemm_nt_bf16_256p")
    ap.add_argument("--last", type=int, default=10)
    ap.add_argument("--rows", type=int, required=True)
    ap.add_argument("--H", type=int, required=True)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch, names = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    write, _ = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    fetch, write = fetch[-a.last:], write[-a.last:]
    # FETCH_SIZE / WRITE_SIZE are in KiB
    f_b = 1024.0 * sum(fetch) / len(fetch)
    w_b = 1024.0 * sum(write) / len(write)
    # bf16: A read + C write + W read + the ReLU bit mask the step's launch writes; fp32: A, C, W
    if a.dtype == "bf16":
        alg = 2.0 * a.rows * a.H * 2 + 2.0 * a.H * a.H + a.rows * a.H / 8.0
    else:
        alg = 2.0 * a.rows * a.H * 4 + 4.0 * a.H * a.H
    out = {"kernel": names[-1] if names else a.kernel, "rows": a.rows, "H": a.H, "dtype": a.dtype,
           "dispatches": len(fetch), "fetch_size_bytes": f_b, "write_size_bytes": w_b,
           "traffic_bytes_per_launch": 2.0 * f_b + w_b, "algorithmic_bytes": alg,
           "traffic_over_algorithmic": (2.0 * f_b + w_b) / alg,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; 2*FETCH_SIZE + WRITE_SIZE"}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
