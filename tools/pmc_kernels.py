"""Counter bytes against algorithmic bytes for the memory-bound kernels of the collab
step and for the SAGE aggregate (profiles/r03_pmc_memory_kernels.json).

Inputs: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes (separate runs) and a
--kernel-trace of the same command.  Beyond-L2 bytes per dispatch = 2 x FETCH_SIZE +
WRITE_SIZE (MI355X_MICROARCH.md, HBM: on gfx950 FETCH_SIZE reports half the bytes of a
wide streaming read; Infinity-Cache hits are counted, so this is L2-miss traffic, an
upper bound on HBM bytes).  Per kernel: the average over its dispatches of the passes
(warm-up dispatches excluded with --skip), the trace's average duration, and
  counter_TBs = counter bytes / duration,   algorithmic_TBs = algorithmic bytes / duration,
each also as a fraction of the 8 TB/s HBM peak (and of the guide's 6.3 TB/s achievable).

    python tools/pmc_kernels.py step --fetch D1 --write D2 --trace D3 --unique 225334 --out F.json
    python tools/pmc_kernels.py sage --fetch D1 --write D2 --plan plan.json --out F.json
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

PEAK = 8.0e12
ACHIEVABLE = 6.3e12


def rows(root, pattern):
    files = glob.glob(os.path.join(root, "**", pattern), recursive=True)
    if not files:
        raise SystemExit(f"no {pattern} under {root}")
    out = []
    for fn in files:
        with open(fn) as f:
            out.extend(csv.DictReader(f))
    return out


def counters(root, counter):
    """Dispatch_Id -> (kernel name, summed counter value, duration ns)."""
    d = {}
    for r in rows(root, "*counter_collection*.csv"):
        if r["Counter_Name"] != counter:
            continue
        k = int(r["Dispatch_Id"])
        name, v, dur = d.get(k, (r["Kernel_Name"], 0.0, int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
        d[k] = (name, v + float(r["Counter_Value"]), dur)
    return d


def trace(root):
    return [(r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            for r in sorted(rows(root, "*kernel_trace*.csv"), key=lambda r: int(r["Start_Timestamp"]))]


def per_kernel(fetch, write, match):
    """Counter bytes per dispatch of kernels whose name contains ``match``, in dispatch order
    (FETCH_SIZE / WRITE_SIZE are reported in KiB)."""
    ids = sorted(k for k, v in fetch.items() if match in v[0])
    return [(fetch[k][0], 1024.0 * (2 * fetch[k][1] + write.get(k, ("", 0.0, 0))[1]), fetch[k][2]) for k in ids]


def short(name):
    """kernel name without the return type, namespace and parameter list"""
    return name.replace("void (anonymous namespace)::", "").split("(")[0]


def entry(name, algo, cbytes, ns, note=""):
    s = ns * 1e-9
    return {"kernel": name, "dispatches": len(cbytes), "avg_us": ns / 1e3,
            "algorithmic_bytes": algo, "counter_bytes": sum(cbytes) / len(cbytes),
            "counter_over_algorithmic": sum(cbytes) / len(cbytes) / algo,
            "algorithmic_TBs": algo / s / 1e12, "counter_TBs": sum(cbytes) / len(cbytes) / s / 1e12,
            "algorithmic_frac": algo / s / PEAK, "counter_frac": sum(cbytes) / len(cbytes) / s / PEAK,
            "counter_frac_of_achievable": sum(cbytes) / len(cbytes) / s / ACHIEVABLE, "note": note}


def step(a):
    B, C, P, H, Ht = a.B, a.C, a.P, a.H, a.Ht
    U, s = a.unique, 2
    BC, R2, L = B * C, B * C + 2 * P, 4 * P
    kernels = {
        # name fragment: (algorithmic bytes, what)
        "hadamard_rows_wave_kernel<unsigned short, 2, 4, 64>": (3 * R2 * H * s + 8 * R2,
            "predictor input h[i] * h[j]: 2 row reads + 1 write per pair row (h rows gathered from the U-row table)"),
        "hadamard_rows_wave_kernel<unsigned short, 1, 4, 32>": (3 * BC * Ht * s + 8 * BC,
            "teacher predictor input t_h[a] * t_h[c] (256 wide)"),
        "colsum_vec_kernel": (2 * R2 * H * s + 4 * R2,
            "head backward: read Z1, write dZ1, dw / db partials"),
        "hadamard_anchor_rows": (2 * BC * H * s + 4 * BC + B * H * s,
            "anchors' sum over contexts of dZ * h[ctx]: dZ context rows + h[ctx] rows, write B rows"),
        "hadamard_bwd_segments_wave_kernel": ((2 * BC + B + 2 * L) * H * s + U * H * s + 12 * (B * (C + 1) + L),
            "per unique node, its target rows in order: dZ row + partner h row (anchor rows: their sum), "
            "one dh row per node; descriptors"),
    }
    fetch, write = counters(a.fetch, "FETCH_SIZE"), counters(a.write, "WRITE_SIZE")
    tr = trace(a.trace) if a.trace else []
    res = []
    for frag, (algo, what) in kernels.items():
        cb = per_kernel(fetch, write, frag)[a.skip:]
        if not cb:
            continue
        durs = [d for n, d in tr if frag in n][a.skip:] or [x[2] for x in cb]
        res.append(entry(short(cb[0][0]), algo, [x[1] for x in cb], sum(durs) / len(durs), what))
    out = {"workload": "ogbl-collab LLP step, bf16", "B": B, "C": C, "P": P, "H": H, "unique_nodes": U,
           "bytes": "counter = 2 x FETCH_SIZE + WRITE_SIZE per dispatch (beyond-L2, MALL hits included)",
           "durations": "kernel trace of the same command (eager steps)" if tr else "PMC pass timestamps",
           "kernels": res}
    json.dump(out, open(a.out, "w"), indent=1)
    for r in res:
        print(f"{r['kernel'][:48]:48s} {r['avg_us']:7.1f} us  algo {r['algorithmic_bytes']/1e9:5.2f} GB "
              f"{r['algorithmic_TBs']:5.2f} TB/s  counter {r['counter_bytes']/1e9:5.2f} GB {r['counter_TBs']:5.2f} TB/s")


def sage(a):
    plan = None
    with open(a.plan) as f:
        for line in f:
            if line.startswith("{") and '"plan"' in line:
                plan = json.loads(line)
    fetch, write = counters(a.fetch, "FETCH_SIZE"), counters(a.write, "WRITE_SIZE")
    cb = per_kernel(fetch, write, "csr_agg")
    res, i = [], 0
    for p in plan["plan"]:
        seg = cb[i:i + p["launches"]][3:]     # the 3 warm-up launches of each configuration excluded
        i += p["launches"]
        name = short(seg[0][0]) if seg else "?"
        e = entry(name, p["algorithmic_bytes"], [x[1] for x in seg], p["ms"] * 1e6,
                  "x rows re-read ~E/N times; the Infinity Cache serves most of them")
        e.update({"order": p.get("order", "id"), "dtype": p["dtype"], "F": p["F"], "mode": p["mode"],
                  "compulsory_bytes": p["compulsory_bytes"], "counter_over_compulsory": e["counter_bytes"] / p["compulsory_bytes"],
                  "compulsory_frac": p["compulsory_bytes"] / (p["ms"] * 1e-3) / PEAK})
        res.append(e)
    out = {"workload": "SAGE mean aggregate over the synthetic ogbl-collab graph", "N": plan["N"], "E": plan["E"],
           "bytes": "counter = 2 x FETCH_SIZE + WRITE_SIZE per dispatch; algorithmic = every neighbour row "
                    "from memory (SURVEY §8d); compulsory = x, col, rowptr read once, out written once",
           "durations": "HIP events in the same run (tools/sage_bench.py --agg-only)", "configs": res}
    json.dump(out, open(a.out, "w"), indent=1)
    for r in res:
        print(f"{r['order']:8s} {r['dtype']} F={r['F']} {r['mode']}: {r['avg_us']:6.1f} us  algo {r['algorithmic_TBs']:5.2f} TB/s "
              f"counter {r['counter_bytes']/1e9:5.3f} GB {r['counter_TBs']:5.2f} TB/s "
              f"({r['counter_over_algorithmic']:.2f} of algo, {r['counter_over_compulsory']:.2f}x compulsory)")


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="what", required=True)
    s1 = sub.add_parser("step")
    s1.add_argument("--fetch", required=True)
    s1.add_argument("--write", required=True)
    s1.add_argument("--trace")
    s1.add_argument("--unique", type=int, required=True)
    s1.add_argument("--B", type=int, default=13110)
    s1.add_argument("--C", type=int, default=36)
    s1.add_argument("--P", type=int, default=65536)
    s1.add_argument("--H", type=int, default=1024)
    s1.add_argument("--Ht", type=int, default=256)
    s1.add_argument("--skip", type=int, default=2, help="dispatches per kernel to drop (warm-up steps)")
    s1.add_argument("--out", required=True)
    s2 = sub.add_parser("sage")
    s2.add_argument("--fetch", required=True)
    s2.add_argument("--write", required=True)
    s2.add_argument("--plan", required=True)
    s2.add_argument("--out", required=True)
    a = ap.parse_args()
    step(a) if a.what == "step" else sage(a)


if __name__ == "__main__":
    main()
