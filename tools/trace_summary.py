"""Per-kernel launch count and duration (avg / min / max, µs) from rocprofv3
--kernel-trace CSVs, for the kernels whose name contains one of the filters:

    python tools/trace_summary.py gpurun_out/trace_a gpurun_out/trace_b -k hadamard_bwd dedup

Each argument is a directory holding t_kernel_trace.csv (the layout the tools/gpu_*.sh
scripts write) or a CSV path.  Used to turn A/B traces into the summaries kept under
profiles/."""
import argparse
import collections
import csv
import os


def load(path):
    f = path if path.endswith(".csv") else os.path.join(path, "t_kernel_trace.csv")
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        name = name[5:] if name.startswith("void ") else name
        name = name.split("(")[0].replace(" ", "")
        out[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("traces", nargs="+")
    ap.add_argument("-k", "--kernels", nargs="*", default=[])
    a = ap.parse_args()
    print("# trace  kernel  launches  avg_us  min_us  max_us")
    for t in a.traces:
        d = load(t)
        for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
            if a.kernels and not any(k in name for k in a.kernels):
                continue
            print(os.path.basename(t.rstrip("/")), name, len(v), round(sum(v) / len(v) / 1e3, 1),
                  round(min(v) / 1e3, 1), round(max(v) / 1e3, 1))


if __name__ == "__main__":
    main()
