"""Per-kernel averages of rocprofv3 --pmc counter_collection CSVs under the given
directories (last N dispatches of each kernel whose name contains FILTER).

    python tools/pmc_table.py FILTER DIR [DIR ...] [--last N]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(root, filt):
    vals = defaultdict(lambda: defaultdict(float))
    name = {}
    for fn in glob.glob(os.path.join(root, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            if filt not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            vals[d][r["Counter_Name"]] += float(r["Counter_Value"])
            name[d] = r["Kernel_Name"]
    return vals, name


def main():
    args = sys.argv[1:]
    last = 3
    if "--last" in args:
        i = args.index("--last")
        last = int(args[i + 1])
        del args[i:i + 2]
    filt, dirs = args[0], args[1:]
    for d in dirs:
        vals, name = load(d, filt)
        ds = sorted(vals)[-last:]
        if not ds:
            print(d, "no dispatches")
            continue
        keys = sorted({k for x in ds for k in vals[x]})
        avg = {k: sum(vals[x][k] for x in ds) / len(ds) for k in keys}
        print(d, name[ds[-1]][:60], " ".join(f"{k}={v:.4g}" for k, v in avg.items()))


if __name__ == "__main__":
    main()
