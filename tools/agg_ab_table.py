"""Summarise tools/gpu_call.sh agg-ab output: per library and aggregate configuration, the best
time over the rounds and its compulsory-byte fraction of 8 TB/s."""
import collections
import json
import sys


def main(path):
    best = collections.defaultdict(lambda: float("inf"))
    comp = {}
    libs = []
    for line in open(path):
        d = json.loads(line)
        lib = d["lib"].split("/")[-1]
        if lib not in libs:
            libs.append(lib)
        for p in d["run"]["plan"]:
            key = (p["dtype"], p["F"], p["mode"])
            best[(lib, key)] = min(best[(lib, key)], p["ms"])
            comp[key] = p["compulsory_bytes"]
    keys = sorted(comp)
    print("config".ljust(18) + "".join(f"{lib[:22]:>24}" for lib in libs))
    for key in keys:
        row = f"{key[0]} F={key[1]} {key[2]}".ljust(18)
        for lib in libs:
            ms = best[(lib, key)]
            row += f"{ms * 1e3:>12.1f}us {comp[key] / (ms * 1e-3) / 8e12:>7.3f}c"
        print(row)


if __name__ == "__main__":
    main(sys.argv[1])
