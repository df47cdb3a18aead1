"""SQ counter pass of ``bench.py --dominant-only N`` (the student layer-2 forward NT GEMM)
into profiles/<round>_pmc_sq_dominant.json: where the waves' cycles go.

Counters (one rocprofv3 --pmc pass, 8 SQ + 1 GRBM): GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS
SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES, averaged over the last N dispatches.
  clock     = GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md, DVFS give-back)
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
  wave_*    = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
              (disjoint; park at s_waitcnt / barrier, issue stall, issuing)

    python tools/pmc_sq.py --dir gpurun_out/r03/pmc_sq --kernel gemm_nt_bf16_pp8p --last 10 \
        --rows 225334 --out profiles/r03_pmc_sq_dominant.json
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--kernel", default="gemm_nt_bf16_pp8p")
    ap.add_argument("--last", type=int, default=10)
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--H", type=int, default=1024)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(float))
    dur, name = {}, {}
    files = glob.glob(os.path.join(a.dir, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {a.dir}")
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                if a.kernel not in r["Kernel_Name"]:
                    continue
                d = int(r["Dispatch_Id"])
                vals[d][r["Counter_Name"]] += float(r["Counter_Value"])
                dur[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                name[d] = r["Kernel_Name"]
    ids = sorted(vals)[-a.last:]
    if not ids:
        raise SystemExit(f"no dispatch of {a.kernel}")
    raw = {c: sum(vals[d][c] for d in ids) / len(ids) for c in vals[ids[0]]}
    ns = sum(dur[d] for d in ids) / len(ids)
    clk = raw["GRBM_GUI_ACTIVE"] / 8 / (ns * 1e-9)
    wc = raw["SQ_WAVE_CYCLES"]
    out = {"kernel": name[ids[-1]].replace("void (anonymous namespace)::", "").split("((")[0], "dispatches": len(ids),
           "method": "rocprofv3 --pmc " + " ".join(sorted(raw)) + " (one pass), last %d dispatches" % len(ids),
           "duration_ms_profiled": ns / 1e6, "clock_ghz": clk / 1e9,
           "mfma_busy": raw["SQ_VALU_MFMA_BUSY_CYCLES"] / (raw["GRBM_GUI_ACTIVE"] / 8 * 1024),
           "wave_wait_any": raw["SQ_WAIT_ANY"] / wc, "wave_wait_inst_any": raw["SQ_WAIT_INST_ANY"] / wc,
           "wave_active_inst_any": raw["SQ_ACTIVE_INST_ANY"] / wc,
           "wave_wait_inst_lds": raw["SQ_WAIT_INST_LDS"] / wc,
           "lds_bank_conflict_cycles": raw["SQ_LDS_BANK_CONFLICT"], "raw": raw}
    if a.rows:
        out["rows"] = a.rows
        out["tflops_profiled"] = 2.0 * a.rows * a.H * a.H / (ns * 1e-9) / 1e12
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "raw"}))


if __name__ == "__main__":
    main()
