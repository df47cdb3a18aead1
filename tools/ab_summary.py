"""ms/step of the A/B runs written by tools/gpu_lib_ab.sh (gpurun_out/ab_{new,old}_*.json);
another prefix as the first argument (e.g. hl for tools/gpu_head_lean.sh)."""
import glob
import json
import sys

pre = sys.argv[1] if len(sys.argv) > 1 else "ab"
for arm in ("new", "old"):
    v = []
    for f in sorted(glob.glob(f"gpurun_out/{pre}_{arm}_*.json")):
        for line in open(f):
            if line.startswith("{"):
                v.append(json.loads(line)["ms_per_step"])
    print(arm, " ".join(f"{x:.3f}" for x in v), f"median {sorted(v)[len(v) // 2]:.3f}" if v else "")
