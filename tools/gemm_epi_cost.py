"""Price of the persistent NT GEMM's epilogue: the M x 1024 x 1024 ReLU-forward launch
(random bf16 operands, event-timed medians) of the default library against diagnostic
builds without the epilogue's C stores (LLP_DIAG_EPI_NOSTORE), without any epilogue
(LLP_DIAG_EPI_SKIP) and with every store of a workgroup aliased onto the same 64 rows, so the
stores stay in L2 (LLP_DIAG_EPI_ALIAS: the stores' instructions without their HBM writes).  (A build whose workgroups started staggered by 1/2 or 1/4 tile, so
that their store bursts would not coincide, measured 1-2 % slower and was removed:
profiles/r03_gemm_epilogue_cost.json.)  Build here: python tools/gemm_epi_cost.py --build; run on the GPU."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "linkless-link-prediction_amd")
VARIANTS = {"nostore": ["LLP_DIAG_EPI_NOSTORE"], "skip": ["LLP_DIAG_EPI_SKIP"], "alias": ["LLP_DIAG_EPI_ALIAS"]}

if "--build" in sys.argv:
    sys.path.insert(0, PKG)
    import build_lib
    for name, defs in VARIANTS.items():
        build_lib.build_variant(os.path.join(REPO, "tools", "bin", f"libllp_hip_epi_{name}.so"), defs,
                                sources=("gemm256.hip",))
    sys.exit(0)

res = {}
for rnd in range(int(sys.argv[sys.argv.index('--rounds') + 1]) if '--rounds' in sys.argv else 2):
    for name in ["default"] + list(VARIANTS):
        env = dict(os.environ)
        if name != "default":
            env["LLP_LIB"] = os.path.join(REPO, "tools", "bin", f"libllp_hip_epi_{name}.so")
        out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "mfma_probe.py")], env=env,
                             capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(out.stdout, out.stderr, file=sys.stderr)
            sys.exit(1)
        d = json.loads(line[-1])["gemm_random"]
        res.setdefault(name, []).append(round(d["median_ms"], 4))
        print(name, rnd, d, flush=True)
print(json.dumps(res))
