"""Same-box A/B of whole library builds, by default on the dominant GEMM (tools/mfma_probe.py
--gemm, random bf16 operands, event-timed medians): python tools/ab_gemm.py NAME=LIB.so ...
[--rounds R] [--script tools/colsum_bench.py | bench.py --args "--no-eval ..."].  Each build runs in its own process (LLP_LIB),
interleaved over the rounds; the script's last JSON line gives median_ms (or bench.py's ms_per_step)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
args = [a for a in sys.argv[1:] if "=" in a]
rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 3
extra = ["--a-one-row"] if "--a-one-row" in sys.argv else []   # passed on to tools/mfma_probe.py
if "--args" in sys.argv:   # extra arguments for the script, one string (e.g. bench.py's --no-* switches)
    extra += sys.argv[sys.argv.index("--args") + 1].split()
script = sys.argv[sys.argv.index("--script") + 1] if "--script" in sys.argv else os.path.join("tools", "mfma_probe.py")
res = {}
for r in range(rounds):
    for a in args:
        name, lib = a.split("=", 1)
        env = dict(os.environ, LLP_LIB=os.path.join(REPO, lib))
        out = subprocess.run([sys.executable, os.path.join(REPO, script)] + extra, env=env,
                             capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(out.stdout, out.stderr, file=sys.stderr)
            sys.exit(1)
        d = json.loads(line[-1])
        d = d.get("gemm_random", d)
        if "runs" in d:   # tools/physics_bench.py: its last run
            d = d["runs"][-1]
        res.setdefault(name, []).append(round(d["median_ms"] if "median_ms" in d else d["ms_per_step"], 4))
        print(name, r, d, flush=True)
print(json.dumps(res))
