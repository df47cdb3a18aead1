"""Table of gpurun_out/epi_ab.json (tools/nt_epi_ab.py lines): per shape, ms / TF/s / checksum per env."""
import json

rows = [json.loads(l) for l in open("gpurun_out/epi_ab.json") if l.startswith("{")]
for n in rows[0]["res"]:
    print(n)
    for r in rows:
        x = r["res"][n]
        env = " ".join(f"{k[4:]}={v}" for k, v in sorted(r["env"].items()))
        print(f"   {env:40s} {x['ms']:.4f} ms {x['tflops']:6.0f} TF  sum={x['sum']}")
