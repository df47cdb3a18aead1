"""Where the head backward (colsum_vec_kernel) stands against plain streaming on the same
bytes: for each shape, median of 20 event-timed launches of
  head_bwd   -- llp_head_bwd: Z read, dZ written, dw / db column sums (the step's call)
  colsum     -- llp_colsum: Z read, column sums only (no dZ)
  copy       -- torch dZ.copy_(Z): read + write of the same bytes
  sum0       -- torch Z.sum(0, dtype=float32): read only
JSON lines {"shape", "kind", "ms", "tbps"} with tbps over the kind's own bytes
(read + write for head_bwd / copy, read for colsum / sum0).  Optional LLP_LIB A/B."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
import llp_hip as K  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for s, t in ev:
        s.record()
        fn()
        t.record()
    torch.cuda.synchronize()
    return sorted(s.elapsed_time(t) for s, t in ev)[n // 2]


def main():
    dev = torch.device("cuda", 0)
    shapes = [(603032, 1024), (400000, 256), (130000, 256)]
    if len(sys.argv) > 1:
        shapes = [tuple(int(v) for v in s.split("x")) for s in sys.argv[1:]]
    for R, H in shapes:
        g = torch.Generator(device="cpu").manual_seed(2)
        Z = torch.relu(torch.randn(R, H, generator=g)).to(torch.bfloat16).to(dev)
        dlogit = (torch.randn(R, generator=g) * 1e-3).to(dev)
        w = torch.randn(H, generator=g).to(dev)
        dZ = torch.empty_like(Z)
        dw = torch.empty(H, device=dev)
        db = torch.empty(1, device=dev)
        ws = torch.empty(K.head_bwd_ws_bytes(R, H) // 4 + 16, device=dev)
        nb = R * H * 2
        for kind, fn, by in (
                ("head_bwd", lambda: K.head_bwd(dlogit, Z, R, H, w, True, dZ, dw, db, ws), 2 * nb),
                ("colsum", lambda: K.colsum(Z, R, H, dw, ws), nb),
                ("copy", lambda: dZ.copy_(Z), 2 * nb),
                ("sum0", lambda: Z.sum(0, dtype=torch.float32), nb)):
            ms = timed(fn)
            print(json.dumps({"shape": [R, H], "kind": kind, "ms": ms, "tbps": by / ms / 1e9,
                              "lib": os.environ.get("LLP_LIB", "default")}), flush=True)


if __name__ == "__main__":
    main()
