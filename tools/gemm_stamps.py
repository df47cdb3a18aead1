"""Where a pp8 NT GEMM workgroup spends its cycles (diagnostic build with -DLLP_GEMM_STAMPS,
tools/bin/libllp_hip_stamps.so; build_lib.build_variant): per workgroup, s_memtime /
s_memrealtime at entry, after the prologue's first K-tile landed, after the main loop and
after the epilogue.  Prints per shape the medians over workgroups of the three spans in
shader cycles, the in-kernel clock (d memtime / d realtime x 100 MHz) and the main loop's
MFMA occupancy against its floor (2 waves per SIMD x K/64 K-tiles x 64 MFMAs x 16 cycles).

    python tools/gemm_stamps.py [--lib tools/bin/libllp_hip_stamps.so]
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(REPO, "tools", "bin", "libllp_hip_stamps.so"))
    ap.add_argument("--warm", type=int, default=40)
    opt = ap.parse_args()
    os.environ["LLP_LIB"] = opt.lib
    sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
    import numpy as np
    import torch
    import llp_hip as K
    L = K.lib()
    fn = L.llp_debug_gemm_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    out = []
    for name, M, N, Kd in (("student L2 fwd (dominant)", 225_334, 1024, 1024), ("predictor L1 fwd", 603_032, 1024, 1024),
                           ("student L1 fwd (K=128)", 225_334, 1024, 128)):
        A = torch.relu(torch.randn(M, Kd, device=dev, generator=g)).to(torch.bfloat16)   # ReLU output: half zeros
        W = (torch.randn(N, Kd, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev, generator=g) * 0.1
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        mask = torch.empty(M, N // 8, device=dev, dtype=torch.uint8)
        a_op, w_op = K.operand(A), K.operand(W)
        for _ in range(opt.warm):
            K.gemm_nt(a_op, w_op, M, N, Kd, C, K.LLP_BF16, bias=b, act=K.ACT_RELU, aux=mask)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        K.gemm_nt(a_op, w_op, M, N, Kd, C, K.LLP_BF16, bias=b, act=K.ACT_RELU, aux=mask)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e)
        tiles = -(-M // 256) * (N // 256)
        buf = np.zeros(tiles * 8, dtype=np.uint64)
        assert fn(buf.ctypes.data, tiles) == 0
        st = buf.reshape(tiles, 8).astype(np.int64)
        t = st[:, 0::2]
        r = st[:, 1::2]
        full = (t[:, 3] > 0) & (t[:, 2] > 0)
        pro, loop, epi = t[full, 1] - t[full, 0], t[full, 2] - t[full, 1], t[full, 3] - t[full, 2]
        clk = (t[full, 3] - t[full, 0]) / np.maximum(r[full, 3] - r[full, 0], 1) * 100e6
        floor = 2 * (Kd // 64) * 64 * 16
        span_rt = (r[full, 3].max() - r[full, 0].min()) / 100e6 * 1e3
        res = {"shape": name, "M": M, "N": N, "K": Kd, "event_ms": ms, "TFs": 2 * M * N * Kd / ms / 1e9,
               "tiles_stamped": int(full.sum()), "prologue_cyc": float(np.median(pro)),
               "loop_cyc": float(np.median(loop)), "epilogue_cyc": float(np.median(epi)),
               "clock_GHz": float(np.median(clk) / 1e9), "mfma_floor_cyc": floor,
               "loop_mfma_occupancy": floor / float(np.median(loop)),
               "tile_cyc": float(np.median(t[full, 3] - t[full, 0])), "realtime_span_ms": float(span_rt),
               "tiles_per_cu": tiles / 256}
        out.append(res)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
