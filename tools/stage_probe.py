"""Staging cost beside back-to-back MFMAs at ONE wave per SIMD (llp_stage_probe, csrc/probe.hip;
DESIGN.md §4.1): shader cycles per v_mfma_f32_32x32x16_bf16 when a wave also moves `pieces`
1-KiB operand pieces per 32 MFMAs by LDS-DMA (mode 1), by global_load_dwordx4 + ds_write_b128
(mode 2), or reads `pieces` ds_read_b128 fragments (mode 3).  A 256 x 256 NT GEMM tile with a
128 x 128 tile per wave moves 4 pieces per 16 MFMAs of this shape (8 per 32): the mode-1 / mode-2
rows at 8 pieces price its staging.  One JSON line per configuration."""
import ctypes as C
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
import llp_hip as K  # noqa: E402

L = K.lib()
L.llp_stage_probe.restype = C.c_int
L.llp_stage_probe.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                              C.c_void_p]
dev = torch.device("cuda", 0)
cus = torch.cuda.get_device_properties(0).multi_processor_count
g = torch.Generator(device="cpu").manual_seed(1)
out = torch.empty(cus * 256, dtype=torch.float32, device=dev)
cyc = torch.zeros(cus, dtype=torch.int64, device=dev)
iters = 2000
for src_mb in (4, 512):
    n_u4 = src_mb * (1 << 20) // 16
    src = (torch.randn(n_u4 * 8, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    for mode, pieces in [(0, 0), (1, 4), (1, 8), (1, 16), (2, 4), (2, 8), (2, 16), (3, 8), (3, 16)]:
        if src_mb != 4 and mode in (0, 3):
            continue
        ms = []
        for rep in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            K.check(L.llp_stage_probe(mode, pieces, src.data_ptr(), n_u4, iters, out.data_ptr(), cyc.data_ptr(),
                                      K.stream_ptr()), "llp_stage_probe")
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        c = cyc.cpu().double() / (iters * 32)
        flops = cus * 4 * iters * 32 * (32.0 * 32 * 16 * 2)
        print(json.dumps({"src_MB": src_mb, "mode": mode, "pieces_per_32_mfma": pieces,
                          "cycles_per_mfma_median": round(float(c.median()), 2),
                          "cycles_per_mfma_max": round(float(c.max()), 2), "ms": round(min(ms), 4),
                          "tflops": round(flops / min(ms) / 1e9, 1)}), flush=True)
