"""What a hipMemsetAsync node does under the segmented capture.

Round 2's segmented multi-rank hipGraph faulted at the collab size in the replay of
the unique-node compaction, whose count buffer was zeroed by hipMemsetAsync; with the
count zeroed by a kernel the same replays are bit-identical to eager steps
(tools/seg_diag.py).  This probe captures, as the segmented capture does (side stream,
shared pool, thread-local mode, a segment before it), one segment holding
hipMemsetAsync(buf, 0, n * 4) followed by a copy of the buffer, and checks at replay
that the copy reads zeros and that the guard words past the buffer are untouched.
buf sits at the start of a guard region 8x its size, so an overrun stays inside memory
this probe owns and is reported instead of faulting.

  python tools/memset_capture_probe.py
"""
import ctypes
import json

import torch


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetAsync.restype = ctypes.c_int
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    res = []
    for n in (2_000, 235_868, 2_000_000):
        for mode in ("thread_local", "global"):
            guard = torch.full((8 * n,), 7, dtype=torch.int32, device=dev)
            buf = guard[:n]
            out = torch.full((n,), -1, dtype=torch.int32, device=dev)
            x = torch.zeros(1024, device=dev)
            torch.cuda.synchronize()
            s = torch.cuda.Stream(device=dev)
            pool = torch.cuda.graph_pool_handle()
            s.wait_stream(torch.cuda.current_stream(dev))
            graphs = []
            with torch.cuda.stream(s):
                g1 = torch.cuda.CUDAGraph()
                g1.capture_begin(pool=pool, capture_error_mode=mode)
                x.add_(1.0)
                g1.capture_end()
                g2 = torch.cuda.CUDAGraph()
                g2.capture_begin(pool=pool, capture_error_mode=mode)
                rc = hip.hipMemsetAsync(buf.data_ptr(), 0, n * 4, s.cuda_stream)
                out.copy_(buf)
                g2.capture_end()
                graphs = [g1, g2]
            torch.cuda.current_stream(dev).wait_stream(s)
            torch.cuda.synchronize()
            rows = []
            for rep in range(3):
                guard.fill_(7)
                out.fill_(-1)
                torch.cuda.synchronize()
                for g in graphs:
                    g.replay()
                torch.cuda.synchronize()
                rows.append({"out_nonzero": int((out != 0).sum().item()),
                             "guard_touched": int((guard[n:] != 7).sum().item()),
                             "buf_nonzero": int((buf != 0).sum().item())})
            res.append({"n": n, "bytes": n * 4, "mode": mode, "memset_rc": rc, "replays": rows})
            print(json.dumps(res[-1]), flush=True)
            del graphs, g1, g2
    ok = all(r["out_nonzero"] == 0 and r["guard_touched"] == 0 for x in res for r in x["replays"])
    print(json.dumps({"memset_node_ok": ok}), flush=True)


if __name__ == "__main__":
    main()
