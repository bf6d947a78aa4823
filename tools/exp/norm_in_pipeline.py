"""Why does EDEN's norm take ~1.1 ms inside the compress pipeline but ~0.87 ms standalone?
Runs the product compress (rocprof shows its eden_norm_kernel), then the experiment norm
(tools/exp/exp_norm_pitch.hip, product flags) on the SAME rotated vectors in the product's
workspace, right after the compress.
    rocprofv3 --kernel-trace --stats -- python3 tools/exp/norm_in_pipeline.py   (GPU box)"""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    import uqdme
    from uqdme_amd import quantizer
    L = ctypes.CDLL(os.path.join(HERE, "libexp_norm_pitch_pf.so"))
    L.exp_norm_pitch.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_void_p]
    L.exp_norm_nc.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                              ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    n, D = 1024, 1 << 20
    x = torch.randn(n, D, generator=torch.Generator(device="cuda").manual_seed(3), device="cuda")
    seeds = torch.randint(0, 100, (n,), generator=torch.Generator().manual_seed(5))
    uqdme.eden_compress(x, 1, seeds=seeds)
    torch.cuda.synchronize()
    ws = next(iter(quantizer._ws_cache.values()))
    vptr = ws.data_ptr() + 256                                 # EdenLayout.vec_off = kCtrlBytes
    nrm = torch.empty(n, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    for rep in range(6):
        uqdme.eden_compress(x, 1, seeds=seeds)
        for nc in (4, 44):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if L.exp_norm_nc(vptr, n, D, D, nrm.data_ptr(), 0, nc, sp) != 0:
                raise RuntimeError("launch failed")
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"rep": rep, "variant": "ahead2" if nc == 44 else "ahead1",
                              "exp_norm_on_pipeline_vectors_ms": round(e0.elapsed_time(e1), 4)}), flush=True)
    # the same vectors copied to a fresh buffer
    v2 = torch.empty(n * D, device="cuda")
    v2.copy_(torch.from_blob if False else ws[256:256 + n * D * 4].view(torch.float32))
    for rep in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        L.exp_norm_pitch(v2.data_ptr(), n, D, D, nrm.data_ptr(), 0, sp)
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"rep": rep, "exp_norm_on_copied_vectors_ms": round(e0.elapsed_time(e1), 4)}), flush=True)


if __name__ == "__main__":
    main()
