"""EDEN norm (experiment copy, product flags) with 1, 2 or 4 clients per workgroup at
1024 x 2^20, after the loader fix (tools/exp/exp_norm_pitch.hip exp_norm_nc).
    python tools/exp/norm_nc.py   (GPU box)"""
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    L = ctypes.CDLL(os.path.join(HERE, "libexp_norm_pitch_pf.so"))
    L.exp_norm_nc.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                              ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    n, D = 1024, 1 << 20
    v = torch.randn(n, D, generator=torch.Generator(device="cuda").manual_seed(7), device="cuda")
    ref = None
    sp = torch.cuda.current_stream().cuda_stream
    for nc in (44, 444, 44, 444, 44, 444):
        nrm = torch.empty(n, device="cuda")
        f = lambda: L.exp_norm_nc(v.data_ptr(), n, D, D, nrm.data_ptr(), 0, nc, sp)  # noqa: E731
        for _ in range(2):
            if f() != 0:
                raise RuntimeError("launch failed")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        ref = nrm.clone() if ref is None else ref
        print(json.dumps({"clients_per_wg": nc % 10, "loads_ahead": {4: 1, 44: 2, 444: 3}[nc], "ms": round(ms, 4), "TB_s": round(n * D * 4 / ms / 1e9, 3),
                          "norms_equal": bool(torch.equal(nrm, ref))}), flush=True)


if __name__ == "__main__":
    main()
