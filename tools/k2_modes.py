"""K2 per-element cost in its two forms at scale: the small-batch kernels (n < 256 clients,
several workgroups per client) against the stream kernel (n >= 256, one workgroup per
client), d = 2^20, q + codes outputs.  Also times the L1 pass.

    python tools/k2_modes.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import uqdme
    from uqdme_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda")
    d = 1 << 20
    m = uqdme.rate_to_m(1, d)
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for n in (1, 2, 4, 8, 16, 32, 64, 128, 255, 256, 512):
        x = torch.randn(n, d, device=dev)
        q = torch.empty_like(x)
        codes = torch.empty((n, d), dtype=torch.int8, device=dev)
        ovf = torch.zeros(n, dtype=torch.int32, device=dev)
        X = torch.rand(n, device=dev)
        l1 = torch.empty(n, device=dev)
        nb = _lib.workspace_bytes(n, d, 1) if hasattr(_lib, "workspace_bytes") else None
        if nb is None:
            import ctypes
            b = ctypes.c_size_t()
            lib.uq_workspace_bytes(n, d, 1, ctypes.byref(b))
            nb = b.value
        ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
        P = lambda t: t.data_ptr()  # noqa: E731

        def l1p():
            _lib.check(lib.uq_l1_torch_order_f32(P(x), n, d, 1, P(l1), P(ws), nb, st), "l1")

        def k2():
            _lib.check(lib.uq_type_unbiased_codes_f32(P(x), P(q), P(codes), P(ovf), n, d, m, P(X), P(l1), None, 1,
                                                      P(ws), nb, st), "k2")
        out = {}
        for name, f in (("l1", l1p), ("k2", k2)):
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            out[name] = {"ms": round(ms, 4), "ns_per_elem": round(ms * 1e6 / (n * d), 5),
                         "GBs": round((4 if name == "l1" else 9) * n * d / ms / 1e6, 1)}
        res[n] = out
        del x, q, codes, ws
        torch.cuda.empty_cache()
    print(json.dumps({"tool": "k2_modes", "d": d, "results": res}))


if __name__ == "__main__":
    main()
