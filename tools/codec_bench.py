"""Time the UQR1 type-message codec (uq_tc_encode / uq_tc_decode) on a resident batch of int8
type codes (C2 shape: 1024 clients x 2^20, R = 1 unless --bits), for rocprofv3 kernel stats.

    python tools/codec_bench.py [--clients N] [--dim D] [--bits R] [--steps K]"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=1024)
    ap.add_argument("--dim", type=int, default=1 << 20)
    ap.add_argument("--bits", type=float, default=1)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    import uqdme
    from uqdme_amd import _lib
    lib = _lib.load()
    n, d = a.clients, a.dim
    x = torch.randn(n, d, generator=torch.Generator(device="cuda").manual_seed(3), device="cuda")
    X = torch.rand(n, generator=torch.Generator().manual_seed(4))
    tc = uqdme.quantize_encode(x, a.bits, X=X, torch_threads=1)
    del x
    b, w = ctypes.c_size_t(), ctypes.c_size_t()
    _lib.check(lib.uq_tc_bound(d, ctypes.byref(b)), "bound")
    _lib.check(lib.uq_tc_workspace_bytes(n, d, ctypes.byref(w)), "ws")
    data = torch.empty(n * b.value, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    ws = torch.empty(w.value, dtype=torch.uint8, device="cuda")
    codes = torch.empty_like(tc.codes)
    l1 = torch.empty_like(tc.l1)
    km = torch.empty_like(tc.overflow)
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    P = lambda t: t.data_ptr()  # noqa: E731
    enc = lambda: _lib.check(lib.uq_tc_encode(P(tc.codes), P(tc.l1), n, d, tc.m, 0, P(data), data.numel(), P(off),  # noqa: E731
                                              P(ws), ws.numel(), sp), "encode")
    dec = lambda: _lib.check(lib.uq_tc_decode(P(data), data.numel(), P(off), n, d, tc.m, P(codes), P(l1), P(km), P(status), sp), "decode")  # noqa: E731
    res = {"clients": n, "d": d, "bits": a.bits}
    for name, f in (("encode", enc), ("decode", dec)):
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            f()
        e1.record()
        torch.cuda.synchronize()
        res[f"{name}_ms"] = round(e0.elapsed_time(e1) / a.steps, 4)
    res["bits_per_dim"] = round(8.0 * int(off[n].item()) / (n * d), 4)
    res["roundtrip_ok"] = bool(torch.equal(codes, torch.where(tc.codes == -1, torch.zeros_like(tc.codes), tc.codes))
                               and int(torch.count_nonzero(status).item()) == 0)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
