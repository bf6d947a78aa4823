"""torch.norm in torch's CPU order on the GPU: the sequential chains (KE2, mode 1) against the
segmented chains (KE2s, mode 2) per batch size, for the choice in uq_eden_norm_f32 / EDEN
(kSegNormMaxN).  Prints one JSON line per (D, n, mode): ms per call (HIP events, 10 calls)
and whether the two modes agree bit for bit.

    python tools/exp/norm_modes.py"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import uqdme  # noqa: E402,F401
from uqdme_amd import _lib  # noqa: E402

L = _lib.load()


def run(x, mode, reps=10):
    n, D = x.shape
    b = ctypes.c_size_t()
    _lib.check(L.uq_eden_norm_workspace_bytes(n, D, ctypes.byref(b)), "ws")
    ws = torch.empty(max(1, b.value), dtype=torch.uint8, device="cuda")
    out = torch.empty(n, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    f = lambda: _lib.check(L.uq_eden_norm_f32(x.data_ptr(), n, D, mode, out.data_ptr(), ws.data_ptr(),  # noqa: E731
                                              ws.numel(), sp), "norm")
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, out.clone()


def main():
    g = torch.Generator(device="cuda").manual_seed(5)
    for D, ns in ((1 << 20, (1, 16, 64, 128, 256, 512, 1024)), (1 << 22, (1, 16, 64, 256))):
        for n in ns:
            x = torch.randn(n, D, generator=g, device="cuda")
            t1, o1 = run(x, 1)
            row = {"D": D, "n": n, "chains_ms": round(t1, 4)}
            if n <= 256:
                t2, o2 = run(x, 2)
                row.update({"segmented_ms": round(t2, 4),
                            "bit_equal": bool(torch.equal(o1.view(torch.int32), o2.view(torch.int32)))})
            print(json.dumps(row), flush=True)
            del x


if __name__ == "__main__":
    main()
