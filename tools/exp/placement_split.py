"""Which allocation decides K2's two speeds: the input x or the outputs (q, codes)?

    phase "outputs": x allocated once; q and codes freed and re-allocated behind a spacer of
                     a different size in every trial (the driver hands out other pages)
    phase "input":   q and codes allocated once; x re-allocated the same way
K2 (q + codes, C2 batch) is timed per trial; q-only beside it.  If only the outputs'
placement moves K2 between 1.7 and 2.0 ms, a placement-checked output pool can keep the
fast mode; if x's does, nothing on the library side can.
    python tools/exp/placement_split.py   (GPU box)"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main(trials=10):
    import uqdme
    from uqdme_amd import _lib
    lib = _lib.load()
    n, d = 1024, 1 << 20
    m = uqdme.rate_to_m(1, d)
    MB = 1 << 20
    X = torch.rand(n, device="cuda")
    l1 = torch.empty(n, device="cuda")
    b = ctypes.c_size_t()
    lib.uq_workspace_bytes(n, d, 1, ctypes.byref(b))
    ws = torch.zeros(b.value, dtype=torch.uint8, device="cuda")
    km = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def timed(f, reps=5):
        for _ in range(2):
            _lib.check(f(), "k2")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / reps, 4)

    def newx():
        x = torch.empty((n, d), device="cuda")
        torch.manual_seed(0)
        x.normal_()
        return x

    bufs = {"x": newx(), "q": torch.empty((n, d), device="cuda"), "c": torch.empty((n, d), dtype=torch.int8, device="cuda")}
    _lib.check(lib.uq_l1_torch_order_f32(bufs["x"].data_ptr(), n, d, 1, l1.data_ptr(), ws.data_ptr(), b.value, st), "l1")
    for phase, moving in (("outputs", ("q", "c")), ("input", ("x",))):
        for trial in range(trials):
            for k in moving:
                bufs[k] = None
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            spacer = torch.empty((trial * 37 + 1) * MB, dtype=torch.uint8, device="cuda")
            for k in moving:
                bufs[k] = newx() if k == "x" else (torch.empty((n, d), device="cuda") if k == "q" else
                                                   torch.empty((n, d), dtype=torch.int8, device="cuda"))
            x, q, c = bufs["x"], bufs["q"], bufs["c"]
            k2 = lambda: lib.uq_type_unbiased_codes_f32(x.data_ptr(), q.data_ptr(), c.data_ptr(), km.data_ptr(), n, d, m,  # noqa: E731
                                                        X.data_ptr(), l1.data_ptr(), None, 1, ws.data_ptr(), b.value, st)
            qo = lambda: lib.uq_type_unbiased_f32(x.data_ptr(), q.data_ptr(), n, d, m, X.data_ptr(), l1.data_ptr(),  # noqa: E731
                                                  None, 1, ws.data_ptr(), b.value, st)
            print(json.dumps({"phase": phase, "trial": trial, "spacer_MB": trial * 37 + 1, "k2_ms": timed(k2),
                              "q_only_ms": timed(qo), "k2_ms_again": timed(k2),
                              "va_GB": [round(t.data_ptr() / 2 ** 30, 3) for t in (x, q, c)]}), flush=True)
            del spacer, x, q, c
    _lib.check(lib.uq_check_status(ws.data_ptr(), st), "status")


if __name__ == "__main__":
    main()
