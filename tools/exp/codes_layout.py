"""Runs tools/exp/exp_codes_layout.hip: K2 (q + codes) with row-major codes (the product
kernel) and with tile-major codes, on the same buffers, across fresh allocations of x, q and
codes in one process (as tools/exp/realloc.py: the two-speed mode follows the allocation).
Also times q only.  Checks that the tile-major codes are the row-major codes permuted.
    python tools/exp/codes_layout.py   (GPU box; build the .so first, see the .hip header)"""
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
    ex = ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libexp_codes_layout.so"))
    ex.exp_k2_tile_major.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 3 + [ctypes.c_void_p] * 3
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

    for trial in range(trials):
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        spacer = torch.empty((trial * 37 + 1) * MB, dtype=torch.uint8, device="cuda")
        x = torch.empty((n, d), device="cuda")
        q = torch.empty((n, d), device="cuda")
        c = torch.empty((n, d), dtype=torch.int8, device="cuda")
        torch.manual_seed(trial)
        x.normal_()
        _lib.check(lib.uq_l1_torch_order_f32(x.data_ptr(), n, d, 1, l1.data_ptr(), ws.data_ptr(), b.value, st), "l1")
        row = lambda: lib.uq_type_unbiased_codes_f32(x.data_ptr(), q.data_ptr(), c.data_ptr(), km.data_ptr(), n, d, m,  # noqa: E731
                                                     X.data_ptr(), l1.data_ptr(), None, 1, ws.data_ptr(), b.value, st)
        tm = lambda: ex.exp_k2_tile_major(x.data_ptr(), q.data_ptr(), c.data_ptr(), km.data_ptr(), n, d, m,  # noqa: E731
                                          X.data_ptr(), l1.data_ptr(), st)
        qo = lambda: lib.uq_type_unbiased_f32(x.data_ptr(), q.data_ptr(), n, d, m, X.data_ptr(), l1.data_ptr(),  # noqa: E731
                                              None, 1, ws.data_ptr(), b.value, st)
        r = {"trial": trial, "spacer_MB": trial * 37 + 1,
             "row_major_ms": timed(row), "tile_major_ms": timed(tm), "row_major_ms_2": timed(row),
             "tile_major_ms_2": timed(tm), "q_only_ms": timed(qo)}
        if trial == 0:
            _lib.check(row(), "k2")
            cr = c.clone()
            _lib.check(tm(), "k2")
            t = d // 4096
            r["tile_major_is_permutation"] = bool(torch.equal(cr.view(n, t, 4096).transpose(0, 1).reshape(-1), c.view(-1)))
            del cr
        print(json.dumps(r), flush=True)
        del x, q, c, spacer
    _lib.check(lib.uq_check_status(ws.data_ptr(), st), "status")


if __name__ == "__main__":
    main()
