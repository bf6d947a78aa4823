"""K2 (q + codes) time across fresh allocations of x, q and codes inside ONE process: each trial
frees the buffers, empties torch's cache, holds a spacer allocation of a different size (so the
driver hands out other physical pages) and allocates x, q, codes again.  If the 1.76 / 1.98 ms
modes follow the allocation rather than the process, the slow mode is physical placement.
    python tools/exp/realloc.py"""
import ctypes, json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
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
    ovf = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for trial in range(12):
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        spacer = torch.empty((trial * 37 + 1) * MB, dtype=torch.uint8, device="cuda")
        order = trial % 3                     # allocation order: x q c / c q x / q c x
        bufs = {}
        for k in (("x", "q", "c"), ("c", "q", "x"), ("q", "c", "x"))[order]:
            bufs[k] = (torch.empty((n, d), device="cuda") if k != "c" else
                       torch.empty((n, d), dtype=torch.int8, device="cuda"))
        x, q, c = bufs["x"], bufs["q"], bufs["c"]
        torch.manual_seed(0)
        x.normal_()
        _lib.check(lib.uq_l1_torch_order_f32(x.data_ptr(), n, d, 1, l1.data_ptr(), ws.data_ptr(), b.value, st), "l1")
        f = lambda: lib.uq_type_unbiased_codes_f32(x.data_ptr(), q.data_ptr(), c.data_ptr(), ovf.data_ptr(), n, d, m,
                                                   X.data_ptr(), l1.data_ptr(), None, 1, ws.data_ptr(), b.value, st)
        for _ in range(2):
            _lib.check(f(), "k2")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        G = 1 << 30
        print(json.dumps({"trial": trial, "order": "xqc cqx qcx".split()[order], "spacer_MB": trial * 37 + 1,
                          "k2_ms": round(e0.elapsed_time(e1) / 5, 4),
                          "va_mod_1G": [t.data_ptr() % G for t in (x, q, c)]}), flush=True)
        del x, q, c, bufs, spacer


if __name__ == "__main__":
    main()
