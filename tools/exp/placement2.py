"""K2 (q + codes) against the placement of x, q and codes (views into pools at byte offsets),
all in one process, plus the virtual addresses (mod 1 GiB) of each configuration.
    python tools/exp/placement2.py"""
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
    xpool = torch.empty(n * d * 4 + 512 * MB, dtype=torch.uint8, device="cuda")
    qpool = torch.empty(n * d * 4 + 512 * MB, dtype=torch.uint8, device="cuda")
    cpool = torch.empty(n * d + 512 * MB, dtype=torch.uint8, device="cuda")
    src = torch.randn(n, d, device="cuda")
    X = torch.rand(n, device="cuda")
    l1 = torch.empty(n, device="cuda")
    b = ctypes.c_size_t()
    lib.uq_workspace_bytes(n, d, 1, ctypes.byref(b))
    ws = torch.zeros(b.value, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ovf = torch.zeros(n, dtype=torch.int32, device="cuda")
    _lib.check(lib.uq_l1_torch_order_f32(src.data_ptr(), n, d, 1, l1.data_ptr(), ws.data_ptr(), b.value, st), "l1")

    def t(xo, qo, co, codes=True):
        xp, qp, cp = xpool.data_ptr() + xo, qpool.data_ptr() + qo, cpool.data_ptr() + co
        torch.cuda.synchronize()
        ctypes.memmove  # noqa
        xv = xpool[xo:xo + n * d * 4].view(torch.float32).view(n, d)
        xv.copy_(src)
        f = lambda: lib.uq_type_unbiased_codes_f32(xp, qp, cp if codes else None, ovf.data_ptr(), n, d, m,
                                                   X.data_ptr(), l1.data_ptr(), None, 1, ws.data_ptr(), b.value, st)
        for _ in range(2):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / 5, 4)

    G = 1 << 30
    print(json.dumps({"xpool": xpool.data_ptr() % G, "qpool": qpool.data_ptr() % G, "cpool": cpool.data_ptr() % G}), flush=True)
    res = {}
    for xo in (0, 2 * MB, 64 * MB, 256 * MB + 4096):
        for qo in (0, 128 * MB + 4096, 384 * MB):
            for co in (0, 192 * MB + 8192):
                res[f"x+{xo // MB}M_q+{qo // MB}M_c+{co // MB}M"] = t(xo, qo, co)
        print(json.dumps(res), flush=True)
    res["ctrl_q_only_x+0"] = t(0, 0, 0, codes=False)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
