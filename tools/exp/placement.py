"""K2 (q + codes) time against the relative placement of its three streams (x read, q and
codes written): q and codes are views into pools at chosen byte offsets.  Checks whether
the box-to-box / process-to-process spread of K2 (1.76 vs 1.98 ms) comes from placement.
    python tools/exp/placement.py"""
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
    x = torch.randn(n, d, device="cuda")
    X = torch.rand(n, device="cuda")
    l1 = torch.empty(n, device="cuda")
    b = ctypes.c_size_t()
    lib.uq_workspace_bytes(n, d, 1, ctypes.byref(b))
    ws = torch.zeros(b.value, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ovf = torch.zeros(n, dtype=torch.int32, device="cuda")
    MB = 1 << 20
    qpool = torch.empty(n * d * 4 + 64 * MB, dtype=torch.uint8, device="cuda")
    cpool = torch.empty(n * d + 64 * MB, dtype=torch.uint8, device="cuda")
    _lib.check(lib.uq_l1_torch_order_f32(x.data_ptr(), n, d, 1, l1.data_ptr(), ws.data_ptr(), b.value, st), "l1")
    print(json.dumps({"x": x.data_ptr() % (1 << 30), "qpool": qpool.data_ptr() % (1 << 30), "cpool": cpool.data_ptr() % (1 << 30)}), flush=True)

    def t(qo, co):
        qp, cp = qpool.data_ptr() + qo, cpool.data_ptr() + co
        f = lambda: lib.uq_type_unbiased_codes_f32(x.data_ptr(), qp, cp, ovf.data_ptr(), n, d, m, X.data_ptr(),
                                                   l1.data_ptr(), None, 1, ws.data_ptr(), b.value, st)
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

    res = {}
    for qo in (0, 4096, 64 * 1024, 1 * MB, 2 * MB + 4096, 8 * MB, 33 * MB):
        for co in (0, 2 * MB + 8192):
            res[f"q+{qo}_c+{co}"] = t(qo, co)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
