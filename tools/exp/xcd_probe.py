"""Times the XCD-resident skeleton (tools/exp/exp_xcd.hip) against the product's K1 + K2 on
the C2 batch (1024 x 2^20, q + codes), same process, same x, several alternations.
Kill criterion: the skeleton is an optimistic bound of the real
single-read kernel; if it is not faster than K1 + K2 here, the real form is not built.

Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
         -fno-gpu-flush-denormals-to-zero -o tools/exp/libexp_xcd.so tools/exp/exp_xcd.hip
Run:   python tools/exp/xcd_probe.py"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import uqdme
    from uqdme_amd import _lib
    lib = _lib.load()
    ex = ctypes.CDLL(os.path.join(ROOT, "tools", "exp", "libexp_xcd.so"))
    ex.exp_xcd.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                           ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                           ctypes.c_void_p]
    props = torch.cuda.get_device_properties(0)
    n, d = 1024, 1 << 20
    m = uqdme.rate_to_m(1, d)
    dev = torch.device("cuda")
    x = torch.randn(n, d, device=dev)
    X = torch.rand(n, device=dev)
    sh = uqdme.DMEPipeline(n, d, m=m, torch_threads=1)
    rep = sh.probe_outputs(x, X, candidates=8, min_candidates=8)
    q, codes = sh.q, sh.codes
    l1x = torch.empty(n, device=dev)
    ws = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def base():
        sh.l1_norms(x)
        sh.quantize(x, X)

    def xcd(mode):
        def f():
            rc = ex.exp_xcd(x.data_ptr(), q.data_ptr(), codes.data_ptr(), n, d, float(m), X.data_ptr(),
                            l1x.data_ptr(), ws.data_ptr(), mode, st)
            if rc != 0:
                raise RuntimeError(f"exp_xcd rc {rc}")
        return f

    def timeit(f, k=10):
        for _ in range(2):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(k):
            f()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / k, 4)

    res = {"device": props.name, "cus": props.multi_processor_count, "probe_k2_ms": rep["k2_ms_chosen"],
           "runs": []}
    err_off = 16 * 9 * 4
    for it in range(3):
        row = {"k1+k2": timeit(base)}
        for mode, name in ((0, "xcd_skeleton"), (1, "xcd_no_waits"), (2, "xcd_skeleton_2wg"), (3, "xcd_no_waits_2wg")):
            ws[:64].zero_()
            row[name] = timeit(xcd(mode))
            row[name + "_err"] = int(ws[err_off:err_off + 4].view(torch.int32).item())
        res["runs"].append(row)
        print(json.dumps(row), flush=True)
    # the team exchange works: the skeleton's L1 (plain f32 sum of the partials) vs torch
    ref = x.abs().sum(dim=1)
    for mode in (0, 2):
        l1x.zero_()
        xcd(mode)()
        torch.cuda.synchronize()
        res[f"l1_maxrel_mode{mode}"] = float(((l1x - ref).abs() / ref).max().item())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
