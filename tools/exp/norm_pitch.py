"""Experiment driver for tools/exp/exp_norm_pitch.hip (EDEN norm vs row pitch, 1024 x 2^20).
    python tools/exp/norm_pitch.py   (GPU box; the .so is built in the container)"""
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    import sys
    L = ctypes.CDLL(os.path.join(HERE, sys.argv[1] if len(sys.argv) > 1 else "libexp_norm_pitch.so"))
    L.exp_norm_pitch.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_void_p]
    n, D = 1024, 1 << 20
    ref = None
    big_a = torch.empty(1 << 30, device="cuda")              # 4 GiB streamed before each timed norm,
    big_b = torch.empty(1 << 30, device="cuda")              # as the high pass precedes it in EDEN
    for extra, off, pad, pre in ((0, 0, 0, False), (0, 0, 0, True), (4096 + 64, 0, 0, True)):
        ld = D + extra                                    # off: row 0 starts `off` floats into the buffer
        buf = torch.randn(n * ld + off, generator=torch.Generator(device="cuda").manual_seed(5), device="cuda")
        v = buf[off:].view(n, ld)
        v[:, :D] = torch.randn(n, D, generator=torch.Generator(device="cuda").manual_seed(7), device="cuda")
        nrm = torch.empty(n, device="cuda")
        sp = torch.cuda.current_stream().cuda_stream
        f = lambda: L.exp_norm_pitch(v.data_ptr(), n, D, ld, nrm.data_ptr(), pad, sp)  # noqa: E731
        for _ in range(2):
            if f() != 0:
                raise RuntimeError("launch failed")
        torch.cuda.synchronize()
        tot = 0.0
        for _ in range(5):
            if pre:
                big_b.copy_(big_a)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            tot += e0.elapsed_time(e1)
        ms = tot / 5
        ref = nrm.clone() if ref is None else ref
        print(json.dumps({"pitch_extra_floats": extra, "base_offset_bytes": 4 * off, "pad_lds": pad, "after_4GiB_copy": pre,
                          "ms": round(ms, 4), "TB_s": round(n * D * 4 / ms / 1e9, 3),
                          "norms_equal": bool(torch.equal(nrm, ref))}), flush=True)
        del buf, v


if __name__ == "__main__":
    main()
