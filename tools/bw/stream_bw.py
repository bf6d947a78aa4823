"""Row-streaming memory-structure calibration (see stream_bw.hip).  Build:
hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/bw/libstream_bw.so tools/bw/stream_bw.hip"""
import ctypes, os, torch
so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libstream_bw.so")
L = ctypes.CDLL(so)
L.bw_stream.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64] * 2 + [ctypes.c_int] * 4 + [ctypes.c_void_p]
n, d = 1024, 1 << 20
x = torch.randn(n, d, device="cuda"); y = torch.empty_like(x); c = torch.empty((n, d), dtype=torch.int8, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
def t(fn, reps=10):
    for _ in range(3): r = fn(); assert not isinstance(r, int) or r == 0
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps
ms = t(lambda: y.copy_(x)); print(f"torch copy_ {ms:.3f} ms {8*n*d/ms/1e6:.0f} GB/s", flush=True)
for codes in (0, 1):
    for nt in (1, 0):
        for depth in (1, 2, 3, 4):
            for spin in (0, 8):
                ms = t(lambda: L.bw_stream(x.data_ptr(), y.data_ptr(), c.data_ptr(), n, d, depth, codes, nt, spin, sp))
                print(f"stream codes={codes} nt={nt} depth={depth} spin={spin}: {ms:.3f} ms {(8+codes)*n*d/ms/1e6:.0f} GB/s", flush=True)
