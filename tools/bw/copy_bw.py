import ctypes, os, sys, torch
so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcopy_bw.so")
L = ctypes.CDLL(so)
L.bw_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
x = torch.randn(1024, 1 << 20, device="cuda"); y = torch.empty_like(x)
sp = torch.cuda.current_stream().cuda_stream
def t(fn, reps=10):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps
nbytes = 2 * x.numel() * 4
ms = t(lambda: y.copy_(x)); print(f"torch copy_      {ms:.3f} ms {nbytes/ms/1e6:.0f} GB/s")
for nt in (0, 1):
    for grid in (1024, 2048, 4096, 8192, 65536):
        ms = t(lambda: L.bw_copy(x.data_ptr(), y.data_ptr(), x.numel() // 4, nt, grid, sp))
        print(f"hip copy nt={nt} grid={grid:6d} {ms:.3f} ms {nbytes/ms/1e6:.0f} GB/s", flush=True)
ms = t(lambda: x.abs().sum(dim=1)); print(f"torch abs-sum rows {ms:.3f} ms {x.numel()*4/ms/1e6:.0f} GB/s read")
