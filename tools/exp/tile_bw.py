"""Strided-tile copy bandwidth (tools/exp/tile_bw.hip) at the EDEN high pass's shape:
1024 vectors of 2^20 floats, rows at a 4096-float stride, 16384 floats per workgroup, row
segments of 64 floats (dword lanes, 256 rows: the product kernel's shape) or 64 / 128 / 256 /
1024 floats (float4 lanes), in place and into a second buffer.
Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/exp/tile_bw.hip -o tools/exp/libtile_bw.so"""
import ctypes, json, os, torch
L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libtile_bw.so"))
L.tile_bw.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                      ctypes.c_void_p]
n, D = 1024, 1 << 20
a = torch.randn(n, D, device="cuda")
b = torch.empty_like(a)
sp = torch.cuda.current_stream().cuda_stream
for stride in (4096,):
    for cols in (0, 64, 128, 256, 1024):
        for inplace in (1, 0):
            dst = a if inplace else b
            f = lambda: L.tile_bw(a.data_ptr(), dst.data_ptr(), n, D, stride, cols, sp)
            rc = f()
            if rc != 0:
                raise RuntimeError(f"tile_bw returned {rc}")
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                f()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 5
            print(json.dumps({"stride": stride, "cols": cols if cols else "64dw", "inplace": inplace, "ms": round(ms, 4),
                              "TBs": round(2 * a.numel() * 4 / ms / 1e9, 3)}), flush=True)
