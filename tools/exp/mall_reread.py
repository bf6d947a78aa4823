"""Cold read vs immediate re-read of one buffer (default vs non-temporal loads), sizes around
the 256 MB Infinity Cache.  A re-read well above HBM rate means the MALL served it.
Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/exp/mall_reread.hip -o tools/exp/libmall_reread.so"""
import ctypes, json, os, torch
L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmall_reread.so"))
L.mall_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
sp = torch.cuda.current_stream().cuda_stream
out = torch.zeros(1, device="cuda")
flush = torch.ones(1 << 29, device="cuda")          # 2 GiB
big = torch.ones(1 << 28, device="cuda")            # 1 GiB pool, sliced
grid = 4096


def read(t, nt):
    L.mall_read(t.data_ptr(), t.numel() // 4, nt, grid, out.data_ptr(), sp)


for nt in (0, 1):
    for mb in (16, 32, 64, 128, 192, 256, 384, 512, 1024):
        buf = big[: mb * (1 << 18)]
        res = []
        for rep in range(5):
            read(flush, 1)
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            read(buf, nt)
            e[1].record()
            read(buf, nt)
            e[2].record()
            torch.cuda.synchronize()
            res.append((e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2])))
        cold = min(r[0] for r in res)
        warm = min(r[1] for r in res)
        nb = buf.numel() * 4
        print(json.dumps({"nt": nt, "MB": mb, "cold_ms": round(cold, 4), "warm_ms": round(warm, 4),
                          "cold_GBs": round(nb / cold / 1e6), "warm_GBs": round(nb / warm / 1e6)}), flush=True)
