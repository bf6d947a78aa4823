"""Times tools/exp/chain_rate.hip: 131072 dependent fmas per lane (d = 2^20 / 8 torch lanes).
Build: cd tools/exp && hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared -o libchain_rate.so chain_rate.hip"""
import ctypes, json, os
import torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libchain_rate.so"))
out = torch.empty(256 * 64, device="cuda")
st = torch.cuda.current_stream().cuda_stream
res = {}
for mode in (0, 1):
    for blocks in (1, 256):
        f = lambda: lib.chain_rate(ctypes.c_void_p(out.data_ptr()), blocks, 131072, mode, ctypes.c_void_p(st))
        f(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); f(); e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        res[f"mode{mode}_blocks{blocks}"] = {"ms": round(ms, 4), "cycles_per_step_at_2.4GHz": round(ms * 1e-3 * 2.4e9 / 131072, 2)}
print(json.dumps(res))
