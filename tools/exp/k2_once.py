"""K2 (q + codes) on the C2 batch, 6 launches, for PMC passes across processes:
    rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum ... -- python3 tools/exp/k2_once.py"""
import ctypes, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import uqdme  # noqa: E402
from uqdme_amd import _lib  # noqa: E402

lib = _lib.load()
n, d = 1024, 1 << 20
m = uqdme.rate_to_m(1, d)
x = torch.randn(n, d, device="cuda")
q = torch.empty_like(x)
codes = torch.empty((n, d), dtype=torch.int8, device="cuda")
ovf = torch.zeros(n, dtype=torch.int32, device="cuda")
X = torch.rand(n, device="cuda")
l1 = torch.empty(n, device="cuda")
b = ctypes.c_size_t()
lib.uq_workspace_bytes(n, d, 1, ctypes.byref(b))
ws = torch.zeros(b.value, dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
lib.uq_l1_torch_order_f32(x.data_ptr(), n, d, 1, l1.data_ptr(), ws.data_ptr(), b.value, st)
for _ in range(6):
    lib.uq_type_unbiased_codes_f32(x.data_ptr(), q.data_ptr(), codes.data_ptr(), ovf.data_ptr(), n, d, m, X.data_ptr(),
                                   l1.data_ptr(), None, 1, ws.data_ptr(), b.value, st)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    lib.uq_type_unbiased_codes_f32(x.data_ptr(), q.data_ptr(), codes.data_ptr(), ovf.data_ptr(), n, d, m, X.data_ptr(),
                                   l1.data_ptr(), None, 1, ws.data_ptr(), b.value, st)
e1.record()
torch.cuda.synchronize()
print(f"K2 {e0.elapsed_time(e1) / 5:.3f} ms  x {x.data_ptr():#x} q {q.data_ptr():#x} codes {codes.data_ptr():#x} "
      f"ws {ws.data_ptr():#x}", flush=True)
