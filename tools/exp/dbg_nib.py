"""Debug: first mismatches between the codes4 pipeline's nibbles and the int8 codes."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import uqdme

n, d, bits = 300, 8192, 1
g = torch.Generator(device="cuda").manual_seed(22)
x = torch.randn(n, d, generator=g, device="cuda")
X = torch.rand(n, generator=torch.Generator().manual_seed(5)).cuda()
r8 = uqdme.DMEPipeline(n, d, bits, torch_threads=1, pipeline="codes")
r8.step(x, X)
p = uqdme.DMEPipeline(n, d, bits, torch_threads=1, pipeline="codes4")
p.step(x, X)
torch.cuda.synchronize()
nib = p.nib
lo = (nib & 0xF).to(torch.int16)
hi = (nib >> 4).to(torch.int16)
v = torch.stack([lo, hi], dim=-1).reshape(n, -1)
v = torch.where(v >= 8, v - 16, v)
c8 = r8.codes.to(torch.int16)
bad = (v != c8).nonzero()
print("kmax max", int(p.kmax.max()), "mismatches", bad.shape[0])
for j, i in bad[:20].tolist():
    print(j, i, "nib", int(v[j, i]), "int8", int(c8[j, i]), "byte", hex(int(nib[j, i // 2])), "kmax", int(p.kmax[j]))
print("int8", c8[0, :48].tolist())
print("nib ", v[0, :48].tolist())
print("int8 t1", c8[0, 4096:4096 + 32].tolist())
print("nib  t1", v[0, 4096:4096 + 32].tolist())
est4 = p.step(x, X).clone()
est8 = r8.step(x, X).clone()
print("est equal", bool(torch.equal(est4, est8)))
