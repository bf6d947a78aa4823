"""Full C2 batch: find clients whose sum(k) != m and compare them with the C oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import uqdme
from oracle import uq_oracle as O, uq_oracle_c as C
from tests import golden_data as G
d = 1 << 20; n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(n, d, generator=g, device="cuda")
X = uqdme.draw_uniforms(n, torch.Generator().manual_seed(1))
m = O.rate_to_m(1, d)
for rep in range(2):
    q, l1 = uqdme.quantize_dequantize(x, m=m, X=X, torch_threads=1, return_l1=True)
    torch.cuda.synchronize(); uqdme.check_status()
    k = torch.round(q.abs().double() * m / l1.double()[:, None])
    s = k.sum(dim=1)
    badc = torch.nonzero(s != m).flatten().tolist()
    print("rep", rep, "clients with sum(k)!=m:", len(badc), badc[:10], [float(s[i]) - m for i in badc[:10]], flush=True)
    for j in badc[:4]:
        xj = x[j].cpu().numpy()
        ref, rl = C.quantize_batch(xj[None], m, X[j:j+1].numpy(), 1)
        gj = q[j].cpu().numpy()
        bad = np.nonzero(gj.view(np.uint32) != ref[0].view(np.uint32))[0]
        print("  client", j, "X", float(X[j]), "l1", float(l1[j]), rl[0], "mismatch", len(bad), bad[:8], "tiles", np.unique(bad // 4096)[:10], flush=True)
        kr = np.round(np.abs(ref[0]).astype(np.float64) * m / rl[0]); print("  oracle sum k - m:", kr.sum() - m)
