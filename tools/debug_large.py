"""Debug helper: compare one large golden spec on the GPU with the C oracle, print the
mismatch pattern (positions, tiles, values) and the protocol status."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import uqdme
from oracle import uq_oracle as O, uq_oracle_c as C
from tests import golden_data as G
for sp, _, pos, qs in G.spec_vectors(large=True):
    if sp["d"] != int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22:
        continue
    x = G.spec_gen(sp)
    m = O.rate_to_m(sp["R"], sp["d"])
    ref, rl1 = C.quantize_batch(x[None], m, [sp["X"]], sp["threads"])
    for rep in range(3):
        got, l1 = uqdme.quantize_dequantize(torch.from_numpy(x[None]).cuda(), m=m, X=[sp["X"]],
                                            torch_threads=sp["threads"], return_l1=True)
        torch.cuda.synchronize()
        try:
            uqdme.check_status(); st = "ok"
        except Exception as e:
            st = str(e)
        g = got[0].cpu().numpy()
        bad = np.nonzero(g.view(np.uint32) != ref[0].view(np.uint32))[0]
        print(sp["dist"], sp["d"], sp["R"], sp["threads"], "rep", rep, "status", st, "l1", l1.item(), rl1[0],
              "mismatches", len(bad), "sha_ok", G.sha(g) == sp["q_sha256"])
        if len(bad):
            tiles = np.unique(bad // 4096)
            print("  first", bad[:12], "tiles", tiles[:20], "ntiles", len(tiles))
            print("  got", g[bad[:6]], "ref", ref[0][bad[:6]])
