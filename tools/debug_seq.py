"""Reproduce the test sequence (mid specs then large specs in one process) and print the
ticket counter / status words after each call plus mismatch details."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import uqdme
from uqdme_amd import quantizer as Q
from oracle import uq_oracle as O, uq_oracle_c as C
from tests import golden_data as G

def ctrl():
    key = (0, torch.cuda.current_stream().cuda_stream)
    ws = Q._ws_cache[key]
    return ws[:8].view(torch.int32).cpu().tolist(), ws.numel(), ws.data_ptr()

def run(sp, pos=None, qs=None, poison=False):
    x = G.spec_gen(sp)
    m = O.rate_to_m(sp["R"], sp["d"])
    if poison:
        for ws in Q._ws_cache.values():
            ws.random_(0, 255)
    got = uqdme.quantize_dequantize(torch.from_numpy(x[None]).cuda(), m=m, X=[sp["X"]], torch_threads=sp["threads"])
    torch.cuda.synchronize()
    c = ctrl()
    g = got[0].cpu().numpy()
    ok = G.sha(g) == sp["q_sha256"]
    tiles = -(-sp["d"] // 4096)
    line = f'{sp["dist"]} d={sp["d"]} R={sp["R"]} T={sp["threads"]} tiles={tiles} ctrl={c[0]} wsbytes={c[1]} ptr={c[2]:#x} ok={ok}'
    if not ok:
        ref, _ = C.quantize_batch(x[None], m, [sp["X"]], sp["threads"])
        bad = np.nonzero(g.view(np.uint32) != ref[0].view(np.uint32))[0]
        tl = np.unique(bad // 4096)
        line += f' mismatches={len(bad)} first={bad[:8].tolist()} tiles={tl[:16].tolist()} ntiles={len(tl)}'
    print(line, flush=True)
    return ok

mode = sys.argv[1] if len(sys.argv) > 1 else "seq"
allok = True
for rnd in range(2):
    for sp, q, _, _ in G.spec_vectors(large=False):
        x = G.spec_gen(sp)
        got = uqdme.quantize_dequantize(torch.from_numpy(x[None]).cuda(), sp["R"], X=[sp["X"]], torch_threads=sp["threads"])
        assert G.bits_equal(got[0].cpu().numpy(), q)
    print("mid ok; ctrl", ctrl(), flush=True)
    for sp, _, pos, qs in G.spec_vectors(large=True):
        allok &= run(sp, poison=(mode == "poison"))
print("ALLOK", allok)
