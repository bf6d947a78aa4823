"""GPU: the DME harness (dme.py, ND:77-221 restricted to the unbiased scheme) against the
reference's own NMSE known answers, and the sharded-mean protocol with the HIP fold."""
import numpy as np
import pytest
import torch

from oracle import uq_oracle as O
from tests import golden_data as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def uq(gpu_ready):
    import uqdme
    return uqdme


def test_nd_harness_known_answers(uq):
    pts = G.nd_points()
    for dist, rows in pts.items():
        res = uq.nmse_simulation(dist, dim=2048, users=(1, 6, 11), num_instances=4)
        k = 0
        for ui, n in enumerate((1, 6, 11)):
            for inst in range(4):
                row = rows[k]
                for r in (1, 2):
                    got = float(res[r]["script"][ui, inst])
                    ref = row[f"nmse{r}"]
                    assert got == ref, (dist, n, inst, r, got, ref)   # bit for bit (north_star: 1e-6 rel)
                k += 1


def test_checkpoint_resume_equals_one_run(uq, tmp_path):
    """A run suspended at a user-count boundary and resumed from its checkpoint gives the rows
    of one uninterrupted run bit for bit (both generator streams continue exactly), with the
    QUIC-FL generator advance (jump-ahead) in the loop."""
    from uqdme_amd.dme import Suspended
    kw = dict(dim=1000, users=(1, 6, 11), num_instances=2, schemes=("eden", "unbiased", "biased"))
    whole = uq.nmse_simulation("gamma", **kw)
    ck = str(tmp_path / "ck.npz")
    with pytest.raises(Suspended):
        uq.nmse_simulation("gamma", checkpoint=ck, time_limit_s=0.0, **kw)      # stops before n = 6
    with pytest.raises(Suspended):
        uq.nmse_simulation("gamma", checkpoint=ck, time_limit_s=0.0, **kw)      # one more user count
    part = uq.nmse_simulation("gamma", checkpoint=ck, **kw)
    again = uq.nmse_simulation("gamma", checkpoint=ck, **kw)                    # finished: same rows
    for k in whole:
        assert np.array_equal(whole[k]["script"], part[k]["script"]), k
        assert np.array_equal(whole[k]["script"], again[k]["script"]), k
    with pytest.raises(ValueError):
        uq.nmse_simulation("normal", checkpoint=ck, **kw)


@pytest.mark.parametrize("dist", ["gamma", "bernoulli", "lognormal", "uniform"])
def test_other_distributions_vs_oracle(uq, dist):
    """Same harness, every scheme call checked bit-for-bit against the CPU oracle."""
    from uqdme_amd.dme import draw_vectors
    vecs, vns = draw_vectors(dist, 5, 2048, np.random.RandomState(3))
    xs = np.stack([v.astype(np.float32) for v in vecs])
    X = np.random.RandomState(4).random_sample(5).astype(np.float32)
    for R in (1, 2):
        q = uq.quantize_dequantize(torch.from_numpy(xs).cuda(), R, X=X, torch_threads=1).cpu().numpy()
        ref = np.stack([O.type_unbiased_quantize(xs[j], R, X[j]) for j in range(5)])
        assert G.bits_equal(q, ref), (dist, R, G.n_mismatch(q, ref))


def test_sharded_mean_single_rank_nccl(uq):
    """The RCCL path of distributed.py with one rank: ordered and reduce modes equal the
    single-call client mean bit-for-bit; ShardedDME's overlapped RCCL reduce likewise."""
    import os
    import socket
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        q = torch.randn(33, 5000, device="cuda")
        ref = uq.client_mean(q, 33.0)
        for mode in ("reduce", "ordered"):
            est = uq.sharded_client_mean(q, 33.0, mode=mode, block=1024)
            torch.cuda.synchronize()
            assert torch.equal(est, ref), mode
        # ShardedDME (the bench's path) over RCCL with the async reduce overlapped with the
        # next step: two estimate buffers alternate; every step's est equals the single-call
        # mean of its own q once drained
        n, d = 40, 8192
        sh = uq.ShardedDME(n, d, n, 1, torch_threads=1, overlap=True)
        assert sh.overlap and len(sh.est_bufs) == 2
        X = torch.rand(n, generator=torch.Generator().manual_seed(9)).cuda()
        outs = []
        for k in range(3):
            x = torch.randn(n, d, generator=torch.Generator(device="cuda").manual_seed(k), device="cuda")
            est = sh.step(x, X)
            q_ref = uq.quantize_dequantize(x, 1, X=X, torch_threads=1)
            outs.append((est, uq.client_mean(q_ref, float(n))))
            if k == 1:
                sh.drain()
                torch.cuda.synchronize()
                assert torch.equal(outs[1][0], outs[1][1])
        sh.drain()
        torch.cuda.synchronize()
        sh.check_status()
        assert outs[2][0].data_ptr() == outs[0][0].data_ptr()
        assert torch.equal(outs[2][0], outs[2][1])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fixture", ["nd_nmse_schemes.json", "nd_nmse_schemes_d4194304.json"])
def test_multi_scheme_nmse_known_answers(gpu_ready, fixture):
    """EDEN 1/2, unbiased 1/2 and biased 1/2 in the driver's call order against the
    reference's own loop (tests/golden/nd_nmse_schemes*.json, made by
    make_golden_nmse_schemes.py): d = 2048, and config C4's d = 2^22 (five distributions,
    n in {1, 6}, two instances each).  Every scheme within 1e-6 relative (north_star), and
    every EDEN scale the reference recorded (EdenSender.compress, AS:335: torch.dot, computed
    here in MKL sdot's order by eden_dot_kernel) bit for bit."""
    import json
    import os
    import uqdme
    from tests.golden_data import GOLDEN
    ref = json.load(open(os.path.join(GOLDEN, fixture)))
    for dist, rows in ref["rows"].items():
        mine = {}
        res = uqdme.nmse_simulation(dist, dim=ref["dim"], users=(1, 6), num_instances=2,
                                    schemes=("eden", "unbiased", "biased"), torch_threads=1, eden_scales_out=mine)
        for row in rows:
            ui = (1, 6).index(row["n"])
            for sc in ("eden", "unbiased", "biased"):
                for r in (1, 2):
                    got = float(res[(sc, r)]["script"][ui, row["inst"]])
                    exp = row[f"{sc}{r}"]
                    assert abs(got - exp) <= 1e-6 * exp, (dist, row["n"], row["inst"], sc, r, got, exp)
        theirs = {}
        for n, inst, client, bits, seed, sbits in ref["eden_scales"][dist]:
            theirs.setdefault((n, inst, bits), []).append(np.uint32(sbits))
        for key, sc_ref in theirs.items():
            assert np.array_equal(mine[key].view(np.uint32), np.asarray(sc_ref, np.uint32)), (dist, key)


@pytest.mark.parametrize("fixture", ["nd_nmse_schemes_quicfl.json", "nd_nmse_schemes_d4194304_quicfl.json"])
def test_nd_loop_with_quicfl_known_answers(gpu_ready, fixture):
    """The driver loop with QUICFL_quantize in its place (ND:141-142, after the biased
    quantizer) against the reference's own loop on synthetic sender tables
    (tests/golden/nd_nmse_schemes_quicfl.json at d = 2048 and nd_nmse_schemes_d4194304_quicfl.json
    at config C4's d = 2^22, normal and laplace; make_golden_nmse_schemes.py --quicfl): the
    QUIC-FL draws (a message seed, then D bernoulli(p_X) words of the global generator per
    call) interleave with EDEN's and the unbiased quantizer's, so every scheme's NMSE is
    checked within 1e-6 relative, QUIC-FL bit for bit.""" 
    import json
    import os
    import sys
    import uqdme
    from tests.golden_data import GOLDEN
    sys.path.insert(0, GOLDEN)
    from quicfl_tables import DATA, sender_tables
    ref = json.load(open(os.path.join(GOLDEN, fixture)))
    rz = np.load(os.path.join(GOLDEN, "quicfl_recv_vectors.npz"))
    tx = uqdme.QuicFLSender(tables={b: (*sender_tables(b), DATA[b]) for b in (1, 2, 3, 4)})
    rx = uqdme.QuicFLReceiver(tables={b: rz[f"recv{b}"] for b in (1, 2, 3, 4)})
    for dist, rows in ref["rows"].items():
        res = uqdme.nmse_simulation(dist, dim=ref["dim"], users=(1, 6), num_instances=2,
                                    schemes=("eden", "unbiased", "biased", "quicfl"), torch_threads=1, quicfl=(tx, rx))
        for row in rows:
            ui = (1, 6).index(row["n"])
            for sc in ("eden", "unbiased", "biased", "quicfl"):
                for r in (1, 2):
                    got = float(res[(sc, r)]["script"][ui, row["inst"]])
                    exp = row[f"{sc}{r}"]
                    assert abs(got - exp) <= 1e-6 * exp, (dist, row["n"], row["inst"], sc, r, got, exp)
            for r in (1, 2):
                got = np.float32(res[("quicfl", r)]["script"][ui, row["inst"]])
                assert got == np.float32(row[f"quicfl{r}"]), (dist, row, r)
