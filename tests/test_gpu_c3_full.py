"""GPU: BASELINE.json configs[2] ("C3") at its full single-GPU size -- n = 8192 clients of
d = 2^20, R = 1 -- for both of its distributions, Laplace(1, 2) (Laplace_dist.py:89) and
U(-1, 1) (build-defined, dme.DISTRIBUTIONS), through the resident DMEPipeline (K1 -> K2 ->
K3c, the path bench.py times; x 32 GiB + q 32 GiB + codes 8 GiB on one MI355X).

Checked against the C restatement oracle/uq_oracle.c (AS:609-641, ND:137-138):
  * every one of the 8192 clients' q bit for bit (the oracle runs over the host's allotted
    cores, slab by slab);
  * est bit for bit against the oracle's client-ordered mean over all 8192 clients;
and at full size, from the GPU's own outputs:
  * no client overflows its int8 codes, and decode(codes) == q bit for bit;
  * sum_i k_i = m +- 1 for every client (AS:636-637 telescopes to floor(c_d - X) - floor(-X);
    the fp64 total c_d sits within a tiny epsilon of an integer), and = m exactly whenever X
    is away from 0 and 1.
The vectors are drawn on the GPU (torch CUDA generator; Laplace by inversion as bench.py
does), so the reference's own NumPy draws are not reproduced here: the parity anchor is the
oracle on the same inputs."""
import os

import numpy as np
import pytest
import torch

from oracle import uq_oracle_c as C

pytestmark = pytest.mark.gpu

N, D = 8192, 1 << 20
SLAB = 512


def _threads() -> int:
    n = len(os.sched_getaffinity(0))
    try:
        n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    except ValueError:
        pass
    return max(1, n)


def _draw(dist, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.empty(N, D, device="cuda", dtype=torch.float32)
    lim = 0.5 - 2.0 ** -25
    for j in range(0, N, 1024):
        u = torch.rand(1024, D, generator=g, device="cuda", dtype=torch.float32)
        if dist == "laplace":           # loc 1, scale 2 (Laplace_dist.py:89), |u - 1/2| < 1/2
            u = (u - 0.5).clamp_(-lim, lim)
            x[j:j + 1024] = 1.0 - 2.0 * torch.sign(u) * torch.log1p(-2.0 * u.abs())
        else:                           # U(-1, 1)
            x[j:j + 1024] = u * 2.0 - 1.0
        del u
    return x


@pytest.mark.parametrize("dist,seed", [("laplace", 31), ("uniform", 32)])
def test_c3_full_size_one_gpu(gpu_ready, dist, seed):
    import uqdme
    m = uqdme.rate_to_m(1, D)
    x = _draw(dist, seed)
    X_cpu = torch.rand(N, generator=torch.Generator().manual_seed(seed))
    X = X_cpu.cuda()
    p = uqdme.DMEPipeline(N, D, 1, torch_threads=1)
    est = p.step(x, X).cpu().numpy()
    p.check_status()
    assert p.overflowed() == 0
    Xh = X_cpu.numpy()
    nth = _threads()
    est_ref = np.zeros(D, np.float32)
    sums = np.empty(N, np.int64)
    dec = torch.empty(SLAB, D, device="cuda", dtype=torch.float32)
    lib = uqdme.load_library()
    from uqdme_amd import _lib as L
    for j0 in range(0, N, SLAB):
        sl = slice(j0, j0 + SLAB)
        # full-size properties from the GPU's own outputs
        c = p.codes[sl].to(torch.int32)
        k = torch.where(c < 0, -c - 1, c)
        sums[sl] = k.sum(dim=1, dtype=torch.int64).cpu().numpy()
        del c, k
        L.check(lib.uq_codes_decode_f32(p.codes[sl].data_ptr(), p.l1[sl].data_ptr(), SLAB, D, m, dec.data_ptr(),
                                        torch.cuda.current_stream().cuda_stream), "decode")
        assert torch.equal(dec.view(torch.int32), p.q[sl].view(torch.int32)), (dist, j0)
        # every client bit for bit against the C oracle, and the oracle's ordered mean
        ref, _, _ = C.quantize_batch_mt(x[sl].cpu().numpy(), m, Xh[sl], 1, nth)
        got = p.q[sl].cpu().numpy()
        bad = np.flatnonzero(np.any(got.view(np.uint32) != ref.view(np.uint32), axis=1))
        assert bad.size == 0, (dist, j0 + bad[:8])
        C.client_mean_acc(ref, float(N), est_ref)
        del ref, got
    assert np.array_equal(est.view(np.uint32), est_ref.view(np.uint32)), (dist, int(np.sum(est != est_ref)))
    dev = sums - m
    assert np.all(np.abs(dev) <= 1), (dist, np.unique(dev))
    mid = (Xh > 0.05) & (Xh < 0.95)
    assert np.all(dev[mid] == 0), (dist, int(np.count_nonzero(dev[mid])))
    print(f"{dist}: sum k - m in {{-1: {int(np.sum(dev == -1))}, 0: {int(np.sum(dev == 0))}, "
          f"+1: {int(np.sum(dev == 1))}}} over {N} clients")
