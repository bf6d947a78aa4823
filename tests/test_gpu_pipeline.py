"""GPU: the resident pipeline (pipeline.DMEPipeline) used by bench.py -- K1 -> K2 (q + codes)
-> client mean from the codes -- equals the batched APIs bit for bit, before and after the
output-placement probe swaps its buffers (ND:133-138, AS:609-641)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,d,bits", [(300, 8192, 1), (5, 40000, 2)])
def test_pipeline_step_matches_batched_apis(gpu_ready, n, d, bits):
    import uqdme
    g = torch.Generator(device="cuda").manual_seed(n + d)
    x = torch.randn(n, d, generator=g, device="cuda")
    X = torch.rand(n, generator=torch.Generator().manual_seed(3)).cuda()
    q_ref = uqdme.quantize_dequantize(x, bits, X=X, torch_threads=1)
    est_ref = uqdme.client_mean(q_ref, float(n))
    p = uqdme.DMEPipeline(n, d, bits, torch_threads=1)
    for probe in (False, True):
        if probe:
            rep = p.probe_outputs(x, X, candidates=3, reps=1)
            assert 1 < rep["candidates"] <= 3 and 0 <= rep["chosen"] < rep["candidates"]
        est = p.step(x, X)
        torch.cuda.synchronize()
        p.check_status()
        assert torch.equal(est.view(torch.int32), est_ref.view(torch.int32)), probe
        assert torch.equal(p.q.view(torch.int32), q_ref.view(torch.int32)), probe
        dec = uqdme.decode(uqdme.TypeCodes(codes=p.codes, l1=p.l1, m=p.m, overflow=p.kmax))
        assert torch.equal(dec.view(torch.int32), q_ref.view(torch.int32)), probe
    with pytest.raises(ValueError):
        p.step(x[:, :-1].contiguous(), X)


def test_pipelines_agree_and_overflowed_client_falls_back_to_q(gpu_ready):
    """a client whose lattice counts overflow its int8 codes (one nonzero
    coordinate: k = m there; or, in a second batch, a NaN / inf coordinate, whose L1 is not
    finite) -- the "codes" pipeline reads that client from q, so est is still the
    client-ordered mean of q bit for bit (ND:137-138); "q" gives the same bits; "encode" (no
    q to fall back to) raises from check_status."""
    import uqdme
    n, d, bits = 70, 8192, 1                       # 2 full 32-client groups + 6 in the tail
    g = torch.Generator(device="cuda").manual_seed(11)
    x0 = torch.randn(n, d, generator=g, device="cuda")
    for j in (3, 40, 67):                          # one client in each group and in the tail
        x0[j].zero_()
        x0[j, 100 + j] = -2.5
    x1 = x0.clone()
    x1[20, 7] = float("nan")
    x1[50, 9] = float("inf")
    X = torch.rand(n, generator=torch.Generator().manual_seed(4)).cuda()
    for x, novf in ((x0, 3), (x1, 5)):
        q_ref = uqdme.quantize_dequantize(x, bits, X=X, torch_threads=1)
        est_ref = uqdme.client_mean(q_ref, float(n))
        for pl in ("codes", "q"):
            p = uqdme.DMEPipeline(n, d, bits, torch_threads=1, pipeline=pl)
            est = p.step(x, X)
            p.check_status()
            assert torch.equal(p.q.view(torch.int32), q_ref.view(torch.int32)), pl
            assert torch.equal(est.view(torch.int32), est_ref.view(torch.int32)), pl
            if pl == "codes":
                assert p.overflowed() == novf
                assert int(p.kmax[3]) == 128 and int(p.kmax[0]) <= 127
        p = uqdme.DMEPipeline(n, d, bits, torch_threads=1, pipeline="encode")
        p.step(x, X)
        with pytest.raises(OverflowError):
            p.check_status()
    # accumulate continues the sum bit-for-bit from a previous est
    x = x0
    q_ref = uqdme.quantize_dequantize(x, bits, X=X, torch_threads=1)
    p = uqdme.DMEPipeline(n, d, bits, torch_threads=1)
    e1 = p.step(x, X, n_div=float(2 * n)).clone()
    e2 = p.step(x, X, n_div=float(2 * n), accumulate=True, est=e1)
    ref2 = uqdme.client_mean(torch.cat([q_ref, q_ref]), float(2 * n))
    assert torch.equal(e2.view(torch.int32), ref2.view(torch.int32))


@pytest.mark.parametrize("d", [1, 5, 4096, 172554, 1 << 20])
def test_vector_entry_x_by_value_matches_batched(gpu_ready, d):
    """uq_type_unbiased_vec_f32 (the per-call drop-in: X by value, no fill) gives the bits of
    the batched entry with n = 1, over repeated calls on one workspace (the record counters
    the tile-sum kernels now reset themselves)."""
    import uqdme
    gen = torch.Generator().manual_seed(d)
    for rep in range(3):
        v = torch.randn(d, generator=gen).cuda()
        torch.manual_seed(100 + rep)
        got = uqdme.Type_unbiased_quantize(v, 1)
        torch.manual_seed(100 + rep)
        X = torch.rand(1)
        ref = uqdme.quantize_dequantize(v.view(1, d), X=X, m=uqdme.rate_to_m(1, d)).view(d)
        assert torch.equal(got.view(torch.int32), ref.view(torch.int32)), (d, rep)


def test_empty_batch_pipeline(gpu_ready):
    """A rank with no clients (more ranks than clients): every launch is a no-op and the
    mean is zeros, so its reduce contributes nothing."""
    import uqdme
    p = uqdme.DMEPipeline(0, 4096, 1, torch_threads=1)
    x = torch.empty((0, 4096), device="cuda")
    X = torch.empty(0, device="cuda")
    for pl in ("codes", "q", "encode"):
        est = p.step(x, X, n_div=5.0, pipeline=pl)
        torch.cuda.synchronize()
        p.check_status()
        assert torch.count_nonzero(est) == 0, pl


def test_output_pool_never_hands_out_a_held_result(gpu_ready):
    """The one-shot APIs' output pool (outpool.py): results the caller still holds -- whole
    tensors, views, NumPy aliases -- are never handed out again; released sets are reused
    (same storage) and every result has the same bits as a plain allocation's."""
    import uqdme
    from uqdme_amd.outpool import POOL
    n, d = 8, 4096
    x = torch.randn(n, d, device="cuda")
    X = torch.rand(n)
    ref = uqdme.quantize_dequantize(x, 1, X=X, torch_threads=1).clone()
    old, was_on = POOL.min_bytes, POOL.enabled
    POOL.min_bytes = 0
    POOL.enabled = True
    POOL.clear()
    try:
        held = [uqdme.quantize_dequantize(x, 1, X=X, torch_threads=1) for _ in range(4)]
        ptrs = {h.data_ptr() for h in held}
        assert len(ptrs) == 4                                    # each held result has its own storage
        for h in held:
            assert torch.equal(h, ref)
        view = held[0][3]
        keep = held[1].cpu()                                     # a host copy: not an alias
        del held
        torch.cuda.synchronize()
        again = [uqdme.quantize_dequantize(x, 1, X=X, torch_threads=1) for _ in range(6)]
        assert all(a.data_ptr() != view.data_ptr() - 3 * d * 4 for a in again)   # held via a view
        assert all(torch.equal(a, ref) for a in again)
        assert torch.equal(keep, ref.cpu())
        del again
        torch.cuda.synchronize()
        loop_ptrs = set()
        for _ in range(12):                                      # the caller's loop: q = f(x)
            q = uqdme.quantize_dequantize(x, 1, X=X, torch_threads=1)
            loop_ptrs.add(q.data_ptr())
            assert torch.equal(q, ref)
        torch.cuda.synchronize()
        assert len(loop_ptrs) <= POOL.explore + POOL.keep        # sets are reused, not allocated per call
        tc, q2 = uqdme.quantize_encode(x, 1, X=X, torch_threads=1, return_q=True)
        assert torch.equal(q2, ref) and torch.equal(uqdme.decode(tc), ref)
        assert torch.equal(view, ref[3])
    finally:
        POOL.min_bytes = old
        POOL.enabled = was_on
        POOL.clear()


def _unpack_nibbles(nib: torch.Tensor) -> torch.Tensor:
    """uint8 [n, d/2] 4-bit fields -> int8 [n, d] codes (sign-extended nibbles)."""
    lo = (nib & 0xF).to(torch.int16)
    hi = (nib >> 4).to(torch.int16)
    v = torch.stack([lo, hi], dim=-1).reshape(nib.shape[0], -1)
    return torch.where(v >= 8, v - 16, v).to(torch.int8)


@pytest.mark.parametrize("bits", [1, 2])
def test_codes4_pipeline_matches_batched_apis(gpu_ready, bits):
    """The 4-bit code pipeline (bench default): est and q bit-identical to the batched APIs,
    before and after the placement probe and with accumulate; its nibbles are the int8
    codes' low nibbles; clients whose counts exceed 7 (an outlier coordinate) or 127 (one
    nonzero coordinate) or whose L1 is not finite are read from q (ND:137-138, AS:609-641)."""
    import uqdme
    n, d = 300, 8192                                   # 9 full 32-client groups + 12 in the tail
    g = torch.Generator(device="cuda").manual_seed(21 + bits)
    x = torch.randn(n, d, generator=g, device="cuda")
    x[5, 77] = 60.0                                    # 7 < kmax <= 127
    x[40].zero_()
    x[40, 100] = -2.5                                  # kmax = 128
    x[299, 3] = float("inf")                           # L1 not finite
    X = torch.rand(n, generator=torch.Generator().manual_seed(5)).cuda()
    q_ref = uqdme.quantize_dequantize(x, bits, X=X, torch_threads=1)
    est_ref = uqdme.client_mean(q_ref, float(n))
    ref8 = uqdme.DMEPipeline(n, d, bits, torch_threads=1, pipeline="codes")
    ref8.step(x, X)
    p = uqdme.DMEPipeline(n, d, bits, torch_threads=1, pipeline="codes4")
    for probe in (False, True):
        if probe:
            rep = p.probe_outputs(x, X, candidates=3, reps=1)
            assert 1 < rep["candidates"] <= 3
        est = p.step(x, X)
        p.check_status()
        assert torch.equal(p.q.view(torch.int32), q_ref.view(torch.int32)), probe
        assert torch.equal(est.view(torch.int32), est_ref.view(torch.int32)), probe
        assert torch.equal(p.kmax, ref8.kmax)
        fits = (p.kmax <= 7).nonzero().flatten()
        assert fits.numel() >= n - 3 and int(p.kmax[5]) > 7 and int(p.kmax[40]) == 128
        assert torch.equal(_unpack_nibbles(p.nib)[fits], ref8.codes[fits]), probe
        assert p.overflowed() >= 3
    e1 = p.step(x, X, n_div=float(2 * n)).clone()
    e2 = p.step(x, X, n_div=float(2 * n), accumulate=True, est=e1)
    ref2 = uqdme.client_mean(torch.cat([q_ref, q_ref]), float(2 * n))
    assert torch.equal(e2.view(torch.int32), ref2.view(torch.int32))
    # no client above 7: the straight-line mean (every client from its nibbles)
    xg = torch.randn(n, d, generator=g, device="cuda")
    qg = uqdme.quantize_dequantize(xg, bits, X=X, torch_threads=1)
    eg = p.step(xg, X)
    assert p.overflowed() == 0
    assert torch.equal(eg.view(torch.int32), uqdme.client_mean(qg, float(n)).view(torch.int32))
    # a step overridden to the int8 kinds and back (the bench's side lines on one pipeline)
    for pl in ("codes", "q", "encode", "codes4"):
        e = p.step(x, X, pipeline=pl)
        if pl != "encode":
            assert torch.equal(e.view(torch.int32), est_ref.view(torch.int32)), pl
    assert uqdme.codes4_fits(n, d, bits) and not uqdme.codes4_fits(n, d, 3) and not uqdme.codes4_fits(255, d, 1)
    for bad in ((255, d), (n, d + 16)):
        with pytest.raises(ValueError):
            uqdme.DMEPipeline(*bad, bits, pipeline="codes4")
