"""GPU: type codes from the quantize kernels (stream and small-batch paths), decode, and the
mean from codes -- all bit-exact against the oracle / the float path."""
import numpy as np
import pytest
import torch

from oracle import uq_oracle as O
from tests import golden_data as G

pytestmark = pytest.mark.gpu
f32 = np.float32


@pytest.fixture(scope="module")
def uq(gpu_ready):
    import uqdme
    return uqdme


@pytest.mark.parametrize("n,d", [(5, 4099), (3, 100003), (300, 4096), (260, 1001), (2, 1 << 20)])
def test_codes_match_oracle_and_decode(uq, n, d):
    rng = np.random.default_rng(n * 7 + d)
    x = rng.laplace(1, 2, (n, d)).astype(f32)
    X = rng.random(n).astype(f32)
    for R in (1, 2):
        m = O.rate_to_m(R, d)
        tc, q = uq.quantize_encode(torch.from_numpy(x).cuda(), m=m, X=X, torch_threads=1, return_q=True)
        q_only = uq.quantize_dequantize(torch.from_numpy(x).cuda(), m=m, X=X, torch_threads=1)
        assert torch.equal(q.view(torch.int32), q_only.view(torch.int32))
        tc.check()
        codes = tc.codes.cpu().numpy()
        for j in range(min(n, 4)):
            ref_code, ref_L, ovf = O.type_codes(x[j], m, X[j])
            assert not ovf
            assert np.array_equal(codes[j], ref_code), (n, d, R, j)
            kk = np.where(ref_code < 0, -ref_code.astype(np.int32) - 1, ref_code.astype(np.int32))
            assert int(tc.overflow[j]) == int(kk.max())
        dec = uq.decode(tc)
        assert G.bits_equal(dec.cpu().numpy(), q.cpu().numpy())
        # encode-only path (no q written) gives the same codes
        tc2 = uq.quantize_encode(torch.from_numpy(x).cuda(), m=m, X=X, torch_threads=1)
        assert torch.equal(tc2.codes, tc.codes)
        est = uq.codes_mean(tc, n)
        assert G.bits_equal(est.cpu().numpy(), uq.client_mean(q, n).cpu().numpy())


def test_codes_mean_accumulate_and_odd_sizes(uq):
    rng = np.random.default_rng(1)
    for n, d in ((1, 7), (33, 1000), (70, 4112)):
        x = rng.normal(size=(n, d)).astype(f32)
        X = rng.random(n).astype(f32)
        tc, q = uq.quantize_encode(torch.from_numpy(x).cuda(), 2, X=X, torch_threads=1, return_q=True)
        h = n // 2
        a = uq.TypeCodes(codes=tc.codes[:h].contiguous(), l1=tc.l1[:h], m=tc.m, overflow=tc.overflow[:h])
        b = uq.TypeCodes(codes=tc.codes[h:].contiguous(), l1=tc.l1[h:], m=tc.m, overflow=tc.overflow[h:])
        est = uq.codes_mean(a, n) if h else torch.zeros(d, device="cuda")
        est = uq.codes_mean(b, n, est=est, accumulate=True)
        assert G.bits_equal(est.cpu().numpy(), uq.client_mean(q, n).cpu().numpy())


def test_overflow_flag_at_high_rate(uq):
    rng = np.random.default_rng(2)
    x = rng.lognormal(1, 2, (3, 5000)).astype(f32)
    tc = uq.quantize_encode(torch.from_numpy(x).cuda(), 10, X=rng.random(3).astype(f32), torch_threads=1)
    assert int(torch.count_nonzero(tc.overflow > 127)) > 0
    with pytest.raises(OverflowError):
        tc.check()


def test_wire_roundtrip_through_bytes(uq):
    rng = np.random.default_rng(3)
    x = rng.normal(size=(4, 2048)).astype(f32)
    X = rng.random(4).astype(f32)
    tc, q = uq.quantize_encode(torch.from_numpy(x).cuda(), 1, X=X, torch_threads=1, return_q=True)
    msg = tc.to_bytes()
    back = uq.TypeCodes.from_bytes(msg, device="cuda")
    assert G.bits_equal(uq.decode(back).cpu().numpy(), q.cpu().numpy())


@pytest.mark.parametrize("d", [4112, 1000])
def test_codes_mean_group_boundaries(uq, d):
    """codes_mean stages client tables 32 at a time and double-buffers code loads in
    batches of 16: client counts on either side of every boundary, vector and bytewise
    columns (d = 4112: a tail workgroup whose last threads go bytewise; d = 1000: all
    bytewise), against the float-path client mean."""
    rng = np.random.default_rng(d)
    x = rng.laplace(1, 2, (97, d)).astype(f32)
    X = rng.random(97).astype(f32)
    tc, q = uq.quantize_encode(torch.from_numpy(x).cuda(), 2, X=X, torch_threads=1, return_q=True)
    for n in (15, 16, 17, 31, 32, 33, 47, 48, 49, 63, 64, 65, 80, 95, 96, 97):
        sub = uq.TypeCodes(codes=tc.codes[:n].contiguous(), l1=tc.l1[:n], m=tc.m, overflow=tc.overflow[:n])
        est = uq.codes_mean(sub, 97).cpu().numpy()
        ref = uq.client_mean(q[:n].contiguous(), 97).cpu().numpy()
        assert G.bits_equal(est, ref), (n, d, G.n_mismatch(est, ref))
