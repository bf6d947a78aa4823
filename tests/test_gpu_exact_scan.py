"""The fp64 scan (AS:635: torch cumsum = SEQUENTIAL fp64 adds, each prefix rounded to f32)
is reproduced exactly by every K2 form.  The inputs are chosen so that a plain parallel
fp64 tree scan (round-1 K2, modelled in tests/scan_models.py) would NOT match: coordinate
mixes with many tiny fractional parts, and X placed on the first f32 prefix where the tree
scan differs, so that the difference reaches the outputs."""
import numpy as np
import pytest
import torch

from oracle import uq_oracle as O
from oracle import uq_oracle_c as C
from tests import golden_data as G
from tests import scan_models as S

pytestmark = pytest.mark.gpu
f32 = np.float32
D = 1 << 20
# seeds of S.tiny_mix(seed, 2^20, 0.5) on which the tree scan's f32 prefixes differ at R=1
# (tools/find_scan_cases.py)
SEEDS = (6, 8, 9, 23, 65)


@pytest.fixture(scope="module")
def uq(gpu_ready):
    import uqdme
    return uqdme


@pytest.fixture(scope="module")
def cases():
    m = O.rate_to_m(1, D)
    xs, Xs = [], []
    for s in SEEDS:
        x = S.tiny_mix(s, D)
        X, i = S.exposing_X(x, m)
        assert X is not None, f"seed {s}: the tree scan no longer differs (model changed?)"
        xs.append(x)
        Xs.append(X)
    x = np.stack(xs)
    X = np.array(Xs, f32)
    ref, _ = C.quantize_batch(x, m, X, 1)
    return x, X, m, ref


def dev(a):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=f32)).cuda()


def test_stream_form_exact(uq, cases):
    """n >= 256: one workgroup per client carries the exact prefix."""
    x, X, m, ref = cases
    n = x.shape[0]
    filler = torch.randn(256 - n, D, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1))
    big = torch.cat([dev(x), filler])
    Xb = np.concatenate([X, np.random.default_rng(2).random(256 - n).astype(f32)])
    got = uq.quantize_dequantize(big, m=m, X=Xb, torch_threads=1)[:n].cpu().numpy()
    assert G.n_mismatch(got, ref) == 0, [G.n_mismatch(got[j], ref[j]) for j in range(n)]


def test_segmented_form_exact(uq, cases):
    """5 clients x 256 tiles: approximate sums -> maps -> exact fold -> segmented outputs."""
    x, X, m, ref = cases
    got = uq.quantize_dequantize(dev(x), m=m, X=X, torch_threads=1).cpu().numpy()
    assert G.n_mismatch(got, ref) == 0, [G.n_mismatch(got[j], ref[j]) for j in range(x.shape[0])]
    tc, q = uq.quantize_encode(dev(x), m=m, X=X, torch_threads=1, return_q=True)
    assert G.bits_equal(q.cpu().numpy(), ref)
    assert G.bits_equal(uq.decode(tc).cpu().numpy(), ref)


def test_per_tile_form_exact_single_client(uq, cases):
    """n = 1 (the drop-in's batch): one workgroup per tile."""
    x, X, m, ref = cases
    for j in range(x.shape[0]):
        got = uq.quantize_dequantize(dev(x[j:j + 1]), m=m, X=X[j:j + 1], torch_threads=1).cpu().numpy()[0]
        assert G.n_mismatch(got, ref[j]) == 0, j


def test_unaligned_rows_exact(uq):
    """d % 4 != 0 with several clients: per-tile kernels on scalar loads."""
    d = D + 3
    m = O.rate_to_m(1, d)
    xs, Xs = [], []
    for s in SEEDS[:3]:
        x = S.tiny_mix(s, d)
        X, _ = S.exposing_X(x, m)
        xs.append(x)
        Xs.append(X if X is not None else f32(0.5))
    x = np.stack(xs)
    X = np.array(Xs, f32)
    ref, _ = C.quantize_batch(x, m, X, 1)
    got = uq.quantize_dequantize(dev(x), m=m, X=X, torch_threads=1).cpu().numpy()
    assert G.n_mismatch(got, ref) == 0


@pytest.mark.parametrize("mix,scale,R", [(0.9, 1e-3, 2), (0.3, 1e-6, 4), (0.99, 1e-5, 0.5)])
def test_tiny_mixes_all_forms(uq, mix, scale, R):
    """Other mixes and rates (more ties, other binades), each client in three forms."""
    d = 1 << 18
    m = O.rate_to_m(R, d)
    x = np.stack([S.tiny_mix(100 + j, d, mix, scale) for j in range(4)])
    X = np.random.default_rng(5).random(4).astype(f32)
    ref, _ = C.quantize_batch(x, m, X, 1)
    got = uq.quantize_dequantize(dev(x), m=m, X=X, torch_threads=1).cpu().numpy()
    assert G.n_mismatch(got, ref) == 0
    one = uq.quantize_dequantize(dev(x[1:2]), m=m, X=X[1:2], torch_threads=1).cpu().numpy()[0]
    assert G.n_mismatch(one, ref[1]) == 0
    big = torch.cat([dev(x), torch.randn(252, d, device="cuda")])
    Xb = np.concatenate([X, np.full(252, 0.5, f32)])
    st = uq.quantize_dequantize(big, m=m, X=Xb, torch_threads=1)[:4].cpu().numpy()
    assert G.n_mismatch(st, ref) == 0


def test_large_d_exact(uq):
    """d = 2^22 (config C4's size): binades up to 2^21, more fine fractions per tile."""
    d = 1 << 22
    m = O.rate_to_m(1, d)
    x = np.stack([S.tiny_mix(7, d, 0.5), np.random.default_rng(8).standard_normal(d).astype(f32)])
    X = np.array([0.25, 0.75], f32)
    ref, _ = C.quantize_batch(x, m, X, 1)
    got = uq.quantize_dequantize(dev(x), m=m, X=X, torch_threads=1).cpu().numpy()
    assert G.n_mismatch(got, ref) == 0
