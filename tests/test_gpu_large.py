"""GPU: maximum sizes -- single client vectors of 2^27 .. 2^29 + 4096 floats (0.5-2 GiB).

Every K2 form at sizes far beyond the configs: the segmented stream (one vector of 2^28,
65 536 tiles), the per-tile forms past the stream's 2^29-element limit (float4 lanes) and
with d % 4 != 0 (scalar lanes), the per-call drop-in (X by value), and the type codes.  m
exceeds 2^24 here, so f32(m) may round (AS:623 / AS:629: the reference casts m to f32).  q is
compared bit for bit with the C oracle; L1 (AS:624) with torch's own CPU sum on this host at
the same intra-op thread count."""
import numpy as np
import pytest
import torch

from oracle import uq_oracle as O
from oracle import uq_oracle_c as C
from tests import golden_data as G

pytestmark = pytest.mark.gpu
f32 = np.float32


@pytest.fixture(scope="module")
def uq(gpu_ready):
    import uqdme
    return uqdme


def torch_l1(x: np.ndarray, T: int) -> np.float32:
    """AS:624 on the CPU with T intra-op threads (the reference's own op)."""
    prev = torch.get_num_threads()
    torch.set_num_threads(T)
    try:
        return np.float32(torch.from_numpy(x).abs().sum().item())
    finally:
        torch.set_num_threads(prev)


@pytest.mark.parametrize("n,d,T,entry", [
    (1, 1 << 28, 1, "drop-in"),                  # segmented stream, uq_type_unbiased_vec_f32
    (1, 1 << 28, 16, "codes"),                   # 16 torch chunks; q + type codes
    (2, (1 << 27) + 3, 1, "batched"),            # d % 4 != 0: per-tile forms, scalar lanes
    (1, (1 << 29) + 4096, 1, "batched"),         # past the stream form's limit: per-tile, float4
])
def test_max_size_vectors_bit_exact(uq, n, d, T, entry):
    rng = np.random.default_rng(d + T)
    x = rng.standard_normal((n, d), dtype=f32)
    m = O.rate_to_m(1, d)
    assert m > (1 << 24)
    X = np.array([0.37, 0.81][:n], f32)
    xt = torch.from_numpy(x).cuda()
    if entry == "drop-in":
        uq.set_torch_threads(T)
        try:
            torch.manual_seed(11)
            got = uq.Type_unbiased_quantize(xt[0], 1).cpu().numpy()[None]
        finally:
            uq.set_torch_threads(None)
        torch.manual_seed(11)
        X = np.array([torch.rand(1).item()], f32)
    elif entry == "codes":
        tc, q = uq.quantize_encode(xt, m=m, X=X, torch_threads=T, return_q=True)
        got = q.cpu().numpy()
        assert torch.equal(uq.decode(tc).view(torch.int32), q.view(torch.int32))
        assert int(tc.overflow.max()) <= 127
    else:
        got = uq.quantize_dequantize(xt, m=m, X=X, torch_threads=T).cpu().numpy()
    del xt
    ref, l1 = C.quantize_batch(x, m, X, T)
    assert G.n_mismatch(got, ref) == 0, (n, d, T)
    for j in range(n):
        assert torch_l1(x[j], T).view(np.uint32) == l1[j].view(np.uint32), (j, T)
        # Counts never exceed m.  (They sum to m up to d = 2^22, but not here: the reference's
        # prefixes c are f32 (AS:635), whose spacing is 2-4 above 2^24-2^25, so most crossings
        # floor(c_i - X) - floor(c_{i-1} - X) == 1 (AS:636-637) are lost -- at d = 2^28 the
        # counts sum to ~0.29 m.  The oracle and the GPU agree on this bit for bit.)
        k = np.rint(np.abs(got[j].astype(np.float64)) * m / np.float64(l1[j]))
        assert int(k.sum()) <= m + 1


def test_max_size_biased_bit_exact(uq):
    """Type_biased_quantize (AS:644-687) on one vector of 2^28 + 64 floats: the k' cascade
    with torch's step 64 (K1a's large-step variant), the radix select over 2^28 keys and --
    when the threshold is tied -- the torch topk replay at that size, bit-exact against the
    C++ oracle with torch's tie choice."""
    d = (1 << 28) + 64
    x = np.random.default_rng(9).standard_normal(d, dtype=f32)
    m = O.rate_to_m(1, d)
    got = uq.biased_quantize(torch.from_numpy(x[None]).cuda(), m=m, torch_threads=1, ties="torch")
    uq.check_status()
    got = got.cpu().numpy()[0]
    ref, L, D, amb = C.biased_quantize(x, m, 1, 0)
    assert G.n_mismatch(got, ref) == 0, (D, amb)
