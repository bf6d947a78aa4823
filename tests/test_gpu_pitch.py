"""GPU: row-pitched outputs (uq_type_unbiased_codes_ld_f32, uq_codes_q_mean_ld_f32).

q row j at out + j*ldq, code row j at codes + j*ldc: every K2 form (stream, segmented
stream, per-tile outputs; float4 and scalar lanes) writes the same bits as into dense [n, d]
buffers and nothing in the pads between rows; the codes mean over pitched codes equals the
dense one (AS:609-641, ND:137-138)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

SENT_F = -12345.5      # sentinel in the pads
SENT_C = 77


def _run(lib, L, x, X, m, ldq, ldc, T=1):
    n, d = x.shape
    b = ctypes.c_size_t()
    L.check(lib.uq_workspace_bytes(n, d, T, ctypes.byref(b)), "ws")
    ws = torch.zeros(max(b.value, 1 << 16), dtype=torch.uint8, device="cuda")
    qs = torch.full((n, ldq), SENT_F, device="cuda")
    cs = torch.full((n, ldc), SENT_C, dtype=torch.int8, device="cuda")
    km = torch.zeros(n, dtype=torch.int32, device="cuda")
    l1 = torch.empty(n, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    L.check(lib.uq_type_unbiased_codes_ld_f32(x.data_ptr(), qs.data_ptr(), ldq, cs.data_ptr(), ldc, km.data_ptr(), n, d,
                                              m, X.data_ptr(), None, l1.data_ptr(), T, ws.data_ptr(), ws.numel(), st),
            "uq_type_unbiased_codes_ld_f32")
    torch.cuda.synchronize()
    return qs, cs, km, l1


# (n, d, ldq - d, ldc - d): stream form (n >= 256), segmented stream (>= 1024 tiles), per-tile
# outputs; pads that keep float4 / 16-byte code stores and odd pads that force scalar lanes
CASES = [
    (300, 8192, 64, 256),
    (300, 8192, 3, 5),
    (8, 1 << 20, 64, 256),
    (3, 40000, 64, 256),
    (3, 40000, 1, 7),
    (1, 4099, 5, 3),
]


@pytest.mark.parametrize("n,d,pq,pc", CASES)
def test_pitched_outputs_bit_identical(gpu_ready, n, d, pq, pc):
    import uqdme
    from uqdme_amd import _lib as L
    lib = L.load()
    g = torch.Generator(device="cuda").manual_seed(n * 7 + d)
    x = torch.randn(n, d, generator=g, device="cuda")
    x[0, : min(d, 300)] = 0.0                         # signed zeros / zero counts in row 0
    x[0, 1] = -0.0
    X = torch.rand(n, generator=torch.Generator().manual_seed(d)).cuda()
    m = uqdme.rate_to_m(1, d)
    q0, c0, k0, l0 = _run(lib, L, x, X, m, d, d)
    q1, c1, k1, l1 = _run(lib, L, x, X, m, d + pq, d + pc)
    assert torch.equal(q1[:, :d].contiguous().view(torch.int32), q0.view(torch.int32))
    assert torch.equal(c1[:, :d], c0) and torch.equal(k1, k0) and torch.equal(l1, l0)
    assert bool((q1[:, d:] == SENT_F).all()), "q pad written"
    assert bool((c1[:, d:] == SENT_C).all()), "codes pad written"
    # the codes mean over the pitched codes (and the pitched q beside them) = the dense mean
    est0 = torch.empty(d, device="cuda")
    est1 = torch.empty(d, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    L.check(lib.uq_codes_q_mean_f32(c0.data_ptr(), q0.data_ptr(), d, l0.data_ptr(), k0.data_ptr(), n, d, m, float(n), 0,
                                    est0.data_ptr(), st), "dense mean")
    L.check(lib.uq_codes_q_mean_ld_f32(c1.data_ptr(), d + pc, q1.data_ptr(), d + pq, l1.data_ptr(), k1.data_ptr(), n,
                                       d, m, float(n), 0, est1.data_ptr(), st), "pitched mean")
    ref = uqdme.client_mean(q0, float(n))
    torch.cuda.synchronize()
    assert torch.equal(est0.view(torch.int32), ref.view(torch.int32))
    assert torch.equal(est1.view(torch.int32), ref.view(torch.int32))
