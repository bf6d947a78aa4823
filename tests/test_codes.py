"""Type-code wire format (codes.py): the decoding rule reproduces the reference's outputs
bit-for-bit (CPU, against the golden fixtures), and the UQT1 message round-trips."""
import numpy as np
import pytest
import torch

from oracle import uq_oracle as O
from tests import golden_data as G

f32 = np.float32


def decode_np(code, L, m):
    k = np.where(code < 0, -code.astype(np.int64) - 1, code.astype(np.int64)).astype(f32)
    with np.errstate(all="ignore"):
        tab = ((f32(L) * k).astype(f32) / f32(m)).astype(f32)
    return np.where(code < 0, -tab, tab).astype(f32)


def test_decode_rule_matches_reference_fixtures():
    z = G.c1()
    for R, key, Xk in ((1, "q1", "X1"), (2, "q2", "X2")):
        for j in range(16):
            m = O.rate_to_m(R, 1024)
            code, L, ovf = O.type_codes(z["x"][j], m, z[Xk][j])
            assert not ovf
            assert G.bits_equal(decode_np(code, L, m), z[key][j])
    n = 0
    for sp, q, _, _ in G.spec_vectors(large=False):
        x = G.spec_gen(sp)
        m = O.rate_to_m(sp["R"], sp["d"])
        code, L, ovf = O.type_codes(x, m, sp["X"], sp["threads"])
        if ovf:
            continue
        assert G.bits_equal(decode_np(code, L, m), q), sp
        n += 1
    assert n >= 30


def test_edge_cases_decode_or_overflow():
    for name, R, X, x, q in G.edge_cases():
        m = O.rate_to_m(R, x.shape[0])
        code, L, ovf = O.type_codes(x, m, X)
        if not ovf:
            assert G.bits_equal(decode_np(code, L, m), q), (name, R)


def test_message_roundtrip_host():
    import uqdme
    rng = np.random.default_rng(0)
    codes = torch.from_numpy(rng.integers(-128, 128, (3, 37), dtype=np.int8))
    tc = uqdme.TypeCodes(codes=codes, l1=torch.tensor([1.5, 2.0, 0.0]), m=7, overflow=torch.zeros(3, dtype=torch.int32))
    buf = tc.to_bytes()
    assert len(buf) == 32 + 12 + 3 * 37
    back = uqdme.TypeCodes.from_bytes(buf)
    assert torch.equal(back.codes, codes) and torch.equal(back.l1, tc.l1) and back.m == 7
    kk = np.where(codes.numpy() < 0, -codes.numpy().astype(np.int32) - 1, codes.numpy().astype(np.int32))
    assert np.array_equal(back.overflow.numpy(), kk.max(axis=1))
    with pytest.raises(ValueError):
        uqdme.TypeCodes.from_bytes(buf[:-1])
    tc.overflow[1] = 128
    with pytest.raises(OverflowError):
        tc.to_bytes()
