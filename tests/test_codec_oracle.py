"""CPU: the UQR1 type-message format (oracle/uq_codec.c, the restatement the GPU codec is
compared with).  Parity unpinned by nature (the reference has no wire format, SURVEY §8(f)
row 4); what is pinned is the round trip to the reference's own output (AS:640):
decode(encode(codes)) gives back the codes -- all of them with exact zero signs, all but
the sign of zero counts in value mode -- and the rate lands near the nominal R."""
import numpy as np
import pytest

from oracle import uq_oracle as O
from oracle import uq_oracle_c as C


def _codes(x, R, X=0.37):
    m = O.rate_to_m(R, x.shape[0])
    code, L, ovf = O.type_codes(x, m, np.float32(X))
    assert not ovf
    return code, L, m


def _value_codes(c):
    return np.where(c == -1, 0, c).astype(np.int8)       # -0 (code ~0) -> +0


@pytest.mark.parametrize("d,R,dist", [(1024, 1, "normal"), (4099, 2, "laplace"), (65536, 0.5, "normal"),
                                      (65537, 1, "normal"), (172554, 1, "normal"), (100003, 4, "normal"),
                                      (3000, 5, "laplace"), (1, 1, "normal"), (63, 2, "normal"), (70000, 6, "normal")])
def test_roundtrip_exact_and_value(d, R, dist):
    rng = np.random.default_rng(d)
    x = (rng.standard_normal(d) if dist == "normal" else rng.laplace(1, 2, d)).astype(np.float32)
    c, L, m = _codes(x, R)
    for exact in (False, True):
        msg = C.codec_encode(c, m, L, exact)
        assert len(msg) % 4 == 0 and len(msg) <= C.lib().uqc_bound(d)
        c2, L2, m2 = C.codec_decode(msg, d)
        assert np.array_equal(c2, c if exact else _value_codes(c)), (d, R, exact)
        assert L2 == L and m2 == m


def test_rate_near_nominal():
    """At d = 2^20 (config C2) the value-mode message costs about R bits per coordinate."""
    rng = np.random.default_rng(1)
    x = rng.standard_normal(1 << 20).astype(np.float32)
    for R, lo, hi in ((1, 0.9, 1.02), (2, 1.85, 2.02), (0.5, 0.45, 0.56)):
        c, L, m = _codes(x, R)
        bits = 8 * len(C.codec_encode(c, m, L, False)) / x.shape[0]
        assert lo <= bits <= hi, (R, bits)


def test_degenerate_inputs():
    # all zero counts (one symbol): the states never move, the payload is empty
    c = np.zeros(5000, np.int8)
    msg = C.codec_encode(c, 10, np.float32(3.0), False)
    c2, L, m = C.codec_decode(msg, 5000)
    assert np.array_equal(c2, c) and L == np.float32(3.0) and m == 10
    # d = 0: a header-only message
    msg = C.codec_encode(np.zeros(0, np.int8), 0, np.float32(0.0), True)
    assert len(msg) == 40
    assert C.codec_decode(msg, 0)[0].shape == (0,)
    # the largest counts (k = 127, both signs) and every symbol present
    c = np.arange(-128, 128, dtype=np.int64).astype(np.int8).repeat(7)
    np.random.default_rng(0).shuffle(c)
    for exact in (False, True):
        c2, _, _ = C.codec_decode(C.codec_encode(c, 999, np.float32(1.5), exact), c.shape[0])
        assert np.array_equal(c2, c if exact else _value_codes(c))


def test_corruption_is_detected():
    rng = np.random.default_rng(2)
    c, L, m = _codes(rng.standard_normal(20000).astype(np.float32), 1)
    msg = bytearray(C.codec_encode(c, m, L, True))
    for pos in (0, 8, 30, len(msg) - 1):
        bad = bytearray(msg)
        bad[pos] ^= 0x5A
        try:
            c2, _, _ = C.codec_decode(bytes(bad), 20000)
        except ValueError:
            continue
        assert not np.array_equal(c2, c) or pos == len(msg) - 1     # last byte may be padding
    with pytest.raises(ValueError):
        C.codec_decode(bytes(msg), 20001)                            # wrong d
