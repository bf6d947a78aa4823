"""GPU: the UQR1 type-message codec (uq_tc_encode / uq_tc_decode, csrc/uq_codec_kernels.h).

* GPU messages are byte-identical to the CPU restatement's (oracle/uq_codec.c) for the same
  codes, and each side decodes the other's messages;
* the whole chain x -> quantize_encode -> encode_messages -> decode_messages -> decode equals
  the reference's output (AS:640) on the same draws: bit for bit with exact zero signs,
  value for value (+0.0 for -0.0) without;
* the rate at config C2's size is ~R bits per coordinate; malformed messages are reported.
Parity of the format itself is unpinned (the reference has no codec)."""
import numpy as np
import pytest
import torch

from oracle import uq_oracle as O
from oracle import uq_oracle_c as C

pytestmark = pytest.mark.gpu


def _batch(n, d, dist, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((n, d)) if dist == "normal" else rng.laplace(1, 2, (n, d))).astype(np.float32)
    X = rng.random(n).astype(np.float32)
    return x, X


@pytest.mark.parametrize("n,d,R,dist", [(16, 1024, 1, "normal"), (3, 65537, 2, "laplace"), (5, 172554, 1, "normal"),
                                        (2, 4099, 4, "normal"), (7, 1, 1, "normal"), (4, 100, 0.5, "laplace"),
                                        (2, 1 << 20, 1, "normal"), (2, 1 << 20, 2, "laplace")])
def test_messages_match_cpu_restatement(gpu_ready, n, d, R, dist):
    import uqdme
    x, X = _batch(n, d, dist, n * d)
    m = O.rate_to_m(R, d)
    tc = uqdme.quantize_encode(torch.from_numpy(x).cuda(), R, X=X, torch_threads=1)
    codes = tc.codes.cpu().numpy()
    l1 = tc.l1.cpu().numpy()
    for exact in (False, True):
        msgs = uqdme.encode_messages(tc, exact_zero_signs=exact)
        gpu = msgs.messages()
        for j in range(n):
            ref = C.codec_encode(codes[j], m, l1[j], exact)
            assert gpu[j] == ref, (n, d, R, exact, j, len(gpu[j]), len(ref))
            c2, L2, m2 = C.codec_decode(gpu[j], d)                        # CPU decodes the GPU's message
            assert np.array_equal(c2, codes[j] if exact else np.where(codes[j] == -1, 0, codes[j]))
        back = uqdme.decode_messages(uqdme.TypeMessages.from_messages([C.codec_encode(codes[j], m, l1[j], exact)
                                                                        for j in range(n)], d))
        want = codes if exact else np.where(codes == -1, 0, codes).astype(np.int8)
        assert np.array_equal(back.codes.cpu().numpy(), want)                # GPU decodes the CPU's messages
        assert np.array_equal(back.l1.cpu().numpy().view(np.uint32), l1.view(np.uint32)) and back.m == m


@pytest.mark.parametrize("R", [1, 2])
def test_chain_reproduces_reference_output(gpu_ready, R):
    import uqdme
    n, d = 6, 1 << 20
    x, X = _batch(n, d, "normal", 11)
    xt = torch.from_numpy(x).cuda()
    q_ref = uqdme.quantize_dequantize(xt, R, X=X, torch_threads=1).cpu().numpy()
    # the GPU q is itself checked against the oracle elsewhere; spot-check one client here
    assert np.array_equal(q_ref[0].view(np.uint32), O.type_unbiased_quantize(x[0], R, X[0]).view(np.uint32))
    tc = uqdme.quantize_encode(xt, R, X=X, torch_threads=1)
    for exact in (True, False):
        msgs = uqdme.encode_messages(tc, exact_zero_signs=exact)
        q = uqdme.decode(uqdme.decode_messages(msgs)).cpu().numpy()
        if exact:
            assert np.array_equal(q.view(np.uint32), q_ref.view(np.uint32))
        else:
            assert np.array_equal(q, q_ref)                                   # -0.0 == +0.0
            bits = msgs.bits_per_dim()
            assert bits <= R + 0.02, bits                                     # ~R bits per coordinate
            assert bits >= 0.9 * R, bits


def test_malformed_messages_are_reported(gpu_ready):
    import uqdme
    x, X = _batch(3, 30000, "normal", 5)
    tc = uqdme.quantize_encode(torch.from_numpy(x).cuda(), 1, X=X, torch_threads=1)
    good = uqdme.encode_messages(tc, exact_zero_signs=True).messages()
    bad = [bytearray(b) for b in good]
    bad[0][0] ^= 1                                       # magic
    bad[1][28] ^= 2                                      # nsym
    bad[2] = bad[2][:-8] + bytes(8)                      # zeroed words at the end
    with pytest.raises(ValueError):
        uqdme.decode_messages(uqdme.TypeMessages.from_messages([bytes(b) for b in bad], 30000))
    ok = uqdme.decode_messages(uqdme.TypeMessages.from_messages(good, 30000))
    assert torch.equal(ok.codes, tc.codes)


def test_empty_vectors_header_only(gpu_ready):
    """d = 0: header-only messages (the d == 0 pack path), byte-identical to the CPU
    restatement's, decoded back to L1 with no codes."""
    import uqdme
    n = 3
    tc = uqdme.TypeCodes(codes=torch.zeros((n, 0), dtype=torch.int8, device="cuda"),
                         l1=torch.tensor([0.0, 1.5, 2.25], device="cuda"), m=0,
                         overflow=torch.zeros(n, dtype=torch.int32, device="cuda"))
    msgs = uqdme.encode_messages(tc, exact_zero_signs=True)
    gpu = msgs.messages()
    for j in range(n):
        assert gpu[j] == C.codec_encode(np.zeros(0, np.int8), 0, np.float32(tc.l1[j].item()), True), j
    back = uqdme.decode_messages(msgs)
    assert back.codes.shape == (n, 0)
    assert torch.equal(back.l1, tc.l1)


def test_offsets_bounds_and_m_checked_on_device(gpu_ready):
    """uq_tc_decode reads nothing outside [msgs, msgs + msgs_bytes) -- offsets past
    the buffer, decreasing or unaligned are status bit 0 -- and a header whose m differs
    from the batch's expected m is status bit 4; the well-formed messages beside them still
    decode.  TypeMessages.from_messages refuses a batch mixing m values on the host."""
    import uqdme
    from uqdme_amd import _lib
    lib = _lib.load()
    n, d = 4, 30000
    x, X = _batch(n, d, "normal", 6)
    tc = uqdme.quantize_encode(torch.from_numpy(x).cuda(), 1, X=X, torch_threads=1)
    msgs = uqdme.encode_messages(tc)
    off = msgs.offsets.clone()
    sp = torch.cuda.current_stream().cuda_stream

    def dec(data, offs, m):
        codes = torch.zeros((n, d), dtype=torch.int8, device="cuda")
        l1 = torch.zeros(n, device="cuda")
        km = torch.zeros(n, dtype=torch.int32, device="cuda")
        st = torch.zeros(n, dtype=torch.int32, device="cuda")
        _lib.check(lib.uq_tc_decode(data.data_ptr(), data.numel(), offs.data_ptr(), n, d, m, codes.data_ptr(),
                                    l1.data_ptr(), km.data_ptr(), st.data_ptr(), sp), "decode")
        torch.cuda.synchronize()
        return codes, st.cpu().tolist()

    want = torch.where(tc.codes == -1, torch.zeros_like(tc.codes), tc.codes)   # value mode: no zero signs
    codes, st = dec(msgs.data, off, tc.m)
    assert st == [0] * n and torch.equal(codes, want)
    codes, st = dec(msgs.data[:int(off[2])], off, tc.m)             # buffer ends inside message 2
    assert st[:2] == [0, 0] and st[2] & 1 and st[3] & 1 and torch.equal(codes[:2], want[:2])
    o2 = off.clone()
    o2[3] = 1 << 40                                                  # far outside, and decreasing after it
    codes, st = dec(msgs.data, o2, tc.m)
    assert st[0] == st[1] == 0 and st[2] & 1 and st[3] & 1
    o3 = off.clone()
    o3[1] += 2                                                       # unaligned start
    _, st = dec(msgs.data, o3, tc.m)
    assert st[1] & 1
    _, st = dec(msgs.data, off, tc.m + 1)                            # another m than the batch's
    assert all(s & 16 for s in st)
    other = uqdme.encode_messages(uqdme.quantize_encode(torch.from_numpy(x).cuda(), 2, X=X, torch_threads=1))
    with pytest.raises(ValueError):
        uqdme.TypeMessages.from_messages(msgs.messages()[:2] + other.messages()[2:], d)


def test_chunked_encode_matches_one_shot(gpu_ready):
    """encode_messages through a small staging buffer (client chunks) returns exactly the
    one-shot messages, in a buffer of exactly their size."""
    import uqdme
    n, d = 7, 20000
    x, X = _batch(n, d, "laplace", 8)
    tc = uqdme.quantize_encode(torch.from_numpy(x).cuda(), 1, X=X, torch_threads=1)
    one = uqdme.encode_messages(tc)
    bound = one.data.numel() // n
    chunked = uqdme.encode_messages(tc, staging_bytes=3 * bound)          # chunks of 3, 3, 1 clients
    assert chunked.messages() == one.messages()
    assert chunked.data.numel() == chunked.total_bytes() == one.total_bytes()
    back = uqdme.decode_messages(chunked)
    assert torch.equal(back.codes, torch.where(tc.codes == -1, torch.zeros_like(tc.codes), tc.codes))
