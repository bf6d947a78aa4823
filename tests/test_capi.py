"""The C-ABI library loads and exports every symbol include/uq_dme.h declares, and its
host-only entry points behave (no GPU needed: no kernel is launched here)."""
import ctypes
import os
import re

import pytest

import uqdme
from uqdme import RATE_TABLE, rate_to_m

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "uq_dme.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(uq_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    return uqdme.load_library()


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for n in ("uq_type_unbiased_f32", "uq_l1_torch_order_f32", "uq_client_mean_f32",
              "uq_workspace_bytes", "uq_last_error", "uq_rate_to_m", "uq_check_status",
              "uq_type_unbiased_mean_f32", "uq_version"):
        assert n in names


def test_library_exports_all_declared_symbols(lib):
    from uqdme_amd import _lib as L
    for n in declared_functions():
        assert hasattr(lib, n), n
        assert n in L.SIGNATURES, f"ctypes signature missing for {n}"


def test_version_and_rate_table(lib):
    assert lib.uq_version() >= 100
    m = ctypes.c_int64()
    for bits, l in RATE_TABLE.items():
        for d in (1, 2, 1000, 1024, 172554, 1 << 20, 1 << 22):
            assert lib.uq_rate_to_m(float(bits), d, ctypes.byref(m)) == 0
            assert m.value == rate_to_m(bits, d) == int(l * d)
    assert lib.uq_rate_to_m(3.3, 10, ctypes.byref(m)) == -1
    assert b"KeyError" in lib.uq_last_error()


def test_workspace_and_argument_errors(lib):
    b = ctypes.c_size_t()
    assert lib.uq_workspace_bytes(1024, 1 << 20, 1, ctypes.byref(b)) == 0
    assert b.value >= 1024 * 256 * 8
    assert lib.uq_workspace_bytes(4, 1000, 0, ctypes.byref(b)) == -1
    assert lib.uq_workspace_bytes(-1, 1000, 1, ctypes.byref(b)) == -1
    # empty batches are no-ops that never touch the device
    assert lib.uq_type_unbiased_f32(None, None, 0, 100, 10, None, None, None, 1, None, 0, None) == 0
    assert lib.uq_type_unbiased_f32(None, None, 4, 0, 0, None, None, None, 1, None, 0, None) == 0
    # invalid arguments are rejected before any launch
    assert lib.uq_type_unbiased_f32(None, None, 4, 100, 10, None, None, None, 1, None, 0, None) == -1
    assert lib.uq_type_unbiased_f32(ctypes.c_void_p(16), ctypes.c_void_p(16), 4, 100, 10, ctypes.c_void_p(16),
                                    None, None, 1, ctypes.c_void_p(16), 10, None) == -3
    assert lib.uq_type_unbiased_f32(ctypes.c_void_p(16), ctypes.c_void_p(16), 4, 100, -5, ctypes.c_void_p(16),
                                    None, None, 1, ctypes.c_void_p(16), 1 << 30, None) == -1
    assert lib.uq_l1_torch_order_f32(ctypes.c_void_p(16), 4, 100, 0, None, ctypes.c_void_p(16), 1 << 30, None) == -1
    # any torch thread count up to 4096: torch splits a sum into min(T, ceil(d/32768))
    # chunks summed through a T-element buffer
    assert lib.uq_workspace_bytes(4, 100, 128, ctypes.byref(b)) == 0
    assert lib.uq_workspace_bytes(4, 1 << 21, 128, ctypes.byref(b)) == 0          # 64 chunks
    assert lib.uq_workspace_bytes(4, 1 << 23, 128, ctypes.byref(b)) == 0          # 128 chunks
    assert lib.uq_workspace_bytes(4, 1 << 23, 4096, ctypes.byref(b)) == 0         # 256 chunks
    assert lib.uq_workspace_bytes(4, 1 << 23, 4097, ctypes.byref(b)) == -1        # beyond the plan
    assert lib.uq_client_mean_f32(None, 3, 10, 10, 3.0, 0, None, None) == -1
    assert lib.uq_client_mean_f32(ctypes.c_void_p(16), 3, 10, 9, 3.0, 0, ctypes.c_void_p(16), None) == -1


def test_drop_in_signature_and_name():
    import inspect
    f = uqdme.Type_unbiased_quantize
    assert f.__name__ == "Type_unbiased_quantize"
    sig = inspect.signature(f)
    assert list(sig.parameters) == ["input_vector", "bits_per_dimension"]
    assert sig.parameters["bits_per_dimension"].default == 1


def test_biased_and_eden_argument_errors(lib):
    """Host-side validation of the biased / EDEN / RHT entry points (no kernel launched)."""
    import ctypes
    from uqdme_amd import _lib as L
    for name, (res, args) in L.SIGNATURES.items():
        getattr(lib, name).restype = res
        getattr(lib, name).argtypes = args
    b = ctypes.c_size_t(0)
    assert lib.uq_biased_workspace_bytes(4, 1000, 1, ctypes.byref(b)) == 0 and b.value > 0
    assert lib.uq_biased_workspace_bytes(-1, 1000, 1, ctypes.byref(b)) < 0
    assert lib.uq_eden_workspace_bytes(4, 1000, ctypes.byref(b)) == 0 and b.value > 0
    # bad n / m / torch_threads / tie policy are rejected before any device work
    assert lib.uq_type_biased_f32(None, None, -1, 10, 2, 1, 0, None, None, None, 0, None) < 0
    assert lib.uq_type_biased_f32(None, None, 1, 10, -2, 1, 0, None, None, None, 0, None) < 0
    assert lib.uq_type_biased_f32(None, None, 1, 10, 2, 0, 0, None, None, None, 0, None) < 0
    assert lib.uq_type_biased_f32(None, None, 1, 10, 2, 1, 7, None, None, None, 0, None) < 0
    assert b"tie_policy" in lib.uq_last_error()
    assert lib.uq_type_biased_f32(None, None, 0, 10, 2, 1, 0, None, None, None, 0, None) == 0   # n = 0: no-op
    # EDEN: only the reference's 1- and 2-bit tables
    assert lib.uq_eden_compress_f32(None, 1, 16, 3, None, None, None, None, None, 0, None) < 0
    assert b"nbits" in lib.uq_last_error()
    assert lib.uq_eden_f32(None, None, 0, 16, 1, None, None, None, None, 0, None) == 0
    assert lib.uq_rht_f32(None, None, -1, 16, 0, None, None, None, 0, None) < 0
    assert lib.uq_rht_signs(None, -1, 16, None, None) < 0


def test_codec_sizes_host_only(lib):
    """uq_tc_bound agrees with the CPU restatement's bound; workspace sizes grow with n, d;
    bad arguments are rejected (no kernel launched)."""
    from oracle import uq_oracle_c as C
    for d in (0, 1, 5, 1023, 1024, 1025, 65536, 65537, 172554, 1 << 20, 3000017):
        b = ctypes.c_size_t()
        assert lib.uq_tc_bound(d, ctypes.byref(b)) == 0
        assert b.value == C.lib().uqc_bound(d), d
    w1, w2 = ctypes.c_size_t(), ctypes.c_size_t()
    assert lib.uq_tc_workspace_bytes(4, 1 << 20, ctypes.byref(w1)) == 0
    assert lib.uq_tc_workspace_bytes(8, 1 << 20, ctypes.byref(w2)) == 0
    assert w2.value > w1.value >= 4 * 2 * (1 << 20)         # the word scratch: 2 B per symbol
    assert lib.uq_tc_bound(-1, ctypes.byref(w1)) != 0
    assert lib.uq_tc_encode(None, None, 1, 10, 5, 2, None, 0, None, None, 0, None) != 0   # unknown flag


def test_round3_entry_points_argument_errors(lib):
    """uq_codes_q_mean_f32 / uq_type_unbiased_vec_f32: host-side checks (no kernel launched)."""
    from uqdme_amd import _lib as L
    for name in ("uq_codes_q_mean_f32", "uq_type_unbiased_vec_f32"):
        res, args = L.SIGNATURES[name]
        getattr(lib, name).restype = res
        getattr(lib, name).argtypes = args
    p = ctypes.c_void_p(16)
    assert lib.uq_codes_q_mean_f32(p, p, 9, p, p, 4, 10, 5, 4.0, 0, p, None) == -1        # ldq < d
    assert b"ldq" in lib.uq_last_error()
    assert lib.uq_codes_q_mean_f32(None, None, 10, None, None, 4, 10, 5, 4.0, 0, p, None) == -1
    assert lib.uq_codes_q_mean_f32(None, None, 10, None, None, 4, 0, 5, 4.0, 0, None, None) == 0   # d = 0
    assert lib.uq_type_unbiased_vec_f32(None, None, 0, 0, 0.5, 1, None, 0, None) == 0      # d = 0: no-op
    assert lib.uq_type_unbiased_vec_f32(p, None, 10, 2, 0.5, 1, p, 1 << 20, None) == -1    # null out
    assert lib.uq_type_unbiased_vec_f32(p, p, 10, -2, 0.5, 1, p, 1 << 20, None) == -1      # m < 0


def test_pitched_entry_points_argument_errors(lib):
    """uq_type_unbiased_codes_ld_f32 / uq_codes_q_mean_ld_f32: row pitches below d are rejected
    before anything is launched (n = 0 for the quantize call, so even a missing check would
    launch nothing)."""
    from uqdme_amd import _lib as L
    for name in ("uq_type_unbiased_codes_ld_f32", "uq_codes_q_mean_ld_f32"):
        res, args = L.SIGNATURES[name]
        getattr(lib, name).restype = res
        getattr(lib, name).argtypes = args
    p = ctypes.c_void_p(16)
    ws = ctypes.create_string_buffer(1 << 16)
    wsp = ctypes.cast(ws, ctypes.c_void_p)
    assert lib.uq_type_unbiased_codes_ld_f32(p, p, 9, p, 10, p, 0, 10, 5, p, None, None, 1, wsp, 1 << 16, None) == -1
    assert b"pitch" in lib.uq_last_error()
    assert lib.uq_type_unbiased_codes_ld_f32(p, p, 10, p, 9, p, 0, 10, 5, p, None, None, 1, wsp, 1 << 16, None) == -1
    assert lib.uq_type_unbiased_codes_ld_f32(p, p, 10, p, 10, p, 0, 10, 5, p, None, None, 1, wsp, 1 << 16, None) == 0
    assert lib.uq_codes_q_mean_ld_f32(p, 9, p, 10, p, p, 4, 10, 5, 4.0, 0, p, None) == -1       # ldc < d
    assert b"ldc" in lib.uq_last_error()


def test_xxh64_and_quicfl_argument_checks(lib):
    """uq_xxh64 (AS:457's hash, host-only) against the oracle's restatement; the sender's
    host-side argument checks (no kernel launched)."""
    from oracle import uq_quicfl as Q
    for s in (0, 1, 42, 99, 123, -3, 10 ** 12):
        b = str(s).encode()
        assert lib.uq_xxh64(b, len(b), 0) == Q.xxh64(b)
    for n in range(0, 70, 3):
        b = bytes((i * 7 + 3) & 255 for i in range(n))
        assert lib.uq_xxh64(b, len(b), 0) == Q.xxh64(b)
    sz = ctypes.c_size_t()
    assert lib.uq_quicfl_workspace_bytes(4, 1000, ctypes.byref(sz)) == 0 and sz.value >= 4 * 1024 * 5
    args = [None, 1, 1000, None, None, None, None, 64 * 3, 64, 0.5, None, None, None, None, None, 0, None, None,
            None, None, None, None, 0, None]
    bad = list(args)
    bad[8] = 300                                   # h_len > 256
    assert lib.uq_quicfl_compress_f32(*bad) == -1
    bad = list(args)
    bad[7] = 100                                   # numel not a multiple of h_len
    assert lib.uq_quicfl_compress_f32(*bad) == -1
    bad = list(args)
    bad[15] = 2                                    # x_kind
    assert lib.uq_quicfl_compress_f32(*bad) == -1
    assert lib.uq_quicfl_compress_f32(*args) == -1  # null pointers
    empty = list(args)
    empty[1] = 0
    assert lib.uq_quicfl_compress_f32(*empty) == 0  # an empty batch is a no-op


def test_build_id_matches_sources(lib):
    """The loaded binary was built from the current sources and flags (content hash, not
    file times: build_ext.needs_build rebuilds on any mismatch)."""
    from uqdme_amd import build_ext
    assert lib.uq_build_id().decode() == build_ext.build_id()
    assert not build_ext.needs_build()


def test_quicfl_workspaces_cover_the_jump_paths(lib):
    """The QUIC-FL workspaces grow by the jump path's scratch where it applies (up to 1024
    messages of >= 8 rounds, by the cost model: the sender's streams, partial windows and run
    records; the receiver's with a workspace entry) and stay as before elsewhere (host-only: no
    kernel runs)."""
    sz = ctypes.c_size_t()
    base = {}
    for n, d in ((1, 2048), (1, 1 << 20), (128, 1 << 20), (300, 1 << 20)):
        assert lib.uq_quicfl_workspace_bytes(n, d, ctypes.byref(sz)) == 0
        base[(n, d)] = sz.value
        assert sz.value >= n * d * 5                       # rotated vectors + h at least
    # one 2^20 message: 2 streams x 33 blocks + >= 1 run's 3 x 4 partial windows more than its vectors
    assert base[(1, 1 << 20)] - (1 << 20) * 5 >= (2 * 33 * 624 + 12 * 624) * 4
    assert lib.uq_quicfl_receive_workspace_bytes(1, 2048, ctypes.byref(sz)) == 0 and sz.value == 0
    assert lib.uq_quicfl_receive_workspace_bytes(1, 1 << 20, ctypes.byref(sz)) == 0 and sz.value >= 33 * 624 * 4
    # 1024 messages of 2^20 take the receiver's jump path too (two runs each, round 6); batches
    # beyond 1024 messages do not
    assert lib.uq_quicfl_receive_workspace_bytes(1024, 1 << 20, ctypes.byref(sz)) == 0
    assert sz.value >= 1024 * 33 * 624 * 4
    assert lib.uq_quicfl_receive_workspace_bytes(2048, 1 << 20, ctypes.byref(sz)) == 0 and sz.value == 0
    assert lib.uq_quicfl_receive_workspace_bytes(-1, 16, ctypes.byref(sz)) < 0
    assert lib.uq_rht_sign_bits(None, -1, 16, None, None) < 0
    assert lib.uq_rht_sign_bits(None, 0, 16, None, None) == 0        # nothing to pack
