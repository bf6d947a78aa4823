"""ctypes binding of the C-ABI in include/uq_dme.h.

Loading fails loudly: there is no CPU fallback anywhere in the product path.  The
library is found in-tree (`_build/libuq_dme.so`); build it with build_ext.py or
`__graft_entry__.build()`.
"""
from __future__ import annotations

import ctypes
import os
import threading

from . import build_ext

_lock = threading.Lock()
_lib = None

# (name, restype, argtypes) — must match include/uq_dme.h exactly.
_i32, _i64, _f32, _f64, _p, _sz = (ctypes.c_int32, ctypes.c_int64, ctypes.c_float,
                                   ctypes.c_double, ctypes.c_void_p, ctypes.c_size_t)
SIGNATURES = {
    "uq_version": (ctypes.c_int, []),
    "uq_last_error": (ctypes.c_char_p, []),
    "uq_build_id": (ctypes.c_char_p, []),
    "uq_test_force_replay_failure": (ctypes.c_int, [ctypes.c_int]),
    "uq_test_set_quicfl_hooks": (ctypes.c_int, [ctypes.c_int]),
    "uq_mt_jump_host": (ctypes.c_int, [_p, _i64, _p]),
    "uq_legacy_draw_f32": (ctypes.c_int, [_p, _p, _p, _p, _i32, _f64, _f64, _i64, _i64, _p, _p, _i32]),
    "uq_legacy_test_params": (ctypes.c_int, [_i64, _i64, _p, _p]),
    "uq_rate_to_m": (ctypes.c_int, [_f64, _i64, ctypes.POINTER(_i64)]),
    "uq_workspace_bytes": (ctypes.c_int, [_i64, _i64, _i32, ctypes.POINTER(_sz)]),
    "uq_l1_torch_order_f32": (ctypes.c_int, [_p, _i64, _i64, _i32, _p, _p, _sz, _p]),
    "uq_type_unbiased_f32": (ctypes.c_int, [_p, _p, _i64, _i64, _i64, _p, _p, _p, _i32, _p, _sz, _p]),
    "uq_type_unbiased_vec_f32": (ctypes.c_int, [_p, _p, _i64, _i64, _f32, _i32, _p, _sz, _p]),
    "uq_client_mean_f32": (ctypes.c_int, [_p, _i64, _i64, _i64, _f32, _i32, _p, _p]),
    "uq_type_unbiased_mean_f32": (ctypes.c_int, [_p, _p, _i64, _i64, _i64, _p, _p, _i32, _f32, _i32, _p,
                                                 _p, _sz, _p]),
    "uq_check_status": (ctypes.c_int, [_p, _p]),
    "uq_type_unbiased_codes_f32": (ctypes.c_int, [_p, _p, _p, _p, _i64, _i64, _i64, _p, _p, _p, _i32, _p, _sz, _p]),
    "uq_codes_decode_f32": (ctypes.c_int, [_p, _p, _i64, _i64, _i64, _p, _p]),
    "uq_codes_mean_f32": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _i64, _f32, _i32, _p, _p]),
    "uq_codes_q_mean_f32": (ctypes.c_int, [_p, _p, _i64, _p, _p, _i64, _i64, _i64, _f32, _i32, _p, _p]),
    "uq_type_unbiased_codes_ld_f32": (ctypes.c_int, [_p, _p, _i64, _p, _i64, _p, _i64, _i64, _i64, _p, _p, _p, _i32,
                                                     _p, _sz, _p]),
    "uq_codes_q_mean_ld_f32": (ctypes.c_int, [_p, _i64, _p, _i64, _p, _p, _i64, _i64, _i64, _f32, _i32, _p, _p]),
    "uq_type_unbiased_nibbles_ld_f32": (ctypes.c_int, [_p, _p, _i64, _p, _i64, _p, _i64, _i64, _i64, _p, _p, _p, _i32,
                                                       _p, _sz, _p]),
    "uq_nibbles_q_mean_ld_f32": (ctypes.c_int, [_p, _i64, _p, _i64, _p, _p, _i64, _i64, _i64, _f32, _i32, _p, _p]),
    "uq_biased_workspace_bytes": (ctypes.c_int, [_i64, _i64, _i32, ctypes.POINTER(_sz)]),
    "uq_type_biased_f32": (ctypes.c_int, [_p, _p, _i64, _i64, _i64, _i32, _i32, _p, _p, _p, _sz, _p]),
    "uq_rht_signs": (ctypes.c_int, [_p, _i64, _i64, _p, _p]),
    "uq_rht_f32": (ctypes.c_int, [_p, _p, _i64, _i64, _i32, _p, _p, _p, _sz, _p]),
    "uq_quicfl_prepare_f32": (ctypes.c_int, [_p, _i64, _i64, _p, _i32, _i32, _p, _p, _p, _p, _p, _p]),
    "uq_quicfl_receive_f32": (ctypes.c_int, [_p, _i32, _i64, _i64, _p, _i32, _i32, _p, _p, _p, _i32, _p, _p, _p, _p, _p]),
    "uq_quicfl_receive_workspace_bytes": (ctypes.c_int, [_i64, _i64, ctypes.POINTER(_sz)]),
    "uq_quicfl_receive_ws_f32": (ctypes.c_int, [_p, _i32, _i64, _i64, _p, _i32, _i32, _p, _p, _p, _i32, _p, _p, _p, _p,
                                                _p, _sz, _p]),
    "uq_quicfl_workspace_bytes": (ctypes.c_int, [_i64, _i64, ctypes.POINTER(_sz)]),
    # x, n, dim, signs, sign_row, table_xp, table_packed, numel, h_len, delta, recv_table, recv_numel, prng_seeds,
    # px_state, px_seeds, px_state_out, out, scale, info, ws, ws_bytes, stream
    "uq_quicfl_quantize_f32": (ctypes.c_int, [_p, _i64, _i64, _p, _p, _p, _p, _i64, _i32, _f32, _p, _i32, _p, _p, _p, _p,
                                              _p, _p, _p, _p, _sz, _p]),
    "uq_quicfl_compress_f32": (ctypes.c_int, [_p, _i64, _i64, _p, _p, _p, _p, _i64, _i32, _f32, _p, _p, _p, _p, _p, _i32,
                                              _p, _p, _p, _p, _p, _p, _sz, _p]),
    "uq_xxh64": (ctypes.c_uint64, [ctypes.c_char_p, _sz, ctypes.c_uint64]),
    "uq_eden_workspace_bytes": (ctypes.c_int, [_i64, _i64, ctypes.POINTER(_sz)]),
    "uq_eden_compress_f32": (ctypes.c_int, [_p, _i64, _i64, _i32, _p, _p, _p, _p, _p, _sz, _p]),
    "uq_eden_decompress_f32": (ctypes.c_int, [_p, _p, _i64, _i64, _i32, _p, _p, _p, _p, _sz, _p]),
    "uq_eden_f32": (ctypes.c_int, [_p, _p, _i64, _i64, _i32, _p, _p, _p, _p, _sz, _p]),
    "uq_rht_sign_bits": (ctypes.c_int, [_p, _i64, _i64, _p, _p]),
    "uq_eden_compress_f32_sb": (ctypes.c_int, [_p, _i64, _i64, _i32, _p, _p, _p, _p, _p, _p, _sz, _p]),
    "uq_eden_decompress_f32_sb": (ctypes.c_int, [_p, _p, _i64, _i64, _i32, _p, _p, _p, _p, _p, _sz, _p]),
    "uq_eden_f32_sb": (ctypes.c_int, [_p, _p, _i64, _i64, _i32, _p, _p, _p, _p, _p, _sz, _p]),
    "uq_eden_norm_workspace_bytes": (ctypes.c_int, [_i64, _i64, ctypes.POINTER(_sz)]),
    "uq_eden_norm_f32": (ctypes.c_int, [_p, _i64, _i64, _i32, _p, _p, _sz, _p]),
    "uq_tc_bound": (ctypes.c_int, [_i64, ctypes.POINTER(_sz)]),
    "uq_tc_workspace_bytes": (ctypes.c_int, [_i64, _i64, ctypes.POINTER(_sz)]),
    "uq_tc_encode": (ctypes.c_int, [_p, _p, _i64, _i64, _i64, _i32, _p, _sz, _p, _p, _sz, _p]),
    "uq_tc_decode": (ctypes.c_int, [_p, _sz, _p, _i64, _i64, _i64, _p, _p, _p, _p, _p]),
}


class UQError(RuntimeError):
    """A C-ABI call returned a negative code."""


def library_path() -> str:
    return build_ext.SO


def load(build_if_missing: bool = False):
    """Load (once) and return the ctypes library.  Raises if it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = library_path()
        if not os.path.exists(path):
            if build_if_missing:
                build_ext.build()
            else:
                raise ImportError(
                    f"HIP extension not built: {path} is missing. Run "
                    "`python unbiased-quantization-distributed-mean-estimation_amd/build_ext.py` "
                    "(no CPU fallback exists by design).")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().uq_last_error()
        raise UQError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
