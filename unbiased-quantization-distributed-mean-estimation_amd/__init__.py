"""MI355X-native unbiased L1-ball type quantizer for distributed mean estimation.

Reference: Ritesh622/Unbiased-Quantization-Distributed-Mean-Estimation,
`Type_unbiased_quantize` (NMSE_Results/Codes/All_Schemes.py:609-641), the client
mean around it (NMSE_Results/Codes/Normal_dist.py:133-138) and the biased variant
`Type_biased_quantize` (All_Schemes.py:644-687).  Import through the
top-level alias `uqdme` (this directory name is not a Python identifier).
"""
from .rates import RATE_TABLE, rate_to_m
from .quantizer import (
    Type_unbiased_quantize, quantize_dequantize, client_mean, quantize_mean,
    l1_torch_order, draw_uniforms, set_torch_threads, get_torch_threads, check_status,
    quantize_encode, decode, codes_mean,
)
from .codes import TypeCodes, TypeMessages, encode_messages, decode_messages
from .biased import Type_biased_quantize, biased_quantize
from .eden import (EDEN_quantize_Hadamard, eden_quantize, eden_compress, eden_decompress, EdenMessage, rht_signs,
                   randomized_hadamard_transform, randomized_inverse_hadamard_transform)
from .quicfl import (QuicFLReceiver, QuicFLSender, QuicFLMessages, QUICFL_quantize, quicfl_compress,
                     quicfl_decompress, quicfl_decompress_messages, quicfl_quantize, set_tables_prefix)
from ._lib import UQError, load as load_library, library_path
from .distributed import ShardedDME, shard_range, sharded_client_mean, sharded_quantize_mean
from .dme import DISTRIBUTIONS, Suspended, legacy_draw, nmse_simulation
from .pipeline import DMEPipeline, codes4_fits
from .fl_stats import compute_nmse_stats_auto, data_format, round_nmse
from .outpool import set_output_pool

__all__ = [
    "QuicFLReceiver", "QuicFLSender", "QuicFLMessages", "QUICFL_quantize", "quicfl_compress", "quicfl_decompress",
    "quicfl_decompress_messages", "quicfl_quantize", "set_tables_prefix",
    "RATE_TABLE", "rate_to_m", "Type_unbiased_quantize", "quantize_dequantize", "client_mean",
    "quantize_mean", "l1_torch_order", "draw_uniforms", "set_torch_threads", "get_torch_threads",
    "check_status", "UQError", "load_library", "library_path", "shard_range", "sharded_client_mean",
    "sharded_quantize_mean", "DISTRIBUTIONS", "Suspended", "legacy_draw", "nmse_simulation", "quantize_encode", "decode", "codes_mean",
    "TypeCodes", "Type_biased_quantize", "biased_quantize", "EDEN_quantize_Hadamard", "eden_quantize",
    "eden_compress", "eden_decompress", "EdenMessage", "rht_signs", "randomized_hadamard_transform",
    "randomized_inverse_hadamard_transform", "compute_nmse_stats_auto", "data_format", "round_nmse",
    "DMEPipeline", "codes4_fits", "ShardedDME", "TypeMessages", "encode_messages", "decode_messages", "set_output_pool",
]
