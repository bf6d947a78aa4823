"""Rate table of the reference (NMSE_Results/Codes/All_Schemes.py:614-620).

For each R (bits per dimension) the reference sets m = int(l_R * d) (AS:622-623):
log2 |{k in Z^d : sum |k_i| = m}| / d ~= R.
"""
from __future__ import annotations

RATE_TABLE = {
    0.5: 0.08282, 1: 0.21403, 1.5: 0.39443, 2: 0.63752,
    2.5: 0.96656, 3: 1.41725, 3.5: 2.04187, 4: 2.91504,
    4.5: 4.14217, 5: 5.87195, 5.5: 8.31416, 6: 11.76507,
    6.5: 16.64332, 7: 23.54075, 7.5: 33.29414, 8: 47.0868,
    8.5: 66.59204, 9: 94.17625, 9.5: 133.18596, 10: 188.35383,
}


def rate_to_m(bits_per_dimension, d: int) -> int:
    """AS:622-623.  Unknown keys raise KeyError exactly like the reference's dict lookup."""
    return int(RATE_TABLE[bits_per_dimension] * d)
