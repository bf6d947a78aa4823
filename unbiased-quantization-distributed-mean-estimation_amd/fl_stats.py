"""FL NMSE statistics of the Flower quantization hook.

Restates SImulation_Results_datasets/MNIST/Codes/NMSE_Results.py (identical in the CIFAR10
and Fashion_MNIST copies):

  compute_nmse_stats_auto(parent_folder, sampled_clients_per_round=5)   NMSE_Results.py:43-140
      walks <parent>/<scheme>/<rate>/NMSE_info_<k>.pkl, the files the client hook writes
      (Type_unbiased.py:171-197: [quantization error vector, ||gradient||]), drops the
      initialisation file NMSE_info_1.pkl, and per round of `sampled_clients_per_round`
      files computes  ||sum(err)/c||^2 / (sum(||g||^2)/c)            (:83-112)
      then the max / mean over rounds (nan-aware, :115-121), formatted by data_format (:7-41)
      and written to an .xlsx (:137-140).
  data_format(x)                                                       NMSE_Results.py:7-41
  round_nmse(errors, grad_norms)                                       the per-round formula

Differences, all on the I/O edge: the reference hard-codes the output name
NMSE_stats_MNIST.xlsx and needs openpyxl; here the name is a parameter and, when openpyxl is
not importable (this image), the same table is written as CSV beside it.  The function also
returns the rows.  Sums of the error vectors stay on the device they were saved from (the
hook saves device tensors), as in the reference.

NMSE_info_*.pkl files are plain pickles (the reference's format), so they are read with
pickle: point this only at directories your own runs wrote.
"""
from __future__ import annotations

import math
import os
import pickle

import numpy as np

__all__ = ["compute_nmse_stats_auto", "data_format", "round_nmse"]


def data_format(data) -> str:
    """NMSE_Results.py:7-41: 3 truncated decimals in [0.01, 1e4), else truncated
    scientific notation (2 significant digits in [0.001, 0.01), 5 otherwise)."""
    if np.isnan(data):
        return "nan"
    if 0.01 <= data < 1e4:
        return f"{int(data * 1000) / 1000:.3f}"
    sig = 2 if 0.001 <= data < 0.01 else 5
    mant, exp = f"{data:.12e}".split("e")
    digits = mant.rstrip("0").rstrip(".").replace(".", "")[:sig]
    new_mant = digits[0] + "." + digits[1:] if len(digits) > 1 else digits
    return f"{new_mant}e{int(exp)}"


def round_nmse(errors, grad_norms, sampled_clients_per_round=None):
    """One round (NMSE_Results.py:94-112): errors = the clients' quantization error vectors
    (tensors or arrays, summed in client order), grad_norms = their ||g|| (floats).  Both
    averages divide by `sampled_clients_per_round` (default: the number of records), also
    when a client's file was missing (:88-90, :103-104)."""
    c = len(errors) if sampled_clients_per_round is None else sampled_clients_per_round
    num = None
    den = None
    for e, g in zip(errors, grad_norms):
        if num is None:
            num, den = e, g ** 2
        else:
            num = num + e                       # the reference's `+=` on the first file's object
            den += g ** 2
    if num is None:
        return None
    avg_error = num / c
    avg_gsq = den / c
    if hasattr(avg_error, "cpu"):
        avg_error = avg_error.cpu().numpy()
    if hasattr(avg_gsq, "cpu"):
        avg_gsq = avg_gsq.cpu().numpy()
    return np.nan if avg_gsq == 0 else np.linalg.norm(avg_error) ** 2 / avg_gsq


def _load_info(path):
    with open(path, "rb") as f:
        return pickle.load(f)                   # [quant_error_vector, gradient_norm]


def compute_nmse_stats_auto(parent_folder: str, sampled_clients_per_round: int = 5,
                            excel_filename: str = "NMSE_stats_MNIST.xlsx", verbose: bool = True):
    """NMSE_Results.py:43-140 over `parent_folder`; returns the result rows."""
    log = print if verbose else (lambda *a, **k: None)
    results = []
    c = sampled_clients_per_round
    for scheme in os.listdir(parent_folder):
        scheme_path = os.path.join(parent_folder, scheme)
        if not os.path.isdir(scheme_path):
            continue
        log(f"Scheme: {scheme}")
        for rate in os.listdir(scheme_path):
            rate_path = os.path.join(scheme_path, rate)
            if not os.path.isdir(rate_path):
                continue
            log(f"  Rate folder: {rate}")
            files = sorted(f for f in os.listdir(rate_path) if f.startswith("NMSE_info_") and f.endswith(".pkl"))
            effective_total = len(files) - 1        # NMSE_info_1.pkl is the initialisation call
            expected_rounds = effective_total // c
            if effective_total % c != 0:
                log(f"Warning: (total files - 1) = {effective_total} is not exactly divisible by {c}.")
                log(f"Processing {expected_rounds} complete rounds only.")
            nmse_rounds = []
            for r in range(expected_rounds):
                errs, norms = [], []
                for j in range(c):
                    path = os.path.join(rate_path, f"NMSE_info_{r * c + j + 2}.pkl")
                    if not os.path.exists(path):
                        log(f"Warning: {os.path.basename(path)} not found; skipping.")
                        continue
                    e, g = _load_info(path)
                    errs.append(e)
                    norms.append(g)
                v = round_nmse(errs, norms, c)
                if v is not None:
                    nmse_rounds.append(v)
            if nmse_rounds:
                arr = np.array(nmse_rounds)
                max_nmse, avg_nmse = np.nanmax(arr), np.nanmean(arr)
                log(f"Computed over {len(arr)} rounds:\nMax NMSE: {max_nmse}\nAvg NMSE: {avg_nmse}")
            else:
                max_nmse = avg_nmse = math.nan
                log("No complete rounds processed.")
            results.append({"Scheme": scheme, "Rate Folder": rate, "Total Files": effective_total,
                            "No of Rounds": expected_rounds, "Clients Per Round": c,
                            "Max NMSE": data_format(max_nmse), "Avg NMSE": data_format(avg_nmse),
                            "max_nmse": float(max_nmse), "avg_nmse": float(avg_nmse)})
    if excel_filename:
        _write_table(results, excel_filename, log)
    return results


def _write_table(rows, excel_filename, log):
    import pandas as pd
    cols = ["Scheme", "Rate Folder", "Total Files", "No of Rounds", "Clients Per Round", "Max NMSE", "Avg NMSE"]
    df = pd.DataFrame([{k: r[k] for k in cols} for r in rows], columns=cols)
    try:
        import openpyxl  # noqa: F401
        df.to_excel(excel_filename, index=False, engine="openpyxl")
        log(f"NMSE statistics saved in: {excel_filename}")
    except ImportError:
        out = os.path.splitext(excel_filename)[0] + ".csv"
        df.to_csv(out, index=False)
        log(f"openpyxl not available: NMSE statistics saved in: {out}")
