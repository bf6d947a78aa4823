"""CPU: the QUIC-FL sender's table checks (host logic, no GPU).  AS:489's bernoulli draws one
32-bit generator word per coordinate only for a float32 p (ATen's bernoulli_distribution<double>
takes a 64-bit draw for a float64 p), so tables are taken as float32 or refused, never cast."""
import numpy as np
import pytest
import torch

import uqdme
from uqdme_amd import quicfl as q


def tables(px=np.float32, pp=np.float32):
    X = (np.arange(12, dtype=np.float64) % 3).reshape(3, 4).astype(px)
    p = (np.arange(12, dtype=np.float64) / 16).reshape(3, 4).astype(pp)
    return {1: (X, p, {"h_len": 4, "delta": 0.5})}


def test_float32_tables_accepted():
    s = uqdme.QuicFLSender(device="cpu", tables=tables())
    assert s.sender_table_p[1].dtype == torch.float32 and s.sender_table_X[1].dtype == torch.float32
    assert s.half_table_size[1] == 4


def test_float64_p_refused():
    with pytest.raises(TypeError, match="float32"):
        uqdme.QuicFLSender(device="cpu", tables=tables(pp=np.float64))


def test_float64_x_exact_values_taken_as_float32():
    s = uqdme.QuicFLSender(device="cpu", tables=tables(px=np.float64))
    assert s.sender_table_X[1].dtype == torch.float32


def test_float64_x_inexact_refused():
    t = tables(px=np.float64)
    t[1][0][0, 0] = 0.1
    with pytest.raises(TypeError, match="exactly"):
        uqdme.QuicFLSender(device="cpu", tables=t)


def test_prefix_tables_keep_their_dtype(tmp_path):
    fn = str(tmp_path / "1_X_6_h_256_q_")
    X, p, dd = tables()[1]
    torch.save(torch.from_numpy(X), fn + "sender_table_X.pt")
    torch.save(torch.from_numpy(p.astype(np.float64)), fn + "sender_table_p.pt")
    open(fn + "data.txt", "w").write(repr(dd))
    tx, tp, d2 = q.QuicFLSender.sender_table(fn)
    assert tp.dtype == torch.float64 and d2 == dd
    with pytest.raises(TypeError):
        uqdme.QuicFLSender(device="cpu", bits=[1], sr_bits=[6], prefix=str(tmp_path) + "/")


def test_tables_prefix(monkeypatch):
    q.set_tables_prefix("/some/dir")
    try:
        assert q.default_tables_prefix() == "/some/dir/"
    finally:
        q.set_tables_prefix(None)
    monkeypatch.setenv("UQDME_QUICFL_TABLES", "/env/dir")
    assert q.default_tables_prefix() == "/env/dir/"
