"""GPU parity of torch.norm's CPU order (AS:329, the EDEN sender's norm) through the C-ABI
entry uq_eden_norm_f32: the sequential chains (KE2, mode 1), the segmented chains (KE2s,
mode 2) and the automatic choice (mode 0) against the C oracle, bit for bit, on vectors
that cross binades at every scale, meet exact ties, underflow, overflow, hold zero runs,
spikes, NaN and Inf (tests/norm_cases.py)."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import uq_oracle_c as C
from tests.norm_cases import norm_cases, same_bits

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib(gpu_ready):
    from uqdme_amd import _lib
    return _lib


def _norm(L, x: torch.Tensor, mode: int) -> np.ndarray:
    n, D = x.shape
    b = ctypes.c_size_t()
    L.check(L.load().uq_eden_norm_workspace_bytes(n, D, ctypes.byref(b)), "norm ws")
    ws = torch.empty(max(1, b.value), dtype=torch.uint8, device=x.device)
    out = torch.full((n,), float("nan"), device=x.device)
    L.check(L.load().uq_eden_norm_f32(x.data_ptr(), n, D, mode, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                      torch.cuda.current_stream().cuda_stream), f"norm mode {mode}")
    return out.cpu().numpy()


@pytest.mark.parametrize("D", [1 << 14, 1 << 17, 1 << 20])
def test_segmented_norm_adversarial_vs_oracle(lib, D):
    cases = norm_cases(D)
    X = np.stack([v for _, v in cases])
    with np.errstate(all="ignore"):
        ref = [C.torch_norm2(v) for v in X]
    x = torch.from_numpy(X).cuda()
    for mode in (2, 1, 0):
        got = _norm(lib, x, mode)
        bad = [(cases[i][0], got[i], ref[i]) for i in range(len(cases)) if not same_bits(got[i], ref[i])]
        assert not bad, (D, mode, bad)


def test_segmented_norm_2pow22_and_scales(lib):
    """C4's d = 2^22 (8192 segments per lane) with per-row scales that put the chains in
    different binade ranges."""
    D = 1 << 22
    rng = np.random.default_rng(22)
    X = np.stack([rng.standard_normal(D) * s for s in (1.0, 3e-7, 2e11)]).astype(np.float32)
    ref = [C.torch_norm2(v) for v in X]
    got = _norm(lib, torch.from_numpy(X).cuda(), 2)
    assert all(same_bits(got[i], ref[i]) for i in range(3)), (got, ref)


def test_segmented_norm_max_batch(lib):
    """The largest batch the segmented form takes (256 rows), each row its own scale and
    distribution; and 257 rows are refused in mode 2 (mode 0 then takes the chains)."""
    D = 1 << 14
    rng = np.random.default_rng(256)
    rows = []
    for j in range(256):
        s = 10.0 ** rng.uniform(-15, 15)
        r = rng.standard_normal(D) if j % 3 else rng.laplace(0, 1, D)
        rows.append(r * s)
    X = np.stack(rows).astype(np.float32)
    ref = np.array([C.torch_norm2(v) for v in X])
    x = torch.from_numpy(X).cuda()
    got = _norm(lib, x, 2)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    X2 = torch.cat([x, x[:1]])
    with pytest.raises(lib.UQError):
        _norm(lib, X2, 2)
    got0 = _norm(lib, X2, 0)
    assert np.array_equal(got0[:256].view(np.uint32), ref.view(np.uint32))


def test_drop_in_uses_segmented_norm_and_matches_batch(lib):
    """The per-call drop-in (n = 1, segmented norm) and a 1024-row batch (sequential
    chains) give the same EDEN output bits for the same row and seed."""
    import uqdme
    rng = np.random.default_rng(4)
    d = 300000                                              # D = 2^19, zero-padded
    x = rng.standard_normal((1024, d)).astype(np.float32)
    seeds = [int(s) for s in rng.integers(0, 100, 1024)]
    xt = torch.from_numpy(x).cuda()
    batch = uqdme.eden_quantize(xt, 1, seeds=seeds)
    for j in (0, 511, 1023):
        one = uqdme.eden_quantize(xt[j:j + 1], 1, seeds=[seeds[j]])
        assert torch.equal(one[0].view(torch.int32), batch[j].view(torch.int32)), j


def test_segmented_norm_fuzz_vs_oracle(lib):
    """256 random rows (the largest segmented batch) at D = 2^15 from many distributions and
    scales, few-bit values among them (ties), each against the C oracle."""
    D, n = 1 << 15, 256
    rng = np.random.default_rng(2025)
    rows = []
    for j in range(n):
        kind = j % 8
        if kind == 0:
            r = rng.standard_normal(D) * 10.0 ** rng.uniform(-20, 18)
        elif kind == 1:
            r = rng.uniform(-1, 1, D) * 10.0 ** rng.uniform(-5, 5)
        elif kind == 2:
            r = rng.laplace(1, 2, D)
        elif kind == 3:
            r = rng.lognormal(1, 2, D)
        elif kind == 4:
            r = rng.integers(-(1 << rng.integers(1, 12)), 1 << rng.integers(1, 12), D) * 2.0 ** rng.integers(-30, 10)
        elif kind == 5:
            r = np.where(rng.random(D) < rng.uniform(0.001, 0.2), rng.standard_normal(D), 0.0)
        elif kind == 6:
            r = rng.standard_normal(D) * np.exp(np.linspace(-rng.uniform(0, 30), rng.uniform(0, 30), D))
        else:
            r = rng.choice([-1.5, -0.75, 0.25, 1.0, 3.0], D) * 2.0 ** rng.integers(-12, 12)
        rows.append(r)
    with np.errstate(all="ignore"):
        X = np.stack(rows).astype(np.float32)
        ref = np.array([C.torch_norm2(v) for v in X])
    got = _norm(lib, torch.from_numpy(X).cuda(), 2)
    bad = [j for j in range(n) if not same_bits(got[j], ref[j])]
    assert not bad, [(j, got[j], ref[j]) for j in bad[:5]]
