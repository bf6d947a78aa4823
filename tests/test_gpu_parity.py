"""GPU parity: the HIP path (through the C-ABI) against the reference's golden fixtures
and the CPU oracle on the same seeded inputs.  Bit-exact unless a test says otherwise;
the north_star's floating-point tolerance (NMSE within 1e-6 relative) is written where
it applies."""
import numpy as np
import pytest
import torch

from oracle import uq_oracle as O
from oracle import uq_oracle_c as C
from tests import golden_data as G

pytestmark = pytest.mark.gpu
f32 = np.float32


@pytest.fixture(scope="module")
def uq(gpu_ready):
    import uqdme
    return uqdme


def dev(a):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=f32)).cuda()


def test_c1_harness_bit_exact(uq):
    z = G.c1()
    x = dev(z["x"])
    q1, l1 = uq.quantize_dequantize(x, 1, X=z["X1"], torch_threads=1, return_l1=True)
    q2 = uq.quantize_dequantize(x, 2, X=z["X2"], torch_threads=1)
    assert G.bits_equal(q1.cpu().numpy(), z["q1"])
    assert G.bits_equal(q2.cpu().numpy(), z["q2"])
    e1 = uq.client_mean(q1, 16).cpu().numpy()
    e2 = uq.client_mean(q2, 16).cpu().numpy()
    assert G.bits_equal(e1, z["est1"])
    assert G.bits_equal(e2, z["est2"])
    n1 = O.script_nmse(e1, z["emp"], float(z["vec_norm_squared"]), 16)
    n2 = O.script_nmse(e2, z["emp"], float(z["vec_norm_squared"]), 16)
    # bit for bit (north_star allows 1e-6 relative): est is bit-exact and the oracle's
    # script_nmse restates torch.norm's f32 order
    assert n1 == float(z["nmse1"]) and n2 == float(z["nmse2"]), (n1, n2)
    ref_l1 = [O.l1_torch_order(z["x"][j], 1) for j in range(16)]
    assert G.bits_equal(l1.cpu().numpy(), np.array(ref_l1, f32))


def test_fused_quantize_mean_matches_two_step(uq):
    z = G.c1()
    x = dev(z["x"])
    est = uq.quantize_mean(x, 1, X=z["X1"], n_div=16, torch_threads=1)
    assert G.bits_equal(est.cpu().numpy(), z["est1"])


def test_edge_cases_bit_exact(uq):
    n = 0
    for name, R, X, x, q in G.edge_cases():
        got = uq.quantize_dequantize(dev(x[None]), R, X=[X], torch_threads=1)[0].cpu().numpy()
        assert G.bits_equal(got, q), (name, R, G.n_mismatch(got, q))
        n += 1
    assert n > 40


def test_spec_vectors_mid_bit_exact(uq):
    for sp, q, _, _ in G.spec_vectors(large=False):
        x = G.spec_gen(sp)
        got, l1 = uq.quantize_dequantize(dev(x[None]), sp["R"], X=[sp["X"]], torch_threads=sp["threads"],
                                         return_l1=True)
        assert l1.cpu().numpy()[0] == f32(sp["l1"]), sp
        got = got[0].cpu().numpy()
        assert G.bits_equal(got, q), (sp["dist"], sp["d"], sp["R"], G.n_mismatch(got, q))


def test_spec_vectors_large_bit_exact(uq):
    for sp, _, pos, qs in G.spec_vectors(large=True):
        x = G.spec_gen(sp)
        got, l1 = uq.quantize_dequantize(dev(x[None]), sp["R"], X=[sp["X"]], torch_threads=sp["threads"],
                                         return_l1=True)
        assert l1.cpu().numpy()[0] == f32(sp["l1"]), sp
        got = got[0].cpu().numpy()
        assert G.bits_equal(got[pos], qs), sp
        assert G.sha(got) == sp["q_sha256"], (sp["dist"], sp["d"], sp["R"], sp["threads"])


@pytest.mark.parametrize("T", [1, 2, 3, 5, 7, 8, 16, 64, 65, 128, 256])
def test_l1_torch_order_sweep(uq, T):
    rng = np.random.default_rng(100 + T)
    sizes = [1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 511, 512, 513, 8191, 8192, 8193,
             32767, 32768, 32769, 65535, 65536, 65537, 100003, 172554, 262144, 1 << 20]
    for d in sizes:
        x = (rng.standard_normal((3, d)) * rng.choice([1e-30, 1e-3, 1.0, 1e3, 1e30])).astype(f32)
        got = uq.l1_torch_order(dev(x), T).cpu().numpy()
        ref = np.array([C.l1_torch_order(x[j], T) for j in range(3)], f32)
        assert G.bits_equal(got, ref), (d, T, got, ref)


def test_random_batches_vs_oracle(uq):
    rng = np.random.default_rng(7)
    gens = [lambda s: rng.normal(0, 1, s), lambda s: rng.laplace(1, 2, s), lambda s: rng.lognormal(1, 2, s),
            lambda s: rng.gamma(2, 2, s), lambda s: rng.choice(2, s, p=[.3, .7]).astype(float),
            lambda s: rng.uniform(-1, 1, s)]
    total = 0
    for d in (1, 3, 4, 17, 100, 1001, 4095, 4096, 4097, 12289, 65536, 100003, 172554):
        for gi, g in enumerate(gens):
            n = 5
            x = g((n, d)).astype(f32)
            for R in (0.5, 1, 2, 6.5, 10):
                X = rng.random(n).astype(f32)
                m = O.rate_to_m(R, d)
                got = uq.quantize_dequantize(dev(x), m=m, X=X, torch_threads=1).cpu().numpy()
                ref, _ = C.quantize_batch(x, m, X, 1)
                bad = G.n_mismatch(got, ref)
                assert bad == 0, (d, gi, R, bad)
                total += 1
    # config C3's two distributions at its d = 2^20 (Laplace(1, 2), U(-1, 1))
    for gi in (1, 5):
        x = gens[gi]((5, 1 << 20)).astype(f32)
        for R in (1, 2):
            X = rng.random(5).astype(f32)
            m = O.rate_to_m(R, 1 << 20)
            got = uq.quantize_dequantize(dev(x), m=m, X=X, torch_threads=1).cpu().numpy()
            ref, _ = C.quantize_batch(x, m, X, 1)
            assert G.n_mismatch(got, ref) == 0, (gi, R)
            total += 1
    assert total > 300


def test_full_size_c2_subset_bit_exact_and_properties(uq):
    """C2 shape (d=2^20): 32 clients bit-exact against the C oracle; then the whole
    1024-client batch through size-independent properties: sum k == m per client and
    |q| = L1*k/m reconstruction."""
    d = 1 << 20
    g = torch.Generator(device="cuda").manual_seed(0)
    n = 1024
    x = torch.randn(n, d, generator=g, device="cuda")
    X = uq.draw_uniforms(n, torch.Generator().manual_seed(1))
    m = O.rate_to_m(1, d)
    q, l1 = uq.quantize_dequantize(x, m=m, X=X, torch_threads=1, return_l1=True)
    torch.cuda.synchronize()
    uq.check_status()
    xs = x[:32].cpu().numpy()
    ref, ref_l1 = C.quantize_batch(xs, m, X[:32].numpy(), 1)
    assert G.bits_equal(l1[:32].cpu().numpy(), ref_l1)
    assert G.n_mismatch(q[:32].cpu().numpy(), ref) == 0
    # Lattice-count sum.  Telescoping AS:636-637 gives sum(r) = floor(c_d - X) + 1 and
    # c_d = m - sum(fl) + eps with |eps| << 1 (f32 rounding of p), so the reference
    # itself yields sum(k) = m exactly unless X is within |eps| of 0 or 1, where it is
    # m -+ 1 (the oracle reproduces those clients bit-for-bit, see tools/debug_full.py).
    k = torch.round(q.abs().double() * m / l1.double()[:, None])
    ks = k.sum(dim=1)
    assert torch.all((ks - m).abs() <= 1)
    mid = (X > 0.05) & (X < 0.95)
    assert torch.all(ks[mid.cuda()] == m)
    # |q| * m / L1 is an integer count up to f32 rounding
    assert torch.all((q.abs().double() * m / l1.double()[:, None] - k).abs() < 1e-3)
    assert torch.all(k >= 0)


def test_unbiasedness_statistical(uq):
    """E[q] = x: average many independent quantizations of one vector."""
    d, reps = 4096, 4000
    rng = np.random.default_rng(3)
    x = rng.standard_normal(d).astype(f32)
    xb = dev(np.repeat(x[None], reps, axis=0))
    X = uq.draw_uniforms(reps, torch.Generator().manual_seed(5))
    q = uq.quantize_dequantize(xb, 1, X=X, torch_threads=1)
    mean = q.double().mean(0).cpu().numpy()
    L = float(np.abs(x).sum())
    m = O.rate_to_m(1, d)
    # per-coordinate std of q is <= L/m * 0.5; the error of the mean shrinks by sqrt(reps)
    tol = 6 * 0.5 * L / m / np.sqrt(reps)
    assert np.max(np.abs(mean - x)) < tol


def test_drop_in_matches_reference_semantics(uq):
    rng = np.random.default_rng(21)
    uq.set_torch_threads(1)
    try:
        for d in (1, 5, 1000, 4099):
            x = rng.standard_normal(d).astype(f32)
            for R in (1, 2):
                torch.manual_seed(77)
                got = uq.Type_unbiased_quantize(x, R)
                assert got.is_cuda and got.dtype == torch.float32 and got.shape == (d,)
                torch.manual_seed(77)
                X = torch.rand(1).item()
                ref = O.type_unbiased_quantize(x, R, X)
                assert G.bits_equal(got.cpu().numpy(), ref)
                # one RNG draw consumed per call, like AS:634
                torch.manual_seed(77)
                uq.Type_unbiased_quantize(torch.from_numpy(x), R)
                a = torch.rand(1)
                torch.manual_seed(77)
                torch.rand(1)
                b = torch.rand(1)
                assert a.item() == b.item()
        xin = torch.from_numpy(rng.standard_normal(64).astype(f32)).cuda()
        keep = xin.clone()
        out = uq.Type_unbiased_quantize(xin, 1)
        assert torch.equal(xin, keep) and out.data_ptr() != xin.data_ptr()
        with pytest.raises(KeyError):
            uq.Type_unbiased_quantize(xin, 3.3)
        with pytest.raises(RuntimeError):
            uq.Type_unbiased_quantize(torch.zeros(4, 4), 1)
        assert uq.Type_unbiased_quantize(torch.zeros(0), 1).numel() == 0
        # float64 and list inputs are rounded to f32 like torch.tensor(..., float32)
        x64 = rng.standard_normal(300)
        torch.manual_seed(3)
        a = uq.Type_unbiased_quantize(x64, 1).cpu().numpy()
        torch.manual_seed(3)
        b = uq.Type_unbiased_quantize(list(x64.astype(f32)), 1).cpu().numpy()
        assert G.bits_equal(a, b)
    finally:
        uq.set_torch_threads(None)


def test_deterministic_repeat_and_unaligned(uq):
    rng = np.random.default_rng(9)
    d = 300001   # not a multiple of 4 -> unaligned rows -> scalar-load path
    x = rng.laplace(1, 2, (6, d)).astype(f32)
    X = rng.random(6).astype(f32)
    a = uq.quantize_dequantize(dev(x), 2, X=X, torch_threads=1).cpu().numpy()
    b = uq.quantize_dequantize(dev(x), 2, X=X, torch_threads=1).cpu().numpy()
    assert G.bits_equal(a, b)
    ref, _ = C.quantize_batch(x, O.rate_to_m(2, d), X, 1)
    assert G.n_mismatch(a, ref) == 0
    # offset view: base pointer not 16-B aligned
    big = dev(np.concatenate([np.zeros(1, f32), x.reshape(-1)]))
    xv = big[1:].view(6, d)
    c = uq.quantize_dequantize(xv, 2, X=X, torch_threads=1).cpu().numpy()
    assert G.bits_equal(a, c)


def test_client_mean_order_and_accumulate(uq):
    rng = np.random.default_rng(4)
    for n, d in ((1, 10), (7, 1001), (33, 4096), (200, 65536)):
        q = rng.standard_normal((n, d)).astype(f32)
        got = uq.client_mean(dev(q), n).cpu().numpy()
        assert G.bits_equal(got, C.client_mean(q, n)), (n, d)
        est = uq.client_mean(dev(q[: n // 2 + 1]), n)
        if n // 2 + 1 < n:
            est = uq.client_mean(dev(q[n // 2 + 1:]), n, est=est, accumulate=True)
        assert G.bits_equal(est.cpu().numpy(), C.client_mean(q, n)), (n, d, "split")


def test_single_row_ragged_d_vector_path_and_many_threads(uq):
    """n = 1 uses the vector loads for any d (the row is 16-byte aligned); the ragged end
    must not read past d; any torch_threads (here up to 128) is accepted."""
    rng = np.random.default_rng(77)
    for d in (172554, 4097, 8195, 1 << 16 | 3):
        x = rng.standard_normal(d).astype(f32)
        for T in (1, 8, 128):
            q = uq.quantize_dequantize(dev(x).view(1, d), 1, X=[0.37], torch_threads=T).cpu().numpy()[0]
            exp = C.quantize_batch(x[None], O.rate_to_m(1, d), np.array([0.37], f32), T)[0][0]
            assert G.bits_equal(q, exp), (d, T, G.n_mismatch(q, exp))


def test_l1_many_chunks_over_finalize_waves(uq):
    """K1b finishes torch chunks on 8 waves (chunk c on wave c % 8) and adds the chunk
    results in chunk order: more than 8 chunks (16, 33) and ragged chunk sizes must keep the
    torch CPU cascade bits (ATen: min(T, ceil(d / 32768)) chunks)."""
    rng = np.random.default_rng(78)
    d = (1 << 20) + 5
    x = rng.standard_normal((2, d)).astype(f32)
    m = O.rate_to_m(1, d)
    X = np.array([0.61, 0.05], f32)
    for T in (16, 37):
        q = uq.quantize_dequantize(dev(x), m=m, X=X, torch_threads=T).cpu().numpy()
        exp = C.quantize_batch(x, m, X, T)[0]
        assert G.bits_equal(q, exp), (T, G.n_mismatch(q, exp))
    # the biased quantizer's m' (k' summed by the same cascade, with its radix histogram)
    qb = uq.biased_quantize(dev(x[:1]), m=m, torch_threads=16, ties="torch").cpu().numpy()[0]
    eb, *_ = C.biased_quantize(x[0], m, 16, 0)
    assert G.bits_equal(qb, eb), G.n_mismatch(qb, eb)


def _division_guard_batch(n, d, rng):
    """Rows that drive every branch of the kernels' x / den (div_plan / div4): ordinary
    rows (fast path), rows with tiny, subnormal, huge and non-finite elements (per-element
    IEEE fallback), zero-heavy rows (zeros stay on the fast path), a row with L1 >= 2^40
    (whole client on the IEEE division), an all-zero row (den = 1e-12) and rows whose
    quotients all fall under the guard threshold."""
    x = rng.standard_normal((n, d)).astype(f32)
    for j in range(n):
        kind = j % 8
        idx = rng.integers(0, d, size=max(1, d // 64))
        if kind == 1:
            x[j, idx] *= np.float32(1e-40)                        # subnormal elements
        elif kind == 2:
            x[j, idx] = (rng.standard_normal(idx.size) * 1e-25).astype(f32)   # tiny normals
        elif kind == 3:
            x[j] *= np.float32(1e10)                              # L1 >= 2^40: IEEE path per client
        elif kind == 4:
            x[j, rng.random(d) < 0.9] = 0.0                       # sparse: zeros on the fast path
        elif kind == 5:
            x[j] *= np.float32(1e-30)                             # every quotient under the threshold
        elif kind == 6:
            x[j, idx[:3]] = [np.inf, -np.inf, np.nan][: min(3, idx.size)]
        elif kind == 7:
            x[j, idx] *= np.float32(1e30)                         # huge elements, q still finite
    x[n // 2] = 0.0                                               # den = 1e-12 exactly
    return x


@pytest.mark.parametrize("n,d", [(264, 4100), (3, 70001)])
def test_division_guards_stream_and_small_batch(uq, n, d):
    """x / den is computed with a per-client reciprocal and two fma corrections; every
    guard branch must give the IEEE quotient's bits (n >= 256: stream kernel, one
    workgroup per client; n = 3: the small-batch kernels)."""
    rng = np.random.default_rng(4242 + n)
    x = _division_guard_batch(n, d, rng)
    assert float(np.abs(x[3 % n]).astype(np.float64).sum()) >= 2.0 ** 40 or n < 4
    X = rng.random(n).astype(f32)
    for R in (1, 4):
        m = O.rate_to_m(R, d)
        got = uq.quantize_dequantize(dev(x), m=m, X=X, torch_threads=1).cpu().numpy()
        ref, _ = C.quantize_batch(x, m, X, 1)
        assert G.n_mismatch(got, ref) == 0, (n, d, R, [G.n_mismatch(got[j], ref[j]) for j in range(n)][:16])


@pytest.mark.parametrize("n,d", [(6, 1 << 20), (6, (1 << 20) + 3), (50, 100004)])
def test_k2_forms_agree_stream_segmented_per_tile(uq, n, d):
    """The K2 forms -- stream (n >= 256, one workgroup per client), segmented stream (a
    few aligned clients with >= 1024 tiles; (50, 100004): 13 segments of 2 tiles, the last
    one a single ragged tile) and one workgroup per tile (n = 1, unaligned rows) -- all
    reproduce the sequential fp64 cumsum, so the same client gives the same bits whichever
    form runs; two rows also against the C oracle."""
    rng = np.random.default_rng(d % 1000 + n)
    x = rng.laplace(1, 2, (n, d)).astype(f32)
    X = rng.random(n).astype(f32)
    m = O.rate_to_m(2, d)
    xd = dev(x)
    phased = uq.quantize_dequantize(xd, m=m, X=X, torch_threads=1).cpu().numpy()
    for j in range(n):
        one = uq.quantize_dequantize(xd[j:j + 1].contiguous(), m=m, X=X[j:j + 1], torch_threads=1).cpu().numpy()[0]
        assert G.n_mismatch(one, phased[j]) == 0, ("n = 1 vs batch", j)
    if d % 4 == 0:
        filler = torch.randn(256 - n, d, device="cuda")
        big = torch.cat([xd, filler])
        Xb = np.concatenate([X, rng.random(256 - n).astype(f32)])
        stream = uq.quantize_dequantize(big, m=m, X=Xb, torch_threads=1)[:n].cpu().numpy()
        assert G.n_mismatch(stream, phased) == 0, "stream vs phased"
    ref, _ = C.quantize_batch(x[:2], m, X[:2], 1)
    assert G.n_mismatch(phased[:2], ref) == 0
    tc, q = uq.quantize_encode(xd, m=m, X=X, torch_threads=1, return_q=True)
    assert G.bits_equal(q.cpu().numpy(), phased)
    assert G.bits_equal(uq.decode(tc).cpu().numpy(), phased)


@pytest.mark.parametrize("R", [0.5, 6.5, 10])
def test_stream_form_all_rates_and_ragged_rows(uq, R):
    """n >= 256 (stream kernel) at low and high rates: k >= 256 takes the arithmetic output
    path (the running-max bound on the table), heavy tails make large k, and d is not a
    multiple of the tile."""
    rng = np.random.default_rng(int(R * 10))
    n, d = 256, 3 * 4096 + 20
    x = rng.laplace(1, 2, (n, d)).astype(f32)
    x[::7] *= np.float32(50.0)
    X = rng.random(n).astype(f32)
    m = O.rate_to_m(R, d)
    got = uq.quantize_dequantize(dev(x), m=m, X=X, torch_threads=1).cpu().numpy()
    ref, _ = C.quantize_batch(x, m, X, 1)
    assert G.n_mismatch(got, ref) == 0
    tc, q = uq.quantize_encode(dev(x), m=m, X=X, torch_threads=1, return_q=True)
    assert G.bits_equal(q.cpu().numpy(), ref)


def test_l1_thread_counts_match_torch_fixture(uq):
    """K1 at T = 1..256 torch threads against torch's own L1 bits (tests/golden/l1_threads.json):
    the two-pass reduction's per-thread buffer is summed by the same cascade."""
    by_vec = {}
    for r, x in G.l1_threads():
        key = (r["seed"], r["d"])
        if key not in by_vec:
            by_vec[key] = (dev(x).view(1, -1), [])
        by_vec[key][1].append(r)
    n = 0
    for xd, recs in by_vec.values():
        for r in recs:
            got = uq.l1_torch_order(xd, r["threads"]).cpu().numpy()[0]
            assert got.view(np.uint32) == np.uint32(r["l1_bits"]), (r["d"], r["threads"], got, r["l1"])
            n += 1
    assert n >= 140


@pytest.mark.parametrize("T", [64, 65, 128, 256])
def test_c4_size_many_torch_threads_bit_exact(uq, T):
    """d = 2^22 (config C4) with as many torch threads as a many-core host gives: 128 chunks
    at T >= 128.  Unbiased and biased quantizers bit-exact against the C oracle."""
    rng = np.random.default_rng(T)
    d = 1 << 22
    x = rng.standard_normal((2, d)).astype(f32)
    X = np.array([0.41, 0.93], f32)
    m = O.rate_to_m(1, d)
    q = uq.quantize_dequantize(dev(x), m=m, X=X, torch_threads=T).cpu().numpy()
    ref, _ = C.quantize_batch(x, m, X, T)
    assert G.n_mismatch(q, ref) == 0, T
    qb = uq.biased_quantize(dev(x[:1]), m=m, torch_threads=T, ties="torch").cpu().numpy()[0]
    eb, *_ = C.biased_quantize(x[0], m, T, 0)
    assert G.bits_equal(qb, eb), G.n_mismatch(qb, eb)


def test_drop_in_default_torch_threads_c4_size(uq):
    """The drop-in with the host's default torch thread count (whatever this box gives,
    often > 64 on a many-core host) at d = 2^22: same bits as the C oracle with that T."""
    uq.set_torch_threads(None)
    T = uq.get_torch_threads()
    rng = np.random.default_rng(5)
    x = rng.standard_normal(1 << 22).astype(f32)
    torch.manual_seed(123)
    got = uq.Type_unbiased_quantize(x, 1).cpu().numpy()
    torch.manual_seed(123)
    X = torch.rand(1).item()
    ref = C.quantize_batch(x[None], O.rate_to_m(1, x.shape[0]), np.array([X], f32), T)[0][0]
    assert G.n_mismatch(got, ref) == 0, T
    torch.manual_seed(123)
    gb = uq.Type_biased_quantize(x, 1).cpu().numpy()
    eb, *_ = C.biased_quantize(x, O.rate_to_m(1, x.shape[0]), T, 0)
    assert G.bits_equal(gb, eb), (T, G.n_mismatch(gb, eb))
