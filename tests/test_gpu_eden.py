"""GPU parity of EDEN + RHT (AS:95-153, 324-413, 792-811) through the C-ABI: diagonal, bins,
scale and outputs bit for bit with the reference fixtures and the oracle (the scale's
torch.dot in MKL sdot's order, eden_dot_kernel; oracle/uq_eden.py:torch_dot)."""
import numpy as np
import pytest
import torch

from oracle import uq_eden as E
from tests import golden_data as G

pytestmark = pytest.mark.gpu


def same_f32(a, b) -> bool:
    a, b = np.float32(a), np.float32(b)
    return bool(a.view(np.uint32) == b.view(np.uint32)) or (np.isnan(a) and np.isnan(b))


@pytest.fixture(scope="module")
def uq(gpu_ready):
    import uqdme
    return uqdme


@pytest.fixture(scope="module")
def fx():
    return G.eden()


def test_rht_signs_known_answers(uq, fx):
    meta, z = fx
    for dg in meta["diag"]:
        got = uq.rht_signs([dg["seed"]], dg["D"]).cpu().numpy()[0]
        assert np.array_equal(got, z[f"diag_{dg['seed']}_{dg['D']}"]), dg


def test_eden_vs_reference_fixtures(uq, fx):
    meta, z = fx
    for case in meta["cases"]:
        x = torch.as_tensor(G.eden_input(case, z)).cuda().view(1, -1)
        msg = uq.eden_compress(x, case["nbits"], seeds=[case["rseed"]])
        bins = msg.bins.cpu().numpy()[0]
        assert bins.shape[0] == case["D"]
        assert G.sha(bins) == case["bins_sha"], case["idx"]
        assert same_f32(msg.scale.cpu()[0], case["scale"]), case["idx"]           # AS:335, bit for bit
        out = uq.eden_decompress(msg).cpu().numpy()[0]
        full = uq.eden_quantize(x, case["nbits"], seeds=[case["rseed"]]).cpu().numpy()[0]
        assert G.bits_equal(out, full)
        i = case["idx"]
        assert G.sha(out) == case["out_sha"], i
        if f"out{i}" in z.files:
            assert G.bits_equal(out, z[f"out{i}"]), i
        else:
            assert G.bits_equal(out[z[f"pos{i}"]], z[f"outs{i}"]), i


def test_eden_batch_vs_oracle(uq):
    rng = np.random.default_rng(3)
    n, d = 12, 3000
    x = rng.standard_normal((n, d)).astype(np.float32)
    seeds = [0, 5, 99, 5, 1234, 7, 0, 42, 64, 99, 3, 100]     # repeats and seeds outside 0..99
    for nbits in (1, 2):
        out, scale = uq.eden_quantize(torch.as_tensor(x).cuda(), nbits, seeds=seeds, return_scale=True)
        out = out.cpu().numpy()
        scale = scale.cpu().numpy()
        for j in range(n):
            bins, sc, _, _ = E.eden_compress(x[j], nbits, seeds[j])
            assert same_f32(scale[j], sc), j
            exp = E.eden_decompress(bins, sc, nbits, seeds[j], d)
            assert G.bits_equal(out[j], exp), (nbits, j)


def test_drop_in(uq, fx):
    meta, z = fx
    for dd in meta["dropin"]:
        x = z[f"dx{dd['tseed']}_{dd['nbits']}"]
        torch.manual_seed(dd["tseed"])
        y = uq.EDEN_quantize_Hadamard(torch.as_tensor(x), dd["nbits"])
        assert isinstance(y, np.ndarray) and y.dtype == np.float32 and y.shape == x.shape
        assert G.bits_equal(y, z[f"dout{dd['tseed']}_{dd['nbits']}"]), dd
        # exactly one randint(0, 100) draw was consumed
        torch.manual_seed(dd["tseed"])
        assert int(torch.randint(0, 100, (1,))) == dd["drawn_seed"]
    with pytest.raises(ValueError):
        uq.EDEN_quantize_Hadamard(torch.randn(64), 3)


def test_rht_forward_inverse_vs_reference(uq, fx):
    meta, z = fx
    from tests.golden_data import spec_gen
    for r in meta["rht"]:
        x = spec_gen({"dist": "normal", "d": r["dim"], "seed": 700 + r["k"]})
        fwd = uq.randomized_hadamard_transform(torch.as_tensor(x).cuda().view(1, -1), [r["seed"]])
        inv = uq.randomized_inverse_hadamard_transform(fwd, [r["seed"]])
        f, i = fwd.cpu().numpy()[0], inv.cpu().numpy()[0]
        assert G.sha(f) == r["fwd_sha"], r
        assert G.sha(i) == r["inv_sha"], r
        if f"rfwd{r['k']}" in z.files:
            assert G.bits_equal(f, z[f"rfwd{r['k']}"])


def test_eden_c4_size_2pow22_vs_oracle(uq):
    """d = 2^22 (three FWHT passes: 12 + 8 + 2 bits) and a padded d = 2^22 - 3."""
    rng = np.random.default_rng(9)
    for d in (1 << 22, (1 << 22) - 3):
        x = rng.standard_normal(d).astype(np.float32)
        for nbits in (1, 2):
            out, scale = uq.eden_quantize(torch.as_tensor(x).cuda().view(1, -1), nbits, seeds=[37],
                                          return_scale=True)
            bins, sc, _, _ = E.eden_compress(x, nbits, 37)
            assert same_f32(scale.cpu()[0], sc), (d, nbits)
            exp = E.eden_decompress(bins, sc, nbits, 37, d)
            assert G.bits_equal(out.cpu().numpy()[0], exp), (d, nbits)


def test_round_trip_fused_path_matches_compress_decompress(uq):
    """uq_eden_f32 fuses the bins into the receiver's first pass when D > 4096: its bits
    equal compress -> decompress, also for norms outside the fast division range
    [2^-39, 2^40) (tiny, huge, zero vectors), and bins / scale match the oracle (a zero
    vector's 0/0 coordinates go to the last bin, as torch.bucketize puts NaN)."""
    rng = np.random.default_rng(11)
    d = 20000                                                  # D = 32768: two passes
    rows = [rng.standard_normal(d) * s for s in (1.0, 1e-13, 1e9, 1e-15, 1e15, 3e-30)]
    rows.append(np.zeros(d))
    x = np.stack(rows).astype(np.float32)
    seeds = [3, 4, 5, 6, 7, 8, 9]
    for nbits in (1, 2):
        xt = torch.as_tensor(x).cuda()
        msg = uq.eden_compress(xt, nbits, seeds=seeds)
        sep = uq.eden_decompress(msg).cpu().numpy()
        fused = uq.eden_quantize(xt, nbits, seeds=seeds).cpu().numpy()
        assert G.bits_equal(sep, fused), nbits
        for j in range(len(seeds)):
            with np.errstate(invalid="ignore"):
                bins, sc, _, _ = E.eden_compress(x[j], nbits, seeds[j])
            assert np.array_equal(msg.bins.cpu().numpy()[j], bins), (nbits, j)   # NaN -> last bin
            assert same_f32(msg.scale.cpu()[j], sc), (nbits, j)
        assert np.isnan(fused[-1]).all()                        # 0 / 0 norm, as the reference


@pytest.mark.parametrize("d", [1 << 20, (1 << 22) - 5])
def test_rht_forward_two_and_three_passes_vs_oracle(uq, d):
    """The forward RHT writes its last pass straight into the output (two passes) or copies
    from the workspace (three passes)."""
    rng = np.random.default_rng(d % 1000)
    x = rng.standard_normal(d).astype(np.float32)
    fwd = uq.randomized_hadamard_transform(torch.as_tensor(x).cuda().view(1, -1), [21]).cpu().numpy()[0]
    assert G.bits_equal(fwd, E.rht(x, 21))


@pytest.mark.parametrize("d", [1, 2, 3, 5, 16, 100, 4095, 4096, 4097, 5000, 8192, 12289])
def test_eden_dims_across_pass_shapes_vs_oracle(uq, d):
    """Dimensions around the pass shapes: a single generic pass (D < 4096), the low pass
    alone (D = 4096, compress + decompress), two and three passes with the fused round
    trip (D > 4096); bins / scale / outputs against the oracle, and the round trip equal to
    compress -> decompress."""
    rng = np.random.default_rng(d)
    n = 3
    x = rng.standard_normal((n, d)).astype(np.float32)
    seeds = [int(s) for s in rng.integers(0, 100, n)]
    for nbits in (1, 2):
        xt = torch.as_tensor(x).cuda()
        out, scale = uq.eden_quantize(xt, nbits, seeds=seeds, return_scale=True)
        msg = uq.eden_compress(xt, nbits, seeds=seeds)
        assert G.bits_equal(uq.eden_decompress(msg).cpu().numpy(), out.cpu().numpy())
        out, scale = out.cpu().numpy(), scale.cpu().numpy()
        for j in range(n):
            bins, sc, _, _ = E.eden_compress(x[j], nbits, seeds[j])
            assert np.array_equal(msg.bins.cpu().numpy()[j], bins), (d, nbits, j)
            assert same_f32(scale[j], sc), (d, nbits, j)
            assert G.bits_equal(out[j], E.eden_decompress(bins, sc, nbits, seeds[j], d)), (d, nbits, j)


def _adv_rows(rng, kind, n, D):
    if kind == "wide":                                   # roundings in every add
        return (rng.standard_normal((n, D)) * np.exp2(rng.integers(-20, 21, (n, D)))).astype(np.float32)
    if kind == "smallint":                               # few distinct values: exact ties in the chains
        return rng.integers(-3, 4, (n, D)).astype(np.float32)
    x = rng.standard_normal((n, D)).astype(np.float32)   # "tiny": quotients that underflow (lowest bin)
    x[:, ::97] = np.float32(1e-44)
    x[:, 1] = np.float32(3e38)
    return x


@pytest.mark.parametrize("n", [1, 5, 300])
def test_scale_dot_order_adversarial(uq, n):
    """The scale's dot (eden_dot_kernel) against the C oracle's MKL-order dot on vectors whose
    f32 sums are order-sensitive (magnitudes over 2^-20 .. 2^20, heavy cancellation), at every
    power-of-two D from 1 to 2^16 (the remainder rules below 64 included) and batch sizes that
    take one and many workgroups: scale bits equal f32(nrm^2) / uqo_torch_dot(c[bins], rot)."""
    from oracle import uq_oracle_c as C
    rng = np.random.default_rng(n)
    for k in range(0, 17):
        D = 1 << k
        x = (rng.standard_normal((n, D)) * np.exp2(rng.integers(-20, 21, (n, D)))).astype(np.float32)
        seeds = [int(s) for s in rng.integers(0, 100, n)]
        for nbits in (1, 2):
            msg = uq.eden_compress(torch.as_tensor(x).cuda(), nbits, seeds=seeds)
            sc = msg.scale.cpu().numpy()
            for j in range(min(n, 7)):
                rot = E.rht(x[j], seeds[j])
                nrm = E.torch_norm2(rot)
                c = E.centroids(nbits)[msg.bins.cpu().numpy()[j]]
                with np.errstate(all="ignore"):
                    exp = np.float32(np.float32(nrm * nrm) / C.torch_dot(c, rot))
                assert same_f32(sc[j], exp), (D, nbits, j)


@pytest.mark.parametrize("kind", ["wide", "smallint", "tiny"])
def test_scale_dot_segmented_and_one_wave_agree(uq, kind):
    """The dot's two forms (KE4s segments for <= kDotSegMaxN clients, one wave per client
    otherwise) on the same rows: identical bins and scales, both equal to the C oracle's
    MKL-order dot, at D = 2^14 .. 2^22 (ties, binade crossings, underflowing quotients)."""
    from oracle import uq_oracle_c as C
    rng = np.random.default_rng(hash(kind) % 1000)
    for D in (1 << 14, 1 << 17, 1 << 20, 1 << 22):
        x = _adv_rows(rng, kind, 2, D)
        seeds = [int(s) for s in rng.integers(0, 100, 2)]
        for nbits in (1, 2):
            few = uq.eden_compress(torch.as_tensor(x).cuda(), nbits, seeds=seeds)            # segmented
            many = uq.eden_compress(torch.as_tensor(np.concatenate([x] * 40)).cuda(), nbits,   # one wave each
                                    seeds=seeds * 40)
            assert torch.equal(few.bins, many.bins[:2]), (D, nbits)
            a, b = few.scale.cpu().numpy(), many.scale.cpu().numpy()[:2]
            for j in range(2):
                assert same_f32(a[j], b[j]), (kind, D, nbits, j)
                rot = E.rht(x[j], seeds[j])
                nrm = E.torch_norm2(rot)
                c = E.centroids(nbits)[few.bins.cpu().numpy()[j]]
                with np.errstate(all="ignore"):
                    exp = np.float32(np.float32(nrm * nrm) / C.torch_dot(c, rot))
                assert same_f32(a[j], exp), (kind, D, nbits, j)


def test_one_bit_batch_fused_norm_dot_and_its_redo(uq):
    """1 bit, > 256 clients, D a multiple of 2048: the norm, the bins and the dot in one read
    (eden_normdot1_kernel), with the exact KE4 rerun for the clients it flags -- a zero row
    (0 / 0 quotients: NaN -> the last bin), rows whose tiny coordinates' quotients underflow to
    0 (the lowest bin although positive), a row with a NaN -- against the oracle, bit for bit."""
    from oracle import uq_oracle_c as C
    rng = np.random.default_rng(77)
    n, d = 300, 1 << 14
    x = rng.standard_normal((n, d)).astype(np.float32)
    x[3] = 0.0
    x[10, ::50] = np.float32(1e-44)
    x[10, 7] = np.float32(3e38)
    x[11] = (rng.standard_normal(d) * 1e-30).astype(np.float32)
    x[12, 100] = np.nan
    seeds = [int(s) for s in rng.integers(0, 100, n)]
    msg = uq.eden_compress(torch.as_tensor(x).cuda(), 1, seeds=seeds)
    bins, sc = msg.bins.cpu().numpy(), msg.scale.cpu().numpy()
    for j in [0, 1, 3, 10, 11, 12, 150, 299]:
        with np.errstate(all="ignore"):
            eb, es, _, _ = E.eden_compress(x[j], 1, seeds[j])
        assert np.array_equal(bins[j], eb), j
        assert same_f32(sc[j], es), (j, sc[j], es)
    out = uq.eden_quantize(torch.as_tensor(x).cuda(), 1, seeds=seeds).cpu().numpy()
    for j in [0, 10, 299]:
        assert G.bits_equal(out[j], E.eden_decompress(bins[j], sc[j], 1, seeds[j], d)), j


@pytest.mark.parametrize("d", [5000, 1 << 20, (1 << 22) - 5])
def test_sign_bits_equal_int8_rows(uq, d):
    """The diagonal as bits (uq_rht_sign_bits; uq_eden_*_sb, what the Python layer calls) and
    as int8 rows (uq_eden_f32 etc.) give the same bits: the sender's first pass (4096- and
    16384-element low passes, padded rows) and the receiver's last pass, 1 and 2 bits, with a
    NaN and infinities in the input."""
    import ctypes
    from uqdme_amd import eden as Ed
    from uqdme_amd._lib import load, check
    rng = np.random.default_rng(d % 1009)
    n = 3
    x = rng.standard_normal((n, d)).astype(np.float32)
    x[1, 7] = np.inf
    x[2, 3] = np.nan
    xt = torch.as_tensor(x).cuda()
    D = Ed.padded_dim(d)
    seeds = torch.tensor([0, 17, 99])
    tab, rows = Ed._sign_rows(seeds, D, xt.device)
    bits = Ed.rht_sign_bits(tab)
    exp_bits = np.packbits((tab.cpu().numpy() < 0).astype(np.uint8), axis=1, bitorder="little")
    assert np.array_equal(bits.cpu().numpy().view(np.uint8), exp_bits)
    L = load()
    b = ctypes.c_size_t()
    check(L.uq_eden_workspace_bytes(n, d, ctypes.byref(b)), "ws")
    ws = torch.empty(b.value, dtype=torch.uint8, device="cuda")
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    for nbits in (1, 2):
        o8 = torch.empty((n, d), device="cuda")
        ob = torch.empty((n, d), device="cuda")
        s8 = torch.empty(n, device="cuda")
        sb = torch.empty(n, device="cuda")
        check(L.uq_eden_f32(p(xt), p(o8), n, d, nbits, p(tab), p(rows), p(s8), p(ws), b.value, None), "int8")
        check(L.uq_eden_f32_sb(p(xt), p(ob), n, d, nbits, p(tab), p(rows), p(bits), p(sb), p(ws), b.value, None),
              "bits")
        torch.cuda.synchronize()
        assert G.bits_equal(o8.cpu().numpy(), ob.cpu().numpy()), nbits
        assert torch.equal(s8.view(torch.int32), sb.view(torch.int32)), nbits
    # and the Python drop-in path (bits) against the oracle on one row
    if d <= 1 << 20:
        out = uq.eden_quantize(xt[:1], 1, seeds=[17]).cpu().numpy()[0]
        assert G.bits_equal(out, E.eden_quantize(x[0], 1, 17))
