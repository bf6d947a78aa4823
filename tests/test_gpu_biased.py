"""GPU parity of the biased type quantizer (AS:669-687) through the C-ABI, against the
reference's fixtures and the C++ oracle (bit-exact; NaN positions compared as NaN)."""
import numpy as np
import pytest
import torch

from oracle import uq_oracle_c as C
from oracle.uq_oracle import rate_to_m
from tests import golden_data as G

pytestmark = pytest.mark.gpu
f32 = np.float32


@pytest.fixture(scope="module")
def uq(gpu_ready):
    import uqdme
    C.build()
    return uqdme


@pytest.fixture(scope="module")
def cases():
    return list(G.biased_vectors())


def run(uq, x, R, T, ties):
    xd = torch.as_tensor(np.ascontiguousarray(x, f32)).cuda().view(1, -1)
    m = rate_to_m(R, x.shape[0])
    out, info = uq.biased_quantize(xd, m=m, torch_threads=T, ties=ties, return_info=True)
    return out.view(-1).cpu().numpy(), info.cpu().numpy()[0]


def test_fixtures_lowest_rule(uq, cases):
    """ties='lowest': bit-exact with the reference wherever no tie straddles the threshold,
    and bit-exact with the oracle's lowest-index rule everywhere."""
    bad = []
    for sp, x, q, h in cases:
        if sp.get("raises"):
            continue
        out, info = run(uq, x, sp["R"], sp["threads"], "lowest")
        assert info[0] == sp["delta"], sp["idx"]
        assert bool(info[1] & 1) == sp["ambiguous"], sp["idx"]
        if not sp["ambiguous"]:
            ok = G.bits_equal(out, q) if q is not None else G.sha(out) == h
        else:
            with np.errstate(all="ignore"):
                exp, *_ = C.biased_quantize(x, rate_to_m(sp["R"], x.shape[0]), sp["threads"], 1)
            ok = G.bits_equal(out, exp)
        if not ok:
            bad.append(sp["idx"])
    assert not bad, f"GPU differs on fixtures {bad}"


def test_raising_cases(uq, cases):
    for sp, x, q, h in cases:
        if not sp.get("raises"):
            continue
        out, info = run(uq, x, sp["R"], sp["threads"], "lowest")
        assert info[1] & 4, sp["idx"]           # |Delta| > d: torch.topk raises
        with pytest.raises(RuntimeError):
            uq.Type_biased_quantize(torch.as_tensor(x), sp["R"])


def test_batch_rows_independent(uq):
    rng = np.random.default_rng(11)
    n, d = 37, 3001
    x = rng.standard_normal((n, d)).astype(f32)
    x[5] = np.round(x[5] * 2) / 2          # some tie-heavy rows
    x[17] = rng.integers(-2, 3, d)
    m = rate_to_m(1, d)
    out = uq.biased_quantize(torch.as_tensor(x).cuda(), m=m, torch_threads=1, ties="lowest").cpu().numpy()
    for j in range(n):
        exp, *_ = C.biased_quantize(x[j], m, 1, 1)
        assert G.bits_equal(out[j], exp), j


def test_large_batch_vs_oracle(uq):
    """n = 64 clients at d = 2^18: the multi-workgroup histogram / tile paths."""
    rng = np.random.default_rng(12)
    n, d = 64, 1 << 18
    x = rng.standard_normal((n, d)).astype(f32)
    x[::4] = np.round(x[::4] * 3) / 3
    for R in (1, 4):
        m = rate_to_m(R, d)
        out = uq.biased_quantize(torch.as_tensor(x).cuda(), m=m, torch_threads=8, ties="lowest").cpu().numpy()
        for j in range(0, n, 7):
            exp, *_ = C.biased_quantize(x[j], m, 8, 1)
            assert G.bits_equal(out[j], exp), (R, j)


def test_unaligned_and_ragged(uq):
    rng = np.random.default_rng(13)
    for d in (1, 3, 7, 31, 4097, 16385, 70001):
        base = torch.as_tensor(rng.standard_normal(d + 1).astype(f32)).cuda()
        xv = base[1:].view(1, d)           # 4-byte offset: scalar paths
        m = rate_to_m(2, d)
        out = uq.biased_quantize(xv, m=m, torch_threads=1, ties="lowest").cpu().numpy()[0]
        exp, *_ = C.biased_quantize(xv.cpu().numpy()[0], m, 1, 1)
        assert G.bits_equal(out, exp), d


def test_drop_in_semantics(uq):
    x = torch.randn(1000)
    with pytest.raises(KeyError):
        uq.Type_biased_quantize(x, 3.3)
    state = torch.get_rng_state()
    y = uq.Type_biased_quantize(x, 1)
    assert torch.equal(state, torch.get_rng_state())     # the biased quantizer draws nothing
    assert y.is_cuda and y.dtype == torch.float32 and y.shape == (1000,)
    assert uq.Type_biased_quantize.__name__ == "Type_biased_quantize"
    assert uq.Type_biased_quantize(torch.empty(0), 1).numel() == 0


def test_fixtures_torch_ties_bit_exact(uq, cases):
    """ties='torch' (the default, KB7 replaying libstdc++'s nth_element / partial_sort):
    bit-exact with the reference on every fixture, ambiguous ties included."""
    bad, replayed = [], 0
    for sp, x, q, h in cases:
        if sp.get("raises"):
            continue
        out, info = run(uq, x, sp["R"], sp["threads"], "torch")
        replayed += bool(info[1] & 8)
        assert bool(info[1] & 8) == sp["ambiguous"], sp["idx"]
        ok = G.bits_equal(out, q) if q is not None else G.sha(out) == h
        if not ok:
            bad.append(sp["idx"])
    uq.check_status()
    assert not bad, f"GPU differs from the reference on fixtures {bad}"
    assert replayed >= 50


def _heap_cases():
    """Tie-heavy vectors whose topk takes partial_sort (k * 64 <= d) with a tie at the threshold."""
    out = []
    for d, scale, R in ((5000, 8, 8), (5000, 16, 2), (20000, 2, 8), (20000, 16, 4), (100000, 8, 2),
                        (100000, 16, 8)):
        x = (np.round(np.random.default_rng(d * 100 + scale + R).standard_normal(d) * scale) / scale).astype(f32)
        out.append((x, R))
    return out


def test_torch_ties_heap_and_select_paths(uq):
    hits = {"heap": 0, "nth": 0}
    for x, R in _heap_cases():
        d = x.shape[0]
        m = rate_to_m(R, d)
        exp, _, D, A = C.biased_quantize(x, m, 1, 0)
        out, info = run(uq, x, R, 1, "torch")
        assert info[0] == D
        assert G.bits_equal(out, exp), (d, R)
        if A:
            hits["heap" if abs(D) * 64 <= d else "nth"] += 1
    uq.check_status()
    assert hits["heap"] >= 2, hits


def test_torch_ties_many_clients(uq):
    """More ambiguous clients than KB7 slots (64): workgroups loop over clients."""
    rng = np.random.default_rng(21)
    n, d = 150, 6007
    x = rng.integers(-3, 4, (n, d)).astype(f32)
    x[1::3] = rng.standard_normal((len(range(1, n, 3)), d)).astype(f32)     # some unambiguous rows
    for R in (1, 4):
        m = rate_to_m(R, d)
        out, info = uq.biased_quantize(torch.as_tensor(x).cuda(), m=m, torch_threads=1, ties="torch",
                                       return_info=True)
        out = out.cpu().numpy()
        info = info.cpu().numpy()
        for j in range(n):
            exp, _, D, A = C.biased_quantize(x[j], m, 1, 0)
            assert info[j, 0] == D and bool(info[j, 1] & 1) == A, j
            assert G.bits_equal(out[j], exp), (R, j)
    uq.check_status()


def test_drop_in_matches_reference_fixtures(uq, cases):
    """The drop-in itself (1-D, torch ties) on the small fixtures, incl. the raising ones."""
    for sp, x, q, h in cases:
        if x.shape[0] > 8192 or sp["threads"] != 1:
            continue
        uq.set_torch_threads(1)
        try:
            if sp.get("raises"):
                with pytest.raises(RuntimeError):
                    uq.Type_biased_quantize(torch.as_tensor(x), sp["R"])
                continue
            y = uq.Type_biased_quantize(torch.as_tensor(x), sp["R"]).cpu().numpy()
        finally:
            uq.set_torch_threads(None)
        assert G.bits_equal(y, q), sp["idx"]


def test_c4_size_2pow22_vs_oracle(uq):
    """Config C4's d = 2^22, torch ties: Gaussian (compaction path) and tie-heavy integers
    (full radix passes + KB7 replay) bit-exact against the oracle's libstdc++ replay."""
    rng = np.random.default_rng(42)
    d = 1 << 22
    for x in (rng.standard_normal(d).astype(f32), rng.integers(-3, 4, d).astype(f32)):
        for R in (1, 2):
            m = rate_to_m(R, d)
            exp, _, D, A = C.biased_quantize(x, m, 1, 0)
            out, info = run(uq, x, R, 1, "torch")
            assert info[0] == D and bool(info[1] & 1) == A
            assert G.bits_equal(out, exp), (R, G.n_mismatch(out, exp))
    uq.check_status()


def test_torch_ties_batch_multiworkgroup_levels(uq):
    """A batch (n >= 32) at d = 2^20 takes KB7a: introselect's levels run over many workgroups
    down to the 4096-pair LDS tails (~10 levels here), marking and tails in 256-thread
    workgroups, then the join.  Tie-heavy integer rows (always ambiguous) and Gaussian rows,
    every client bit-exact against the oracle's libstdc++ replay."""
    rng = np.random.default_rng(77)
    n, d = 40, 1 << 20
    x = rng.standard_normal((n, d)).astype(f32)
    x[::4] = rng.integers(-3, 4, (len(range(0, n, 4)), d)).astype(f32)
    m = rate_to_m(1, d)
    out, info = uq.biased_quantize(torch.as_tensor(x).cuda(), m=m, torch_threads=1, ties="torch", return_info=True)
    out = out.cpu().numpy()
    info = info.cpu().numpy()
    amb = 0
    for j in range(n):
        exp, _, D, A = C.biased_quantize(x[j], m, 1, 0)
        assert info[j, 0] == D and bool(info[j, 1] & 1) == A, j
        assert G.bits_equal(out[j], exp), j
        amb += int(A)
    assert amb >= n // 4, amb
    uq.check_status()


def test_torch_ties_gaussian_ambiguous_fine_clients(uq):
    """Gaussian rows whose threshold key repeats (~2 % of rows at d = 2^18, picked with the
    oracle): their threshold bin is small, so KB6f writes the rows, KB7a replays the ties and
    KB6t patches the selected bin coordinates (no full-row rewrite).  A 40-client batch (KB7a),
    every client bit-exact against the oracle."""
    rng = np.random.default_rng(91)
    d = 1 << 18
    m = rate_to_m(1, d)
    amb_rows = []
    for _ in range(600):
        x = rng.standard_normal(d).astype(f32)
        if C.biased_quantize(x, m, 1, 0)[3]:
            amb_rows.append(x)
            if len(amb_rows) == 6:
                break
    assert len(amb_rows) >= 3
    n = 40
    x = rng.standard_normal((n, d)).astype(f32)
    slots = [1, 7, 8, 20, 33, 39][:len(amb_rows)]
    for j, r in zip(slots, amb_rows):
        x[j] = r
    out, info = uq.biased_quantize(torch.as_tensor(x).cuda(), m=m, torch_threads=1, ties="torch", return_info=True)
    out = out.cpu().numpy()
    info = info.cpu().numpy()
    for j in range(n):
        exp, _, D, A = C.biased_quantize(x[j], m, 1, 0)
        assert info[j, 0] == D and bool(info[j, 1] & 1) == A, j
        assert G.bits_equal(out[j], exp), j
        if j in slots:
            assert A, j
    uq.check_status()


def test_torch_ties_many_listed_clients_stop_levels_early(uq):
    """>= 128 listed clients: KB7a's levels stop at ranges of 65536 and the 1024-thread
    replays resume those slots after the join (plus the list entries beyond the 256 slots).
    Every client tie-heavy (ambiguous), bit-exact against the oracle."""
    rng = np.random.default_rng(78)
    n, d = 300, 1 << 17
    x = rng.integers(-3, 4, (n, d)).astype(f32)
    m = rate_to_m(1, d)
    out, info = uq.biased_quantize(torch.as_tensor(x).cuda(), m=m, torch_threads=1, ties="torch", return_info=True)
    out = out.cpu().numpy()
    info = info.cpu().numpy()
    amb = 0
    for j in range(n):
        exp, _, D, A = C.biased_quantize(x[j], m, 1, 0)
        assert info[j, 0] == D and bool(info[j, 1] & 1) == A, j
        assert G.bits_equal(out[j], exp), j
        amb += int(A)
    assert amb >= 128, amb
    uq.check_status()


def test_tiny_vectors_several_selections(uq):
    """d < 8 (a single scalar torch chunk, K1b's lane-0 path) with |Delta| >= 2: the first
    radix digit's histogram must count each coordinate once.  Both tie rules, against the
    oracle."""
    rng = np.random.default_rng(5)
    rows = []
    while len(rows) < 24:
        d = int(rng.integers(2, 8))
        R = int(rng.choice([1, 2, 3, 4, 5, 6, 8]))
        x = (rng.standard_normal(d) * rng.choice([1, 10, 0.1])).astype(f32)
        _, _, D, _ = C.biased_quantize(x, rate_to_m(R, d), 1, 1)
        if abs(D) >= 2:
            rows.append((x, R))
    for x, R in rows:
        m = rate_to_m(R, x.shape[0])
        for ties, rule in (("lowest", 1), ("torch", 0)):
            exp, _, D, A = C.biased_quantize(x, m, 1, rule)
            out, info = run(uq, x, R, 1, ties)
            assert info[0] == D and bool(info[1] & 1) == A, (x, R, ties)
            assert G.bits_equal(out, exp), (x, R, ties)
    uq.check_status()


def test_fuzz_small_vectors_vs_oracle(uq):
    """Seeded fuzz over d = 1..600: Gaussian, wide-range, tie-heavy integer and zero-heavy
    rows at random rates, both tie rules, bit-exact against the oracle."""
    rng = np.random.default_rng(2024)
    rates = [0.5, 1, 1.5, 2, 3, 4, 6, 8]
    for t in range(160):
        d = int(rng.integers(1, 601))
        kind = t % 4
        if kind == 0:
            x = rng.standard_normal(d)
        elif kind == 1:
            x = rng.standard_normal(d) * np.exp(rng.uniform(-20, 20, d))
        elif kind == 2:
            x = rng.integers(-3, 4, d)
        else:
            x = rng.standard_normal(d) * (rng.random(d) < 0.2)
        x = x.astype(f32)
        R = float(rng.choice(rates))
        m = rate_to_m(R, d)
        for ties, rule in (("lowest", 1), ("torch", 0)):
            with np.errstate(all="ignore"):
                exp, _, D, A = C.biased_quantize(x, m, 1, rule)
            out, info = run(uq, x, R, 1, ties)
            assert info[0] == D and bool(info[1] & 1) == A, (t, d, R, ties)
            assert G.bits_equal(out, exp), (t, d, R, ties)
    uq.check_status()


@pytest.mark.parametrize("n,d", [(3, 1 << 16), (40, 1 << 20)])
def test_failed_replay_falls_back_to_index_order(uq, n, d):
    """a torch-tie replay that fails its consistency checks (forced here through
    the library's test hook uq_test_force_replay_failure) reports the internal error through
    check_status and leaves a DEFINED output: the client's threshold ties ranked in index
    order, i.e. exactly the UQ_TIES_LOWEST_INDEX result (the replay kernel counts the tile
    ties that rez_tiecount_kernel skipped for listed clients).  Both replay forms: one kernel
    (few clients) and KB7a's levels (n >= 32)."""
    from uqdme_amd._lib import load
    rng = np.random.default_rng(n)
    x = torch.as_tensor(rng.integers(-3, 4, (n, d)).astype(f32)).cuda()
    m = rate_to_m(1, d)
    assert load().uq_test_force_replay_failure(1) == 0
    try:
        out_t, info = uq.biased_quantize(x, m=m, torch_threads=1, ties="torch", return_info=True)
        torch.cuda.synchronize()
        with pytest.raises(uq.UQError):
            uq.check_status()
    finally:
        assert load().uq_test_force_replay_failure(0) == 1
    assert int((info[:, 1] & 1).sum()) >= n // 2 and int((info[:, 1] & 8).sum()) == 0   # ambiguous, none replayed
    out_l = uq.biased_quantize(x, m=m, torch_threads=1, ties="lowest")
    assert torch.equal(out_t.view(torch.int32), out_l.view(torch.int32))
    uq.check_status()


@pytest.mark.parametrize("d", [(1 << 17) + 5, 1 << 20])
def test_candidate_digits_few_and_many_clients_agree(uq, d):
    """Batches of <= 16 clients run the candidate digits (KB4d) over many workgroups per
    client, larger ones one workgroup per client: the same rows give the same bits either
    way (torch ties and lowest index), and both match the oracle."""
    rng = np.random.default_rng(d % 977)
    x = rng.standard_normal((17, d)).astype(f32)
    x[3] = np.round(x[3] * 4) / 4                      # tie-heavy rows
    x[9] = rng.integers(-3, 4, d)
    xt = torch.as_tensor(x).cuda()
    m = rate_to_m(1, d)
    for ties, code in (("torch", 0), ("lowest", 1)):
        few = uq.biased_quantize(xt[:16], m=m, torch_threads=1, ties=ties).cpu().numpy()
        many = uq.biased_quantize(xt, m=m, torch_threads=1, ties=ties).cpu().numpy()
        assert G.bits_equal(few, many[:16]), ties
        one = uq.biased_quantize(xt[9:10], m=m, torch_threads=1, ties=ties).cpu().numpy()
        assert G.bits_equal(one[0], many[9]), ties
        for j in (0, 3, 9):
            exp, *_ = C.biased_quantize(x[j], m, 1, code)
            assert G.bits_equal(many[j], exp), (ties, j)


def test_few_clients_2pow22_take_level_replay(uq):
    """A few clients at d >= 2^21 replay torch's tie choice through KB7a's levels (one
    workgroup walking 2^22 keys took milliseconds): Gaussian and tie-heavy rows, bit-exact
    against the oracle, at least one row replayed."""
    rng = np.random.default_rng(622)
    d, n = 1 << 22, 4
    x = rng.standard_normal((n, d)).astype(f32)
    x[1] = np.round(x[1] * 4) / 4
    x[3] = np.round(x[3] * 8) / 8
    m = rate_to_m(1, d)
    out, info = uq.biased_quantize(torch.as_tensor(x).cuda(), m=m, torch_threads=1, ties="torch", return_info=True)
    out, info = out.cpu().numpy(), info.cpu().numpy()
    assert (info[:, 1] & 8).any(), info
    for j in range(n):
        exp, *_ = C.biased_quantize(x[j], m, 1, 0)
        assert G.bits_equal(out[j], exp), (j, G.n_mismatch(out[j], exp))
    uq.check_status()


@pytest.mark.parametrize("d", [(1 << 21) + 3, 1 << 22])
def test_host_check_skips_replay_with_same_bits(uq, d):
    """UQ_TIES_HOST_CHECK (the per-vector drop-in's policy): when no row needs the torch-tie
    replay its kernels are skipped; when some do, they run.  Same bits as the plain call either
    way, for tie-free and tie-heavy rows, one row and a few."""
    rng = np.random.default_rng(d % 1013)
    smooth = rng.standard_normal((3, d)).astype(f32)
    ties = rng.integers(-3, 4, (3, d)).astype(f32)
    m = rate_to_m(1, d)
    for x in (smooth, ties, np.stack([smooth[0], ties[1]])):
        xt = torch.as_tensor(x).cuda()
        for rows in (xt[:1], xt):
            a, ia = uq.biased_quantize(rows, m=m, torch_threads=1, ties="torch", return_info=True)
            b, ib = uq.biased_quantize(rows, m=m, torch_threads=1, ties="torch", return_info=True, host_check=True)
            assert torch.equal(a.view(torch.int32), b.view(torch.int32)) and torch.equal(ia, ib)
    out = uq.Type_biased_quantize(torch.as_tensor(ties[2]).cuda(), 1)
    ref = uq.biased_quantize(torch.as_tensor(ties[2:3]).cuda(), m=rate_to_m(1, d), ties="torch")
    assert torch.equal(out.view(torch.int32), ref.view(d).view(torch.int32))
    uq.check_status()


@pytest.mark.parametrize("d", [1, 5, 8, 100, 1023, 1024, 2048, 4097, 32767])
def test_small_vector_single_launch(uq, d):
    """KB-small (d < GRAIN, one launch): the lowest-index rule for any batch, and torch ties
    under the host check (the drop-in's policy; an ambiguous row reruns the multi-kernel
    path), bit-exact with the oracle on smooth, tie-heavy and zero-heavy rows, info pairs
    included; R = 1 and 4."""
    rng = np.random.default_rng(d)
    rows = [rng.standard_normal(d), rng.integers(-3, 4, d), np.where(rng.random(d) < 0.7, 0, rng.standard_normal(d)),
            rng.laplace(1, 2, d)]
    x = np.stack(rows).astype(f32)
    xt = torch.as_tensor(x).cuda()
    for R in (1, 4):
        m = rate_to_m(R, d)
        lo, ilo = uq.biased_quantize(xt, m=m, torch_threads=1, ties="lowest", return_info=True)
        to, ito = uq.biased_quantize(xt, m=m, torch_threads=1, ties="torch", return_info=True, host_check=True)
        for j in range(x.shape[0]):
            for rule, got, info in ((1, lo, ilo), (0, to, ito)):
                try:
                    with np.errstate(all="ignore"):
                        exp, _, D, A = C.biased_quantize(x[j], m, 1, rule)
                except (RuntimeError, ValueError):         # the reference raises (AS:656 / AS:660)
                    assert int(info[j, 1]) & 6, (d, R, j, rule)
                    continue
                assert int(info[j, 0]) == D and bool(int(info[j, 1]) & 1) == A, (d, R, j, rule)
                assert G.bits_equal(got[j].cpu().numpy(), exp), (d, R, j, rule)
    uq.check_status()
