"""Test infrastructure: a model of the ROUND-1 K2 prefix scheme (parallel fp64 tree scan),
used to show that the exact-scan tests have teeth: on the inputs they use, that scheme's
f32 prefixes differ from torch's sequential fp64 cumsum (AS:635), and X is chosen so the
difference reaches the outputs.  Not a reference restatement (that is oracle/)."""
import numpy as np

from oracle import uq_oracle as O
from oracle import uq_oracle_c as C

f32, f64 = np.float32, np.float64
TILE, ITEMS, BLOCK, WAVE = 4096, 16, 256, 64


def tree_prefix(fr):
    """Per-element fp64 prefixes of round-1 K2: thread sums from 0, wave Hillis-Steele scan,
    waves added in order, thread base = P_t + exclusive, P_{t+1} = P_t + A_t."""
    d = fr.shape[0]
    tiles = (d + TILE - 1) // TILE
    frp = np.zeros(tiles * TILE, f64)
    frp[:d] = fr.astype(f64)
    out = np.empty(tiles * TILE, f64)
    P = f64(0)
    lanes = np.arange(WAVE)[None, :]
    for t in range(tiles):
        v = frp[t * TILE:(t + 1) * TILE].reshape(BLOCK, ITEMS)
        ts = np.zeros(BLOCK, f64)
        for k in range(ITEMS):
            ts = ts + v[:, k]
        w = ts.reshape(BLOCK // WAVE, WAVE)
        o = 1
        while o < WAVE:
            sh = np.concatenate([np.zeros((w.shape[0], o)), w[:, :-o]], axis=1)
            w = np.where(lanes >= o, sh + w, w)
            o <<= 1
        wexcl = np.concatenate([np.zeros((w.shape[0], 1)), w[:, :-1]], axis=1)
        wbase = np.zeros(BLOCK // WAVE, f64)
        acc = f64(0)
        for i in range(BLOCK // WAVE):
            wbase[i] = acc
            acc = acc + w[i, -1]
        s = P + (wbase[:, None] + wexcl).reshape(BLOCK)
        for k in range(ITEMS):
            s = s + v[:, k]
            out[t * TILE + k + np.arange(BLOCK) * ITEMS] = s
        P = P + acc
    return out[:d]


# ---- the exact scheme (restated from the K2 design), per tile with the
# exact start P: regular tiles by the two parity chains and ordered tie resolution,
# irregular tiles thread by thread (clean threads by their chains, edge threads one add at
# a time).  It checks the arithmetic argument, not the kernel.
def binade(s):
    return int(np.frexp(s)[1]) - 1          # s in [2^E, 2^(E+1))


def par(s):
    return int(np.array(s, f64).view(np.uint64)) & 1


def chains(vrow, E):
    G = np.ldexp(1.0, E - 52)
    B0 = np.ldexp(1.0, E)
    B1 = B0 + G
    c0, c1 = B0, B1
    for f in vrow:
        c0 = c0 + f
        c1 = c1 + f
    return c0 - B0, c1 - B1


def exact_tile(P, v):
    """v: [256, 16] fp64 fractions; returns (thread bases, P_next)."""
    base = np.empty(BLOCK, f64)
    if P >= 32.0:
        E = binade(P)
        B0 = np.ldexp(1.0, E)
        G = np.ldexp(1.0, E - 52)
        c0 = np.full(BLOCK, B0)
        c1 = np.full(BLOCK, B0 + G)
        for k in range(ITEMS):
            c0 = c0 + v[:, k]
            c1 = c1 + v[:, k]
        T0 = c0 - B0
        T1 = c1 - (B0 + G)
        excl0 = np.concatenate([[0.0], np.cumsum(T0)[:-1]])     # any order: exact
        total0 = T0.sum()
        if P + total0 + 1.0 < np.ldexp(1.0, E + 1):
            delta = 0.0
            corr = np.zeros(BLOCK)
            for k in np.nonzero(T0 != T1)[0]:
                Sk = (P + excl0[k]) + delta
                dk = (T1[k] if par(Sk) else T0[k]) - T0[k]
                delta = delta + dk
                corr[k + 1:] = delta
            base = (P + excl0) + corr
            return base, (P + total0) + delta
    # irregular tile: serial walk over threads
    ts = v.sum(axis=1)
    sa = P + np.concatenate([[0.0], np.cumsum(ts)[:-1]])
    S = P
    for i in range(BLOCK):
        base[i] = S
        s_a = sa[i]
        clean = False
        if s_a >= 32.0:
            Et = binade(s_a)
            clean = s_a >= np.ldexp(1.0, Et) * (1 + 2.0 ** -20) and s_a + ts[i] + 1.0 < np.ldexp(1.0, Et + 1)
        if clean:
            T0, T1 = chains(v[i], Et)
            assert binade(S) == Et
            S = S + (T1 if par(S) else T0)
        else:
            for f in v[i]:
                S = S + f
    return base, S


def exact_prefix(fr):
    d = fr.shape[0]
    tiles = (d + TILE - 1) // TILE
    frp = np.zeros(tiles * TILE, f64)
    frp[:d] = fr.astype(f64)
    out = np.empty(tiles * TILE, f64)
    P = 0.0
    nirr = 0
    for t in range(tiles):
        v = frp[t * TILE:(t + 1) * TILE].reshape(BLOCK, ITEMS)
        base, Pn = exact_tile(P, v)
        s = base.copy()
        for k in range(ITEMS):
            s = s + v[:, k]
            out[t * TILE + k + np.arange(BLOCK) * ITEMS] = s
        P = Pn
    return out[:d]



def tiny_mix(seed, d, mix=0.5, scale=1e-4):
    """N(0,1) with a fraction `mix` of the coordinates replaced by N(0, scale^2): many
    fractional parts with bits below the fp64 spacing of the running sum."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(d).astype(f32)
    sel = rng.random(d) < mix
    x[sel] = (rng.standard_normal(int(sel.sum())) * scale).astype(f32)
    return x


def exposing_X(x, m, torch_threads=1):
    """(X, i) such that with this X the round-1 tree scheme's output differs from the
    reference at element i, or (None, None) when its prefixes all agree."""
    l1 = C.l1_torch_order(x, torch_threads)
    _, _, fr = O.fractional_parts(x, m, l1)
    seq = np.cumsum(fr.astype(f64)).astype(f32)
    tre = tree_prefix(fr).astype(f32)
    bad = np.nonzero(seq != tre)[0]
    if bad.size == 0:
        return None, None
    i = int(bad[0])
    hi = max(seq[i], tre[i])
    X = f32(hi - np.floor(hi))                 # c_hi - X is an integer, c_lo - X is not
    return X, i
