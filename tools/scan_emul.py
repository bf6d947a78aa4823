"""CPU emulation of K2's fp64 prefix schemes, to find inputs on which the parallel tree
scan (round-1 K2: thread sums from 0, wave Hillis-Steele scan, waves added in order,
P_{t+1} = P_t + A_t) gives f32 prefixes different from torch's sequential fp64 cumsum
(AS:635), and to check the exact emulation against the sequential definition.

usage: python tools/scan_emul.py [d] [vectors] [mix]"""
import sys
import numpy as np

f32, f64 = np.float32, np.float64
TILE, ITEMS, BLOCK, WAVE = 4096, 16, 256, 64


def tree_prefix(fr):
    """Thread-start prefixes s_i (fp64) of the round-1 K2 tree scan, per element prefix c."""
    d = fr.shape[0]
    tiles = (d + TILE - 1) // TILE
    frp = np.zeros(tiles * TILE, f64)
    frp[:d] = fr.astype(f64)
    out = np.empty(tiles * TILE, f64)
    P = f64(0)
    for t in range(tiles):
        v = frp[t * TILE:(t + 1) * TILE].reshape(BLOCK, ITEMS)
        ts = np.zeros(BLOCK, f64)
        for k in range(ITEMS):
            ts = ts + v[:, k]
        w = ts.reshape(BLOCK // WAVE, WAVE).copy()
        o = 1
        while o < WAVE:
            sh = np.concatenate([np.zeros((w.shape[0], o)), w[:, :-o]], axis=1)
            w = np.where(np.arange(WAVE)[None, :] >= o, sh + w, w)
            o <<= 1
        incl = w
        wexcl = np.concatenate([np.zeros((incl.shape[0], 1)), incl[:, :-1]], axis=1)
        wsum = incl[:, -1]
        wbase = np.zeros(BLOCK // WAVE, f64)
        acc = f64(0)
        for i in range(BLOCK // WAVE):
            wbase[i] = acc
            acc = acc + wsum[i]
        total = acc
        texcl = (wbase[:, None] + wexcl).reshape(BLOCK)
        s = P + texcl
        for k in range(ITEMS):
            s = s + v[:, k]
            out[t * TILE + k + np.arange(BLOCK) * ITEMS] = s
        P = P + total
    return out[:d]


def frac_parts(x, m):
    L = np.float32(np.abs(x).astype(f32).sum(dtype=f32))   # any L1: the scan is what is compared
    den = f32(L + f32(1e-12))
    v = (x / den).astype(f32)
    mp = (f32(m) * np.abs(v)).astype(f32)
    return (mp - np.floor(mp)).astype(f32)


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    nv = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    mix = float(sys.argv[3]) if len(sys.argv) > 3 else 0.3
    rng = np.random.default_rng(7)
    m = int(0.21403 * d)
    tot_mis = 0
    for j in range(nv):
        x = rng.standard_normal(d).astype(f32)
        sel = rng.random(d) < mix
        x[sel] = (rng.standard_normal(sel.sum()) * 1e-4).astype(f32)
        fr = frac_parts(x, m)
        seq = np.cumsum(fr.astype(f64))
        tre = tree_prefix(fr)
        mis = int(np.sum(seq.astype(f32) != tre.astype(f32)))
        dev = np.max(np.abs(seq - tre))
        tot_mis += mis
        print(f"vector {j}: f32 prefix mismatches {mis}, max |fp64 diff| {dev:.3e}, final {seq[-1]:.6f}", flush=True)
    print("total", tot_mis)


if __name__ == "__main__":
    main()


# ---------------------------------------------------------------------------------------
# Exact emulation (the K2 design): per tile, with the exact prefix P known.
#   regular tile (P >= 32, binade E of P, P + tile total + 1 < 2^(E+1)): each thread runs
#     its 16 adds from B0 = 2^E and from B1 = 2^E + G (G = ulp in binade E); T_p = chain_p
#     - B_p is the thread's exact increment when its true start has parity p (the fp64 add
#     S + f depends on S only through S mod 2G while S stays in binade E).  Block scan of
#     T0 (exact: multiples of G below 2^E); threads with T0 != T1 ("ties") are resolved in
#     order from their exact start parity.
#   irregular tile: per-thread binade from the approximate start; clean threads use their
#     own (T0, T1), the rest add their 16 values one by one; a serial walk over threads.
# ---------------------------------------------------------------------------------------
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
            clean = s_a >= np.ldexp(1.0, Et) * (1 + 2.0 ** -30) and s_a + ts[i] + 1.0 < np.ldexp(1.0, Et + 1)
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


def check_exact(d=1 << 20, nv=8, mix=0.5, seed=11):
    rng = np.random.default_rng(seed)
    m = int(0.21403 * d)
    bad = 0
    for j in range(nv):
        x = rng.standard_normal(d).astype(f32)
        sel = rng.random(d) < mix
        x[sel] = (rng.standard_normal(sel.sum()) * 1e-4).astype(f32)
        fr = frac_parts(x, m)
        seq = np.cumsum(fr.astype(f64))
        ex = exact_prefix(fr)
        nb = int(np.sum(seq.view(np.uint64) != ex.view(np.uint64)))
        bad += nb
        print(f"exact vector {j}: fp64 prefix mismatches {nb}", flush=True)
    return bad
