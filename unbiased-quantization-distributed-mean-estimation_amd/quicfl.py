"""QUIC-FL on the GPU — SURVEY §8(f) row 2 (baseline): sender, receiver and the drop-in.

    QuicFLSender(device=..., bits=[1, 2, 3, 4], sr_bits=[6, 5, 4, 4], prefix=.../tables/)
        mirrors NMSE_Results/Codes/All_Schemes.py:429-503: per bit width the sender tables
        `<b>_X_<s>_h_256_q_sender_table_X.pt` / `..._p.pt` (torch.load(weights_only=True)) and
        `data.txt` (ast.literal_eval, not eval); compress(data) returns the reference's message
        dict and draws its bernoulli(p_X) words from torch's global CPU generator, which it
        leaves where the reference would.
    QuicFLReceiver(...)    AS:507-535, decompress(data) -> vec[:dim] on the GPU.
    QUICFL_quantize(input_vector, bits_per_dimension=1)
        AS:814-832: one torch.randint(0, 100) draw of the global CPU generator, compress,
        decompress, NumPy f32 result.  Tables come from `set_tables_prefix()` /
        $UQDME_QUICFL_TABLES (the reference reads its own tables/ directory).
    quicfl_compress(x[n, d], nbits, seeds, rotation_seeds, sender=...)  -> QuicFLMessages
    quicfl_decompress(X[n, D], nbits, prng_seeds, rotation_seeds, scale[n], dim, recv_table)

Bit-identical to the reference's QuicFLSender.compress (X, exact_indeces, exact_values, scale,
the global generator's state after the call) on synthetic sender tables
(tests/golden/quicfl_sender_vectors.*), and to its QuicFLReceiver.decompress on its own
receiver tables (tests/golden/quicfl_recv_vectors.*).  The published sender tables are not in
the reference, so outputs on them remain unpinned.
"""
from __future__ import annotations

import ast
import ctypes
import os
import struct
import threading
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .eden import _sign_rows, padded_dim, randomized_inverse_hadamard_transform
from .quantizer import _as_device_f32_2d, _device, _ptr, _stream_ptr, _workspace

__all__ = ["QuicFLReceiver", "QuicFLSender", "QuicFLMessages", "QUICFL_quantize", "quicfl_compress",
           "quicfl_decompress", "quicfl_decompress_messages", "quicfl_quantize", "prng_seed", "set_tables_prefix"]

STATE_WORDS = 626                  # UQ_QFL_STATE_WORDS: (left, next, 624 words)
_FLAG_P, _FLAG_INDEX, _FLAG_PX, _FLAG_X, _FLAG_TIMEOUT, _FLAG_EXACT, _FLAG_RECV_INDEX = 1, 2, 4, 8, 16, 32, 64  # UQ_QFL_*
_tables_prefix = None
_USE_PACKED = os.environ.get("UQDME_QUICFL_PACKED", "1") == "1"     # the 4-byte table when it is valid
_dropin_lock = threading.Lock()
_dropin: dict = {}


def set_tables_prefix(prefix) -> None:
    """Directory (with trailing separator or not) holding the QUIC-FL tables the drop-in
    QUICFL_quantize loads, as the reference's `str(path) + '/tables/'` (AS:431, AS:509)."""
    global _tables_prefix
    _tables_prefix = None if prefix is None else os.path.join(str(prefix), "")


def default_tables_prefix() -> str:
    if _tables_prefix is not None:
        return _tables_prefix
    env = os.environ.get("UQDME_QUICFL_TABLES")
    if env:
        return os.path.join(env, "")
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "tables", "")


def prng_seed(seed) -> int:
    """AS:457: xxh64(str(seed)).intdigest() % 2^16 (xxHash64 in the C library)."""
    b = str(seed).encode()
    return int(_lib.load().uq_xxh64(b, len(b), 0)) % (1 << 16)


# ---- torch CPU generator state <-> (left, next, 624 words) --------------------------------------
def generator_words(gen: torch.Generator):
    """(get_state() bytes, uint32 [626] = left, next, state words) of a CPU generator."""
    st = gen.get_state().numpy().copy()
    _, left, _, nxt = struct.unpack_from("<QiiQ", st.tobytes(), 0)
    out = np.empty(STATE_WORDS, np.uint32)
    out[0], out[1] = left, nxt
    out[2:] = np.frombuffer(st[24:24 + 624 * 8].tobytes(), dtype=np.uint64).astype(np.uint32)
    return st, out


def set_generator_words(gen: torch.Generator, st: np.ndarray, words: np.ndarray) -> None:
    b = bytearray(st.tobytes())
    struct.pack_into("<i", b, 8, int(words[0]))
    struct.pack_into("<Q", b, 16, int(words[1]))
    b[24:24 + 624 * 8] = np.asarray(words[2:], np.uint32).astype(np.uint64).tobytes()
    gen.set_state(torch.frombuffer(bytearray(b), dtype=torch.uint8).clone())


def advance_generator(gen: torch.Generator, nwords: int) -> None:
    """Leave the CPU generator where `nwords` 32-bit draws leave it -- torch.rand(nwords,
    generator=gen) on CPU takes one word per f32 element, so this stands for the D bernoulli(p_X)
    words of AS:489 -- by MT19937 jump-ahead (uq_mt_jump_host) instead of drawing them."""
    if nwords < 0:
        raise ValueError("nwords must be >= 0")
    st, w = generator_words(gen)
    left, nxt = int(w[0]), int(w[1])
    rem = left - 1                                   # words left in the current block
    if nwords <= rem:
        w[0], w[1] = left - nwords, nxt + nwords
    else:
        after = nwords - rem                         # words read from the following blocks
        k = (after + 623) // 624                     # twists
        r = after - 624 * (k - 1)                    # words read from the last one (1..624)
        out = np.empty(624, np.uint32)
        key = np.ascontiguousarray(w[2:], np.uint32)
        _lib.check(_lib.load().uq_mt_jump_host(key.ctypes.data, k, out.ctypes.data), "uq_mt_jump_host")
        w[2:] = out
        w[0], w[1] = 625 - r, r
    set_generator_words(gen, st, w)


def _check_state(words: np.ndarray) -> None:
    left, nxt = int(words[0]), int(words[1])
    if not 1 <= left <= 624 or (left > 1 and nxt != 625 - left):
        raise ValueError("generator state with left/next outside ATen mt19937's invariant")


# ---- sender ------------------------------------------------------------------------------------------
class QuicFLSender:
    """AS:429-503 with the same constructor arguments and compress(data) contract."""

    def __init__(self, device=None, bits=(1, 2, 3, 4), sr_bits=(6, 5, 4, 4), prefix=None, tables=None):
        self.device = device if device is not None else _device()
        self.sender_table_X, self.sender_table_p, self.data, self.half_table_size = {}, {}, {}, {}
        self._xp = {}
        if tables is not None:                      # {nbits: (table_X, table_p, data dict)}
            for b, (tx, tp, dd) in tables.items():
                self._add(int(b), torch.as_tensor(tx), torch.as_tensor(tp), dict(dd))
        else:
            prefix = default_tables_prefix() if prefix is None else prefix
            for b, s in zip(bits, sr_bits):
                fn = f"{prefix}{b}_X_{s}_h_256_q_"
                self._add(b, *self.sender_table(fn, self.device))

    def _add(self, b, tx, tp, dd):
        if tx.numel() != tp.numel():
            raise ValueError("sender_table_X and sender_table_p differ in size")
        # AS:489 bernoulli(table_p[idx]) draws ONE 32-bit generator word per coordinate and
        # compares in f32 only for a float32 p; ATen's bernoulli_distribution<double> (a float64
        # p) takes one 64-bit draw (two words) and compares in double, which the kernel does not
        # reproduce: such tables are refused rather than cast (the cast would shift the global
        # generator for every later draw of the caller)
        if tp.dtype != torch.float32:
            raise TypeError(f"sender_table_p must be float32 (got {tp.dtype}): a {tp.dtype} p makes the reference's "
                            "bernoulli draw other generator words (AS:489); not supported")
        if tx.dtype != torch.float32:
            t32 = tx.to(torch.float32)
            if not torch.equal(t32.to(tx.dtype), tx):
                raise TypeError(f"sender_table_X ({tx.dtype}) holds values float32 cannot represent exactly")
            tx = t32
        self.sender_table_X[b], self.sender_table_p[b], self.data[b] = tx, tp, dd
        h = int(dd["h_len"])
        self.half_table_size[b] = ((tx.numel() // h) - 1) * h // 2                      # AS:443

    @staticmethod
    def sender_table(prefix, device=None):
        """AS:447-451 with safe loaders: torch.load(weights_only=True), ast.literal_eval."""
        tx = torch.load(prefix + "sender_table_X.pt", weights_only=True)     # dtypes kept: checked in _add
        tp = torch.load(prefix + "sender_table_p.pt", weights_only=True)
        with open(prefix + "data.txt") as f:
            dd = ast.literal_eval(f.read())
        return tx, tp, dd

    def table_packed(self, nbits: int, dev):
        """The table as u32 (X << 25) | ceil(p * 2^24) on the device (one 4-byte gather per
        coordinate), or None when some X is not an integer in 0..127 or some p is outside
        [0, 1] (then the (X, p) pairs, whose kernel path also flags a bad p like AS:489)."""
        key = ("packed", nbits, dev.index)
        if key not in self._xp:
            X = self.sender_table_X[nbits].reshape(-1).to(torch.float64)
            p = self.sender_table_p[nbits].reshape(-1).to(torch.float64)
            ok = bool(((X == torch.round(X)) & (X >= 0) & (X <= 127)).all() and ((p >= 0) & (p <= 1)).all())
            t = None
            if ok:          # p * 2^24 is exact (a power-of-two scale of an f32), its ceil <= 2^24
                P = torch.ceil(p * float(1 << 24)).to(torch.int64)
                t = ((X.to(torch.int64) << 25) | P).to(torch.int64)
                t = torch.where(t >= (1 << 31), t - (1 << 32), t).to(torch.int32).to(dev).contiguous()
            self._xp[key] = t
        return self._xp[key]

    def table_xp(self, nbits: int, dev) -> torch.Tensor:
        """(X, p) pairs [numel, 2] f32 on the device (one 8-byte gather per coordinate)."""
        key = (nbits, dev.index)
        t = self._xp.get(key)
        if t is None:
            t = torch.stack([self.sender_table_X[nbits].reshape(-1), self.sender_table_p[nbits].reshape(-1)], 1)
            t = t.to(dev).contiguous()
            self._xp[key] = t
        return t

    def compress(self, data, generator: torch.Generator | None = None):
        """AS:455-503.  The bernoulli(p_X) words come from `generator` (default: torch's
        global CPU generator, as the reference on CPU) and advance it by D words."""
        nbits = data["nbits"]
        dd = self.data[nbits]                                          # KeyError like AS:465
        vec = data["vec"]
        v = vec.detach() if torch.is_tensor(vec) else torch.as_tensor(np.asarray(vec))
        v = v.reshape(1, -1)
        if v.shape[1] == 0:
            raise ValueError("empty vector (the reference's RHT and norm of an empty vector are degenerate)")
        gen = generator if generator is not None else torch.default_generator
        st, words = generator_words(gen)
        msg, new = quicfl_compress(v, nbits, [data["seed"]], [data["rotation_seed"]], sender=self,
                                   px_states=words[None, :], x_dtype=torch.int64, _state_out=True)
        set_generator_words(gen, st, new[0])
        cnt = int(msg.exact_count[0])
        return {
            "X": msg.X[0],
            "exact_values": msg.exact_vals[0, :cnt],
            "exact_indeces": msg.exact_mask[0],
            "seed": data["seed"],
            "prng_seed": int(msg.prng_seeds[0]),
            "rotation_seed": data["rotation_seed"],
            "dim": int(v.shape[1]),
            "scale": msg.scale[0],
            "nbits": nbits,
            "h_len": dd["h_len"],
        }


@dataclass
class QuicFLMessages:
    X: torch.Tensor             # [n, D] uint8 or int64
    exact_mask: torch.Tensor    # [n, D] bool (exact_indeces)
    exact_vals: torch.Tensor    # [n, D] f32, row j's exact values in its first exact_count[j] entries
    exact_count: torch.Tensor   # [n] int32 (host)
    scale: torch.Tensor         # [n] f32
    prng_seeds: torch.Tensor    # [n] int64 (host)
    rotation_seeds: torch.Tensor
    dim: int
    nbits: int
    h_len: int

    def exact_dense(self) -> torch.Tensor:
        """[n, D] f32: each message's exact values at their coordinates, 0 elsewhere.  (In row
        blocks of < 2^31 elements: boolean indexing of larger tensors overflows on this torch.)"""
        n, D = self.exact_mask.shape
        dev = self.exact_vals.device
        dense = torch.zeros((n, D), dtype=torch.float32, device=dev)
        cnt = self.exact_count.to(dev)
        ar = torch.arange(D, device=dev)[None, :]
        rows = max(1, ((1 << 31) - 1) // max(D, 1))
        for j0 in range(0, n, rows):
            j1 = min(n, j0 + rows)
            keep = ar < cnt[j0:j1, None]
            dense[j0:j1][self.exact_mask[j0:j1]] = self.exact_vals[j0:j1][keep]
        return dense


def _ws(n, d, dev):
    b = ctypes.c_size_t(0)
    _lib.check(_lib.load().uq_quicfl_workspace_bytes(n, d, ctypes.byref(b)), "uq_quicfl_workspace_bytes")
    return _workspace(dev, int(b.value))


def _send_inputs(ps, n, px_seeds, px_states, dev):
    """The small per-message inputs in ONE host-to-device copy (prng seeds, then the generator
    states or the px seeds): each pageable copy would otherwise wait for the stream on its own.
    -> (prng seeds, states or None, px seeds or None, state words out)."""
    if px_states is not None:
        w = np.asarray(px_states, np.uint32).reshape(n, STATE_WORDS)
        for r in w:
            _check_state(r)
        tail = w.view(np.int32).reshape(-1)
    else:
        if px_seeds is None:
            raise ValueError("px_seeds or px_states is required")
        pxs = np.asarray(torch.as_tensor(px_seeds, dtype=torch.int64).reshape(-1).numpy(), np.int64)
        if pxs.size != n:
            raise ValueError("one px seed per message")
        tail = (pxs & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
    hin = np.empty(n + tail.size, np.int32)
    hin[:n] = ps.numpy().astype(np.int32)
    hin[n:] = tail
    din = torch.from_numpy(hin).to(dev)
    ps_d, tail_d = din[:n], din[n:]
    if px_states is not None:
        return ps_d, tail_d.view(n, STATE_WORDS), None, n * STATE_WORDS
    return ps_d, None, tail_d, 0


def _raise_send_flags(flags: int) -> None:
    if flags & _FLAG_P:
        raise RuntimeError("Expected p_in >= 0 && p_in <= 1 to be true, but got false.")   # AS:484 bernoulli
    if flags & _FLAG_INDEX:
        raise IndexError("out of range: a sender-table index outside the table (AS:486 torch.take)")
    if flags & _FLAG_PX:
        raise RuntimeError("Expected p_in >= 0 && p_in <= 1 to be true, but got false.")   # AS:489 bernoulli
    if flags & _FLAG_X:
        raise OverflowError("X outside 0..255: use x_dtype=torch.int64")
    if flags & _FLAG_TIMEOUT:
        raise RuntimeError("uq_quicfl_compress_f32: internal wait ran out (results invalid)")


def quicfl_compress(x, nbits: int, seeds, rotation_seeds, *, sender: QuicFLSender, px_seeds=None, px_states=None,
                    x_dtype=torch.uint8, _state_out: bool = False):
    """QuicFLSender.compress (AS:455-503) for every row of x [n, d].  seeds: the messages'
    `seed` (hashed to the local generator's seed, AS:457); rotation_seeds: the RHT seeds.
    The bernoulli(p_X) draws (AS:489) of message j come from a fresh generator seeded with
    px_seeds[j], or from px_states[j] ([626] = left, next, state words of a torch CPU
    generator, see generator_words).  X is returned as uint8 (x_dtype=torch.uint8, values
    outside 0..255 raise) or int64 (the reference's X.long())."""
    dev = _device()
    dd = sender.data[nbits]
    x = _as_device_f32_2d(x, dev)
    n, d = x.shape
    D = padded_dim(d)
    s = [int(v) for v in torch.as_tensor(seeds).reshape(-1).tolist()] if not isinstance(seeds, (list, tuple)) else list(seeds)
    rs = torch.as_tensor(rotation_seeds, dtype=torch.int64).reshape(-1)
    if len(s) != n or rs.numel() != n:
        raise ValueError("one seed and one rotation seed per message")
    ps = torch.tensor([prng_seed(v) for v in s], dtype=torch.int64)
    if x_dtype not in (torch.uint8, torch.int64):
        raise ValueError("x_dtype must be torch.uint8 or torch.int64")
    X = torch.empty((n, D), dtype=x_dtype, device=dev)
    mask = torch.empty((n, D), dtype=torch.bool, device=dev)
    ev = torch.empty((n, D), dtype=torch.float32, device=dev)
    scale = torch.empty(n, dtype=torch.float32, device=dev)
    ps_d, st_in, pxs_d, nst = _send_inputs(ps, n, px_seeds, px_states, dev)
    dout = torch.zeros(2 * n + nst, dtype=torch.int32, device=dev)
    info, cnt_d = dout[:n], dout[n:2 * n]
    st_out = dout[2 * n:].view(n, STATE_WORDS) if nst else None
    hout = np.zeros(2 * n + nst, np.int32)
    if n and d:
        tab, rows = _sign_rows(rs, D, dev)
        xp = sender.table_xp(nbits, dev)
        tp = sender.table_packed(nbits, dev) if _USE_PACKED else None
        ws = _ws(n, d, dev)
        _lib.check(_lib.load().uq_quicfl_compress_f32(
            _ptr(x), n, d, _ptr(tab), _ptr(rows), _ptr(xp), _ptr(tp), xp.shape[0], int(dd["h_len"]),
            float(np.float32(dd["delta"])), _ptr(ps_d), _ptr(st_in), _ptr(pxs_d), _ptr(st_out),
            _ptr(X), 0 if x_dtype == torch.int64 else 1, _ptr(mask), _ptr(ev), _ptr(cnt_d), _ptr(scale), _ptr(info),
            _ptr(ws), ws.numel(), _stream_ptr(dev)), "uq_quicfl_compress_f32")
        hout = dout.cpu().numpy()
        _raise_send_flags(int(np.bitwise_or.reduce(hout[:n])) if n else 0)
    msg = QuicFLMessages(X=X, exact_mask=mask, exact_vals=ev, exact_count=torch.from_numpy(hout[n:2 * n].copy()),
                         scale=scale, prng_seeds=ps, rotation_seeds=rs, dim=d, nbits=nbits, h_len=int(dd["h_len"]))
    if _state_out:
        new = hout[2 * n:].reshape(n, STATE_WORDS).view(np.uint32).copy() if nst else None
        return msg, new
    return msg


# ---- receiver ----------------------------------------------------------------------------------------
_X_KIND = {torch.int64: 0, torch.uint8: 1, torch.int32: 2}


def quicfl_decompress(X, nbits: int, prng_seeds, rotation_seeds, scale, dim: int, recv_table, h_len: int | None = None,
                      exact_mask=None, exact_vals=None, exact_count=None, _defer_check: bool = False) -> torch.Tensor:
    """Batched QuicFLReceiver.decompress (AS:526-535).  X [n, D] integers (int64, uint8 or int32
    are read in place on the device) with D a power of two; recv_table [rows, h_len];
    exact_mask bool [n, D] with exact_vals f32 [n, D], or both None.  exact_vals is dense (the
    value at its coordinate) when exact_count is None, else compact: row j's exact values in
    index order in its first exact_count[j] entries (quicfl_compress's layout).  scale [n];
    returns [n, dim] f32.  Raises IndexError where torch.take would (AS:530) and RuntimeError
    when a compact row's count does not match its mask (AS:531)."""
    dev = _device()
    X = torch.as_tensor(X)
    if X.dim() == 1:
        X = X.view(1, -1)
    n, D = X.shape
    if D != padded_dim(D):
        raise ValueError("X rows are the padded (power-of-two) dimension (AS:461-467)")
    if not 0 < dim <= D:
        raise ValueError("dim must be in 1..D")
    tab = torch.as_tensor(recv_table, dtype=torch.float32).to(dev).contiguous()
    rows, hl = (tab.shape[0], tab.shape[1]) if tab.dim() == 2 else (1, tab.numel())
    if h_len is not None and int(h_len) != hl:
        raise ValueError("h_len does not match the receiver table")
    if X.dtype not in _X_KIND:
        X = X.to(torch.int64)
    Xd = X.to(dev).contiguous()
    ps = torch.as_tensor(prng_seeds, dtype=torch.int64).reshape(-1)
    rs = torch.as_tensor(rotation_seeds, dtype=torch.int64).reshape(-1)
    sc = torch.as_tensor(scale, dtype=torch.float32).reshape(-1).to(dev)
    if ps.numel() != n or rs.numel() != n or sc.numel() != n:
        raise ValueError("one prng seed, rotation seed and scale per message")
    if (exact_mask is None) != (exact_vals is None):
        raise ValueError("exact_mask and exact_vals go together")
    m = v = None
    compact = exact_count is not None
    if exact_mask is not None:
        m = torch.as_tensor(exact_mask).to(device=dev).reshape(n, D)
        m = (m if m.dtype in (torch.bool, torch.uint8) else m != 0).contiguous()
        v = torch.as_tensor(exact_vals, dtype=torch.float32).to(dev).reshape(n, D).contiguous()
    pre = torch.empty((n, D), dtype=torch.float32, device=dev)
    info = torch.zeros(n, dtype=torch.int32, device=dev)
    if n:
        # prng seeds (and the exact counts) in one host-to-device copy
        hin = np.empty(2 * n if (compact and m is not None) else n, np.int32)
        hin[:n] = (ps.numpy() & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
        if hin.size > n:
            c = np.asarray(torch.as_tensor(exact_count).reshape(-1).cpu().numpy(), np.int64)
            if c.size != n:
                raise ValueError("one exact count per message")
            hin[n:] = c.astype(np.int32)
        din = torch.from_numpy(hin).to(dev)
        seeds32, cnt = din[:n], (din[n:] if hin.size > n else None)
        L = _lib.load()
        wb = ctypes.c_size_t()
        _lib.check(L.uq_quicfl_receive_workspace_bytes(n, D, ctypes.byref(wb)), "uq_quicfl_receive_workspace_bytes")
        ws = torch.empty(max(int(wb.value), 1), dtype=torch.uint8, device=dev)
        _lib.check(L.uq_quicfl_receive_ws_f32(
            _ptr(Xd), _X_KIND[Xd.dtype], n, D, _ptr(tab), rows, hl, _ptr(seeds32), _ptr(m), _ptr(v),
            1 if (compact and m is not None) else 0, _ptr(cnt), _ptr(sc), _ptr(pre), _ptr(info), _ptr(ws), wb.value,
            _stream_ptr(dev)), "uq_quicfl_receive_ws_f32")
        if not _defer_check:
            _raise_recv_flags(int(np.bitwise_or.reduce(info.cpu().numpy())))
    out = randomized_inverse_hadamard_transform(pre, rs)[:, :dim]
    return (out, info) if _defer_check else out


def _raise_recv_flags(flags: int) -> None:
    if flags & _FLAG_TIMEOUT:
        raise RuntimeError("uq_quicfl_receive_f32: internal wait ran out (results invalid)")
    if flags & _FLAG_INDEX:
        raise IndexError("index out of range in self (AS:530 recv_table.take)")
    if flags & _FLAG_EXACT:
        raise RuntimeError("shape mismatch: exact_values do not match exact_indeces (AS:531)")


def quicfl_decompress_messages(msg: QuicFLMessages, recv_table) -> torch.Tensor:
    """The receiver (AS:526-535) on every message of a quicfl_compress batch -> [n, dim]
    (X, mask and the compact exact values read in place)."""
    return quicfl_decompress(msg.X, msg.nbits, msg.prng_seeds, msg.rotation_seeds, msg.scale, msg.dim, recv_table,
                             msg.h_len, msg.exact_mask, msg.exact_vals, msg.exact_count)


class QuicFLReceiver:
    """AS:507-535 with the same constructor arguments and decompress(data) contract."""

    def __init__(self, device=None, bits=(1, 2, 3, 4), sr_bits=(6, 5, 4, 4), prefix=None, tables=None):
        self.device = device if device is not None else _device()
        self.recv_table = {}
        if tables is not None:                      # {nbits: [rows, h_len] tensor or array}
            for b, t in tables.items():
                self.recv_table[int(b)] = torch.as_tensor(t, dtype=torch.float32)
        else:
            prefix = default_tables_prefix() if prefix is None else prefix
            for b, s in zip(bits, sr_bits):
                fn = f"{prefix}{b}_X_{s}_h_256_q_"
                self.recv_table[b] = self.receiver_table(fn, self.device)

    @staticmethod
    def receiver_table(prefix, device):
        """AS:520-523, loading with weights_only=True (no code from the file runs)."""
        return torch.load(prefix + "recv_table.pt", weights_only=True).to(torch.float32)

    @staticmethod
    def table_params(prefix):
        """The data.txt dictionary next to a table (parsed with ast.literal_eval, not eval)."""
        with open(prefix + "data.txt") as f:
            return ast.literal_eval(f.read())

    def _table(self, nbits):
        """The receiver table on the device (copied once per device)."""
        dev = _device()
        key = ("_dev", int(nbits), dev.index)
        t = self._dev_tables.get(key) if hasattr(self, "_dev_tables") else None
        if t is None:
            if not hasattr(self, "_dev_tables"):
                self._dev_tables = {}
            t = self.recv_table[int(nbits)].to(dev).contiguous()
            self._dev_tables[key] = t
        return t

    def decompress(self, data, _defer_check: bool = False):
        """AS:526-535: the message dict of QuicFLSender.compress -> vec[:dim] (on the GPU)."""
        X = torch.as_tensor(data["X"]).reshape(1, -1)
        D = X.shape[1]
        mask = vals = cnt = None
        ei = data.get("exact_indeces")
        if ei is not None:
            dev = _device()
            mask = torch.as_tensor(ei).reshape(1, D).to(dev)
            ev = torch.as_tensor(data["exact_values"], dtype=torch.float32).reshape(-1)
            if ev.numel() == 1:
                # AS:531 vec[exact_indeces] = exact_values broadcasts a one-element value over
                # every masked coordinate: expand it to the mask's popcount (compact layout)
                k = int(torch.count_nonzero(mask).item())
                if k != 1:
                    ev = ev.expand(k)
            if ev.numel() > D:
                raise RuntimeError("shape mismatch: more exact_values than coordinates (AS:531)")
            vals = torch.zeros((1, D), dtype=torch.float32, device=dev)   # compact: the values, then room to D
            vals[0, :ev.numel()] = ev.to(dev)
            cnt = [ev.numel()]
        self.recv_table[int(data["nbits"])]                              # KeyError like the reference
        res = quicfl_decompress(X, data["nbits"], [int(data["prng_seed"])], [int(data["rotation_seed"])],
                                data["scale"], int(data["dim"]), self._table(data["nbits"]),
                                int(data["h_len"]), mask, vals, cnt, _defer_check=_defer_check)
        if _defer_check:
            return res[0].view(-1), res[1]
        return res.view(-1)


def _dropin_pair():
    prefix = default_tables_prefix()
    dev = _device()
    key = (prefix, dev.index)
    with _dropin_lock:
        pair = _dropin.get(key)
        if pair is None:
            pair = (QuicFLSender(device=dev, prefix=prefix), QuicFLReceiver(device=dev, prefix=prefix))
            _dropin[key] = pair
    return pair


def quicfl_quantize(x, nbits: int, seeds, rotation_seeds, *, sender: QuicFLSender, recv_table, px_seeds=None,
                    px_states=None, _host_out: bool = False):
    """QUICFL_quantize (AS:814-832) on every row of x [n, d]: the sender of quicfl_compress with
    the receiver (AS:526-535, recv_table) fused into it (uq_quicfl_quantize_f32: the receiver's
    h is the sender's own randint stream, so it is not regenerated, and no message is written),
    then the inverse RHT.  Returns (out [n, d], end states [n, 626] or None, scale [n]).
    Raises like the sender, then like the receiver (IndexError from its take, AS:530)."""
    dev = _device()
    dd = sender.data[nbits]
    x = _as_device_f32_2d(x, dev)
    n, d = x.shape
    D = padded_dim(d)
    s = [int(v) for v in torch.as_tensor(seeds).reshape(-1).tolist()] if not isinstance(seeds, (list, tuple)) else list(seeds)
    rs = torch.as_tensor(rotation_seeds, dtype=torch.int64).reshape(-1)
    if len(s) != n or rs.numel() != n:
        raise ValueError("one seed and one rotation seed per message")
    ps = torch.tensor([prng_seed(v) for v in s], dtype=torch.int64)
    rt = torch.as_tensor(recv_table, dtype=torch.float32).to(dev).contiguous().reshape(-1)
    ps_d, st_in, pxs_d, nst = _send_inputs(ps, n, px_seeds, px_states, dev)
    out = torch.empty((n, d), dtype=torch.float32, device=dev)
    scale = torch.empty(n, dtype=torch.float32, device=dev)
    dout = torch.zeros(n + nst, dtype=torch.int32, device=dev)
    info = dout[:n]
    st_out = dout[n:].view(n, STATE_WORDS) if nst else None
    if n and d:
        tab, rows = _sign_rows(rs, D, dev)
        xp = sender.table_xp(nbits, dev)
        tp = sender.table_packed(nbits, dev) if _USE_PACKED else None
        ws = _ws(n, d, dev)
        _lib.check(_lib.load().uq_quicfl_quantize_f32(
            _ptr(x), n, d, _ptr(tab), _ptr(rows), _ptr(xp), _ptr(tp), xp.shape[0], int(dd["h_len"]),
            float(np.float32(dd["delta"])), _ptr(rt), rt.numel(), _ptr(ps_d), _ptr(st_in), _ptr(pxs_d), _ptr(st_out),
            _ptr(out), _ptr(scale), _ptr(info), _ptr(ws), ws.numel(), _stream_ptr(dev)), "uq_quicfl_quantize_f32")
    if _host_out:                          # the result and the flags / states in one synchronisation
        host = torch.empty(out.numel(), dtype=torch.float32, pin_memory=True)
        hsmall = torch.empty(dout.numel(), dtype=torch.int32, pin_memory=True)
        host.copy_(out.view(-1), non_blocking=True)
        hsmall.copy_(dout, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        out, hout = host.view(n, d), hsmall.numpy()
    else:
        hout = dout.cpu().numpy()
    flags = int(np.bitwise_or.reduce(hout[:n])) if n else 0
    _raise_send_flags(flags)
    new = hout[n:].reshape(n, STATE_WORDS).view(np.uint32).copy() if nst else None
    if flags & _FLAG_RECV_INDEX:           # the sender returned (its draws happened), the receiver raises
        raise _RecvIndexError(new)
    return out, new, scale


class _RecvIndexError(IndexError):
    """The receiver's take raised after the sender had drawn (the caller restores the states)."""

    def __init__(self, states):
        super().__init__("index out of range in self (AS:530 recv_table.take)")
        self.states = states


def QUICFL_quantize(input_vector, bits_per_dimension=1):
    """Drop-in for AS:814-832 (same name for the drivers' result keys): one torch.randint(0, 100)
    draw of the global CPU generator (the message seed), the sender (bernoulli(p_X) from the same
    generator, left where the reference leaves it) and the receiver fused in one pass
    (quicfl_quantize); returns a NumPy f32 array of length d."""
    dev = _device()
    if torch.is_tensor(input_vector):
        v = input_vector.detach().to(device=dev, dtype=torch.float32).reshape(-1)
    else:
        v = torch.tensor(np.asarray(input_vector), dtype=torch.float32, device=dev).reshape(-1)
    sender, receiver = _dropin_pair()
    seed = int(torch.randint(0, 100, (1,)).item())
    nbits = bits_per_dimension
    sender.data[nbits]                                                    # KeyError like the sender
    if v.numel() == 0:
        raise ValueError("empty vector (the reference's RHT and norm of an empty vector are degenerate)")
    if nbits not in receiver.recv_table:                                  # the reference's receiver raises
        sender.compress({"vec": v, "seed": seed, "nbits": nbits, "rotation_seed": 123})   # after its sender
        receiver.recv_table[nbits]
    gen = torch.default_generator
    st, words = generator_words(gen)
    try:
        out, new, _ = quicfl_quantize(v.view(1, -1), nbits, [seed], [123], sender=sender,
                                      recv_table=receiver._table(nbits), px_states=words[None, :], _host_out=True)
    except _RecvIndexError as e:
        set_generator_words(gen, st, e.states[0])
        raise IndexError(str(e)) from None
    set_generator_words(gen, st, new[0])
    return out.view(-1).numpy()
