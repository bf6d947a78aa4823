"""Golden vectors for the QUIC-FL sender (AS:429-503) and the QUICFL_quantize drop-in
(AS:814-832), produced by running the reference's own QuicFLSender.compress here.

The reference's sender tables are missing, but its constructor takes a
`prefix` (AS:431) and loads `sender_table_X.pt`, `sender_table_p.pt` and `data.txt` from it
(AS:447-451).  This script writes synthetic tables (tests/golden/quicfl_tables.py: the shape
rule of AS:443, the reference's own data.txt parameters) into a temporary prefix, runs the
reference's compress on them, and commits inputs and outputs.  The data.txt files it writes
are literals built here, so the reference's `eval` (AS:450) only ever reads text from this
script.  QUICFL_quantize is run end to end by pointing QuicFLSender's default prefix at the
temporary tables (its receiver keeps the reference's real receiver tables).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_quicfl_sender.py
"""
import hashlib
import json
import os
import struct
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from quicfl_tables import DATA, SR_BITS, data_txt, sender_tables  # noqa: E402

REF = "/root/reference/NMSE_Results/Codes"


def write_prefix(root, x_len=None, delta=None):
    os.makedirs(root, exist_ok=True)
    for b in (1, 2, 3, 4):
        fn = os.path.join(root, f"{b}_X_{SR_BITS[b]}_h_256_q_")
        X, p = sender_tables(b, x_len=x_len)
        torch.save(torch.from_numpy(X), fn + "sender_table_X.pt")
        torch.save(torch.from_numpy(p), fn + "sender_table_p.pt")
        over = {}
        if x_len is not None:
            over["x_len"] = x_len
        if delta is not None:
            over["delta"] = delta
        with open(fn + "data.txt", "w") as f:
            f.write(data_txt(b, **over))
    return root + "/"


def gen(kind, seed, dim):
    rs = np.random.RandomState(seed)
    if kind == "normal":
        v = rs.normal(0, 1, dim)
    elif kind == "laplace":
        v = rs.laplace(1, 2, dim)
    elif kind == "zeros":
        v = np.zeros(dim)
    elif kind == "spike":                       # one huge coordinate (the RHT spreads it out)
        v = rs.normal(0, 1, dim)
        v[dim // 3] = 3000.0
    else:
        raise ValueError(kind)
    return v.astype(np.float32)


def gen_state():
    st = torch.default_generator.get_state().numpy()
    _, left, _, nxt = struct.unpack_from("<QiiQ", st, 0)
    words = np.frombuffer(st[24:24 + 624 * 8].tobytes(), dtype=np.uint64).astype(np.uint32)
    return int(left), int(nxt), words


def main():
    sys.path.insert(0, REF)
    import All_Schemes as AS  # noqa: E402  (the reference)
    torch.set_num_threads(1)
    tmp = tempfile.mkdtemp(prefix="qfl_sender_")
    prefixes = {"pub": write_prefix(os.path.join(tmp, "pub")),           # data.txt of the reference
                "small": write_prefix(os.path.join(tmp, "small"), x_len=101, delta=0.06),
                "oor": write_prefix(os.path.join(tmp, "oor"), x_len=101, delta=0.05)}
    senders = {k: AS.QuicFLSender(device="cpu", prefix=v) for k, v in prefixes.items()}
    rx = AS.QuicFLReceiver(device="cpu")                                  # the reference's receiver tables
    arrays, cases = {}, []

    def run(tag, kind, vseed, dim, nbits, seed, rot, gseed, pre, store_x):
        k = len(cases)
        x = gen(kind, vseed, dim)
        torch.manual_seed(gseed)
        if pre:
            torch.rand(pre)                      # move the global generator off its seeded state
        left0, next0, words0 = gen_state()
        c = {"idx": k, "tables": tag, "kind": kind, "vseed": vseed, "dim": dim, "nbits": nbits, "seed": seed,
             "rotation_seed": rot, "gseed": gseed, "pre": pre, "left0": left0, "next0": next0}
        try:
            msg = senders[tag].compress({"vec": torch.from_numpy(x.copy()), "seed": seed, "nbits": nbits,
                                         "rotation_seed": rot})
        except Exception as e:                   # noqa: BLE001  (the reference's own error)
            c["error"] = type(e).__name__
            c["message"] = str(e)[:80]
            cases.append(c)
            return
        left1, next1, words1 = gen_state()
        X = msg["X"].numpy()
        assert X.dtype == np.int64 and X.min() >= 0 and X.max() < 256
        ei = np.flatnonzero(msg["exact_indeces"].numpy()).astype(np.int32)
        c.update({"prng_seed": int(msg["prng_seed"]), "scale_bits": int(np.float32(msg["scale"].item()).view(np.uint32)),
                  "D": int(X.size), "h_len": int(msg["h_len"]), "n_exact": int(ei.size), "left1": left1,
                  "next1": next1, "x_stored": bool(store_x)})
        assert msg["scale"].dtype == torch.float32 and msg["scale"].dim() == 0
        assert msg["exact_values"].dtype == torch.float32
        if store_x:
            arrays[f"x{k}"] = x
        arrays[f"X{k}"] = X.astype(np.uint8)
        arrays[f"ei{k}"] = ei
        arrays[f"ev{k}"] = msg["exact_values"].numpy().astype(np.float32)
        arrays[f"st0_{k}"] = words0
        arrays[f"st1_{k}"] = words1
        if tag == "pub":                         # the reference's receiver on the reference's message
            out = rx.decompress(msg).numpy().astype(np.float32)
            if out.size <= 1 << 17:
                arrays[f"rx{k}"] = out
            else:                                # large: sha256 of the bits + a sample
                pos = np.random.default_rng(k).choice(out.size, 4096, replace=False).astype(np.int64)
                c["rx_sha"] = hashlib.sha256(out.tobytes()).hexdigest()
                arrays[f"rxpos{k}"] = pos
                arrays[f"rxs{k}"] = out[pos]
        cases.append(c)

    seeds = iter(range(1000, 100000, 37))
    for nbits in (1, 2, 3, 4):
        for kind, dim in (("normal", 1000), ("laplace", 4096), ("normal", 65536), ("laplace", 70000)):
            s = next(seeds)
            run("pub", kind, s, dim, nbits, s % 100, 123, s, (0, 1, 623, 700)[nbits - 1], dim <= 4096)
    for dim in (1, 2, 3, 5, 8, 17):
        s = next(seeds)
        run("pub", "normal", s, dim, 1 + dim % 4, s % 100, 7, s, 624 if dim == 3 else 0, True)
    run("pub", "spike", 77, 2048, 2, 5, 123, 77, 1249, True)
    run("pub", "spike", 78, 5000, 4, 99, 11, 78, 3, True)
    run("pub", "zeros", 0, 512, 1, 3, 123, 5, 0, True)                     # ||v|| = 0: bernoulli(NaN) raises
    run("pub", "normal", 501, 1 << 20, 1, 42, 123, 501, 5, False)          # config-scale message
    run("small", "normal", 502, 3000, 2, 17, 123, 502, 0, True)            # a 101-row table
    run("small", "laplace", 503, 1024, 4, 18, 9, 503, 10, True)
    run("oor", "normal", 504, 4096, 1, 19, 123, 504, 0, True)              # index beyond the table: raises

    # QUICFL_quantize (AS:814-832) end to end: seed draw, compress, decompress on the global generator
    AS.QuicFLSender.__init__.__defaults__ = ("cpu", [1, 2, 3, 4], [6, 5, 4, 4], prefixes["pub"])
    dropin = []
    for j, (kind, dim, nbits, gseed) in enumerate((("normal", 1024, 1, 42), ("laplace", 3000, 2, 7),
                                                    ("normal", 4096, 4, 11))):
        x = gen(kind, 900 + j, dim)
        torch.manual_seed(gseed)
        outs = [AS.QUICFL_quantize(x, nbits).astype(np.float32) for _ in range(2)]   # two calls in a row
        left1, next1, words1 = gen_state()
        arrays[f"dx{j}"] = x
        for t, o in enumerate(outs):
            arrays[f"dout{j}_{t}"] = o
        arrays[f"dst1_{j}"] = words1
        dropin.append({"idx": j, "kind": kind, "dim": dim, "nbits": nbits, "gseed": gseed, "left1": left1,
                       "next1": next1})

    np.savez_compressed(os.path.join(HERE, "quicfl_sender_vectors.npz"), **arrays)
    meta = {"data": {str(b): DATA[b] for b in DATA}, "sr_bits": {str(b): SR_BITS[b] for b in SR_BITS},
            "small": {"x_len": 101, "delta": 0.06}, "oor": {"x_len": 101, "delta": 0.05},
            "cases": cases, "dropin": dropin}
    json.dump(meta, open(os.path.join(HERE, "quicfl_sender_vectors.json"), "w"), indent=1)
    print(len(cases), "compress cases,", len(dropin), "drop-in cases;",
          sum("error" in c for c in cases), "raising")


if __name__ == "__main__":
    main()
