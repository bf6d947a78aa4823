"""Golden vectors for the QUIC-FL sender (AS:429-503), its receiver (AS:507-535) and the
QUICFL_quantize drop-in (AS:814-832) at config C4's size, D = 2^22, produced by running the
reference's own code here on the synthetic sender tables of quicfl_tables.py (the published
sender tables are missing; see make_golden_quicfl_sender.py).

Cases: dim = 2^22 (a power of two) and dim = 2^22 - 5 (padded to D = 2^22), 1 and 2 bits,
generator states on and off a block edge.  Messages are stored as SHA-256 of X (int64 bytes),
of the mask (bool bytes) and of the exact values (f32 bytes) plus 4096 sampled positions, the
global generator's end state, and the reference receiver's output (SHA-256 + samples).
Inputs are regenerated from their seeds (numpy RandomState, as in make_golden_quicfl_sender).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_quicfl_c4.py
"""
import hashlib
import json
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden_quicfl_sender import REF, gen, gen_state, write_prefix  # noqa: E402

CASES = [  # (kind, vseed, dim, nbits, seed, gseed, pre)
    ("normal", 4101, 1 << 22, 1, 42, 4101, 0),
    ("laplace", 4102, (1 << 22) - 5, 1, 7, 4102, 311),
    ("normal", 4103, 1 << 22, 2, 93, 4103, 624),
    ("laplace", 4104, (1 << 22) - 5, 2, 0, 4104, 1000),
]
DROPIN = [("normal", 4201, 1 << 22, 1, 42)]   # (kind, vseed, dim, nbits, gseed): QUICFL_quantize


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    sys.path.insert(0, REF)
    import All_Schemes as AS  # noqa: E402  (the reference)
    torch.set_num_threads(1)
    pre_dir = write_prefix(os.path.join(tempfile.mkdtemp(prefix="qfl_c4_"), "pub"))
    snd = AS.QuicFLSender(device="cpu", prefix=pre_dir)
    rx = AS.QuicFLReceiver(device="cpu")
    arrays, cases = {}, []
    for k, (kind, vseed, dim, nbits, seed, gseed, pre) in enumerate(CASES):
        x = gen(kind, vseed, dim)
        torch.manual_seed(gseed)
        if pre:
            torch.rand(pre)
        left0, next0, _ = gen_state()
        msg = snd.compress({"vec": torch.from_numpy(x.copy()), "seed": seed, "nbits": nbits, "rotation_seed": 123})
        left1, next1, words1 = gen_state()
        X = msg["X"].numpy()
        mask = msg["exact_indeces"].numpy()
        ev = msg["exact_values"].numpy().astype(np.float32)
        out = rx.decompress(msg).numpy().astype(np.float32)
        rng = np.random.default_rng(k)
        pos = np.sort(rng.choice(X.size, 4096, replace=False)).astype(np.int64)
        opos = np.sort(rng.choice(out.size, 4096, replace=False)).astype(np.int64)
        c = {"idx": k, "kind": kind, "vseed": vseed, "dim": dim, "nbits": nbits, "seed": seed, "gseed": gseed,
             "pre": pre, "left0": left0, "next0": next0, "left1": left1, "next1": next1, "D": int(X.size),
             "prng_seed": int(msg["prng_seed"]), "scale_bits": int(np.float32(msg["scale"].item()).view(np.uint32)),
             "n_exact": int(ev.size), "X_sha": sha(X.astype(np.int64)), "mask_sha": sha(mask.astype(np.bool_)),
             "ev_sha": sha(ev), "rx_sha": sha(out)}
        arrays[f"pos{k}"] = pos
        arrays[f"Xs{k}"] = X[pos].astype(np.uint8)
        arrays[f"ms{k}"] = mask[pos]
        arrays[f"ev{k}"] = ev                                   # a few thousand values
        arrays[f"opos{k}"] = opos
        arrays[f"rxs{k}"] = out[opos]
        arrays[f"st1_{k}"] = words1
        cases.append(c)
        print(k, dim, nbits, "exact", ev.size, flush=True)
    AS.QuicFLSender.__init__.__defaults__ = ("cpu", [1, 2, 3, 4], [6, 5, 4, 4], pre_dir)
    dropin = []
    for j, (kind, vseed, dim, nbits, gseed) in enumerate(DROPIN):
        x = gen(kind, vseed, dim)
        torch.manual_seed(gseed)
        out = AS.QUICFL_quantize(x, nbits).astype(np.float32)
        left1, next1, words1 = gen_state()
        opos = np.sort(np.random.default_rng(100 + j).choice(out.size, 4096, replace=False)).astype(np.int64)
        arrays[f"dpos{j}"] = opos
        arrays[f"douts{j}"] = out[opos]
        arrays[f"dst1_{j}"] = words1
        dropin.append({"idx": j, "kind": kind, "vseed": vseed, "dim": dim, "nbits": nbits, "gseed": gseed,
                       "left1": left1, "next1": next1, "out_sha": sha(out)})
    np.savez_compressed(os.path.join(HERE, "quicfl_c4_vectors.npz"), **arrays)
    json.dump({"cases": cases, "dropin": dropin}, open(os.path.join(HERE, "quicfl_c4_vectors.json"), "w"), indent=1)
    print(len(cases), "compress cases,", len(dropin), "drop-in")


if __name__ == "__main__":
    main()
