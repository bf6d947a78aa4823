"""Golden vectors for the QUIC-FL receiver (AS:507-535), produced by running the reference's
QuicFLReceiver.decompress here on synthetic messages (its sender cannot run: the sender tables
are missing from the reference).  Also stores the reference's receiver tables and their
data.txt parameters as fixture data (the GPU box has no /root/reference).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_quicfl.py
"""
import ast
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/NMSE_Results/Codes"


def main():
    sys.path.insert(0, REF)
    import All_Schemes as AS  # noqa: E402  (the reference, imported for its receiver)
    rx = AS.QuicFLReceiver(device="cpu")
    tables, meta = {}, {"tables": {}, "cases": []}
    for b, s in ((1, 6), (2, 5), (3, 4), (4, 4)):
        pre = os.path.join(REF, "tables", f"{b}_X_{s}_h_256_q_")
        t = torch.load(pre + "recv_table.pt", weights_only=True)
        data = ast.literal_eval(open(pre + "data.txt").read())
        tables[f"recv{b}"] = t.numpy().astype(np.float32)
        meta["tables"][str(b)] = {"h_len": int(data["h_len"]), "shape": list(t.shape), "delta": data["delta"],
                                  "T": data["T"], "x_len": data["x_len"]}
    rng = np.random.default_rng(2025)
    arrays = dict(tables)
    k = 0
    for nbits in (1, 2, 3, 4):
        h_len = meta["tables"][str(nbits)]["h_len"]
        for dim in (1000, 4096, 70000):
            D = 1 << int(np.ceil(np.log2(dim)))
            X = rng.integers(0, 1 << nbits, size=D).astype(np.int64)
            mask = rng.random(D) < 0.004
            vals = (rng.standard_normal(int(mask.sum())) * 3.5).astype(np.float32)
            scale = torch.tensor(float(np.sqrt(D) / (rng.random() * 50 + 10)), dtype=torch.float32)
            msg = {"X": torch.from_numpy(X), "exact_values": torch.from_numpy(vals),
                   "exact_indeces": torch.from_numpy(mask), "seed": 0, "prng_seed": int(rng.integers(0, 1 << 16)),
                   "rotation_seed": int(rng.integers(0, 100)), "dim": dim, "scale": scale, "nbits": nbits,
                   "h_len": h_len}
            out = rx.decompress(msg).numpy().astype(np.float32)
            arrays[f"X{k}"] = X.astype(np.int32)
            arrays[f"mask{k}"] = mask
            arrays[f"vals{k}"] = vals
            arrays[f"out{k}"] = out
            meta["cases"].append({"idx": k, "nbits": nbits, "dim": dim, "D": D, "prng_seed": msg["prng_seed"],
                                  "rotation_seed": msg["rotation_seed"], "scale": float(scale.item()), "h_len": h_len})
            k += 1
    np.savez_compressed(os.path.join(HERE, "quicfl_recv_vectors.npz"), **arrays)
    json.dump(meta, open(os.path.join(HERE, "quicfl_recv_vectors.json"), "w"), indent=1)
    print(f"{k} cases")


if __name__ == "__main__":
    main()
