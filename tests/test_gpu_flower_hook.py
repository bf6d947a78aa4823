"""Config C5: the Flower client's quantization hook on the
reference's own model, without flwr.

tests/fl_harness.py restates FlowerClient.get_parameters (FLM:148-212) and Net (FLM:37-56,
d = 172 554).  Two FedAvg rounds of 5 clients (plus the initialisation call) run through the
hook with the drop-in Type_unbiased_quantize at the host's default torch thread count (the
order torch's CPU sum would use in this process, AS:624); every quantized update is
compared bit for bit with the C oracle on the same delta, the same X (the draw the drop-in
took from the global generator, AS:634) and the same T.  The NMSE_info files the hook wrote
then go through compute_nmse_stats_auto (NMSE_Results.py:43-140), checked against the same
statistic computed from the oracle's outputs.  Published FL numbers (accuracy, CIFAR-10
NMSE) need flwr + MNIST/CIFAR data and stay statistically pinned only."""
import os

import numpy as np
import pytest
import torch

from tests.fl_harness import HookClient, Net, local_train, synthetic_batches

pytestmark = pytest.mark.gpu


def _oracle_q(gradient, X, bits, T):
    from oracle import uq_oracle_c as C
    from oracle.uq_oracle import rate_to_m
    out, _ = C.quantize_batch(gradient[None].astype(np.float32), rate_to_m(bits, gradient.size),
                              np.array([X], np.float32), T)
    return out[0]


def _x_of(rng_state):
    cur = torch.get_rng_state()
    torch.set_rng_state(rng_state)
    X = float(torch.rand(1).item())
    torch.set_rng_state(cur)
    return X


def test_hook_fedavg_rounds_bit_exact_and_nmse_stats(gpu_ready, tmp_path):
    import uqdme
    T = uqdme.get_torch_threads()
    assert T == torch.get_num_threads()            # the drop-in follows the host's default
    nmse_dir = str(tmp_path / "NMSE_Results_MNIST")
    hand = {}
    for bits in (1, 2):
        torch.manual_seed(42)                      # FLM:30
        server = Net(num_classes=10)
        d = sum(p.numel() for p in server.parameters())
        assert d == 172554
        glob = [v.cpu().numpy().copy() for v in server.state_dict().values()]
        init = HookClient(Net(num_classes=10), uqdme.Type_unbiased_quantize, bits, nmse_dir)
        init.model.load_state_dict(server.state_dict())
        init.get_parameters()                      # the server's initial parameter request (NMSE_info_1)
        q0 = init.last
        assert np.array_equal(q0["quantized"].view(np.uint32),
                              _oracle_q(q0["gradient"], _x_of(q0["rng_before"]), bits, T).view(np.uint32))
        rounds = []
        for r in range(2):
            updates = []
            errs, norms = [], []
            for j in range(5):
                cl = HookClient(Net(num_classes=10), uqdme.Type_unbiased_quantize, bits, nmse_dir)
                cl.set_parameters(glob)
                local_train(cl.model, synthetic_batches(100 * bits + 10 * r + j))
                layers = cl.get_parameters()
                g, X = cl.last["gradient"], _x_of(cl.last["rng_before"])
                want = _oracle_q(g, X, bits, T)
                got = cl.last["quantized"]
                assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), \
                    (bits, r, j, int(np.count_nonzero(got.view(np.uint32) != want.view(np.uint32))))
                # conv3 / conv4 are not used by forward: their deltas and quantized deltas are 0
                assert np.all(want[12832 + 416:12832 + 416 + 18496 + 73856] == 0)
                assert [a.shape for a in layers] == [v.shape for v in glob]
                updates.append(layers)
                errs.append(torch.from_numpy(want - g))
                norms.append(float(torch.norm(torch.from_numpy(g)).item()))
            rounds.append(uqdme.round_nmse(errs, norms, 5))
            glob = [np.mean([u[i] for u in updates], axis=0).astype(np.float32) for i in range(len(glob))]
        hand[bits] = rounds
    rows = uqdme.compute_nmse_stats_auto(nmse_dir, 5, excel_filename=str(tmp_path / "stats.xlsx"), verbose=False)
    assert {r["Rate Folder"] for r in rows} == {"rate_1", "rate_2"}
    for row in rows:
        bits = int(row["Rate Folder"].split("_")[1])
        assert row["Scheme"] == "Type_unbiased_quantize" and row["No of Rounds"] == 2
        want_max, want_avg = max(hand[bits]), float(np.mean(hand[bits]))
        assert abs(row["max_nmse"] - want_max) <= 1e-5 * want_max, (row, hand[bits])
        assert abs(row["avg_nmse"] - want_avg) <= 1e-5 * want_avg, (row, hand[bits])
        assert 0.0 < row["avg_nmse"] < (1.0 if bits == 1 else 0.3)


def test_hook_other_drop_ins_on_net(gpu_ready, tmp_path):
    """Biased and EDEN drop-ins through the same hook: names key the result folders
    (FLM:177), outputs reload into Net (FLM:141-146)."""
    import uqdme
    torch.manual_seed(42)
    base = Net(num_classes=10)
    glob = [v.cpu().numpy().copy() for v in base.state_dict().values()]
    names = set()
    for qfunc, bits in ((uqdme.Type_biased_quantize, 1), (uqdme.EDEN_quantize_Hadamard, 2)):
        cl = HookClient(Net(num_classes=10), qfunc, bits, str(tmp_path))
        cl.set_parameters(glob)
        local_train(cl.model, synthetic_batches(7))
        layers = cl.get_parameters()
        names.add(qfunc.__name__)
        sd = {k: torch.as_tensor(v) for k, v in zip(base.state_dict().keys(), layers)}
        Net(num_classes=10).load_state_dict(sd, strict=True)
        err = cl.last["quantized"] - cl.last["gradient"]
        rel = float(np.sum(err.astype(np.float64) ** 2) / np.sum(cl.last["gradient"].astype(np.float64) ** 2))
        assert np.isfinite(rel) and 0.0 < rel < 10.0
        assert os.path.isdir(tmp_path / qfunc.__name__ / f"rate_{bits}")
    assert names == {"Type_biased_quantize", "EDEN_quantize_Hadamard"}


def test_hook_unbiasedness_over_rounds(gpu_ready):
    """Unbiased quantizer: the average of many quantized updates approaches the update."""
    import uqdme
    g = torch.randn(4096, device="cuda")
    acc = torch.zeros_like(g)
    for _ in range(200):
        acc += uqdme.Type_unbiased_quantize(g, 1)
    rel = (torch.norm(acc / 200 - g) / torch.norm(g)).item()
    assert rel < 0.25, rel
