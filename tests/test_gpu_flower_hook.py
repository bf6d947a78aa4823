"""Config C5: the Flower client's quantization hook, exercised without
flwr.  Emulates the contract of SImulation_Results_datasets/MNIST/Codes/Type_unbiased.py
(FLM:147-212) around the drop-ins: flat model update -> quantization_func(tensor, bits) ->
quantization error / norm (tensor or ndarray result) -> update + global params reshaped per
layer; the function's __name__ keys the result directories (FLM:177)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Flatten(), torch.nn.Linear(28 * 28, 200), torch.nn.ReLU(),
                               torch.nn.Linear(200, 10))


def _client_round(qfunc, bits, model, global_flat):
    arrays = [v.detach().cpu().numpy() for v in model.state_dict().values()]
    shapes = [a.shape for a in arrays]
    sizes = [a.size for a in arrays]
    flat = np.concatenate([a.reshape(-1) for a in arrays])
    grad_t = torch.from_numpy(flat - global_flat).float().cuda()                 # FLM:158
    out = qfunc(grad_t, bits)                                                     # FLM:159
    q_t = torch.from_numpy(out).cuda() if isinstance(out, np.ndarray) else out    # FLM:166-169
    err = q_t - grad_t                                                            # FLM:170
    gnorm = torch.norm(grad_t).item()                                             # FLM:171
    q_np = out if isinstance(out, np.ndarray) else out.cpu().numpy()              # FLM:197-205
    params = q_np + global_flat
    layers, off = [], 0
    for shp, sz in zip(shapes, sizes):
        layers.append(params[off:off + sz].reshape(shp))
        off += sz
    return layers, float(torch.norm(err).item() ** 2 / max(gnorm ** 2, 1e-30)), qfunc.__name__


def test_hook_with_the_drop_ins(gpu_ready):
    import uqdme
    model = _model()
    with torch.no_grad():
        global_flat = np.concatenate([v.cpu().numpy().reshape(-1) for v in model.state_dict().values()])
        for p in model.parameters():                                   # a "local training" step
            p.add_(0.01 * torch.randn_like(p))
    d = global_flat.size
    names = set()
    for qfunc, bits in ((uqdme.Type_unbiased_quantize, 1), (uqdme.Type_unbiased_quantize, 2),
                        (uqdme.Type_biased_quantize, 1), (uqdme.EDEN_quantize_Hadamard, 2)):
        layers, nmse, name = _client_round(qfunc, bits, model, global_flat)
        names.add(name)
        assert [l.shape for l in layers] == [v.shape for v in model.state_dict().values()]
        assert all(l.dtype == np.float32 for l in layers)
        assert np.isfinite(nmse) and 0.0 < nmse < 10.0, (name, bits, nmse)
        # the quantized update loads back into the model (set_parameters, FLM:140-145)
        sd = {k: torch.as_tensor(v) for k, v in zip(model.state_dict().keys(), layers)}
        _model().load_state_dict(sd, strict=True)
    assert names == {"Type_unbiased_quantize", "Type_biased_quantize", "EDEN_quantize_Hadamard"}
    assert d == 28 * 28 * 200 + 200 + 200 * 10 + 10


def test_hook_unbiasedness_over_rounds(gpu_ready):
    """Unbiased quantizer: the average of many quantized updates approaches the update."""
    import uqdme
    g = torch.randn(4096, device="cuda")
    acc = torch.zeros_like(g)
    for _ in range(200):
        acc += uqdme.Type_unbiased_quantize(g, 1)
    rel = (torch.norm(acc / 200 - g) / torch.norm(g)).item()
    assert rel < 0.25, rel
