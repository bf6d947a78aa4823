"""GPU: the resident pipeline (pipeline.DMEPipeline) used by bench.py -- K1 -> K2 (q + codes)
-> client mean from the codes -- equals the batched APIs bit for bit, before and after the
output-placement probe swaps its buffers (ND:133-138, AS:609-641)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,d,bits", [(300, 8192, 1), (5, 40000, 2)])
def test_pipeline_step_matches_batched_apis(gpu_ready, n, d, bits):
    import uqdme
    g = torch.Generator(device="cuda").manual_seed(n + d)
    x = torch.randn(n, d, generator=g, device="cuda")
    X = torch.rand(n, generator=torch.Generator().manual_seed(3)).cuda()
    q_ref = uqdme.quantize_dequantize(x, bits, X=X, torch_threads=1)
    est_ref = uqdme.client_mean(q_ref, float(n))
    p = uqdme.DMEPipeline(n, d, bits, torch_threads=1)
    for probe in (False, True):
        if probe:
            rep = p.probe_outputs(x, X, candidates=3, reps=1)
            assert 1 < rep["candidates"] <= 3 and 0 <= rep["chosen"] < rep["candidates"]
        est = p.step(x, X)
        torch.cuda.synchronize()
        p.check_status()
        assert torch.equal(est.view(torch.int32), est_ref.view(torch.int32)), probe
        assert torch.equal(p.q.view(torch.int32), q_ref.view(torch.int32)), probe
        dec = uqdme.decode(uqdme.TypeCodes(codes=p.codes, l1=p.l1, m=p.m, overflow=p.kmax))
        assert torch.equal(dec.view(torch.int32), q_ref.view(torch.int32)), probe
    with pytest.raises(ValueError):
        p.step(x[:, :-1].contiguous(), X)
