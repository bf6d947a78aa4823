"""The same rows give the same bits whichever internal path a call takes: one-vector calls
(the drop-in's entry; the segmented norm) against batches (the stream / small-batch forms;
the sequential norm chains above 256 rows), at the sizes where the dispatch changes."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def uq(gpu_ready):
    import uqdme
    return uqdme


def _bits(t):
    return t.contiguous().view(torch.int32)


def test_unbiased_one_vector_entry_matches_batch(uq):
    rng = np.random.default_rng(31)
    d = (1 << 20) + 12
    x = torch.as_tensor(rng.standard_normal((5, d)).astype(np.float32)).cuda()
    X = torch.rand(5, generator=torch.Generator().manual_seed(31))
    batch = uq.quantize_dequantize(x, 1, X=X, torch_threads=1)
    for j in range(5):
        one = uq.quantize_dequantize(x[j:j + 1], 1, X=X[j:j + 1], torch_threads=1)
        assert torch.equal(_bits(one[0]), _bits(batch[j])), j


def test_eden_2pow22_segmented_and_chain_norms_agree(uq):
    """D = 2^22 (14 + 8 passes, compress + decompress): a 300-row batch (sequential norm
    chains) and one-row calls (segmented chains) give the same outputs bit for bit."""
    rng = np.random.default_rng(32)
    d = 1 << 22
    n = 300
    g = torch.Generator(device="cuda").manual_seed(32)
    x = torch.randn(n, d, generator=g, device="cuda")
    seeds = [int(s) for s in rng.integers(0, 100, n)]
    batch = uq.eden_quantize(x, 1, seeds=seeds)
    for j in (0, 137, 299):
        one = uq.eden_quantize(x[j:j + 1], 1, seeds=[seeds[j]])
        assert torch.equal(_bits(one[0]), _bits(batch[j])), j
    del batch, x
    torch.cuda.empty_cache()
