"""The fused sampler's specification (oracle/model.py sample_topk_spec / inverse_cdf) against the reference's own
torch ops on the CPU (generate/base.py:30-41): torch.topk's kept values, softmax(logits / T) in bf16, and the
inverse CDF torch.multinomial draws from. CPU only."""

import numpy as np
import pytest
import torch

from oracle import model as om


def _logits(n, seed, ties=False):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, generator=g) * 3
    if ties:
        x = x.round()
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("n,k,ties", [(1000, 1, False), (32000, 200, False), (32000, 200, True), (50, 50, False),
                                      (300, 1024, True), (4096, 37, True)])
def test_spec_matches_torch_ops(n, k, ties):
    x = _logits(n, n + k, ties)
    kept, p, tok = om.sample_topk_spec(x, k, 0.8, 0.37)
    kk = min(k, n)
    # the kept set holds exactly torch.topk's values; ties at the k-th value are the lowest indices
    v, i = torch.topk(x.float(), kk)
    assert sorted(x[kept].float().tolist()) == sorted(v.tolist())
    kth = float(v.min())
    tied = [j for j in range(n) if float(x[j]) == kth]
    assert [j for j in kept if float(x[j]) == kth] == tied[:len([j for j in kept if float(x[j]) == kth])]
    # probabilities: the reference's bf16 softmax over the scattered logits, within one bf16 ulp
    full = torch.full_like(x, float("-inf")).scatter_(-1, torch.tensor(kept), x[kept])
    ref = torch.softmax(full / 0.8, dim=-1)[kept].float()
    assert torch.allclose(p, ref, rtol=2 ** -7, atol=0)
    assert tok in kept


def test_inverse_cdf_is_first_index_reaching_u():
    p = np.array([0.0, 0.25, 0.0, 0.5, 0.25], dtype=np.float32)
    assert om.inverse_cdf(p, 1e-6) == 1
    assert om.inverse_cdf(p, 0.25) == 1
    assert om.inverse_cdf(p, 0.2500001) == 3
    assert om.inverse_cdf(p, 0.75) == 3
    assert om.inverse_cdf(p, 0.9999) == 4
    # frequencies over a uniform grid follow p
    us = (np.arange(10000) + 0.5) / 10000
    counts = np.bincount([om.inverse_cdf(p, u) for u in us], minlength=5)
    assert np.allclose(counts / 10000, p, atol=1e-3)


def test_spec_nan_is_kept_first():
    x = _logits(100, 3)
    x[17] = float("nan")
    kept = om.sample_topk_spec(x, 5, 1.0, 0.5)[0]
    assert 17 in kept  # torch.topk orders NaN above every number
    assert sorted(kept) == kept and len(kept) == 5
