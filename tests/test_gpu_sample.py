"""The fused top-k + temperature + softmax + multinomial sampler (csrc/sample.hip lga_sample_topk) on the MI355X.

generate/base.py:30-41 with top_k and temperature > 0. Checked against oracle/model.py sample_topk_spec (itself
pinned to torch's CPU ops by tests/test_sample_oracle.py): the kept set bit-exact (and equal to torch.topk's
values on the device), the probabilities within one bf16 ulp, and the drawn token equal to the oracle's inverse
CDF on the same uniform — exactly over the kernel's own probabilities, and over the oracle's wherever u is not
within 1e-3 of a CDF step. Then the RNG path: counter-driven draws follow the distribution, replay in a HIP graph,
and a sampled decode through DecodeGraph equals the eager decode with the same seed.
"""

import numpy as np
import pytest
import torch

from oracle import model as om

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    from lit_gpt import ops as _ops

    _ops.load_library()
    return _ops


def _logits(n, seed, ties=False, scale=3.0):
    """ties False / True (rounded: heavy ties) / "peaked" (one logit far above the rest: the k-th largest lies
    outside the kernel's window below the max, so its radix fallback runs) / "ninf" (all but 5 logits -inf: the
    k-th is a tie among -inf, taken lowest index first)."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, generator=g) * scale
    if ties is True:
        x = x.round()
    elif ties == "peaked":
        x[n // 3] = 1000.0
    elif ties == "ninf":
        x = torch.full((n,), float("-inf"))
        x[torch.randperm(n, generator=g)[:5]] = torch.randn(5, generator=g)
    return x.to(torch.bfloat16)


def _draw(ops, x, k, T, u):
    kk = min(k, x.numel())
    kept = torch.full((kk,), -1, dtype=torch.int32, device=DEV)
    probs = torch.zeros(kk, dtype=torch.bfloat16, device=DEV)
    uni = torch.tensor([u], dtype=torch.float32, device=DEV)
    tok = ops.sample_topk(x.to(DEV), k, T, uniform=uni, kept_out=kept, probs_out=probs)
    torch.cuda.synchronize()
    return kept.cpu().tolist(), probs.float().cpu(), int(tok.item())


CASES = [(32000, 200, False), (32000, 200, True), (32000, 1, False), (32000, 1024, True), (50304, 200, True),
         (1000, 1000, False), (7, 200, True), (65536, 64, True), (32000, 200, "peaked"), (50304, 100, "peaked"),
         (32000, 50, "ninf"), (3000, 7, "ninf")]


@pytest.mark.parametrize("n,k,ties", CASES)
@pytest.mark.parametrize("T", [0.8, 1.7])
def test_sampler_matches_oracle(ops, n, k, ties, T):
    x = _logits(n, n * 7 + k, ties)
    for u in (0.013, 0.37, 0.5, 0.93, 0.9999):
        kept, p, tok = _draw(ops, x, k, T, u)
        ref_kept, ref_p, ref_tok = om.sample_topk_spec(x, k, T, u)
        assert kept == ref_kept  # bit-exact kept set, in index order
        assert torch.allclose(p, ref_p, rtol=2 ** -7, atol=0)  # one bf16 ulp
        assert tok == kept[om.inverse_cdf(p.numpy(), u)]  # the inverse CDF of the kernel's own probabilities
        cdf = np.cumsum(ref_p.numpy(), dtype=np.float32) / ref_p.sum().item()
        if np.min(np.abs(cdf - u)) > 1e-3:
            assert tok == ref_tok
    # the kept values are torch.topk's on the device
    v, _ = torch.topk(x.to(DEV), min(k, n))
    assert sorted(x[kept].float().tolist()) == sorted(v.float().cpu().tolist())


def test_sampler_rejects_bad_arguments(ops):
    x = _logits(100, 1).to(DEV)
    c = torch.zeros(1, dtype=torch.int64, device=DEV)
    with pytest.raises(ValueError):
        ops.sample_topk(x, 0, 0.8, counter=c)
    with pytest.raises(ValueError):
        ops.sample_topk(x, 2000, 0.8, counter=c)
    with pytest.raises(RuntimeError):
        ops.sample_topk(x, 10, 0.0, counter=c)
    with pytest.raises(RuntimeError):
        ops.sample_topk(_logits(70000, 1).to(DEV), 10, 0.8, counter=c)


def test_sampler_bookkeeping_and_embedding(ops):
    n, C = 32000, 4096
    x = _logits(n, 5).to(DEV)
    table = (torch.randn(n, C, generator=torch.Generator().manual_seed(2)) * 0.02).bfloat16().to(DEV)
    emb = torch.empty(C, dtype=torch.bfloat16, device=DEV)
    tok = torch.zeros(1, dtype=torch.int32, device=DEV)
    pos = torch.tensor([41], device=DEV)
    uni = torch.tensor([0.6], dtype=torch.float32, device=DEV)
    idx = ops.sample_topk(x, 200, 0.8, uniform=uni, token_out=tok, pos_inout=pos, table=table, emb_out=emb)
    t = int(idx.item())
    assert tok.item() == t and pos.item() == 42
    assert torch.equal(emb, table[t])


def test_counter_rng_follows_the_distribution_and_replays_in_a_graph(ops):
    # 8 kept logits with known probabilities; 4000 counter-driven draws
    x = torch.full((1000,), -30.0)
    vals = torch.tensor([2.0, 1.5, 1.0, 0.5, 0.0, -0.5, -1.0, -1.5])
    where = torch.tensor([900, 3, 500, 77, 78, 10, 999, 0])
    x[where] = vals
    x = x.bfloat16().to(DEV)
    _, p, _ = om.sample_topk_spec(x.cpu(), 8, 1.0, 0.5)
    kept = sorted(where.tolist())
    counter = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = torch.zeros(4000, dtype=torch.int64, device=DEV)
    for i in range(4000):
        ops.sample_topk(x, 8, 1.0, seed=1234, counter=counter, out_idx=out[i:i + 1])
    assert counter.item() == 4000
    got = out.cpu()
    freq = torch.tensor([(got == j).sum().item() for j in kept], dtype=torch.float64) / 4000
    sd = torch.sqrt(p.double() * (1 - p.double()) / 4000)
    assert torch.all((freq - p.double()).abs() < 5 * sd + 1e-3), (freq, p)
    # graph capture: replays continue the same counter sequence as the eager calls
    c2 = torch.zeros(1, dtype=torch.int64, device=DEV)
    o2 = torch.zeros(1, dtype=torch.int64, device=DEV)
    g = torch.cuda.CUDAGraph()
    ops.sample_topk(x, 8, 1.0, seed=1234, counter=c2, out_idx=o2)  # warm (counter 0 -> 1)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        ops.sample_topk(x, 8, 1.0, seed=1234, counter=c2, out_idx=o2)
    c2.fill_(0)
    seq = []
    for _ in range(50):
        g.replay()
        seq.append(int(o2.item()))
    assert c2.item() == 50
    assert seq == got[:50].tolist()
    # another seed, another sequence
    c3 = torch.zeros(1, dtype=torch.int64, device=DEV)
    o3 = torch.zeros(50, dtype=torch.int64, device=DEV)
    for i in range(50):
        ops.sample_topk(x, 8, 1.0, seed=99, counter=c3, out_idx=o3[i:i + 1])
    assert o3.cpu().tolist() != seq


@pytest.mark.parametrize("quantize", [None, "bnb.nf4"])
def test_sampled_decode_graph_equals_eager(quantize):
    """generate(temperature 0.8, top_k 200): the captured decode graph (and its 8-step chunks) draws the same tokens
    as the eager per-step loop for the same seed; every token is inside the step's top-200."""
    from generate.base import build_model, generate
    from lit_gpt import Config

    cfg = (Config.from_name("pythia-160m", n_layer=2) if quantize is None else
           Config.from_name("Llama-2-7b-hf", n_layer=2, n_embd=1024, n_head=8, n_query_groups=8,
                            intermediate_size=2816))
    model = build_model(cfg, quantize=quantize, device=torch.device(DEV), max_seq_length=64)
    prompt = torch.randint(0, cfg.vocab_size, (9,), generator=torch.Generator().manual_seed(0)).to(DEV)
    outs = []
    for use_graph in (True, False):
        torch.manual_seed(1234)
        for b in model.transformer.h:
            b.attn.kv_cache.reset_parameters()
        outs.append(generate(model, prompt, 9 + 30, temperature=0.8, top_k=200, use_graph=use_graph).cpu())
    assert torch.equal(outs[0], outs[1])
    assert outs[0].numel() == 39
    torch.manual_seed(7)
    for b in model.transformer.h:
        b.attn.kv_cache.reset_parameters()
    other = generate(model, prompt, 9 + 30, temperature=0.8, top_k=200).cpu()
    assert not torch.equal(other, outs[0])
