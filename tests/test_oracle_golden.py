"""Pin the CPU oracle against golden vectors produced by the reference itself (tests/golden/make_golden.py)."""

import numpy as np
import pytest
import torch

from oracle import model as om
from oracle import quant, synth
from oracle.tp import shard_linear


def _cfg(name, **kw):
    from lit_gpt.config import Config

    return Config.from_name(name, **kw)


TINY = {
    "llama_mha": ("Llama-2-7b-hf", dict(n_layer=2, n_embd=256, n_head=4, intermediate_size=640, vocab_size=1000,
                                         padding_multiple=64, block_size=256)),
    "llama_gqa": ("Llama-2-70b-hf", dict(n_layer=2, n_embd=256, n_head=4, n_query_groups=2, intermediate_size=512,
                                          vocab_size=1000, padding_multiple=64, block_size=256)),
    "llama_mqa": ("Llama-2-7b-hf", dict(n_layer=2, n_embd=256, n_head=4, n_query_groups=1, intermediate_size=384,
                                         vocab_size=1000, padding_multiple=64, block_size=256)),
    "mixtral": ("Mixtral-8x7B-v0.1", dict(n_layer=2, n_embd=256, n_head=4, n_query_groups=2, intermediate_size=384,
                                           n_expert=4, n_expert_per_token=2, padded_vocab_size=1024, vocab_size=1024,
                                           block_size=256)),
}


def teacher_forced(m, prompt, steps):
    T = prompt.numel()
    logits = [m.forward(prompt, torch.arange(T))[-1]]
    tok = torch.argmax(logits[-1]).view(1).to(prompt.dtype)
    toks = [tok]
    for s in range(steps - 1):
        logits.append(m.forward(tok, torch.tensor([T + s]))[-1])
        tok = torch.argmax(logits[-1]).view(1).to(prompt.dtype)
        toks.append(tok)
    return torch.cat(toks), torch.stack(logits).float()


def _quant_override(fmt):
    def f(k, v):
        if k.endswith(".weight") and v.ndim == 2 and not k.startswith("transformer.wte"):
            if fmt == "q4g":
                return quant.dequantize_q4g(*quant.quantize_q4g(v, 128), 128)
            return quant.dequantize_nf4(*quant.quantize_nf4(v, 64), 64)
        return v

    return f


@pytest.mark.parametrize("key", list(TINY))
def test_tiny_models_fp32_match_reference(key, golden):
    g = golden("g2_tiny_models.npz")
    name, kw = TINY[key]
    cfg = _cfg(name, **kw)
    sd = synth.state_dict(cfg, seed=7)
    prompt = torch.from_numpy(g[f"{key}_prompt"])
    np.testing.assert_array_equal(prompt.numpy(), synth.token_ids(24, cfg.vocab_size, seed=7))
    m = om.OracleGPT(cfg, sd)
    m.set_kv_cache(24 + 16)
    toks, logits = teacher_forced(m, prompt, 16)
    np.testing.assert_array_equal(toks.numpy(), g[f"{key}_fp32_tokens"])
    np.testing.assert_allclose(logits.numpy(), g[f"{key}_fp32_logits"], rtol=0, atol=2e-5)
    # no-cache path (input_pos=None)
    full = torch.cat([prompt, toks[:-1]])
    m2 = om.OracleGPT(cfg, sd)
    np.testing.assert_allclose(m2.forward(full).numpy(), g[f"{key}_nocache_logits"], rtol=0, atol=2e-5)


@pytest.mark.parametrize("fmt", ["q4g", "nf4"])
def test_tiny_llama_quantized_weights_match_reference(fmt, golden):
    g = golden("g2_tiny_models.npz")
    name, kw = TINY["llama_mha"]
    cfg = _cfg(name, **kw)
    m = om.OracleGPT(cfg, synth.state_dict(cfg, seed=7), weight_override=_quant_override(fmt))
    m.set_kv_cache(40)
    toks, logits = teacher_forced(m, torch.from_numpy(g["llama_mha_prompt"]), 16)
    np.testing.assert_array_equal(toks.numpy(), g[f"llama_mha_{fmt}_tokens"])
    np.testing.assert_allclose(logits.numpy(), g[f"llama_mha_{fmt}_logits"], rtol=0, atol=2e-5)


@pytest.mark.parametrize("key", ["llama_mha", "llama_gqa", "mixtral"])
def test_tiny_models_bf16_close_to_reference(key, golden):
    """bf16-true: the oracle mirrors the reference's cast points; CPU bf16 kernels may round differently."""
    g = golden("g2_tiny_models.npz")
    name, kw = TINY[key]
    cfg = _cfg(name, **kw)
    m = om.OracleGPT(cfg, synth.state_dict(cfg, seed=7), dtype=torch.bfloat16)
    m.set_kv_cache(40)
    prompt = torch.from_numpy(g[f"{key}_prompt"])
    # teacher-force the reference's bf16 token stream so a single flipped argmax cannot cascade
    ref_toks = torch.from_numpy(g[f"{key}_bf16_tokens"])
    T = prompt.numel()
    logits = [m.forward(prompt, torch.arange(T))[-1].float()]
    for s in range(15):
        logits.append(m.forward(ref_toks[s:s + 1], torch.tensor([T + s]))[-1].float())
    logits = torch.stack(logits).numpy()
    ref = g[f"{key}_bf16_logits"]
    scale = np.abs(ref).max()
    assert np.abs(logits - ref).max() <= 0.05 * scale


def test_pythia160m_greedy_128_matches_reference(golden):
    """BASELINE config 1: pythia-160m fp32, random init, 16-token prompt, greedy 128 tokens."""
    g = golden("g1_pythia160m_greedy.npz")
    cfg = _cfg("pythia-160m")
    prompt = torch.from_numpy(synth.token_ids(16, cfg.vocab_size, seed=1234))
    np.testing.assert_array_equal(prompt.numpy(), g["prompt"])
    m = om.OracleGPT(cfg, synth.state_dict(cfg, seed=1234))
    m.set_kv_cache(16 + 128)
    rec = []
    y = om.generate(m, prompt, 16 + 128, temperature=0.0, record_logits=rec)
    np.testing.assert_array_equal(y.numpy(), g["tokens"])
    np.testing.assert_allclose(rec[0].numpy(), g["step0_logits"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(torch.stack(rec).sum(-1).numpy(), g["logits_sum"], rtol=1e-4, atol=1e-2)


def test_rope_cache_and_apply(golden):
    g = golden("g3_ops.npz")
    for pos_dtype, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
        cos, sin = om.build_rope_cache(2304, 128, 10000, 1, pos_dtype)
        np.testing.assert_allclose(cos[2040:2050].numpy(), g[f"rope_cos_{tag}"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(sin[2040:2050].numpy(), g[f"rope_sin_{tag}"], rtol=0, atol=1e-6)
    # the bf16 default-dtype quirk rounds positions > 256 — the two caches must differ there
    assert not np.allclose(g["rope_cos_f32"], g["rope_cos_bf16"])
    cos, sin = om.build_rope_cache(64, 16, 1000000, 2)
    np.testing.assert_allclose(cos.numpy(), g["rope_small_cos"], rtol=0, atol=1e-6)
    y = om.apply_rope(torch.from_numpy(g["rope_x"]), cos, sin)
    np.testing.assert_allclose(y.numpy(), g["rope_y"], rtol=0, atol=1e-5)


def test_rope_long_context_rows_match_reference(golden):
    """The oracle's rope tables at 4k-32k positions (config 5's 32k context, rope_base 1e6; Llama-2's 1e4) against the
    reference's own build_rope_cache (tests/golden/make_golden_rope.py), under an fp32 and a bf16 default dtype — the
    bf16 position rounding that the 8k / 32k Mixtral prefill tests depend on."""
    g = golden("g5_rope_long.npz")
    rows = g["rows"]
    for base in (10000, 1000000):
        for pos_dtype, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
            cos, sin = om.build_rope_cache(32768, 128, base, 1, pos_dtype)
            np.testing.assert_allclose(cos[rows].numpy(), g[f"cos_{base}_{tag}"], rtol=0, atol=1e-6)
            np.testing.assert_allclose(sin[rows].numpy(), g[f"sin_{base}_{tag}"], rtol=0, atol=1e-6)
        assert not np.allclose(g[f"cos_{base}_f32"], g[f"cos_{base}_bf16"])


def test_rmsnorm(golden):
    g = golden("g3_ops.npz")
    x, w = torch.from_numpy(g["rms_x"]), torch.from_numpy(g["rms_w"])
    np.testing.assert_allclose(om.rms_norm(x, w, 1e-5).numpy(), g["rms_y"], rtol=0, atol=1e-6)
    yb = om.rms_norm(x.bfloat16(), w.bfloat16(), 1e-5).float().numpy()
    np.testing.assert_array_equal(yb, g["rms_y_bf16"])


def test_sample_known_answers(golden):
    g = golden("g3_ops.npz")
    logits = torch.from_numpy(g["sample_logits"])
    assert om.sample(logits[0], temperature=0.0).tolist() == g["sample_t0"].tolist() == [0]
    tl = torch.from_numpy(g["sample_ties_logits"])[0]
    assert om.sample(tl, temperature=0.0).tolist() == g["sample_ties_t0"].tolist()
    assert om.sample(tl, temperature=0.0, top_k=2).tolist() == g["sample_ties_t0_k2"].tolist()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_tp_shards_match_reference(world, golden):
    g = golden("g4_tp.npz")
    w = np.arange(24 * 16, dtype=np.float32).reshape(24, 16)
    b = np.arange(24, dtype=np.float32)
    for rank in range(world):
        for style in ("colwise", "rowwise"):
            key = f"w{world}_r{rank}_{style}"
            if f"{key}_error" in g:
                with pytest.raises(ValueError):
                    shard_linear(w, b, style, world, rank)
                continue
            ws, bs = shard_linear(w, b, style, world, rank)
            np.testing.assert_array_equal(ws, g[f"{key}_weight"])
            np.testing.assert_array_equal(bs, g[f"{key}_bias"])


def test_quant_formats_roundtrip():
    w = synth.normal((64, 256), "qw", 3, 0.02)
    p, s = quant.quantize_q4g(w, 128)
    assert p.shape == (64, 128) and p.dtype == np.uint8 and s.shape == (64, 2)
    d = quant.dequantize_q4g(p, s, 128)
    scale = quant.bf16_bits_to_f32(s)
    assert np.all(np.abs(d - w).reshape(64, 2, 128) <= scale[..., None] * 0.5 * 1.01 + 1e-12)
    p2, s2 = quant.quantize_q4g(d, 128)  # idempotent on its own output
    np.testing.assert_array_equal(quant.dequantize_q4g(p2, s2, 128), d)
    pn, a = quant.quantize_nf4(w, 64)
    dn = quant.dequantize_nf4(pn, a, 64)
    assert np.abs(dn - w).max() <= a.max() * 0.2
    np.testing.assert_array_equal(quant.dequantize_nf4(*quant.quantize_nf4(dn, 64), 64), dn)


def test_synth_is_deterministic():
    a = synth.normal((1000,), "x", 1)
    b = synth.normal((1000,), "x", 1)
    np.testing.assert_array_equal(a, b)
    assert abs(a.std() - 0.02) < 0.002 and abs(a.mean()) < 0.002
    assert not np.array_equal(a, synth.normal((1000,), "y", 1))


@pytest.mark.parametrize("fam", ["llama", "mixtral", "neox"])
@pytest.mark.parametrize("world", [2, 4])
def test_reference_tp_logits_equal_unsharded_oracle(fam, world, golden):
    """G4: the reference's own tensor_parallel under gloo TP=2/4 (tests/golden/make_golden_tp.py)
    computes what the unsharded oracle computes: same greedy tokens, logits within fp32 reordering of the
    row-parallel sums; and with per-shard int4 weights, what the oracle computes on those assembled shards."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).parent / "golden"))
    from make_golden_tp import FAMILIES, STEPS, T, fit_group

    g = golden("g4_tp_logits.npz")
    name, kw = FAMILIES[fam]
    cfg = _cfg(name, **kw)
    sd = synth.state_dict(cfg, seed=17)
    prompt = torch.from_numpy(g[f"{fam}_prompt"])
    ref = g[f"{fam}_w{world}_fp32_float32_logits"]
    toks = g[f"{fam}_w{world}_fp32_float32_tokens"]
    m = om.OracleGPT(cfg, sd)
    m.set_kv_cache(T + STEPS + 1)
    got = [m.forward(prompt, torch.arange(T))[-1]]
    for s in range(STEPS):
        got.append(m.forward(torch.tensor([int(toks[s])]), torch.tensor([T + s]))[-1])
    got = torch.stack(got).float().numpy()
    assert np.abs(got - ref).max() <= 1e-4 * np.abs(ref).max()
    assert np.array_equal(got.argmax(-1), toks)

    # int4 per shard: colwise shards (dim 0) keep the unsharded groups; rowwise shards (dim 1) are quantized with
    # the group that fits the shard's width, i.e. the unsharded matrix quantized with that group
    def deq(k, v):
        if not (k.endswith(".weight") and v.ndim == 2) or k.startswith("transformer.wte"):
            return v
        rowwise = k.endswith("attn.proj.weight") or (k.endswith("proj.weight") and ".mlp" in k)
        gsz = fit_group(v.shape[1] // world if rowwise else v.shape[1])
        return quant.dequantize_q4g(*quant.quantize_q4g(v, gsz), gsz)

    mq = om.OracleGPT(cfg, sd, weight_override=deq)
    mq.set_kv_cache(T + STEPS + 1)
    ref_q = g[f"{fam}_w{world}_q4g_bfloat16_logits"]
    toks_q = g[f"{fam}_w{world}_q4g_bfloat16_tokens"]
    got_q = [mq.forward(prompt, torch.arange(T))[-1]]
    for s in range(STEPS):
        got_q.append(mq.forward(torch.tensor([int(toks_q[s])]), torch.tensor([T + s]))[-1])
    got_q = torch.stack(got_q).float().numpy()
    # reference side ran in bf16: bf16 activation rounding vs the fp32 oracle
    assert np.abs(got_q - ref_q).max() <= 0.03 * np.abs(ref_q).max()


@pytest.mark.parametrize("name,kw", [("Llama-2-7b-hf", dict(n_embd=128, n_head=8, n_query_groups=2,
                                                             intermediate_size=256)),
                                     ("Mixtral-8x7B-v0.1", dict(n_embd=128, n_head=8, n_query_groups=2,
                                                                intermediate_size=96))])
def test_one_block_rows_equal_full_forward(name, kw):
    """oracle.one_block_rows (linear-cost rows of a one-block forward, used for the 32k-prompt prefill parity) ==
    OracleGPT.forward's rows, exactly, in float64 — the full causal forward is the reference restatement."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "lit-gpt_amd"))
    from lit_gpt import Config

    cfg = Config.from_name(name, n_layer=1, vocab_size=256, padded_vocab_size=256, **kw)
    og = om.OracleGPT(cfg, synth.state_dict(cfg, seed=4), dtype=torch.float64)
    T = 70
    idx = torch.from_numpy(synth.token_ids(T, cfg.vocab_size, seed=4))
    full = og.forward(idx)
    rows = [0, 1, 33, T - 2, T - 1]
    gaps = []
    got = om.one_block_rows(og, idx, rows, router_gaps=gaps)
    assert torch.allclose(got, full[rows], rtol=1e-12, atol=1e-12)
    assert len(gaps) == (len(rows) if cfg._mlp_class == "LLaMAMoE" else 0) and all(g >= 0 for g in gaps)
