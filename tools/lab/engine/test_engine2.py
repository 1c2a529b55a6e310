"""LAB (not collected by the product suite): the persistent decode engine VERSION 2 (lga_decode_engine of
tools/lab/engine/engine2.hip) against the per-op kernels and the oracle.
Run: python -m pytest tools/lab/engine/test_engine2.py -m gpu

The engine runs a whole greedy decode step (every block + ln_f + lm_head + argmax; reference generate/base.py:44-47,
lit_gpt/model.py:499-519) as ONE launch. Its GEMVs reproduce the per-op kernels' arithmetic (same chunk mapping,
x staging, RMSNorm order, butterflies and epilogues), so every GEMV output is compared BIT-EXACTLY with lga_q4_gemv /
lga_q4_gemv_swiglu fed the engine's own input vector (op_limit stops the launch after that op and leaves the
per-layer activations in the scratch). The attention merges its key splits in a different order than
lga_attention_decode_fused: compared within 2 bf16 ulps. End to end, the engine's greedy tokens and logits are
checked against the oracle (tests/parity.py bounds) and against the per-op HIP-graph decode.

Geometry: Llama-2-7B width (C 4096, 32 heads, I 11008, V 32000), two blocks, int4-g128 (BASELINE config 3).
"""

from __future__ import annotations

import math
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

_HERE = Path(__file__).resolve().parent
sys.path[:0] = [str(_HERE), str(_HERE.parents[2] / "tests"), str(_HERE.parents[2] / "lit-gpt_amd"),
                str(_HERE.parents[2])]
from oracle import synth  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _model(T, extra=40, seed=5, n_layer=2):
    from generate.base import build_model
    from lit_gpt import Config

    cfg = Config.from_name("Llama-2-7b-hf", n_layer=n_layer)
    model = build_model(cfg, quantize="int4-g128", device=DEV, seed=seed, max_seq_length=T + extra)
    prompt = torch.from_numpy(synth.token_ids(T, cfg.vocab_size, seed=seed)).to(DEV)
    lg = model(prompt.view(1, -1), torch.arange(T, device=DEV), last_token_only=True)
    first = int(torch.argmax(lg[0, -1].float()))
    return model, cfg, first


def _ulps_close(a: torch.Tensor, b: torch.Tensor, ulps: int = 2) -> bool:
    a, b = a.float(), b.float()
    tol = ulps * torch.maximum(a.abs(), b.abs()) * 2 ** -8 + 1e-6
    return bool(((a - b).abs() <= tol).all())


@pytest.mark.timeout(300)
@pytest.mark.parametrize("T", [300, 2048])
@torch.inference_mode()
def test_engine_ops_match_per_op_kernels(T):
    from lit_gpt import ops
    from engine2 import DecodeEngine

    model, cfg, first = _model(T)
    eng = DecodeEngine(model)
    emb = ops.embedding(torch.tensor([first], device=DEV, dtype=torch.int32), model.transformer.wte.weight).view(-1)
    kv0 = [(b.attn.kv_cache.k.clone(), b.attn.kv_cache.v.clone()) for b in model.transformer.h]

    def restore():
        for b, (k, v) in zip(model.transformer.h, kv0):
            b.attn.kv_cache.k.copy_(k)
            b.attn.kv_cache.v.copy_(v)

    def run(limit):
        restore()
        eng.reset()
        eng.set_embedding(emb)
        pos = torch.tensor([T], device=DEV)
        eng.step(pos, op_limit=limit)
        torch.cuda.synchronize()
        assert eng.errors() == 0
        return pos

    cos, sin = model._rope_tables()
    H, G, hs = cfg.n_head, cfg.n_query_groups, cfg.head_size
    for l, blk in enumerate(model.transformer.h):
        a, m = blk.attn, blk.mlp
        k0 = 5 * l
        # 1. RMSNorm + qkv GEMV on the engine's block input x_l
        run(k0 + 1)
        xl = eng.buffer("x", l).clone()
        qkv = eng.buffer("qkv", l).clone()
        ref = ops.q4_gemv(xl, a.attn.qweight, a.attn.scales, a.attn.out_features, cfg.n_embd, a.attn.group,
                          a.attn.fmt, norm_weight=blk.norm_1.weight, eps=blk.norm_1.eps)
        assert torch.equal(qkv, ref), f"layer {l}: qkv GEMV differs from lga_q4_gemv"
        # 2. RoPE + KV append + attention (the per-op fused kernel on the engine's qkv, same caches)
        run(k0 + 2)
        y = eng.buffer("y", l).clone()
        k_eng, v_eng = a.kv_cache.k.clone(), a.kv_cache.v.clone()
        restore()
        p = torch.tensor([T], device=DEV)
        splits = ops.decode_splits(G, H // G, hs, a.kv_cache.k.size(-2))
        y_ref = ops.attention_decode_fused(qkv.view(1, -1), a.kv_cache.k, a.kv_cache.v, p, p, cos, sin, H, G, hs, hs,
                                           1.0 / math.sqrt(hs), splits)
        assert torch.equal(k_eng, a.kv_cache.k) and torch.equal(v_eng, a.kv_cache.v), f"layer {l}: KV append differs"
        assert _ulps_close(y, y_ref.view(-1)), (l, (y.float() - y_ref.view(-1).float()).abs().max())
        # 3. o_proj + residual on the engine's attention output
        run(k0 + 3)
        xp = eng.buffer("xp", l).clone()
        ref = ops.q4_gemv(eng.buffer("y", l), a.proj.qweight, a.proj.scales, cfg.n_embd, cfg.n_embd, a.proj.group,
                          a.proj.fmt, residual=xl)
        assert torch.equal(xp, ref), f"layer {l}: o_proj GEMV differs"
        # 4. RMSNorm + fc_1 || fc_2 + SwiGLU
        run(k0 + 4)
        g = eng.buffer("g", l).clone()
        ref = ops.q4_gemv_swiglu(eng.buffer("xp", l), m.fc_1.qweight, m.fc_1.scales, m.fc_2.qweight,
                                 m.fc_2.scales, cfg.intermediate_size, cfg.n_embd, m.fc_1.group, m.fc_1.fmt,
                                 norm_weight=blk.norm_2.weight, eps=blk.norm_2.eps)
        assert torch.equal(g, ref), f"layer {l}: fc_1/fc_2 SwiGLU GEMV differs"
        # 5. mlp.proj + residual
        run(k0 + 5)
        x1 = eng.buffer("x", l + 1).clone()
        ref = ops.q4_gemv(eng.buffer("g", l), m.proj.qweight, m.proj.scales, cfg.n_embd, cfg.intermediate_size,
                          m.proj.group, m.proj.fmt, residual=eng.buffer("xp", l))
        assert torch.equal(x1, ref), f"layer {l}: mlp.proj GEMV differs"
    # 6. the whole step: ln_f + lm_head bit-exact on the engine's last activation, argmax, pos, next embedding
    tok = torch.zeros(1, dtype=torch.int32, device=DEV)
    restore()
    eng.reset()
    eng.set_embedding(emb)
    pos = torch.tensor([T], device=DEV)
    eng.step(pos, token=tok)
    torch.cuda.synchronize()
    assert eng.errors() == 0
    lm = model.lm_head
    ref = ops.q4_gemv(eng.buffer("x", cfg.n_layer), lm.qweight, lm.scales, lm.out_features, cfg.n_embd, lm.group,
                      lm.fmt, norm_weight=model.transformer.ln_f.weight, eps=model.transformer.ln_f.eps)
    assert torch.equal(eng.logits, ref), "lm_head GEMV differs"
    assert int(tok) == int(ops.argmax(eng.logits)), "argmax differs"
    assert int(pos) == T + 1
    assert torch.equal(eng.x0, model.transformer.wte.weight[int(tok)]), "next-step embedding differs"


@pytest.mark.timeout(400)
@torch.inference_mode()
def test_engine_greedy_decode_matches_per_op_graph_and_oracle():
    """16 greedy steps after a 2048-token prefill: the engine (eager launches, then captured in a HIP graph) vs the
    per-op DecodeGraph — identical tokens up to the first step whose per-op top-2 margin is inside the logit
    tolerance, and every engine step's logits within the tests/parity.py bounds of the oracle."""
    from lit_gpt import ops
    from engine2 import DecodeEngine
    from lit_gpt.runtime import DecodeGraph
    from parity import check_step
    from oracle import model as om
    from test_gpu_geometry import oracle_state_from_model

    T, N = 2048, 16
    model, cfg, first = _model(T, extra=N + 4)
    kv0 = [(b.attn.kv_cache.k.clone(), b.attn.kv_cache.v.clone()) for b in model.transformer.h]
    # per-op path: captured decode graph, logits per step
    dg = DecodeGraph(model, torch.tensor([first], device=DEV), T)
    ref_toks = [int(dg.token)]
    for _ in range(N - 1):
        ref_toks.append(int(dg.step()))
    for b, (k, v) in zip(model.transformer.h, kv0):
        b.attn.kv_cache.k.copy_(k)
        b.attn.kv_cache.v.copy_(v)
    eng = DecodeEngine(model)
    eng.set_embedding(model.transformer.wte.weight[first])
    pos = torch.tensor([T], device=DEV)
    tok = torch.zeros(1, dtype=torch.int32, device=DEV)
    toks, logits = [], []
    for i in range(N):
        if i == 4:  # from here on through a captured graph (fixed pointers, device-side pos / epoch)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                eng.step(pos, token=tok)
        if i >= 4:
            g.replay()
        else:
            eng.step(pos, token=tok)
        torch.cuda.synchronize()
        toks.append(int(tok))
        logits.append(eng.logits.float().cpu())
    eng.check()
    assert int(pos) == T + N
    # tokens vs the per-op path while the margin is clear
    for i in range(N):
        lg = logits[i]
        top = torch.topk(lg, 2).values
        if float(top[0] - top[1]) <= 0.03 * float(lg.abs().max()):
            break
        assert toks[i] == ref_toks[i], (i, toks, ref_toks)
    # logits vs the oracle (teacher-forced on the engine's tokens)
    sd = oracle_state_from_model(model)
    prompt = torch.from_numpy(synth.token_ids(T, cfg.vocab_size, seed=5))
    exp = {}
    for dt in (torch.bfloat16, torch.float64):
        ref = om.OracleGPT(cfg, sd, dtype=dt, rope_pos_dtype=torch.bfloat16)
        ref.set_kv_cache(T + N + 4)
        ref.forward(prompt.long(), torch.arange(T), last_only=True)
        fed = [first] + toks[:-1]
        exp[dt] = [ref.forward(torch.tensor([t]), torch.tensor([T + i]))[-1].double() for i, t in enumerate(fed[:6])]
    for s in range(6):
        check_step(logits[s].numpy(), exp[torch.bfloat16][s].numpy(), exp[torch.float64][s].numpy(), f"engine step {s}")


@pytest.mark.timeout(120)
@torch.inference_mode()
def test_engine_declines_unsupported_models():
    from generate.base import build_model
    from lit_gpt import Config
    from engine2 import DecodeEngine

    cfg = Config.from_name("Llama-2-7b-hf", n_layer=1, n_embd=256, n_head=2, intermediate_size=640)
    model = build_model(cfg, quantize="int4-g128", device=DEV, max_seq_length=64)
    ok, why = DecodeEngine.supported(model)
    assert not ok and why
    with pytest.raises(NotImplementedError):
        DecodeEngine(model)
