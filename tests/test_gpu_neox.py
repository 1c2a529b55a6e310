"""BASELINE config 1 on the MI355X: pythia-160m (GPT-NeoX blocks — LayerNorm with bias, partial rotary 16 of 64
dims, parallel residual, biased Linears, exact-erf GELU MLP; reference lit_gpt/model.py:572-593, 691-702) through
the product's GPT.forward / generate, against

* the reference's own fp32 greedy run (tests/golden/g1_pythia160m_greedy.npz, made by importing /root/reference:
  tokens, step-0 logits, per-step margins), and
* the oracle (CPU restatement of the reference) on the same synthetic weights in bf16 and float64, with the bounds
  of tests/parity.py.

The product has no CPU path, so config 1 runs on the GPU in bf16 (the reference's CPU plumbing run is fp32): the
bound is "as accurate as the reference's own bf16 execution", and the greedy tokens must equal the fp32 reference's
wherever its top-1/top-2 margin clears the bf16 error.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import model as om
from oracle import quant, synth
from parity import check_step, rel_err

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _pythia(mode="bf16", max_seq=16 + 128):
    """mode: "bf16" (bf16-true), "fp32" (32-true, the reference's config-1 precision) or a 4-bit quantize mode."""
    from lit_gpt import GPT, Config
    from lit_gpt.quantize import QuantizedPrecision

    cfg = Config.from_name("pythia-160m")
    sd = synth.state_dict(cfg, seed=1234)
    model = GPT(cfg)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    dt = torch.float32 if mode == "fp32" else torch.bfloat16
    model = model.to(device=DEV, dtype=dt)
    if mode not in ("bf16", "fp32"):
        QuantizedPrecision(mode).convert_module(model, DEV)
    model.max_seq_length = max_seq
    model.set_kv_cache(1, device=DEV, dtype=dt)
    return cfg, sd, model.eval()


def _oracles(cfg, sd, mode):
    def deq(k, v):
        if k.endswith(".weight") and v.ndim == 2 and not k.startswith("transformer.wte"):
            vb = quant.bf16_bits_to_f32(quant.f32_to_bf16_bits(v))
            return vb if mode == "bf16" else quant.dequantize_q4g(*quant.quantize_q4g(vb, 128), 128)
        return quant.bf16_bits_to_f32(quant.f32_to_bf16_bits(v)) if v.dtype == np.float32 else v

    return {dt: om.OracleGPT(cfg, sd, dtype=dt, weight_override=deq) for dt in (torch.bfloat16, torch.float64)}


@pytest.mark.parametrize("mode", ["bf16", "int4-g128"])
@torch.inference_mode()
def test_pythia160m_teacher_forced_on_reference_tokens(golden, mode):
    """Prefill the fixture's 16-token prompt, then decode teacher-forced on the reference's greedy tokens; every
    48th-or-so step (and the first 8) checked against the bf16 / float64 oracles; step 0 also against the fixture."""
    g = golden("g1_pythia160m_greedy.npz")
    cfg, sd, model = _pythia(mode)
    toks = torch.from_numpy(g["tokens"]).long()
    T = 16
    steps = list(range(8)) + list(range(8, 128, 13))
    got = {0: model(toks[:T].view(1, -1).to(DEV), torch.arange(T, device=DEV))[0, -1].float().cpu()}
    for i in range(1, 128):
        lg = model(toks[T + i - 1:T + i].view(1, 1).to(DEV), torch.tensor([T + i - 1], device=DEV))[0, -1]
        if i in steps:
            got[i] = lg.float().cpu()
    refs = {}
    for dt, ref in _oracles(cfg, sd, mode).items():
        ref.set_kv_cache(T + 128)
        out = {0: ref.forward(toks[:T], torch.arange(T))[-1]}
        for i in range(1, 128):
            lg = ref.forward(toks[T + i - 1:T + i], torch.tensor([T + i - 1]))[-1]
            if i in steps:
                out[i] = lg
        refs[dt] = out
    for i in steps:
        check_step(got[i], refs[torch.bfloat16][i], refs[torch.float64][i], f"pythia {mode} step {i}")
    if mode == "bf16":
        # the reference's own fp32 logits at step 0 (fixture): within the bf16 path's distance to exact arithmetic
        mx, rms, _ = rel_err(got[0], g["step0_logits"])
        fmx, frms, _ = rel_err(refs[torch.bfloat16][0], g["step0_logits"])
        assert mx <= 1.25 * fmx + 0.0025 and rms <= 1.25 * frms + 0.0025, (mx, rms, fmx, frms)


@torch.inference_mode()
def test_pythia160m_greedy_generate_follows_reference():
    """generate/base.py's loop (prefill + HIP-graph decode) on config 1: the 128 greedy tokens equal the fp32
    reference's (fixture) at every step whose reference margin exceeds the bf16 error bound — until the first step
    where the reference's own margin is within it (after that the two greedy streams may legitimately fork)."""
    from generate.base import generate

    g = np.load(__import__("pathlib").Path(__file__).parent / "golden" / "g1_pythia160m_greedy.npz")
    cfg, sd, model = _pythia("bf16")
    prompt = torch.from_numpy(g["prompt"]).to(DEV)
    y = generate(model, prompt, 16 + 128, temperature=0.0).cpu().numpy()
    ref, margins, absmax = g["tokens"], g["margins"], g["logits_absmax"]
    checked = 0
    for i in range(128):
        if margins[i] <= 0.03 * absmax[i]:
            break
        assert y[16 + i] == ref[16 + i], f"step {i}: {y[16 + i]} vs reference {ref[16 + i]}"
        checked += 1
    assert checked >= 4, checked


FP32_TOL = 2e-5  # relative to max |logit|: fp32 summation-order differences over 12 blocks (measured ~1e-6)


@torch.inference_mode()
def test_pythia160m_fp32_step0_logits_match_reference_fixture(golden):
    """BASELINE config 1 in its own precision (--precision 32-true, csrc/fp32.hip): the prefill's last-row logits
    equal the reference's fp32 logits (fixture g1, generated by importing /root/reference) to fp32 summation-order
    noise — no bf16 rounding anywhere on the path."""
    g = golden("g1_pythia160m_greedy.npz")
    cfg, sd, model = _pythia("fp32")
    prompt = torch.from_numpy(g["prompt"]).long().view(1, -1).to(DEV)
    lg = model(prompt, torch.arange(prompt.shape[1], device=DEV))[0, -1].cpu()
    assert lg.dtype == torch.float32
    ref = torch.from_numpy(g["step0_logits"]).float()
    err = float((lg - ref).abs().max() / ref.abs().max())
    assert err <= FP32_TOL, err


@torch.inference_mode()
def test_pythia160m_fp32_greedy_128_tokens_equal_reference():
    """generate/base.py's loop in fp32 (prefill + HIP-graph decode, fp32 argmax on the device): the 128 greedy
    tokens equal the reference's fp32 run (fixture) at every step up to the first whose reference top-1/top-2 margin
    is within the fp32 noise bound (after which two correct fp32 executions may legitimately fork)."""
    from generate.base import generate

    g = np.load(__import__("pathlib").Path(__file__).parent / "golden" / "g1_pythia160m_greedy.npz")
    cfg, sd, model = _pythia("fp32")
    prompt = torch.from_numpy(g["prompt"]).to(DEV)
    y = generate(model, prompt, 16 + 128, temperature=0.0).cpu().numpy()
    ref, margins, absmax = g["tokens"], g["margins"], g["logits_absmax"]
    checked = 0
    for i in range(128):
        if margins[i] <= 4 * FP32_TOL * absmax[i]:
            break
        assert y[16 + i] == ref[16 + i], f"step {i}: {y[16 + i]} vs reference {ref[16 + i]}"
        checked += 1
    assert checked >= 64, checked
    print(f"fp32: {checked} of 128 greedy tokens checked against the reference's fp32 run")
