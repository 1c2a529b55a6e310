"""How far is the bf16 reference from exact arithmetic at Llama-2-7B geometry? (test-tolerance derivation)

Runs the oracle (CPU restatement of the reference forward) twice on the same dequantized int4-g128 weights of a
2-block Llama-2-7B (C 4096, I 11008, V 32000): once in float64 (exact-arithmetic stand-in) and once in bf16 (the
reference's ``--precision bf16-true`` rounding points), prefill T tokens then ``--steps`` decode steps, and prints
per step max|d|/max|logit| and rms(d)/rms(logit) of bf16 vs fp64. The GPU parity tests
(tests/test_gpu_geometry.py) bound the product's distance to the bf16 oracle by a multiple of this floor: two
independent bf16 computations of the same math land about sqrt(2) x floor apart.

    python tools/bf16_noise_floor.py --T 2048 --steps 3
"""

from __future__ import annotations

import argparse
import math
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "lit-gpt_amd")]

from lit_gpt import Config  # noqa: E402
from oracle import model as om  # noqa: E402
from oracle import quant, synth  # noqa: E402


def rel(a: torch.Tensor, b: torch.Tensor):
    d = (a.double() - b.double()).abs()
    return float(d.max() / b.double().abs().max()), float(d.pow(2).mean().sqrt() / b.double().pow(2).mean().sqrt())


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--mode", default="int4-g128", choices=["int4-g128", "bf16"])
    args = ap.parse_args()
    cfg = Config.from_name("Llama-2-7b-hf", n_layer=args.layers)
    sd = synth.state_dict(cfg, seed=7)

    def deq(k, v):
        v = quant.bf16_bits_to_f32(quant.f32_to_bf16_bits(v))
        if args.mode == "int4-g128" and k.endswith(".weight") and v.ndim == 2 and not k.startswith("transformer.wte"):
            return quant.dequantize_q4g(*quant.quantize_q4g(v, 128), 128)
        return v

    sd = {k: deq(k, v) for k, v in sd.items()}
    prompt = torch.from_numpy(synth.token_ids(args.T, cfg.vocab_size, seed=7)).long()
    runs, toks = {}, []
    for dt in (torch.float64, torch.bfloat16):
        t0 = time.time()
        m = om.OracleGPT(cfg, sd, dtype=dt, rope_pos_dtype=torch.bfloat16)
        m.set_kv_cache(args.T + args.steps + 1)
        out = [m.forward(prompt, torch.arange(args.T), last_only=True)[-1]]
        for i in range(args.steps):
            if dt == torch.float64:  # both runs are teacher-forced on the fp64 run's greedy tokens
                toks.append(int(torch.argmax(out[-1])))
            out.append(m.forward(torch.tensor([toks[i]]), torch.tensor([args.T + i]))[-1])
        runs[dt] = out
        print(f"{dt}: {time.time() - t0:.1f} s", flush=True)
    for i, (a, b) in enumerate(zip(runs[torch.bfloat16], runs[torch.float64])):
        mx, rms = rel(a, b)
        print(f"step {i}: bf16 vs fp64 max|d|/max = {mx:.3%}  rms(d)/rms = {rms:.3%}")


if __name__ == "__main__":
    main()
