"""A/B of the sparse-MoE prefill GEMM tiles: one full-width Mixtral-8x7B block (int4-g128), prefill of T tokens,
variants by LGA_GROUPED_BN (128: 256 x 128 tiles for > 512 routed rows, the round-4 choice; 256: 256 x 256), timed
with HIP events around the whole one-block forward (best of AB_ROUNDS, variants alternating).

usage: python tools/moe_prefill_ab.py [T ...]       (AB_ROUNDS=3)
"""

import os
import sys
import time
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]


@torch.inference_mode()
def main():
    from generate.base import build_model
    from lit_gpt import Config
    from oracle import synth

    Ts = [int(v) for v in sys.argv[1:]] or [8192]
    rounds = int(os.environ.get("AB_ROUNDS", "3"))
    dev = torch.device("cuda")
    cfg = Config.from_name("Mixtral-8x7B-v0.1", n_layer=1)
    model = build_model(cfg, quantize="int4-g128", device=dev, seed=11, max_seq_length=max(Ts) + 2)
    for T in Ts:
        prompt = torch.from_numpy(synth.token_ids(T, cfg.vocab_size, seed=11)).to(dev)
        res, outs = {}, {}
        for r in range(rounds):
            for bn in ("128", "256"):
                os.environ["LGA_GROUPED_BN"] = bn
                model.transformer.h[0].attn.kv_cache.reset_parameters()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                lg = model(prompt.view(1, -1), torch.arange(T, device=dev), last_token_only=True)
                e.record()
                e.synchronize()
                res.setdefault(bn, []).append(s.elapsed_time(e))
                outs[bn] = lg.float().cpu()
        same = torch.equal(outs["128"], outs["256"])
        print(f"T={T}: one Mixtral block prefill ms  bn128 {min(res['128']):.2f}  bn256 {min(res['256']):.2f}"
              f"  (logits bit-identical: {same})", flush=True)


if __name__ == "__main__":
    main()
