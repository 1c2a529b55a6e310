"""Is the oracle a fair stand-in for the reference's CPU decode?  (bench.py ``cpu_baseline``, kind "port")

Times one decode step at context 2048 of a 2-block Llama-2-7B (full width: C 4096, 32 heads, I 11008, V 32000;
bf16 weights and activations, the reference's ``--precision bf16-true``) on this host's cores, twice on the same
weights and the same cached context:
  * the REFERENCE itself — /root/reference/lit_gpt/model.py imported with stubs for the absent Lightning package
    (tests/golden/make_golden.py import_reference), GPT.forward(idx, input_pos) as generate/base.py:84-92 calls it;
  * the oracle — oracle/model.py OracleGPT.forward, what bench.py times on the GPU box.
and prints both per-step times, their ratio, and the 32-block extrapolation (per block x 32 + lm_head) that
bench.py reports. Run here, in the container (the reference does not exist on the GPU box):

    python tools/cpu_baseline_check.py [--threads 8] [--steps 12]
"""

from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "tests" / "golden")]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--context", type=int, default=2048)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    import make_golden  # imports the reference lit_gpt with stubs (no Lightning here)

    config, model_mod, _, _ = make_golden.import_reference()
    from oracle import model as om
    from oracle import synth

    cfg = config.Config.from_name("Llama-2-7b-hf", n_layer=2)
    P, S = args.context, args.context + args.steps + 2
    g = torch.Generator().manual_seed(0)
    sd = {}
    for name, shape, kind in synth.param_shapes(cfg):
        sd[name] = ((torch.randn(shape, generator=g) * 0.02) if kind == "normal" else
                    (torch.ones(shape) if kind == "ones" else torch.zeros(shape))).numpy()
    kv = [(torch.randn(cfg.n_query_groups, P, cfg.head_size).bfloat16(),
           torch.randn(cfg.n_query_groups, P, cfg.head_size).bfloat16()) for _ in range(cfg.n_layer)]
    tok = torch.tensor([[1]])
    results = {}

    with torch.inference_mode():
        # reference: bf16 module, KV cache of S rows, context rows 0..P-1 written directly (same values as oracle)
        ref = model_mod.GPT(cfg)
        ref.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
        ref = ref.to(torch.bfloat16).eval()
        ref.max_seq_length = S
        ref.set_kv_cache(batch_size=1)
        for i, blk in enumerate(ref.transformer.h):
            blk.attn.kv_cache.k[0, :, :P] = kv[i][0]  # n_query_groups == n_head for Llama-2-7B: no expansion
            blk.attn.kv_cache.v[0, :, :P] = kv[i][1]
        ref(tok, torch.tensor([P]))  # warm-up
        t0 = time.perf_counter()
        for s in range(args.steps):
            ref(tok, torch.tensor([P + 1 + s]))
        results["reference"] = (time.perf_counter() - t0) / args.steps
        x = torch.randn(1, 1, cfg.n_embd).bfloat16()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ref.lm_head(ref.transformer.ln_f(x))
        head_ref = (time.perf_counter() - t0) / args.steps
        del ref

        orc = om.OracleGPT(cfg, sd, dtype=torch.bfloat16)
        orc.set_kv_cache(S)
        for i in range(cfg.n_layer):
            orc.cache.write(i, torch.arange(P), kv[i][0], kv[i][1])
        orc.forward(tok.view(-1), torch.tensor([P]))
        t0 = time.perf_counter()
        for s in range(args.steps):
            orc.forward(tok.view(-1), torch.tensor([P + 1 + s]))
        results["oracle"] = (time.perf_counter() - t0) / args.steps
        x2 = x.view(1, -1)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            orc._lin("lm_head", orc._norm("transformer.ln_f", x2))
        head_orc = (time.perf_counter() - t0) / args.steps

    for name, per, head in (("reference", results["reference"], head_ref), ("oracle", results["oracle"], head_orc)):
        block = (per - head) / cfg.n_layer
        full = block * 32 + head
        print(f"{name:9s}: {per * 1e3:8.1f} ms per 2-block step  -> 32 blocks {full * 1e3:8.1f} ms/token "
              f"({1 / full:.3f} tok/s) on {args.threads} threads")
    print(f"oracle / reference time ratio: {results['oracle'] / results['reference']:.3f}")


if __name__ == "__main__":
    main()
