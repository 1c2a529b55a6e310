"""Where the cold 2048-token prefill's extra time goes (bench `prefill_s` vs `warm_seconds`).

    python tools/prefill_cold.py [--order small-first|big-first] [--model NAME]

Builds random-init Llama-2-7B int4-g128 and times prefills in one process: with `small-first` a 16-token prefill
runs before the 2048-token ones (it loads every kernel the prefill path launches but allocates little), with
`big-first` the 2048-token prefill is the first call (the bench's order). For a sparse-MoE model the small-first
order runs 16 and 600 tokens (both grouped-GEMM tile shapes) before the 2048-token ones. Under
`rocprofv3 --kernel-trace --hip-runtime-trace` the trace shows which runtime calls fill the cold call's gaps.
"""

from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
for p in (str(REPO / "lit-gpt_amd"), str(REPO)):
    if p not in sys.path:
        sys.path.insert(0, p)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", choices=("small-first", "big-first"), default="big-first")
    ap.add_argument("--model", default="Llama-2-7b-hf")
    args = ap.parse_args()
    import torch

    from generate.base import build_model
    from lit_gpt import Config

    T = 2048
    dev = torch.device("cuda", 0)
    cfg = Config.from_name(args.model)
    model = build_model(cfg, quantize="int4-g128", device=dev, max_seq_length=T + 16)
    g = torch.Generator(device="cpu").manual_seed(1234)
    prompt = torch.randint(0, cfg.vocab_size, (T,), generator=g, dtype=torch.int32).to(dev)

    def prefill(n: int) -> float:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        model(prompt[:n].view(1, -1), torch.arange(n, device=dev), last_token_only=True)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    with torch.inference_mode():
        moe = cfg._mlp_class == "LLaMAMoE"
        small = [16, 600] if moe else [16]
        seq = small + [T, T, T] if args.order == "small-first" else [T, T] + small + [T]
        for n in seq:
            print(f"prefill T={n:5d}: {prefill(n) * 1e3:8.2f} ms", flush=True)


if __name__ == "__main__":
    main()
