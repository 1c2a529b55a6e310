"""Prefill flash-attention timing (lga_attention with T query rows, causal): us per layer and TFLOP/s.

Llama-2-7B geometry (H = G = 32, hs = 128), T = 2048 at positions 0..T-1, 8 distinct caches, graph-captured.
usage: python tools/prefill_attn_bench.py [T]
"""
import math
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
from lit_gpt import ops  # noqa: E402
import os  # noqa: E402

if os.environ.get("ATT_LIB"):  # lab build of the library
    ops.LIB_PATH = Path(os.environ["ATT_LIB"])


def main(T=2048, H=32, G=32, hs=128, S=2304, layers=8):
    dev = torch.device("cuda")
    caches = [(torch.randn(G, S, hs, device=dev).bfloat16(), torch.randn(G, S, hs, device=dev).bfloat16())
              for _ in range(layers)]
    q = torch.randn(T, H, hs, device=dev).bfloat16()
    full = os.environ.get("ATT_FULL") == "1"  # every query row sees all T keys (no causal imbalance)
    pos = torch.full((T,), T - 1, device=dev, dtype=torch.long) if full else torch.arange(T, device=dev)
    y = torch.empty(T, H * hs, device=dev, dtype=torch.bfloat16)
    scale = 1.0 / math.sqrt(hs)

    def run():
        for kc, vc in caches:
            ops.attention(q, kc, vc, pos, H, G, hs, scale, 1, out=y)

    run()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / (5 * layers) * 1e3
    fl = 2.0 * 2.0 * H * hs * T * (T if full else (T + 1) / 2)
    print(f"prefill attention {'full' if full else 'causal'} T={T} H={H} G={G} hs={hs}: {us:8.1f} us/layer  {fl / us / 1e6:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
