"""A/B of decode-attention builds in ONE process on one box (box-to-box spread is ~4 %, larger than the effects).

usage: AB_LIBS=lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so,tools/_lab5/attn_old.so python tools/attn_ab.py
       (AB_HEADS=32 AB_GROUPS=AB_HEADS AB_CACHE=2304 AB_LAYERS=32 AB_SPLITS=product AB_POS=2063,2302)
Per library: 32 fused decode-attention launches (Llama-2-7B geometry, one KV cache per block, 8 splits) captured in
one HIP graph, replayed back to back — bench.py's time_attention — at several positions; rounds alternate the
libraries so drift hits both. Prints us per launch (median over rounds).
"""

import math
import os
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]

from lit_gpt import ops  # noqa: E402


def main():
    libs = os.environ["AB_LIBS"].split(",")
    H = int(os.environ.get("AB_HEADS", "32"))
    G = int(os.environ.get("AB_GROUPS", str(H)))
    hs, S = 128, int(os.environ.get("AB_CACHE", "2304"))
    layers = int(os.environ.get("AB_LAYERS", "32"))
    positions = [int(v) for v in os.environ.get("AB_POS", "2063,2302").split(",")]
    rounds = int(os.environ.get("AB_ROUNDS", "5"))
    dev = torch.device("cuda")
    loaded = [ops.load_library(Path(p), strict=False) for p in libs]
    caches = [(torch.randn(G, S, hs, device=dev).bfloat16(), torch.randn(G, S, hs, device=dev).bfloat16())
              for _ in range(layers)]
    qkv = torch.randn(1, (H + 2 * G) * hs, device=dev).bfloat16()
    cos, sin = torch.randn(S, hs, device=dev), torch.randn(S, hs, device=dev)
    split_list = [int(v) for v in os.environ.get("AB_SPLITS", "0").split(",")]
    split_list = [v or ops.decode_splits(G, H // G, hs, S) for v in split_list]
    splits = split_list[0]
    variants = [(i, sp) for i in range(len(libs)) for sp in split_list]  # (library, split count)
    out = torch.empty(1, H * hs, device=dev, dtype=torch.bfloat16)
    res = {}
    for p in positions:
        pos = torch.tensor([p], device=dev)
        graphs = []
        for li, sp in variants:
            ops._lib = loaded[li]
            ws = ops.AttentionWorkspace(1, H, G, hs, sp, dev)

            def launch_all(ws=ws, splits=sp):
                for kc, vc in caches:
                    ops.attention_decode_fused(qkv, kc, vc, pos, pos, cos, sin, H, G, hs, hs, 1.0 / math.sqrt(hs),
                                               splits, workspace=ws, out=out)

            launch_all()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                launch_all()
            g.replay()
            torch.cuda.synchronize()
            graphs.append((g, ws))
        for r in range(rounds):
            for i, (g, _) in enumerate(graphs):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    g.replay()
                e.record()
                e.synchronize()
                res.setdefault((p, i), []).append(s.elapsed_time(e) * 1e3 / (10 * layers))
    for p in positions:
        nbytes = 2 * G * hs * 2 * (p + 1) + (H + 2 * G) * hs * 2 + H * hs * 2
        for i, (li, sp) in enumerate(variants):
            v = res[(p, i)]
            med = float(np.median(v))
            print(f"p={p} {Path(libs[li]).name:28s} splits {sp:3d} {med:7.2f} us  (min {min(v):.2f} max {max(v):.2f})  "
                  f"{nbytes / med / 1e3:7.1f} GB/s = {nbytes / med / 1e3 / 8000:.3f} of 8 TB/s", flush=True)


if __name__ == "__main__":
    main()
