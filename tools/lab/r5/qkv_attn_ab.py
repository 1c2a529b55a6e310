"""A/B of the decode step's attention half: qkv GEMV (RMSNorm fused) + fused decode attention as two launches vs
lga_qkv_attention_decode (one launch, the K/V stream beside the qkv weights), Llama-2-7B geometry, 32 blocks with
their own weights and caches in one HIP graph each, at the bench's positions.

usage: python tools/qkv_attn_ab.py        (AB_POS=2063,2302  AB_ROUNDS=7  AB_LIBS=lab .so list  AB_VARIANTS=0:0,2:0: LGA_QA_KV_WAIT:LGA_QA_KV_DELAY)
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
from lit_gpt.quantize import QuantLinear  # noqa: E402


def main():
    dev = torch.device("cuda")
    H = G = 32
    hs, C, S, layers = 128, 4096, 2304, 32
    N = (H + 2 * G) * hs
    positions = [int(v) for v in os.environ.get("AB_POS", "2063,2302").split(",")]
    rounds = int(os.environ.get("AB_ROUNDS", "7"))
    ab_libs = [v for v in os.environ.get("AB_LIBS", "").split(",") if v]  # lab builds, same entry points
    ops.load_library()
    ab_loaded = [ops.load_library(Path(v), strict=False) for v in ab_libs]
    lins = [QuantLinear.from_float(torch.randn(N, C, device=dev) * 0.02, None, "int4-g128", dev)
            for _ in range(layers)]
    caches = [(torch.randn(G, S, hs, device=dev).bfloat16(), torch.randn(G, S, hs, device=dev).bfloat16())
              for _ in range(layers)]
    x = torch.randn(1, C, device=dev).bfloat16()
    nw = torch.ones(C, device=dev).bfloat16()
    cos, sin = torch.randn(S, hs, device=dev), torch.randn(S, hs, device=dev)
    splits = ops.decode_splits(G, 1, hs, S)
    ws = ops.AttentionWorkspace(1, H, G, hs, splits, dev)
    qkv = torch.empty(N, device=dev, dtype=torch.bfloat16)
    y = torch.empty(1, H * hs, device=dev, dtype=torch.bfloat16)
    scale = 1.0 / math.sqrt(hs)
    for p in positions:
        pos = torch.tensor([p], device=dev)

        def two():
            for lin, (kc, vc) in zip(lins, caches):
                ops.q4_gemv(x.view(-1), lin.qweight, lin.scales, N, C, 128, 0, norm_weight=nw, out=qkv)
                ops.attention_decode_fused(qkv.view(1, -1), kc, vc, pos, pos, cos, sin, H, G, hs, hs, scale, splits,
                                           workspace=ws, out=y)

        def one():
            for lin, (kc, vc) in zip(lins, caches):
                ops.qkv_attention_decode(x, nw, 1e-5, lin, kc, vc, pos, pos, cos, sin, H, G, hs, scale, splits, ws,
                                         qkv, out=y)

        def gemv():
            for lin in lins:
                ops.q4_gemv(x.view(-1), lin.qweight, lin.scales, N, C, 128, 0, norm_weight=nw, out=qkv)

        graphs = {}
        variants = [("qkv gemv", gemv, None), ("gemv + attention", two, None)]
        variants += [(f"fused {v}", one, v) for v in os.environ.get("AB_VARIANTS", "0:0").split(",")]
        variants += [(f"fused {Path(lp).stem}", one, ("lib", lib)) for lp, lib in zip(ab_libs, ab_loaded)]
        default_lib = ops._lib
        for name, fn, v in variants:
            ops._lib = default_lib
            if isinstance(v, tuple):
                ops._lib = v[1]
            elif v is not None:  # "wait:delay" -> LGA_QA_KV_WAIT, LGA_QA_KV_DELAY
                os.environ["LGA_QA_KV_WAIT"], os.environ["LGA_QA_KV_DELAY"] = v.split(":")
            fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fn()
            g.replay()
            torch.cuda.synchronize()
            graphs[name] = g
        ops._lib = default_lib
        t = {}
        for _ in range(rounds):
            for name, g in graphs.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    g.replay()
                e.record()
                e.synchronize()
                t.setdefault(name, []).append(s.elapsed_time(e) * 1e3 / (10 * layers))
        print(f"p={p}: " + "  ".join(f"{k} {np.median(v):6.2f}" for k, v in t.items()) + " us per block", flush=True)


if __name__ == "__main__":
    main()
