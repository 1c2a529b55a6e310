"""Lab: launch variants of the routed fc_1 || fc_2 + SwiGLU decode GEMV (lga_q4_gemv_swiglu_experts, Mixtral geometry:
8 experts x [14336, 4096] int4-g128 per matrix, k = 2, RMSNorm fused): per-call time over distinct expert stacks in
one HIP graph, each variant (gemv.hip: bit 0 more rows per wave, bit 3 half the rows, bits 4..7 workgroups per CU)
alternating; outputs checked bit-identical across variants that keep the row grouping.

usage: python tools/moe_fc_variants.py [variants, default -1,0,1,8]
"""
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
from lit_gpt import ops  # noqa: E402


def main():
    variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "-1,0,1,8").split(",")]
    dev = torch.device("cuda")
    E, N, K, g, n = 8, 14336, 4096, 128, 4
    stacks = []
    for _ in range(n):
        q1, s1 = zip(*[ops.quantize(torch.randn(N, K, device=dev) * 0.02, 0, g) for _ in range(E)])
        q2, s2 = zip(*[ops.quantize(torch.randn(N, K, device=dev) * 0.02, 0, g) for _ in range(E)])
        stacks.append((torch.stack(q1), torch.stack(s1), torch.stack(q2), torch.stack(s2)))
    x = torch.randn(K, device=dev).bfloat16()
    nw = (1 + 0.1 * torch.randn(K, device=dev)).bfloat16()
    ids = torch.tensor([5, 2], dtype=torch.int32, device=dev)
    graphs = {}
    outs = {}
    for v in variants:
        ys = [torch.empty(2, N, dtype=torch.bfloat16, device=dev) for _ in range(n)]

        def run(v=v, ys=ys):
            for (q1, s1, q2, s2), y in zip(stacks, ys):
                ops.q4_gemv_swiglu_experts(x, q1, s1, q2, s2, ids, N, K, g, 0, norm_weight=nw, out=y, variant=v)

        run()
        torch.cuda.synchronize()
        outs[v] = [y.clone() for y in ys]
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            run()
        gr.replay()
        torch.cuda.synchronize()
        graphs[v] = gr
    t = {v: [] for v in variants}
    for _ in range(7):
        for v, gr in graphs.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                gr.replay()
            e.record()
            e.synchronize()
            t[v].append(s.elapsed_time(e) * 1e3 / (10 * n))
    nbytes = 2 * 2 * (N * K // 2 + N * (K // g) * 2)
    ref = outs[variants[0]]
    for v in variants:
        same = all(torch.equal(a, b) for a, b in zip(ref, outs[v]))
        us = np.median(t[v])
        print(f"variant {v:4d}: {us:6.2f} us per launch (min {min(t[v]):.2f}) = {nbytes / us / 1e3:7.1f} GB/s, "
              f"bit-identical to variant {variants[0]}: {same}", flush=True)


if __name__ == "__main__":
    main()
