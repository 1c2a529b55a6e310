"""A/B of the one-token routed down-projection + combine launch (lga_q4_gemv_experts_pair_combine) between library
builds, Mixtral geometry (8 experts x [4096, 14336] int4-g128, k = 2): 8 launches on distinct expert stacks in one HIP
graph, libraries alternating; outputs compared bit for bit.

usage: AB_LIBS=lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so,tools/_ab/liblitgpt_cpt8.so python tools/moe_down_ab.py
"""

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
    loaded = [ops.load_library(Path(p), strict=False) for p in libs]
    dev = torch.device("cuda")
    E, N, K, n, g = 8, 4096, 14336, 8, 128
    stacks = []
    for _ in range(n):
        qs, ss = zip(*[ops.quantize(torch.randn(N, K, device=dev) * 0.02, 0, g) for _ in range(E)])
        stacks.append((torch.stack(qs), torch.stack(ss)))
    x = torch.randn(2 * K, device=dev).bfloat16()
    ids = torch.tensor([5, 2], dtype=torch.int32, device=dev)
    probs = torch.tensor([0.6, 0.4], device=dev).bfloat16()
    res = torch.randn(N, device=dev).bfloat16()
    outs, graphs = [], []
    for lib in loaded:
        ops._lib = lib
        ws = ops.ExpertsPairWorkspace(N, dev)
        ys = [torch.empty(N, dtype=torch.bfloat16, device=dev) for _ in range(n)]

        def run():
            for (qw, sc), y in zip(stacks, ys):
                ops.q4_gemv_experts_pair_combine(x, qw, sc, ids, probs, res, N, K, g, 0, ws, out=y)

        run()
        torch.cuda.synchronize()
        outs.append([y.clone() for y in ys])
        for rep in range(20):  # the same launches again: any run-to-run difference is a hand-off race
            run()
            torch.cuda.synchronize()
            if not all(torch.equal(a, b) for a, b in zip(outs[-1], ys)):
                print(f"{Path(lib._name).name}: repeat {rep} differs from the first run", flush=True)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            run()
        gr.replay()
        torch.cuda.synchronize()
        graphs.append(gr)
    same = True
    for i in range(1, len(outs)):
        eq = all(torch.equal(a, b) for a, b in zip(outs[0], outs[i]))
        d = max((a.float() - b.float()).abs().max().item() for a, b in zip(outs[0], outs[i]))
        print(f"{Path(libs[i]).name} vs {Path(libs[0]).name}: bit-identical {eq} (max |diff| {d:.3e})", flush=True)
        same &= eq
    t = {}
    for _ in range(7):
        for i, gr in enumerate(graphs):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                gr.replay()
            e.record()
            e.synchronize()
            t.setdefault(i, []).append(s.elapsed_time(e) * 1e3 / (10 * n))
    nbytes = 2 * (N * K // 2 + N * (K // g) * 2)
    for i, lib in enumerate(libs):
        us = np.median(t[i])
        print(f"{Path(lib).name:28s} down + combine {us:6.2f} us per launch (min {min(t[i]):.2f}) = "
              f"{nbytes / us / 1e3:7.1f} GB/s", flush=True)
    raise SystemExit(0 if same else 1)


if __name__ == "__main__":
    main()
