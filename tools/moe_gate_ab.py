"""A/B of the one-token router gate + routing launch (lga_moe_gate_route) between library builds, Mixtral geometry
(8 experts x 4096, k = 2, RMSNorm fused): 32 launches on distinct gate weights in one HIP graph, libraries alternating.

usage: AB_LIBS=lit-gpt_amd/lit_gpt/_lib/liblitgpt_amd.so,tools/_lab5/old.so python tools/moe_gate_ab.py
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
    E, K, k, n = 8, 4096, 2, 32
    gates = [ops.quantize(torch.randn(E, K, device=dev) * 0.02, 0, 128) for _ in range(n)]
    x = torch.randn(K, device=dev).bfloat16()
    nw = torch.ones(K, device=dev).bfloat16()
    ids = torch.empty(1, k, dtype=torch.int32, device=dev)
    pr = torch.empty(1, k, dtype=torch.bfloat16, device=dev)
    graphs = []
    for lib in loaded:
        ops._lib = lib

        def run():
            for qw, sc in gates:
                ops.moe_gate_route(x, qw, sc, E, K, 128, 0, k, norm_weight=nw, ids=ids, probs=pr)

        run()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            run()
        g.replay()
        torch.cuda.synchronize()
        graphs.append(g)
    res = {}
    for _ in range(7):
        for i, g in enumerate(graphs):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                g.replay()
            e.record()
            e.synchronize()
            res.setdefault(i, []).append(s.elapsed_time(e) * 1e3 / (10 * n))
    for i, lib in enumerate(libs):
        print(f"{Path(lib).name:28s} gate + route {np.median(res[i]):6.2f} us per launch", flush=True)


if __name__ == "__main__":
    main()
