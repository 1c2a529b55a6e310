"""Lab: Mixtral decode MoE proj timing — lga_q4_gemv_experts_combine (one launch) vs lga_q4_gemv_experts +
lga_moe_combine (two), per call, from graph replays that cycle over 16 expert pairs of two stacked weight sets
(470 MB, past the 256 MB Infinity Cache). LGA_MOE_NW=8 selects the two-8-wave-workgroups-per-CU build of the fused
kernel (read once per process).

    python tools/moe_combine_ab.py            # 16-wave workgroups (default)
    LGA_MOE_NW=8 python tools/moe_combine_ab.py
"""
import os
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
from lit_gpt import ops  # noqa: E402

dev = torch.device("cuda")
N, K, E, G = 4096, 14336, 8, 128
g = torch.Generator().manual_seed(0)
stacks = []
for _ in range(2):
    qw = torch.empty(E, N, K // 2, dtype=torch.uint8, device=dev)
    sc = torch.empty(E, N, K // G, dtype=torch.bfloat16, device=dev)
    for e in range(E):
        q, s = ops.quantize(torch.randn(N, K, device=dev) * 0.02, 0, G)
        qw[e].copy_(q)
        sc[e].copy_(s)
    stacks.append((qw, sc))
pairs = [(i % E, (i * 3 + 1) % E) for i in range(16)]
pairs = [(a, b if b != a else (b + 1) % E) for a, b in pairs]
ids = [torch.tensor(p, dtype=torch.int32, device=dev) for p in pairs]
x = torch.randn(2, K, generator=g).bfloat16().to(dev)
probs = torch.tensor([0.6, 0.4]).bfloat16().to(dev)
res = torch.randn(N, generator=g).bfloat16().to(dev)
y = torch.empty(N, dtype=torch.bfloat16, device=dev)
eout = torch.empty(2, N, dtype=torch.bfloat16, device=dev)


def fused():
    for i, d in enumerate(ids):
        qw, sc = stacks[i % 2]
        ops.q4_gemv_experts_combine(x, qw, sc, d, probs, res, N, K, G, 0, out=y)


def split():
    for i, d in enumerate(ids):
        qw, sc = stacks[i % 2]
        ops.q4_gemv_experts(x, qw, sc, d, N, K, G, 0, out=eout)
        ops.moe_combine(eout.view(1, 2, N), probs.view(1, 2), d.view(1, 2), residual=res.view(1, N), out=y.view(1, N))


def timed(fn):
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        fn()
    best = 1e9
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        gr.replay()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) * 1000 / len(ids))
    return best


nw = os.environ.get("LGA_MOE_NW", "16")
for _ in range(2):
    print(f"NW={nw}: fused {timed(fused):6.2f} us/call   split (experts GEMV + combine) {timed(split):6.2f} us/call",
          flush=True)
