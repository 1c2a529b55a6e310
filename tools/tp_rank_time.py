"""Per-rank decode launch costs at tensor-parallel geometries, measured in ONE process on one GPU.

usage: python tools/tp_rank_time.py [--pos 2200] [--layers 32]

For each geometry (Llama-2-7B at TP = 1/2/4/8, Llama-2-70B at TP = 8) this builds the rank's shard shapes of
generate/tp.py's split — qkv / fc_1 / fc_2 column-parallel, attn.proj / mlp.proj row-parallel — as int4-g128
weights, one distinct copy per layer (so nothing is served from the caches a real step would not have warm), and
times each op of the rank's decode layer as HIP-graph replays of `layers` back-to-back launches: the fused RMSNorm +
qkv GEMV, the fused decode attention (its split count and head slices as the product picks them), the row-parallel
projections as the plain GEMV (the xGMI all-reduce folded into them is a separate, cross-GPU term), and the fused
RMSNorm + fc_1||fc_2 + SwiGLU GEMV. Also the qkv-inside-attention chain as two launches in one graph, and the
lm_head + argmax once per step. Prints us per launch and the per-layer sum.
"""

import argparse
import math
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]

from lit_gpt import ops  # noqa: E402

GEOMS = {  # name: (C, n_head, n_query_groups, intermediate, tp)
    "7B tp1": (4096, 32, 32, 11008, 1),
    "7B tp2": (4096, 32, 32, 11008, 2),
    "7B tp4": (4096, 32, 32, 11008, 4),
    "7B tp8": (4096, 32, 32, 11008, 8),
    "70B tp8": (8192, 64, 8, 28672, 8),
}


def time_graph(fn, layers, reps=10):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            g.replay()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / (reps * layers))
    return best


def q4(N, K, dev):
    from lit_gpt.quantize import _fit_group  # the group the product fits to a shard's K (e.g. 1376 at 7B TP = 8)

    g = _fit_group(K, 128)
    return ops.quantize(torch.randn(N, K, device=dev) * 0.02, ops.FMT_Q4G, g) + (g,)


def run(name, C, H, G, I, tp, pos, layers, dev):
    hs = 128
    Hr, Gr = H // tp, max(1, G // tp)
    Ir = I // tp
    Kp = Hr * hs  # row-parallel proj input per rank
    S = pos + 64
    qkv_n = (Hr + 2 * Gr) * hs
    W = [dict(qkv=q4(qkv_n, C, dev), proj=q4(C, Kp, dev), fc1=q4(Ir, C, dev), fc2=q4(Ir, C, dev),
              down=q4(C, Ir, dev), kc=torch.randn(Gr, S, hs, device=dev).bfloat16(),
              vc=torch.randn(Gr, S, hs, device=dev).bfloat16()) for _ in range(layers)]
    x = torch.randn(C, device=dev).bfloat16()
    nw = torch.ones(C, device=dev).bfloat16()
    qkv = torch.empty(qkv_n, device=dev, dtype=torch.bfloat16)
    y = torch.empty(Hr * hs, device=dev, dtype=torch.bfloat16)
    o = torch.empty(C, device=dev, dtype=torch.bfloat16)
    g = torch.empty(Ir, device=dev, dtype=torch.bfloat16)
    cos, sin = torch.randn(S, hs, device=dev), torch.randn(S, hs, device=dev)
    p = torch.tensor([pos], device=dev)
    splits = ops.decode_splits(Gr, Hr // Gr, hs, S)
    ws = ops.AttentionWorkspace(1, Hr, Gr, hs, splits, dev)
    scale = 1.0 / math.sqrt(hs)
    qkv_init = torch.randn(1, qkv_n, device=dev).bfloat16()

    def f_qkv():
        for w in W:
            ops.q4_gemv(x, *w["qkv"][:2], qkv_n, C, w["qkv"][2], 0, norm_weight=nw, out=qkv)

    def f_attn():
        for w in W:
            ops.attention_decode_fused(qkv_init, w["kc"], w["vc"], p, p, cos, sin, Hr, Gr, hs, hs, scale, splits,
                                       workspace=ws, out=y.view(1, -1))

    def f_proj():
        for w in W:
            ops.q4_gemv(y, *w["proj"][:2], C, Kp, w["proj"][2], 0, residual=x, out=o)

    def f_fc():
        for w in W:
            ops.q4_gemv_swiglu(x, *w["fc1"][:2], *w["fc2"][:2], Ir, C, w["fc1"][2], 0, norm_weight=nw, out=g)

    def f_down():
        for w in W:
            ops.q4_gemv(g, *w["down"][:2], C, Ir, w["down"][2], 0, residual=x, out=o)

    def f_layer():
        for w in W:
            ops.q4_gemv(x, *w["qkv"][:2], qkv_n, C, w["qkv"][2], 0, norm_weight=nw, out=qkv)
            ops.attention_decode_fused(qkv.view(1, -1), w["kc"], w["vc"], p, p, cos, sin, Hr, Gr, hs, hs, scale,
                                       splits, workspace=ws, out=y.view(1, -1))
            ops.q4_gemv(y, *w["proj"][:2], C, Kp, w["proj"][2], 0, residual=x, out=o)
            ops.q4_gemv_swiglu(o, *w["fc1"][:2], *w["fc2"][:2], Ir, C, w["fc1"][2], 0, norm_weight=nw, out=g)
            ops.q4_gemv(g, *w["down"][:2], C, Ir, w["down"][2], 0, residual=o, out=x)

    t = {k: time_graph(f, layers) for k, f in (("qkv", f_qkv), ("attn", f_attn), ("proj", f_proj), ("fc", f_fc),
                                               ("down", f_down), ("layer", f_layer))}
    parts = sum(t[k] for k in ("qkv", "attn", "proj", "fc", "down"))
    print(f"{name:8s} rank H={Hr:2d} G={Gr:2d} I={Ir:5d} splits={splits:2d}: " +
          " ".join(f"{k} {t[k]:5.2f}" for k in ("qkv", "attn", "proj", "fc", "down")) +
          f" | sum {parts:5.2f}, chained layer {t['layer']:5.2f} us", flush=True)
    del W
    torch.cuda.empty_cache()
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pos", type=int, default=2200)
    ap.add_argument("--layers", type=int, default=32)
    args = ap.parse_args()
    dev = torch.device("cuda")
    for name, (C, H, G, I, tp) in GEOMS.items():
        run(name, C, H, G, I, tp, args.pos, args.layers if not name.startswith("70B") else 20, dev)


if __name__ == "__main__":
    main()
