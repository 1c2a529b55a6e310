"""Sweep decode-attention split counts on the GPU (Llama-2-7B geometry unless overridden).

Each launch reads a different layer's KV cache (32 distinct caches, > 1 GiB in total) so the timed launches
stream from HBM as in the decode step, not from the 256 MB MALL; launches are captured in a HIP graph.
Prints us/launch and effective GB/s (K + V bytes of keys 0..p) per (p, splits, path).
"""

import math
import os
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]

from lit_gpt import ops  # noqa: E402


def main(H=32, G=32, hs=128, S=4096, layers=32):
    import os
    libs = [x for x in os.environ.get("ATTN_LIBS", "").split(",") if x] or [None]
    for lib in libs:
        if lib is not None:
            import ctypes
            raw = ctypes.CDLL(lib)
            saved = dict(ops.SIGNATURES)
            for name in list(ops.SIGNATURES):  # older lab builds lack newer entry points
                if not hasattr(raw, name):
                    del ops.SIGNATURES[name]
            ops._lib = ops.load_library(Path(lib))
            ops.SIGNATURES.update(saved)
        print(f"=== library {lib or 'default'}", flush=True)
        mode = os.environ.get("ATTN_MODE", "fused" if lib is not None else "both")
        sweep(H, G, hs, S, layers, mode=mode)


def sweep(H, G, hs, S, layers, mode="both"):
    dev = torch.device("cuda")
    caches = [(torch.randn(G, S, hs, device=dev).bfloat16(), torch.randn(G, S, hs, device=dev).bfloat16())
              for _ in range(layers)]
    qkv = torch.randn(1, (H + 2 * G) * hs, device=dev).bfloat16()
    q = torch.randn(1, H, hs, device=dev).bfloat16()
    cos = torch.randn(S, hs, device=dev)
    sin = torch.randn(S, hs, device=dev)
    y = torch.empty(1, H * hs, device=dev, dtype=torch.bfloat16)
    scale = 1.0 / math.sqrt(hs)
    for p in [int(x) for x in os.environ.get("ATTN_POS", "128,1024,2048,2303,4000").split(",")]:
        pos = torch.tensor([p], device=dev)
        nbytes = 2 * G * (p + 1) * hs * 2
        for splits in [int(x) for x in os.environ.get("ATTN_SPLITS", "4,8,12,16,24,32,48,64").split(",")]:
            ws = ops.AttentionWorkspace(1, H, G, hs, splits, dev)
            if ws.counters.numel() < 64 * G:  # libraries built before the 256-B counter stride want G words
                ws.counters = torch.zeros(64 * G, dtype=torch.int32, device=dev)
            for fused in {"both": (False, True), "fused": (True,), "unfused": (False,)}[mode]:
                def run(i):
                    kc, vc = caches[i % layers]
                    if fused:
                        ops.attention_decode_fused(qkv, kc, vc, pos, pos, cos, sin, H, G, hs, hs, scale, splits,
                                                   workspace=ws, out=y)
                    else:
                        ops.attention(q, kc, vc, pos, H, G, hs, scale, splits, workspace=ws, out=y)

                for i in range(layers):
                    run(i)
                torch.cuda.synchronize()
                reps = 2 * layers
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for i in range(reps):
                        run(i)
                g.replay()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                g.replay()
                e.record()
                e.synchronize()
                us = s.elapsed_time(e) / reps * 1e3
                print(f"p={p:5d} splits={splits:4d} fused={int(fused)}  {us:7.2f} us  {nbytes / us / 1e3:7.1f} GB/s",
                      flush=True)
                del g


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
