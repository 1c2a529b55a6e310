"""Lab: decode-GEMV launch time per shape for lab builds of the library (gemv.hip compiled with -DLGA_LAB_NOX /
-DLGA_LAB_NOSCALE / -DLGA_LAB_NOCOMPUTE): what the activation fetch, the scale loads and the dequant-dot cost.

usage: python tools/gemv_variants.py lib1.so [lib2.so ...]   (graph of back-to-back launches over distinct weights)
       GEMV_VARIANTS=-1,4,6 ... times each launch variant (gemv.hip: bit 2 streaming form, bit 1 one row per tile,
       bits 4..7 workgroups per CU) of every library
"""
import os
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
from lit_gpt import ops  # noqa: E402

SHAPES = {"qkv": (12288, 4096, False, "norm"), "o_proj": (4096, 4096, False, "res"),
          "gate_up": (11008, 4096, True, "norm"), "down": (4096, 11008, False, "res"),
          "lm_head": (32000, 4096, False, "norm")}
if os.environ.get("GEMV_SHAPES") == "mixtral":  # Mixtral-8x7B decode shapes (qkv with 8 kv heads, attn.proj)
    SHAPES = {"mix_qkv": (6144, 4096, False, "norm"), "mix_proj": (4096, 4096, False, "res"),
              "gate": (8, 4096, False, "norm")}
dev = torch.device("cuda")
data = {}
for name, (N, K, dual, kind) in SHAPES.items():
    copies = max(4, int(1.0e9 // (N * K // 2 * (2 if dual else 1))))
    mats = [(ops.quantize(torch.randn(N, K, device=dev) * 0.02, 0, 128),
             ops.quantize(torch.randn(N, K, device=dev) * 0.02, 0, 128) if dual else None) for _ in range(copies)]
    data[name] = mats
x = {K: torch.randn(K, device=dev).bfloat16() for K in (4096, 11008)}
nw = torch.ones(4096, device=dev).bfloat16()
res = torch.randn(32000, device=dev).bfloat16()
y = torch.empty(32000, device=dev, dtype=torch.bfloat16)

import os  # noqa: E402

VARIANTS = [int(v) for v in os.environ.get("GEMV_VARIANTS", "-1").split(",")]
for lib, var in [(lib, v) for lib in sys.argv[1:] for v in VARIANTS]:
    ops._lib = ops.load_library(Path(lib))  # load_library(path) does not install it as the default
    line = []
    for name, (N, K, dual, kind) in SHAPES.items():
        mats = data[name]

        def run():
            for (qa, sa), q2 in mats:
                if dual:
                    ops.q4_gemv_swiglu(x[K], qa, sa, q2[0], q2[1], N, K, 128, 0, norm_weight=nw, out=y[:N],
                                       variant=var)
                elif kind == "norm":
                    ops.q4_gemv(x[K], qa, sa, N, K, 128, 0, norm_weight=nw, out=y[:N], variant=var)
                else:
                    ops.q4_gemv(x[K], qa, sa, N, K, 128, 0, residual=res[:N], out=y[:N], variant=var)

        run()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            run()
        best = 1e9
        for _ in range(4):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e) * 1e3 / len(mats))
        line.append(f"{name} {best:6.2f}")
    print(f"{Path(lib).name:16s} v={var:4d} " + "  ".join(line), flush=True)
