"""Lab probe: how much faster are the decode kernels when their bytes are already in the Infinity Cache (MALL)?

Llama-2-7B decode shapes, 32 "layers" with distinct buffers. Mode "cold": each kernel reads bytes no recent kernel
touched (HBM). Mode "warm": before each kernel, a bare read kernel streams exactly that kernel's bytes (filling
MALL), then a 64 MB read of unrelated data flushes the 32 MB of L2, then the kernel runs. Run under
``rocprofv3 --kernel-trace --stats`` and compare the kernels' average durations between the two modes.

usage: python tools/mall_lab.py cold|warm     (needs tools/_lab/overlap_lab.so)
"""
import ctypes
import math
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
from lit_gpt import ops  # noqa: E402

lab = ctypes.CDLL(str(REPO / "tools/_lab/overlap_lab.so"))
lab.lab_read.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                         ctypes.c_void_p]
mode = sys.argv[1]  # cold | warm (plain-load fill) | warmnt (nt-load fill)
dev = torch.device("cuda")
LAYERS, C, I, G, H, S, P = 16, 4096, 11008, 128, 32, 2304, 2200


def q(N, K):
    return ops.quantize(torch.randn(N, K, device=dev) * 0.02, 0, G)


layers = []
for _ in range(LAYERS):
    layers.append(dict(qkv=q(3 * C, C), o=q(C, C), fc1=q(I, C), fc2=q(I, C), down=q(C, I),
                       k=torch.randn(H, S, 128, device=dev).bfloat16(), v=torch.randn(H, S, 128, device=dev).bfloat16()))
junk = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
sink = torch.zeros(4, dtype=torch.int32, device=dev)
x = torch.randn(C, device=dev).bfloat16()
xi = torch.randn(I, device=dev).bfloat16()
nw = torch.ones(C, device=dev).bfloat16()
qkv = torch.randn(1, 3 * C, device=dev).bfloat16()
cos, sin = torch.randn(S, 128, device=dev), torch.randn(S, 128, device=dev)
pos = torch.tensor([P], device=dev)
ws = ops.AttentionWorkspace(1, H, H, 128, 8, dev)
y = torch.empty(3 * C, device=dev).bfloat16()
cur = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731


def touch(t, unr=-8 if mode == "warm" else 8):  # noqa: B008  # warm: plain (default-policy) loads; nt loads do not fill MALL
    lab.lab_read(t.data_ptr(), t.numel() * t.element_size(), 512, unr, sink.data_ptr(), cur())


def warm(*ts):
    if mode.startswith("warm"):
        for t in ts:
            touch(t)
        touch(junk, 8)


def step():
    for L in layers:
        warm(*L["qkv"])
        ops.q4_gemv(x, L["qkv"][0], L["qkv"][1], 3 * C, C, G, 0, norm_weight=nw, out=y)
        warm(L["k"], L["v"])
        ops.attention_decode_fused(qkv, L["k"], L["v"], pos, pos, cos, sin, H, H, 128, 128, 1 / math.sqrt(128), 8,
                                   workspace=ws)
        warm(*L["o"])
        ops.q4_gemv(x, L["o"][0], L["o"][1], C, C, G, 0, residual=x, out=y[:C])
        warm(*L["fc1"], *L["fc2"])
        ops.q4_gemv_swiglu(x, *L["fc1"], *L["fc2"], I, C, G, 0, norm_weight=nw, out=y[:I] if I <= 3 * C else None)
        warm(*L["down"])
        ops.q4_gemv(xi, L["down"][0], L["down"][1], C, I, G, 0, residual=x, out=y[:C])


step()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    step()
for _ in range(10):
    g.replay()
torch.cuda.synchronize()
print("done", mode)
