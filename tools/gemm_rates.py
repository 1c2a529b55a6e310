"""Lab: prefill GEMM rates at Llama-2-7B layer shapes (M = 2048 prompt rows) — the product's int4 GEMM, its
dequantize pass + bf16 GEMM (gemm.hip's MFMA tiles), and torch.matmul (the vendor library) on the same bf16
operands for comparison.

usage: python tools/gemm_rates.py [M]   (per-call GPU time from graph replays over distinct weight copies; the
bf16 rows re-read one weight from the MALL, so they are optimistic at small M)
"""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
from lit_gpt import ops  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
if len(sys.argv) > 2 and sys.argv[2]:  # an alternative build of the library (lab A/B)
    ops._lib = ops.load_library(Path(sys.argv[2]))
ONLY = sys.argv[3].split(",") if len(sys.argv) > 3 else None
dev = torch.device("cuda")
SHAPES = {"qkv": (12288, 4096), "proj": (4096, 4096), "fc": (11008, 4096), "down": (4096, 11008)}


def timed(fn, reps=16):
    """GPU time per call: `reps` calls captured in a HIP graph and replayed, so short launches (M = 64) are timed
    without the Python / ctypes launch overhead (which would otherwise exceed the kernels themselves). fn(i) may
    pick one of several weight copies so the weights stream from HBM as in a prefill, not from the 256 MB MALL."""
    fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(reps):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


tot = {}
for name, (N, K) in SHAPES.items():
    w = torch.randn(N, K, device=dev) * 0.02
    qw, sc = ops.quantize(w, 0, 128)
    wb = ops.q4_dequantize(qw, sc, N, K, 128, 0)
    # enough distinct copies of the packed weights that one replay streams > 512 MB of them
    C = max(1, min(16, -(-512 * 2 ** 20 // (N * K // 2))))
    qws = [qw] + [qw.clone() for _ in range(C - 1)]
    scs = [sc] + [sc.clone() for _ in range(C - 1)]
    x = torch.randn(M, K, device=dev).bfloat16()
    fl = 2.0 * M * N * K
    r = {"q4f": timed(lambda i: ops.q4_gemm_fused(x, qws[i % C], scs[i % C], N, K, 128, 0)),
         "q4_gemm": timed(lambda i: ops.q4_gemm(x, qws[i % C], scs[i % C], N, K, 128, 0)),
         "dequant": timed(lambda i: ops.q4_dequantize(qws[i % C], scs[i % C], N, K, 128, 0, out=wb)),
         "bf16_gemm": timed(lambda i: ops.bf16_gemm(x, wb)),
         "q4f_bf16w": timed(lambda i: ops.q4_gemm_fused(x, wb, None, N, K, 64, 2)),
         "torch_mm": timed(lambda i: torch.matmul(x, wb.t()))}
    if name == "fc":  # fc_1 || fc_2 + SwiGLU in one launch (counts as both GEMMs of the layer)
        r["q4f_swiglu/2"] = timed(lambda i: ops.q4_gemm_swiglu(x, qws[i % C], scs[i % C], qws[(i + 1) % C],
                                                               scs[(i + 1) % C], N, K, 128, 0)) / 2
    if ONLY:
        r = {k: v for k, v in r.items() if k in ONLY}
    for k, v in r.items():
        tot[k] = tot.get(k, 0.0) + v * (2 if name == "fc" else 1)
    print(f"{name:5s} N={N:6d} K={K:6d}  " + "  ".join(
        f"{k} {v:8.1f} us" + (f" ({fl / v / 1e6:6.1f} TF/s)" if k != "dequant" else
                              f" ({(N * K * 2.5) / v / 1e3:6.1f} GB/s)") for k, v in r.items()), flush=True)
print("per layer: " + "  ".join(f"{k} {v:8.1f} us" for k, v in tot.items()) + "  (fc counted twice)")
fl_layer = 2.0 * M * sum(N * K * (2 if n == "fc" else 1) for n, (N, K) in SHAPES.items())
print("per-layer TF/s: " + "  ".join(f"{k} {fl_layer / v / 1e6:6.1f}" for k, v in tot.items()), flush=True)
