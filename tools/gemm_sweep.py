"""Prefill GEMM timing at the Llama-2-7B prefill shapes (M = 2048): us per call and TFLOP/s (graph-captured)."""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
from lit_gpt import ops  # noqa: E402

SHAPES = {"qkv": (12288, 4096), "o_proj": (4096, 4096), "fc": (11008, 4096), "down": (4096, 11008)}


def main(M=2048):
    dev = torch.device("cuda")
    tot_us, tot_fl = 0.0, 0.0
    for name, (N, K) in SHAPES.items():
        for fmt, group in ((0, 128), (1, 64)):
            q, s = ops.quantize(torch.randn(N, K, device=dev) * 0.02, fmt, group)
            x = torch.randn(M, K, device=dev).bfloat16()
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            for _ in range(3):
                ops.q4_gemm(x, q, s, N, K, group, fmt, out=y)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(10):
                    ops.q4_gemm(x, q, s, N, K, group, fmt, out=y)
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) / 10 * 1e3
            fl = 2.0 * M * N * K
            if fmt == 0:
                tot_us += us * (2 if name == "fc" else 1)
                tot_fl += fl * (2 if name == "fc" else 1)
            print(f"{name:7s} fmt={fmt} M={M} N={N} K={K}: {us:9.1f} us  {fl / us / 1e6:7.1f} TFLOP/s", flush=True)
    print(f"int4-g128 layer total (qkv+o+2fc+down): {tot_us:.1f} us, {tot_fl / tot_us / 1e6:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
