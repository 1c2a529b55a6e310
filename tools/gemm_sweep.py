"""Prefill GEMM timing at the Llama-2-7B prefill shapes (M = 2048): us per call and TFLOP/s (graph-captured)."""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
from lit_gpt import ops  # noqa: E402
import os  # noqa: E402

if os.environ.get("GEMM_LIB"):  # lab build of the library
    ops.LIB_PATH = Path(os.environ["GEMM_LIB"])

SHAPES = {"qkv": (12288, 4096), "o_proj": (4096, 4096), "fc": (11008, 4096), "down": (4096, 11008)}


def main(M=2048):
    dev = torch.device("cuda")
    tot_us, tot_fl = 0.0, 0.0
    for name, (N, K) in SHAPES.items():
        for fmt, group in ((0, 128), (1, 64), (2, 0)):
            w = torch.randn(N, K, device=dev) * 0.02
            if fmt == 2:
                wb = w.bfloat16()
            else:
                q, s = ops.quantize(w, fmt, group)
            x = torch.randn(M, K, device=dev).bfloat16()
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

            def call():
                if fmt == 2:
                    ops.bf16_gemm(x, wb, out=y)
                else:
                    ops.q4_gemm(x, q, s, N, K, group, fmt, out=y)
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(10):
                    call()
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
