"""Per-wave phase timeline of one decode-GEMV launch from a lab build with -DLGA_GEMV_TRACE.

usage: GEMV_LIB=tools/_lab/gtrace.so python tools/gemv_trace.py
Stamps (lane 0 of each wave, s_memrealtime 100 MHz): 0 start, 1 all loads issued, 2 x landed + sum of
squares (NORM only), 3 x staged in LDS (after the barrier), 4 every weight landed (vmcnt(0)), 5 output stored
(incl. the store's completion). Times in us from the earliest wave start.
"""

import ctypes
import os
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]

from lit_gpt import ops  # noqa: E402

SHAPES = {"gate_up": (11008, 4096, True, "norm"), "qkv": (12288, 4096, False, "norm"),
          "down": (4096, 11008, False, "res"), "o_proj": (4096, 4096, False, "res"),
          "lm_head": (32000, 4096, False, "norm")}


def main():
    lib = ops.load_library(Path(os.environ["GEMV_LIB"]))
    ops._lib = lib
    lib.lga_gemv_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda")
    for name, (N, K, dual, kind) in SHAPES.items():
        copies = max(3, int(1.2e9 // (N * K // 2 * (2 if dual else 1))))
        mats = []
        for _ in range(copies):
            q = ops.quantize(torch.randn(N, K, device=dev) * 0.02, 0, 128)
            q2 = ops.quantize(torch.randn(N, K, device=dev) * 0.02, 0, 128) if dual else None
            mats.append((q, q2))
        x = torch.randn(K, device=dev).bfloat16()
        nw = torch.ones(K, device=dev).bfloat16()
        res = torch.randn(N, device=dev).bfloat16()
        y = torch.empty(N, device=dev, dtype=torch.bfloat16)

        def run(i):
            (qa, sa), q2 = mats[i]
            if dual:
                ops.q4_gemv_swiglu(x, qa, sa, q2[0], q2[1], N, K, 128, 0, norm_weight=nw, out=y)
            elif kind == "norm":
                ops.q4_gemv(x, qa, sa, N, K, 128, 0, norm_weight=nw, out=y)
            else:
                ops.q4_gemv(x, qa, sa, N, K, 128, 0, residual=res, out=y)

        for i in range(1, copies):
            run(i)
        torch.cuda.synchronize()
        lib.lga_gemv_trace_read(np.zeros(8, dtype=np.uint64).ctypes.data, 8)  # clear
        run(0)
        torch.cuda.synchronize()
        nw_max = 65536
        buf = np.zeros(nw_max * 8, dtype=np.uint64)
        lib.lga_gemv_trace_read(buf.ctypes.data, nw_max * 8)
        tr = buf.reshape(nw_max, 8).astype(np.int64)
        tr = tr[tr[:, 0] > 0]
        if len(tr) == 0:  # the streaming form (gemv_stream.h) carries no stamps
            print(f"== {name} N={N} K={K}: no stamps (streaming form)", flush=True)
            continue
        t0 = tr[:, 0].min()
        rel = (tr - t0) / 100.0
        print(f"== {name} N={N} K={K} waves={len(tr)}", flush=True)
        labels = ["start", "issued", "x+ss", "x staged", "w landed", "stored"]
        for k, lab in enumerate(labels):
            col = rel[:, k][tr[:, k] > 0]
            if len(col) == 0:
                continue
            q = np.percentile(col, [0, 10, 50, 90, 100])
            print(f"   {lab:9s} " + "  ".join(f"{v:6.2f}" for v in q), flush=True)
        d = (tr[:, 4] - tr[:, 1]) / 100.0
        print(f"   issue->landed per wave: p10 {np.percentile(d, 10):.2f} p50 {np.median(d):.2f} "
              f"p90 {np.percentile(d, 90):.2f}", flush=True)
        d = (tr[:, 5] - tr[:, 4]) / 100.0
        print(f"   landed->stored per wave: p10 {np.percentile(d, 10):.2f} p50 {np.median(d):.2f} "
              f"p90 {np.percentile(d, 90):.2f}", flush=True)
        # occupancy over time: waves alive per 0.5 us bin
        end = rel[:, 5].max()
        bins = np.arange(0, end + 0.5, 0.5)
        alive = [int(((rel[:, 0] <= b) & (rel[:, 5] > b)).sum()) for b in bins]
        print("   alive waves per 0.5us: " + " ".join(str(a) for a in alive), flush=True)
        del mats
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
