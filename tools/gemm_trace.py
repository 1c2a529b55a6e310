"""Lab: per-workgroup phase timeline of the fused prefill GEMM at the Llama-2-7B layer shapes (M = 2048), from a
build with -DLGA_Q4F_TRACE (make -C lit-gpt_amd/csrc lab-lib LABSRC=gemm_q4f LABFLAGS=-DLGA_Q4F_TRACE
LABLIB=../../tools/_lab/q4f_trace.so). Phases per workgroup (thread 0, 100 MHz clock): 0 start, 1 prologue done
(first stages landed + first dequantization), 2 K-loop done, 3 epilogue stores retired. Prints, per shape, the
start skew, prologue, loop and epilogue times (median / p90 / max, us) and the kernel span.
usage: python tools/gemm_trace.py tools/_lab/q4f_trace.so"""
import ctypes
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]
from lit_gpt import ops  # noqa: E402

lib = ops.load_library(Path(sys.argv[1]))
ops._lib = lib
lib.lga_q4f_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
dev = torch.device("cuda")
M = 2048
SHAPES = {"qkv": (12288, 4096, False), "proj": (4096, 4096, False), "fc": (11008, 4096, True),
          "down": (4096, 11008, False)}
buf = np.zeros(8192 * 4, dtype=np.uint64)
for name, (N, K, dual) in SHAPES.items():
    w = torch.randn(N, K, device=dev) * 0.02
    qw, sc = ops.quantize(w, 0, 128)
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    if dual:
        w2 = torch.randn(N, K, device=dev) * 0.02
        q2, s2 = ops.quantize(w2, 0, 128)
        run = lambda: ops.q4_gemm_swiglu(x, qw, sc, q2, s2, N, K, 128, 0)  # noqa: E731
    else:
        run = lambda: ops.q4_gemm_fused(x, qw, sc, N, K, 128, 0)  # noqa: E731
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    lib.lga_q4f_trace_read(buf.ctypes.data, buf.size)  # clear
    run()
    torch.cuda.synchronize()
    lib.lga_q4f_trace_read(buf.ctypes.data, buf.size)
    tr = buf.reshape(-1, 4).astype(np.int64)
    tr = tr[tr[:, 0] > 0]
    t0 = tr[:, 0].min()
    rel = (tr - t0) / 100.0  # us
    ph = {"start": rel[:, 0], "prologue": rel[:, 1] - rel[:, 0], "loop": rel[:, 2] - rel[:, 1],
          "epilogue": rel[:, 3] - rel[:, 2], "end": rel[:, 3]}
    print(f"{name}: {len(tr)} workgroups, span {rel[:, 3].max():.1f} us")
    for k, v in ph.items():
        print(f"   {k:9s} median {np.median(v):7.2f}  p90 {np.percentile(v, 90):7.2f}  max {v.max():7.2f}  "
              f"min {v.min():7.2f}")
    # rounds: workgroups sorted by start, the start of each 256-block round
    order = np.argsort(rel[:, 0])
    starts = rel[order, 0]
    print("   round starts:", " ".join(f"{starts[i]:.1f}" for i in range(0, len(starts), 256)))
