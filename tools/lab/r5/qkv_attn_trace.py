"""Phase timeline of lga_qkv_attention_decode from a lab build with -DLGA_QA_TRACE (make lab-lib LABSRC=qkv_attention
LABFLAGS=-DLGA_QA_TRACE LABLIB=../../tools/_lab5/qa_trace.so). Per workgroup (thread 0, 100 MHz): 0 start, 1 x staged,
2 qkv rows computed, 3 group rows exchanged + q roped, 4 keys scored, 5 published + arrival returned, 6 combined (last
split). The traced launch runs right after 16 untraced ones (each on its own weights and caches), us from the
earliest workgroup start.

usage: QA_LIB=tools/_lab5/qa_trace.so python tools/qkv_attn_trace.py
"""

import ctypes
import math
import os
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]

from lit_gpt import ops  # noqa: E402
from lit_gpt.quantize import QuantLinear  # noqa: E402


def main():
    lib = ops.load_library(Path(os.environ["QA_LIB"]), strict=False)
    ops._lib = lib
    lib.lga_qa_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda")
    H = G = 32
    hs, C, S, layers = 128, 4096, 2304, 17
    N = (H + 2 * G) * hs
    lins = [QuantLinear.from_float(torch.randn(N, C, device=dev) * 0.02, None, "int4-g128", dev)
            for _ in range(layers)]
    caches = [(torch.randn(G, S, hs, device=dev).bfloat16(), torch.randn(G, S, hs, device=dev).bfloat16())
              for _ in range(layers)]
    x = torch.randn(1, C, device=dev).bfloat16()
    nw = torch.ones(C, device=dev).bfloat16()
    cos, sin = torch.randn(S, hs, device=dev), torch.randn(S, hs, device=dev)
    splits = ops.decode_splits(G, 1, hs, S)
    ws = ops.AttentionWorkspace(1, H, G, hs, splits, dev)
    qkv = torch.empty(N, device=dev, dtype=torch.bfloat16)
    for p in (2063, 2302):
        pos = torch.tensor([p], device=dev)
        for i in range(layers):
            if i == layers - 1:
                torch.cuda.synchronize()
                lib.lga_qa_trace_read(np.zeros(8, dtype=np.uint64).ctypes.data, 8)  # clear
            ops.qkv_attention_decode(x, nw, 1e-5, lins[i], caches[i][0], caches[i][1], pos, pos, cos, sin, H, G, hs,
                                     1.0 / math.sqrt(hs), splits, ws, qkv)
        torch.cuda.synchronize()
        n = splits * G
        buf = np.zeros(n * 8, dtype=np.uint64)
        lib.lga_qa_trace_read(buf.ctypes.data, n * 8)
        tr = buf.reshape(n, 8).astype(np.int64)
        t0 = tr[:, 0].min()
        rel = (tr - t0) / 100.0
        print(f"p={p}", flush=True)
        for k, name in enumerate(["start", "x staged", "qkv rows", "q ready", "scored", "published", "combined"]):
            col = rel[:, k][tr[:, k] > 0]
            print(f"   {name:9s} min {col.min():6.2f}  med {np.median(col):6.2f}  max {col.max():6.2f}  (n={len(col)})",
                  flush=True)


if __name__ == "__main__":
    main()
