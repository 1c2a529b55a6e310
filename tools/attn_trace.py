"""Phase timeline of one decode-attention launch from a lab build with -DLGA_ATTN_TRACE.

usage: ATTN_LIBS=tools/_lab/trace_4_4.so,... python tools/attn_trace.py
Per block (thread 0): 0 start, 1 position known, 2 q ready (+ first KV batch landed), 3 key loop done,
4 block merge done, 5 partial published + arrival counter returned, 6 combine done (last block). Times in us from the
earliest block start (s_memrealtime, 100 MHz).
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


def run(lib_path, H=32, G=32, hs=128, S=4096, layers=16):
    lib = ops.load_library(Path(lib_path))
    ops._lib = lib
    lib.lga_attn_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda")
    caches = [(torch.randn(G, S, hs, device=dev).bfloat16(), torch.randn(G, S, hs, device=dev).bfloat16())
              for _ in range(layers)]
    qkv = torch.randn(1, (H + 2 * G) * hs, device=dev).bfloat16()
    cos = torch.randn(S, hs, device=dev)
    sin = torch.randn(S, hs, device=dev)
    scale = 1.0 / math.sqrt(hs)
    for p in [int(v) for v in os.environ.get("ATTN_POS", "2048,2302").split(",")]:
        pos = torch.tensor([p], device=dev)
        for splits in [int(v) for v in os.environ.get("ATTN_SPLITS", "8").split(",")]:
            ws = ops.AttentionWorkspace(1, H, G, hs, splits, dev)
            for i in range(layers):
                kc, vc = caches[i]
                ops.attention_decode_fused(qkv, kc, vc, pos, pos, cos, sin, H, G, hs, hs, scale, splits, workspace=ws)
            torch.cuda.synchronize()
            lib.lga_attn_trace_read(np.zeros(8, dtype=np.uint64).ctypes.data, 8)  # clear (read-and-clear)
            kc, vc = caches[0]
            ops.attention_decode_fused(qkv, kc, vc, pos, pos, cos, sin, H, G, hs, hs, scale, splits, workspace=ws)
            torch.cuda.synchronize()
            nblk = splits * G
            buf = np.zeros(nblk * 8, dtype=np.uint64)
            lib.lga_attn_trace_read(buf.ctypes.data, nblk * 8)
            tr = buf.reshape(nblk, 8).astype(np.int64)
            t0 = tr[:, 0].min()
            rel = (tr - t0) / 100.0  # us
            last = tr[:, 6] > 0
            print(f"{Path(lib_path).name} p={p} splits={splits}")
            for k, name in enumerate(["start", "pos", "q+kv0", "loop", "merge"]):
                col = rel[:, k]
                print(f"   {name:7s} min {col.min():6.2f}  med {np.median(col):6.2f}  max {col.max():6.2f}")
            col = rel[:, 5]
            print(f"   {'atomic':7s} min {col.min():6.2f}  med {np.median(col):6.2f}  max {col.max():6.2f}")
            col = rel[last, 6]
            print(f"   {'combine':7s} min {col.min():6.2f}  med {np.median(col):6.2f}  max {col.max():6.2f}"
                  f"  (n={last.sum()})", flush=True)


if __name__ == "__main__":
    for lib in os.environ["ATTN_LIBS"].split(","):
        run(lib)
