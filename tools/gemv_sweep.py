"""Sweep GEMV launch variants for the Llama-2-7B decode shapes on the GPU; prints GB/s per (shape, variant).

Weights are rotated over enough copies (> 1 GiB) that each launch streams from HBM as in the decode step;
launches run back to back between two HIP events (as inside the captured step).
"""

import os
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]

from lit_gpt import ops  # noqa: E402

if os.environ.get("GEMV_LIB"):  # lab build of the library (e.g. -DLGA_GEMV_LAB variants)
    ops.LIB_PATH = Path(os.environ["GEMV_LIB"])

SHAPES = {  # name: (N, K, dual)
    "qkv": (12288, 4096, False),
    "o_proj": (4096, 4096, False),
    "gate_up": (11008, 4096, True),
    "down": (4096, 11008, False),
    "lm_head": (32000, 4096, False),
}


def main(fmt=0, group=128):
    dev = torch.device("cuda")
    res = {}
    for name, (N, K, dual) in SHAPES.items():
        per = N * K // 2 * (2 if dual else 1)
        copies = int(os.environ["GEMV_COPIES"]) if "GEMV_COPIES" in os.environ else max(2, int(1.5e9 // per))
        mats = []
        for c in range(copies):
            w = torch.randn(N, K, device=dev) * 0.02
            q1 = ops.quantize(w, fmt, group)
            q2 = ops.quantize(torch.randn(N, K, device=dev) * 0.02, fmt, group) if dual else None
            mats.append((q1, q2))
        x = torch.randn(K, device=dev).bfloat16()
        nw = torch.ones(K, device=dev).bfloat16()
        y = torch.empty(N, device=dev, dtype=torch.bfloat16)
        nbytes = per + (N * K // group) * (2 if fmt == 0 else 4) * (2 if dual else 1)
        best = None
        variants = [int(v) for v in os.environ.get("GEMV_VARIANTS", "0,1").split(",")]
        for v in variants:  # bit0: rows per wave small/large
            rw, blocks = v & 1, v >> 4
            if True:

                def run(i):
                    (qa, sa), q2 = mats[i % copies]
                    if dual:
                        ops.q4_gemv_swiglu(x, qa, sa, q2[0], q2[1], N, K, group, fmt, norm_weight=nw, out=y,
                                           variant=v)
                    else:
                        ops.q4_gemv(x, qa, sa, N, K, group, fmt, norm_weight=nw, out=y, variant=v)

                for i in range(copies):
                    run(i)
                torch.cuda.synchronize()
                # capture the launches in a HIP graph: Python/ctypes submission (~8 us/launch) would otherwise
                # starve the GPU and the sweep would time the host, not the kernel
                reps = 4 * copies
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
                gbs = nbytes / us / 1e3
                if best is None or us < best[0]:
                    best = (us, v, gbs)
                print(f"{name:8s} variant={v:3d} (big={rw} stream={(v >> 2) & 1} bpc={blocks})  {us:8.2f} us  "
                      f"{gbs:8.1f} GB/s", flush=True)
        res[name] = best
        print(f"BEST {name}: variant={best[1]} ({best[1] & 15}, {best[1] >> 4}) {best[0]:.2f} us {best[2]:.1f} GB/s",
              flush=True)
        del mats
        torch.cuda.empty_cache()
    print(res)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
