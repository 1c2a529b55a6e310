"""Lab (round 6): the fused int4 prefill GEMM's 4-wave 128 x 128 tile (LGA_Q4F_W4=1, two
workgroups per CU) against the default 8-wave tiles — outputs and rates.

usage: make -C lit-gpt_amd/csrc lab-lib LABSRC=gemm_q4f LABFLAGS=-DLGA_Q4F_W4_LAB LABLIB=../../tools/_lab/liblitgpt_w4.so
       LGA_Q4F_W4=1 python tools/q4f_tile_ab.py save OUT.pt [M] [LIB]   (and once without the env / LIB)
       python tools/q4f_tile_ab.py compare A.pt B.pt
The saved file holds every 7B layer GEMM's output (qkv, proj + residual, fc_1 || fc_2 + SwiGLU, down + residual) on
fixed seeded inputs; compare reports bit equality per GEMM.
"""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]


def save(out, M, lib=None):
    from lit_gpt import ops

    if lib:
        ops._lib = ops.load_library(Path(lib))
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(7)
    res = {}
    for name, (N, K, dual) in {"qkv": (12288, 4096, False), "proj": (4096, 4096, False), "fc": (11008, 4096, True),
                               "down": (4096, 11008, False)}.items():
        x = (torch.randn(M, K, generator=g) * 0.5).bfloat16().to(dev)
        w1 = (torch.randn(N, K, generator=g) * 0.02).to(dev)
        group = 128 if K % 128 == 0 else 64
        qw, sc = ops.quantize(w1, ops.FMT_Q4G, group)
        if dual:
            qw2, sc2 = ops.quantize((torch.randn(N, K, generator=g) * 0.02).to(dev), ops.FMT_Q4G, group)
            y = ops.q4_gemm_swiglu(x, qw, sc, qw2, sc2, N, K, group, ops.FMT_Q4G)
        else:
            r = (torch.randn(M, N, generator=g) * 0.5).bfloat16().to(dev) if name in ("proj", "down") else None
            y = ops.q4_gemm_fused(x, qw, sc, N, K, group, ops.FMT_Q4G, residual=r)
        torch.cuda.synchronize()
        res[name] = y.cpu()
    torch.save(res, out)
    print("saved", out, {k: tuple(v.shape) for k, v in res.items()}, flush=True)


def compare(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    ok = True
    for k in A:
        same = torch.equal(A[k], B[k])
        d = (A[k].float() - B[k].float()).abs().max().item()
        print(f"{k:5s} bit-identical {same}  max |diff| {d:.3e}", flush=True)
        ok &= same
    raise SystemExit(0 if ok else 1)


if __name__ == "__main__":
    if sys.argv[1] == "save":
        save(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 2048, sys.argv[4] if len(sys.argv) > 4 else None)
    else:
        compare(sys.argv[2], sys.argv[3])
