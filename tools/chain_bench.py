"""Times the chained decode GEMVs (lga_q4_decode_chain) against the same four GEMVs launched one by one.

32 Llama-2-7B blocks' worth of distinct int4-g128 weights (attn.proj, fc_1, fc_2, mlp.proj, next qkv), each
variant captured in one HIP graph over all 32 blocks and replayed; prints us per block and the weight-stream rate.
usage: python tools/chain_bench.py [--layers 32] [--reps 20]
"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "lit-gpt_amd"))
import torch  # noqa: E402

from lit_gpt import ops  # noqa: E402
from lit_gpt.quantize import QuantLinear  # noqa: E402
from lit_gpt.rmsnorm import RMSNorm  # noqa: E402


def lin(N, K, dev):
    return QuantLinear.from_float(torch.randn(N, K, device=dev) * 0.02, None, "int4-g128", dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--C", type=int, default=4096)
    ap.add_argument("--I", type=int, default=11008)
    ap.add_argument("--Nn", type=int, default=12288)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    C, I, Nn = a.C, a.I, a.Nn
    L = []
    for _ in range(a.layers):
        n2, nn_ = RMSNorm(C).to(dev).to(torch.bfloat16), RMSNorm(C).to(dev).to(torch.bfloat16)
        L.append(dict(proj=lin(C, C, dev), f1=lin(I, C, dev), f2=lin(I, C, dev), down=lin(C, I, dev),
                      nxt=lin(Nn, C, dev), n2=n2, nn=nn_))
    wbytes = sum(m.qweight.numel() + m.scales.numel() * 2 for l in L for m in
                 (l["proj"], l["f1"], l["f2"], l["down"], l["nxt"]))
    y_att = torch.randn(C, device=dev).to(torch.bfloat16)
    x_in = torch.randn(C, device=dev).to(torch.bfloat16)
    ws = ops.ChainWorkspace(dev)
    outs_c = [(torch.empty(C, dtype=torch.bfloat16, device=dev), torch.empty(Nn, dtype=torch.bfloat16, device=dev))
              for _ in L]

    def per_op():
        res = []
        for l in L:
            h_mid = ops.q4_gemv(y_att, l["proj"].qweight, l["proj"].scales, C, C, 128, 0, residual=x_in)
            act = ops.q4_gemv_swiglu(h_mid, l["f1"].qweight, l["f1"].scales, l["f2"].qweight, l["f2"].scales, I, C,
                                     128, 0, norm_weight=l["n2"].weight, eps=1e-5)
            h = ops.q4_gemv(act, l["down"].qweight, l["down"].scales, C, I, 128, 0, residual=h_mid)
            res.append(ops.q4_gemv(h, l["nxt"].qweight, l["nxt"].scales, Nn, C, 128, 0, norm_weight=l["nn"].weight,
                                   eps=1e-5, variant=0))
        return res

    def chained():
        res = []
        for l, (ho, o) in zip(L, outs_c):
            res.append(ops.q4_decode_chain(y_att, x_in, l["proj"], l["f1"], l["f2"], l["n2"], l["down"], l["nxt"],
                                           l["nn"], ws, out=o)[1])
        return res

    s = torch.cuda.Stream()
    results = {}
    for name, fn in (("per_op", per_op), ("chain", chained)):
        with torch.cuda.stream(s):
            fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                out = fn()
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.reps):
                g.replay()
            e1.record(s)
            torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        results[name] = [o.clone() for o in out]
        print(f"{name:7s} {ms * 1e3 / a.layers:8.2f} us/block  {wbytes / (ms * 1e-3) / 1e9:8.1f} GB/s "
              f"(weights {wbytes / a.layers / 1e6:.1f} MB/block)", flush=True)
    same = all(torch.equal(p, q) for p, q in zip(results["per_op"], results["chain"]))
    print(f"chain == per_op: {same}; err word {int(ws.err.item())}", flush=True)


if __name__ == "__main__":
    main()
