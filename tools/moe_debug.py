"""Lab: one LLaMAMoE layer on the GPU vs a CPU torch restatement with the same dequantized weights."""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]

from oracle import model as om  # noqa: E402
from tests.test_gpu_model import _cfg, build_gpu_model, oracle_for  # noqa: E402
from oracle import synth  # noqa: E402


@torch.inference_mode()
def main():
    cfg = _cfg("moe")
    sd = synth.state_dict(cfg, seed=21)
    model = build_gpu_model(cfg, sd, "int4-g128", 64)
    ref = oracle_for(cfg, sd, "int4-g128")
    blk = model.transformer.h[0]
    C = cfg.n_embd
    for T in (1, 5):
        x = torch.randn(T, C).bfloat16()
        got = blk.mlp(x.view(1, T, C).cuda(), norm=blk.norm_2, residual=x.view(1, T, C).cuda()).view(T, C).cpu()
        n = om.rms_norm(x, ref.p["transformer.h.0.norm_2.weight"], cfg.norm_eps)
        router = ref._lin("transformer.h.0.mlp.gate", n)
        gr = model.transformer.h[0].mlp.gate(blk.norm_2(x.cuda())).cpu()
        print("T", T, "router max diff", (router.float() - gr.float()).abs().max().item())
        exp = x + ref._mlp(0, n)
        d = (got.float() - exp.float()).abs()
        print("  out max diff", d.max().item(), "ref max", exp.abs().max().item())
        probs, idx = torch.topk(router, 2)
        ids, pr = __import__("lit_gpt").ops.moe_route(gr.cuda().contiguous(), 2)
        print("  ids ref", idx.tolist(), "gpu", ids.cpu().tolist())


if __name__ == "__main__":
    main()


@torch.inference_mode()
def full():
    cfg = _cfg("moe")
    sd = synth.state_dict(cfg, seed=21)
    T, N = 20, 12
    model = build_gpu_model(cfg, sd, "int4-g128", T + N)
    ref = oracle_for(cfg, sd, "int4-g128")
    ref.set_kv_cache(T + N)
    g_router, r_router = [], []
    for i, b in enumerate(model.transformer.h):
        b.mlp.gate.register_forward_hook(lambda m, a, o, i=i: g_router.append((i, o.float().cpu().view(-1, 8))))
    orig = ref._lin

    def lin(name, x, *a, **k):
        y = orig(name, x, *a, **k)
        if name.endswith("mlp.gate"):
            r_router.append((int(name.split(".")[2]), y.float().view(-1, 8)))
        return y

    ref._lin = lin
    prompt = torch.from_numpy(synth.token_ids(T, cfg.vocab_size, seed=21))
    stream = torch.from_numpy(synth.token_ids(N, cfg.vocab_size, seed=22))
    dev = torch.device("cuda")
    got = [model(prompt.view(1, -1).to(dev), torch.arange(T, device=dev))[0, -1].float().cpu()]
    exp = [ref.forward(prompt, torch.arange(T))[-1].float()]
    for i in range(N - 1):
        got.append(model(stream[i:i + 1].view(1, 1).to(dev), torch.tensor([T + i], device=dev))[0, -1].float().cpu())
        exp.append(ref.forward(stream[i:i + 1], torch.tensor([T + i]))[-1].float())
    for s, (g, e) in enumerate(zip(got, exp)):
        print("step", s, "err", (g - e).abs().max().item(), "max", e.abs().max().item())
    for (li, gr), (lr, rr) in zip(g_router, r_router):
        gi = torch.topk(gr.bfloat16(), 2).indices
        ri = torch.topk(rr.bfloat16(), 2).indices
        print("layer", li, lr, "router diff", (gr - rr).abs().max().item(), "ids equal", torch.equal(gi, ri))


if __name__ == "__main__":
    full()
