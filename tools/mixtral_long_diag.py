"""Localise a full-width Mixtral one-block prefill mismatch: the same model's logits with the grouped expert GEMMs
vs the per-expert loop, and with the MFMA flash attention vs a torch fp32 softmax, at several prompt lengths.

usage: python tools/mixtral_long_diag.py [T ...]
"""

import math
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO), str(REPO / "tests")]

from oracle import synth  # noqa: E402


def rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-30))


@torch.inference_mode()
def main():
    from generate.base import build_model
    from lit_gpt import Config, ops
    from lit_gpt import model as M

    dev = torch.device("cuda")
    Ts = [int(v) for v in sys.argv[1:] if not v.startswith("--")] or [1024, 4096, 8192]
    cfg = Config.from_name("Mixtral-8x7B-v0.1", n_layer=1)
    model = build_model(cfg, quantize="int4-g128", device=dev, seed=11, max_seq_length=max(Ts) + 2)
    moe = model.transformer.h[0].mlp
    if "--experts" in sys.argv:
        from oracle import quant
        import numpy as np
        torch.manual_seed(0)
        x = torch.randn(64, cfg.n_embd, device=dev).bfloat16()
        rec = {}
        orig_route = ops.moe_route

        def spy(router, k):
            ids, probs = orig_route(router, k)
            rec["ids"], rec["probs"] = ids.clone(), probs.clone()
            return ids, probs

        ops.moe_route = spy
        y = moe(x.view(1, 64, -1)).view(64, -1).float()
        ops.moe_route = orig_route

        def deq(lin):
            qw = lin.qweight.cpu().numpy()
            sc = lin.scales.view(torch.int16).cpu().numpy().view(np.uint16)
            return torch.from_numpy(quant.dequantize_q4g(qw, sc, lin.group)).float().to(dev)

        W = {e: {n: deq(getattr(moe.experts[e], n)) for n in ("fc_1", "fc_2", "proj")} for e in range(cfg.n_expert)}
        ref = torch.zeros(64, cfg.n_embd, device=dev)
        xf = x.float()
        for t in range(64):
            for sl in range(2):
                e = int(rec["ids"][t, sl])
                w = W[e]
                h = torch.nn.functional.silu(xf[t] @ w["fc_1"].T) * (xf[t] @ w["fc_2"].T)
                ref[t] += float(rec["probs"][t, sl]) * (h @ w["proj"].T)
        d = (y - ref).abs().amax(-1) / ref.abs().amax(-1)
        for t in range(64):
            if d[t] > 0.03:
                print(f"row {t}: rel {float(d[t]):.3f} experts {rec['ids'][t].tolist()}", flush=True)
        print(f"experts check: worst {float(d.max()):.4f}; expert counts "
              f"{torch.bincount(rec['ids'].view(-1).long(), minlength=cfg.n_expert).tolist()}", flush=True)
        # per-expert single-linear check
        for e in range(cfg.n_expert):
            lin = moe.experts[e].fc_1
            yy = ops.q4_gemm(x, lin.qweight, lin.scales, lin.out_features, cfg.n_embd, lin.group, lin.fmt).float() \
                if hasattr(ops, "q4_gemm") else None
            if yy is not None:
                print(f"expert {e} fc_1 gemm rel {rel(yy, xf @ W[e]['fc_1'].T):.4f}", flush=True)
        return
    if "--oracle" in sys.argv:
        from oracle import model as om
        from test_gpu_geometry import oracle_state_from_model

        sd = oracle_state_from_model(model)
        og = om.OracleGPT(cfg, sd, dtype=torch.bfloat16, rope_pos_dtype=torch.bfloat16)
        for T in Ts:
            prompt = torch.from_numpy(synth.token_ids(T, cfg.vocab_size, seed=11)).to(dev)
            model.transformer.h[0].attn.kv_cache.reset_parameters()
            lg = model(prompt.view(1, -1), torch.arange(T, device=dev))[0].float().cpu()
            rows = sorted({0, 1, 255, 256, 257, T // 2, T - 1} | set(range(max(0, T - 6), T)) |
                          ({507, 508, 509, 510, 511} if T > 512 else set()))
            print(f"T={T}: tokens " + " ".join(f"{r}:{int(prompt[r])}" for r in rows), flush=True)
            rec = {}
            orig_route = ops.moe_route

            def spy(router, k):
                rec["router"] = router.float().cpu()
                return orig_route(router, k)

            ops.moe_route = spy
            model.transformer.h[0].attn.kv_cache.reset_parameters()
            model(prompt.view(1, -1), torch.arange(T, device=dev))
            ops.moe_route = orig_route
            for r in (T - 2, T - 1):
                v, i = torch.sort(rec["router"][r], descending=True)
                print(f"  row {r}: router top-4 {[round(float(x), 5) for x in v[:4]]} experts {i[:4].tolist()}")
            ref = om.one_block_rows(og, prompt.cpu().long(), rows)
            print(f"T={T}: product vs bf16 oracle per row: " +
                  " ".join(f"{r}:{rel(lg[r], ref[i]):.3f}" for i, r in enumerate(rows)), flush=True)
        return
    for T in Ts:
        prompt = torch.from_numpy(synth.token_ids(T, cfg.vocab_size, seed=11)).to(dev)
        outs = {}
        orig = M.LLaMAMoE._grouped_ok
        for name, grouped in (("grouped", True), ("loop", False)):
            M.LLaMAMoE._grouped_ok = orig if grouped else (lambda self, C: False)
            model.transformer.h[0].attn.kv_cache.reset_parameters()
            outs[name] = model(prompt.view(1, -1), torch.arange(T, device=dev))[0].float()
        M.LLaMAMoE._grouped_ok = orig
        d = (outs["grouped"] - outs["loop"]).abs().amax(-1) / outs["loop"].abs().amax(-1)
        bad = (d > 0.05).nonzero().view(-1)
        print(f"T={T}: grouped vs loop logits rel max {float(d.max()):.4f}, rows > 5%: {bad.numel()}"
              f" (first {bad[:8].tolist()})", flush=True)
        # MoE alone on random x, grouped vs loop
        x = torch.randn(1, T, cfg.n_embd, device=dev).bfloat16()
        M.LLaMAMoE._grouped_ok = lambda self, C: False
        y_loop = moe(x)
        M.LLaMAMoE._grouped_ok = orig
        y_grp = moe(x)
        d = (y_grp - y_loop).float().abs().amax(-1) / y_loop.float().abs().amax(-1)
        bad = (d.view(-1) > 0.05).nonzero().view(-1)
        print(f"T={T}: MoE grouped vs loop rel max {float(d.max()):.4f}, rows > 5%: {bad.numel()}"
              f" (first {bad[:8].tolist()})", flush=True)
        # flash attention, Mixtral geometry, vs fp32 torch on sampled rows
        H, G, hs = cfg.n_head, cfg.n_query_groups, cfg.head_size
        q = torch.randn(T, H, hs, device=dev).bfloat16()
        k = torch.randn(G, T, hs, device=dev).bfloat16()
        v = torch.randn(G, T, hs, device=dev).bfloat16()
        y = ops.attention(q, k, v, torch.arange(T, device=dev), H, G, hs, 1.0 / math.sqrt(hs)).float().view(T, H, hs)
        worst = 0.0
        for t in sorted({0, 127, 128, T // 2, T - 129, T - 128, T - 1}):
            for h in (0, 13, 31):
                kk, vv = k[h // (H // G), : t + 1].float(), v[h // (H // G), : t + 1].float()
                ref = torch.softmax(kk @ q[t, h].float() / math.sqrt(hs), 0) @ vv
                worst = max(worst, rel(y[t, h], ref))
        print(f"T={T}: flash attention sampled rows rel max {worst:.4f}", flush=True)


if __name__ == "__main__":
    main()
