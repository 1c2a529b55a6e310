"""Stage-by-stage comparison of lga_decode_layer against the per-op kernels for one Llama-2-7B block."""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]

from lit_gpt import ops  # noqa: E402


@torch.inference_mode()
def main(p=37):
    from generate.base import build_model
    from lit_gpt import Config

    dev = torch.device("cuda")
    cfg = Config.from_name("Llama-2-7b-hf", n_layer=1, vocab_size=512, padding_multiple=64, block_size=4096)
    S = 128
    model = build_model(cfg, quantize="int4-g128", device=dev, seed=7, max_seq_length=S)
    blk = model.transformer.h[0]
    kv = blk.attn.kv_cache
    kv.k.normal_()
    kv.v.normal_()
    x = (torch.randn(cfg.n_embd, device=dev)).bfloat16()
    pos = torch.tensor([p], device=dev)
    cos, sin = model.cos.float().contiguous(), model.sin.float().contiguous()
    C, H, G, hs = cfg.n_embd, cfg.n_head, cfg.n_query_groups, cfg.head_size
    # per-op reference
    k_ref, v_ref = kv.k.clone(), kv.v.clone()
    at, mlp = blk.attn, blk.mlp
    qkv = ops.q4_gemv(x, at.attn.qweight, at.attn.scales, at.attn.out_features, C, 128, 0,
                      norm_weight=blk.norm_1.weight, eps=blk.norm_1.eps)
    q = ops.rope_kv_append(qkv.view(1, -1), k_ref, v_ref, pos, pos, cos, sin, H, G, hs, hs)
    y = ops.attention(q, k_ref, v_ref, pos, H, G, hs, hs ** -0.5, n_splits=1).view(-1)
    h_mid = ops.q4_gemv(y, at.proj.qweight, at.proj.scales, C, C, 128, 0, residual=x)
    act = ops.q4_gemv_swiglu(h_mid, mlp.fc_1.qweight, mlp.fc_1.scales, mlp.fc_2.qweight, mlp.fc_2.scales,
                             mlp.fc_1.out_features, C, 128, 0, norm_weight=blk.norm_2.weight, eps=blk.norm_2.eps)
    h_out = ops.q4_gemv(act, mlp.proj.qweight, mlp.proj.scales, C, mlp.fc_1.out_features, 128, 0, residual=h_mid)
    # layer kernel
    I = mlp.fc_1.out_features
    ws = ops.DecodeLayerWorkspace(C, I, H, G, hs, dev)
    k2, v2 = kv.k.clone(), kv.v.clone()
    out = ops.decode_layer(x, blk, cos, sin, pos, k2, v2, ws)
    torch.cuda.synchronize()
    print("err flag", int(ws.err.item()), "counters", int(ws.counters.abs().sum()))

    def cmp(name, a, b):
        a, b = a.float().view(-1), b.float().view(-1)
        d = (a - b).abs()
        i = int(d.argmax())
        print(f"{name:6s} max|diff| {d.max().item():10.4g} at {i} (ref {b[i].item():.4g} got {a[i].item():.4g})  "
              f"ref max {b.abs().max().item():.4g}  frac>1e-2 {(d > 1e-2 * b.abs().max()).float().mean().item():.4f}")

    cmp("qkv", ws.qkv, qkv)
    cmp("kcache", k2[0, :, p], k_ref[0, :, p])
    cmp("vcache", v2[0, :, p], v_ref[0, :, p])
    cmp("y", ws.y, y)
    cmp("h_mid", ws.h_mid, h_mid)
    cmp("act", ws.act, act)
    cmp("h_out", out, h_out)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
