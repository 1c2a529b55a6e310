"""CPU tests of scripts/convert_hf_checkpoint.py (reference tests/test_convert_hf_checkpoint.py): the 70B shape
case, the fused-qkv group interleave against the reference formula, and a full round trip through sharded
safetensors / .bin files into lit_model.pth + lit_config.json that generate/base.py's loader reads."""

import json

import pytest
import torch


def test_llama2_70b_conversion_shapes():
    from lit_gpt import Config
    from scripts.convert_hf_checkpoint import copy_weights_hf_llama

    C, I = 8192, 28672
    layer = {"input_layernorm.weight": (C,), "mlp.down_proj.weight": (C, I), "mlp.gate_proj.weight": (I, C),
             "mlp.up_proj.weight": (I, C), "post_attention_layernorm.weight": (C,),
             "self_attn.o_proj.weight": (C, C)}
    shapes = {"model.embed_tokens.weight": (32000, C)}
    for l in range(5):
        shapes.update({f"model.layers.{l}.{k}": s for k, s in layer.items()})
    shapes.update({"model.layers.0.self_attn.k_proj.weight": (1024, C), "model.layers.0.self_attn.q_proj.weight":
                   (C, C), "model.layers.0.self_attn.v_proj.weight": (1024, C),
                   "model.layers.5.mlp.gate_proj.weight": (I, C), "model.layers.5.self_attn.o_proj.weight": (C, C)})
    config = Config.from_name("Llama-2-70b-hf")
    holder, qkv_weights = {}, {}
    with torch.device("meta"):
        weights = {k: torch.empty(s) for k, s in shapes.items()}
    copy_weights_hf_llama(config, qkv_weights, holder, weights)
    assert len(qkv_weights) == 5 and all(v is None for qkv in qkv_weights.values() for v in qkv)
    got = {k: tuple(t.shape) for k, t in holder.items()}
    want = {"transformer.wte.weight": (32000, C), "transformer.h.0.attn.attn.weight": (10240, C),
            "transformer.h.5.attn.proj.weight": (C, C), "transformer.h.5.mlp.fc_1.weight": (I, C)}
    for l in range(5):
        want.update({f"transformer.h.{l}.attn.proj.weight": (C, C), f"transformer.h.{l}.mlp.fc_1.weight": (I, C),
                     f"transformer.h.{l}.mlp.fc_2.weight": (I, C), f"transformer.h.{l}.mlp.proj.weight": (C, I),
                     f"transformer.h.{l}.norm_1.weight": (C,), f"transformer.h.{l}.norm_2.weight": (C,)})
    assert got == want


@pytest.mark.parametrize("n_head,G", [(8, 8), (8, 2), (8, 1)])
def test_fuse_qkv_matches_reference_interleave(n_head, G):
    from lit_gpt import Config
    from scripts.convert_hf_checkpoint import fuse_qkv

    cfg = Config.from_name("Llama-2-7b-hf", n_embd=64, n_head=n_head, n_query_groups=G)
    hs = cfg.head_size
    g = torch.Generator().manual_seed(0)
    q, k, v = (torch.randn(r, 64, generator=g) for r in (n_head * hs, G * hs, G * hs))
    # reference scripts/convert_hf_checkpoint.py:180-187: split, zip per group, cat
    qs, ks, vs = torch.split(q, hs * (n_head // G)), torch.split(k, hs), torch.split(v, hs)
    ref = torch.cat([t for grp in zip(qs, ks, vs) for t in grp])
    assert torch.equal(fuse_qkv(cfg, q, k, v), ref)
    with pytest.raises(ValueError):
        fuse_qkv(cfg, q[:-1], k, v)


def _hf_state(cfg, lit):
    """Invert the conversion: a lit state dict -> HF names with split q/k/v."""
    hs, G = cfg.head_size, cfg.n_query_groups
    qpk = cfg.n_head // G
    hf = {"model.embed_tokens.weight": lit["transformer.wte.weight"], "model.norm.weight":
          lit["transformer.ln_f.weight"], "lm_head.weight": lit["lm_head.weight"]}
    for l in range(cfg.n_layer):
        p = f"transformer.h.{l}."
        w = lit[p + "attn.attn.weight"].view(G, (qpk + 2) * hs, -1)
        hf[f"model.layers.{l}.self_attn.q_proj.weight"] = w[:, :qpk * hs].reshape(-1, w.shape[-1]).clone()
        hf[f"model.layers.{l}.self_attn.k_proj.weight"] = w[:, qpk * hs:(qpk + 1) * hs].reshape(-1, w.shape[-1]).clone()
        hf[f"model.layers.{l}.self_attn.v_proj.weight"] = w[:, (qpk + 1) * hs:].reshape(-1, w.shape[-1]).clone()
        hf[f"model.layers.{l}.self_attn.o_proj.weight"] = lit[p + "attn.proj.weight"]
        hf[f"model.layers.{l}.input_layernorm.weight"] = lit[p + "norm_1.weight"]
        hf[f"model.layers.{l}.post_attention_layernorm.weight"] = lit[p + "norm_2.weight"]
        if cfg._mlp_class == "LLaMAMoE":
            hf[f"model.layers.{l}.block_sparse_moe.gate.weight"] = lit[p + "mlp.gate.weight"]
            for e in range(cfg.n_expert):
                for h, n in (("w1", "fc_1"), ("w3", "fc_2"), ("w2", "proj")):
                    hf[f"model.layers.{l}.block_sparse_moe.experts.{e}.{h}.weight"] = lit[f"{p}mlp.experts.{e}.{n}.weight"]
        else:
            for h, n in (("gate_proj", "fc_1"), ("up_proj", "fc_2"), ("down_proj", "proj")):
                hf[f"model.layers.{l}.mlp.{h}.weight"] = lit[f"{p}mlp.{n}.weight"]
    return hf


@pytest.mark.parametrize("name,kw,fmt", [
    ("Llama-2-70b-hf", dict(n_layer=2, n_embd=128, n_head=8, n_query_groups=2, intermediate_size=96), "safetensors"),
    ("Mixtral-8x7B-v0.1", dict(n_layer=2, n_embd=64, n_head=4, n_query_groups=2, intermediate_size=32), "bin")])
def test_convert_round_trip(tmp_path, monkeypatch, name, kw, fmt):
    import scripts.convert_hf_checkpoint as cth
    from lit_gpt import GPT, Config

    cfg = Config.from_name(name, vocab_size=100, padding_multiple=64, block_size=32, **kw)
    torch.manual_seed(0)
    lit = {k: torch.randn_like(v) for k, v in GPT(cfg).state_dict().items() if not k.endswith(("cos", "sin"))}
    hf = _hf_state(cfg, lit)
    # two shards with layer 0's q in the first and its k/v in the second (the "split across files" case)
    names = sorted(hf)
    first = [n for n in names if "layers.0.self_attn.q_proj" in n or "embed" in n or "layers.1" in n]
    shards = {f"model-00001.{fmt}": first, f"model-00002.{fmt}": [n for n in names if n not in first]}
    for fname, keys in shards.items():
        part = {k: hf[k].contiguous() for k in keys}
        if fmt == "safetensors":
            from safetensors.torch import save_file
            save_file(part, str(tmp_path / fname))
        else:
            torch.save(part, tmp_path / fname)
    index = "model.safetensors.index.json" if fmt == "safetensors" else "pytorch_model.bin.index.json"
    (tmp_path / index).write_text(json.dumps({"weight_map": {k: f for f, ks in shards.items() for k in ks}}))

    class TinyConfig(Config):
        @classmethod
        def from_name(cls, n, **k):
            return Config.from_name(n, vocab_size=100, padding_multiple=64, block_size=32, **kw)

    monkeypatch.setattr(cth, "Config", TinyConfig)
    cth.convert_hf_checkpoint(checkpoint_dir=tmp_path, model_name=name)
    out = torch.load(tmp_path / "lit_model.pth", weights_only=True)
    assert set(out) == set(lit)
    for k in lit:
        assert torch.equal(out[k], lit[k]), k
    back = Config.from_json(tmp_path / "lit_config.json")
    assert (back.n_layer, back.n_query_groups, back._mlp_class) == (cfg.n_layer, cfg.n_query_groups, cfg._mlp_class)


def test_convert_rejects_unsupported(tmp_path):
    from scripts.convert_hf_checkpoint import convert_hf_checkpoint

    with pytest.raises(NotImplementedError):
        convert_hf_checkpoint(checkpoint_dir=tmp_path, model_name="pythia-14m")


def test_convert_rejects_a_layer_without_attention(tmp_path, monkeypatch):
    """A shard set whose layer 1 has no q/k/v at all is refused at conversion time (not later as a KeyError in
    generate/base.py build_model)."""
    import scripts.convert_hf_checkpoint as cth
    from lit_gpt import GPT, Config
    from safetensors.torch import save_file

    kw = dict(n_layer=2, n_embd=64, n_head=4, n_query_groups=2, intermediate_size=32)
    cfg = Config.from_name("Llama-2-7b-hf", vocab_size=100, padding_multiple=64, block_size=32, **kw)
    lit = {k: torch.randn_like(v) for k, v in GPT(cfg).state_dict().items() if not k.endswith(("cos", "sin"))}
    hf = {k: v.contiguous() for k, v in _hf_state(cfg, lit).items() if ".layers.1.self_attn." not in k
          or "o_proj" in k}
    save_file(hf, str(tmp_path / "model.safetensors"))

    class TinyConfig(Config):
        @classmethod
        def from_name(cls, n, **k):
            return Config.from_name(n, vocab_size=100, padding_multiple=64, block_size=32, **kw)

    monkeypatch.setattr(cth, "Config", TinyConfig)
    with pytest.raises(ValueError, match="transformer.h.1.attn.attn.weight"):
        cth.convert_hf_checkpoint(checkpoint_dir=tmp_path, model_name="Llama-2-7b-hf")
    assert not (tmp_path / "lit_model.pth").exists()
