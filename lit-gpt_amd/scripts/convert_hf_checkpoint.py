"""HuggingFace Llama / Mixtral checkpoint -> ``lit_model.pth`` + ``lit_config.json`` (the files generate/base.py,
generate/tp.py, generate/sequentially.py and chat/base.py load).

Follows /root/reference/scripts/convert_hf_checkpoint.py for the families whose blocks this build runs
(``LLaMAMLP`` / ``LLaMAMoE``): ``copy_weights_hf_llama`` (:111-188) — the same name map, the fused
``attn.attn.weight`` laid out per query group as ``[q_g (q_per_kv * hs rows), k_g (hs), v_g (hs)]``
(:174-188), q/k/v halves that arrive in different shard files held until all three are present — and
``convert_hf_checkpoint`` (:282-338): ``lit_config.json`` is ``asdict(Config.from_name(model_name))``, shards come
from ``pytorch_model.bin.index.json`` (or every ``*.bin`` but ``training_args.bin``). Differences:
  * ``*.safetensors`` shards (``model.safetensors.index.json``) are read too, through safetensors;
  * ``.bin`` shards load with ``torch.load(weights_only=True, mmap=True)`` — nothing in the file executes;
  * the whole converted state is written with one ``torch.save`` instead of the reference's incremental saver;
  * GPT-NeoX / Falcon / Phi layouts raise ``NotImplementedError`` (no MI355X blocks for them in this build).
"""

from __future__ import annotations

import argparse
import json
import re
import sys
from dataclasses import asdict
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import torch

wd = Path(__file__).parent.parent.resolve()
if str(wd) not in sys.path:
    sys.path.append(str(wd))

from lit_gpt import Config  # noqa: E402


def layer_template(name: str, idx: int) -> Tuple[str, int]:
    """``model.layers.7.mlp...`` -> (``model.layers.{}.mlp...``, 7): the ``idx``-th dotted field is the number."""
    split = name.split(".")
    number = int(split[idx])
    split[idx] = "{}"
    return ".".join(split), number


def _weight_map(config: Config) -> Dict[str, Optional[str]]:
    wm: Dict[str, Optional[str]] = {
        "model.embed_tokens.weight": "transformer.wte.weight",
        "model.layers.{}.input_layernorm.weight": "transformer.h.{l}.norm_1.weight",
        "model.layers.{}.input_layernorm.bias": "transformer.h.{l}.norm_1.bias",
        "model.layers.{}.self_attn.q_proj.weight": None,
        "model.layers.{}.self_attn.k_proj.weight": None,
        "model.layers.{}.self_attn.v_proj.weight": None,
        "model.layers.{}.self_attn.o_proj.weight": "transformer.h.{l}.attn.proj.weight",
        "model.layers.{}.self_attn.rotary_emb.inv_freq": None,
        "model.layers.{}.post_attention_layernorm.weight": "transformer.h.{l}.norm_2.weight",
        "model.layers.{}.post_attention_layernorm.bias": "transformer.h.{l}.norm_2.bias",
        "model.norm.weight": "transformer.ln_f.weight",
        "model.norm.bias": "transformer.ln_f.bias",
        "lm_head.weight": "lm_head.weight",
    }
    if config._mlp_class == "LLaMAMoE":
        moe = "model.layers.{}.block_sparse_moe."
        wm[moe + "gate.weight"] = "transformer.h.{l}.mlp.gate.weight"
        for hf, lit in (("w1", "fc_1"), ("w3", "fc_2"), ("w2", "proj")):
            wm[moe + "experts.{}." + hf + ".weight"] = "transformer.h.{l}.mlp.experts.{e}." + lit + ".weight"
    elif config._mlp_class == "LLaMAMLP":
        for hf, lit in (("gate_proj", "fc_1"), ("up_proj", "fc_2"), ("down_proj", "proj")):
            wm["model.layers.{}.mlp." + hf + ".weight"] = "transformer.h.{l}.mlp." + lit + ".weight"
    else:
        raise NotImplementedError(f"{config._mlp_class} checkpoints have no MI355X blocks in this build")
    return wm


def fuse_qkv(config: Config, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """HF q/k/v projections -> lit-gpt's fused weight, grouped per KV head (reference :180-188)."""
    hs = config.head_size
    q_per_kv = config.n_head // config.n_query_groups
    G = config.n_query_groups
    if q.shape[0] != config.n_head * hs or k.shape[0] != G * hs or v.shape[0] != G * hs:
        raise ValueError(f"q/k/v rows {q.shape[0]}/{k.shape[0]}/{v.shape[0]} do not match n_head={config.n_head},"
                         f" n_query_groups={G}, head_size={hs}")
    C = q.shape[1]
    fused = torch.cat((q.reshape(G, q_per_kv * hs, C), k.reshape(G, hs, C), v.reshape(G, hs, C)), dim=1)
    return fused.reshape(-1, C)


def copy_weights_hf_llama(config: Config, qkv_weights: Dict[int, List[Optional[torch.Tensor]]],
                          state_dict: Dict[str, torch.Tensor], hf_weights: Dict[str, torch.Tensor],
                          dtype: Optional[torch.dtype] = None) -> None:
    """Rename one shard's tensors into ``state_dict``; fuse each layer's q/k/v once all three have been seen."""
    wm = _weight_map(config)
    for name, param in hf_weights.items():
        if "model.layers" in name:
            from_name, layer = layer_template(name, 2)
            expert = None
            if "block_sparse_moe.experts" in name:
                from_name, expert = layer_template(from_name, 5)
            qkv = qkv_weights.setdefault(layer, [None, None, None])  # every layer seen gets a holder (:160)
            for i, key in enumerate(("q_proj", "k_proj", "v_proj")):
                if f"self_attn.{key}." in name:
                    qkv[i] = param
            if from_name not in wm:
                raise KeyError(f"unexpected checkpoint tensor {name!r}")
            to_name = wm[from_name]
            if to_name is None:
                continue
            to_name = to_name.format(l=layer, e=expert)
        else:
            if name not in wm:
                raise KeyError(f"unexpected checkpoint tensor {name!r}")
            to_name = wm[name]
        state_dict[to_name] = param if dtype is None else param.to(dtype)
    for layer, (q, k, v) in list(qkv_weights.items()):
        if q is None or k is None or v is None:
            continue  # the rest is in a later shard
        qkv = fuse_qkv(config, q, k, v)
        state_dict[f"transformer.h.{layer}.attn.attn.weight"] = qkv if dtype is None else qkv.to(dtype)
        del qkv_weights[layer]


def _load_shard(path: Path) -> Dict[str, torch.Tensor]:
    if path.suffix == ".safetensors":
        from safetensors.torch import load_file

        return load_file(str(path))
    try:
        return torch.load(str(path), map_location="cpu", mmap=True, weights_only=True)
    except RuntimeError as e:  # legacy (non-zip) .bin shards cannot be memory-mapped; load them whole
        if "mmap" not in str(e) and "zip" not in str(e):
            raise
        return torch.load(str(path), map_location="cpu", weights_only=True)


def expected_keys(config: Config) -> set:
    """State-dict names of GPT(config) (rope tables and KV caches are buffers, not checkpoint entries)."""
    from lit_gpt import GPT

    with torch.device("meta"):
        model = GPT(config)
    return {k for k in model.state_dict() if not k.endswith((".cos", ".sin")) and k not in ("cos", "sin")
            and ".kv_cache." not in k}


def shard_files(checkpoint_dir: Path) -> List[Path]:
    for index in ("model.safetensors.index.json", "pytorch_model.bin.index.json"):
        p = checkpoint_dir / index
        if p.is_file():
            with open(p) as fp:
                return sorted({checkpoint_dir / f for f in json.load(fp)["weight_map"].values()})
    files = sorted(checkpoint_dir.glob("*.safetensors"))
    if not files:
        files = sorted(f for f in checkpoint_dir.glob("*.bin") if f.name != "training_args.bin")
    if not files:
        raise ValueError(f"Expected {str(checkpoint_dir)!r} to contain .bin or .safetensors files")
    return files


@torch.inference_mode()
def convert_hf_checkpoint(*, checkpoint_dir: Path = Path("checkpoints/meta-llama/Llama-2-7b-hf"),
                          model_name: Optional[str] = None, dtype: Optional[str] = None) -> None:
    checkpoint_dir = Path(checkpoint_dir)
    model_name = model_name or checkpoint_dir.name
    tdtype = getattr(torch, dtype) if dtype is not None else None
    config = Config.from_name(model_name)
    if re.search("falcon|phi", model_name) or config._mlp_class not in ("LLaMAMLP", "LLaMAMoE"):
        raise NotImplementedError(f"{model_name}: only Llama-family (LLaMAMLP / LLaMAMoE) layouts are converted")
    config_dict = asdict(config)
    print(f"Model config {config_dict}")
    with open(checkpoint_dir / "lit_config.json", "w") as fp:
        json.dump(config_dict, fp)
    qkv_weights: Dict[int, List[Optional[torch.Tensor]]] = {}
    sd: Dict[str, torch.Tensor] = {}
    for f in shard_files(checkpoint_dir):
        print("Processing", f)
        copy_weights_hf_llama(config, qkv_weights, sd, _load_shard(f), dtype=tdtype)
    partial = sorted(l for l, qkv in qkv_weights.items() if any(t is not None for t in qkv))
    if partial:
        raise ValueError(f"layers {partial} are missing q, k or v projections")
    want = expected_keys(config)
    missing, extra = sorted(want - set(sd)), sorted(set(sd) - want)
    if missing or extra:  # fail here, not later as a KeyError in generate/base.py build_model
        raise ValueError(f"converted state does not match {model_name}: missing {missing[:8]}"
                         f"{' ...' if len(missing) > 8 else ''}, unexpected {extra[:8]}{' ...' if len(extra) > 8 else ''}")
    # RAM: the whole converted state is held until this single save (~2 bytes/param with --dtype bfloat16, e.g.
    # ~140 GB for Llama-2-70B); shards are memory-mapped while converting
    print("Saving converted checkpoint")
    torch.save(sd, checkpoint_dir / "lit_model.pth")


def _cli(argv=None) -> None:
    p = argparse.ArgumentParser(description="Convert a HuggingFace Llama-family checkpoint to lit_model.pth")
    p.add_argument("--checkpoint_dir", type=Path, default=Path("checkpoints/meta-llama/Llama-2-7b-hf"))
    p.add_argument("--model_name", default=None)
    p.add_argument("--dtype", default=None)
    a = p.parse_args(argv)
    convert_hf_checkpoint(checkpoint_dir=a.checkpoint_dir, model_name=a.model_name, dtype=a.dtype)


if __name__ == "__main__":
    _cli()
