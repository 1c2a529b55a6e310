"""Model hyper-parameters for the MI355X decode path.

Mirrors the public surface of the reference ``Config`` dataclass
(/root/reference/lit_gpt/config.py:16-144): the same field names and defaults, the same derived
fields computed in ``__post_init__`` (``head_size``, ``padded_vocab_size``, ``n_query_groups``,
``intermediate_size``, ``rope_n_elem``; reference :63-89), ``from_name`` / ``from_json`` /
``from_checkpoint`` (:91-130) and the ``mlp_class`` / ``norm_class`` indirection (:132-144).

Only the model families this build targets are registered ("fields + the 4 target
configs"): GPT-NeoX/pythia (CPU plumbing config), Llama-2 7B/13B/70B (+chat), Mixtral-8x7B, plus
the tiny configs the test-suite uses.
"""

from __future__ import annotations

import json
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, List, Literal, Optional, Type, Union

from lit_gpt.utils import find_multiple


@dataclass
class Config:
    name: str = ""
    hf_config: dict = field(default_factory=dict)
    block_size: int = 4096
    vocab_size: int = 50254
    padding_multiple: int = 512
    padded_vocab_size: Optional[int] = None
    n_layer: int = 16
    n_head: int = 32
    n_embd: int = 4096
    rotary_percentage: float = 0.25
    parallel_residual: bool = True
    bias: bool = True
    lm_head_bias: bool = False
    # MHA: n_query_groups == n_head; MQA: 1; GQA: in between (reference :31-50)
    n_query_groups: Optional[int] = None
    shared_attention_norm: bool = False
    _norm_class: Literal["LayerNorm", "RMSNorm"] = "LayerNorm"
    norm_eps: float = 1e-5
    _mlp_class: Literal["GptNeoxMLP", "LLaMAMLP", "LLaMAMoE"] = "GptNeoxMLP"
    gelu_approximate: str = "none"
    intermediate_size: Optional[int] = None
    rope_condense_ratio: int = 1
    rope_base: int = 10000
    n_expert: int = 0
    n_expert_per_token: int = 0

    def __post_init__(self) -> None:
        if not self.name:
            self.name = self.hf_config.get("name", self.name)
        assert self.n_embd % self.n_head == 0
        self.head_size = self.n_embd // self.n_head
        if self.padded_vocab_size is None:
            self.padded_vocab_size = find_multiple(self.vocab_size, self.padding_multiple)
        else:
            self.vocab_size = min(self.vocab_size, self.padded_vocab_size)
        if self.n_query_groups is None:
            self.n_query_groups = self.n_head
        else:
            assert self.n_head % self.n_query_groups == 0
        if self.intermediate_size is None:
            if self._mlp_class == "LLaMAMLP":
                raise ValueError("The config needs to set the `intermediate_size`")
            self.intermediate_size = 4 * self.n_embd
        self.rope_n_elem = int(self.rotary_percentage * self.head_size)

    @classmethod
    def from_name(cls, name: str, **kwargs: Any) -> "Config":
        conf = name_to_config.get(name)
        if conf is None:
            conf = next((c for c in configs if c["hf_config"].get("name") == name), None)
            if conf is None:
                raise ValueError(f"{name!r} is not a supported config name")
        conf = dict(conf)
        if "condense_ratio" in kwargs:  # legacy spelling
            kwargs["rope_condense_ratio"] = kwargs.pop("condense_ratio")
        conf.update(kwargs)
        return cls(**conf)

    @classmethod
    def from_json(cls, path: Union[str, Path], **kwargs: Any) -> "Config":
        with open(path, encoding="utf-8") as fp:
            loaded = json.load(fp)
        for d in (loaded, kwargs):
            if "condense_ratio" in d:
                d["rope_condense_ratio"] = d.pop("condense_ratio")
        if "org" in loaded:
            loaded["hf_config"] = {"name": loaded["name"], "org": loaded.pop("org")}
        if "org" in kwargs:
            kwargs["hf_config"] = {"name": kwargs.get("name", loaded["name"]), "org": kwargs.pop("org")}
        loaded.update(kwargs)
        return cls(**loaded)

    @classmethod
    def from_checkpoint(cls, path: Path, **kwargs: Any) -> "Config":
        path = Path(path)
        if (path / "lit_config.json").is_file():
            return cls.from_json(path / "lit_config.json", **kwargs)
        if path.name in name_to_config:
            return cls.from_name(path.name, **kwargs)
        raise FileNotFoundError(f"For {str(path)!r} neither 'lit_config.json' nor matching config exists.")

    @property
    def mlp_class(self) -> Type:
        import lit_gpt.model

        return getattr(lit_gpt.model, self._mlp_class)

    @property
    def norm_class(self) -> Type:
        if self._norm_class == "RMSNorm":
            from lit_gpt.rmsnorm import RMSNorm

            return RMSNorm
        import lit_gpt.model

        return getattr(lit_gpt.model, self._norm_class)


# --------------------------------------------------------------------------------------------
# Registry. Values follow the HF configs the reference cites (pythia: config.py:200-260,
# Llama-2: :726-776, Mixtral: :1290-1307).
# --------------------------------------------------------------------------------------------
configs: List[Dict[str, Any]] = []


def _register(name: str, org: str, **kw: Any) -> None:
    configs.append(dict(name=name, hf_config=dict(org=org, name=name), **kw))


for _name, _block, _layers, _embd, _heads in (
    ("pythia-14m", 512, 6, 128, 4),
    ("pythia-31m", 1024, 6, 256, 8),
    ("pythia-70m", 2048, 6, 512, 8),
    ("pythia-160m", 2048, 12, 768, 12),
    ("pythia-410m", 2048, 24, 1024, 16),
    ("pythia-1b", 2048, 16, 2048, 8),
):
    _register(_name, "EleutherAI", block_size=_block, n_layer=_layers, n_embd=_embd, n_head=_heads,
              padding_multiple=128)

_LLAMA2 = dict(vocab_size=32000, padding_multiple=64, rotary_percentage=1.0, parallel_residual=False,
               bias=False, _norm_class="RMSNorm", _mlp_class="LLaMAMLP")
for _kind in ("", "-chat"):
    _register(f"Llama-2-7b{_kind}-hf", "meta-llama", n_layer=32, intermediate_size=11008, **_LLAMA2)
    _register(f"Llama-2-13b{_kind}-hf", "meta-llama", n_layer=40, n_head=40, n_embd=5120,
              intermediate_size=13824, **_LLAMA2)
    _register(f"Llama-2-70b{_kind}-hf", "meta-llama", n_layer=80, n_head=64, n_embd=8192, n_query_groups=8,
              intermediate_size=28672, **_LLAMA2)

for _kind in ("", "Instruct-"):
    _register(f"Mixtral-8x7B-{_kind}v0.1", "mistralai", padded_vocab_size=32000, block_size=32768, n_layer=32,
              n_query_groups=8, rotary_percentage=1.0, parallel_residual=False, bias=False,
              _norm_class="RMSNorm", norm_eps=1e-05, _mlp_class="LLaMAMoE", intermediate_size=14336,
              rope_base=1000000, n_expert=8, n_expert_per_token=2)

name_to_config: Dict[str, Dict[str, Any]] = {c["name"]: c for c in configs}
