"""Deterministic synthetic weights and prompts — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Weights follow the reference's random init (``GPT._init_weights``, /root/reference/lit_gpt/model.py:490-497:
Linear/Embedding ~ N(0, 0.02), biases 0) and norm defaults (RMSNorm weight 1, rmsnorm.py:15; LayerNorm
weight 1 / bias 0). Values come from a counter-based generator (splitmix64 of a per-tensor key + element
index, Box-Muller), so the same tensors are produced on any host without torch's RNG state.
"""

from __future__ import annotations

from typing import Dict, Iterable, Tuple

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform01(n: int, key: int, start: int = 0) -> np.ndarray:
    """n doubles in (0, 1) from counter ``start..start+n`` under ``key``."""
    idx = np.arange(start, start + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        bits = _splitmix64(idx ^ np.uint64(key) * np.uint64(0xD6E8FEB86659FD93))
    return ((bits >> np.uint64(11)).astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)


def normal(shape: Tuple[int, ...], name: str, seed: int = 1234, std: float = 0.02,
           chunk: int = 1 << 24) -> np.ndarray:
    """float32 N(0, std) tensor keyed by (seed, name)."""
    n = int(np.prod(shape)) if len(shape) else 1
    key = _fnv1a64(f"{seed}:{name}")
    out = np.empty(n, dtype=np.float32)
    half = (n + 1) // 2
    for s in range(0, half, chunk):
        m = min(chunk, half - s)
        u1 = uniform01(m, key, 2 * s)
        u2 = uniform01(m, key ^ 0x5BD1E995, 2 * s)
        r = np.sqrt(-2.0 * np.log(u1))
        z = np.empty(2 * m, dtype=np.float64)
        z[0::2] = r * np.cos(2 * np.pi * u2)
        z[1::2] = r * np.sin(2 * np.pi * u2)
        e = min(2 * (s + m), n)
        out[2 * s:e] = (z[: e - 2 * s] * std).astype(np.float32)
    return out.reshape(shape)


def token_ids(n: int, vocab_size: int, seed: int = 1234, name: str = "prompt") -> np.ndarray:
    """int32 ids uniform in [0, vocab_size) (SURVEY §8d synthetic prompt)."""
    u = uniform01(n, _fnv1a64(f"{seed}:{name}"))
    return np.minimum((u * vocab_size).astype(np.int64), vocab_size - 1).astype(np.int32)


def param_shapes(cfg) -> Iterable[Tuple[str, Tuple[int, ...], str]]:
    """(state-dict name, shape, init kind) for every parameter of the reference GPT
    (/root/reference/lit_gpt/model.py:445-460, 562-570, 596-607, 691-723)."""
    C, V = cfg.n_embd, cfg.padded_vocab_size
    qkv = (cfg.n_head + 2 * cfg.n_query_groups) * cfg.head_size
    norm_bias = cfg._norm_class == "LayerNorm"
    yield "transformer.wte.weight", (V, C), "normal"

    def norm(prefix):
        yield f"{prefix}.weight", (C,), "ones"
        if norm_bias:
            yield f"{prefix}.bias", (C,), "zeros"

    def linear(prefix, n_out, n_in, bias):
        yield f"{prefix}.weight", (n_out, n_in), "normal"
        if bias:
            yield f"{prefix}.bias", (n_out,), "zeros"

    for i in range(cfg.n_layer):
        p = f"transformer.h.{i}"
        yield from norm(f"{p}.norm_1")
        yield from linear(f"{p}.attn.attn", qkv, C, cfg.bias)
        yield from linear(f"{p}.attn.proj", C, C, cfg.bias)
        if not cfg.shared_attention_norm:
            yield from norm(f"{p}.norm_2")
        I = cfg.intermediate_size
        if cfg._mlp_class == "GptNeoxMLP":
            yield from linear(f"{p}.mlp.fc", I, C, cfg.bias)
            yield from linear(f"{p}.mlp.proj", C, I, cfg.bias)
        elif cfg._mlp_class == "LLaMAMLP":
            yield from linear(f"{p}.mlp.fc_1", I, C, cfg.bias)
            yield from linear(f"{p}.mlp.fc_2", I, C, cfg.bias)
            yield from linear(f"{p}.mlp.proj", C, I, cfg.bias)
        elif cfg._mlp_class == "LLaMAMoE":
            yield from linear(f"{p}.mlp.gate", cfg.n_expert, C, False)
            for e in range(cfg.n_expert):
                yield from linear(f"{p}.mlp.experts.{e}.fc_1", I, C, cfg.bias)
                yield from linear(f"{p}.mlp.experts.{e}.fc_2", I, C, cfg.bias)
                yield from linear(f"{p}.mlp.experts.{e}.proj", C, I, cfg.bias)
        else:
            raise NotImplementedError(cfg._mlp_class)
    yield from norm("transformer.ln_f")
    yield from linear("lm_head", V, C, cfg.lm_head_bias)


def state_dict(cfg, seed: int = 1234, std: float = 0.02) -> Dict[str, np.ndarray]:
    """Full float32 state dict with the reference's parameter names."""
    out: Dict[str, np.ndarray] = {}
    for name, shape, kind in param_shapes(cfg):
        if kind == "normal":
            out[name] = normal(shape, name, seed, std)
        elif kind == "ones":
            out[name] = np.ones(shape, dtype=np.float32)
        else:
            out[name] = np.zeros(shape, dtype=np.float32)
    return out
