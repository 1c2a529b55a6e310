"""CPU restatement of the reference GPT forward / generate — TEST INFRASTRUCTURE ONLY (oracle/__init__.py).

A functional (no nn.Module) restatement over a state dict carrying the reference's parameter names.
Every function cites the reference code it follows. ``dtype`` selects the activation/parameter dtype
the reference would run in (fp32 for the CPU config; bf16 to mirror ``--precision bf16-true``): the
op-by-op promotions (fp32 RMSNorm, fp32 RoPE products, dtype casts) are those of the reference.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F


def find_multiple(n: int, k: int) -> int:  # lit_gpt/utils.py:74-78
    assert k > 0
    return n if n % k == 0 else n + k - n % k


def build_rope_cache(seq_len: int, n_elem: int, base: int = 10000, condense_ratio: int = 1,
                     pos_dtype: torch.dtype = torch.float32):
    """lit_gpt/model.py:746-764. ``pos_dtype`` is the default dtype the reference runs
    ``torch.arange(seq_len) / condense_ratio`` in (fp32 on CPU; bf16 under ``fabric.init_tensor()``
    with bf16-true — the "bf16 RoPE position quirk" of SURVEY §7)."""
    theta = 1.0 / (base ** (torch.arange(0, n_elem, 2, dtype=torch.float32) / n_elem))
    # the reference's expression under that default dtype: an int64 range true-divided, i.e. each position rounded
    # to nearest-even in pos_dtype (torch.arange(n, dtype=torch.bfloat16) itself rounds differently above 4096)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(pos_dtype)
    try:
        seq_idx = torch.arange(seq_len) / condense_ratio
    finally:
        torch.set_default_dtype(prev)
    idx_theta = torch.outer(seq_idx, theta).repeat(1, 2)
    return torch.cos(idx_theta), torch.sin(idx_theta)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """rotate-half RoPE in promoted precision, cast back (lit_gpt/model.py:767-773)."""
    half = x.size(-1) // 2
    rotated = torch.cat((-x[..., half:], x[..., :half]), dim=-1)
    return ((x * cos) + (rotated * sin)).to(x.dtype)


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    """fp32 math, weight multiply in promoted dtype, one cast back (lit_gpt/rmsnorm.py:19-25)."""
    xf = x.float()
    normed = xf * torch.rsqrt(torch.mean(xf * xf, dim=-1, keepdim=True) + eps)
    return (w * normed).to(x.dtype)


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    """torch.nn.LayerNorm (lit_gpt/config.py:137-144 norm_class for GPT-NeoX)."""
    return F.layer_norm(x, (x.size(-1),), w, b, eps)


def topk_order(values: List[float], k: int) -> List[int]:
    """Indices of ``torch.topk(values, k)`` on the CPU (lit_gpt/model.py:737, the MoE router) including its tie
    order, restated: ATen's CPU topk (k * 64 > n) runs libstdc++ std::nth_element(begin, begin + k - 1, end)
    with the comparator "NaN first, then >" followed by std::sort(begin, begin + k - 1). nth_element is
    introselect: median-of-3 pivot moved to the front, unguarded Hoare partition while the range is longer than
    3, then insertion sort; for n <= 8 its depth limit is never reached. This is the specification of
    lga_moe_route (csrc/moe.hip); tests/test_host_logic.py checks it against torch.topk on tie-heavy inputs."""
    def gt(a, b):
        return (math.isnan(a[0]) and not math.isnan(b[0])) or (a[0] > b[0])

    def insertion(q, f, l):
        for i in range(f + 1, l):
            v = q[i]
            if gt(v, q[f]):
                q[f + 1:i + 1] = q[f:i]
                q[f] = v
            else:
                j = i
                while gt(v, q[j - 1]):
                    q[j] = q[j - 1]
                    j -= 1
                q[j] = v

    q = [(float(v), i) for i, v in enumerate(values)]
    n = len(q)
    if n > 8 or not 1 <= k <= n:
        raise ValueError("topk_order restates the n <= 8 case")
    first, last, nth = 0, n, k - 1
    while last - first > 3:
        mid = first + (last - first) // 2
        a, b, c = first + 1, mid, last - 1
        if gt(q[a], q[b]):
            s = b if gt(q[b], q[c]) else (c if gt(q[a], q[c]) else a)
        else:
            s = a if gt(q[a], q[c]) else (c if gt(q[b], q[c]) else b)
        q[first], q[s] = q[s], q[first]
        lo, hi = first + 1, last
        while True:
            while gt(q[lo], q[first]):
                lo += 1
            hi -= 1
            while gt(q[first], q[hi]):
                hi -= 1
            if not lo < hi:
                break
            q[lo], q[hi] = q[hi], q[lo]
            lo += 1
        if lo <= nth:
            first = lo
        else:
            last = lo
    insertion(q, first, last)
    insertion(q, 0, k - 1)
    return [i for _, i in q[:k]]


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    return F.linear(x, w, b)


@dataclass
class Cache:
    """Per-layer K/V for positions written so far (lit_gpt/model.py:776-799), in the activation dtype (the
    reference's cache dtype); stored un-expanded (G heads: the attention below runs SDPA with enable_gqa, the same
    math as the reference's expand-to-H-heads)."""
    k: List[torch.Tensor] = field(default_factory=list)  # (G, S, hs) per layer
    v: List[torch.Tensor] = field(default_factory=list)

    def write(self, i: int, pos, k: torch.Tensor, v: torch.Tensor) -> None:
        """KVCache.forward's index_copy_ (model.py:788-795) at positions ``pos`` of layer i; k, v (G, T, hs)."""
        self.k[i][:, pos] = k
        self.v[i][:, pos] = v


class OracleGPT:
    """Functional restatement of GPT/Block/CausalSelfAttention/MLPs (lit_gpt/model.py:445-743)."""

    def __init__(self, cfg, sd: Dict[str, np.ndarray], dtype: torch.dtype = torch.float32,
                 weight_override: Optional[Callable[[str, np.ndarray], np.ndarray]] = None,
                 rope_pos_dtype: torch.dtype = torch.float32):
        self.cfg = cfg
        self.dtype = dtype
        self.p: Dict[str, torch.Tensor] = {}
        for k, v in sd.items():
            if weight_override is not None:
                v = weight_override(k, v)
            self.p[k] = torch.from_numpy(np.ascontiguousarray(v)).to(dtype)
        self.rope_pos_dtype = rope_pos_dtype
        self.max_seq_length = cfg.block_size
        self.cache: Optional[Cache] = None
        # tests only: route_override(router_logits (T, E), topk_idx (T, k)) -> idx (T, k). Random-init routers put
        # experts within a bf16 ulp of each other; where the product broke such a near-tie the other way, a parity test
        # lets the oracle take the product's expert set (both are valid evaluations) so the later steps stay comparable
        self.route_override: Optional[Callable[[torch.Tensor, torch.Tensor], torch.Tensor]] = None

    # GPT.max_seq_length setter + rope cache (model.py:466-484, 525-532)
    def set_kv_cache(self, max_seq_length: int) -> None:
        if max_seq_length > self.cfg.block_size:
            raise ValueError(f"Cannot attend to {max_seq_length}, block size is only {self.cfg.block_size}")
        self.max_seq_length = max_seq_length
        self.cos, self.sin = build_rope_cache(max_seq_length, self.cfg.rope_n_elem, self.cfg.rope_base,
                                              self.cfg.rope_condense_ratio, self.rope_pos_dtype)
        c = self.cfg
        S = max_seq_length
        shape = (c.n_query_groups, S, c.head_size)
        self.cache = Cache(
            k=[torch.zeros(shape, dtype=self.dtype) for _ in range(c.n_layer)],
            v=[torch.zeros(shape, dtype=self.dtype) for _ in range(c.n_layer)])

    def _norm(self, prefix: str, x: torch.Tensor) -> torch.Tensor:
        c = self.cfg
        if c._norm_class == "RMSNorm":
            return rms_norm(x, self.p[f"{prefix}.weight"], c.norm_eps)
        return layer_norm(x, self.p[f"{prefix}.weight"], self.p[f"{prefix}.bias"], c.norm_eps)

    def _lin(self, prefix: str, x: torch.Tensor) -> torch.Tensor:
        return linear(x, self.p[f"{prefix}.weight"], self.p.get(f"{prefix}.bias"))

    def _attn(self, i: int, x: torch.Tensor, cos, sin, input_pos: Optional[torch.Tensor]) -> torch.Tensor:
        """CausalSelfAttention.forward (model.py:609-656) + SDPA (:658-665)."""
        c = self.cfg
        T = x.size(0)
        G, hs, H = c.n_query_groups, c.head_size, c.n_head
        qpk = H // G
        qkv = self._lin(f"transformer.h.{i}.attn.attn", x).view(T, G, qpk + 2, hs)
        q = qkv[:, :, :qpk].reshape(T, H, hs).transpose(0, 1)  # (H, T, hs)
        k = qkv[:, :, qpk].transpose(0, 1)  # (G, T, hs)
        v = qkv[:, :, qpk + 1].transpose(0, 1)
        n = c.rope_n_elem
        q = torch.cat((apply_rope(q[..., :n], cos, sin), q[..., n:]), dim=-1)
        k = torch.cat((apply_rope(k[..., :n], cos, sin), k[..., n:]), dim=-1)
        scale = 1.0 / math.sqrt(hs)
        if input_pos is not None:
            if self.cache is None:
                raise TypeError("You need to call `gpt.set_kv_cache()`")
            self.cache.write(i, input_pos, k, v)
            kk, vv = self.cache.k[i], self.cache.v[i]  # the whole cache, as KVCache.forward returns it
            # mask_cache rows input_pos (model.py:509): key j visible to query t iff j <= input_pos[t]
            mask = torch.arange(kk.size(1))[None, :] <= input_pos[:, None]
            y = F.scaled_dot_product_attention(q[None], kk[None], vv[None], attn_mask=mask[None, None], scale=scale,
                                               enable_gqa=G != H)
        else:
            y = F.scaled_dot_product_attention(q[None], k[None], v[None], is_causal=True, scale=scale,
                                               enable_gqa=G != H)
        # SDPA in the activation dtype, exactly the reference's call (model.py:658-665)
        y = y[0].transpose(0, 1).reshape(T, H * hs)
        return self._lin(f"transformer.h.{i}.attn.proj", y)

    def _mlp(self, i: int, x: torch.Tensor) -> torch.Tensor:
        c = self.cfg
        p = f"transformer.h.{i}.mlp"
        if c._mlp_class == "LLaMAMLP":  # model.py:712-716
            return self._lin(f"{p}.proj", F.silu(self._lin(f"{p}.fc_1", x)) * self._lin(f"{p}.fc_2", x))
        if c._mlp_class == "GptNeoxMLP":  # model.py:699-702
            return self._lin(f"{p}.proj", F.gelu(self._lin(f"{p}.fc", x), approximate=c.gelu_approximate))
        if c._mlp_class == "LLaMAMoE":  # model.py:727-743
            router = self._lin(f"{p}.gate", x)
            probs, idx = torch.topk(router, c.n_expert_per_token)
            if self.route_override is not None:  # test hook: adopt another implementation's tie-break (see below)
                idx = self.route_override(router, idx)
                probs = torch.gather(router, 1, idx)
            probs = probs.softmax(dim=1, dtype=torch.float).to(x.dtype)
            y = torch.zeros_like(x)
            for e in range(c.n_expert):
                tok, slot = torch.where(idx == e)
                if tok.numel() == 0:
                    continue
                xe = x[tok]
                ye = self._lin(f"{p}.experts.{e}.proj",
                               F.silu(self._lin(f"{p}.experts.{e}.fc_1", xe)) * self._lin(f"{p}.experts.{e}.fc_2", xe))
                y[tok] += probs[tok, slot, None] * ye
            return y
        raise NotImplementedError(c._mlp_class)

    def forward(self, idx: torch.Tensor, input_pos: Optional[torch.Tensor] = None,
                last_only: bool = False) -> torch.Tensor:
        """GPT.forward (model.py:499-519) for B=1: idx (T,) int -> logits (T, V) in ``dtype`` (``last_only``: the
        last row only, (1, V) — all that generate samples from, generate/base.py:31)."""
        c = self.cfg
        T = idx.numel()
        if self.max_seq_length < T:
            raise ValueError(f"Cannot forward sequence of length {T}, max seq length is only {self.max_seq_length}.")
        if input_pos is not None:
            if self.cache is None:
                raise TypeError("You need to call `gpt.set_kv_cache()`")
            cos, sin = self.cos[input_pos], self.sin[input_pos]
        else:
            cos, sin = build_rope_cache(T, c.rope_n_elem, c.rope_base, c.rope_condense_ratio, self.rope_pos_dtype)
        x = self.p["transformer.wte.weight"][idx.long()]
        for i in range(c.n_layer):
            pre = f"transformer.h.{i}"
            n1 = self._norm(f"{pre}.norm_1", x)
            h = self._attn(i, n1, cos, sin, input_pos)
            if c.parallel_residual:  # Block.forward model.py:580-593
                n2 = n1 if c.shared_attention_norm else self._norm(f"{pre}.norm_2", x)
                x = self._mlp(i, n2) + h + x
            else:
                if c.shared_attention_norm:
                    raise NotImplementedError("non-parallel residual and shared attention norm")
                x = h + x
                x = self._mlp(i, self._norm(f"{pre}.norm_2", x)) + x
        if last_only:
            x = x[-1:]
        x = self._norm("transformer.ln_f", x)
        return self._lin("lm_head", x)


def one_block_rows(og: OracleGPT, idx: torch.Tensor, rows: List[int],
                   router_gaps: Optional[List[float]] = None) -> torch.Tensor:
    """Rows ``rows`` of GPT.forward's logits (model.py:499-519, no cache) for a ONE-block model over idx (T,),
    without the T x T work of a full forward: the qkv Linear and RoPE run over every position (the keys and values
    every query sees), the query, attention, projection, MLP and head only for the requested rows. Row t of the
    causal forward attends keys 0..t (SDPA is_causal, model.py:658-665) — exactly one query row over the prefix —
    and is also what a decode step at input_pos t computes from a cache filled by the prefix (model.py:509, 788-795).
    Long-prompt prefill parity (32k tokens) at a cost linear in T. ``router_gaps`` (a list, sparse-MoE configs):
    receives per row the gap between the k-th and (k+1)-th router logit over max |router| — a row whose gap is at
    the rounding noise can route to another expert in any other evaluation order (a parity test skips it)."""
    c = og.cfg
    if c.n_layer != 1 or c.parallel_residual:
        raise NotImplementedError("one_block_rows: one sequential-residual block")
    T = idx.numel()
    G, hs, H = c.n_query_groups, c.head_size, c.n_head
    qpk, n = H // G, c.rope_n_elem
    cos, sin = build_rope_cache(T, n, c.rope_base, c.rope_condense_ratio, og.rope_pos_dtype)
    x = og.p["transformer.wte.weight"][idx.long()]
    qkv = og._lin("transformer.h.0.attn.attn", og._norm("transformer.h.0.norm_1", x)).view(T, G, qpk + 2, hs)
    k = qkv[:, :, qpk].transpose(0, 1)  # (G, T, hs)
    v = qkv[:, :, qpk + 1].transpose(0, 1)
    k = torch.cat((apply_rope(k[..., :n], cos, sin), k[..., n:]), dim=-1)
    out = []
    for t in rows:
        q = qkv[t, :, :qpk].reshape(H, 1, hs)
        q = torch.cat((apply_rope(q[..., :n], cos[t:t + 1], sin[t:t + 1]), q[..., n:]), dim=-1)
        y = F.scaled_dot_product_attention(q[None], k[None, :, : t + 1], v[None, :, : t + 1],
                                           scale=1.0 / math.sqrt(hs), enable_gqa=G != H)
        h = og._lin("transformer.h.0.attn.proj", y[0].transpose(0, 1).reshape(1, H * hs))
        xr = h + x[t:t + 1]
        n2 = og._norm("transformer.h.0.norm_2", xr)
        if router_gaps is not None and c._mlp_class == "LLaMAMoE":
            r = torch.sort(og._lin("transformer.h.0.mlp.gate", n2)[0].double(), descending=True)[0]
            ne = c.n_expert_per_token
            router_gaps.append(float((r[ne - 1] - r[ne]) / r.abs().max()))
        xr = og._mlp(0, n2) + xr
        out.append(og._lin("lm_head", og._norm("transformer.ln_f", xr)))
    return torch.cat(out)


def sample(logits: torch.Tensor, temperature: float = 1.0, top_k: Optional[int] = None,
           multinomial: Optional[Callable[[torch.Tensor], torch.Tensor]] = None) -> torch.Tensor:
    """generate/base.py:30-41 on the last row of (T, V) logits; returns (1,) int64."""
    logits = logits[-1]
    if top_k is not None:
        v, i = torch.topk(logits, min(top_k, logits.size(-1)))
        logits = torch.full_like(logits, float("-inf")).scatter_(-1, i, v)
    if temperature > 0.0:
        probs = torch.softmax(logits / temperature, dim=-1)
        return (multinomial or (lambda p: torch.multinomial(p, num_samples=1)))(probs)
    return torch.argmax(logits, dim=-1, keepdim=True)


def inverse_cdf(probs: np.ndarray, u: float) -> int:
    """torch.multinomial(probs, 1) on the CPU given its uniform draw u (generate/base.py:27, 40): the fp32 running sum
    in index order, divided by its total, and the first index whose value reaches u (ATen's CPU multinomial
    cumulative distribution + binary search). The specification of lga_sample_topk's draw."""
    cum = np.cumsum(np.asarray(probs, dtype=np.float32), dtype=np.float32)
    cdf = (cum / cum[-1]).astype(np.float32)
    return int(np.searchsorted(cdf, np.float32(u), side="left"))


def sample_topk_spec(logits_bf16: torch.Tensor, top_k: int, temperature: float, u: float):
    """generate/base.py:30-41 (top_k, temperature > 0) on 1-D bf16 logits, stated as lga_sample_topk computes it:
    the kept set is torch.topk's (ties at the k-th value kept lowest index first), probabilities are the bf16
    softmax of bf16(v / temperature) over the kept set, the token is inverse_cdf of those probabilities.
    Returns (kept indices in index order, their probabilities (fp32 holding bf16 values), token)."""
    x = logits_bf16.float()
    n = x.numel()
    k = min(top_k, n)
    xs = x.tolist()
    # NaN above everything, then value descending (-0 == +0), then index ascending
    order = sorted(range(n), key=lambda i: (not math.isnan(xs[i]), -xs[i] if not math.isnan(xs[i]) else 0.0, i))
    kept = sorted(order[:k])
    v = (x[kept] / temperature).to(torch.bfloat16).float()
    e = torch.exp(v - v.max())
    p = (e / e.sum()).to(torch.bfloat16).float()
    j = inverse_cdf(p.numpy(), u)
    return kept, p, kept[j]


def generate(model: OracleGPT, prompt: torch.Tensor, max_returned_tokens: int, *, temperature: float = 1.0,
             top_k: Optional[int] = None, eos_id: Optional[int] = None,
             multinomial=None, record_logits: Optional[list] = None) -> torch.Tensor:
    """generate/base.py:50-93: prefill at arange(T), then single-token steps at input_pos = T, T+1, ..."""
    T = prompt.numel()
    assert max_returned_tokens > T
    if model.max_seq_length < max_returned_tokens - 1:
        raise NotImplementedError(f"max_seq_length {model.max_seq_length} needs to be >= {max_returned_tokens - 1}")
    tokens = [prompt]
    logits = model.forward(prompt, torch.arange(T))
    if record_logits is not None:
        record_logits.append(logits[-1].float().clone())
    token = sample(logits, temperature, top_k, multinomial).to(prompt.dtype)
    tokens.append(token)
    pos = T
    for _ in range(2, max_returned_tokens - T + 1):
        logits = model.forward(token.view(-1), torch.tensor([pos]))
        if record_logits is not None:
            record_logits.append(logits[-1].float().clone())
        token = sample(logits, temperature, top_k, multinomial).to(prompt.dtype)
        tokens.append(token)
        if eos_id is not None and int(token) == eos_id:
            break
        pos += 1
    return torch.cat(tokens)
