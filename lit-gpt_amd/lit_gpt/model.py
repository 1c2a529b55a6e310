"""GPT / Block / CausalSelfAttention / KVCache with the reference's module API and an MI355X HIP hot path.

Public surface kept from /root/reference/lit_gpt/model.py: ``GPT(config)``; ``GPT.forward(idx,
input_pos=None)`` (:499-519); ``max_seq_length`` property/setter (:462-484); ``rope_cache`` (:525-532);
``set_kv_cache`` / ``clear_kv_cache`` (:534-559); ``from_name`` (:521-523); ``_init_weights`` (:490-497);
attributes ``config, lm_head, transformer.{wte,h,ln_f}, cos, sin, mask_cache``. ``Block.forward(x, cos, sin,
mask=None, input_pos=None)`` (:572-593) with ``norm_1, attn, norm_2, mlp``; ``CausalSelfAttention.forward``
(:609-656) with ``attn`` (fused qkv Linear), ``proj``, ``kv_cache``, ``build_kv_cache``,
``scaled_dot_product_attention``; ``KVCache`` (:776-799); ``LLaMAMLP`` / ``LLaMAMoE`` / ``GptNeoxMLP`` classes
(``generate/tp.py`` isinstance-checks them); ``build_rope_cache`` / ``apply_rope`` / ``build_mask_cache``.

What runs underneath (GPU, bf16 activations, Linears converted by ``QuantizedPrecision``): every op is a HIP
kernel from ``liblitgpt_amd.so`` — embedding gather, RMSNorm fused into the qkv / fc GEMV prologue, RoPE fused
with the KV-cache append, split-sequence decode attention, the out-projections with the residual add in their
epilogue, SwiGLU fused into the dual fc_1/fc_2 GEMV, and greedy argmax. Differences from the reference that do
not change results: the KV cache holds ``n_query_groups`` heads (un-expanded GQA) and the bool mask is never
materialised on the hot path (the kernels read keys ``<= input_pos``). RoPE positions follow the reference's
default-dtype semantics (``build_rope_cache``), so ``generate.base.build_model`` reproduces the bf16 rounding of
positions > 256 that the reference's bf16 ``init_tensor`` context produces.
"""

from __future__ import annotations

import math
import os
from typing import Any, Optional, Tuple

import torch
import torch.nn as nn

from lit_gpt import ops
from lit_gpt.config import Config
from lit_gpt.rmsnorm import RMSNorm



def _gpu_only(what: str) -> None:
    raise RuntimeError(f"{what}: this build computes on the MI355X only (no CPU path); move the model to 'cuda'")


def _dense_weight(linear: nn.Linear) -> torch.Tensor:
    """The bf16 weight of an unquantized Linear, made contiguous once in place (a TP row shard from
    ``generate/tp.py``'s ``tensor_split(dim=1)`` is a strided view)."""
    w = linear.weight
    if w.dtype != torch.bfloat16:
        raise TypeError(f"unquantized Linear on the MI355X path expects bf16 weights (bf16-true), got {w.dtype}")
    if not w.is_contiguous():
        linear.weight.data = w.data.contiguous()
        w = linear.weight
    return w


def _dense(linear: nn.Linear, x: torch.Tensor, *, residual: Optional[torch.Tensor] = None,
           norm_weight: Optional[torch.Tensor] = None, norm_eps: float = 1e-5) -> torch.Tensor:
    """F.linear with bf16 weights (BASELINE config 2): one token -> lga_bf16_gemv (RMSNorm / residual fused),
    several -> lga_bf16_gemm (MFMA)."""
    w = _dense_weight(linear)
    N, K = w.shape
    lead = x.shape[:-1]
    x2 = x.reshape(-1, K)
    if x2.dtype != torch.bfloat16:
        raise TypeError(f"Linear expects bf16 activations (bf16-true), got {x2.dtype}")
    x2 = x2.contiguous()
    M = x2.shape[0]
    b = None if linear.bias is None else linear.bias.to(torch.bfloat16)
    res = None if residual is None else residual.reshape(M, N).contiguous()
    if M == 1:
        y = ops.bf16_gemv(x2.view(-1), w, bias=b, residual=None if res is None else res.view(-1),
                          norm_weight=norm_weight, eps=norm_eps)
    else:
        if norm_weight is not None:
            x2 = ops.rmsnorm(x2, norm_weight, norm_eps)
        if _fused_prefill(M, N, K, 64, 2):  # MFMA tiles with the weight DMA'd as stored (csrc/gemm_q4f.hip)
            y = ops.q4_gemm_fused(x2, w, None, N, K, 64, 2, bias=b, residual=res)
        else:
            y = ops.bf16_gemm(x2, w, bias=b, residual=res)
    return y.view(*lead, N)


def _dense_f32(linear: nn.Linear, x: torch.Tensor, *, residual: Optional[torch.Tensor] = None,
               norm_weight: Optional[torch.Tensor] = None, norm_eps: float = 1e-5) -> torch.Tensor:
    """F.linear in float32 (the reference's --precision 32-true, BASELINE config 1): lga_f32_linear."""
    if norm_weight is not None:
        raise NotImplementedError("fp32 path: RMSNorm-family blocks are not built in fp32 (GPT-NeoX LayerNorm is)")
    w = linear.weight
    if not w.is_contiguous():
        linear.weight.data = w.data.contiguous()
        w = linear.weight
    N, K = w.shape
    if x.dtype != torch.float32:
        raise TypeError(f"fp32 Linear expects fp32 activations (32-true), got {x.dtype}")
    lead = x.shape[:-1]
    x2 = x.reshape(-1, K).contiguous()
    res = None if residual is None else residual.reshape(x2.shape[0], N).contiguous()
    return ops.f32_linear(x2, w, bias=linear.bias, residual=res).view(*lead, N)


def _fused_prefill(M: int, N: int, K: int, group: int, fmt: int) -> bool:
    return M > 1 and ops.q4f_fits(M, N, K, group, fmt)


def _lin(linear: nn.Module, x: torch.Tensor, *, reduce=None, **kw) -> torch.Tensor:
    """Run a Linear on the MI355X kernels. ``reduce``: the TP all-reduce hook of a row-parallel projection
    (generate/tp.py) — the partial output is summed over the ranks (+ ``residual``), fused into the GEMV launch for
    one-token inputs (lit_gpt/comm.py linear_reduce)."""
    from lit_gpt.quantize import QuantLinear

    if reduce is not None:
        from lit_gpt import comm

        res = kw.pop("residual", None)
        return comm.linear_reduce(reduce, linear, x, res, lambda: _lin(linear, x, **kw))

    if isinstance(linear, QuantLinear):
        return linear(x, **kw)
    if isinstance(linear, nn.Linear) and linear.weight.is_cuda and linear.weight.dtype == torch.float32:
        return _dense_f32(linear, x, **kw)
    if isinstance(linear, nn.Linear) and linear.weight.is_cuda:
        return _dense(linear, x, **kw)
    raise NotImplementedError(
        "Linear without MI355X weights: move the model to the GPU in bf16, or convert it with "
        "lit_gpt.quantize.QuantizedPrecision('int4-g128' | 'nf4').convert_module(model) (the --quantize flag)")


class GPT(nn.Module):
    def __init__(self, config: Config) -> None:
        super().__init__()
        assert config.padded_vocab_size is not None
        self.config = config
        self.lm_head = nn.Linear(config.n_embd, config.padded_vocab_size, bias=config.lm_head_bias)
        self.transformer = nn.ModuleDict(dict(
            wte=nn.Embedding(config.padded_vocab_size, config.n_embd),
            h=nn.ModuleList(Block(config) for _ in range(config.n_layer)),
            ln_f=config.norm_class(config.n_embd, eps=config.norm_eps),
        ))
        self.max_seq_length = self.config.block_size
        self.mask_cache: Optional[torch.Tensor] = None

    @property
    def max_seq_length(self) -> int:
        return self._max_seq_length

    @max_seq_length.setter
    def max_seq_length(self, value: int) -> None:
        if value > self.config.block_size:
            raise ValueError(f"Cannot attend to {value}, block size is only {self.config.block_size}")
        self._max_seq_length = value
        if not hasattr(self, "cos"):
            cos, sin = self.rope_cache()
            self.register_buffer("cos", cos, persistent=False)
            self.register_buffer("sin", sin, persistent=False)
        elif value != self.cos.size(0):
            self.cos, self.sin = self.rope_cache(device=self.cos.device)

    def reset_parameters(self) -> None:
        self.cos, self.sin = self.rope_cache()

    def _init_weights(self, module: nn.Module) -> None:
        if isinstance(module, nn.Linear):
            torch.nn.init.normal_(module.weight, mean=0.0, std=0.02)
            if module.bias is not None:
                torch.nn.init.zeros_(module.bias)
        elif isinstance(module, nn.Embedding):
            torch.nn.init.normal_(module.weight, mean=0.0, std=0.02)

    def _rope_tables(self) -> Tuple[torch.Tensor, torch.Tensor]:
        # model.to(bf16) would also cast the rope buffers; the kernels need the exact fp32 tables
        if self.cos.dtype != torch.float32 or self.cos.size(0) != self.max_seq_length:
            self.cos, self.sin = self.rope_cache(device=self.cos.device)
        return self.cos, self.sin

    def forward(self, idx: torch.Tensor, input_pos: Optional[torch.Tensor] = None, *,
                last_token_only: bool = False, embedded: Optional[torch.Tensor] = None,
                hidden_only: bool = False) -> torch.Tensor:
        """(B=1, T) ids -> (1, T, padded_vocab) logits; ``last_token_only`` computes only the last row (1, 1, V)
        — all that ``generate`` samples from (generate/base.py:31). ``embedded`` (T * n_embd bf16) is
        ``transformer.wte(idx)`` already gathered — by the previous decode step's ``ops.argmax_embed`` in
        ``DecodeGraph`` — and replaces the embedding launch. ``hidden_only`` stops before ln_f / lm_head and returns
        the last block's output (DecodeGraph runs the head fused with the greedy argmax)."""
        B, T = idx.shape
        if self.max_seq_length < T:
            raise ValueError(f"Cannot forward sequence of length {T}, max seq length is only {self.max_seq_length}.")
        if input_pos is not None and self.mask_cache is None:
            raise TypeError("You need to call `gpt.set_kv_cache()`")
        if not idx.is_cuda:
            _gpu_only("GPT.forward")
        if B != 1:
            raise NotImplementedError("the MI355X decode path runs batch size 1 (as generate/base.py does)")
        cos, sin = self._rope_tables()
        if input_pos is not None:
            input_pos = input_pos.to(device=idx.device, dtype=torch.int64).contiguous()
        if embedded is not None:
            if embedded.numel() != T * self.transformer.wte.weight.shape[1] or embedded.dtype != torch.bfloat16:
                raise ValueError("embedded must hold T * n_embd bf16 values (the gathered wte rows of idx)")
            x = embedded.view(1, T, -1)
        else:
            x = ops.embedding(idx.reshape(-1).contiguous(), self.transformer.wte.weight).view(1, T, -1)
        for block in self.transformer.h:
            x = block(x, cos, sin, None, input_pos)
        if last_token_only:
            x = x[:, -1:].contiguous()
        if hidden_only:
            return x
        ln = self.transformer.ln_f
        if isinstance(ln, RMSNorm):
            return _lin(self.lm_head, x, norm_weight=ln.weight, norm_eps=ln.eps)
        return _lin(self.lm_head, ln(x))

    @classmethod
    def from_name(cls, name: str, **kwargs: Any) -> "GPT":
        return cls(Config.from_name(name, **kwargs))

    def rope_cache(self, device: Optional[torch.device] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        return build_rope_cache(seq_len=self.max_seq_length, n_elem=self.config.rope_n_elem, device=device,
                                condense_ratio=self.config.rope_condense_ratio, base=self.config.rope_base)

    def set_kv_cache(self, batch_size: int, rope_cache_length: Optional[int] = None,
                     device: Optional[torch.device] = None, dtype: Optional[torch.dtype] = None) -> None:
        if rope_cache_length is None:
            rope_cache_length = self.cos.size(-1)
        for block in self.transformer.h:
            block.attn.kv_cache = block.attn.build_kv_cache(batch_size, self.max_seq_length, rope_cache_length,
                                                            device, dtype)
        if self.mask_cache is None or self.mask_cache.size(3) != self.max_seq_length:
            self.mask_cache = CausalMask(self.max_seq_length, device or self.transformer.wte.weight.device)

    def clear_kv_cache(self) -> None:
        self.mask_cache = None
        for block in self.transformer.h:
            block.attn.kv_cache = None


class Block(nn.Module):
    def __init__(self, config: Config) -> None:
        super().__init__()
        self.norm_1 = config.norm_class(config.n_embd, eps=config.norm_eps)
        self.attn = CausalSelfAttention(config)
        self.norm_2 = None if config.shared_attention_norm else config.norm_class(config.n_embd, eps=config.norm_eps)
        self.mlp = config.mlp_class(config)
        self.config = config

    def forward(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, mask: Optional[torch.Tensor] = None,
                input_pos: Optional[torch.Tensor] = None) -> torch.Tensor:
        c = self.config
        if c.shared_attention_norm and not c.parallel_residual:
            raise NotImplementedError("No checkpoint amongst the ones we support uses this configuration"
                                      " (non-parallel residual and shared attention norm).")
        if c.parallel_residual:
            return self._parallel_forward(x, cos, sin, mask, input_pos)
        if not isinstance(self.norm_1, RMSNorm) or not isinstance(self.mlp, (LLaMAMLP, LLaMAMoE)):
            raise NotImplementedError(f"{type(self.mlp).__name__} / {type(self.norm_1).__name__} blocks have no "
                                      "MI355X kernels in this build")
        # The norms ride the qkv / fc GEMV prologues and the residual adds the out-projection epilogues. Under
        # tensor parallelism (generate/tp.py's all_reduce_output hook on attn / mlp) the projections yield partial
        # sums: the module then runs without its hook and the reduction + residual add is one fused kernel
        # (lit_gpt/comm.py); any other forward hook keeps the reference's call-the-module semantics.
        from lit_gpt import comm

        ha = comm.tp_hook(self.attn)
        hm = comm.tp_hook(self.mlp)
        if ha is not None:
            x = self.attn.forward(x, cos, sin, mask, input_pos, norm=self.norm_1, residual=x, reduce=ha)
        elif not self.attn._forward_hooks:
            x = self.attn(x, cos, sin, mask, input_pos, norm=self.norm_1, residual=x)
        else:
            x = ops.add(self.attn(self.norm_1(x), cos, sin, mask, input_pos).contiguous(), x.contiguous())
        if hm is not None and isinstance(self.mlp, LLaMAMLP):
            return self.mlp.forward(x, norm=self.norm_2, residual=x, reduce=hm)
        if hm is not None:
            return comm.reduce_add(hm, self.mlp, self.mlp.forward(x, norm=self.norm_2), x)
        if not self.mlp._forward_hooks:  # (a sparse-MoE block applies its experts' TP hooks itself)
            return self.mlp(x, norm=self.norm_2, residual=x)
        return ops.add(self.mlp(self.norm_2(x)).contiguous(), x)


    def _parallel_forward(self, x, cos, sin, mask, input_pos) -> torch.Tensor:
        """GPT-NeoX block (reference model.py:572-593, parallel_residual): n_1 = norm_1(x), h = attn(n_1),
        n_2 = n_1 if shared_attention_norm else norm_2(x), x = mlp(n_2) + h + x — the reference's association:
        bf16(mlp + h) (fused into the mlp.proj epilogue) then + x. Under tensor parallelism the attn / mlp outputs
        go through their all-reduce hooks first (generate/tp.py), as in the reference."""
        n_1 = self.norm_1(x)
        h = self.attn(n_1, cos, sin, mask, input_pos).contiguous()
        n_2 = n_1 if self.config.shared_attention_norm else self.norm_2(x)
        if self.mlp._forward_hooks:  # TP: the hook must see the mlp output alone
            m = ops.add(self.mlp(n_2).contiguous(), h)
        else:
            m = self.mlp(n_2, residual=h)
        return ops.add(m.contiguous(), x.contiguous()).view_as(x)


class CausalSelfAttention(nn.Module):
    def __init__(self, config: Config) -> None:
        super().__init__()
        shape = (config.n_head + 2 * config.n_query_groups) * config.head_size
        self.attn = nn.Linear(config.n_embd, shape, bias=config.bias)
        self.proj = nn.Linear(config.n_embd, config.n_embd, bias=config.bias)
        self.kv_cache: Optional[KVCache] = None
        self.config = config

    # decode tokens (T = 1) with full 128-dim rotary use lga_attention_decode_fused; False keeps the two-launch
    # rope_kv_append + attention path (bit-identical; tests compare the two)
    fuse_decode = True

    def forward(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, mask: Optional[torch.Tensor] = None,
                input_pos: Optional[torch.Tensor] = None, *, norm: Optional["RMSNorm"] = None,
                residual: Optional[torch.Tensor] = None, reduce=None) -> torch.Tensor:
        """``norm`` / ``residual`` / ``reduce`` are fusion hooks used by Block.forward: the RMSNorm runs in the qkv
        GEMV prologue, the residual add (and under TP the all-reduce hook ``reduce``) in the proj epilogue. Without
        them this is the reference forward."""
        B, T, C = x.size()
        c = self.config
        H, G, hs = c.n_head, c.n_query_groups, c.head_size
        qkv = _lin(self.attn, x, norm_weight=None if norm is None else norm.weight,
                   norm_eps=c.norm_eps if norm is None else norm.eps).view(T, -1)
        dev = x.device
        if input_pos is None:
            # no cache (training-style causal forward, model.py:510-513): a private cache of T rows
            pos = torch.arange(T, device=dev, dtype=torch.int64)
            kc = torch.empty(G, T, hs, dtype=torch.bfloat16, device=dev)
            vc = torch.empty_like(kc)
            rope_pos = pos
        else:
            if not isinstance(self.kv_cache, KVCache):
                raise TypeError("You need to call `gpt.set_kv_cache()`")
            kv = self.kv_cache
            if kv.k.dtype != qkv.dtype:  # reference KVCache.forward casts to the activation dtype (:790-791)
                kv.k, kv.v = kv.k.to(qkv.dtype), kv.v.to(qkv.dtype)
            kc, vc = kv.k, kv.v
            pos = input_pos
            # callers may pass the full cos/sin tables (our GPT.forward) or rows pre-selected by input_pos (the
            # reference's GPT.forward, model.py:505-506)
            rope_pos = pos if (cos.size(0) != T or T == kc.size(-2)) else torch.arange(T, device=dev)
        cos = cos.to(device=dev, dtype=torch.float32).contiguous()
        sin = sin.to(device=dev, dtype=torch.float32).contiguous()
        S = kc.size(-2)
        ws = None
        n_splits = 1
        if T == 1 and qkv.dtype == torch.bfloat16:
            n_splits = ops.decode_splits(G, H // G, hs, S)
            ws = getattr(self, "_attn_ws", None)
            if ws is None or ws.key != (1, H, G, hs, n_splits) or ws.counters.device != dev:
                ws = self._attn_ws = ops.AttentionWorkspace(1, H, G, hs, n_splits, dev)
        if T == 1 and self.fuse_decode and ops.decode_fusable(hs, c.rope_n_elem) and qkv.dtype == torch.bfloat16:
            # decode token: RoPE + KV-append + attention in a single launch
            y = ops.attention_decode_fused(qkv, kc, vc, pos, rope_pos, cos, sin, H, G, hs, c.rope_n_elem,
                                           1.0 / math.sqrt(hs), n_splits, workspace=ws)
        else:
            q = ops.rope_kv_append(qkv, kc, vc, pos, rope_pos, cos, sin, H, G, hs, c.rope_n_elem)
            y = ops.attention(q, kc, vc, pos, H, G, hs, 1.0 / math.sqrt(hs), n_splits, workspace=ws)
        out = _lin(self.proj, y.view(1, T, H * hs), residual=residual, reduce=reduce)
        return out.view(B, T, -1)

    def scaled_dot_product_attention(self, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor,
                                     mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Reference-compatible helper (model.py:658-665); the fused path uses ``ops.attention`` instead."""
        scale = 1.0 / math.sqrt(self.config.head_size)
        y = torch.nn.functional.scaled_dot_product_attention(q, k, v, attn_mask=mask, dropout_p=0.0, scale=scale,
                                                             is_causal=mask is None)
        return y.transpose(1, 2)

    def build_kv_cache(self, batch_size: int, max_seq_length: int, rope_cache_length: Optional[int] = None,
                       device: Optional[torch.device] = None, dtype: Optional[torch.dtype] = None) -> "KVCache":
        heads = self.config.n_query_groups  # un-expanded groups (the reference stores n_head, model.py:675)
        v_shape = (batch_size, heads, max_seq_length, self.config.head_size)
        if rope_cache_length is None:
            if self.config.rotary_percentage != 1.0:
                raise TypeError("Please pass the `rope_cache_length=gpt.cos.size(-1)` value")
            k_shape = v_shape
        else:
            k_shape = (batch_size, heads, max_seq_length,
                       rope_cache_length + self.config.head_size - self.config.rope_n_elem)
        if device is None:
            device = self.attn.weight.device
        return KVCache(k_shape, v_shape, device=device, dtype=dtype or torch.bfloat16)


class GptNeoxMLP(nn.Module):
    """GPT-NeoX / pythia MLP (reference model.py:691-702): fc (+bias) -> GELU -> proj (+bias). The Linears run the
    GEMV / GEMM kernels (4-bit or bf16), the activation ``lga_gelu`` (exact erf, or tanh per
    ``config.gelu_approximate``) with the reference's bf16 rounding points."""

    def __init__(self, config: Config) -> None:
        super().__init__()
        self.fc = nn.Linear(config.n_embd, config.intermediate_size, bias=config.bias)
        self.proj = nn.Linear(config.intermediate_size, config.n_embd, bias=config.bias)
        self.config = config

    def forward(self, x: torch.Tensor, *, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``residual`` fuses an add into the proj epilogue (bf16(bf16(proj(x)) + residual)); Block uses it for the
        parallel residual's ``mlp(n_2) + h``."""
        if not x.is_cuda:
            _gpu_only("GptNeoxMLP")
        h = _lin(self.fc, x)
        h = ops.gelu(h.contiguous(), self.config.gelu_approximate)
        return _lin(self.proj, h, residual=residual)


class LLaMAMLP(nn.Module):
    def __init__(self, config: Config) -> None:
        super().__init__()
        self.fc_1 = nn.Linear(config.n_embd, config.intermediate_size, bias=config.bias)
        self.fc_2 = nn.Linear(config.n_embd, config.intermediate_size, bias=config.bias)
        self.proj = nn.Linear(config.intermediate_size, config.n_embd, bias=config.bias)

    def forward(self, x: torch.Tensor, *, norm: Optional["RMSNorm"] = None,
                residual: Optional[torch.Tensor] = None, reduce=None) -> torch.Tensor:
        """proj(silu(fc_1 x) * fc_2 x) (model.py:712-716); ``norm``/``residual``/``reduce`` are Block fusion hooks
        (``reduce``: the TP all-reduce of the row-parallel proj, see CausalSelfAttention.forward)."""
        from lit_gpt.quantize import QuantLinear

        lead, C = x.shape[:-1], x.shape[-1]
        x2 = x.reshape(-1, C).contiguous()
        M = x2.shape[0]
        f1, f2 = self.fc_1, self.fc_2
        fusable = (M == 1 and isinstance(f1, QuantLinear) and isinstance(f2, QuantLinear) and f1.bias is None
                   and f2.bias is None and (f1.fmt, f1.group) == (f2.fmt, f2.group))
        dense = (M == 1 and type(f1) is nn.Linear and type(f2) is nn.Linear and f1.bias is None and f2.bias is None
                 and f1.weight.is_cuda and f1.weight.shape == f2.weight.shape)
        if dense:  # bf16 weights: fc_1 || fc_2 + SwiGLU in one GEMV launch, norm_2 fused
            g = ops.bf16_gemv_swiglu(x2.view(-1), _dense_weight(f1), _dense_weight(f2),
                                     norm_weight=None if norm is None else norm.weight,
                                     eps=1e-5 if norm is None else norm.eps).view(1, -1)
        elif fusable:
            if norm is not None and not ops.gemv_fuses_norm(C, dual=True):
                x2, norm = norm(x2), None
            g = ops.q4_gemv_swiglu(x2.view(-1), f1.qweight, f1.scales, f2.qweight, f2.scales, f1.out_features, C,
                                   f1.group, f1.fmt, norm_weight=None if norm is None else norm.weight,
                                   eps=1e-5 if norm is None else norm.eps).view(1, -1)
        else:
            n = x2 if norm is None else norm(x2)
            g = None
            if f1.bias is None and f2.bias is None:  # fc_1 || fc_2 + SwiGLU in one fused GEMM launch
                I = f1.out_features
                if (isinstance(f1, QuantLinear) and isinstance(f2, QuantLinear)
                        and (f1.fmt, f1.group) == (f2.fmt, f2.group) and _fused_prefill(M, I, C, f1.group, f1.fmt)):
                    g = ops.q4_gemm_swiglu(n, f1.qweight, f1.scales, f2.qweight, f2.scales, I, C, f1.group, f1.fmt)
                elif (type(f1) is nn.Linear and type(f2) is nn.Linear and f1.weight.is_cuda
                      and f1.weight.shape == f2.weight.shape and _fused_prefill(M, I, C, 64, 2)):
                    g = ops.q4_gemm_swiglu(n, _dense_weight(f1), None, _dense_weight(f2), None, I, C, 64, 2)
            if g is None:
                g = ops.swiglu(_lin(f1, n).contiguous(), _lin(f2, n).contiguous())
        out = _lin(self.proj, g, residual=residual, reduce=reduce)
        return out.view(*lead, -1)


# decode routing through the fused gate + route launch (lga_moe_gate_route); False keeps lga_q4_gemv + lga_moe_route
# (tests A/B the two)
moe_gate_route = True
# one-token sparse-MoE: the routed proj GEMVs of both slots + the combine + residual in one launch whose second-arriving
# workgroup per row block combines (lga_q4_gemv_experts_pair_combine, bit-identical to the two launches); False keeps
# lga_q4_gemv_experts + lga_moe_combine
moe_pair_combine = os.environ.get("LGA_MOE_PAIR_COMBINE", "1") != "0"


class LLaMAMoE(nn.Module):
    """Sparse MoE (lit_gpt/model.py:719-743): router gate, top-k experts per token, prob-weighted bf16 sum.

    Decode (one token) never leaves the device: ``lga_moe_route`` picks the experts, the routed GEMVs stream
    only the k selected experts' weights (``lga_q4_gemv_swiglu_experts`` with the fused norm_2, then
    ``lga_q4_gemv_experts``), ``lga_moe_combine`` adds them in ascending expert order plus the Block residual.
    Prefill (T > 1) groups the (token, slot) pairs per expert on the device (``lga_moe_group``: the reference's
    ``torch.where`` loop as a stable counting sort and a tile table) and runs all experts in two grouped MFMA GEMM
    launches (fc_1||fc_2 + SwiGLU, proj); shapes the grouped kernel does not take fall back to the per-expert loop. Forward hooks registered on the experts (``generate/tp.py`` registers the TP
    all-reduce on each expert, tp.py:58-62) are applied to the stacked (T, k, C) expert outputs: a per-element
    sum over ranks, identical to reducing every expert call separately.
    """

    def __init__(self, config: Config) -> None:
        super().__init__()
        self.gate = nn.Linear(config.n_embd, config.n_expert, bias=False)
        self.experts = nn.ModuleList(LLaMAMLP(config) for _ in range(config.n_expert))
        self.config = config
        self._stacks = None

    def _stack(self):
        """Stack the experts' packed weights per Linear ((E, N, K/2) / (E, N, K/group)) and re-point every
        expert's buffers at its slice, so the routed GEMVs and the grouped GEMMs index experts with one stride
        (done once: ``build_model`` calls it right after quantizing the block, so the first prompt does not pay the
        copy — 32 ms of Mixtral-8x7B's cold prefill in round 4)."""
        from lit_gpt.quantize import QuantLinear

        if self._stacks is not None and self._stacks[0][0].data_ptr() == self.experts[0].fc_1.qweight.data_ptr():
            return self._stacks
        out = []
        for name in ("fc_1", "fc_2", "proj"):
            lins = [getattr(e, name) for e in self.experts]
            l0 = lins[0]
            if not all(isinstance(l, QuantLinear) and l.bias is None and (l.fmt, l.group, l.qweight.shape) ==
                       (l0.fmt, l0.group, l0.qweight.shape) for l in lins):
                raise NotImplementedError("LLaMAMoE on the MI355X needs bias-free QuantLinear experts of one format")
            qw = torch.stack([l.qweight for l in lins])
            sc = torch.stack([l.scales for l in lins])
            for i, l in enumerate(lins):
                l.qweight, l.scales = qw[i], sc[i]
            out.append((qw, sc))
        self._stacks = out
        return out

    def _grouped_ok(self, C: int) -> bool:
        """The grouped prefill GEMMs take 4-bit experts whose shapes the fused MFMA kernel covers (else the loop)."""
        from lit_gpt.quantize import QuantLinear

        f1, pj = self.experts[0].fc_1, self.experts[0].proj
        if not isinstance(f1, QuantLinear) or not isinstance(pj, QuantLinear):
            return False
        return bool(ops.q4f_fits(64, f1.out_features, C, f1.group, f1.fmt)
                    and ops.q4f_fits(64, pj.out_features, pj.in_features, pj.group, pj.fmt))

    def _gate_route_ok(self, C: int) -> bool:
        """One-token routing through ``lga_moe_gate_route``: a bias-free 4-bit gate without forward hooks (the
        reference's TP keeps the gate replicated and hook-free, generate/tp.py:58-62) whose shape the kernel takes."""
        from lit_gpt.quantize import QuantLinear

        g = self.gate
        return (moe_gate_route and isinstance(g, QuantLinear) and g.bias is None and not g._forward_hooks
                and g.in_features == C and ops.moe_gate_route_fits(g.out_features, C))

    def _expert_hooks(self, x: torch.Tensor, eout: torch.Tensor) -> torch.Tensor:
        hooks = [list(e._forward_hooks.values()) for e in self.experts]
        if any(len(h) != len(hooks[0]) for h in hooks):
            raise NotImplementedError("LLaMAMoE: experts carry different forward hooks")
        for hook in hooks[0]:
            r = hook(self.experts[0], (x,), eout)
            eout = eout if r is None else r
        return eout

    def forward(self, x: torch.Tensor, *, norm: Optional["RMSNorm"] = None,
                residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``norm`` / ``residual``: Block fusion hooks (norm_2 in the gate / fc GEMV prologues, the residual in the
        combine)."""
        c = self.config
        lead, C = x.shape[:-1], x.shape[-1]
        x2 = x.reshape(-1, C).contiguous()
        T, k, E = x2.size(0), c.n_expert_per_token, c.n_expert
        (q1, s1), (q2, s2), (qp, sp) = self._stack()
        f1, pj = self.experts[0].fc_1, self.experts[0].proj
        res = None if residual is None else residual.reshape(T, C).contiguous()
        if T == 1:
            fuse_norm = norm is not None and ops.gemv_fuses_norm(C, dual=True)
            xin = x2 if (norm is None or fuse_norm) else norm(x2)
            nw = norm.weight if fuse_norm else None
            eps = norm.eps if fuse_norm else 1e-5
            if self._gate_route_ok(C):  # gate GEMV + routing in one launch (same bits as the pair below)
                g = self.gate
                ids, probs = ops.moe_gate_route(xin.view(-1), g.qweight, g.scales, E, C, g.group, g.fmt, k,
                                                norm_weight=nw, eps=eps)
            else:
                router = _lin(self.gate, xin, norm_weight=nw, norm_eps=eps).view(1, E)
                ids, probs = ops.moe_route(router, k)
            act = ops.q4_gemv_swiglu_experts(xin.view(-1), q1, s1, q2, s2, ids.view(-1), f1.out_features, C,
                                             f1.group, f1.fmt, norm_weight=nw, eps=eps)
            if (moe_pair_combine and res is not None and k == 2 and not any(e._forward_hooks for e in self.experts)
                    and ops.experts_pair_supported(pj.out_features, pj.in_features, pj.group, pj.fmt)):
                pw = getattr(self, "_pair_ws", None)
                if pw is None or pw.scratch.numel() != 2 * pj.out_features or pw.scratch.device != act.device:
                    pw = self._pair_ws = ops.ExpertsPairWorkspace(pj.out_features, act.device)
                return ops.q4_gemv_experts_pair_combine(act, qp, sp, ids.view(-1), probs.view(-1), res.view(-1),
                                                        pj.out_features, pj.in_features, pj.group, pj.fmt,
                                                        pw).view(*lead, C)
            eout = ops.q4_gemv_experts(act, qp, sp, ids.view(-1), pj.out_features, pj.in_features, pj.group,
                                       pj.fmt).view(1, k, C)
        else:
            n = x2 if norm is None else norm(x2)
            router = _lin(self.gate, n)
            ids, probs = ops.moe_route(router.contiguous(), k)
            if self._grouped_ok(C):
                # the reference's per-expert token groups (model.py:740-742) as two grouped launches over a
                # device-built tile table: no torch.where host sync, no gathered / scattered copies
                rows, bm = T * k, ops.moe_grouped_bm(T * k)
                tiles, x_rows, y_rows = ops.moe_group(ids, E, bm)
                g = ops.q4_gemm_swiglu_grouped(n.contiguous(), q1, s1, q2, s2, tiles, x_rows, rows,
                                               f1.out_features, C, f1.group, f1.fmt, bm, E)
                eout = ops.q4_gemm_grouped(g, qp, sp, tiles, y_rows, rows, pj.out_features, pj.in_features,
                                           pj.group, pj.fmt, bm, E).view(T, k, C)
            else:
                eout = torch.empty(T, k, C, dtype=torch.bfloat16, device=x2.device)
                for e in range(E):  # the reference's per-expert token groups (model.py:740-742)
                    tok, slot = torch.where(ids == e)
                    if tok.numel() == 0:
                        continue
                    xe = n.index_select(0, tok)
                    ex = self.experts[e]
                    g = ops.swiglu(_lin(ex.fc_1, xe).contiguous(), _lin(ex.fc_2, xe).contiguous())
                    eout[tok, slot] = _lin(ex.proj, g)
        eout = self._expert_hooks(x2, eout)
        return ops.moe_combine(eout.contiguous(), probs, ids, residual=res).view(*lead, C)


class LayerNorm(nn.LayerNorm):
    """config.norm_class for GPT-NeoX (reference config.py:137-144: torch.nn.LayerNorm) on the ``lga_layernorm``
    kernel: same parameters (weight, bias) and state-dict names, fp32 statistics, one bf16 cast."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:
            _gpu_only("LayerNorm")
        dt = torch.float32 if x.dtype == torch.float32 else torch.bfloat16  # 32-true or bf16-true
        w = self.weight.to(dt) if self.weight.dtype != dt else self.weight
        b = None if self.bias is None else (self.bias.to(dt) if self.bias.dtype != dt else self.bias)
        return ops.layernorm(x.contiguous(), w, b, self.eps)


class KVCache(nn.Module):
    def __init__(self, k_shape: Tuple[int, int, int, int], v_shape: Tuple[int, int, int, int],
                 device: Optional[torch.device] = None, dtype: Optional[torch.dtype] = None) -> None:
        super().__init__()
        self.register_buffer("k", torch.zeros(k_shape, device=device, dtype=dtype), persistent=False)
        self.register_buffer("v", torch.zeros(v_shape, device=device, dtype=dtype), persistent=False)

    def forward(self, input_pos: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Reference API (model.py:788-795); the fused path writes the cache inside ``lga_rope_kv_append``."""
        self.k = self.k.to(k.dtype)
        self.v = self.v.to(v.dtype)
        return self.k.index_copy_(2, input_pos, k), self.v.index_copy_(2, input_pos, v)

    def reset_parameters(self) -> None:
        torch.nn.init.zeros_(self.k)
        torch.nn.init.zeros_(self.v)


def build_rope_cache(seq_len: int, n_elem: int, device: Optional[torch.device] = None, base: int = 10000,
                     condense_ratio: int = 1) -> Tuple[torch.Tensor, torch.Tensor]:
    """cos/sin tables (seq_len, n_elem) in fp32 (model.py:746-764).

    The positions are a true division of an integer range, so (as in the reference) they take the DEFAULT dtype:
    under a bf16 default — the reference's ``fabric.init_tensor()`` with bf16-true / bnb precision around
    ``model.max_seq_length = ...`` (generate/base.py:153-157, generate/tp.py) — positions above 256 round to bf16
    before the fp32 outer product. ``generate.base.build_model(rope_positions=...)`` chooses that context.

    The tables are computed on the CPU (as the reference's CPU run computes them) and then moved to ``device``: the
    GPU's fp32 cos / sin of angles in the thousands of radians differ from the CPU's by up to ~1.6e-3 (measured at
    the 4k-32k rows of tests/golden/g5_rope_long.npz), the CPU's are the reference's values bit for bit."""
    inv_freq = torch.arange(0, n_elem, 2).float().div(n_elem)
    theta = 1.0 / torch.pow(float(base), inv_freq)
    positions = torch.arange(seq_len).div(condense_ratio)  # default dtype, see above
    angles = torch.outer(positions, theta).repeat(1, 2)
    cos, sin = torch.cos(angles), torch.sin(angles)
    return (cos, sin) if device is None else (cos.to(device), sin.to(device))


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """Reference helper (model.py:767-773); the hot path applies RoPE inside ``lga_rope_kv_append``."""
    half = x.size(-1) // 2
    rotated = torch.cat((-x[..., half:], x[..., :half]), dim=-1)
    return ((x * cos) + (rotated * sin)).to(dtype=x.dtype)


def build_mask_cache(max_seq_length: int, device: Optional[torch.device] = None) -> torch.Tensor:
    ones = torch.ones((max_seq_length, max_seq_length), device=device, dtype=torch.bool)
    return torch.tril(ones).unsqueeze(0).unsqueeze(0)


class CausalMask:
    """``GPT.mask_cache`` without the (1, 1, S, S) bool tensor (reference model.py:551-554,802-804 build it in
    ``set_kv_cache``): no kernel reads it — attention derives the mask row from ``input_pos`` — and at Mixtral's
    S = 32768 it would hold 1 GiB of HBM per rank. It keeps the reference's shape for ``size()`` / ``shape`` and
    materialises the tril tensor only if a caller indexes it (``mask_cache.index_select(2, input_pos)`` style)."""

    def __init__(self, max_seq_length: int, device: Optional[torch.device] = None) -> None:
        self.max_seq_length = max_seq_length
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self._t: Optional[torch.Tensor] = None

    @property
    def shape(self) -> torch.Size:
        return torch.Size((1, 1, self.max_seq_length, self.max_seq_length))

    def size(self, dim: Optional[int] = None):
        return self.shape if dim is None else self.shape[dim]

    def tensor(self) -> torch.Tensor:
        if self._t is None:
            self._t = build_mask_cache(self.max_seq_length, self.device)
        return self._t

    def __getitem__(self, item):
        return self.tensor()[item]

    def index_select(self, dim: int, index: torch.Tensor) -> torch.Tensor:
        return self.tensor().index_select(dim, index)
