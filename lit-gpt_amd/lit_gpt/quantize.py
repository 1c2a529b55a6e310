"""4-bit weight-only quantized Linear — the drop-in for bitsandbytes' ``Linear4bit``.

Reference boundary ("Operator boundary being replaced"): any object used where ``nn.Linear`` is
expected — ``forward(x[..., in_features]) -> y[..., out_features]`` with attributes ``weight``, ``bias``,
``in_features``, ``out_features``. The reference gets it from Lightning's ``BitsandbytesPrecision(mode, dtype)``
whose ``convert_module`` swaps every ``nn.Linear`` (lm_head included: ``ignore_modules`` is not passed,
generate/base.py:133) and quantizes on the move to the GPU (generate/base.py:128-136, 168; generate/tp.py:171,
190). ``QuantizedPrecision`` mirrors that: ``convert_module`` swaps the Linears of a (possibly TP-sharded,
still float) model for ``QuantLinear`` modules that quantize their weight on the device with the HIP quantizer.

Modes:
  "int4-g128" (also "int4-g64", "int4-g32")  symmetric int4, per-group bf16 scale (BASELINE config 3)
  "nf4"  / "bnb.nf4"                          NF4 codebook, fp32 absmax per 64 (bitsandbytes nf4 layout)
  "bnb.nf4-dq"                                nf4 + bitsandbytes double quantization of the absmax (offset =
                                              mean, 8-bit dynamic-map codes per 256 blocks, fp32 absmax2): the
                                              kernels scale by the dequantized statistic code[q]*absmax2+offset,
                                              held expanded as fp32 per 64-block (lga_nf4_double_quant)
  "bnb.fp4" / "bnb.fp4-dq"                    bitsandbytes FP4 code ({0, .0625, 8, 12, 4, 6, 2, 3} / 12, sign
                                              bit), fp32 absmax per 64 (+ the same double quantization)
Group sizes must divide in_features; for a TP row-shard whose width is not a multiple of the requested group
(e.g. Llama-2-7B mlp.proj at TP=8: 1376) the largest of {128, 64, 32} that divides it is used.
"""

from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn as nn

from lit_gpt import ops

_DOUBLE_QUANT = {"bnb.nf4-dq", "bnb.fp4-dq"}
_CODE_CACHE = {}


def bnb_dynamic_map(device) -> torch.Tensor:
    """bitsandbytes create_dynamic_map(signed=True, max_exponent_bits=7, total_bits=8): the 256 sorted fp32 codes
    of the absmax double quantization (7 decades of 2^i linearly spaced means, +-, plus 0 and 1)."""
    key = str(device)
    if key not in _CODE_CACHE:
        data = []
        for i in range(7):
            b = torch.linspace(0.1, 1, 2 ** i + 1)
            means = ((b[:-1] + b[1:]) / 2.0) * (10 ** (-6 + i))
            data += means.tolist() + (-means).tolist()
        data += [0.0, 1.0]
        _CODE_CACHE[key] = torch.tensor(sorted(data), dtype=torch.float32, device=device)
    return _CODE_CACHE[key]


_MODES = {
    "int4-g128": (ops.FMT_Q4G, 128),
    "int4-g64": (ops.FMT_Q4G, 64),
    "int4-g32": (ops.FMT_Q4G, 32),
    "nf4": (ops.FMT_NF4, 64),
    "bnb.nf4": (ops.FMT_NF4, 64),
    "bnb.nf4-dq": (ops.FMT_NF4, 64),
    "bnb.fp4": (ops.FMT_FP4, 64),
    "bnb.fp4-dq": (ops.FMT_FP4, 64),
}


def parse_mode(mode: str):
    if mode not in _MODES:
        raise NotImplementedError(
            f"quantize mode {mode!r} is not supported on this build (supported: {sorted(_MODES)}); "
            "bnb.int8 (LLM.int8 outlier decomposition) has no MI355X kernel")
    return _MODES[mode]


def _fit_group(K: int, group: int) -> int:
    for g in (group, 128, 64, 32):
        if g <= group and K % g == 0:
            return g
    raise ValueError(f"in_features={K} is not a multiple of 32; no 4-bit group layout fits")


class QuantLinear(nn.Module):
    """Packed 4-bit weight ``qweight`` (N, K/2) uint8 + ``scales`` (N, K/group) on the GPU.

    ``forward`` dispatches like bitsandbytes' ``matmul_4bit``: one token -> fused dequant-GEMV
    (``lga_q4_gemv``), several -> MFMA GEMM with the dequantization fused (``lga_q4_gemm_fused``). ``weight`` is kept as an alias of the packed
    buffer so code that inspects ``linear.weight`` (e.g. ``.device``/``.dtype``) keeps working.
    """

    # lga_q4_gemv launch variant for one-token inputs (-1: the library's heuristic). The opt-in fused kernels
    # (attention + out-projection, out-projection + MoE gate) reproduce the 4-rows-per-wave form (variant 0); their
    # bit-identity A/B tests pin the unfused side to it
    gemv_variant = -1

    def __init__(self, in_features: int, out_features: int, fmt: int, group: int,
                 bias: Optional[torch.Tensor] = None, device=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.fmt, self.group = fmt, group
        self.register_buffer("qweight", torch.empty(out_features, in_features // 2, dtype=torch.uint8, device=device))
        sdt = torch.bfloat16 if fmt == ops.FMT_Q4G else torch.float32
        self.register_buffer("scales", torch.empty(out_features, in_features // group, dtype=sdt, device=device))
        self.bias = None if bias is None else nn.Parameter(bias.to(torch.bfloat16), requires_grad=False)

    @property
    def weight(self) -> torch.Tensor:
        return self.qweight

    @classmethod
    def from_float(cls, weight: torch.Tensor, bias: Optional[torch.Tensor], mode: str,
                   device: Optional[torch.device] = None) -> "QuantLinear":
        fmt, group = parse_mode(mode)
        N, K = weight.shape
        group = _fit_group(K, group)
        device = device or (weight.device if weight.is_cuda else torch.device("cuda", torch.cuda.current_device()))
        w = weight.detach().to(device)
        m = cls(K, N, fmt, group, None if bias is None else bias.detach().to(device), device=device)
        qw, sc = ops.quantize(w, fmt, group)
        m.qweight.copy_(qw)
        m.scales.copy_(sc)
        if mode in _DOUBLE_QUANT:
            m.dq_offset = ops.nf4_double_quant(m.scales, bnb_dynamic_map(device))
        return m

    def forward(self, x: torch.Tensor, *, residual: Optional[torch.Tensor] = None,
                norm_weight: Optional[torch.Tensor] = None, norm_eps: float = 1e-5) -> torch.Tensor:
        lead = x.shape[:-1]
        x2 = x.reshape(-1, self.in_features)
        if x2.dtype != torch.bfloat16:
            raise TypeError(f"QuantLinear expects bf16 activations (bf16-true), got {x2.dtype}")
        x2 = x2.contiguous()
        M = x2.shape[0]
        res = None if residual is None else residual.reshape(M, self.out_features).contiguous()
        if M == 1:
            if norm_weight is not None and not ops.gemv_fuses_norm(self.in_features, dual=False):
                x2, norm_weight = ops.rmsnorm(x2, norm_weight, norm_eps), None
            y = ops.q4_gemv(x2.view(-1), self.qweight, self.scales, self.out_features, self.in_features, self.group,
                            self.fmt, bias=self.bias, residual=None if res is None else res.view(-1),
                            norm_weight=norm_weight, eps=norm_eps, variant=self.gemv_variant)
        else:
            if norm_weight is not None:
                x2 = ops.rmsnorm(x2, norm_weight, norm_eps)
            if ops.q4f_fits(M, self.out_features, self.in_features, self.group, self.fmt):
                # several rows (prefill): the dequantization runs inside the MFMA tiles (csrc/gemm_q4f.hip) to the
                # bits bnb's dequantize_4bit writes — the reference's M > 1 path without a bf16 weight in HBM
                y = ops.q4_gemm_fused(x2, self.qweight, self.scales, self.out_features, self.in_features,
                                      self.group, self.fmt, bias=self.bias, residual=res)
            else:  # group 32 / K % 64: gemm.hip's 128 x 128 tiles (same staged weight bits)
                y = ops.q4_gemm(x2, self.qweight, self.scales, self.out_features, self.in_features, self.group,
                                self.fmt, bias=self.bias, residual=res)
        return y.view(*lead, self.out_features)

    def extra_repr(self) -> str:
        kind = {ops.FMT_Q4G: "int4", ops.FMT_NF4: "nf4", ops.FMT_FP4: "fp4"}[self.fmt]
        return f"in_features={self.in_features}, out_features={self.out_features}, {kind}, group={self.group}"


class QuantizedPrecision:
    """Stand-in for Lightning's ``BitsandbytesPrecision(mode, dtype)`` (generate/base.py:128-134)."""

    def __init__(self, mode: str, dtype: torch.dtype = torch.bfloat16) -> None:
        parse_mode(mode)
        if dtype != torch.bfloat16:
            raise NotImplementedError("the MI355X 4-bit path computes in bf16 (precision bf16-true)")
        self.mode, self.dtype = mode, dtype

    def convert_module(self, module: nn.Module, device: Optional[torch.device] = None) -> nn.Module:
        """Replace every ``nn.Linear`` (lm_head included) by a ``QuantLinear`` quantized on ``device``."""
        for name, child in list(module.named_children()):
            if isinstance(child, nn.Linear):
                setattr(module, name, QuantLinear.from_float(child.weight, child.bias, self.mode, device))
            else:
                self.convert_module(child, device)
        return module
