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
Group sizes must divide in_features; for a TP row-shard whose width is not a multiple of the requested group
(e.g. Llama-2-7B mlp.proj at TP=8: 1376) the largest of {128, 64, 32} that divides it is used.
"""

from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn as nn

from lit_gpt import ops

_DOUBLE_QUANT = {"bnb.nf4-dq"}
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
}


def parse_mode(mode: str):
    if mode not in _MODES:
        raise NotImplementedError(
            f"quantize mode {mode!r} is not supported on this build (supported: {sorted(_MODES)}); "
            "bnb.fp4 / bnb.int8 have no MI355X kernel")
    return _MODES[mode]


def _fit_group(K: int, group: int) -> int:
    for g in (group, 128, 64, 32):
        if g <= group and K % g == 0:
            return g
    raise ValueError(f"in_features={K} is not a multiple of 32; no 4-bit group layout fits")


# Prefill GEMM for M > 1 rows: "fused" = lga_q4_gemm_fused (dequantization inside the MFMA tiles) from
# FUSED_GEMM_MIN_M rows; "blaslt" = dequantize + hipBLASLt (LGA_PREFILL_GEMM=blaslt, for A/B runs).
PREFILL_GEMM = os.environ.get("LGA_PREFILL_GEMM", "blaslt")
FUSED_GEMM_MIN_M = 16

# prefill rows from which dequantize + the library bf16 GEMM beats the fused int4 GEMM (tools/gemm_rates.py, Llama-2-7B
# layer: 0.21 vs 0.44 ms at M = 64, 0.63 vs 1.04 ms at M = 2048; gemm.hip's 128-row tiles idle most CUs below M = 256)
DEQUANT_GEMM_MIN_M = 16
_SCRATCH: dict = {}


# Prefill weight cache: a Linear keeps the bf16 weight its first long prefill dequantized (the same bits
# lga_q4_dequantize writes every time) and later prefills skip the dequantize pass — 0.13 ms of HBM-bound work per
# Llama-2-7B layer, the largest non-GEMM cost of a warm 2048-token prefill. Decode keeps streaming the packed 4-bit
# weights. Costs 2 bytes per weight of HBM: 13 GB for Llama-2-7B of an MI355X's 288 GB, so it is bounded per device
# by PREFILL_CACHE_FRACTION of the device memory and by what is free (keeping PREFILL_CACHE_HEADROOM free); a Linear
# that does not fit dequantizes into the shared scratch as before. LGA_PREFILL_CACHE=0 turns it off.
PREFILL_CACHE = os.environ.get("LGA_PREFILL_CACHE", "1") != "0"
PREFILL_CACHE_FRACTION = 0.25
PREFILL_CACHE_HEADROOM = 16 << 30
_CACHED_BYTES: dict = {}


def _cache_admits(nbytes: int, device: torch.device) -> bool:
    if not PREFILL_CACHE:
        return False
    free, total = torch.cuda.mem_get_info(device)
    used = _CACHED_BYTES.get(device, 0)
    return used + nbytes <= PREFILL_CACHE_FRACTION * total and free - nbytes >= PREFILL_CACHE_HEADROOM


def _dequant_scratch(numel: int, device: torch.device) -> torch.Tensor:
    """One growing bf16 buffer per device for dequantized weights: the Linears of a forward run one after
    another on the device's stream, so one buffer serves them all."""
    buf = _SCRATCH.get(device)
    if buf is None or buf.numel() < numel:
        buf = _SCRATCH[device] = torch.empty(numel, dtype=torch.bfloat16, device=device)
    return buf


class QuantLinear(nn.Module):
    """Packed 4-bit weight ``qweight`` (N, K/2) uint8 + ``scales`` (N, K/group) on the GPU.

    ``forward`` dispatches like bitsandbytes' ``matmul_4bit``: one token -> fused dequant-GEMV
    (``lga_q4_gemv``), several -> MFMA GEMM (``lga_q4_gemm``). ``weight`` is kept as an alias of the packed
    buffer so code that inspects ``linear.weight`` (e.g. ``.device``/``.dtype``) keeps working.
    """

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
                            norm_weight=norm_weight, eps=norm_eps)
        else:
            if norm_weight is not None:
                x2 = ops.rmsnorm(x2, norm_weight, norm_eps)
            if PREFILL_GEMM == "fused" and M >= FUSED_GEMM_MIN_M and ops.q4f_fits(M, self.out_features,
                                                                                  self.in_features, self.group,
                                                                                  self.fmt):
                # dequantization fused into the MFMA tiles (csrc/gemm_q4f.hip): no bf16 weight in HBM
                y = ops.q4_gemm_fused(x2, self.qweight, self.scales, self.out_features, self.in_features,
                                      self.group, self.fmt, bias=self.bias, residual=res)
            elif M >= DEQUANT_GEMM_MIN_M:
                # long prefill: dequantize to bf16 once (bnb's dequantize_4bit, the reference's own M > 1 path),
                # then the library bf16 GEMM (hipBLASLt): 1.1-1.25 PFLOP/s vs 0.5-0.7 for the fused int4 GEMM at
                # M = 2048, the dequantize pass included (tools/gemm_rates.py)
                y = ops.bf16_gemm(x2, self._prefill_weight(x2.device), bias=self.bias, residual=res)
            else:
                y = ops.q4_gemm(x2, self.qweight, self.scales, self.out_features, self.in_features, self.group,
                                self.fmt, bias=self.bias, residual=res)
        return y.view(*lead, self.out_features)

    def _prefill_weight(self, device: torch.device) -> torch.Tensor:
        """bf16(dequant(W)) for the library GEMM: the cached copy when it is current (same packed weights and
        scales as when it was made), else a fresh dequantize — into a cache buffer if the device budget admits one,
        into the shared scratch otherwise."""
        try:
            key = (self.qweight.data_ptr(), self.qweight._version, self.scales.data_ptr(), self.scales._version)
        except RuntimeError:  # inference tensors keep no version counter: an in-place change would go unseen
            key = None
        cached = getattr(self, "_w_bf16", None)
        if cached is not None and self._w_key == key:
            return cached
        if cached is not None:  # weights changed in place (e.g. load_state_dict): drop the stale copy
            _CACHED_BYTES[cached.device] = _CACHED_BYTES.get(cached.device, 0) - cached.numel() * 2
            self._w_bf16 = None
        N, K = self.out_features, self.in_features
        if key is not None and _cache_admits(N * K * 2, device):
            out = torch.empty(N, K, dtype=torch.bfloat16, device=device)
            _CACHED_BYTES[device] = _CACHED_BYTES.get(device, 0) + N * K * 2
            self._w_bf16, self._w_key = out, key
        else:
            out = _dequant_scratch(N * K, device)
        return ops.q4_dequantize(self.qweight, self.scales, N, K, self.group, self.fmt, out=out)

    def extra_repr(self) -> str:
        kind = "int4" if self.fmt == ops.FMT_Q4G else "nf4"
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
