"""Python view of the C-ABI library ``liblitgpt_amd.so`` (declared in ``include/litgpt_amd.h``).

Every hot op of the decode path is a HIP kernel in ``lit-gpt_amd/csrc`` reached through these thin wrappers:
they validate dtype / shape / contiguity / device, pass raw device pointers and sizes, launch on torch's
current HIP stream (so the calls can be captured into a HIP graph), and turn a non-zero return code into a
``RuntimeError`` carrying ``lga_last_error_string()``. There is no CPU fallback: without the library, or on a
non-GPU tensor, every op raises.

Reference boundary replaced: bitsandbytes' ctypes C functions behind ``Linear4bit`` and the ATen
kernels that ``lit_gpt/model.py`` issues (RMSNorm, RoPE, index_copy_, SDPA, embedding, argmax).
"""

from __future__ import annotations

import ctypes
import math
import os
from pathlib import Path
from typing import Optional

import torch

LIB_PATH = Path(os.environ.get("LGA_LIB", Path(__file__).resolve().parent / "_lib" / "liblitgpt_amd.so"))

FMT_Q4G = 0  # int4, symmetric, per-group bf16 scale
FMT_NF4 = 1  # bitsandbytes NF4 codebook, per-block fp32 absmax
FMT_BF16 = 2  # (prefill GEMM only) unquantized bf16 weight
FMT_FP4 = 3  # bitsandbytes FP4 code, per-block fp32 absmax

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_F = ctypes.c_float
_SZ = ctypes.c_size_t

# symbol -> argtypes; the exported surface of include/litgpt_amd.h (tests check the .so exports each one)
SIGNATURES = {
    "lga_version": [],
    "lga_last_error_string": [],
    "lga_device_info": [_I, _P, _P, _I],
    "lga_preload_kernels": [],
    "lga_quantize": [_P, _I, _P, _P, _I, _I, _I, _I, _P],
    "lga_nf4_double_quant": [_P, _L, _P, _P, _P],
    "lga_q4_gemv": [_P, _P, _P, _P, _P, _P, _F, _P, _I, _I, _I, _I, _I, _P],
    "lga_q4_gemv_swiglu": [_P, _P, _P, _P, _P, _P, _F, _P, _I, _I, _I, _I, _I, _P],
    "lga_q4_gemm": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "lga_q4f_fits": [_I, _I, _I, _I, _I],
    "lga_q4f_workspace_bytes": [_I, _I, _I, _I],
    "lga_q4_gemm_fused": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P],
    "lga_q4_gemm_swiglu": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P],
    "lga_q4_dequantize": [_P, _P, _P, _I, _I, _I, _I, _P],
    "lga_bf16_gemv": [_P, _P, _P, _P, _P, _F, _P, _I, _I, _P],
    "lga_bf16_gemv_swiglu": [_P, _P, _P, _P, _F, _P, _I, _I, _P],
    "lga_bf16_gemm": [_P, _P, _P, _P, _P, _I, _I, _I, _P],
    "lga_rmsnorm": [_P, _P, _P, _I, _I, _F, _P],
    "lga_rope_kv_append": [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P],
    "lga_embedding": [_P, _I, _P, _P, _I, _I, _I, _P],
    "lga_add": [_P, _P, _P, _L, _P],
    "lga_swiglu": [_P, _P, _P, _L, _P],
    "lga_layernorm": [_P, _P, _P, _P, _I, _I, _F, _P],
    "lga_gelu": [_P, _P, _L, _I, _P],
    "lga_attention": [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _F, _P],
    "lga_attention_workspace_bytes": [_I, _I, _I, _I],
    "lga_attention_decode_fused": [_P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _I, _F, _P],
    "lga_argmax": [_P, _I, _P, _P, _P, _P],
    "lga_q4_gemv_argmax_work_bytes": [_I, _I],
    "lga_q4_gemv_argmax_embed": [_P, _P, _P, _P, _F, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _I, _I, _P, _P],
    "lga_argmax_embed": [_P, _I, _P, _P, _P, _P, _I, _I, _P, _P],
    "lga_moe_route": [_P, _I, _I, _I, _P, _P, _P],
    "lga_moe_gate_route": [_P, _P, _P, _P, _F, _I, _I, _I, _I, _I, _P, _P, _P],
    "lga_q4_gemv_experts_pair_supported": [_I, _I, _I, _I],
    "lga_q4_gemv_experts_pair_counters": [_I],
    "lga_q4_gemv_experts_pair_combine": [_P, _P, _P, _P, _P, _P, _I, ctypes.c_longlong, ctypes.c_longlong, _P, _P,
                                         _P, _I, _I, _I, _I, _P],
    "lga_q4_gemv_experts": [_P, _P, _P, _P, _I, _I, ctypes.c_longlong, ctypes.c_longlong, _I, _P, _I, _I, _I, _I,
                            _I, _P],
    "lga_q4_gemv_swiglu_experts": [_P, _P, _P, _P, _P, _P, _I, _I, ctypes.c_longlong, ctypes.c_longlong, _P, _F,
                                   _P, _I, _I, _I, _I, _I, _P],
    "lga_moe_combine": [_P, _P, _P, _P, _P, _I, _I, _I, _P],
    "lga_moe_group_tiles": [_I, _I, _I],
    "lga_moe_group": [_P, _I, _I, _I, _I, _P, _P, _P, _P],
    "lga_q4_gemm_swiglu_grouped": [_P, _P, _P, _P, _P, ctypes.c_longlong, ctypes.c_longlong, _P, _P, _P, _I, _I, _I,
                                   _I, _I, _I, _I, _P],
    "lga_q4_gemm_grouped": [_P, _P, _P, ctypes.c_longlong, ctypes.c_longlong, _P, _P, _P, _P, _I, _I, _I, _I, _I,
                            _I, _I, _P],
    "lga_comm_mailbox_bytes": [_I],
    "lga_comm_alloc": [ctypes.c_size_t, ctypes.POINTER(_P), _P],
    "lga_comm_open": [_P, ctypes.POINTER(_P)],
    "lga_comm_close": [_P],
    "lga_comm_free": [_P],
    "lga_comm_trace": [_P, _I],
    "lga_allreduce_bf16": [_P, _P, _P, _I, ctypes.POINTER(_P), _I, _I, _I, _P, _P, _P],
    "lga_f32_linear": [_P, _P, _P, _P, _P, _I, _I, _I, _P],
    "lga_f32_layernorm": [_P, _P, _P, _P, _I, _I, _F, _P],
    "lga_f32_gelu": [_P, _P, _L, _I, _P],
    "lga_f32_add": [_P, _P, _P, _L, _P],
    "lga_f32_rope_kv_append": [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P],
    "lga_f32_attention": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _F, _P],
    "lga_argmax_f32": [_P, _I, _P, _P, _P, _P],
    "lga_sample_topk": [_P, _I, _I, _F, _P, ctypes.c_ulonglong, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P],
    "lga_q4_gemv_allreduce": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, ctypes.POINTER(_P), _I, _I, _I, _P, _P, _P,
                              _P],
    "lga_q4_gemv_allreduce_tagged": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, ctypes.POINTER(_P), _I, _I, _I, _P, _P,
                                     _P, _P],
}
_RESTYPES = {"lga_q4_gemv_experts_pair_counters": ctypes.c_size_t, "lga_q4f_workspace_bytes": ctypes.c_size_t, "lga_last_error_string": ctypes.c_char_p, "lga_attention_workspace_bytes": ctypes.c_size_t,
             "lga_comm_mailbox_bytes": ctypes.c_size_t, "lga_q4_gemv_argmax_work_bytes": ctypes.c_size_t}

_lib: Optional[ctypes.CDLL] = None


class NativeLibraryError(RuntimeError):
    pass


def load_library(path: Optional[Path] = None, strict: bool = True) -> ctypes.CDLL:
    """Load (once) and return the HIP library. Raises loudly when it is missing: there is no fallback.
    ``strict=False`` (lab A/B of older builds only) skips the symbols a library does not export."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path or LIB_PATH)
    if not p.is_file():
        raise NativeLibraryError(
            f"HIP library not found at {p}. Build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C lit-gpt_amd/csrc` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(str(p))
    for name, argtypes in SIGNATURES.items():
        if not strict and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    if path is None:
        _lib = lib
    return lib


def _check(rc: int) -> None:
    if rc != 0:
        msg = load_library().lga_last_error_string()
        raise RuntimeError(f"liblitgpt_amd error {rc}: {msg.decode() if msg else ''}")


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _dev(t: torch.Tensor, name: str, dtype: Optional[torch.dtype] = None) -> int:
    if not t.is_cuda:
        raise RuntimeError(f"{name}: expected a GPU tensor (this build has no CPU path), got {t.device}")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous tensor")
    return t.data_ptr()


def _opt(t: Optional[torch.Tensor], name: str, dtype=None) -> Optional[int]:
    return None if t is None else _dev(t, name, dtype)


# ------------------------------------------------------------------------------------------------ quantizer
def quantize(weight: torch.Tensor, fmt: int, group: int):
    """(N, K) fp32/bf16 device weight -> (packed uint8 (N, K/2), scales) on the same device."""
    N, K = weight.shape
    w = weight.contiguous()
    if w.dtype not in (torch.float32, torch.bfloat16):
        w = w.float()
    qw = torch.empty(N, K // 2, dtype=torch.uint8, device=w.device)
    sdt = torch.bfloat16 if fmt == FMT_Q4G else torch.float32
    sc = torch.empty(N, K // group, dtype=sdt, device=w.device)
    _check(load_library().lga_quantize(_dev(w, "weight"), int(w.dtype == torch.bfloat16), qw.data_ptr(),
                                       sc.data_ptr(), N, K, group, fmt, _stream()))
    return qw, sc


# ------------------------------------------------------------------------------------------------ linear
def nf4_double_quant(absmax: torch.Tensor, code: torch.Tensor) -> torch.Tensor:
    """In place: nf4 absmax (fp32, contiguous) -> bitsandbytes' double-quantized statistic; returns the offset."""
    off = torch.empty(1, dtype=torch.float32, device=absmax.device)
    _check(load_library().lga_nf4_double_quant(_dev(absmax, "absmax", torch.float32), absmax.numel(),
                                               _dev(code, "code", torch.float32), _dev(off, "offset", torch.float32),
                                               _stream()))
    return off


def q4_gemv(x, qweight, scales, N, K, group, fmt, *, bias=None, residual=None, norm_weight=None, eps=1e-5,
            out=None, variant=-1):
    """y (N,) = x (K,) . dequant(W)^T  [+bias] [+residual]; optional fused RMSNorm of x (norm_weight)."""
    y = out if out is not None else torch.empty(N, dtype=torch.bfloat16, device=x.device)
    _check(load_library().lga_q4_gemv(_dev(x, "x", torch.bfloat16), _dev(qweight, "qweight", torch.uint8),
                                      _dev(scales, "scales"), _opt(bias, "bias", torch.bfloat16),
                                      _opt(residual, "residual", torch.bfloat16),
                                      _opt(norm_weight, "norm_weight", torch.bfloat16), float(eps),
                                      _dev(y, "y", torch.bfloat16), N, K, group, fmt, variant, _stream()))
    return y


def q4_gemv_swiglu(x, qw1, sc1, qw2, sc2, N, K, group, fmt, *, norm_weight=None, eps=1e-5, out=None, variant=-1):
    """y (N,) = bf16(silu(bf16(x W1^T))) * bf16(x W2^T), optional fused RMSNorm of x."""
    y = out if out is not None else torch.empty(N, dtype=torch.bfloat16, device=x.device)
    _check(load_library().lga_q4_gemv_swiglu(_dev(x, "x", torch.bfloat16), _dev(qw1, "qw1", torch.uint8),
                                             _dev(sc1, "sc1"), _dev(qw2, "qw2", torch.uint8), _dev(sc2, "sc2"),
                                             _opt(norm_weight, "norm_weight", torch.bfloat16), float(eps),
                                             _dev(y, "y", torch.bfloat16), N, K, group, fmt, variant, _stream()))
    return y


def q4_gemm(x, qweight, scales, N, K, group, fmt, *, bias=None, residual=None, out=None):
    """Y (M, N) = X (M, K) . dequant(W)^T [+bias] [+residual] with MFMA tiles."""
    M = x.shape[0]
    y = out if out is not None else torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
    _check(load_library().lga_q4_gemm(_dev(x, "x", torch.bfloat16), _dev(qweight, "qweight", torch.uint8),
                                      _dev(scales, "scales"), _opt(bias, "bias", torch.bfloat16),
                                      _opt(residual, "residual", torch.bfloat16), _dev(y, "y", torch.bfloat16),
                                      M, N, K, group, fmt, _stream()))
    return y


def q4f_fits(M, N, K, group, fmt) -> bool:
    """Whether lga_q4_gemm_fused / lga_q4_gemm_swiglu take this shape (fmt 2 = bf16 weights)."""
    return bool(load_library().lga_q4f_fits(int(M), int(N), int(K), int(group), int(fmt)))


_Q4F_WS: dict = {}


def _q4f_workspace(M, N, K, swiglu, device):
    """The split-K workspace of a short-prompt fused GEMM: one zeroed buffer per device, grown as needed (its
    per-tile counters are left zeroed by every launch). Returns (ptr, bytes) or (None, 0)."""
    need = int(load_library().lga_q4f_workspace_bytes(int(M), int(N), int(K), int(bool(swiglu))))
    if need == 0:
        return None, 0
    ws = _Q4F_WS.get(device)
    if ws is None or ws.numel() < need:
        ws = _Q4F_WS[device] = torch.zeros(need, dtype=torch.uint8, device=device)
    return ws.data_ptr(), ws.numel()


def q4_gemm_fused(x, weight, scales, N, K, group, fmt, *, bias=None, residual=None, out=None):
    """Y (M, N) = X (M, K) . dequant(W)^T [+bias] [+residual], dequantization fused into the MFMA tiles
    (fmt 2: ``weight`` is the bf16 (N, K) matrix, ``scales`` None)."""
    M = x.shape[0]
    y = out if out is not None else torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
    wdt = torch.bfloat16 if fmt == 2 else torch.uint8
    ws, nws = _q4f_workspace(M, N, K, False, x.device)
    _check(load_library().lga_q4_gemm_fused(_dev(x, "x", torch.bfloat16), _dev(weight, "weight", wdt),
                                            _opt(scales, "scales"), _opt(bias, "bias", torch.bfloat16),
                                            _opt(residual, "residual", torch.bfloat16), _dev(y, "y", torch.bfloat16),
                                            M, N, K, group, fmt, ws, nws, _stream()))
    return y


def q4_gemm_swiglu(x, w1, s1, w2, s2, N, K, group, fmt, *, out=None):
    """G (M, N) = bf16(silu(bf16(X W1^T))) * bf16(X W2^T) in one launch (LLaMAMLP fc_1 / fc_2 / silu*mul)."""
    M = x.shape[0]
    y = out if out is not None else torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
    wdt = torch.bfloat16 if fmt == 2 else torch.uint8
    ws, nws = _q4f_workspace(M, N, K, True, x.device)
    _check(load_library().lga_q4_gemm_swiglu(_dev(x, "x", torch.bfloat16), _dev(w1, "w1", wdt), _opt(s1, "s1"),
                                             _dev(w2, "w2", wdt), _opt(s2, "s2"), _dev(y, "y", torch.bfloat16),
                                             M, N, K, group, fmt, ws, nws, _stream()))
    return y


def q4_dequantize(qweight, scales, N, K, group, fmt, *, out=None):
    """W (N, K) bf16 = bf16(value(nibble) * scale): the bits lga_q4_gemm stages (bnb dequantize_4bit)."""
    w = out if out is not None else torch.empty(N, K, dtype=torch.bfloat16, device=qweight.device)
    if w.numel() < N * K:
        raise ValueError(f"q4_dequantize: out holds {w.numel()} elements, needs {N * K}")
    _check(load_library().lga_q4_dequantize(_dev(qweight, "qweight", torch.uint8), _dev(scales, "scales"),
                                            _dev(w, "w", torch.bfloat16), N, K, group, fmt, _stream()))
    return w[: N * K].view(N, K) if w.dim() == 1 else w


def bf16_gemv(x, weight, *, bias=None, residual=None, norm_weight=None, eps=1e-5, out=None):
    """y (N,) = x (K,) . W (N, K)^T [+bias] [+residual] with bf16 weights; optional fused RMSNorm of x."""
    N, K = weight.shape
    y = out if out is not None else torch.empty(N, dtype=torch.bfloat16, device=x.device)
    _check(load_library().lga_bf16_gemv(_dev(x, "x", torch.bfloat16), _dev(weight, "weight", torch.bfloat16),
                                        _opt(bias, "bias", torch.bfloat16), _opt(residual, "residual", torch.bfloat16),
                                        _opt(norm_weight, "norm_weight", torch.bfloat16), float(eps),
                                        _dev(y, "y", torch.bfloat16), N, K, _stream()))
    return y


def bf16_gemv_swiglu(x, w1, w2, *, norm_weight=None, eps=1e-5, out=None):
    """y (N,) = bf16(silu(bf16(x W1^T))) * bf16(x W2^T) with bf16 weights, optional fused RMSNorm of x."""
    N, K = w1.shape
    if tuple(w2.shape) != (N, K):
        raise ValueError(f"bf16_gemv_swiglu: weight shapes differ {tuple(w1.shape)} vs {tuple(w2.shape)}")
    y = out if out is not None else torch.empty(N, dtype=torch.bfloat16, device=x.device)
    _check(load_library().lga_bf16_gemv_swiglu(_dev(x, "x", torch.bfloat16), _dev(w1, "w1", torch.bfloat16),
                                               _dev(w2, "w2", torch.bfloat16),
                                               _opt(norm_weight, "norm_weight", torch.bfloat16), float(eps),
                                               _dev(y, "y", torch.bfloat16), N, K, _stream()))
    return y


def bf16_gemm(x, weight, *, bias=None, residual=None, out=None):
    """Y (M, N) = X (M, K) . W (N, K)^T [+bias] [+residual] with bf16 weights on gemm.hip's MFMA tiles (bias and
    residual fused in its epilogue; the residual added after the product's bf16 rounding, as Block adds it)."""
    M = x.shape[0]
    N, K = weight.shape
    y = out if out is not None else torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
    _check(load_library().lga_bf16_gemm(_dev(x, "x", torch.bfloat16), _dev(weight, "weight", torch.bfloat16),
                                        _opt(bias, "bias", torch.bfloat16), _opt(residual, "residual", torch.bfloat16),
                                        _dev(y, "y", torch.bfloat16), M, N, K, _stream()))
    return y


# ------------------------------------------------------------------------------------------------ row ops
def rmsnorm(x, weight, eps, out=None):
    n = x.shape[-1]
    rows = x.numel() // n
    y = out if out is not None else torch.empty_like(x)
    _check(load_library().lga_rmsnorm(_dev(x, "x", torch.bfloat16), _dev(weight, "weight", torch.bfloat16),
                                      _dev(y, "y", torch.bfloat16), rows, n, float(eps), _stream()))
    return y


def rope_kv_append(qkv, k_cache, v_cache, cache_pos, rope_pos, cos, sin, n_head, n_query_groups, head_size,
                   rope_n_elem, q_out=None):
    """qkv (T, (H+2G)*hs) -> q (T, H, hs) roped with cos/sin rows rope_pos; k (roped) and v written into the
    (G, max_seq, hs) caches at rows cache_pos."""
    T = qkv.shape[0]
    max_seq = k_cache.shape[-2]
    q = q_out if q_out is not None else torch.empty(T, n_head, head_size, dtype=qkv.dtype, device=qkv.device)
    if qkv.dtype == torch.float32:  # --precision 32-true (csrc/fp32.hip)
        _check(load_library().lga_f32_rope_kv_append(
            _dev(qkv, "qkv", torch.float32), _dev(q, "q", torch.float32), _dev(k_cache, "k_cache", torch.float32),
            _dev(v_cache, "v_cache", torch.float32), _dev(cache_pos, "cache_pos", torch.int64),
            _dev(rope_pos, "rope_pos", torch.int64), _dev(cos, "cos", torch.float32), _dev(sin, "sin", torch.float32),
            cos.shape[0], T, n_head, n_query_groups, head_size, rope_n_elem, max_seq, _stream()))
        return q
    _check(load_library().lga_rope_kv_append(
        _dev(qkv, "qkv", torch.bfloat16), _dev(q, "q", torch.bfloat16), _dev(k_cache, "k_cache", torch.bfloat16),
        _dev(v_cache, "v_cache", torch.bfloat16), _dev(cache_pos, "cache_pos", torch.int64),
        _dev(rope_pos, "rope_pos", torch.int64), _dev(cos, "cos", torch.float32), _dev(sin, "sin", torch.float32),
        cos.shape[0], T, n_head, n_query_groups, head_size, rope_n_elem, max_seq, _stream()))
    return q


ATTN_COUNTER_STRIDE = 64  # uint32 per (row, group) arrival counter (kCounterStride in attention.hip)


class AttentionWorkspace:
    """Persistent split-attention scratch: fp32 partials + per-(row, group) arrival counters. The counters are
    zeroed once here; the kernel's last-arriving workgroup re-arms them, so the buffers are reusable across
    launches and HIP-graph replays (allocate before capture)."""

    def __init__(self, T: int, n_head: int, n_query_groups: int, head_size: int, n_splits: int, device) -> None:
        nbytes = load_library().lga_attention_workspace_bytes(T, n_head, head_size, n_splits)
        self.key = (T, n_head, n_query_groups, head_size, n_splits)
        self.partials = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=device)
        # one counter per (row, query group, head slice): at most n_head of them per row (csrc/attention.hip
        # attn_hsplit deals a group's heads to up to q_per_kv workgroups when the groups are few)
        self.counters = torch.zeros(T * n_head * ATTN_COUNTER_STRIDE, dtype=torch.int32, device=device)


def attention(q, k_cache, v_cache, input_pos, n_head, n_query_groups, head_size, scale, n_splits=1,
              workspace: Optional[AttentionWorkspace] = None, out=None):
    """y (T, H*hs): causal attention of q (T, H, hs) over the (G, max_seq, hs) caches, keys <= input_pos[t]."""
    T = q.shape[0]
    max_seq = k_cache.shape[-2]
    y = out if out is not None else torch.empty(T, n_head * head_size, dtype=q.dtype, device=q.device)
    if q.dtype == torch.float32:  # --precision 32-true: one workgroup per (row, head), no splits (csrc/fp32.hip)
        _check(load_library().lga_f32_attention(
            _dev(q, "q", torch.float32), _dev(k_cache, "k_cache", torch.float32),
            _dev(v_cache, "v_cache", torch.float32), _dev(input_pos, "input_pos", torch.int64),
            _dev(y, "y", torch.float32), T, n_head, n_query_groups, head_size, max_seq, float(scale), _stream()))
        return y
    if n_splits > 1:
        if workspace is None or workspace.key != (T, n_head, n_query_groups, head_size, n_splits):
            workspace = AttentionWorkspace(T, n_head, n_query_groups, head_size, n_splits, q.device)
        ws, cnt = _dev(workspace.partials, "workspace", torch.float32), _dev(workspace.counters, "counters", torch.int32)
    else:
        ws = cnt = None
    _check(load_library().lga_attention(
        _dev(q, "q", torch.bfloat16), _dev(k_cache, "k_cache", torch.bfloat16),
        _dev(v_cache, "v_cache", torch.bfloat16), _dev(input_pos, "input_pos", torch.int64),
        _dev(y, "y", torch.bfloat16), ws, cnt, T, n_head, n_query_groups, head_size, max_seq, n_splits, float(scale),
        _stream()))
    return y


def attention_decode_fused(qkv, k_cache, v_cache, cache_pos, rope_pos, cos, sin, n_head, n_query_groups,
                           head_size, rope_n_elem, scale, n_splits=1, workspace: Optional[AttentionWorkspace] = None,
                           out=None):
    """One decode token: RoPE + KV-append + attention in one launch. qkv (1, (H+2G)*hs) is the fused projection
    row; returns y (1, H*hs) and leaves roped k / v stored in the caches at cache_pos[0]."""
    if qkv.shape[0] != 1:
        raise ValueError("attention_decode_fused handles exactly one token (T = 1)")
    max_seq = k_cache.shape[-2]
    y = out if out is not None else torch.empty(1, n_head * head_size, dtype=torch.bfloat16, device=qkv.device)
    if n_splits > 1:
        if workspace is None or workspace.key != (1, n_head, n_query_groups, head_size, n_splits):
            workspace = AttentionWorkspace(1, n_head, n_query_groups, head_size, n_splits, qkv.device)
        ws, cnt = _dev(workspace.partials, "workspace", torch.float32), _dev(workspace.counters, "counters", torch.int32)
    else:
        ws = cnt = None
    _check(load_library().lga_attention_decode_fused(
        _dev(qkv, "qkv", torch.bfloat16), _dev(k_cache, "k_cache", torch.bfloat16),
        _dev(v_cache, "v_cache", torch.bfloat16), _dev(cache_pos, "cache_pos", torch.int64),
        _dev(rope_pos, "rope_pos", torch.int64), _dev(cos, "cos", torch.float32), _dev(sin, "sin", torch.float32),
        cos.shape[0], _dev(y, "y", torch.bfloat16), ws, cnt, n_head, n_query_groups, head_size, rope_n_elem, max_seq,
        n_splits, float(scale), _stream()))
    return y


class HeadWorkspace:
    """Scratch of the fused greedy head (lga_q4_gemv_argmax_embed): per-workgroup winners + arrival counters,
    zeroed once; the kernel re-arms its counters, so it is reusable across launches and graph replays."""

    def __init__(self, N: int, K: int, device) -> None:
        nbytes = load_library().lga_q4_gemv_argmax_work_bytes(N, K)
        self.key = (N, K)
        self.buf = torch.zeros((nbytes + 7) // 8, dtype=torch.int64, device=device)


def head_argmax_supported(lin) -> bool:
    """Whether lga_q4_gemv_argmax_embed covers this lm_head: a 4-bit QuantLinear with K <= 4096, no bias."""
    from lit_gpt.quantize import QuantLinear

    return (isinstance(lin, QuantLinear) and lin.bias is None and lin.in_features <= 4096
            and lin.in_features % 32 == 0 and lin.qweight.is_cuda)


def q4_gemv_argmax_embed(x, lin, work: HeadWorkspace, *, norm_weight=None, eps=1e-5, table=None, emb_out=None,
                         logits=None, out_idx=None, token_out=None, pos_inout=None):
    """Greedy decode head in one launch: logits = lm_head(RMSNorm(x)), token = argmax(logits) (torch.argmax order),
    the lga_argmax_embed bookkeeping (token_out, out_idx, pos_inout += 1, table row -> emb_out). Returns logits."""
    N, K = lin.out_features, lin.in_features
    logits = logits if logits is not None else torch.empty(N, dtype=torch.bfloat16, device=x.device)
    V, C = (table.shape if table is not None else (0, 0))
    _check(load_library().lga_q4_gemv_argmax_embed(
        _dev(x.reshape(-1), "x", torch.bfloat16), _dev(lin.qweight, "qweight", torch.uint8), _dev(lin.scales, "scales"),
        _opt(norm_weight, "norm_weight", torch.bfloat16), float(eps), _dev(logits, "logits", torch.bfloat16), N, K,
        lin.group, lin.fmt, _dev(work.buf, "work"), _opt(out_idx, "out_idx", torch.int64),
        _opt(token_out, "token_out", torch.int32), _opt(pos_inout, "pos_inout", torch.int64),
        _opt(table, "table", torch.bfloat16), C, V, _opt(emb_out, "emb_out", torch.bfloat16), _stream()))
    return logits


def preload_kernels() -> None:
    """Build the prefill path's kernel objects now (model load) rather than at their first launch
    (lga_preload_kernels; nothing runs on the GPU)."""
    _check(load_library().lga_preload_kernels())


_N_CU = None


def num_cus() -> int:
    """Compute units of the current device (lga_device_info)."""
    global _N_CU
    if _N_CU is None:
        n = ctypes.c_int(0)
        arch = ctypes.create_string_buffer(64)
        _check(load_library().lga_device_info(torch.cuda.current_device(), ctypes.byref(n), arch, 64))
        _N_CU = int(n.value)
    return _N_CU


def decode_fusable(head_size: int, rope_n_elem: int) -> bool:
    """Whether lga_attention_decode_fused covers this geometry (full rotary over 128-dim heads)."""
    return head_size == 128 and rope_n_elem == 128


def decode_splits(n_query_groups: int, q_per_kv: int, head_size: int, max_seq: int, n_cu: int = 256) -> int:
    """Sequence splits for T = 1 attention: one workgroup per CU across all query groups, at most 16 splits
    (tools/attn_sweep.py on MI355X, p = 2048..4000: 8 splits beat 16 for Llama-2-7B's 32 groups; with the few
    groups per rank of tensor parallelism 16 splits beat 32/64/128 — G = 4: 7.8 vs 10.9 us at 64 splits; G = 1,
    8 heads per group: 21 vs 34 us at 64 — because the last-arriving split's combine grows with the split count).
    Caches of >= 12k rows (a long prompt: generate/base.py sizes the cache to prompt + new tokens) take up to 32:
    with the log2-domain softmax, Mixtral 18.6 vs 19.3 us at p = 16000 and 28.4 vs 31.3 at 32066, its TP = 2 rank
    13.8 vs 14.9 and 20.3 vs 24.4; at 8000 16 still wins for Mixtral (13.0 vs 14.4) and ties at TP = 2
    (tools/attn_ab.py interleaved, round 5, profiles/r05z_attn_long_context.txt)."""
    s = max(1, min(n_cu // max(1, n_query_groups), 32 if max_seq >= 12288 else 16))
    return min(s, max(1, max_seq // 16), 256)


def embedding(idx, table, out=None):
    """out[t] = table[idx[t]]; bf16 or fp32 rows (fp32 rows move as pairs of 16-bit words: a byte copy)."""
    T = idx.numel()
    V, C = table.shape
    y = out if out is not None else torch.empty(T, C, dtype=table.dtype, device=table.device)
    if idx.dtype not in (torch.int32, torch.int64):
        raise TypeError(f"embedding: idx must be int32/int64, got {idx.dtype}")
    if table.dtype not in (torch.bfloat16, torch.float32):
        raise TypeError(f"embedding: table must be bf16 or fp32, got {table.dtype}")
    words = C * (2 if table.dtype == torch.float32 else 1)
    _check(load_library().lga_embedding(_dev(idx, "idx"), int(idx.dtype == torch.int64),
                                        _dev(table, "table", table.dtype), _dev(y, "y", table.dtype), T, words, V,
                                        _stream()))
    return y


def add(a, b, out=None):
    y = out if out is not None else torch.empty_like(a)
    if a.dtype == torch.float32:
        _check(load_library().lga_f32_add(_dev(a, "a", torch.float32), _dev(b, "b", torch.float32),
                                          _dev(y, "y", torch.float32), a.numel(), _stream()))
        return y
    _check(load_library().lga_add(_dev(a, "a", torch.bfloat16), _dev(b, "b", torch.bfloat16),
                                  _dev(y, "y", torch.bfloat16), a.numel(), _stream()))
    return y


def layernorm(x, weight, bias, eps, out=None):
    """torch.nn.LayerNorm over the last dim of a contiguous bf16 GPU tensor (GPT-NeoX)."""
    n = x.shape[-1]
    y = out if out is not None else torch.empty_like(x)
    if x.dtype == torch.float32:
        _check(load_library().lga_f32_layernorm(_dev(x, "x", torch.float32), _dev(weight, "weight", torch.float32),
                                                _opt(bias, "bias", torch.float32), _dev(y, "y", torch.float32),
                                                x.numel() // n, n, float(eps), _stream()))
        return y
    _check(load_library().lga_layernorm(_dev(x, "x", torch.bfloat16), _dev(weight, "weight", torch.bfloat16),
                                        _opt(bias, "bias", torch.bfloat16), _dev(y, "y", torch.bfloat16),
                                        x.numel() // n, n, float(eps), _stream()))
    return y


def gelu(a, approximate: str = "none", out=None):
    """bf16(F.gelu(a, approximate)) (GptNeoxMLP)."""
    if approximate not in ("none", "tanh"):
        raise ValueError(f"gelu approximate must be 'none' or 'tanh', got {approximate!r}")
    y = out if out is not None else torch.empty_like(a)
    if a.dtype == torch.float32:
        _check(load_library().lga_f32_gelu(_dev(a, "a", torch.float32), _dev(y, "y", torch.float32), a.numel(),
                                           int(approximate == "tanh"), _stream()))
        return y
    _check(load_library().lga_gelu(_dev(a, "a", torch.bfloat16), _dev(y, "y", torch.bfloat16), a.numel(),
                                   int(approximate == "tanh"), _stream()))
    return y


def swiglu(a, b, out=None):
    y = out if out is not None else torch.empty_like(a)
    _check(load_library().lga_swiglu(_dev(a, "a", torch.bfloat16), _dev(b, "b", torch.bfloat16),
                                     _dev(y, "y", torch.bfloat16), a.numel(), _stream()))
    return y


def argmax(logits, out_idx=None, token_out=None, pos_inout=None):
    """Greedy token (lowest index on ties); optionally writes the token buffer and advances input_pos."""
    n = logits.numel()
    idx = out_idx if out_idx is not None else torch.empty(1, dtype=torch.int64, device=logits.device)
    if logits.dtype == torch.float32:
        _check(load_library().lga_argmax_f32(_dev(logits, "logits", torch.float32), n,
                                             _dev(idx, "out_idx", torch.int64), _opt(token_out, "token_out", torch.int32),
                                             _opt(pos_inout, "pos_inout", torch.int64), _stream()))
        return idx
    _check(load_library().lga_argmax(_dev(logits, "logits", torch.bfloat16), n, _dev(idx, "out_idx", torch.int64),
                                     _opt(token_out, "token_out", torch.int32),
                                     _opt(pos_inout, "pos_inout", torch.int64), _stream()))
    return idx


def f32_linear(x, weight, bias=None, residual=None, out=None):
    """y (M, N) = x (M, K) . W (N, K)^T (+ bias) (+ residual), all fp32 (--precision 32-true, csrc/fp32.hip)."""
    N, K = weight.shape
    M = x.numel() // K
    y = out if out is not None else torch.empty(M, N, dtype=torch.float32, device=x.device)
    _check(load_library().lga_f32_linear(_dev(x, "x", torch.float32), _dev(weight, "weight", torch.float32),
                                         _opt(bias, "bias", torch.float32), _opt(residual, "residual", torch.float32),
                                         _dev(y, "y", torch.float32), M, N, K, _stream()))
    return y


def argmax_embed(logits, table, emb_out, out_idx=None, token_out=None, pos_inout=None):
    """argmax (as ``argmax``) + the embedding row of the chosen token written to ``emb_out`` (n_embd,) bf16 in
    the same launch (the next decode step's input)."""
    n = logits.numel()
    V, C = table.shape
    if emb_out.numel() != C:
        raise ValueError(f"argmax_embed: emb_out holds {emb_out.numel()} elements, the table rows {C}")
    idx = out_idx if out_idx is not None else torch.empty(1, dtype=torch.int64, device=logits.device)
    _check(load_library().lga_argmax_embed(_dev(logits, "logits", torch.bfloat16), n, _dev(idx, "out_idx", torch.int64),
                                           _opt(token_out, "token_out", torch.int32),
                                           _opt(pos_inout, "pos_inout", torch.int64), _dev(table, "table", torch.bfloat16),
                                           C, V, _dev(emb_out, "emb_out", torch.bfloat16), _stream()))
    return idx


MAX_TOP_K = 1024  # lga_sample_topk keeps at most this many logits
MAX_SAMPLE_VOCAB = 65536  # ... out of at most this many (one workgroup holds them in LDS)


def sample_topk(logits, top_k, temperature, *, uniform=None, seed=0, counter=None, out_idx=None, token_out=None,
                pos_inout=None, table=None, emb_out=None, kept_out=None, probs_out=None):
    """generate/base.py:30-41 at temperature > 0 with top_k (1..1024) in ONE launch (csrc/sample.hip
    topk_sample_kernel): top-k (ties lowest index first), softmax(logits / temperature) in bf16, inverse-CDF draw.
    ``uniform`` (1,) fp32 on the device fixes the draw (tests); otherwise ``counter`` (1,) int64 on the device is the
    RNG state (hash of ``seed`` and the counter; advanced per call, so the launch replays in a HIP graph). With
    ``table``/``emb_out`` the chosen token's embedding row is gathered as ``argmax_embed`` does. Returns out_idx."""
    n = logits.numel()
    if not 1 <= top_k <= MAX_TOP_K:
        raise ValueError(f"sample_topk: top_k must be in [1, {MAX_TOP_K}], got {top_k}")
    if uniform is None and counter is None:
        raise ValueError("sample_topk: needs uniform or an RNG counter")
    idx = out_idx if out_idx is not None else torch.empty(1, dtype=torch.int64, device=logits.device)
    V, C = (table.shape if table is not None else (0, 0))
    if emb_out is not None and (table is None or emb_out.numel() != C):
        raise ValueError("sample_topk: emb_out needs the embedding table and one row of it")
    _check(load_library().lga_sample_topk(
        _dev(logits, "logits", torch.bfloat16), n, int(top_k), float(temperature), _opt(uniform, "uniform", torch.float32),
        int(seed) & (2**64 - 1), _opt(counter, "counter", torch.int64), _dev(idx, "out_idx", torch.int64),
        _opt(token_out, "token_out", torch.int32), _opt(pos_inout, "pos_inout", torch.int64),
        _opt(table, "table", torch.bfloat16), C, V, _opt(emb_out, "emb_out", torch.bfloat16),
        _opt(kept_out, "kept_out", torch.int32), _opt(probs_out, "probs_out", torch.bfloat16), _stream()))
    return idx


# ------------------------------------------------------------------------------------------------ sparse MoE
def moe_route(logits, k, ids=None, probs=None):
    """(T, E) bf16 router logits -> (ids (T, k) int32, probs (T, k) bf16): torch.topk (CPU tie order) + fp32
    softmax over the k values, cast to bf16 (lit_gpt/model.py:737-738)."""
    T, E = logits.shape
    ids = ids if ids is not None else torch.empty(T, k, dtype=torch.int32, device=logits.device)
    probs = probs if probs is not None else torch.empty(T, k, dtype=torch.bfloat16, device=logits.device)
    _check(load_library().lga_moe_route(_dev(logits, "logits", torch.bfloat16), T, E, k, _dev(ids, "ids", torch.int32),
                                        _dev(probs, "probs", torch.bfloat16), _stream()))
    return ids, probs


def moe_gate_route_fits(n_expert: int, K: int) -> bool:
    """Whether lga_moe_gate_route takes this router gate (E <= 8 rows, K <= 6144, K % 32 == 0)."""
    return 0 < n_expert <= 8 and K % 32 == 0 and 0 < K <= 6144


def moe_gate_route(x, qweight, scales, n_expert, K, group, fmt, k, *, norm_weight=None, eps=1e-5, ids=None,
                   probs=None):
    """One token: router logits = gate(x) (4-bit GEMV, optional fused RMSNorm) and their routing in ONE launch ->
    (ids (1, k) int32, probs (1, k) bf16), bit-identical to q4_gemv + moe_route (lit_gpt/model.py:736-738)."""
    ids = ids if ids is not None else torch.empty(1, k, dtype=torch.int32, device=x.device)
    probs = probs if probs is not None else torch.empty(1, k, dtype=torch.bfloat16, device=x.device)
    _check(load_library().lga_moe_gate_route(_dev(x, "x", torch.bfloat16), _dev(qweight, "qweight", torch.uint8),
                                             _dev(scales, "scales"), _opt(norm_weight, "norm_weight", torch.bfloat16),
                                             float(eps), n_expert, K, group, fmt, k, _dev(ids, "ids", torch.int32),
                                             _dev(probs, "probs", torch.bfloat16), _stream()))
    return ids, probs


def experts_pair_supported(N: int, K: int, group: int, fmt: int) -> bool:
    """Whether lga_q4_gemv_experts_pair_combine covers this routed proj shape."""
    return bool(load_library().lga_q4_gemv_experts_pair_supported(N, K, group, fmt))


class ExpertsPairWorkspace:
    """Persistent scratch of lga_q4_gemv_experts_pair_combine for one MoE block (allocate before graph capture): the
    first-arriving slot's rows [2][N] bf16 and the per-row-block arrival counters (zeroed once, re-armed by the kernel)."""

    def __init__(self, N: int, device) -> None:
        self.scratch = torch.empty(2 * N, dtype=torch.bfloat16, device=device)
        self.counters = torch.zeros(int(load_library().lga_q4_gemv_experts_pair_counters(N)), dtype=torch.int32,
                                    device=device)


def q4_gemv_experts_pair_combine(x, qweight, scales, ids, probs, residual, N, K, group, fmt, ws, out=None):
    """One token, k = 2: y (N,) = residual + combine of the two routed proj GEMVs (slot s: x[s] against expert ids[s]
    of the (E, N, K/2) stack), bit-identical to q4_gemv_experts + moe_combine, in one launch."""
    if ids.numel() != 2 or probs.numel() != 2 or x.numel() != 2 * K or residual.numel() != N:
        raise ValueError("q4_gemv_experts_pair_combine: needs 2 slots (ids, probs, x of 2 x K) and a residual of N")
    y = out if out is not None else torch.empty(N, dtype=torch.bfloat16, device=x.device)
    ws_, ss_ = _expert_strides(qweight, scales)
    _check(load_library().lga_q4_gemv_experts_pair_combine(
        _dev(x, "x", torch.bfloat16), _dev(qweight, "qweight", torch.uint8), _dev(scales, "scales"),
        _dev(ids, "ids", torch.int32), _dev(probs, "probs", torch.bfloat16), _dev(residual, "residual", torch.bfloat16),
        qweight.size(0), ws_, ss_, _dev(y, "y", torch.bfloat16), _dev(ws.scratch, "scratch", torch.bfloat16),
        _dev(ws.counters, "counters", torch.int32), N, K, group, fmt, _stream()))
    return y


def _expert_strides(qweight, scales):
    if qweight.dim() != 3 or scales.dim() != 3:
        raise ValueError("expert weights must be stacked as (E, N, K/2) / (E, N, K/group)")
    return qweight.stride(0) * qweight.element_size(), scales.stride(0) * scales.element_size()


def q4_gemv_experts(x, qweight, scales, ids, N, K, group, fmt, *, out=None, variant=-1):
    """y (k, N): slot s = x[s] (k, K) . dequant(W[ids[s]])^T with W stacked (E, N, K/2)."""
    k = ids.numel()
    ws, ss = _expert_strides(qweight, scales)
    y = out if out is not None else torch.empty(k, N, dtype=torch.bfloat16, device=x.device)
    _check(load_library().lga_q4_gemv_experts(_dev(x, "x", torch.bfloat16), _dev(qweight, "qweight", torch.uint8),
                                              _dev(scales, "scales"), _dev(ids, "ids", torch.int32), k,
                                              qweight.size(0), ws, ss, K, _dev(y, "y", torch.bfloat16), N, K, group,
                                              fmt, variant, _stream()))
    return y


def q4_gemv_swiglu_experts(x, qw1, sc1, qw2, sc2, ids, N, K, group, fmt, *, norm_weight=None, eps=1e-5, out=None,
                           variant=-1):
    """y (k, N): slot s = bf16(silu(bf16(x W1[ids[s]]^T))) * bf16(x W2[ids[s]]^T), optional fused RMSNorm of x."""
    k = ids.numel()
    ws, ss = _expert_strides(qw1, sc1)
    if _expert_strides(qw2, sc2) != (ws, ss):
        raise ValueError("fc_1 and fc_2 expert stacks must share one stride")
    y = out if out is not None else torch.empty(k, N, dtype=torch.bfloat16, device=x.device)
    _check(load_library().lga_q4_gemv_swiglu_experts(
        _dev(x, "x", torch.bfloat16), _dev(qw1, "qw1", torch.uint8), _dev(sc1, "sc1"), _dev(qw2, "qw2", torch.uint8),
        _dev(sc2, "sc2"), _dev(ids, "ids", torch.int32), k, qw1.size(0), ws, ss,
        _opt(norm_weight, "norm_weight", torch.bfloat16), float(eps), _dev(y, "y", torch.bfloat16), N, K, group, fmt,
        variant, _stream()))
    return y


def moe_group(ids, n_expert, bm):
    """(T, k) int32 expert ids -> (tiles, x_rows, y_rows) of the grouped prefill GEMMs (lga_moe_group): the
    (token, slot) pairs sorted by expert on the device, m-tiles of ``bm`` rows; no host synchronisation."""
    T, k = ids.shape
    lib = load_library()
    cap = int(lib.lga_moe_group_tiles(T * k, int(n_expert), int(bm)))
    tiles = torch.empty(1 + 3 * cap, dtype=torch.int32, device=ids.device)
    x_rows = torch.empty(T * k, dtype=torch.int32, device=ids.device)
    y_rows = torch.empty(T * k, dtype=torch.int32, device=ids.device)
    _check(lib.lga_moe_group(_dev(ids, "ids", torch.int32), T, k, int(n_expert), int(bm), _dev(tiles, "tiles"),
                             _dev(x_rows, "x_rows"), _dev(y_rows, "y_rows"), _stream()))
    return tiles, x_rows, y_rows


def moe_grouped_bm(rows: int) -> int:
    """Tile height of the grouped prefill GEMMs for ``rows`` permuted rows (T * k)."""
    return 64 if rows <= 512 else 256


def q4_gemm_swiglu_grouped(x, w1, s1, w2, s2, tiles, x_rows, rows, N, K, group, fmt, bm, n_expert, *, out=None):
    """g (rows, N): permuted row r = bf16(silu(bf16(x[x_rows[r]] W1_e^T))) * bf16(x[x_rows[r]] W2_e^T), e the row's
    expert, W stacked (E, N, K/2) — every expert's rows in one launch."""
    ws, ss = _expert_strides(w1, s1)
    y = out if out is not None else torch.empty(rows, N, dtype=torch.bfloat16, device=x.device)
    _check(load_library().lga_q4_gemm_swiglu_grouped(
        _dev(x, "x", torch.bfloat16), _dev(w1, "w1", torch.uint8), _dev(s1, "s1"), _dev(w2, "w2", torch.uint8),
        _dev(s2, "s2"), ws, ss, _dev(tiles, "tiles", torch.int32), _dev(x_rows, "x_rows", torch.int32),
        _dev(y, "y", torch.bfloat16), int(rows), int(N), int(K), int(group), int(fmt), int(bm), int(n_expert),
        _stream()))
    return y


def q4_gemm_grouped(x, w, s, tiles, y_rows, rows, N, K, group, fmt, bm, n_expert, *, x_rows=None, out=None):
    """y[y_rows[r]] = x[r] W_e^T for every permuted row r (x rows in permuted order unless ``x_rows``)."""
    ws, ss = _expert_strides(w, s)
    y = out if out is not None else torch.empty(rows, N, dtype=torch.bfloat16, device=x.device)
    _check(load_library().lga_q4_gemm_grouped(
        _dev(x, "x", torch.bfloat16), _dev(w, "w", torch.uint8), _dev(s, "s"), ws, ss,
        _dev(tiles, "tiles", torch.int32), _opt(x_rows, "x_rows", torch.int32), _opt(y_rows, "y_rows", torch.int32),
        _dev(y, "y", torch.bfloat16), int(rows), int(N), int(K), int(group), int(fmt), int(bm), int(n_expert),
        _stream()))
    return y


def moe_combine(expert_out, probs, ids, residual=None, out=None):
    """(T, k, C) expert outputs -> (T, C): [residual +] sum over slots in ascending expert id of bf16(p * E)."""
    T, k, C = expert_out.shape
    y = out if out is not None else torch.empty(T, C, dtype=torch.bfloat16, device=expert_out.device)
    _check(load_library().lga_moe_combine(_dev(expert_out, "expert_out", torch.bfloat16),
                                          _dev(probs, "probs", torch.bfloat16), _dev(ids, "ids", torch.int32),
                                          _opt(residual, "residual", torch.bfloat16), _dev(y, "y", torch.bfloat16),
                                          T, k, C, _stream()))
    return y


def gemv_fuses_norm(K: int, dual: bool) -> bool:
    """Whether lga_q4_gemv(_swiglu) can fuse the RMSNorm prologue: the row must fit one K tile
    (64 lanes x 2 chunks x 32 for the dual SwiGLU GEMV, x 4 chunks otherwise)."""
    return K // 32 <= (128 if dual else 256)
