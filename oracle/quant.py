"""Weight formats of the build (int4-g128, nf4-b64) — TEST INFRASTRUCTURE ONLY (oracle/__init__.py).

The reference's quantized arithmetic lives in bitsandbytes 0.41.0 (requirements-all.txt:3), reached through
Lightning's ``BitsandbytesPrecision`` (generate/base.py:128-136). Neither is in this container, so
nf4/int4 arithmetic parity is *unpinned* against the reference; the contract is
"dequantize with this restatement, then the reference fp math". This module restates both formats
byte-for-byte so the HIP quantizer (csrc/quant.hip) and the GEMV/GEMM dequant are checked bit-exactly.

Formats (row-major over an (N, K) Linear weight, groups run along K):

int4-g128 ("q4g"): per group of G consecutive k (default 128):
    absmax = max |w| (computed in fp32); scale = bf16(absmax / 7); inv = 1/float(scale) (0 if scale == 0)
    q = clamp(rint(w * inv), -8, 7) (round-half-even); nibble = q + 8
    packed byte j of a row holds k = 2j in its low nibble and k = 2j + 1 in its high nibble
    dequant: w' = float(nibble - 8) * float(scale)
nf4-b64 ("nf4"): bitsandbytes' NF4 codebook (bnb ``get_4bit_type('nf4')``),
    blocks of 64 along K, absmax fp32; code = argmin_i |w/absmax - NF4[i]| (ties -> lower index)
    using the codebook midpoints; same nibble packing; dequant: w' = NF4[code] * absmax.
"""

from __future__ import annotations

from typing import Tuple

import numpy as np

NF4 = np.array([
    -1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453, -0.28444138169288635,
    -0.18477343022823334, -0.09105003625154495, 0.0, 0.07958029955625534, 0.16093020141124725,
    0.24611230194568634, 0.33791524171829224, 0.44070982933044434, 0.5626170039176941,
    0.7229568362236023, 1.0], dtype=np.float32)
NF4_MID = ((NF4[1:] + NF4[:-1]) * np.float32(0.5)).astype(np.float32)


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even fp32 -> bf16 bit pattern (uint16)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = np.isnan(x)
    if nan.any():
        r[nan] = 0x7FC0
    return r


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (b.astype(np.uint32) << 16).view(np.float32)


def _pack_nibbles(codes: np.ndarray) -> np.ndarray:
    codes = codes.astype(np.uint8)
    return (codes[..., 0::2] | (codes[..., 1::2] << 4)).astype(np.uint8)


def _unpack_nibbles(packed: np.ndarray) -> np.ndarray:
    lo = packed & 0x0F
    hi = packed >> 4
    out = np.empty(packed.shape[:-1] + (packed.shape[-1] * 2,), dtype=np.uint8)
    out[..., 0::2] = lo
    out[..., 1::2] = hi
    return out


def quantize_q4g(w: np.ndarray, group: int = 128) -> Tuple[np.ndarray, np.ndarray]:
    """(N, K) float32 -> (packed uint8 (N, K/2), scales bf16-bits uint16 (N, K/group))."""
    w = np.ascontiguousarray(w, dtype=np.float32)
    N, K = w.shape
    if K % group or group % 2:
        raise ValueError(f"K={K} must be a multiple of the group size {group}")
    g = w.reshape(N, K // group, group)
    absmax = np.abs(g).max(axis=-1)
    scale_bits = f32_to_bf16_bits(absmax / np.float32(7.0))
    scale = bf16_bits_to_f32(scale_bits)
    with np.errstate(divide="ignore"):
        inv = np.where(scale > 0, np.float32(1.0) / scale, np.float32(0.0)).astype(np.float32)
    q = np.clip(np.rint(g * inv[..., None]), -8, 7).astype(np.int32) + 8
    return _pack_nibbles(q.reshape(N, K)), scale_bits


def dequantize_q4g(packed: np.ndarray, scale_bits: np.ndarray, group: int = 128) -> np.ndarray:
    N = packed.shape[0]
    codes = _unpack_nibbles(packed).astype(np.float32) - np.float32(8.0)
    K = codes.shape[1]
    scale = bf16_bits_to_f32(scale_bits)
    return (codes.reshape(N, K // group, group) * scale[..., None]).reshape(N, K).astype(np.float32)


def quantize_nf4(w: np.ndarray, block: int = 64) -> Tuple[np.ndarray, np.ndarray]:
    """(N, K) float32 -> (packed uint8 (N, K/2), absmax float32 (N, K/block))."""
    w = np.ascontiguousarray(w, dtype=np.float32)
    N, K = w.shape
    if K % block:
        raise ValueError(f"K={K} must be a multiple of the block size {block}")
    g = w.reshape(N, K // block, block)
    absmax = np.abs(g).max(axis=-1).astype(np.float32)
    with np.errstate(divide="ignore"):
        inv = np.where(absmax > 0, np.float32(1.0) / absmax, np.float32(0.0)).astype(np.float32)
    xn = (g * inv[..., None]).astype(np.float32)
    # code = number of midpoints strictly below xn  (ties at a midpoint go to the lower code)
    codes = np.searchsorted(NF4_MID, xn.ravel(), side="left").reshape(xn.shape)
    return _pack_nibbles(codes.reshape(N, K)), absmax


def dequantize_nf4(packed: np.ndarray, absmax: np.ndarray, block: int = 64) -> np.ndarray:
    N = packed.shape[0]
    codes = _unpack_nibbles(packed)
    K = codes.shape[1]
    vals = NF4[codes].reshape(N, K // block, block)
    return (vals * absmax[..., None]).reshape(N, K).astype(np.float32)
