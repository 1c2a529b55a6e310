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
fp4-b64 ("fp4"): bitsandbytes' FP4 code (get_4bit_type('fp4') = {0, .0625, 8, 12, 4, 6, 2, 3, -0, ...} / 12),
    blocks of 64, absmax fp32; code = dQuantizeFP4(w * (1/absmax)) — sign bit for x < 0, magnitude by strict >
    against bnb's seven literal pivots; dequant: w' = FP4[code] * absmax (dDequantizeFP4Tree's values).
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

# bitsandbytes 0.41.0 functional.get_4bit_type('fp4') (upstream, not vendored): the list divided by its absmax 12 in
# float32; the same values dDequantizeFP4Tree (csrc/kernels.cu) returns per code
FP4 = (np.array([0, 0.0625, 8.0, 12.0, 4.0, 6.0, 2.0, 3.0, -0.0, -0.0625, -8.0, -12.0, -4.0, -6.0, -2.0, -3.0],
                dtype=np.float32) / np.float32(12.0)).astype(np.float32)
# dQuantizeFP4's pivots (float literals in kernels.cu) between the sorted magnitudes and the code of each rank
FP4_PIVOTS = np.array([0.00260417, 0.0859375, 0.20833333, 0.29166667, 0.4166667, 0.583333, 0.8333333],
                      dtype=np.float32)
FP4_CODE_OF_RANK = np.array([0, 1, 6, 7, 4, 5, 2, 3], dtype=np.uint8)


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


def quantize_fp4(w: np.ndarray, block: int = 64) -> Tuple[np.ndarray, np.ndarray]:
    """(N, K) float32 -> (packed uint8 (N, K/2), absmax float32 (N, K/block)) — bnb quantize_4bit(quant_type='fp4')."""
    w = np.ascontiguousarray(w, dtype=np.float32)
    N, K = w.shape
    if K % block:
        raise ValueError(f"K={K} must be a multiple of the block size {block}")
    g = w.reshape(N, K // block, block)
    absmax = np.abs(g).max(axis=-1).astype(np.float32)
    with np.errstate(divide="ignore"):
        inv = np.where(absmax > 0, np.float32(1.0) / absmax, np.float32(0.0)).astype(np.float32)
    xn = (g * inv[..., None]).astype(np.float32)
    rank = (np.abs(xn)[..., None] > FP4_PIVOTS).sum(axis=-1)
    codes = FP4_CODE_OF_RANK[rank] + np.where(xn < 0, 8, 0).astype(np.uint8)
    return _pack_nibbles(codes.reshape(N, K)), absmax


def dequantize_fp4(packed: np.ndarray, absmax: np.ndarray, block: int = 64) -> np.ndarray:
    N = packed.shape[0]
    codes = _unpack_nibbles(packed)
    K = codes.shape[1]
    vals = FP4[codes].reshape(N, K // block, block)
    return (vals * absmax[..., None]).reshape(N, K).astype(np.float32)


def dequantize_nf4(packed: np.ndarray, absmax: np.ndarray, block: int = 64) -> np.ndarray:
    N = packed.shape[0]
    codes = _unpack_nibbles(packed)
    K = codes.shape[1]
    vals = NF4[codes].reshape(N, K // block, block)
    return (vals * absmax[..., None]).reshape(N, K).astype(np.float32)


def quantize_fmt(w: np.ndarray, fmt: int, group: int):
    """By the C-ABI format code: 0 int4-g, 1 nf4, 3 fp4 (include/litgpt_amd.h LGA_FMT_*)."""
    return {0: quantize_q4g, 1: quantize_nf4, 3: quantize_fp4}[fmt](w, group)


def dequantize_fmt(packed: np.ndarray, scales: np.ndarray, fmt: int, group: int) -> np.ndarray:
    return {0: dequantize_q4g, 1: dequantize_nf4, 3: dequantize_fp4}[fmt](packed, scales, group)


# ---- bitsandbytes double quantization of the nf4 absmax ("bnb.nf4-dq", compress_statistics=True) --------------
# Restated from bitsandbytes 0.41.0 (requirements-all.txt:3; not vendored in /root/reference, not importable here —
# parity unpinned): functional.quantize_4bit(compress_statistics=True) computes the per-64 absmax as nf4 does, then
#   offset = absmax.mean(); qabsmax, state2 = quantize_blockwise(absmax - offset, blocksize=256)
# with the signed 8-bit dynamic map (create_dynamic_map(signed=True, max_exponent_bits=7, total_bits=8)) and the
# kQuantizeBlockwise nearest-code binary search (dQuantize<0>); dequantize_4bit uses
#   absmax' = code[qabsmax] * absmax2[block] + offset      (fp32 multiply, then fp32 add)
# The 4-bit codes themselves stay those computed from the exact absmax.

def dynamic_map(max_exponent_bits: int = 7, total_bits: int = 8) -> np.ndarray:
    """bitsandbytes create_dynamic_map(signed=True): 256 sorted float32 values in [-1, 1]."""
    import torch

    data = []
    non_sign_bits = total_bits - 1
    additional_items = 2 ** (non_sign_bits - max_exponent_bits) - 1
    for i in range(max_exponent_bits):
        fraction_items = int(2 ** (i + non_sign_bits - max_exponent_bits) + 1)
        boundaries = torch.linspace(0.1, 1, fraction_items)
        means = (boundaries[:-1] + boundaries[1:]) / 2.0
        data += ((10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
        data += (-(10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
    if additional_items > 0:
        boundaries = torch.linspace(0.1, 1, additional_items + 1)
        means = (boundaries[:-1] + boundaries[1:]) / 2.0
        data += ((10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
        data += (-(10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
    data.append(0)
    data.append(1.0)
    data += [0] * (256 - len(data))
    data.sort()
    return np.array(data, dtype=np.float32)


def _dquantize(code: np.ndarray, x: np.float32) -> int:
    """kQuantizeBlockwise's dQuantize<0>: binary search over the sorted code, nearest of the bracketing pair."""
    pivot, upper_pivot, lower_pivot = 127, 255, 0
    lower, upper = np.float32(-1.0), np.float32(1.0)
    val = code[pivot]
    i = 64
    while i > 0:
        if x > val:
            lower_pivot, lower = pivot, val
            pivot += i
        else:
            upper_pivot, upper = pivot, val
            pivot -= i
        val = code[pivot]
        i >>= 1
    if upper_pivot == 255:
        upper = code[upper_pivot]
    if lower_pivot == 0:
        lower = code[lower_pivot]
    if x > val:
        mid = np.float32((upper + val) * np.float32(0.5))
        return upper_pivot if x > mid else pivot
    mid = np.float32((lower + val) * np.float32(0.5))
    return lower_pivot if x < mid else pivot


def double_quant_absmax(absmax: np.ndarray, block: int = 256):
    """nf4 absmax (any shape, flattened row-major as bnb's blocks) -> (qabsmax uint8, absmax2 float32 per 256,
    offset float32, absmax' float32 in the input shape: the dequantized statistic the GEMV / GEMM scale by).
    The mean is accumulated in float64 (the product's kernel does the same; bnb uses torch's fp32 mean)."""
    a = np.ascontiguousarray(absmax, dtype=np.float32).ravel()
    code = dynamic_map()
    offset = np.float32(a.astype(np.float64).sum() / a.size)
    v = (a - offset).astype(np.float32)
    n_blk = (a.size + block - 1) // block
    q = np.zeros(a.size, dtype=np.uint8)
    amax2 = np.zeros(n_blk, dtype=np.float32)
    for b in range(n_blk):
        blk = v[b * block:(b + 1) * block]
        m = np.float32(np.abs(blk).max())
        amax2[b] = m
        inv = np.float32(1.0) / m if m > 0 else np.float32(0.0)
        for j, x in enumerate(blk):
            q[b * block + j] = _dquantize(code, np.float32(x * inv)) if m > 0 else int(np.argmin(np.abs(code)))
    deq = (code[q] * np.repeat(amax2, block)[: a.size]).astype(np.float32)
    out = (deq + offset).astype(np.float32)
    return q, amax2, offset, out.reshape(np.shape(absmax))

