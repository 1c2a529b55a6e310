// Device helpers shared by the decode kernels (gemv.hip, attention.hip, layer.hip): int4/nf4 dequant-dot,
// wave reductions, bf16 unpacking, RoPE of a 16-lane key row, write-through (sc1) stores/loads.
#pragma once
#include "common.h"

namespace lga {

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ld_nt16(const void* p) {  // 16-B non-temporal load (weights are read once)
  const u32x4_t v = __builtin_nontemporal_load((const u32x4_t*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float dot2_f16(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2_t, a), __builtin_bit_cast(f16x2_t, b), c, false);
}

__device__ __forceinline__ float dot2_bf16(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), c,
                                         false);
}

#define LGA_DPP(v, ctrl) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xF, 0xF, false))

// DPP wave reduction -> uniform wave sum (used once per wave for the RMSNorm sum of squares)
__device__ __forceinline__ float wave_sum_uniform(float v) {
  v += LGA_DPP(v, 0xB1);   // quad [1,0,3,2]
  v += LGA_DPP(v, 0x4E);   // quad [2,3,0,1]
  v += LGA_DPP(v, 0x141);  // row half mirror
  v += LGA_DPP(v, 0x140);  // row mirror
  const int i = __float_as_int(v);
  return (__int_as_float(__builtin_amdgcn_readlane(i, 0)) + __int_as_float(__builtin_amdgcn_readlane(i, 16))) +
         (__int_as_float(__builtin_amdgcn_readlane(i, 32)) + __int_as_float(__builtin_amdgcn_readlane(i, 48)));
}

// Transposed butterfly over R in {2, 4, 8} per-lane partials a[0..R). Level with lane-distance D keeps one half
// of the values and adds the partner's other half. Afterwards lanes whose low log2(64/R) bits are 0 hold the
// full wave sum of value index  bfly_index<R>(lane).
template <int R>
__device__ __forceinline__ float butterfly(float* a, int lane) {
  constexpr int L = R == 8 ? 3 : (R == 4 ? 2 : 1);
#pragma unroll
  for (int lev = 0; lev < L; ++lev) {
    const int D = 32 >> lev;
    const int n = R >> (lev + 1);
    const bool h = lane & D;
#pragma unroll
    for (int i = 0; i < n; ++i) {
      // the pair as register values first: on two loads of the array, LLVM folds the selects below into ONE load
      // through a selected pointer, and the dynamically indexed array then lives in scratch (a store + load round
      // trip per level in every wave's tail; round 6)
      float lo = a[i], hi = a[i + n];
      asm volatile("" : "+v"(lo), "+v"(hi));
      const float send = h ? lo : hi, keep = h ? hi : lo;
      float recv;
      if (D == 8) recv = LGA_DPP(send, 0x128);  // row_ror:8 == xor 8 inside a 16-lane row
      else recv = __shfl_xor(send, D);
      a[i] = keep + recv;
    }
  }
  float d = a[0];
  // reduce over the remaining 64/R lanes (bits below the last exchange distance)
  d += LGA_DPP(d, 0xB1);
  d += LGA_DPP(d, 0x4E);
  d += LGA_DPP(d, 0x141);  // 8-lane groups done (R = 8)
  if (R <= 4) d += LGA_DPP(d, 0x140);  // 16-lane groups (R = 4)
  if (R <= 2) d += __shfl_xor(d, 16);  // 32-lane groups (R = 2)
  return d;
}
template <int R>
__device__ __forceinline__ int bfly_index(int lane) {
  return R == 8 ? ((lane >> 5) & 1) * 4 + ((lane >> 4) & 1) * 2 + ((lane >> 3) & 1)
                : (R == 4 ? ((lane >> 5) & 1) * 2 + ((lane >> 4) & 1) : ((lane >> 5) & 1));
}

#define kNF4v (kCode4[0])  // (lab engine)

// Scales stay raw bits until used: converting at load time makes the compiler wait for the scale load at once,
// and vmcnt is in order, so that wait would also drain every weight load issued before it.
template <int FMT>
__device__ __forceinline__ uint32_t load_scale_bits(const void* sc, size_t i) {
  return FMT == 0 ? (uint32_t)((const uint16_t*)sc)[i] : ((const uint32_t*)sc)[i];
}
template <int FMT>
__device__ __forceinline__ float scale_of(uint32_t bits) {
  return FMT == 0 ? __uint_as_float(bits << 16) : __uint_as_float(bits);
}

// (v & mask) | magic in ONE VOP3 op (v_and_or_b32): gfx9 VOP3 takes no literal, so both constants live in
// registers materialised once per kernel — the mask in a VGPR, the magic in an SGPR — behind asm the compiler
// cannot constant-fold (with literals it emits the two-op VOP2 and/or pair; as inline asm of its own the op
// would cost an s_nop hazard slot in front of every dependent v_dot2c).
__device__ __forceinline__ uint32_t and_or_magic(uint32_t v, uint32_t mask_vgpr, uint32_t magic_sgpr) {
  return (v & mask_vgpr) | magic_sgpr;
}
__device__ __forceinline__ uint32_t nibble_mask() {  // 0x000F000F in a VGPR, materialised once per kernel
  uint32_t m;
  asm volatile("v_mov_b32 %0, 0x000F000F" : "=v"(m));
  return m;
}

__device__ __forceinline__ uint32_t nibble_mask_hi() {  // 0x00F000F0 in a VGPR (fp16 int4 dot)
  uint32_t m;
  asm volatile("v_mov_b32 %0, 0x00F000F0" : "=v"(m));
  return m;
}
__device__ __forceinline__ uint32_t f16_magic() {  // 0x64006400 (fp16 pair 1024, 1024) in an SGPR
  uint32_t m;
  asm volatile("s_mov_b32 %0, 0x64006400" : "=s"(m));
  return m;
}

// Stage 8 activations (bf16 pairs d = (x0,x1) (x2,x3) (x4,x5) (x6,x7)) as the LDS pair layout the chunk dot reads:
// (x0,x4) (x1,x5) (x2,x6) (x3,x7); returns this thread's share of the chunk correction. nf4: bf16 pairs by byte
// permutes (the codebook FMAs read them), correction unused. int4: fp16 pairs with the odd slots pre-divided by 16
// (bf16 values convert exactly for |x| in [2^-10, 65504]; smaller ones round toward zero in fp16's subnormals, at
// most 2^-24 absolute), correction = 1032 sum x_even + 72 sum x_odd (see chunk_dot_rows).
template <int FMT>
__device__ __forceinline__ float stage_x8(const uint32_t (&d)[4], uint4& out) {
  if (FMT == 0) {
    const float x0 = bflo(d[0]), x1 = bfhi(d[0]), x2 = bflo(d[1]), x3 = bfhi(d[1]);
    const float x4 = bflo(d[2]), x5 = bfhi(d[2]), x6 = bflo(d[3]), x7 = bfhi(d[3]);
    const float k = 0.0625f;
    out = make_uint4(__builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(x0, x4)),
                     __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(x1 * k, x5 * k)),
                     __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(x2, x6)),
                     __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(x3 * k, x7 * k)));
    return 1032.0f * ((x0 + x2) + (x4 + x6)) + 72.0f * ((x1 + x3) + (x5 + x7));
  }
  out = make_uint4(__builtin_amdgcn_perm(d[2], d[0], 0x05040100u), __builtin_amdgcn_perm(d[2], d[0], 0x07060302u),
                   __builtin_amdgcn_perm(d[3], d[1], 0x05040100u), __builtin_amdgcn_perm(d[3], d[1], 0x07060302u));
  return ((bflo(d[0]) + bfhi(d[0])) + (bflo(d[1]) + bfhi(d[1]))) + ((bflo(d[2]) + bfhi(d[2])) + (bflo(d[3]) + bfhi(d[3])));
}

// Dot of R 16-byte weight chunks (32 nibbles each: the rows / matrices of a wave) against ONE x chunk, interleaved
// pair by pair: R independent accumulation chains give the scheduler work between each unpack and its dependent
// v_dot2c (one chain at a time leaves an s_nop hazard slot in front of every dot). Every caller (one-shot and
// streaming GEMV, every epilogue) goes through this function, so their results agree bit for bit.
//
// int4: fp16 magic bias — (w & 0x000F000F) | 0x64006400 = fp16 (1024 + q) and (w & 0x00F000F0) | 0x64006400 =
// fp16 (1024 + 16 q) need no shift for nibbles 0, 1 (4, 5) and one shared w >> 8 for 2, 3 (6, 7): 5 unpack ops
// per 8 weights (bf16's 128 + q bias needed 7: three shifts), fed to v_dot2c_f32_f16; with the odd x slots staged
// / 16, sum x (q - 8) = dot - (1032 sum x_even + 72 sum x_odd) = dot - corr. tools/gemv_variants.py, 7B shapes:
// qkv -0.2..0.4, o_proj -0.2, fc_1||fc_2 -0.6..0.8, mlp.proj -0.1..0.3, lm_head -0.8..1.1 us per launch vs the
// bf16 form. nf4: codebook values from LDS, fp32 FMAs against the bf16 x pairs.
template <int FMT, int R>
__device__ __forceinline__ void chunk_dot_rows(const uint4 (&w)[R], const uint4* xc, float corr, const float* nf4,
                                               uint32_t mask, uint32_t magic, uint32_t mask_hi, float (&d)[R]) {
#pragma unroll
  for (int r = 0; r < R; ++r) d[r] = 0.0f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint4 xv = xc[j];
    const uint32_t xp[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t wd = j == 0 ? w[r].x : (j == 1 ? w[r].y : (j == 2 ? w[r].z : w[r].w));
      if (FMT == 0) {
        const uint32_t w8 = wd >> 8;
        d[r] = dot2_f16(xp[0], and_or_magic(wd, mask, magic), d[r]);
        d[r] = dot2_f16(xp[1], and_or_magic(wd, mask_hi, magic), d[r]);
        d[r] = dot2_f16(xp[2], and_or_magic(w8, mask, magic), d[r]);
        d[r] = dot2_f16(xp[3], and_or_magic(w8, mask_hi, magic), d[r]);
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          d[r] = fmaf(nf4[(wd >> (4 * s)) & 0xF], bflo(xp[s]), d[r]);
          d[r] = fmaf(nf4[(wd >> (4 * s + 16)) & 0xF], bfhi(xp[s]), d[r]);
        }
      }
    }
  }
  if (FMT == 0) {  // ONE explicit op: left to -ffp-contract the compiler could fuse it differently per variant
#pragma unroll
    for (int r = 0; r < R; ++r) d[r] = __builtin_fmaf(-1.0f, corr, d[r]);
  }
}

// One workgroup = 4 independent waves (row slots); a wave handles RPR consecutive rows.
template <int LPR>
__device__ __forceinline__ float row_group_sum(float v) {
  // LPR = 16: full DPP row; LPR = 8: half row
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  if (LPR == 16) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
  return v;
}

__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
  const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = bflo(d[i]);
    f[2 * i + 1] = bfhi(d[i]);
  }
}

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// RoPE of the 8 dims a lane holds (full rotary, n_elem == HS == 128): rotate-half partner dims live 8 lanes away
// inside the 16-lane row group (DPP row_ror:8). Same math and rounding as lga_rope_kv_append / the reference
// (x*cos + rotated*sin in fp32, no FMA contraction, one bf16 cast).
__device__ __forceinline__ uint4 rope8(const uint4 raw, const float* cr, const float* sr, int sub) {
  const uint32_t d[4] = {raw.x, raw.y, raw.z, raw.w};
  uint32_t pd[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) pd[i] = __builtin_amdgcn_update_dpp(0, d[i], 0x128, 0xF, 0xF, false);
  const bool lo_half = sub < 8;
  uint32_t out[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float r0 = bflo(pd[i]), r1 = bfhi(pd[i]);
    if (lo_half) {
      r0 = -r0;
      r1 = -r1;
    }
    const float x0 = bflo(d[i]), x1 = bfhi(d[i]);
    out[i] = pack2(add_rn(mul_rn(x0, cr[2 * i]), mul_rn(r0, sr[2 * i])),
                   add_rn(mul_rn(x1, cr[2 * i + 1]), mul_rn(r1, sr[2 * i + 1])));
  }
  return make_uint4(out[0], out[1], out[2], out[3]);
}

}  // namespace lga
