// Batch-1 decode GEMV over packed 4-bit weights: y[n] = sum_k x[k] * dequant(W)[n, k]  (+ fused epilogues)
//
// Replaces the bitsandbytes 4-bit GEMV that `Linear4bit.forward` dispatches for one-token inputs
// (bnb `matmul_4bit` -> `gemv_4bit`, reached via BitsandbytesPrecision at reference generate/base.py:128-136)
// for every Linear of the decode step: qkv (lit_gpt/model.py:619), attn proj (:656), LLaMAMLP fc_1/fc_2/proj
// (:712-716) and lm_head (:519).
//
// MI355X design (HBM-bound, ~1 flop/byte):
//  * weights stream once from HBM as 16-byte-per-lane coalesced loads (1 KiB per wave-instruction);
//  * the activation row is staged once per workgroup in LDS (bf16, pair-permuted so that one AND-OR turns
//    a nibble pair into a bf16 pair "128 + q"), optionally RMS-normalised in the prologue (fused RMSNorm,
//    lit_gpt/rmsnorm.py:19-25), with per-32-element sums for the "-8" offset;
//  * int4-g: v_dot2c_f32_bf16 on (x_k, x_k+4) x (128+q_k, 128+q_k+4) pairs, one scale FMA per 32 weights;
//    nf4: 16-entry codebook in LDS, fp32 FMAs, one absmax multiply per 32 weights;
//  * a wave owns RW rows x (1/KS of K); 4 waves per 256-thread workgroup; wave sums via DPP + readlane;
//  * epilogues: +bias, +residual (Block residual add, model.py:591-592), dual-weight SwiGLU
//    (silu(fc_1 x) * fc_2 x, model.py:715) with the reference's bf16 rounding points.
#include "common.h"

namespace lga {

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt16(const void* p) {  // 16-B non-temporal load (weights are read once)
  const u32x4_t v = __builtin_nontemporal_load((const u32x4_t*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ float dot2_bf16(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), c,
                                         false);
}

// DPP wave reduction: every lane of each 16-lane row gets the row sum, then 4 readlanes -> uniform sum.
__device__ __forceinline__ float dpp_row_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));  // quad [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));  // quad [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));  // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));  // row_mirror
  return v;
}
__device__ __forceinline__ float wave_sum_uniform(float v) {
  v = dpp_row_sum(v);
  const int i = __float_as_int(v);
  return __int_as_float(__builtin_amdgcn_readlane(i, 0)) + __int_as_float(__builtin_amdgcn_readlane(i, 16)) +
         __int_as_float(__builtin_amdgcn_readlane(i, 32)) + __int_as_float(__builtin_amdgcn_readlane(i, 48));
}

struct GemvArgs {
  const uint16_t* x;         // [K] bf16
  const uint8_t* qw;         // [N][K/2]
  const void* sc;            // q4g: bf16 [N][K/G]; nf4: f32 [N][K/G]
  const uint8_t* qw2;        // dual: second weight (fc_2)
  const void* sc2;
  const uint16_t* bias;      // [N] or null
  const uint16_t* residual;  // [N] or null
  const uint16_t* norm_w;    // [K] or null (fused RMSNorm)
  uint16_t* y;               // [N]
  int N, K, G;
  float eps;
};

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;

__device__ __forceinline__ float load_scale(const void* sc, size_t i, int fmt) {
  return fmt == 0 ? bf2f(((const uint16_t*)sc)[i]) : ((const float*)sc)[i];
}

// dot of one 16-byte weight chunk (32 nibbles) with the LDS x chunk; returns the *unscaled* partial
template <int FMT>
__device__ __forceinline__ float chunk_dot(const uint4 w, const uint4* xl, float xsum, const float* nf4) {
  const uint32_t wd[4] = {w.x, w.y, w.z, w.w};
  if (FMT == 0) {
    float d = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 xv = xl[j];
      const uint32_t xp[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const uint32_t q = ((wd[j] >> (4 * s)) & 0x000F000Fu) | 0x43004300u;  // bf16 pair (128+q_s, 128+q_s+4)
        d = dot2_bf16(xp[s], q, d);
      }
    }
    return d - 136.0f * xsum;
  } else {
    float d = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 xv = xl[j];
      const uint32_t xp[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        d = fmaf(nf4[(wd[j] >> (4 * s)) & 0xF], bflo(xp[s]), d);
        d = fmaf(nf4[(wd[j] >> (4 * s + 16)) & 0xF], bfhi(xp[s]), d);
      }
    }
    return d;
  }
}

// Stage x (optionally RMS-normalised, rounded to bf16 like the reference's `.to(dtype)`) into LDS.
// Layout: per 8-element group, dwords (x0,x4),(x1,x5),(x2,x6),(x3,x7); xsum[c] = sum of chunk c (32 elems).
__device__ void stage_x(const GemvArgs& a, uint4* xl, float* xsum, float* red) {
  const int tid = threadIdx.x;
  const int n8 = a.K / 8;
  float rs = 1.0f;
  if (a.norm_w) {
    float ss = 0.0f;
    for (int i = tid; i < n8; i += kThreads) {
      const uint4 v = ((const uint4*)a.x)[i];
      const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float lo = bflo(d[j]), hi = bfhi(d[j]);
        ss = fmaf(lo, lo, ss);
        ss = fmaf(hi, hi, ss);
      }
    }
    ss = wave_sum_uniform(ss);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
    __syncthreads();
    const float tot = red[0] + red[1] + red[2] + red[3];
    rs = 1.0f / sqrtf(tot / (float)a.K + a.eps);
  }
  for (int i = tid; i < n8; i += kThreads) {
    const uint4 v = ((const uint4*)a.x)[i];
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
    float e[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      e[2 * j] = bflo(d[j]);
      e[2 * j + 1] = bfhi(d[j]);
    }
    if (a.norm_w) {
      const uint4 wv = ((const uint4*)a.norm_w)[i];
      const uint32_t wd[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        e[2 * j] = round_bf(__fmul_rn(bflo(wd[j]), __fmul_rn(e[2 * j], rs)));
        e[2 * j + 1] = round_bf(__fmul_rn(bfhi(wd[j]), __fmul_rn(e[2 * j + 1], rs)));
      }
    }
    xl[i] = make_uint4(pack2(e[0], e[4]), pack2(e[1], e[5]), pack2(e[2], e[6]), pack2(e[3], e[7]));
    float s = ((e[0] + e[1]) + (e[2] + e[3])) + ((e[4] + e[5]) + (e[6] + e[7]));
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    if ((i & 3) == 0) xsum[i >> 2] = s;
  }
}

template <int RW, int KS, int FMT, bool DUAL>
__global__ void __launch_bounds__(kThreads) gemv_q4_kernel(GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* xl = (uint4*)smem;                                  // K * 2 bytes
  float* xsum = (float*)(smem + (size_t)a.K * 2);            // K/32 floats
  float* part = xsum + a.K / 32;                             // [4 waves][RW][2]
  float* nf4 = part + kWaves * RW * 2;                       // 16 floats
  float* red = nf4 + 16;                                     // 4 floats
  if (FMT == 1 && threadIdx.x < 16) {
    const float cb[16] = {-1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
                          -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
                          0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f,
                          0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
                          0.7229568362236023f, 1.0f};
    nf4[threadIdx.x] = cb[threadIdx.x];
  }
  stage_x(a, xl, xsum, red);
  __syncthreads();

  constexpr int RS = kWaves / KS;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rs = wave / KS, ks = wave % KS;
  const int row0 = (blockIdx.x * RS + rs) * RW;
  const int NC = a.K / 32, groups = a.K / a.G;
  const int cps = (NC + KS - 1) / KS;
  const int c_beg = ks * cps, c_end = min(NC, c_beg + cps);
  const size_t row_bytes = (size_t)a.K / 2;

  const uint8_t* wrow[RW];
  const uint8_t* wrow2[RW];
  int srow[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int n = min(row0 + r, a.N - 1);
    wrow[r] = a.qw + (size_t)n * row_bytes;
    wrow2[r] = DUAL ? a.qw2 + (size_t)n * row_bytes : nullptr;
    srow[r] = n * groups;
  }
  float acc[RW], acc2[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) acc[r] = acc2[r] = 0.0f;

#pragma unroll 2
  for (int c = c_beg + lane; c < c_end; c += kWave) {
    uint4 wv[RW], wv2[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      wv[r] = ld_nt16(wrow[r] + (size_t)c * 16);
      if (DUAL) wv2[r] = ld_nt16(wrow2[r] + (size_t)c * 16);
    }
    const int gi = (c * 32) / a.G;
    float s[RW], s2[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      s[r] = load_scale(a.sc, (size_t)srow[r] + gi, FMT);
      if (DUAL) s2[r] = load_scale(a.sc2, (size_t)srow[r] + gi, FMT);
    }
    const float xs = xsum[c];
    const uint4* xc = xl + c * 4;
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      acc[r] = fmaf(s[r], chunk_dot<FMT>(wv[r], xc, xs, nf4), acc[r]);
      if (DUAL) acc2[r] = fmaf(s2[r], chunk_dot<FMT>(wv2[r], xc, xs, nf4), acc2[r]);
    }
  }

  float tot[RW], tot2[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    tot[r] = wave_sum_uniform(acc[r]);
    tot2[r] = DUAL ? wave_sum_uniform(acc2[r]) : 0.0f;
  }
  if (KS > 1) {
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        part[(wave * RW + r) * 2] = tot[r];
        part[(wave * RW + r) * 2 + 1] = tot2[r];
      }
    }
    __syncthreads();
    if (ks != 0) return;
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      float t = 0.0f, t2 = 0.0f;
      for (int k = 0; k < KS; ++k) {
        t += part[((rs * KS + k) * RW + r) * 2];
        t2 += part[((rs * KS + k) * RW + r) * 2 + 1];
      }
      tot[r] = t;
      tot2[r] = t2;
    }
  }
  if (lane < RW) {
    // select this lane's row without dynamic register indexing
    float t = tot[0], t2 = tot2[0];
#pragma unroll
    for (int r = 1; r < RW; ++r)
      if (lane == r) {
        t = tot[r];
        t2 = tot2[r];
      }
    const int n = row0 + lane;
    if (n < a.N) {
      float out;
      if (DUAL) {
        const float g = round_bf(silu_f(round_bf(t)));  // silu(bf16(fc_1 x)) -> bf16
        out = __fmul_rn(g, round_bf(t2));               // * bf16(fc_2 x)
      } else {
        out = a.bias ? t + bf2f(a.bias[n]) : t;
        if (a.residual) out = round_bf(out) + bf2f(a.residual[n]);
      }
      a.y[n] = f2bf(out);
    }
  }
}

template <int RW, int KS, int FMT, bool DUAL>
static void launch(const GemvArgs& a, hipStream_t stream) {
  constexpr int rows_per_block = (kWaves / KS) * RW;
  const dim3 grid((a.N + rows_per_block - 1) / rows_per_block);
  const size_t lds = (size_t)a.K * 2 + (a.K / 32) * 4 + kWaves * RW * 2 * 4 + 16 * 4 + 4 * 4;
  gemv_q4_kernel<RW, KS, FMT, DUAL><<<grid, kThreads, lds, stream>>>(a);
}

template <int FMT, bool DUAL>
static void dispatch(const GemvArgs& a, int variant, hipStream_t stream) {
  // variant: rows-per-wave x k-split; picked by the host heuristic (or a tuning sweep)
  switch (variant) {
    case 0: launch<1, 1, FMT, DUAL>(a, stream); break;
    case 1: launch<2, 1, FMT, DUAL>(a, stream); break;
    case 2: launch<4, 1, FMT, DUAL>(a, stream); break;
    case 3: launch<2, 2, FMT, DUAL>(a, stream); break;
    case 4: launch<4, 2, FMT, DUAL>(a, stream); break;
    case 5: launch<2, 4, FMT, DUAL>(a, stream); break;
    case 6: launch<4, 4, FMT, DUAL>(a, stream); break;
    default: launch<1, 4, FMT, DUAL>(a, stream); break;
  }
}

static int pick_variant(int N, int K, bool dual) {
  // aim for >= ~1024 workgroups (4 per CU) with >= 4 rows of loads in flight per wave
  const long rows = dual ? 2L * N : N;
  if (rows >= 16384) return 2;         // 4 rows/wave, 16 rows/block
  if (rows >= 8192) return 4;          // 4 rows/wave, k-split 2 -> 8 rows/block
  if (K >= 8192) return 6;             // 4 rows/wave, k-split 4 -> 4 rows/block
  return 4;
}

}  // namespace lga

extern "C" int lga_q4_gemv(const void* x, const uint8_t* qweight, const void* scales, const void* bias,
                           const void* residual, const void* norm_weight, float norm_eps, void* y, int N, int K,
                           int group, int fmt, int variant, hipStream_t stream) {
  LGA_CHECK_ARG(x && qweight && scales && y, "lga_q4_gemv: null pointer");
  LGA_CHECK_ARG(N > 0 && K > 0 && K % 32 == 0, "lga_q4_gemv: K must be a positive multiple of 32");
  LGA_CHECK_ARG(group >= 32 && group % 32 == 0 && K % group == 0, "lga_q4_gemv: group must be a multiple of 32 dividing K");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1, "lga_q4_gemv: fmt must be 0 (int4-g) or 1 (nf4)");
  LGA_CHECK_ARG((size_t)K * 2 + (K / 32) * 4 + 256 <= 160 * 1024, "lga_q4_gemv: K too large for the LDS-staged row");
  lga::GemvArgs a{(const uint16_t*)x, qweight, scales, nullptr, nullptr, (const uint16_t*)bias,
                  (const uint16_t*)residual, (const uint16_t*)norm_weight, (uint16_t*)y, N, K, group, norm_eps};
  if (variant < 0) variant = lga::pick_variant(N, K, false);
  if (fmt == 0) lga::dispatch<0, false>(a, variant, stream);
  else lga::dispatch<1, false>(a, variant, stream);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_q4_gemv_swiglu(const void* x, const uint8_t* qweight1, const void* scales1,
                                  const uint8_t* qweight2, const void* scales2, const void* norm_weight,
                                  float norm_eps, void* y, int N, int K, int group, int fmt, int variant,
                                  hipStream_t stream) {
  LGA_CHECK_ARG(x && qweight1 && scales1 && qweight2 && scales2 && y, "lga_q4_gemv_swiglu: null pointer");
  LGA_CHECK_ARG(N > 0 && K > 0 && K % 32 == 0, "lga_q4_gemv_swiglu: K must be a positive multiple of 32");
  LGA_CHECK_ARG(group >= 32 && group % 32 == 0 && K % group == 0, "lga_q4_gemv_swiglu: bad group");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1, "lga_q4_gemv_swiglu: fmt must be 0 or 1");
  LGA_CHECK_ARG((size_t)K * 2 + (K / 32) * 4 + 256 <= 160 * 1024, "lga_q4_gemv_swiglu: K too large");
  lga::GemvArgs a{(const uint16_t*)x, qweight1, scales1, qweight2, scales2, nullptr, nullptr,
                  (const uint16_t*)norm_weight, (uint16_t*)y, N, K, group, norm_eps};
  if (variant < 0) variant = lga::pick_variant(N, K, true);
  if (fmt == 0) lga::dispatch<0, true>(a, variant, stream);
  else lga::dispatch<1, true>(a, variant, stream);
  LGA_LAUNCH_RETURN();
}
