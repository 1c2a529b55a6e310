// Batch-1 decode GEMV over packed 4-bit weights: y[n] = sum_k x[k] * dequant(W)[n, k]  (+ fused epilogues)
//
// Replaces the bitsandbytes 4-bit GEMV that `Linear4bit.forward` dispatches for one-token inputs
// (bnb `matmul_4bit` -> `gemv_4bit`, reached via BitsandbytesPrecision at reference generate/base.py:128-136)
// for every Linear of the decode step: qkv (lit_gpt/model.py:619), attn proj (:656), LLaMAMLP fc_1/fc_2/proj
// (:712-716) and lm_head (:519).
//
// MI355X design. A batch-1 GEMV is a pure weight stream (~1 flop/byte) whose launches are only 8-66 MB, so the
// launch ramp and load latency dominate unless the whole kernel's weights are in flight at once
// (tools/bw_probe: a bare 16-B/lane read of 8 / 25 / 46 / 66 MB takes 3.0 / 5.5 / 8.6 / 11.7 us).
// Measured cost split for the 25 MB qkv shape (tools/gemv_lab): streaming 5.0 us, + int4 dequant-dot 0.9 us,
// + per-row wave reductions 1.3-2.0 us, + the butterfly below only 0.4 us.
//  * One wave per row slot: a wave owns RPR consecutive rows; lane l owns 32-element chunk columns
//    l, l+64, ... (CPT of them). Every wave issues ALL its 16-B non-temporal weight loads (RPR*CPT per lane)
//    up front, one round per wave; enough waves (~3 workgroups per CU) hide the latency.
//  * The activation row is fetched BEFORE the weights (vmcnt is in order, so the wait for x leaves the weight
//    loads in flight), then staged once per workgroup in LDS as bf16 pairs (x_k, x_k+4) with per-chunk sums;
//    the fused RMSNorm (lit_gpt/rmsnorm.py:19-25: bf16(w * (x * rsqrt(mean(x^2) + eps))), the reference's
//    rounding point) runs during that staging, while the weights stream.
//  * int4-g: one AND-OR turns two nibbles into the bf16 pair (128+q_k, 128+q_k+4) for v_dot2c_f32_bf16, and
//    sum x*(q-8) = dot - 136*sum(x); nf4: codebook in LDS, fp32 FMAs; one scale/absmax FMA per 32 weights.
//  * Reduction: a transposed butterfly sums R = RPR (x2 for the dual GEMV) row partials across the wave with
//    log2(R) halving exchanges + DPP, instead of R separate wave reductions.
//  * Epilogues: +bias, +residual (Block residual add, model.py:591-592), dual-weight SwiGLU
//    (silu(fc_1 x) * fc_2 x, model.py:715) with the reference's bf16 rounding points.
#include "common.h"

namespace lga {

#ifdef LGA_GEMV_TRACE  // lab builds only (tools/gemv_trace.py): per-wave phase timestamps, 100 MHz clock
__device__ unsigned long long g_gemv_trace[65536 * 8];
#define LGA_GTRACE(i)                                                                                        \
  do {                                                                                                     \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                          \
    if ((threadIdx.x & 63) == 0)                                                                         \
      g_gemv_trace[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define LGA_GTRACE_NOWAIT(i)                                                                                 \
  do {                                                                                                     \
    if ((threadIdx.x & 63) == 0)                                                                         \
      g_gemv_trace[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define LGA_GTRACE(i) \
  do {                \
  } while (0)
#define LGA_GTRACE_NOWAIT(i) \
  do {                       \
  } while (0)
#endif


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
      const float send = h ? a[i] : a[i + n], keep = h ? a[i + n] : a[i];
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

__constant__ float kNF4v[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f, -0.28444138169288635f,
    -0.18477343022823334f, -0.09105003625154495f, 0.0f, 0.07958029955625534f, 0.16093020141124725f,
    0.24611230194568634f, 0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
    0.7229568362236023f, 1.0f};

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

// (v & mask) | 0x43004300 in ONE VOP3 op: the compiler only emits the two-op VOP2 and/or pair (gfx9 VOP3 takes
// no literal), which makes the nibble unpack 2 ops per bf16 pair instead of 1 (+1 shift for nibbles 1-3)
__device__ __forceinline__ uint32_t and_or_magic(uint32_t v, uint32_t mask_vgpr) {
  uint32_t r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(v), "v"(mask_vgpr), "s"(0x43004300u));
  return r;
}
__device__ __forceinline__ uint32_t nibble_mask() {  // 0x000F000F in a VGPR, materialised once per kernel
  uint32_t m;
  asm volatile("v_mov_b32 %0, 0x000F000F" : "=v"(m));
  return m;
}

// dot of one 16-byte weight chunk (32 nibbles) with the LDS x chunk (4 uint4 of (x_i, x_i+4) pairs)
template <int FMT>
__device__ __forceinline__ float chunk_dot(const uint4 w, const uint4* xc, float xsum, const float* nf4,
                                           uint32_t mask) {
  const uint32_t wd[4] = {w.x, w.y, w.z, w.w};
  float d = 0.0f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint4 xv = xc[j];
    const uint32_t xp[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (FMT == 0) {
        d = dot2_bf16(xp[s], and_or_magic(s == 0 ? wd[j] : wd[j] >> (4 * s), mask), d);
      } else {
        d = fmaf(nf4[(wd[j] >> (4 * s)) & 0xF], bflo(xp[s]), d);
        d = fmaf(nf4[(wd[j] >> (4 * s + 16)) & 0xF], bfhi(xp[s]), d);
      }
    }
  }
  return FMT == 0 ? d - 136.0f * xsum : d;  // int4: sum x*(128+q) - 136*sum x = sum x*(q-8)
}

// One workgroup = 4 independent waves (row slots); a wave handles RPR consecutive rows.
template <int RPR, int CPT, int FMT, bool DUAL, bool NORM, bool RES>
__global__ void __launch_bounds__(256) gemv_q4_kernel(GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* xl = (uint4*)smem;                        // K/8 uint4 (bf16 pairs)
  float* xsum = (float*)(smem + (size_t)a.K * 2);  // K/32 chunk sums
  float* red = xsum + a.K / 32;                    // 4
  float* nf4 = red + 4;                            // 16
  constexpr int R = DUAL ? 2 * RPR : RPR;          // values per lane entering the butterfly
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int NC = a.K / 32, n8 = a.K / 8, groups = a.K / a.G;
  const int row0 = (blockIdx.x * 4 + wave) * RPR;
  if (FMT == 1 && t < 16) nf4[t] = kNF4v[t];
  LGA_GTRACE_NOWAIT(0);

  // 1. activation (and norm weight) share of this thread: uint4 t, t+256, ... (clamped, branch-free)
  uint4 xr[CPT], nr[CPT];
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int u = min(t + 256 * i, n8 - 1);
    xr[i] = ((const uint4*)a.x)[u];
    if (NORM) nr[i] = ((const uint4*)a.norm_w)[u];
  }
  // 2. every weight / scale / residual load of this wave (rows past N re-read row N-1; never stored)
  uint4 w[RPR][CPT], w2[DUAL ? RPR : 1][DUAL ? CPT : 1];
  uint32_t s[RPR][CPT], s2[DUAL ? RPR : 1][DUAL ? CPT : 1];
  uint32_t res = 0;
#pragma unroll
  for (int i = 0; i < RPR; ++i) {
    const size_t rb = (size_t)min(row0 + i, a.N - 1) * (a.K / 2);
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int c = min(lane + 64 * j, NC - 1);
      w[i][j] = ld_nt16(a.qw + rb + (size_t)c * 16);
      if (DUAL) w2[i][j] = ld_nt16(a.qw2 + rb + (size_t)c * 16);
    }
  }
#pragma unroll
  for (int i = 0; i < RPR; ++i) {
    const size_t n = (size_t)min(row0 + i, a.N - 1);
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int g = (min(lane + 64 * j, NC - 1) * 32) / a.G;
      s[i][j] = load_scale_bits<FMT>(a.sc, n * groups + g);
      if (DUAL) s2[i][j] = load_scale_bits<FMT>(a.sc2, n * groups + g);
    }
  }
  if (RES) res = a.residual[min(row0 + (lane & (RPR - 1)), a.N - 1)];
  __builtin_amdgcn_sched_barrier(0);  // nothing that waits on x may move above the weight loads
  LGA_GTRACE_NOWAIT(1);

  // 3. stage x into LDS (RMS-normalised when NORM) while the weights stream
  float rs = 1.0f;
  if (NORM) {
    float ss = 0.0f;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const bool ok = t + 256 * i < n8;
      const uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float lo = ok ? bflo(d[q]) : 0.0f, hi = ok ? bfhi(d[q]) : 0.0f;
        ss = fmaf(lo, lo, ss);
        ss = fmaf(hi, hi, ss);
      }
    }
    ss = wave_sum_uniform(ss);
    if (lane == 0) red[wave] = ss;
    LGA_GTRACE_NOWAIT(2);
    __syncthreads();
    rs = 1.0f / sqrtf(((red[0] + red[1]) + (red[2] + red[3])) / (float)a.K + a.eps);
  }
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int u = t + 256 * i;
    uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};  // bf16 pairs (x0,x1) (x2,x3) (x4,x5) (x6,x7)
    if (NORM) {  // bf16(w * (x * rs)), rounded in hardware, two elements per instruction
      const uint32_t nw[4] = {nr[i].x, nr[i].y, nr[i].z, nr[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        d[q] = pack2(__fmul_rn(bflo(nw[q]), __fmul_rn(bflo(d[q]), rs)),
                     __fmul_rn(bfhi(nw[q]), __fmul_rn(bfhi(d[q]), rs)));
    }
    float cs = ((bflo(d[0]) + bfhi(d[0])) + (bflo(d[1]) + bfhi(d[1]))) +
               ((bflo(d[2]) + bfhi(d[2])) + (bflo(d[3]) + bfhi(d[3])));
    cs += __shfl_xor(cs, 1);  // 4 consecutive threads hold one 32-element chunk
    cs += __shfl_xor(cs, 2);
    if (u < n8) {
      // (x0,x4) (x1,x5) (x2,x6) (x3,x7): byte permutes of the bf16 pairs
      xl[u] = make_uint4(__builtin_amdgcn_perm(d[2], d[0], 0x05040100u), __builtin_amdgcn_perm(d[2], d[0], 0x07060302u),
                         __builtin_amdgcn_perm(d[3], d[1], 0x05040100u), __builtin_amdgcn_perm(d[3], d[1], 0x07060302u));
      if ((u & 3) == 0) xsum[u >> 2] = cs;
    }
  }
  __syncthreads();
  LGA_GTRACE_NOWAIT(3);
  LGA_GTRACE(4);

  // 4. dequant-dot every row of this wave, then one butterfly for all of them
  const uint32_t nmask = nibble_mask();
  float part[R];
#pragma unroll
  for (int i = 0; i < R; ++i) part[i] = 0.0f;
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = lane + 64 * j;
    const bool ok = c < NC;
    const int cc = min(c, NC - 1);
    const uint4* xc = xl + cc * 4;
    const float xs = xsum[cc];
#pragma unroll
    for (int i = 0; i < RPR; ++i) {
      const float d = chunk_dot<FMT>(w[i][j], xc, xs, nf4, nmask);
      if (DUAL) {  // value index = 2*row + matrix (so the pair of one row lands in lanes l and l^8 / l^16 / l^32)
        part[2 * i] = fmaf(ok ? scale_of<FMT>(s[i][j]) : 0.0f, d, part[2 * i]);
        const float d2 = chunk_dot<FMT>(w2[i][j], xc, xs, nf4, nmask);
        part[2 * i + 1] = fmaf(ok ? scale_of<FMT>(s2[i][j]) : 0.0f, d2, part[2 * i + 1]);
      } else {
        part[i] = fmaf(ok ? scale_of<FMT>(s[i][j]) : 0.0f, d, part[i]);
      }
    }
  }
  const float tot = butterfly<R>(part, lane);
  const int vi = bfly_index<R>(lane);  // value index held by this lane
  constexpr int GROUP = 64 / R;        // lanes per value after the butterfly
  if (DUAL) {
    // partner value (other matrix, same row) sits in the lane whose value index differs in bit 0
    constexpr int PD = R == 8 ? 8 : (R == 4 ? 16 : 32);
    const float other = PD == 8 ? LGA_DPP(tot, 0x128) : __shfl_xor(tot, PD);
    const int row = row0 + (vi >> 1);
    if ((lane & (GROUP - 1)) == 0 && (vi & 1) == 0 && row < a.N) {
      const float g = round_bf(silu_f(round_bf(tot)));  // silu(bf16(fc_1 x)) -> bf16
      a.y[row] = f2bf(__fmul_rn(g, round_bf(other)));   // * bf16(fc_2 x)
    }
    LGA_GTRACE(5);
  } else {
    const int row = row0 + vi;
    float o = tot;
    if (RES) {
      // residual of row vi sits in lane vi (loaded up front); fetch it into this lane
      o = round_bf(a.bias ? o + bf2f(a.bias[min(row, a.N - 1)]) : o) +
          __uint_as_float(((uint32_t)__shfl(res, vi)) << 16);
    } else if (a.bias) {
      o += bf2f(a.bias[min(row, a.N - 1)]);
    }
    if ((lane & (GROUP - 1)) == 0 && row < a.N) a.y[row] = f2bf(o);
    LGA_GTRACE(5);
  }
}

template <int RPR, int CPT, int FMT, bool DUAL>
static void launch(const GemvArgs& a, hipStream_t stream) {
  const int waves = (a.N + RPR - 1) / RPR;
  const int blocks = (waves + 3) / 4;
  const size_t lds = (size_t)a.K * 2 + (a.K / 32) * 4 + 4 * 4 + 16 * 4;
  const bool norm = a.norm_w != nullptr, res = a.residual != nullptr;
  if (DUAL) {
    if (norm) gemv_q4_kernel<RPR, CPT, FMT, DUAL, true, false><<<blocks, 256, lds, stream>>>(a);
    else gemv_q4_kernel<RPR, CPT, FMT, DUAL, false, false><<<blocks, 256, lds, stream>>>(a);
  } else if (norm) {
    if (res) gemv_q4_kernel<RPR, CPT, FMT, DUAL, true, true><<<blocks, 256, lds, stream>>>(a);
    else gemv_q4_kernel<RPR, CPT, FMT, DUAL, true, false><<<blocks, 256, lds, stream>>>(a);
  } else {
    if (res) gemv_q4_kernel<RPR, CPT, FMT, DUAL, false, true><<<blocks, 256, lds, stream>>>(a);
    else gemv_q4_kernel<RPR, CPT, FMT, DUAL, false, false><<<blocks, 256, lds, stream>>>(a);
  }
}

// variant: 0 = fewer rows per wave (more waves), 1 = more rows per wave; < 0 = heuristic
template <int FMT, bool DUAL>
static int dispatch(const GemvArgs& a, int variant, hipStream_t stream) {
  const int cpt = (a.K / 32 + 63) / 64;  // chunks per lane (== uint4 of x per thread)
  if (variant < 0) {
    const long rows = DUAL ? 2L * a.N : a.N;
    variant = rows >= 24000 ? 1 : 0;  // tall matrices: more rows per wave keep the grid ~3-4 workgroups per CU
  }
  // A persistent, double-buffered streaming form of this kernel (few workgroups per CU walking row tiles) measured
  // 10-70 % slower on every decode shape (tools/gemv_sweep.py, round 1) and was dropped.
  const bool big = (variant & 1) != 0;
#define LGA_L(RS, RB, CPT)                                                         \
  do {                                                                             \
    if (big) launch<(DUAL ? (RB) / 2 : (RB)), CPT, FMT, DUAL>(a, stream);          \
    else launch<(DUAL ? (RS) / 2 : (RS)), CPT, FMT, DUAL>(a, stream);              \
  } while (0)
  switch (cpt) {
    case 1: LGA_L(4, 8, 1); break;
    case 2: LGA_L(4, 8, 2); break;
    case 3: LGA_L(4, 8, 3); break;
    case 4: LGA_L(2, 4, 4); break;
    case 5:
    case 6: LGA_L(2, 4, 6); break;
    case 7:
    case 8: LGA_L(2, 4, 8); break;
    default:
      if (cpt <= 16) {
        LGA_L(2, 2, 16);
        break;
      }
      lga_set_error("lga_q4_gemv: K > 32768 is not supported");
      return (int)hipErrorInvalidValue;
  }
#undef LGA_L
  return 0;
}

}  // namespace lga

extern "C" int lga_q4_gemv(const void* x, const uint8_t* qweight, const void* scales, const void* bias,
                           const void* residual, const void* norm_weight, float norm_eps, void* y, int N, int K,
                           int group, int fmt, int variant, hipStream_t stream) {
  LGA_CHECK_ARG(x && qweight && scales && y, "lga_q4_gemv: null pointer");
  LGA_CHECK_ARG(N > 0 && K > 0 && K % 32 == 0, "lga_q4_gemv: K must be a positive multiple of 32");
  LGA_CHECK_ARG(group >= 32 && group % 32 == 0 && K % group == 0, "lga_q4_gemv: group must be a multiple of 32 dividing K");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1, "lga_q4_gemv: fmt must be 0 (int4-g) or 1 (nf4)");
  lga::GemvArgs a{(const uint16_t*)x, qweight, scales, nullptr, nullptr, (const uint16_t*)bias,
                  (const uint16_t*)residual, (const uint16_t*)norm_weight, (uint16_t*)y, N, K, group, norm_eps};
  const int rc = fmt == 0 ? lga::dispatch<0, false>(a, variant, stream) : lga::dispatch<1, false>(a, variant, stream);
  if (rc) return rc;
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
  lga::GemvArgs a{(const uint16_t*)x, qweight1, scales1, qweight2, scales2, nullptr, nullptr,
                  (const uint16_t*)norm_weight, (uint16_t*)y, N, K, group, norm_eps};
  const int rc = fmt == 0 ? lga::dispatch<0, true>(a, variant, stream) : lga::dispatch<1, true>(a, variant, stream);
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}

#ifdef LGA_GEMV_TRACE
extern "C" int lga_gemv_trace_read(unsigned long long* host, int n) {
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(lga::g_gemv_trace), (size_t)n * sizeof(unsigned long long));
  void* dptr = nullptr;
  if (e == hipSuccess) e = hipGetSymbolAddress(&dptr, HIP_SYMBOL(lga::g_gemv_trace));
  if (e == hipSuccess) e = hipMemset(dptr, 0, sizeof(lga::g_gemv_trace));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}
#endif
