// GEMV ablation (lab, not product): where do the ~5 us between lga_q4_gemv and a bare one-shot read of the same
// bytes go? One-shot int4-g128 GEMV (same load order as csrc/gemv.hip) with switches:
//   XM 0: x + norm weight from global, RMSNorm, 2 barriers (product)   1: x from global, no norm, 1 barrier
//      2: no global x (LDS filled with a constant), 1 barrier          3: no LDS / barrier (x constant in regs)
//   CM 1: dequant-dot + butterfly + store    0: xor of the loaded words + store
// build: hipcc --offload-arch=gfx950 -O3 -o tools/gemv_ab tools/gemv_ab.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t err_ = (x);                                               \
    if (err_ != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); \
      exit(1);                                                           \
    }                                                                    \
  } while (0)

__device__ __forceinline__ float dot2(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), c, false);
}
__device__ __forceinline__ uint4 ldnt(const void* p) {
  const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float bflo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bfhi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }
#define DPP(v, c) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), c, 0xF, 0xF, false))

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
      a[i] = keep + (D == 8 ? DPP(send, 0x128) : __shfl_xor(send, D));
    }
  }
  float d = a[0];
  d += DPP(d, 0xB1);
  d += DPP(d, 0x4E);
  d += DPP(d, 0x141);
  if (R <= 4) d += DPP(d, 0x140);
  if (R <= 2) d += __shfl_xor(d, 16);
  return d;
}

__device__ __forceinline__ uint32_t and_or_magic(uint32_t v, uint32_t m) {
  uint32_t r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(v), "v"(m), "s"(0x43004300u));
  return r;
}

template <int RPR, int CPT, bool DUAL, int XM, int CM, int NW = 4, int PRIO = 0, int ORD = 0>
__global__ void __launch_bounds__(NW * 64) gemv(const uint16_t* __restrict__ x, const uint16_t* __restrict__ nw,
                                            const uint8_t* __restrict__ qw, const uint16_t* __restrict__ sc,
                                            const uint8_t* __restrict__ qw2, const uint16_t* __restrict__ sc2,
                                            uint16_t* __restrict__ y, int N, int K, int rpb) {
  __shared__ uint4 xl[1024];
  __shared__ float xsum[256], red[16];
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int NC = K / 32, n8 = K / 8, groups = K / 128;
  const int row0 = rpb ? blockIdx.x * rpb + wave * RPR : (blockIdx.x * NW + wave) * RPR;
  const int row_end = rpb ? min(blockIdx.x * rpb + rpb, N) : N;
  constexpr int NT = NW * 64;
  if (PRIO == 1) __builtin_amdgcn_s_setprio(3);
  uint4 xr[CPT], nr[CPT];
  if (XM <= 1) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int u = min(t + NT * i, n8 - 1);
      xr[i] = ((const uint4*)x)[u];
      if (XM == 0) nr[i] = ((const uint4*)nw)[u];
    }
  }
  uint4 w[RPR][CPT], w2[DUAL ? RPR : 1][DUAL ? CPT : 1];
  uint32_t s[RPR][CPT], s2[DUAL ? RPR : 1][DUAL ? CPT : 1];
  if (ORD == 0) {
#pragma unroll
  for (int i = 0; i < RPR; ++i) {
    const size_t rb = (size_t)min(row0 + i, row_end - 1) * (K / 2);
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int c = min(lane + 64 * j, NC - 1);
      w[i][j] = ldnt(qw + rb + (size_t)c * 16);
      if (DUAL) w2[i][j] = ldnt(qw2 + rb + (size_t)c * 16);
    }
  }
#pragma unroll
  for (int i = 0; i < RPR; ++i) {
    const size_t n = (size_t)min(row0 + i, row_end - 1);
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int g = (min(lane + 64 * j, NC - 1) * 32) / 128;
      s[i][j] = sc[n * groups + g];
      if (DUAL) s2[i][j] = sc2[n * groups + g];
    }
  }
  } else {  // ORD 1: consumption order (j outer, i inner), each scale right after its weights
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = min(lane + 64 * j, NC - 1);
#pragma unroll
    for (int i = 0; i < RPR; ++i) {
      const size_t n = (size_t)min(row0 + i, row_end - 1);
      w[i][j] = ldnt(qw + n * (K / 2) + (size_t)c * 16);
      s[i][j] = sc[n * groups + (c * 32) / 128];
      if (DUAL) {
        w2[i][j] = ldnt(qw2 + n * (K / 2) + (size_t)c * 16);
        s2[i][j] = sc2[n * groups + (c * 32) / 128];
      }
    }
  }
  }
  __builtin_amdgcn_sched_barrier(0);
  if (PRIO == 1) __builtin_amdgcn_s_setprio(0);
  if (XM <= 2) {
    float rs = 1.0f;
    if (XM == 0) {
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) ss = fmaf(bflo(d[q]), bflo(d[q]), fmaf(bfhi(d[q]), bfhi(d[q]), ss));
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
      if (lane == 0) red[wave] = ss;
      __syncthreads();
      float tot = 0.f;
      for (int i = 0; i < NW; ++i) tot += red[i];
      rs = 1.0f / sqrtf(tot / K + 1e-5f);
    }
#pragma unroll
    for (int i = 0; i < (CPT * 256 + NT - 1) / NT; ++i) {
      const int u = t + NT * i;
      uint4 v = XM == 2 ? make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u) : xr[i];
      if (XM == 0) {
        v.x = __builtin_bit_cast(uint32_t, (bf16x2_t){(__bf16)(bflo(nr[i].x) * bflo(v.x) * rs), (__bf16)(bfhi(nr[i].x) * bfhi(v.x) * rs)});
      }
      if (u < n8) {
        xl[u] = v;
        if ((u & 3) == 0) xsum[u >> 2] = 1.0f;
      }
    }
    __syncthreads();
  }
  float part[DUAL ? 2 * RPR : RPR];
  constexpr int R = DUAL ? 2 * RPR : RPR;
#pragma unroll
  for (int i = 0; i < R; ++i) part[i] = 0.f;
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = min(lane + 64 * j, NC - 1);
    uint4 xc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) xc[q] = XM <= 2 ? xl[c * 4 + q] : make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);
    const float xs = XM <= 2 ? xsum[c] : 1.0f;
#pragma unroll
    for (int i = 0; i < RPR; ++i) {
#pragma unroll
      for (int m = 0; m < (DUAL ? 2 : 1); ++m) {
        const uint4 ww = m ? w2[DUAL ? i : 0][DUAL ? j : 0] : w[i][j];
        const uint32_t sb = m ? s2[DUAL ? i : 0][DUAL ? j : 0] : s[i][j];
        float d = 0.f;
        if (CM == 1) {
          const uint32_t wd[4] = {ww.x, ww.y, ww.z, ww.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t xp[4] = {xc[q].x, xc[q].y, xc[q].z, xc[q].w};
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) d = dot2(xp[s4], ((wd[q] >> (4 * s4)) & 0x000F000Fu) | 0x43004300u, d);
          }
          d -= 136.f * xs;
        } else if (CM >= 2) {
          uint32_t mk;
          asm volatile("v_mov_b32 %0, 0x000F000F" : "=v"(mk));
          const uint32_t wd[4] = {ww.x, ww.y, ww.z, ww.w};
          float dd[2] = {0.f, 0.f};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t xp[4] = {xc[q].x, xc[q].y, xc[q].z, xc[q].w};
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
              const uint32_t b = and_or_magic(s4 ? wd[q] >> (4 * s4) : wd[q], mk);
              if (CM == 3) dd[s4 & 1] = dot2(xp[s4], b, dd[s4 & 1]);
              else d = dot2(xp[s4], b, d);
            }
          }
          d = (CM == 3 ? dd[0] + dd[1] : d) - 136.f * xs;
        } else {
          d = __uint_as_float((ww.x ^ ww.y ^ ww.z ^ ww.w) & 0x3FFFFFFFu);
        }
        part[DUAL ? 2 * i + m : i] = fmaf(__uint_as_float(sb << 16), d, part[DUAL ? 2 * i + m : i]);
      }
    }
  }
  const float tot = butterfly<R>(part, lane);
  if ((lane & (64 / R - 1)) == 0 && row0 < row_end) y[min(row0 + (lane >> 3) % RPR, N - 1)] = (uint16_t)(__float_as_uint(tot) >> 16);
}

template <int RPR, int CPT, bool DUAL, int XM, int CM, int NW = 4, int PRIO = 0, int ORD = 0>
float run(uint8_t* base, size_t wbytes, int copies, uint16_t* scb, size_t sbytes, uint16_t* x, uint16_t* y, int N, int K,
          int cu_blocks = 0, int pad_lds = 0) {
  const int rpb = cu_blocks ? (N + cu_blocks - 1) / cu_blocks : 0;
  if (rpb && (rpb + RPR - 1) / RPR > NW) return -1.0f;  // config cannot cover its rows
  const int blocks = cu_blocks ? cu_blocks : ((N + RPR - 1) / RPR + NW - 1) / NW;
  auto launch = [&](int c) {
    uint8_t* q = base + (size_t)c * wbytes;
    uint16_t* s = (uint16_t*)((char*)scb + (size_t)c * sbytes);
    gemv<RPR, CPT, DUAL, XM, CM, NW, PRIO, ORD><<<blocks, NW * 64, pad_lds>>>(x, x, q, s, q + wbytes / 2, s + sbytes / 4, y, N, K, rpb);
  };
  for (int c = 0; c < copies; ++c) launch(c);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 4 * copies;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch(r % copies);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

int main(int argc, char** argv) {
  const bool one = argc > 1;
  const bool warm = argc > 2;  // same weights every launch: MALL-resident (< 256 MiB)
  const size_t total = 2ull << 30;
  uint8_t* base;
  uint16_t *scb, *x, *y;
  CK(hipMalloc(&base, total));
  CK(hipMalloc(&scb, 128u << 20));
  CK(hipMalloc(&x, 1 << 20));
  CK(hipMalloc(&y, 1 << 20));
  CK(hipMemset(base, 0x37, total));
  CK(hipMemset(scb, 0x3C, 128u << 20));
  CK(hipMemset(x, 0x3F, 1 << 20));
  struct Shape { const char* name; int N, K; bool dual; };
  const Shape shapes[] = {{"gate_up dual", 11008, 4096, true}, {"qkv", 12288, 4096, false}, {"o_proj", 4096, 4096, false},
                          {"down", 4096, 11008, false}, {"lm_head", 32000, 4096, false}};
  for (const Shape& sh : shapes) {
    const int N = sh.N, K = sh.K;
    const size_t wb = (sh.dual ? 2ull : 1ull) * N * K / 2, sb = (sh.dual ? 2ull : 1ull) * N * (K / 128) * 2;
    const int copies = warm ? 1 : ((int)(total / wb) > 64 ? 64 : (int)(total / wb));
    printf("%s (%.1f MB)\n", sh.name, (wb + sb) / 1e6);
#define R(RPR, CPT, NW, CUB, PAD) \
  (sh.dual ? run<RPR, CPT, true, 0, 2, NW>(base, wb, copies, scb, sb, x, y, N, K, CUB, PAD) \
           : run<RPR, CPT, false, 0, 2, NW>(base, wb, copies, scb, sb, x, y, N, K, CUB, PAD))
    if (one) {
#define RO(RPR, CPT, XM, CM, ORD) \
  (sh.dual ? run<RPR, CPT, true, XM, CM, 4, 0, ORD>(base, wb, copies, scb, sb, x, y, N, K) \
           : run<RPR, CPT, false, XM, CM, 4, 0, ORD>(base, wb, copies, scb, sb, x, y, N, K))
      if (K == 4096) {
        printf("  RPR2: ord0 %7.2f ord1 %7.2f bare %7.2f | RPR4: ord0 %7.2f ord1 %7.2f bare %7.2f\n", RO(2, 2, 0, 2, 0),
               RO(2, 2, 0, 2, 1), RO(2, 2, 3, 0, 0), RO(4, 2, 0, 2, 0), RO(4, 2, 0, 2, 1), RO(4, 2, 3, 0, 0));
      } else {
        printf("  RPR2: ord0 %7.2f ord1 %7.2f bare %7.2f\n", RO(2, 6, 0, 2, 0), RO(2, 6, 0, 2, 1), RO(2, 6, 3, 0, 0));
      }
      continue;
    }
    if (K == 4096) {
      printf("  grid-by-rows RPR2 NW4       %7.2f\n", R(2, 2, 4, 0, 0));
      printf("  grid-by-rows RPR4 NW4       %7.2f\n", R(4, 2, 4, 0, 0));
      printf("  256 blocks NW16 RPR1/2/3/4/8 %7.2f %7.2f %7.2f %7.2f %7.2f\n", R(1, 2, 16, 256, 0), R(2, 2, 16, 256, 0),
             R(3, 2, 16, 256, 0), R(4, 2, 16, 256, 0), R(8, 2, 16, 256, 0));
      printf("  256 blocks NW16 pad96K RPR1/2/3/4/8 %7.2f %7.2f %7.2f %7.2f %7.2f\n", R(1, 2, 16, 256, 98304),
             R(2, 2, 16, 256, 98304), R(3, 2, 16, 256, 98304), R(4, 2, 16, 256, 98304), R(8, 2, 16, 256, 98304));
      printf("  256 blocks NW8 RPR1/2/4/8   %7.2f %7.2f %7.2f %7.2f\n", R(1, 2, 8, 256, 0), R(2, 2, 8, 256, 0),
             R(4, 2, 8, 256, 0), R(8, 2, 8, 256, 0));
      printf("  512 blocks NW8 RPR1/2/3/4/8 %7.2f %7.2f %7.2f %7.2f %7.2f\n", R(1, 2, 8, 512, 0), R(2, 2, 8, 512, 0),
             R(3, 2, 8, 512, 0), R(4, 2, 8, 512, 0), R(8, 2, 8, 512, 0));
    } else {
      printf("  grid-by-rows RPR2 NW4       %7.2f\n", R(2, 6, 4, 0, 0));
      printf("  256 blocks NW16 RPR1/2      %7.2f %7.2f\n", R(1, 6, 16, 256, 0), R(2, 6, 16, 256, 0));
      printf("  256 blocks NW16 pad RPR1/2  %7.2f %7.2f\n", R(1, 6, 16, 256, 98304), R(2, 6, 16, 256, 98304));
      printf("  512 blocks NW8 RPR1/2       %7.2f %7.2f\n", R(1, 6, 8, 512, 0), R(2, 6, 8, 512, 0));
    }
#undef R
  }
  return 0;
}
