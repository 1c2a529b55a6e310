// GEMV ablation lab (not product code): QKV-shaped int4 GEMV (N=12288, K=4096, 25 MB) with switches, to split
// the kernel time into streaming / dequant-math / reduction / prologue. Back-to-back launches over rotating
// weight copies (> 1 GiB) timed with HIP events from C++ (no Python submission overhead).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/gemv_lab tools/gemv_lab.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float dot2(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), c, false);
}
__device__ __forceinline__ float wsum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
  const int i = __float_as_int(v);
  return (__int_as_float(__builtin_amdgcn_readlane(i, 0)) + __int_as_float(__builtin_amdgcn_readlane(i, 16))) +
         (__int_as_float(__builtin_amdgcn_readlane(i, 32)) + __int_as_float(__builtin_amdgcn_readlane(i, 48)));
}

// transposed butterfly: 8 per-lane row partials -> lane l holds the full wave sum of row
// 4*bit5(l) + 2*bit4(l) + bit3(l); 7 exchanges + 3 DPP instead of 8 separate wave reductions
__device__ __forceinline__ float tr8(const float* a, int lane) {
  const bool h1 = lane & 32, h2 = lane & 16, h3 = lane & 8;
  float b[4], c[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float send = h1 ? a[i] : a[i + 4], keep = h1 ? a[i + 4] : a[i];
    b[i] = keep + __shfl_xor(send, 32);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float send = h2 ? b[i] : b[i + 2], keep = h2 ? b[i + 2] : b[i];
    c[i] = keep + __shfl_xor(send, 16);
  }
  const float send = h3 ? c[0] : c[1], keep = h3 ? c[1] : c[0];
  float d = keep + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(send), 0x128, 0xF, 0xF, false));
  d += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0xB1, 0xF, 0xF, false));
  d += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0x4E, 0xF, 0xF, false));
  d += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d), 0x141, 0xF, 0xF, false));
  return d;
}

// MODE 0: loads + xor (probe-like) ; 1: + int4 dequant dot (no reduction) ; 2: + per-row wave reduction + store
// MODE 3: + transposed 8-row butterfly reduction + store
// Each thread: chunk c = t % 128 of rows slot + 2*i (RPR rows per round), rounds over the block's rows.
template <int MODE, int RPR>
__global__ void __launch_bounds__(256) lab(const uint8_t* __restrict__ w, const uint32_t* __restrict__ x,
                                          float* __restrict__ y, int N, int R) {
  const int t = threadIdx.x, c = t & 127, slot = t >> 7, lane = t & 63;
  const int row_beg = blockIdx.x * R, row_end = min(row_beg + R, N);
  uint32_t xp[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) xp[i] = x[c * 16 + i];
  float xs = 0.f;
  unsigned acc_x = 0;
  float acc_f = 0.f;
  for (int r0 = row_beg + slot * RPR; r0 < row_end; r0 += 2 * RPR) {
    u32x4 v[RPR];
#pragma unroll
    for (int i = 0; i < RPR; ++i)
      v[i] = __builtin_nontemporal_load((const u32x4*)(w + (size_t)min(r0 + i, N - 1) * 2048 + c * 16));
    if (MODE == 3) {
      float part[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const u32x4 vi = v[i % RPR];
        const uint32_t wd[4] = {vi.x, vi.y, vi.z, vi.w};
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s) d = dot2(xp[j * 4 + s], ((wd[j] >> (4 * s)) & 0x000F000Fu) | 0x43004300u, d);
        part[i] = d - 136.f * xs;
      }
      const float tot = tr8(part, lane);
      const int row = r0 + ((lane >> 5) & 1) * 4 + ((lane >> 4) & 1) * 2 + ((lane >> 3) & 1);
      if ((lane & 7) == 0 && row < row_end) y[row] = tot;
      continue;
    }
#pragma unroll
    for (int i = 0; i < RPR; ++i) {
      if (MODE == 0) {
        acc_x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
      } else {
        const uint32_t wd[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s) d = dot2(xp[j * 4 + s], ((wd[j] >> (4 * s)) & 0x000F000Fu) | 0x43004300u, d);
        d -= 136.f * xs;
        if (MODE == 1) {
          acc_f += d;
        } else {
          const float tot = wsum(d);
          if (lane == 0 && r0 + i < row_end) y[r0 + i] = tot;  // (partial of one wave: lab only)
        }
      }
    }
  }
  if (MODE == 0 && acc_x == 0x1234567u) y[0] = 1.f;
  if (MODE == 1 && acc_f == 1234.5f) y[0] = acc_f;
}

// MODE 4: butterfly kernel + per-(row, chunk) bf16 scale loads (raw bits, converted at use)
// MODE 5: MODE 4 + x staged through LDS as the product does (x loads first, RMSNorm sum, 2 barriers)
template <int MODE>
__global__ void __launch_bounds__(256) lab2(const uint8_t* __restrict__ w, const uint16_t* __restrict__ sc,
                                           const uint32_t* __restrict__ x, float* __restrict__ y, int N, int R) {
  __shared__ uint32_t xl[2048];
  __shared__ float red[4];
  const int t = threadIdx.x, c = t & 127, slot = t >> 7, lane = t & 63, wave = t >> 6;
  const int row_beg = blockIdx.x * R, row_end = min(row_beg + R, N);
  uint32_t xp[16];
  uint4 xr[2];
  if (MODE == 4) {
#pragma unroll
    for (int i = 0; i < 16; ++i) xp[i] = x[c * 16 + i];
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i) xr[i] = ((const uint4*)x)[t + 256 * i];
  }
  const int r0 = row_beg + slot * 8;
  u32x4 v[8];
  uint32_t s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    v[i] = __builtin_nontemporal_load((const u32x4*)(w + (size_t)min(r0 + i, N - 1) * 2048 + c * 16));
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = sc[(size_t)min(r0 + i, N - 1) * 32 + c / 4];
  __builtin_amdgcn_sched_barrier(0);
  if (MODE == 5) {
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) ss += __uint_as_float(d[q] << 16) * __uint_as_float(d[q] << 16);
    }
    ss = wsum(ss);
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    const float rs = 1.f / sqrtf(red[0] + red[1] + red[2] + red[3] + 1e-5f);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      uint4 o = xr[i];
      o.x = __float_as_uint(__uint_as_float(o.x) * rs);
      ((uint4*)xl)[t + 256 * i] = o;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) xp[i] = xl[c * 16 + i];
  }
  float part[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t wd[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
    float d = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) d = dot2(xp[j * 4 + q], ((wd[j] >> (4 * q)) & 0x000F000Fu) | 0x43004300u, d);
    part[i] = __uint_as_float(s[i] << 16) * d;
  }
  const float tot = tr8(part, lane);
  const int row = r0 + ((lane >> 5) & 1) * 4 + ((lane >> 4) & 1) * 2 + ((lane >> 3) & 1);
  if ((lane & 7) == 0 && row < row_end) y[row] = tot;
}

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t err_ = (x);                                             \
    if (err_ != hipSuccess) {                                          \
      printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

template <int MODE, int RPR>
void run(const char* name, uint8_t* base, size_t bytes, int copies, uint32_t* x, float* y, int N, int blocks) {
  const int R = (N + blocks - 1) / blocks;
  for (int c = 0; c < copies; ++c) lab<MODE, RPR><<<blocks, 256>>>(base + (size_t)c * bytes, x, y, N, R);
  CK(hipDeviceSynchronize());
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  const int reps = 4 * copies;
  CK(hipEventRecord(s));
  for (int r = 0; r < reps; ++r) lab<MODE, RPR><<<blocks, 256>>>(base + (size_t)(r % copies) * bytes, x, y, N, R);
  CK(hipEventRecord(e));
  CK(hipEventSynchronize(e));
  float ms;
  CK(hipEventElapsedTime(&ms, s, e));
  const float us = ms * 1e3f / reps;
  printf("%-28s RPR %d blocks %4d: %7.2f us  %6.0f GB/s\n", name, RPR, blocks, us, bytes / us / 1e3);
}

template <int MODE>
void run2(const char* name, uint8_t* base, size_t bytes, int copies, uint16_t* sc, uint32_t* x, float* y, int N) {
  const int blocks = N / 16, R = 16;
  for (int c = 0; c < copies; ++c) lab2<MODE><<<blocks, 256>>>(base + (size_t)c * bytes, sc, x, y, N, R);
  CK(hipDeviceSynchronize());
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  const int reps = 4 * copies;
  CK(hipEventRecord(s));
  for (int r = 0; r < reps; ++r) lab2<MODE><<<blocks, 256>>>(base + (size_t)(r % copies) * bytes, sc, x, y, N, R);
  CK(hipEventRecord(e));
  CK(hipEventSynchronize(e));
  float ms;
  CK(hipEventElapsedTime(&ms, s, e));
  const float us = ms * 1e3f / reps;
  printf("%-28s blocks %4d: %7.2f us  %6.0f GB/s\n", name, blocks, us, bytes / us / 1e3);
}

extern "C" int lga_q4_gemv(const void* x, const uint8_t* qweight, const void* scales, const void* bias,
                           const void* residual, const void* norm_weight, float norm_eps, void* y, int N, int K,
                           int group, int fmt, int variant, hipStream_t stream);

void run_product(const char* name, uint8_t* base, size_t bytes, int copies, uint16_t* sc, uint16_t* x, uint16_t* nw,
                 uint16_t* y, int N, int K, int variant) {
  for (int c = 0; c < copies; ++c)
    lga_q4_gemv(x, base + (size_t)c * bytes, sc, nullptr, nullptr, nw, 1e-5f, y, N, K, 128, 0, variant, 0);
  CK(hipDeviceSynchronize());
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  const int reps = 4 * copies;
  CK(hipEventRecord(s));
  for (int r = 0; r < reps; ++r)
    lga_q4_gemv(x, base + (size_t)(r % copies) * bytes, sc, nullptr, nullptr, nw, 1e-5f, y, N, K, 128, 0, variant, 0);
  CK(hipEventRecord(e));
  CK(hipEventSynchronize(e));
  float ms;
  CK(hipEventElapsedTime(&ms, s, e));
  const float us = ms * 1e3f / reps;
  printf("%-28s variant %d: %7.2f us  %6.0f GB/s\n", name, variant, us, bytes / us / 1e3);
}

int main() {
  const int N = 12288, K = 4096;
  const size_t bytes = (size_t)N * K / 2;
  const int copies = 48;
  uint8_t* base;
  uint32_t* x;
  float* y;
  CK(hipMalloc(&base, bytes * copies));
  CK(hipMalloc(&x, K * 2));
  CK(hipMalloc(&y, N * 4));
  CK(hipMemset(base, 0x37, bytes * copies));
  CK(hipMemset(x, 0x3f, K * 2));
  uint16_t* sc;
  CK(hipMalloc(&sc, (size_t)N * 32 * 2));
  CK(hipMemset(sc, 0x3c, (size_t)N * 32 * 2));
  for (int rep = 0; rep < 2; ++rep) {
    run<3, 8>("butterfly8 (lab)", base, bytes, copies, x, y, N, 768);
    run2<4>("+scales", base, bytes, copies, sc, x, y, N);
    run2<5>("+scales+LDS x staging/norm", base, bytes, copies, sc, x, y, N);
    run_product("product lga_q4_gemv norm", base, bytes, copies, sc, (uint16_t*)x, (uint16_t*)x, (uint16_t*)y, N, K, 0);
    run_product("product lga_q4_gemv norm", base, bytes, copies, sc, (uint16_t*)x, (uint16_t*)x, (uint16_t*)y, N, K, 1);
    run_product("product no-norm", base, bytes, copies, sc, (uint16_t*)x, nullptr, (uint16_t*)y, N, K, 0);
  }
  for (int blocks : {768}) {
    run<0, 4>("loads+xor", base, bytes, copies, x, y, N, blocks);
    run<0, 8>("loads+xor", base, bytes, copies, x, y, N, blocks);
    run<1, 4>("loads+dequant-dot", base, bytes, copies, x, y, N, blocks);
    run<1, 8>("loads+dequant-dot", base, bytes, copies, x, y, N, blocks);
    run<2, 4>("loads+dot+wave-reduce+store", base, bytes, copies, x, y, N, blocks);
    run<2, 8>("loads+dot+wave-reduce+store", base, bytes, copies, x, y, N, blocks);
    run<3, 8>("loads+dot+butterfly8+store", base, bytes, copies, x, y, N, blocks);
  }
  return 0;
}
