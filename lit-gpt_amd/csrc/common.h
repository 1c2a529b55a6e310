// Shared device helpers for the lit-gpt MI355X (gfx950) decode path.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lga {

constexpr int kWave = 64;  // CDNA wavefront

// 4-bit codebook formats (kernel template FMT 1, weight = code[nibble] * fp32 block absmax, one fp32 multiply):
//   row 0 — bitsandbytes NF4 (LGA_FMT_NF4 = 1), get_4bit_type('nf4');
//   row 1 — bitsandbytes FP4 (LGA_FMT_FP4 = 3), get_4bit_type('fp4') = {0, .0625, 8, 12, 4, 6, 2, 3, -0, -.0625,
//           -8, -12, -4, -6, -2, -3} / 12: the sign-bit / 2-bit exponent / 1-bit mantissa code whose values
//           dDequantizeFP4Tree returns (bnb 0.41.0 csrc/kernels.cu, upstream; reference generate/base.py:105).
// Kernels take the row as a runtime index (`cb`), so FP4 shares every NF4 instantiation.
constexpr int kFmtFP4 = 3;
__host__ __device__ constexpr int codebook_of(int fmt) { return fmt == kFmtFP4 ? 1 : 0; }
__host__ __device__ constexpr int kernel_fmt(int fmt) { return fmt == kFmtFP4 ? 1 : fmt; }
static __constant__ float kCode4[2][16] = {
    {-1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f, -0.28444138169288635f,
     -0.18477343022823334f, -0.09105003625154495f, 0.0f, 0.07958029955625534f, 0.16093020141124725f,
     0.24611230194568634f, 0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
     0.7229568362236023f, 1.0f},
    {0.0f, 0.005208333333333333f, 0.6666666666666666f, 1.0f, 0.3333333333333333f, 0.5f, 0.16666666666666666f,
     0.25f, -0.0f, -0.005208333333333333f, -0.6666666666666666f, -1.0f, -0.3333333333333333f, -0.5f,
     -0.16666666666666666f, -0.25f}};

// ---- bf16 <-> f32 (bf16 stored as raw uint16_t; RNE on the way down, NaN kept a NaN) ----
__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }
__device__ __forceinline__ float bflo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bfhi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }
// fp32 -> bf16 round-to-nearest-even in hardware (v_cvt_pk_bf16_f32: one instruction per PAIR, NaN stays NaN);
// hipcc has no builtin that emits the packed form for two independent values, hence the asm.
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}
__device__ __forceinline__ uint16_t f2bf(float f) {
  return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f));
}
__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }

// ---- wave-level reductions (64 lanes) ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
// sum over aligned groups of `W` lanes (W power of two <= 64)
template <int W>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// exact-order (no FMA contraction) helpers used where the reference's CPU math does mul then add. HIP's
// __fmul_rn / __fadd_rn are plain `a * b` / `a + b` (clang __clang_hip_math.h) and -ffp-contract may fuse them;
// the pragma drops the `contract` flag from these ops, which survives inlining.
__device__ __forceinline__ float mul_rn(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float add_rn(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }

// The runtime builds a kernel's device-side object at the kernel's first launch (about 0.5 ms each on ROCm 7.2,
// profiles/r03c_cold_prefill.txt); hipFuncGetAttributes builds it ahead of time. Each file lists the kernels of the
// prefill path it owns; lga_preload_kernels (capi.hip) runs them all at model load.
template <class F>
inline int preload(F* f) {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, (const void*)f) == hipSuccess ? 0 : 1;
}
// compute units of the current device (cached; 256 if the query fails)
inline int num_cu() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}
int preload_gemm_q4f();
int preload_attention();
int preload_norm_rope();
int preload_sample();
int preload_gemv();
int preload_moe();

}  // namespace lga

// error plumbing shared by every C entry point
extern "C" void lga_set_error(const char* msg);

#define LGA_CHECK_ARG(cond, msg)    \
  do {                              \
    if (!(cond)) {                  \
      lga_set_error(msg);           \
      return (int)hipErrorInvalidValue; \
    }                               \
  } while (0)

#define LGA_LAUNCH_RETURN()                          \
  do {                                               \
    hipError_t e_ = hipGetLastError();               \
    if (e_ != hipSuccess) {                          \
      lga_set_error(hipGetErrorString(e_));          \
      return (int)e_;                                \
    }                                                \
    return 0;                                        \
  } while (0)
