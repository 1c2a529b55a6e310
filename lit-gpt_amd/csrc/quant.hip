// Load-time weight quantizer: (N, K) fp32/bf16 Linear weight -> packed int4 + per-group scale.
//
// Replaces the bitsandbytes quantize-on-device step that Lightning's BitsandbytesPrecision triggers on
// `fabric.setup_module` / `fabric.to_device` (reference generate/base.py:168, generate/tp.py:190; bnb
// `cquantize_blockwise_*_nf4`, upstream). Formats are specified byte-for-byte in oracle/quant.py:
//   LGA_FMT_Q4G (0): symmetric int4, group G along K, scale = bf16(absmax / 7), nibble = q + 8
//   LGA_FMT_NF4 (1): bnb NF4 codebook, block G along K, fp32 absmax
//   LGA_FMT_FP4 (3): bnb FP4 codebook (common.h kCode4[1]), block G along K, fp32 absmax; the code of w / absmax
//                    is bnb's dQuantizeFP4 (csrc/kernels.cu, upstream): sign bit for x < 0, then the magnitude
//                    against the seven literal pivots below (strict >, so a tie takes the smaller magnitude)
// Packed byte j of a row holds k = 2j (low nibble) and k = 2j + 1 (high nibble).
//
// lga_nf4_double_quant: bitsandbytes' double quantization of the nf4 statistics ("bnb.nf4-dq",
// quantize_4bit(compress_statistics=True), generate/base.py:105): offset = mean(absmax), the centred absmax
// quantized in blocks of 256 to the signed 8-bit dynamic map (kQuantizeBlockwise + dQuantize<0>), and the
// statistic the kernels scale by replaced IN PLACE by its dequantized value code[q] * absmax2 + offset (fp32
// multiply, fp32 add — dequantize_4bit's order). Restated and tested against oracle/quant.py double_quant_absmax.
#include "common.h"

namespace lga {


// dQuantizeFP4: pivots between the sorted magnitudes {0, 1/192, 1/6, 1/4, 1/3, 1/2, 2/3, 1} (codes 0, 1, 6, 7, 4,
// 5, 2, 3), the float literals bitsandbytes compares against
__device__ __forceinline__ unsigned fp4_code(float x) {
  const unsigned sign = x < 0.0f ? 8u : 0u;
  const float a = fabsf(x);
  const float piv[7] = {0.00260417f, 0.0859375f, 0.20833333f, 0.29166667f, 0.4166667f, 0.583333f, 0.8333333f};
  unsigned r = 0;
#pragma unroll
  for (int j = 0; j < 7; ++j) r += a > piv[j] ? 1u : 0u;
  const unsigned code_of_rank = 0x32547610u;  // rank r -> code nibble r of this word: 0 1 6 7 4 5 2 3
  return ((code_of_rank >> (4 * r)) & 0xFu) + sign;
}

template <bool IN_BF16>
__device__ __forceinline__ float load_w(const void* w, size_t i) {
  if (IN_BF16) return bf2f(((const uint16_t*)w)[i]);
  return ((const float*)w)[i];
}

// one thread per (row, group)
template <bool IN_BF16, int FMT>
__global__ void __launch_bounds__(256) quantize_kernel(const void* __restrict__ w, uint8_t* __restrict__ qw,
                                                      void* __restrict__ scales, int N, int K, int G) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int groups = K / G;
  if (gid >= (long)N * groups) return;
  const int n = (int)(gid / groups), g = (int)(gid % groups);
  const size_t base = (size_t)n * K + (size_t)g * G;
  float amax = 0.0f;
  for (int i = 0; i < G; ++i) amax = fmaxf(amax, fabsf(load_w<IN_BF16>(w, base + i)));
  float inv;
  if (FMT == 0) {
    const uint16_t sb = f2bf(__fdiv_rn(amax, 7.0f));
    ((uint16_t*)scales)[(size_t)n * groups + g] = sb;
    const float s = bf2f(sb);
    inv = s > 0.0f ? __fdiv_rn(1.0f, s) : 0.0f;
  } else {
    ((float*)scales)[(size_t)n * groups + g] = amax;
    inv = amax > 0.0f ? __fdiv_rn(1.0f, amax) : 0.0f;
  }
  uint8_t* out = qw + ((size_t)n * K + (size_t)g * G) / 2;
  for (int i = 0; i < G; i += 2) {
    unsigned c[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float v = __fmul_rn(load_w<IN_BF16>(w, base + i + h), inv);
      if (FMT == 0) {
        float q = rintf(v);
        q = fminf(fmaxf(q, -8.0f), 7.0f);
        c[h] = (unsigned)((int)q + 8);
      } else if (FMT == 3) {
        c[h] = fp4_code(v);
      } else {
        unsigned code = 0;
#pragma unroll
        for (int j = 0; j < 15; ++j) {
          const float mid = __fmul_rn(__fadd_rn(kCode4[0][j + 1], kCode4[0][j]), 0.5f);
          code += (mid < v) ? 1u : 0u;
        }
        c[h] = code;
      }
    }
    out[i / 2] = (uint8_t)(c[0] | (c[1] << 4));
  }
}

// offset = mean(absmax), accumulated in fp64 in a fixed order (one workgroup)
__global__ void __launch_bounds__(1024) absmax_mean_kernel(const float* __restrict__ a, long n, float* __restrict__ out) {
  __shared__ double part[1024];
  double s = 0.0;
  for (long i = threadIdx.x; i < n; i += 1024) s += (double)a[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = (float)(part[0] / (double)n);
}

// dQuantize<0> of bitsandbytes' kQuantizeBlockwise: binary search in the sorted 256-entry code, then the nearer
// of the bracketing pair (midpoint rule, ties to the lower pivot / pivot as the upstream comparisons fall)
__device__ int dq_index(const float* code, float x) {
  int pivot = 127, upper_pivot = 255, lower_pivot = 0;
  float lower = -1.0f, upper = 1.0f, val = code[pivot];
  for (int i = 64; i > 0; i >>= 1) {
    if (x > val) {
      lower_pivot = pivot;
      lower = val;
      pivot += i;
    } else {
      upper_pivot = pivot;
      upper = val;
      pivot -= i;
    }
    val = code[pivot];
  }
  if (upper_pivot == 255) upper = code[upper_pivot];
  if (lower_pivot == 0) lower = code[lower_pivot];
  if (x > val) return x > __fmul_rn(__fadd_rn(upper, val), 0.5f) ? upper_pivot : pivot;
  return x < __fmul_rn(__fadd_rn(lower, val), 0.5f) ? lower_pivot : pivot;
}

// one workgroup per 256 statistics
__global__ void __launch_bounds__(256) double_quant_kernel(float* __restrict__ a, long n, const float* __restrict__ code_g,
                                                           const float* __restrict__ offset_p) {
  __shared__ float code[256];
  __shared__ float red[4];
  code[threadIdx.x] = code_g[threadIdx.x];
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const float offset = *offset_p;
  const float v = i < n ? __fsub_rn(a[i], offset) : 0.0f;
  float m = fabsf(v);
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  const float amax2 = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  if (i >= n) return;
  int q;
  if (amax2 > 0.0f) {
    q = dq_index(code, __fmul_rn(v, __fdiv_rn(1.0f, amax2)));
  } else {  // all statistics of the block equal the offset: the code's zero
    q = 0;
    for (int j = 1; j < 256; ++j)
      if (fabsf(code[j]) < fabsf(code[q])) q = j;
  }
  {
    // two roundings, as bitsandbytes (kDequantizeBlockwise multiplies, then `absmax += offset` is a separate op):
    // HIP's __fmul_rn / __fadd_rn alone do not stop -ffp-contract from fusing them into one fma
#pragma clang fp contract(off)
    const float deq = code[q] * amax2;
    a[i] = deq + offset;
  }
}

// Dequantise packed 4-bit rows to bf16: w[n][k] = bf16(value(nibble) * scale), value = nibble - 8 (int4-g, bf16
// group scale) or NF4[nibble] (nf4, fp32 block absmax) — bit for bit the B tiles gemm_q4_kernel stages, so a bf16
// GEMM over the result equals lga_q4_gemm. One thread: 8 weights (4 B in, 16 B out), so every wave instruction
// reads 256 and writes 1024 contiguous bytes.
template <int FMT>
__global__ void __launch_bounds__(256) dequant_kernel(const uint32_t* __restrict__ qw, const void* __restrict__ sc,
                                                       uint4* __restrict__ w, long words, int K, int group, int cb) {
  const long c = (long)blockIdx.x * 256 + threadIdx.x;
  if (c >= words) return;
  const long n = c / (K / 8), k0 = (c % (K / 8)) * 8;
  const uint32_t q = __builtin_nontemporal_load(qw + c);
  const size_t si = (size_t)n * (K / group) + k0 / group;
  const float s = FMT == 0 ? bf2f(((const uint16_t*)sc)[si]) : ((const float*)sc)[si];
  uint32_t o[4];
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const uint32_t lo = (q >> (4 * e)) & 0xF, hi = (q >> (4 * e + 4)) & 0xF;
    const float vl = FMT == 0 ? (float)((int)lo - 8) : kCode4[cb][lo];
    const float vh = FMT == 0 ? (float)((int)hi - 8) : kCode4[cb][hi];
    o[e / 2] = pack2(mul_rn(vl, s), mul_rn(vh, s));
  }
  w[c] = make_uint4(o[0], o[1], o[2], o[3]);
}

}  // namespace lga

extern "C" int lga_q4_dequantize(const uint8_t* qweight, const void* scales, void* w, int N, int K, int group,
                                 int fmt, hipStream_t stream) {
  LGA_CHECK_ARG(qweight && scales && w, "lga_q4_dequantize: null pointer");
  LGA_CHECK_ARG(N > 0 && K > 0 && K % 32 == 0 && group >= 32 && group % 32 == 0 && K % group == 0,
                "lga_q4_dequantize: K must be a positive multiple of 32 and of the group (a multiple of 32)");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1 || fmt == 3, "lga_q4_dequantize: fmt must be 0 (int4-g), 1 (nf4) or 3 (fp4)");
  LGA_CHECK_ARG(((uintptr_t)qweight | (uintptr_t)w) % 16 == 0, "lga_q4_dequantize: 16-B aligned buffers required");
  const long words = (long)N * (K / 8);
  const dim3 grid((unsigned)((words + 255) / 256));
  if (fmt == 0) lga::dequant_kernel<0><<<grid, 256, 0, stream>>>((const uint32_t*)qweight, scales, (uint4*)w, words, K, group, 0);
  else lga::dequant_kernel<1><<<grid, 256, 0, stream>>>((const uint32_t*)qweight, scales, (uint4*)w, words, K, group,
                                                        lga::codebook_of(fmt));
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_nf4_double_quant(float* absmax, long n, const float* code, float* offset_out,
                                    hipStream_t stream) {
  LGA_CHECK_ARG(absmax && code && offset_out && n > 0, "lga_nf4_double_quant: bad arguments");
  lga::absmax_mean_kernel<<<1, 1024, 0, stream>>>(absmax, n, offset_out);
  lga::double_quant_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(absmax, n, code, offset_out);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_quantize(const void* w, int w_is_bf16, uint8_t* qweight, void* scales, int N, int K,
                            int group, int fmt, hipStream_t stream) {
  LGA_CHECK_ARG(w && qweight && scales, "lga_quantize: null pointer");
  LGA_CHECK_ARG(N > 0 && K > 0 && group > 0 && group % 2 == 0 && K % group == 0,
                "lga_quantize: K must be a positive multiple of an even group size");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1 || fmt == 3, "lga_quantize: fmt must be 0 (int4-g), 1 (nf4) or 3 (fp4)");
  const long total = (long)N * (K / group);
  const dim3 grid((unsigned)((total + 255) / 256)), block(256);
  if (w_is_bf16) {
    if (fmt == 0) lga::quantize_kernel<true, 0><<<grid, block, 0, stream>>>(w, qweight, scales, N, K, group);
    else if (fmt == 1) lga::quantize_kernel<true, 1><<<grid, block, 0, stream>>>(w, qweight, scales, N, K, group);
    else lga::quantize_kernel<true, 3><<<grid, block, 0, stream>>>(w, qweight, scales, N, K, group);
  } else {
    if (fmt == 0) lga::quantize_kernel<false, 0><<<grid, block, 0, stream>>>(w, qweight, scales, N, K, group);
    else if (fmt == 1) lga::quantize_kernel<false, 1><<<grid, block, 0, stream>>>(w, qweight, scales, N, K, group);
    else lga::quantize_kernel<false, 3><<<grid, block, 0, stream>>>(w, qweight, scales, N, K, group);
  }
  LGA_LAUNCH_RETURN();
}
