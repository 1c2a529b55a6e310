// Row-wise and elementwise kernels of the decode/prefill step:
//   lga_rmsnorm        RMSNorm (lit_gpt/rmsnorm.py:19-25): fp32 math, weight multiply in fp32, one bf16 cast
//   lga_rope_kv_append RoPE on q,k (lit_gpt/model.py:641-644, apply_rope :767-773) fused with the KV-cache
//                      write (KVCache.forward :788-795, index_copy_ at input_pos) — cache kept un-expanded
//                      (n_query_groups heads) instead of the reference's expanded copy (:633-635, :675)
//   lga_embedding      token-embedding gather (model.py:515)
//   lga_add            bf16 residual add (Block.forward :591-592) when the add cannot ride a GEMV epilogue (TP)
//   lga_swiglu         silu(a) * b with the reference's rounding points (LLaMAMLP.forward :715)
//   lga_layernorm      torch.nn.LayerNorm (GPT-NeoX / pythia norm_class, reference config.py:137-144): fp32 mean and
//                      variance, (x - mean) * rstd * w + b in fp32, one bf16 cast
//   lga_gelu           GptNeoxMLP's activation (model.py:699-702): F.gelu exact (erf) or tanh, fp32, one bf16 cast
#include <algorithm>

#include "common.h"

namespace lga {

__global__ void __launch_bounds__(256) rmsnorm_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                      uint16_t* __restrict__ y, int n, float eps) {
  const size_t row = blockIdx.x;
  const uint16_t* xr = x + row * n;
  uint16_t* yr = y + row * n;
  __shared__ float red[4];
  float ss = 0.0f;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float v = bf2f(xr[i]);
    ss = fmaf(v, v, ss);
  }
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float rs = 1.0f / sqrtf((red[0] + red[1] + red[2] + red[3]) / (float)n + eps);
  for (int i = threadIdx.x; i < n; i += 256) yr[i] = f2bf(__fmul_rn(bf2f(w[i]), __fmul_rn(bf2f(xr[i]), rs)));
}

// 16-B form for rows of n % 8 == 0, n <= 8 * 256 * VPT: every thread loads its VPT uint4 of x and of the weight
// once (all in flight together), keeps x in registers for the scaling pass — one read of x instead of two 2-B
// scalar passes. Same math (fp32 sum of squares, w * (x * rs) rounded once); the sum runs in another order.
template <int VPT>
__global__ void __launch_bounds__(256) rmsnorm_vec_kernel(const uint4* __restrict__ x, const uint4* __restrict__ w,
                                                          uint4* __restrict__ y, int n8, float eps) {
  const size_t row = blockIdx.x;
  const uint4* xr = x + row * n8;
  uint4* yr = y + row * n8;
  uint4 xv[VPT], wv[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int u = min((int)threadIdx.x + 256 * i, n8 - 1);
    xv[i] = xr[u];
    wv[i] = w[u];
  }
  float ss = 0.0f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    if ((int)threadIdx.x + 256 * i < n8) {
      const uint32_t d[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        ss = fmaf(bflo(d[q]), bflo(d[q]), ss);
        ss = fmaf(bfhi(d[q]), bfhi(d[q]), ss);
      }
    }
  }
  __shared__ float red[4];
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float rs = 1.0f / sqrtf((red[0] + red[1] + red[2] + red[3]) / (float)(n8 * 8) + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int u = (int)threadIdx.x + 256 * i;
    if (u < n8) {
      const uint32_t d[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
      const uint32_t m[4] = {wv[i].x, wv[i].y, wv[i].z, wv[i].w};
      uint32_t o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        o[q] = pack2(__fmul_rn(bflo(m[q]), __fmul_rn(bflo(d[q]), rs)), __fmul_rn(bfhi(m[q]), __fmul_rn(bfhi(d[q]), rs)));
      yr[u] = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
}

__global__ void __launch_bounds__(256) layernorm_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                        const uint16_t* __restrict__ b, uint16_t* __restrict__ y,
                                                        int n, float eps) {
  const size_t row = blockIdx.x;
  const uint16_t* xr = x + row * n;
  uint16_t* yr = y + row * n;
  __shared__ float red[4];
  float s = 0.0f;
  for (int i = threadIdx.x; i < n; i += 256) s += bf2f(xr[i]);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const float mean = ((red[0] + red[1]) + (red[2] + red[3])) / (float)n;
  __syncthreads();
  float ss = 0.0f;  // two-pass variance (biased, as torch.nn.LayerNorm)
  for (int i = threadIdx.x; i < n; i += 256) {
    const float d = bf2f(xr[i]) - mean;
    ss = fmaf(d, d, ss);
  }
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float rstd = 1.0f / sqrtf(((red[0] + red[1]) + (red[2] + red[3])) / (float)n + eps);
  for (int i = threadIdx.x; i < n; i += 256) {
    const float v = __fmul_rn(__fmul_rn(bf2f(xr[i]) - mean, rstd), bf2f(w[i]));
    yr[i] = f2bf(b ? v + bf2f(b[i]) : v);
  }
}

__global__ void __launch_bounds__(256) gelu_kernel(const uint16_t* __restrict__ a, uint16_t* __restrict__ y, size_t n,
                                                   int approximate_tanh) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float v = bf2f(a[i]);
    float g;
    if (approximate_tanh) {
      const float inner = 0.7978845608028654f * (v + 0.044715f * v * v * v);
      g = 0.5f * v * (1.0f + tanhf(inner));
    } else {
      g = 0.5f * v * (1.0f + erff(v * 0.7071067811865476f));
    }
    y[i] = f2bf(g);
  }
}

// grid (T, G): one workgroup per (token, query group); slots 0..qpk-1 = q heads, qpk = k, qpk+1 = v
__global__ void __launch_bounds__(256) rope_kv_kernel(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ q_out,
                                                      uint16_t* __restrict__ k_cache, uint16_t* __restrict__ v_cache,
                                                      const int64_t* __restrict__ cache_pos,
                                                      const int64_t* __restrict__ rope_pos,
                                                      const float* __restrict__ cos, const float* __restrict__ sin,
                                                      int n_head, int n_groups, int hs, int n_elem, int max_seq,
                                                      int rope_rows) {
  const int t = blockIdx.x, g = blockIdx.y;
  const int qpk = n_head / n_groups;
  const long p = cache_pos[t];
  const long rp = rope_pos[t];
  if (p < 0 || p >= max_seq || rp < 0 || rp >= rope_rows) return;  // host validates; never go out of bounds
  const uint16_t* src = qkv + ((size_t)t * (n_head + 2 * n_groups) + (size_t)g * (qpk + 2)) * hs;
  const float* cr = cos + (size_t)rp * n_elem;
  const float* sr = sin + (size_t)rp * n_elem;
  const int half = n_elem / 2;
  const int items = (qpk + 2) * hs;
  for (int it = threadIdx.x; it < items; it += blockDim.x) {
    const int slot = it / hs, d = it % hs;
    const uint16_t* xs = src + (size_t)slot * hs;
    uint16_t out = xs[d];
    if (slot <= qpk && d < n_elem) {
      const float x = bf2f(xs[d]);
      const float r = d < half ? -bf2f(xs[d + half]) : bf2f(xs[d - half]);
      out = f2bf(add_rn(mul_rn(x, cr[d]), mul_rn(r, sr[d])));
    }
    if (slot < qpk) {
      q_out[((size_t)t * n_head + (size_t)g * qpk + slot) * hs + d] = out;
    } else if (slot == qpk) {
      k_cache[((size_t)g * max_seq + p) * hs + d] = out;
    } else {
      v_cache[((size_t)g * max_seq + p) * hs + d] = out;
    }
  }
}

// Vector form of rope_kv_kernel (same arithmetic per element): one thread moves one 16-B chunk (8 elements) of a
// (token, group, slot) row; the rotate-half partner is the chunk half / 8 away. Needs hs % 8 == 0 and
// (rope_n_elem / 2) % 8 == 0 (Llama: 128 / 64, pythia: 16 / 8); other geometries take the scalar kernel.
__global__ void __launch_bounds__(256) rope_kv_vec_kernel(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ q_out,
                                                          uint16_t* __restrict__ k_cache,
                                                          uint16_t* __restrict__ v_cache,
                                                          const int64_t* __restrict__ cache_pos,
                                                          const int64_t* __restrict__ rope_pos,
                                                          const float* __restrict__ cos, const float* __restrict__ sin,
                                                          int T, int n_head, int n_groups, int hs, int n_elem,
                                                          int max_seq, int rope_rows) {
  const int qpk = n_head / n_groups, cph = hs / 8, half = n_elem / 2;
  const long per_t = (long)n_groups * (qpk + 2) * cph;  // chunks per token
  const long total = (long)T * per_t;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int t = (int)(i / per_t);
    const int rem = (int)(i % per_t);
    const int g = rem / ((qpk + 2) * cph), slot = (rem / cph) % (qpk + 2), c = rem % cph;
    const long p = cache_pos[t], rp = rope_pos[t];
    if (p < 0 || p >= max_seq || rp < 0 || rp >= rope_rows) continue;  // host validates; never out of bounds
    const uint16_t* xs = qkv + ((size_t)t * (n_head + 2 * n_groups) + (size_t)g * (qpk + 2) + slot) * hs;
    uint4 v = ((const uint4*)xs)[c];
    const int d0 = c * 8;
    if (slot <= qpk && d0 < n_elem) {
      const bool lo = d0 < half;
      const uint4 pv = ((const uint4*)xs)[lo ? c + half / 8 : c - half / 8];
      const float4* cr = (const float4*)(cos + (size_t)rp * n_elem + d0);
      const float4* sr = (const float4*)(sin + (size_t)rp * n_elem + d0);
      const float4 c0 = cr[0], c1 = cr[1], s0 = sr[0], s1 = sr[1];
      const float cf[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      const float sf[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      const uint32_t xw[4] = {v.x, v.y, v.z, v.w}, pw[4] = {pv.x, pv.y, pv.z, pv.w};
      uint32_t ow[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float x0 = bflo(xw[k]), x1 = bfhi(xw[k]);
        const float r0 = lo ? -bflo(pw[k]) : bflo(pw[k]), r1 = lo ? -bfhi(pw[k]) : bfhi(pw[k]);
        const float o0 = add_rn(mul_rn(x0, cf[2 * k]), mul_rn(r0, sf[2 * k]));
        const float o1 = add_rn(mul_rn(x1, cf[2 * k + 1]), mul_rn(r1, sf[2 * k + 1]));
        ow[k] = (uint32_t)f2bf(o0) | ((uint32_t)f2bf(o1) << 16);
      }
      v = make_uint4(ow[0], ow[1], ow[2], ow[3]);
    }
    uint4* dst = slot < qpk ? (uint4*)(q_out + ((size_t)t * n_head + (size_t)g * qpk + slot) * hs)
                            : (uint4*)((slot == qpk ? k_cache : v_cache) + ((size_t)g * max_seq + p) * hs);
    dst[c] = v;
  }
}

__global__ void __launch_bounds__(256) add_vec_kernel(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                                      uint4* __restrict__ y, size_t n8) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
    const uint4 u = a[i], w = b[i];
    const uint32_t ua[4] = {u.x, u.y, u.z, u.w}, wa[4] = {w.x, w.y, w.z, w.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      o[k] = (uint32_t)f2bf(bflo(ua[k]) + bflo(wa[k])) | ((uint32_t)f2bf(bfhi(ua[k]) + bfhi(wa[k])) << 16);
    y[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

__global__ void __launch_bounds__(256) swiglu_vec_kernel(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                                         uint4* __restrict__ y, size_t n8) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
    const uint4 u = a[i], w = b[i];
    const uint32_t ua[4] = {u.x, u.y, u.z, u.w}, wa[4] = {w.x, w.y, w.z, w.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float g0 = round_bf(silu_f(bflo(ua[k]))), g1 = round_bf(silu_f(bfhi(ua[k])));
      o[k] = (uint32_t)f2bf(__fmul_rn(g0, bflo(wa[k]))) | ((uint32_t)f2bf(__fmul_rn(g1, bfhi(wa[k]))) << 16);
    }
    y[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

template <typename IDX>
__global__ void __launch_bounds__(256) embedding_kernel(const IDX* __restrict__ idx, const uint16_t* __restrict__ table,
                                                        uint16_t* __restrict__ out, int C, int V) {
  const int t = blockIdx.x;
  long id = (long)idx[t];
  id = id < 0 ? 0 : (id >= V ? V - 1 : id);  // host validates ids; clamp keeps the gather in bounds
  const uint4* src = (const uint4*)(table + (size_t)id * C);
  uint4* dst = (uint4*)(out + (size_t)t * C);
  for (int i = threadIdx.x; i < C / 8; i += 256) dst[i] = src[i];
}

__global__ void __launch_bounds__(256) add_kernel(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b,
                                                  uint16_t* __restrict__ y, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    y[i] = f2bf(bf2f(a[i]) + bf2f(b[i]));
}

__global__ void __launch_bounds__(256) swiglu_kernel(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b,
                                                     uint16_t* __restrict__ y, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float g = round_bf(silu_f(bf2f(a[i])));
    y[i] = f2bf(__fmul_rn(g, bf2f(b[i])));
  }
}

static unsigned elementwise_grid(size_t n) {
  size_t g = (n + 255) / 256;
  return (unsigned)(g > 4096 ? 4096 : (g == 0 ? 1 : g));
}

}  // namespace lga

int lga::preload_norm_rope() {
  return lga::preload(lga::rmsnorm_vec_kernel<1>) + lga::preload(lga::rmsnorm_vec_kernel<2>) +
         lga::preload(lga::rmsnorm_vec_kernel<3>) + lga::preload(lga::rmsnorm_vec_kernel<4>) +
         lga::preload(lga::rope_kv_vec_kernel) + lga::preload(lga::embedding_kernel<int64_t>) +
         lga::preload(lga::embedding_kernel<int32_t>);
}

extern "C" int lga_rmsnorm(const void* x, const void* weight, void* y, int rows, int n, float eps,
                           hipStream_t stream) {
  LGA_CHECK_ARG(x && weight && y && rows > 0 && n > 0, "lga_rmsnorm: bad arguments");
  const bool al = (((uintptr_t)x | (uintptr_t)weight | (uintptr_t)y) & 15) == 0;
  const int n8 = n / 8, vpt = (n8 + 255) / 256;
  if (al && n % 8 == 0 && vpt <= 4) {
#define LGA_RMS(V)                                                                                               \
  lga::rmsnorm_vec_kernel<V><<<rows, 256, 0, stream>>>((const uint4*)x, (const uint4*)weight, (uint4*)y, n8, eps)
    if (vpt == 1) LGA_RMS(1);
    else if (vpt == 2) LGA_RMS(2);
    else if (vpt == 3) LGA_RMS(3);
    else LGA_RMS(4);
#undef LGA_RMS
  } else {
    lga::rmsnorm_kernel<<<rows, 256, 0, stream>>>((const uint16_t*)x, (const uint16_t*)weight, (uint16_t*)y, n, eps);
  }
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_rope_kv_append(const void* qkv, void* q_out, void* k_cache, void* v_cache,
                                  const int64_t* cache_pos, const int64_t* rope_pos, const float* cos,
                                  const float* sin, int rope_rows, int T, int n_head, int n_query_groups,
                                  int head_size, int rope_n_elem, int max_seq, hipStream_t stream) {
  LGA_CHECK_ARG(qkv && q_out && k_cache && v_cache && cache_pos && rope_pos && (rope_n_elem == 0 || (cos && sin)),
                "lga_rope_kv_append: null pointer");
  LGA_CHECK_ARG(T > 0 && n_query_groups > 0 && n_head % n_query_groups == 0 && head_size > 0,
                "lga_rope_kv_append: bad head geometry");
  LGA_CHECK_ARG(rope_n_elem >= 0 && rope_n_elem <= head_size && rope_n_elem % 2 == 0,
                "lga_rope_kv_append: rope_n_elem must be even and <= head_size");
  if (head_size % 8 == 0 && (rope_n_elem / 2) % 8 == 0 &&
      ((uintptr_t)qkv | (uintptr_t)q_out | (uintptr_t)k_cache | (uintptr_t)v_cache | (uintptr_t)cos | (uintptr_t)sin) % 16 == 0) {
    const long chunks = (long)T * (n_head + 2 * n_query_groups) * (head_size / 8);
    const unsigned blocks = (unsigned)std::min<long>((chunks + 255) / 256, 8192);
    lga::rope_kv_vec_kernel<<<blocks, 256, 0, stream>>>((const uint16_t*)qkv, (uint16_t*)q_out, (uint16_t*)k_cache,
                                                       (uint16_t*)v_cache, cache_pos, rope_pos, cos, sin, T, n_head,
                                                       n_query_groups, head_size, rope_n_elem, max_seq, rope_rows);
    LGA_LAUNCH_RETURN();
  }
  const dim3 grid(T, n_query_groups);
  lga::rope_kv_kernel<<<grid, 256, 0, stream>>>((const uint16_t*)qkv, (uint16_t*)q_out, (uint16_t*)k_cache,
                                                (uint16_t*)v_cache, cache_pos, rope_pos, cos, sin, n_head,
                                                n_query_groups, head_size, rope_n_elem, max_seq, rope_rows);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_embedding(const void* idx, int idx_is_int64, const void* table, void* out, int T, int C, int V,
                             hipStream_t stream) {
  LGA_CHECK_ARG(idx && table && out && T > 0 && C > 0 && C % 8 == 0 && V > 0, "lga_embedding: bad arguments");
  if (idx_is_int64)
    lga::embedding_kernel<int64_t><<<T, 256, 0, stream>>>((const int64_t*)idx, (const uint16_t*)table,
                                                          (uint16_t*)out, C, V);
  else
    lga::embedding_kernel<int32_t><<<T, 256, 0, stream>>>((const int32_t*)idx, (const uint16_t*)table,
                                                          (uint16_t*)out, C, V);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_add(const void* a, const void* b, void* y, long n, hipStream_t stream) {
  LGA_CHECK_ARG(a && b && y && n > 0, "lga_add: bad arguments");
  if (n % 8 == 0 && ((uintptr_t)a | (uintptr_t)b | (uintptr_t)y) % 16 == 0) {
    lga::add_vec_kernel<<<lga::elementwise_grid(n / 8), 256, 0, stream>>>((const uint4*)a, (const uint4*)b, (uint4*)y,
                                                                         (size_t)n / 8);
    LGA_LAUNCH_RETURN();
  }
  lga::add_kernel<<<lga::elementwise_grid(n), 256, 0, stream>>>((const uint16_t*)a, (const uint16_t*)b,
                                                                 (uint16_t*)y, (size_t)n);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_swiglu(const void* a, const void* b, void* y, long n, hipStream_t stream) {
  LGA_CHECK_ARG(a && b && y && n > 0, "lga_swiglu: bad arguments");
  if (n % 8 == 0 && ((uintptr_t)a | (uintptr_t)b | (uintptr_t)y) % 16 == 0) {
    lga::swiglu_vec_kernel<<<lga::elementwise_grid(n / 8), 256, 0, stream>>>((const uint4*)a, (const uint4*)b,
                                                                            (uint4*)y, (size_t)n / 8);
    LGA_LAUNCH_RETURN();
  }
  lga::swiglu_kernel<<<lga::elementwise_grid(n), 256, 0, stream>>>((const uint16_t*)a, (const uint16_t*)b,
                                                                    (uint16_t*)y, (size_t)n);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_layernorm(const void* x, const void* weight, const void* bias, void* y, int rows, int n, float eps,
                             hipStream_t stream) {
  LGA_CHECK_ARG(x && weight && y && rows > 0 && n > 0, "lga_layernorm: bad arguments");
  lga::layernorm_kernel<<<rows, 256, 0, stream>>>((const uint16_t*)x, (const uint16_t*)weight, (const uint16_t*)bias,
                                                   (uint16_t*)y, n, eps);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_gelu(const void* a, void* y, long n, int approximate_tanh, hipStream_t stream) {
  LGA_CHECK_ARG(a && y && n > 0, "lga_gelu: bad arguments");
  lga::gelu_kernel<<<lga::elementwise_grid(n), 256, 0, stream>>>((const uint16_t*)a, (uint16_t*)y, (size_t)n,
                                                                  approximate_tanh);
  LGA_LAUNCH_RETURN();
}
