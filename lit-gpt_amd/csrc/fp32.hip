// fp32 forward path: the reference's `--precision 32-true` (generate/base.py:132, Fabric precision "32-true":
// weights and activations in float32). BASELINE config 1 is quoted in it (pythia-160m fp32, greedy 128 tokens);
// the bf16 kernels round every activation to bf16, which the fp32 fixture (tests/golden/g1) does not.
//
// Plumbing-sized, not tuned: config 1 is the reference's CPU-runnable case (a 160M model), so these kernels keep
// the reference's per-op arithmetic — fp32 products and sums, no bf16 rounding anywhere — in simple forms:
//   lga_f32_linear          F.linear (lit_gpt/model.py:619, 656, 699-702, 519): y = x W^T (+ b) (+ residual)
//   lga_f32_layernorm       torch.nn.LayerNorm (GPT-NeoX norm_class, config.py:137-144): two-pass mean / biased var
//   lga_f32_gelu            F.gelu exact (erf) or tanh (GptNeoxMLP, model.py:699-702)
//   lga_f32_add             the Block's residual adds (model.py:584-593)
//   lga_f32_rope_kv_append  apply_rope (model.py:767-773, partial rotary) + KVCache.forward (:788-795)
//   lga_f32_attention       SDPA over the cache with the input_pos mask rows (model.py:651, 658-665)
// (the token-embedding gather is lga_embedding over the fp32 rows as pairs of 16-bit words — a byte copy; greedy
// sampling is lga_argmax_f32 in sample.hip)
#include "common.h"

namespace lga {

// one wave per output (m, n): lanes stride over K (16-B loads when K % 4 == 0), then a wave sum
__global__ void __launch_bounds__(256) f32_linear_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ b, const float* __restrict__ res,
                                                         float* __restrict__ y, int N, int K) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + wave, m = blockIdx.y;
  if (n >= N) return;
  const float* xr = x + (size_t)m * K;
  const float* wr = w + (size_t)n * K;
  float acc = 0.0f;
  if ((K & 3) == 0) {
    for (int k = lane * 4; k < K; k += 256) {
      const float4 xv = *(const float4*)(xr + k), wv = *(const float4*)(wr + k);
      acc = fmaf(xv.x, wv.x, acc);
      acc = fmaf(xv.y, wv.y, acc);
      acc = fmaf(xv.z, wv.z, acc);
      acc = fmaf(xv.w, wv.w, acc);
    }
  } else {
    for (int k = lane; k < K; k += 64) acc = fmaf(xr[k], wr[k], acc);
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    if (b) acc += b[n];
    if (res) acc += res[(size_t)m * N + n];
    y[(size_t)m * N + n] = acc;
  }
}

__global__ void __launch_bounds__(256) f32_layernorm_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ b, float* __restrict__ y, int n,
                                                            float eps) {
  const size_t row = blockIdx.x;
  const float* xr = x + row * n;
  float* yr = y + row * n;
  __shared__ float red[4];
  float s = 0.0f;
  for (int i = threadIdx.x; i < n; i += 256) s += xr[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const float mean = ((red[0] + red[1]) + (red[2] + red[3])) / (float)n;
  __syncthreads();
  float ss = 0.0f;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float d = xr[i] - mean;
    ss = fmaf(d, d, ss);
  }
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float rstd = 1.0f / sqrtf(((red[0] + red[1]) + (red[2] + red[3])) / (float)n + eps);
  for (int i = threadIdx.x; i < n; i += 256) {
    const float v = mul_rn(mul_rn(xr[i] - mean, rstd), w[i]);
    yr[i] = b ? add_rn(v, b[i]) : v;
  }
}

__global__ void __launch_bounds__(256) f32_gelu_kernel(const float* __restrict__ a, float* __restrict__ y, size_t n,
                                                       int approximate_tanh) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float v = a[i];
    if (approximate_tanh) {
      const float inner = 0.7978845608028654f * (v + 0.044715f * v * v * v);
      y[i] = 0.5f * v * (1.0f + tanhf(inner));
    } else {
      y[i] = 0.5f * v * (1.0f + erff(v * 0.7071067811865476f));
    }
  }
}

__global__ void __launch_bounds__(256) f32_add_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                      float* __restrict__ y, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) y[i] = a[i] + b[i];
}

// grid (T, G): the q heads, k and v of query group g for token t (qkv row layout per group [q_0..q_{qpk-1}, k, v],
// scripts/convert_hf_checkpoint.py:174-188); x * cos + rotate_half(x) * sin on the first n_elem dims, two roundings
__global__ void __launch_bounds__(256) f32_rope_kv_kernel(const float* __restrict__ qkv, float* __restrict__ q_out,
                                                          float* __restrict__ k_cache, float* __restrict__ v_cache,
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
  const float* src = qkv + ((size_t)t * (n_head + 2 * n_groups) + (size_t)g * (qpk + 2)) * hs;
  const float* cr = cos + (size_t)rp * n_elem;
  const float* sr = sin + (size_t)rp * n_elem;
  const int half = n_elem / 2;
  for (int it = threadIdx.x; it < (qpk + 2) * hs; it += blockDim.x) {
    const int slot = it / hs, d = it % hs;
    const float* xs = src + (size_t)slot * hs;
    float out = xs[d];
    if (slot <= qpk && d < n_elem) {
      const float r = d < half ? -xs[d + half] : xs[d - half];
      out = add_rn(mul_rn(xs[d], cr[d]), mul_rn(r, sr[d]));
    }
    if (slot < qpk) q_out[((size_t)t * n_head + (size_t)g * qpk + slot) * hs + d] = out;
    else if (slot == qpk) k_cache[((size_t)g * max_seq + p) * hs + d] = out;
    else v_cache[((size_t)g * max_seq + p) * hs + d] = out;
  }
}

// grid (T, H): softmax(q . K^T * scale) . V over keys 0..input_pos[t] of the query's group; scores kept in LDS
// (max_seq floats), exact max, fp32 exp and sums
__global__ void __launch_bounds__(256) f32_attention_kernel(const float* __restrict__ q, const float* __restrict__ kc,
                                                            const float* __restrict__ vc,
                                                            const int64_t* __restrict__ input_pos, float* __restrict__ y,
                                                            int n_head, int n_groups, int hs, int max_seq, float scale) {
  extern __shared__ float sc[];  // [max_seq] scores, then [256] partials
  __shared__ float red[4];
  __shared__ float qs[256];
  const int t = blockIdx.x, h = blockIdx.y;
  const int g = h / (n_head / n_groups);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long p = input_pos[t];
  const int L = (int)min(max(p + 1, 1L), (long)max_seq);
  const float* qr = q + ((size_t)t * n_head + h) * hs;
  for (int d = threadIdx.x; d < hs; d += 256) qs[d] = qr[d];
  __syncthreads();
  const float* kb = kc + (size_t)g * max_seq * hs;
  const float* vb = vc + (size_t)g * max_seq * hs;
  float mx = -INFINITY;
  for (int j = wave; j < L; j += 4) {
    float d = 0.0f;
    for (int e = lane; e < hs; e += 64) d = fmaf(qs[e], kb[(size_t)j * hs + e], d);
    d = wave_sum(d) * scale;
    mx = fmaxf(mx, d);
    if (lane == 0) sc[j] = d;
  }
  if (lane == 0) red[wave] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.0f;
  for (int j = threadIdx.x; j < L; j += 256) {
    const float e = expf(sc[j] - mx);
    sc[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  if (lane == 0) red[wave] = sum;
  __syncthreads();
  sum = (red[0] + red[1]) + (red[2] + red[3]);
  // P.V: thread -> (dim d = tid % hs', key phase tid / hs') with hs' = min(hs, 256); partials reduced in LDS
  float* part = sc + max_seq;
  const int HSP = hs < 256 ? hs : 256, phases = 256 / HSP;
  const int ph = threadIdx.x / HSP, dd = threadIdx.x % HSP;
  for (int d0 = 0; d0 < hs; d0 += HSP) {
    float o = 0.0f;
    if (ph < phases)
      for (int j = ph; j < L; j += phases) o = fmaf(sc[j], vb[(size_t)j * hs + d0 + dd], o);
    part[threadIdx.x] = o;
    __syncthreads();
    if (threadIdx.x < HSP) {
      float acc = 0.0f;
      for (int k = 0; k < phases; ++k) acc += part[k * HSP + threadIdx.x];
      y[((size_t)t * n_head + h) * hs + d0 + threadIdx.x] = acc / sum;
    }
    __syncthreads();
  }
}

static unsigned elementwise_blocks(size_t n) { return (unsigned)std::min<size_t>((n + 255) / 256, 65535); }

}  // namespace lga

extern "C" int lga_f32_linear(const float* x, const float* w, const float* bias, const float* residual, float* y,
                              int M, int N, int K, hipStream_t stream) {
  LGA_CHECK_ARG(x && w && y && M > 0 && N > 0 && K > 0 && M <= 65535, "lga_f32_linear: bad arguments");
  LGA_CHECK_ARG(((uintptr_t)x | (uintptr_t)w) % 16 == 0 || K % 4 != 0, "lga_f32_linear: 16-B aligned x, w needed");
  lga::f32_linear_kernel<<<dim3((N + 3) / 4, M), 256, 0, stream>>>(x, w, bias, residual, y, N, K);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_f32_layernorm(const float* x, const float* w, const float* b, float* y, int rows, int n, float eps,
                                 hipStream_t stream) {
  LGA_CHECK_ARG(x && w && y && rows > 0 && n > 0, "lga_f32_layernorm: bad arguments");
  lga::f32_layernorm_kernel<<<rows, 256, 0, stream>>>(x, w, b, y, n, eps);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_f32_gelu(const float* a, float* y, long n, int approximate_tanh, hipStream_t stream) {
  LGA_CHECK_ARG(a && y && n > 0, "lga_f32_gelu: bad arguments");
  lga::f32_gelu_kernel<<<lga::elementwise_blocks((size_t)n), 256, 0, stream>>>(a, y, (size_t)n, approximate_tanh);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_f32_add(const float* a, const float* b, float* y, long n, hipStream_t stream) {
  LGA_CHECK_ARG(a && b && y && n > 0, "lga_f32_add: bad arguments");
  lga::f32_add_kernel<<<lga::elementwise_blocks((size_t)n), 256, 0, stream>>>(a, b, y, (size_t)n);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_f32_rope_kv_append(const float* qkv, float* q_out, float* k_cache, float* v_cache,
                                      const int64_t* cache_pos, const int64_t* rope_pos, const float* cos,
                                      const float* sin, int rope_rows, int T, int n_head, int n_query_groups,
                                      int head_size, int rope_n_elem, int max_seq, hipStream_t stream) {
  LGA_CHECK_ARG(qkv && q_out && k_cache && v_cache && cache_pos && rope_pos && cos && sin,
                "lga_f32_rope_kv_append: null pointer");
  LGA_CHECK_ARG(T > 0 && n_query_groups > 0 && n_head % n_query_groups == 0 && head_size > 0 &&
                    rope_n_elem % 2 == 0 && rope_n_elem <= head_size && max_seq > 0 && rope_rows > 0,
                "lga_f32_rope_kv_append: bad geometry");
  lga::f32_rope_kv_kernel<<<dim3(T, n_query_groups), 256, 0, stream>>>(qkv, q_out, k_cache, v_cache, cache_pos,
                                                                       rope_pos, cos, sin, n_head, n_query_groups,
                                                                       head_size, rope_n_elem, max_seq, rope_rows);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_f32_attention(const float* q, const float* k_cache, const float* v_cache, const int64_t* input_pos,
                                 float* y, int T, int n_head, int n_query_groups, int head_size, int max_seq,
                                 float scale, hipStream_t stream) {
  LGA_CHECK_ARG(q && k_cache && v_cache && input_pos && y, "lga_f32_attention: null pointer");
  LGA_CHECK_ARG(T > 0 && T <= 65535 && n_query_groups > 0 && n_head % n_query_groups == 0 && head_size > 0 &&
                    head_size <= 256,
                "lga_f32_attention: bad geometry (head_size <= 256)");
  LGA_CHECK_ARG(max_seq > 0 && max_seq <= 32768, "lga_f32_attention: max_seq must be in [1, 32768] (scores in LDS)");
  const size_t lds = ((size_t)max_seq + 256) * sizeof(float);
  lga::f32_attention_kernel<<<dim3(T, n_head), 256, lds, stream>>>(q, k_cache, v_cache, input_pos, y, n_head,
                                                                    n_query_groups, head_size, max_seq, scale);
  LGA_LAUNCH_RETURN();
}
