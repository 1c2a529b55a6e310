// Cached causal attention for decode (T = 1, split over the sequence) and prefill (T rows, one split).
//
// Replaces CausalSelfAttention.scaled_dot_product_attention (lit_gpt/model.py:651, :658-665): SDPA of q
// against the full max_seq-long cache under the bool mask row(s) selected by input_pos (model.py:509). The
// mask allows key j for query t iff j <= input_pos[t]; this kernel reads only those keys.
//
// KV cache layout (HBM): k, v = [G][max_seq][hs] bf16 per layer (un-expanded query groups); one key row is
// hs*2 contiguous bytes, read by a "row group" of hs/8 lanes at 16 B per lane.
//
// Work decomposition: grid (splits, G, T); a 256-thread workgroup owns one (split, group, query row) and all
// q_per_kv query heads of that group (GQA/MQA read each K/V row once). Inside, every row group streams its
// own keys with an independent online softmax; states are merged per wave with shuffles, then across the
// 4 waves in LDS. With splits > 1 the per-split (m, l, o) go to an fp32 workspace that lga_attention_combine
// merges (flash-decoding); with one split the bf16 output is written directly.
#include "common.h"

namespace lga {

template <int LPR>
__device__ __forceinline__ float row_group_sum(float v) {
  // LPR = 16: full DPP row; LPR = 8: half row
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  if (LPR == 16) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
  return v;
}

template <int HS, int QPK>
__global__ void __launch_bounds__(256) attn_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                                   const uint16_t* __restrict__ vc,
                                                   const int64_t* __restrict__ input_pos, uint16_t* __restrict__ y,
                                                   float* __restrict__ ws, int n_head, int max_seq, int chunk,
                                                   float scale) {
  constexpr int LPR = HS / 8;      // lanes per key row
  constexpr int RGW = 64 / LPR;    // row groups per wave
  constexpr int RG = 4 * RGW;      // row groups per workgroup
  const int split = blockIdx.x, g = blockIdx.y, t = blockIdx.z;
  const int n_splits = gridDim.x, G = gridDim.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rg = wave * RGW + lane / LPR;  // row group id in the workgroup
  const int sub = lane % LPR;              // 8-dim slice of the row
  const long p = input_pos[t];
  const int k_lo = split * chunk;
  const int k_hi = (int)min(min((long)k_lo + chunk, p + 1), (long)max_seq);  // never read past the cache

  float qf[QPK][8];
#pragma unroll
  for (int h = 0; h < QPK; ++h) {
    const uint4 qv = *(const uint4*)(q + ((size_t)t * n_head + (size_t)g * QPK + h) * HS + sub * 8);
    const uint32_t d[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      qf[h][2 * j] = bflo(d[j]);
      qf[h][2 * j + 1] = bfhi(d[j]);
    }
  }
  float m[QPK], l[QPK], o[QPK][8];
#pragma unroll
  for (int h = 0; h < QPK; ++h) {
    m[h] = -INFINITY;
    l[h] = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[h][i] = 0.0f;
  }
  const uint16_t* kbase = kc + (size_t)g * max_seq * HS + sub * 8;
  const uint16_t* vbase = vc + (size_t)g * max_seq * HS + sub * 8;
  for (int j = k_lo + rg; j < k_hi; j += RG) {
    const uint4 kv = *(const uint4*)(kbase + (size_t)j * HS);
    const uint4 vv = *(const uint4*)(vbase + (size_t)j * HS);
    const uint32_t kd[4] = {kv.x, kv.y, kv.z, kv.w};
    const uint32_t vd[4] = {vv.x, vv.y, vv.z, vv.w};
    float kf[8], vf[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      kf[2 * i] = bflo(kd[i]);
      kf[2 * i + 1] = bfhi(kd[i]);
      vf[2 * i] = bflo(vd[i]);
      vf[2 * i + 1] = bfhi(vd[i]);
    }
#pragma unroll
    for (int h = 0; h < QPK; ++h) {
      float s = 0.0f;
#pragma unroll
      for (int i = 0; i < 8; ++i) s = fmaf(qf[h][i], kf[i], s);
      s = row_group_sum<LPR>(s) * scale;
      const float mn = fmaxf(m[h], s);
      const float c = expf(m[h] - mn);  // m = -inf on the first key -> 0
      const float e = expf(s - mn);
      l[h] = fmaf(l[h], c, e);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[h][i] = fmaf(o[h][i], c, e * vf[i]);
      m[h] = mn;
    }
  }
  // merge the RGW row groups of this wave (lanes differing in the bits above log2(LPR))
#pragma unroll
  for (int off = LPR; off < 64; off <<= 1) {
#pragma unroll
    for (int h = 0; h < QPK; ++h) {
      const float mo = __shfl_xor(m[h], off), lo = __shfl_xor(l[h], off);
      const float mn = fmaxf(m[h], mo);
      const float ca = mn == -INFINITY ? 0.0f : expf(m[h] - mn);
      const float cb = mn == -INFINITY ? 0.0f : expf(mo - mn);
      l[h] = l[h] * ca + lo * cb;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float oo = __shfl_xor(o[h][i], off);
        o[h][i] = o[h][i] * ca + oo * cb;
      }
      m[h] = mn;
    }
  }
  // merge the 4 waves through LDS
  __shared__ float sm[4][QPK], sl[4][QPK];
  __shared__ float so[4][QPK][HS];
  if (lane < LPR) {
#pragma unroll
    for (int h = 0; h < QPK; ++h) {
      if (lane == 0) {
        sm[wave][h] = m[h];
        sl[wave][h] = l[h];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) so[wave][h][sub * 8 + i] = o[h][i];
    }
  }
  __syncthreads();
  for (int it = threadIdx.x; it < QPK * HS; it += 256) {
    const int h = it / HS, d = it % HS;
    float mx = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) mx = fmaxf(mx, sm[w][h]);
    float lt = 0.0f, ot = 0.0f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float c = mx == -INFINITY ? 0.0f : expf(sm[w][h] - mx);
      lt += sl[w][h] * c;
      ot += so[w][h][d] * c;
    }
    const int head = g * QPK + h;
    if (n_splits == 1) {
      y[((size_t)t * n_head + head) * HS + d] = f2bf(ot / lt);
    } else {
      float* wsr = ws + (((size_t)t * n_head + head) * n_splits + split) * (HS + 2);
      wsr[2 + d] = ot;
      if (d == 0) {
        wsr[0] = mx;
        wsr[1] = lt;
      }
    }
  }
  (void)G;
}

template <int HS>
__global__ void __launch_bounds__(HS) combine_kernel(const float* __restrict__ ws, uint16_t* __restrict__ y,
                                                     int n_head, int n_splits) {
  const int h = blockIdx.x, t = blockIdx.y, d = threadIdx.x;
  const float* base = ws + ((size_t)t * n_head + h) * n_splits * (HS + 2);
  float mx = -INFINITY;
  for (int s = 0; s < n_splits; ++s) mx = fmaxf(mx, base[s * (HS + 2)]);
  float lt = 0.0f, ot = 0.0f;
  for (int s = 0; s < n_splits; ++s) {
    const float* r = base + s * (HS + 2);
    if (r[1] == 0.0f) continue;
    const float c = expf(r[0] - mx);
    lt += r[1] * c;
    ot += r[2 + d] * c;
  }
  y[((size_t)t * n_head + h) * HS + d] = f2bf(ot / lt);
}

template <int HS>
static int launch_hs(const void* q, const void* kc, const void* vc, const int64_t* pos, void* y, float* ws, int T,
                     int H, int G, int max_seq, int n_splits, float scale, hipStream_t stream) {
  const int qpk = H / G;
  const int chunk = (max_seq + n_splits - 1) / n_splits;
  const dim3 grid(n_splits, G, T);
#define LGA_ATTN(QPK)                                                                                         \
  attn_kernel<HS, QPK><<<grid, 256, 0, stream>>>((const uint16_t*)q, (const uint16_t*)kc, (const uint16_t*)vc, \
                                                 pos, (uint16_t*)y, ws, H, max_seq, chunk, scale)
  switch (qpk) {
    case 1: LGA_ATTN(1); break;
    case 2: LGA_ATTN(2); break;
    case 4: LGA_ATTN(4); break;
    case 8: LGA_ATTN(8); break;
    default: lga_set_error("lga_attention: q_per_kv must be 1, 2, 4 or 8"); return (int)hipErrorInvalidValue;
  }
#undef LGA_ATTN
  if (n_splits > 1) combine_kernel<HS><<<dim3(H, T), HS, 0, stream>>>(ws, (uint16_t*)y, H, n_splits);
  return 0;
}

}  // namespace lga

extern "C" int lga_attention(const void* q, const void* k_cache, const void* v_cache, const int64_t* input_pos,
                             void* y, float* workspace, int T, int n_head, int n_query_groups, int head_size,
                             int max_seq, int n_splits, float scale, hipStream_t stream) {
  LGA_CHECK_ARG(q && k_cache && v_cache && input_pos && y, "lga_attention: null pointer");
  LGA_CHECK_ARG(T > 0 && n_query_groups > 0 && n_head % n_query_groups == 0, "lga_attention: bad head geometry");
  LGA_CHECK_ARG(n_splits >= 1 && n_splits <= max_seq, "lga_attention: bad n_splits");
  LGA_CHECK_ARG(n_splits == 1 || workspace, "lga_attention: split attention needs a workspace");
  int rc;
  if (head_size == 128)
    rc = lga::launch_hs<128>(q, k_cache, v_cache, input_pos, y, workspace, T, n_head, n_query_groups, max_seq,
                             n_splits, scale, stream);
  else if (head_size == 64)
    rc = lga::launch_hs<64>(q, k_cache, v_cache, input_pos, y, workspace, T, n_head, n_query_groups, max_seq,
                            n_splits, scale, stream);
  else {
    lga_set_error("lga_attention: head_size must be 64 or 128");
    return (int)hipErrorInvalidValue;
  }
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}

extern "C" size_t lga_attention_workspace_bytes(int T, int n_head, int head_size, int n_splits) {
  return n_splits <= 1 ? 0 : (size_t)T * n_head * n_splits * (head_size + 2) * sizeof(float);
}
