// Cached causal attention for decode (T = 1, split over the sequence) and prefill (T rows).
//
// Replaces CausalSelfAttention.scaled_dot_product_attention (lit_gpt/model.py:651, :658-665): SDPA of q
// against the full max_seq-long cache under the bool mask row(s) selected by input_pos (model.py:509). The
// mask allows key j for query t iff j <= input_pos[t]; this kernel reads only those keys.
//
// KV cache layout (HBM): k, v = [G][max_seq][hs] bf16 per layer (un-expanded query groups); one key row is
// hs*2 contiguous bytes, read by a "row group" of hs/8 lanes at 16 B per lane.
//
// Work decomposition: grid (splits, G, T); a 256-thread workgroup owns one (split, query group, query row) and
// all q_per_kv heads of that group (GQA/MQA read each K/V row once). The split boundaries are computed in the
// kernel from the live position (chunk = ceil((p+1)/splits)), so every split is busy whatever the context
// length and a captured HIP graph stays valid as p grows. Inside, each row group streams UNR keys per step
// (2*UNR 16-B loads in flight per lane) with an online softmax; row groups merge with shuffles, waves via LDS.
// With splits > 1 every workgroup publishes (m, l, o) write-through (sc1) and bumps a per-(t, group) counter;
// the workgroup that arrives last merges the splits and writes the bf16 output (flash-decoding combine inside
// the same launch; MI355X_MICROARCH.md "Valid forms" row 1), then re-arms the counter for the next launch.
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

template <int HS, int QPK, int UNR>
__global__ void __launch_bounds__(256) attn_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                                   const uint16_t* __restrict__ vc,
                                                   const int64_t* __restrict__ input_pos, uint16_t* __restrict__ y,
                                                   float* __restrict__ ws, unsigned* __restrict__ cnt, int n_head,
                                                   int max_seq, float scale) {
  constexpr int LPR = HS / 8;    // lanes per key row
  constexpr int RGW = 64 / LPR;  // row groups per wave
  constexpr int RG = 4 * RGW;    // row groups per workgroup
  const int split = blockIdx.x, g = blockIdx.y, t = blockIdx.z;
  const int n_splits = gridDim.x, G = gridDim.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rg = wave * RGW + lane / LPR;
  const int sub = lane % LPR;
  const long p = input_pos[t];
  const int L = (int)min(p + 1, (long)max_seq);  // keys 0..p (never past the cache)
  const int chunk = (L + n_splits - 1) / n_splits;
  const int k_lo = split * chunk;
  const int k_hi = min(k_lo + chunk, L);

  float qf[QPK][8];
#pragma unroll
  for (int h = 0; h < QPK; ++h)
    unpack8(*(const uint4*)(q + ((size_t)t * n_head + (size_t)g * QPK + h) * HS + sub * 8), qf[h]);
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
  for (int j0 = k_lo + rg; j0 < k_hi; j0 += RG * UNR) {
    uint4 kv[UNR], vv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int j = min(j0 + u * RG, k_hi - 1);  // clamped duplicate rows are masked below
      kv[u] = *(const uint4*)(kbase + (size_t)j * HS);
      vv[u] = *(const uint4*)(vbase + (size_t)j * HS);
    }
#pragma unroll
    for (int h = 0; h < QPK; ++h) {
      float s[UNR];
      float mx = m[h];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        float kf[8];
        unpack8(kv[u], kf);
        float d = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) d = fmaf(qf[h][i], kf[i], d);
        const float sd = row_group_sum<LPR>(d) * scale;  // whole row group active: DPP stays inside it
        s[u] = (j0 + u * RG < k_hi) ? sd : -INFINITY;
        mx = fmaxf(mx, s[u]);
      }
      const float c = expf(m[h] - mx);  // m = -inf (first step) -> 0
      l[h] *= c;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[h][i] *= c;
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const float e = expf(s[u] - mx);  // masked keys: exp(-inf) = 0
        l[h] += e;
        float vf[8];
        unpack8(vv[u], vf);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[h][i] = fmaf(e, vf[i], o[h][i]);
      }
      m[h] = mx;
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
      for (int i = 0; i < 8; ++i) o[h][i] = o[h][i] * ca + __shfl_xor(o[h][i], off) * cb;
      m[h] = mn;
    }
  }
  __shared__ float sm[4][QPK], sl[4][QPK];
  __shared__ float so[4][QPK][HS];
  __shared__ unsigned s_last;
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
  const size_t row0 = (size_t)t * n_head + (size_t)g * QPK;  // first head row of this group
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
    if (n_splits == 1) {
      y[(row0 + h) * HS + d] = f2bf(ot / lt);
    } else {
      float* wsr = ws + ((row0 + h) * n_splits + split) * (HS + 2);
      st_sc1(wsr + 2 + d, ot);
      if (d == 0) {
        st_sc1(wsr, mx);
        st_sc1(wsr + 1, lt);
      }
    }
  }
  if (n_splits == 1) return;
  // ---- publish, then the last-arriving split of this (t, group) merges all splits ----
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(cnt + (size_t)t * G + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_last != (unsigned)(n_splits - 1)) return;
  float* wm = &so[0][0][0];  // reuse LDS: [QPK][n_splits] weights (n_splits <= 4*HS)
  for (int it = threadIdx.x; it < QPK * n_splits; it += 256) {
    const int h = it / n_splits, s = it % n_splits;
    wm[it] = ld_sc1(ws + ((row0 + h) * n_splits + s) * (HS + 2));
  }
  __syncthreads();
  for (int it = threadIdx.x; it < QPK * HS; it += 256) {
    const int h = it / HS, d = it % HS;
    float mx = -INFINITY;
    for (int s = 0; s < n_splits; ++s) mx = fmaxf(mx, wm[h * n_splits + s]);
    float lt = 0.0f, ot = 0.0f;
    const float* base = ws + (row0 + h) * n_splits * (HS + 2);
    // no data-dependent branch: empty splits carry m = -inf (weight exp(-inf) = 0), l = 0, o = 0, so every
    // load is independent and the compiler keeps them all in flight
#pragma unroll 8
    for (int s = 0; s < n_splits; ++s) {
      const float c = expf(wm[h * n_splits + s] - mx);
      lt = fmaf(ld_sc1(base + s * (HS + 2) + 1), c, lt);
      ot = fmaf(ld_sc1(base + s * (HS + 2) + 2 + d), c, ot);
    }
    y[(row0 + h) * HS + d] = f2bf(ot / lt);
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt + (size_t)t * G + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int HS>
static int launch_hs(const void* q, const void* kc, const void* vc, const int64_t* pos, void* y, float* ws,
                     unsigned* cnt, int T, int H, int G, int max_seq, int n_splits, float scale, hipStream_t stream) {
  const dim3 grid(n_splits, G, T);
#define LGA_ATTN(QPK, UNR)                                                                                    \
  attn_kernel<HS, QPK, UNR><<<grid, 256, 0, stream>>>((const uint16_t*)q, (const uint16_t*)kc,                 \
                                                      (const uint16_t*)vc, pos, (uint16_t*)y, ws, cnt, H, max_seq, \
                                                      scale)
  switch (H / G) {
    case 1: LGA_ATTN(1, 4); break;
    case 2: LGA_ATTN(2, 4); break;
    case 4: LGA_ATTN(4, 2); break;
    case 8: LGA_ATTN(8, 2); break;
    default: lga_set_error("lga_attention: q_per_kv must be 1, 2, 4 or 8"); return (int)hipErrorInvalidValue;
  }
#undef LGA_ATTN
  return 0;
}

}  // namespace lga

extern "C" int lga_attention(const void* q, const void* k_cache, const void* v_cache, const int64_t* input_pos,
                             void* y, float* workspace, unsigned* counters, int T, int n_head, int n_query_groups,
                             int head_size, int max_seq, int n_splits, float scale, hipStream_t stream) {
  LGA_CHECK_ARG(q && k_cache && v_cache && input_pos && y, "lga_attention: null pointer");
  LGA_CHECK_ARG(T > 0 && n_query_groups > 0 && n_head % n_query_groups == 0, "lga_attention: bad head geometry");
  LGA_CHECK_ARG(n_splits >= 1 && n_splits <= 512, "lga_attention: n_splits must be in [1, 512]");
  LGA_CHECK_ARG(n_splits == 1 || (workspace && counters), "lga_attention: split attention needs workspace + counters");
  LGA_CHECK_ARG(n_splits * (n_head / n_query_groups) <= 4 * head_size, "lga_attention: too many splits for the LDS merge");
  int rc;
  if (head_size == 128)
    rc = lga::launch_hs<128>(q, k_cache, v_cache, input_pos, y, workspace, counters, T, n_head, n_query_groups,
                             max_seq, n_splits, scale, stream);
  else if (head_size == 64)
    rc = lga::launch_hs<64>(q, k_cache, v_cache, input_pos, y, workspace, counters, T, n_head, n_query_groups,
                            max_seq, n_splits, scale, stream);
  else {
    lga_set_error("lga_attention: head_size must be 64 or 128");
    return (int)hipErrorInvalidValue;
  }
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}

// fp32 partials (T * H * n_splits * (hs + 2)); the counters (T * G uint32) must be zeroed once at allocation
extern "C" size_t lga_attention_workspace_bytes(int T, int n_head, int head_size, int n_splits) {
  return n_splits <= 1 ? 0 : (size_t)T * n_head * n_splits * (head_size + 2) * sizeof(float);
}
