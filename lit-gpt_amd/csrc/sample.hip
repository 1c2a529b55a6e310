// Greedy sampling on the device: argmax over the last row of logits (generate/base.py:30-41 with
// temperature == 0; torch.argmax returns the first maximal index, so ties break to the LOWEST index).
// Top-k masking never changes the arg-max (the maximal element is always inside the top-k set), so
// `sample(..., top_k=k, temperature=0)` is this same kernel.
//
// The kernel also performs the decode loop's bookkeeping so the whole step stays on the GPU (and inside
// one HIP graph): it writes the new token id (the `next.to(dtype=x.dtype)` of next_token, base.py:47) into
// the token buffer the next step's embedding reads, and advances input_pos (`input_pos.add_(1)`, base.py:92).
#include "common.h"

namespace lga {

// torch.argmax semantics: NaN compares greater than every number; among equals the lowest index wins
__device__ __forceinline__ bool better(float v, int i, float bv, int bi) {
  const bool vn = v != v, bn = bv != bv;
  if (vn || bn) return vn && (!bn || i < bi);
  return (v > bv) || (v == bv && i < bi);
}

__device__ __forceinline__ void take(float v, int i, float& bv, int& bi) {
  const bool t = better(v, i, bv, bi);
  bv = t ? v : bv;
  bi = t ? i : bi;
}

// One workgroup; every lane issues all of its 16-B loads (8 logits each, up to kVec per lane per pass) before
// comparing, so a 32000-entry vocabulary costs one memory round trip instead of one per element.
constexpr int kVec = 8;

// EMB: the same workgroup then gathers row `token` of the embedding table into emb_out — the next decode step's
// transformer.wte(idx) (lit_gpt/model.py:515), so that step needs no embedding launch of its own.
template <bool VEC, bool EMB = false>
__global__ void __launch_bounds__(1024) argmax_kernel(const uint16_t* __restrict__ logits, int n,
                                                      int64_t* __restrict__ out_idx, int32_t* __restrict__ token_out,
                                                      int64_t* __restrict__ pos_inout,
                                                      const uint16_t* __restrict__ table = nullptr, int C = 0,
                                                      int V = 0, uint16_t* __restrict__ emb_out = nullptr) {
  float bv = -INFINITY;
  int bi = 0x7FFFFFFF;
  int done = 0;
  // the position is read before the logits (in-order vmcnt: its wait never holds the logit loads back), so the
  // bookkeeping at the end is a store instead of a dependent load round trip
  const int64_t p0 = (pos_inout && threadIdx.x == 0) ? *pos_inout : 0;
  if (VEC) {
    const int nvec = n / 8;
    const uint4* lv = (const uint4*)logits;
    for (int base = 0; base < nvec; base += 1024 * kVec) {
      uint4 r[kVec];
#pragma unroll
      for (int u = 0; u < kVec; ++u) r[u] = lv[min(base + u * 1024 + (int)threadIdx.x, nvec - 1)];
#pragma unroll
      for (int u = 0; u < kVec; ++u) {
        const int vi = base + u * 1024 + threadIdx.x;
        const uint32_t d[4] = {r[u].x, r[u].y, r[u].z, r[u].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (vi < nvec) {  // clamped duplicate vectors are skipped (the loads above stay unconditional)
            take(bflo(d[e]), vi * 8 + 2 * e, bv, bi);
            take(bfhi(d[e]), vi * 8 + 2 * e + 1, bv, bi);
          }
        }
      }
    }
    done = nvec * 8;
  }
  for (int i = done + threadIdx.x; i < n; i += blockDim.x) take(bf2f(logits[i]), i, bv, bi);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(bv, off);
    const int oi = __shfl_xor(bi, off);
    take(ov, oi, bv, bi);
  }
  __shared__ float sv[16];
  __shared__ int si[16];
  __shared__ int s_tok;
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sv[wave] = bv;
    si[wave] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = blockDim.x >> 6;
    for (int w = 1; w < nw; ++w) take(sv[w], si[w], bv, bi);
    if (bi >= n) bi = 0;
    if (out_idx) *out_idx = bi;
    if (token_out) *token_out = bi;
    if (pos_inout) *pos_inout = p0 + 1;
    s_tok = bi;
  }
  if (EMB) {
    __syncthreads();
    const long id = min(max(s_tok, 0), V - 1);  // as lga_embedding: the gather stays in bounds
    const uint4* src = (const uint4*)(table + (size_t)id * C);
    for (int i = threadIdx.x; i < C / 8; i += blockDim.x) ((uint4*)emb_out)[i] = src[i];
  }
}

// fp32 logits (the reference's --precision 32-true, lit_gpt/fp32 path): same selection, one workgroup
__global__ void __launch_bounds__(1024) argmax_f32_kernel(const float* __restrict__ logits, int n,
                                                          int64_t* __restrict__ out_idx, int32_t* __restrict__ token_out,
                                                          int64_t* __restrict__ pos_inout) {
  float bv = -INFINITY;
  int bi = 0x7FFFFFFF;
  for (int i = threadIdx.x; i < n; i += blockDim.x) take(logits[i], i, bv, bi);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(bv, off);
    const int oi = __shfl_xor(bi, off);
    take(ov, oi, bv, bi);
  }
  __shared__ float sv[16];
  __shared__ int si[16];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sv[wave] = bv;
    si[wave] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) take(sv[w], si[w], bv, bi);
    if (bi >= n) bi = 0;
    if (out_idx) *out_idx = bi;
    if (token_out) *token_out = bi;
    if (pos_inout) *pos_inout += 1;
  }
}

// ---- temperature > 0: top-k + softmax + multinomial on the device (generate/base.py:30-41) -----------------------
// The reference's default invocation (generate/base.py:102-103: top_k 200, temperature 0.8) as ONE launch inside the
// decode graph:
//   v, i = torch.topk(logits, k); logits = full(-inf).scatter(i, v)      -> the kept set, in index order
//   probs = softmax(logits / temperature) in the logits' dtype (bf16)     -> p = bf16(exp(x - max) / sum), x = bf16(v / T)
//   multinomial(probs, 1)                                                 -> first index whose normalised running sum
//                                                                            reaches a uniform u (torch's CPU inverse CDF)
// Top-k is a two-pass radix select on the bf16 bits (256-bin LDS histograms) of a 16-bit order key (NaN highest, -0 ==
// +0); ties at the k-th value are kept lowest-index first (CUDA torch.topk's order; the CPU one is the heap order of
// std::partial_sort). u comes from `uniform` when given (tests: the reference's test patches the draw,
// tests/test_generate.py:19-46), else from a counter-based hash of (seed, *counter) — the counter lives on the device
// and advances per call, so the launch replays in a HIP graph. Then the argmax kernel's bookkeeping: token, input_pos,
// the next step's embedding row.
__device__ __forceinline__ unsigned order_key(uint16_t b) {
  if ((b & 0x7F80u) == 0x7F80u && (b & 0x7Fu)) return 0xFFFFu;  // NaN: above everything
  if (b == 0x8000u) b = 0;                                      // -0 == +0
  return (b & 0x8000u) ? (~(unsigned)b & 0xFFFFu) : ((unsigned)b | 0x8000u);
}
__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {  // splitmix64 finaliser
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

#ifdef LGA_SAMPLE_TRACE  // lab builds only: phase timestamps of the sampler (100 MHz clock)
__device__ unsigned long long g_sample_trace[16];
#define LGA_STRACE(i)                                                   \
  do {                                                                  \
    if (threadIdx.x == 0) g_sample_trace[(i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define LGA_STRACE(i) \
  do {                \
  } while (0)
#endif

constexpr int kMaxTopK = 1024;

__device__ __forceinline__ unsigned wave_max_u(unsigned v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (unsigned)__shfl_xor((int)v, o));
  return v;
}
__device__ __forceinline__ unsigned wave_incl_scan(unsigned v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned u = (unsigned)__shfl_up((int)v, o);
    if (lane >= o) v += u;
  }
  return v;
}

// One workgroup of 1024 threads; thread t owns logits [t EPT, t EPT + EPT) (index order = thread order, so every
// "in index order" below is a block prefix sum). The logits are staged once in LDS (coalesced), padded with -inf
// (pads sit after every real index, so a tie rule that takes the lowest indices never reaches them: k <= n).
template <int EPT>
__global__ void __launch_bounds__(1024) topk_sample_kernel(
    const uint16_t* __restrict__ logits, int n, int k, float temperature, const float* __restrict__ uniform,
    unsigned long long seed, unsigned long long* __restrict__ counter, int64_t* __restrict__ out_idx,
    int32_t* __restrict__ token_out, int64_t* __restrict__ pos_inout, const uint16_t* __restrict__ table, int C,
    int V, uint16_t* __restrict__ emb_out, int32_t* __restrict__ kept_out, uint16_t* __restrict__ probs_out) {
  constexpr int NT = 1024, NW = 16;
  static_assert(EPT % 8 == 0, "16-B LDS reads");
  __shared__ __attribute__((aligned(16))) uint16_t sx[NT * EPT];
  __shared__ __attribute__((aligned(16))) float kval[kMaxTopK];
  __shared__ __attribute__((aligned(16))) float kcum[kMaxTopK];
  __shared__ int kidx[kMaxTopK];
  __shared__ unsigned hist[NW][256];  // one histogram per wave: 16x fewer atomics on one address
  __shared__ unsigned wsum[NW], wsum2[NW], wmax_s[NW];
  __shared__ float red[NW], red2[NW];
  __shared__ unsigned s_sel, s_before, s_found;
  __shared__ float s_tot, s_u;
  __shared__ int s_tok;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  k = min(k, n);
  float u0 = 0.0f;  // thread 0: the draw's uniform, fetched now so its global round trip overlaps the selection
  if (t == 0) {
    if (uniform) {
      u0 = *uniform;
    } else {
      const unsigned long long cn = *counter;
      *counter = cn + 1;
      u0 = ((float)(mix64(seed ^ (cn * 0xD1B54A32D192ED03ull)) >> 41) + 0.5f) * 0x1.0p-23f;  // exact, in (0, 1)
    }
  }
  // stage the logits (pairs of bf16 per load when the row is 4-B aligned), -inf past n; clear the first histogram
  if (((uintptr_t)logits & 3) == 0) {
    for (int i2 = t; i2 < NT * EPT / 2; i2 += NT) {
      const int i = 2 * i2;
      uint32_t v = 0xFF80FF80u;
      if (i + 1 < n) v = ((const uint32_t*)logits)[i2];
      else if (i < n) v = (uint32_t)logits[i] | 0xFF800000u;
      ((uint32_t*)sx)[i2] = v;
    }
  } else {
    for (int i = t; i < NT * EPT; i += NT) sx[i] = i < n ? logits[i] : (uint16_t)0xFF80u;
  }
  for (int i = t; i < NW * 256; i += NT) (&hist[0][0])[i] = 0;
  if (t == 0) s_found = 0;
  __syncthreads();
  LGA_STRACE(0);
  // this thread's order keys, two 16-bit keys per register (element 2j low, 2j+1 high); at 64 per thread they
  // would not fit beside the rest (1024 threads: 128 VGPRs), so that form reads them from the LDS copy instead
  constexpr bool REG = EPT <= 32;
  uint32_t key2[REG ? EPT / 2 : 1];
  if constexpr (REG) {
    const uint4* src = (const uint4*)(sx + t * EPT);
#pragma unroll
    for (int c = 0; c < EPT / 8; ++c) {
      const uint4 v = src[c];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int h = 0; h < 4; ++h)
        key2[4 * c + h] = order_key((uint16_t)(w[h] & 0xFFFFu)) | (order_key((uint16_t)(w[h] >> 16)) << 16);
    }
  }
  auto key = [&](int e) -> unsigned {
    if constexpr (REG) return (key2[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
    else return order_key(sx[t * EPT + e]);
  };
  // one selection pass: a 256-bin histogram of digit d (d ascending = key descending) over the keys `digit` maps
  // into [0, 256), then the bin where the running count from d = 0 first reaches `need` (s_sel) and the count
  // before it (s_before); s_found stays 0 when the binned keys number fewer than `need`. `clear`: zero the
  // histogram first (the first pass finds it cleared by the staging phase)
  auto select = [&](auto digit, unsigned need, bool clear) {
    if (clear) {
      for (int i = t; i < NW * 256; i += NT) (&hist[0][0])[i] = 0;
      __syncthreads();
    }
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const unsigned d = digit(key(e));
      if (d < 256u) atomicAdd(&hist[wave][d], 1u);
    }
    __syncthreads();
    unsigned c = 0;
    if (t < 256)
#pragma unroll
      for (int w = 0; w < NW; ++w) c += hist[w][t];
    const unsigned inc = wave_incl_scan(c, lane);
    if (lane == 63 && wave < 4) wsum[wave] = inc;
    __syncthreads();
    if (t < 256) {
      unsigned pre = inc;
      for (int w = 0; w < wave; ++w) pre += wsum[w];
      if (pre >= need && pre - c < need) {
        s_sel = t;
        s_before = pre - c;
        s_found = 1;
      }
    }
    __syncthreads();
  };
  // ---- the k-th largest key. First the 256 keys just below the maximum (one pass, atomics only for the keys near
  // the top: logits are dense around their mean, and the top-k of a vocabulary usually sits within two binades of
  // the max); otherwise an MSD radix select on the high byte, then the low byte. ----
  unsigned kmax;
  {
    unsigned m = 0;
    if constexpr (REG) {  // two keys per v_pk_max_u16
      typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
      u16x2 mm = __builtin_bit_cast(u16x2, key2[0]);
#pragma unroll
      for (int j = 1; j < EPT / 2; ++j) mm = __builtin_elementwise_max(mm, __builtin_bit_cast(u16x2, key2[j]));
      m = max((unsigned)mm[0], (unsigned)mm[1]);
    } else {
#pragma unroll
      for (int e = 0; e < EPT; ++e) m = max(m, key(e));
    }
    m = wave_max_u(m);
    if (lane == 0) wmax_s[wave] = m;
    __syncthreads();
    kmax = wmax_s[0];
    for (int w = 1; w < NW; ++w) kmax = max(kmax, wmax_s[w]);
  }
  LGA_STRACE(1);
  unsigned kth, gt;
  select([&](unsigned kk) { return kmax - kk; }, (unsigned)k, false);
  if (s_found) {
    kth = kmax - s_sel;
    gt = s_before;
  } else {
    select([&](unsigned kk) { return 255u - (kk >> 8); }, (unsigned)k, true);
    const unsigned hi = 255u - s_sel, above = s_before;
    select([&](unsigned kk) { return (kk >> 8) == hi ? 255u - (kk & 255u) : 256u; }, (unsigned)k - above, true);
    kth = (hi << 8) | (255u - s_sel);
    gt = above + s_before;
  }
  LGA_STRACE(2);
  // ---- the kept set in index order: every key above the k-th, then ties lowest index first. One block scan of
  // (ties, above): before thread t sit above_before keys above the k-th and min(tie_before, need) taken ties ----
  const unsigned need = (unsigned)k - gt;
  unsigned ties = 0, above = 0;
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    ties += key(e) == kth;
    above += key(e) > kth;
  }
  unsigned tie_before, above_before;
  {
    const unsigned ti = wave_incl_scan(ties, lane), ai = wave_incl_scan(above, lane);
    if (lane == 63) {
      wsum[wave] = ti;
      wsum2[wave] = ai;
    }
    __syncthreads();
    unsigned tb = 0, ab = 0;
    for (int w = 0; w < wave; ++w) {
      tb += wsum[w];
      ab += wsum2[w];
    }
    tie_before = tb + ti - ties;
    above_before = ab + ai - above;
  }
  unsigned pos = above_before + min(tie_before, need);
  unsigned tie_seen = tie_before;
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const unsigned ke = key(e);
    bool keep = ke > kth;
    if (ke == kth) keep = tie_seen++ < need;
    if (keep) {
      kidx[pos] = t * EPT + e;
      kval[pos] = bf2f(sx[t * EPT + e]);
      ++pos;
    }
  }
  __syncthreads();
  LGA_STRACE(3);
  // ---- softmax over the kept logits / temperature, in bf16 like the reference's bf16 tensor ops ----
  const bool mine = t < k;
  const float x = mine ? round_bf(kval[t] / temperature) : -INFINITY;
  float m = wave_max(x);
  if (lane == 0) red[wave] = m;
  __syncthreads();
  m = red[0];
  for (int w = 1; w < NW; ++w) m = fmaxf(m, red[w]);
  const float e = mine ? expf(x - m) : 0.0f;
  float sum = wave_sum(e);
  if (lane == 0) red2[wave] = sum;
  __syncthreads();
  sum = 0.0f;
  for (int w = 0; w < NW; ++w) sum += red2[w];
  const float p = mine ? round_bf(e / sum) : 0.0f;
  if (t < ((k + 15) & ~15)) kval[t] = p;  // zero past k: the sequential sum below reads whole groups of 16
  if (mine && kept_out) kept_out[t] = kidx[t];
  if (mine && probs_out) probs_out[t] = f2bf(p);
  __syncthreads();
  LGA_STRACE(4);
  // ---- multinomial: torch's CPU inverse CDF — the running fp32 sum in index order (one thread: the order is the
  // specification), normalised, the first index reaching u (every kept thread tests its own step) ----
  if (t == 0) {
    // probabilities past k are zero (kval padded below), so whole float4 groups need no bounds test: the running
    // sum stays put over them
    float c = 0.0f;
    for (int j = 0; j < k; j += 16) {
      float4 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = *(const float4*)&kval[j + 4 * q];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4 o;
        o.x = c += v[q].x;
        o.y = c += v[q].y;
        o.z = c += v[q].z;
        o.w = c += v[q].w;
        *(float4*)&kcum[j + 4 * q] = o;
      }
    }
    s_tot = c;
    s_u = u0;
    s_tok = kidx[k - 1];
  }
  __syncthreads();
  if (mine) {
    const float tot = s_tot, u = s_u;
    const float cdf = kcum[t] / tot, prev = t ? kcum[t - 1] / tot : -1.0f;
    if (cdf >= u && prev < u) s_tok = kidx[t];
  }
  __syncthreads();
  LGA_STRACE(5);
  const int pick = s_tok;
  if (t == 0) {
    if (out_idx) *out_idx = pick;
    if (token_out) *token_out = pick;
    if (pos_inout) *pos_inout += 1;
  }
  if (emb_out) {
    const long id = min(max(pick, 0), V - 1);
    const uint4* src = (const uint4*)(table + (size_t)id * C);
    for (int i = t; i < C / 8; i += NT) ((uint4*)emb_out)[i] = src[i];
  }
}

}  // namespace lga

int lga::preload_sample() {
  return lga::preload(lga::argmax_kernel<true>) + lga::preload(lga::argmax_kernel<false>) +
         lga::preload(lga::topk_sample_kernel<16>) + lga::preload(lga::topk_sample_kernel<32>) +
         lga::preload(lga::topk_sample_kernel<64>);
}

extern "C" int lga_argmax(const void* logits, int n, int64_t* out_idx, int32_t* token_out, int64_t* pos_inout,
                          hipStream_t stream) {
  LGA_CHECK_ARG(logits && n > 0, "lga_argmax: bad arguments");
  if (((uintptr_t)logits & 15) == 0 && n >= 8)
    lga::argmax_kernel<true><<<1, 1024, 0, stream>>>((const uint16_t*)logits, n, out_idx, token_out, pos_inout);
  else
    lga::argmax_kernel<false><<<1, 1024, 0, stream>>>((const uint16_t*)logits, n, out_idx, token_out, pos_inout);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_argmax_embed(const void* logits, int n, int64_t* out_idx, int32_t* token_out, int64_t* pos_inout,
                                const void* table, int n_embd, int vocab, void* emb_out, hipStream_t stream) {
  LGA_CHECK_ARG(logits && n > 0 && table && emb_out && n_embd > 0 && n_embd % 8 == 0 && vocab > 0,
                "lga_argmax_embed: bad arguments");
  LGA_CHECK_ARG(((uintptr_t)table & 15) == 0 && ((uintptr_t)emb_out & 15) == 0,
                "lga_argmax_embed: table and emb_out must be 16-B aligned");
  if (((uintptr_t)logits & 15) == 0 && n >= 8)
    lga::argmax_kernel<true, true><<<1, 1024, 0, stream>>>((const uint16_t*)logits, n, out_idx, token_out, pos_inout,
                                                           (const uint16_t*)table, n_embd, vocab, (uint16_t*)emb_out);
  else
    lga::argmax_kernel<false, true><<<1, 1024, 0, stream>>>((const uint16_t*)logits, n, out_idx, token_out, pos_inout,
                                                            (const uint16_t*)table, n_embd, vocab, (uint16_t*)emb_out);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_argmax_f32(const float* logits, int n, int64_t* out_idx, int32_t* token_out, int64_t* pos_inout,
                              hipStream_t stream) {
  LGA_CHECK_ARG(logits && n > 0, "lga_argmax_f32: bad arguments");
  lga::argmax_f32_kernel<<<1, 1024, 0, stream>>>(logits, n, out_idx, token_out, pos_inout);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_sample_topk(const void* logits, int n, int top_k, float temperature, const float* uniform,
                               unsigned long long seed, unsigned long long* counter, int64_t* out_idx,
                               int32_t* token_out, int64_t* pos_inout, const void* table, int n_embd, int vocab,
                               void* emb_out, int32_t* kept_out, void* probs_out, hipStream_t stream) {
  LGA_CHECK_ARG(logits && n > 0 && n <= 1024 * 64, "lga_sample_topk: needs 0 < n <= 65536 logits");
  LGA_CHECK_ARG(top_k >= 1 && top_k <= lga::kMaxTopK, "lga_sample_topk: top_k must be in [1, 1024]");
  LGA_CHECK_ARG(temperature > 0.0f, "lga_sample_topk: temperature must be > 0 (0 is lga_argmax)");
  LGA_CHECK_ARG(uniform || counter, "lga_sample_topk: needs a uniform or an RNG counter");
  LGA_CHECK_ARG(!emb_out || (table && n_embd > 0 && n_embd % 8 == 0 && vocab > 0 && ((uintptr_t)table & 15) == 0 &&
                             ((uintptr_t)emb_out & 15) == 0),
                "lga_sample_topk: the embedding gather needs a 16-B aligned table and emb_out, n_embd % 8 == 0");
#define LGA_TOPK(EPT)                                                                                           \
  lga::topk_sample_kernel<EPT><<<1, 1024, 0, stream>>>((const uint16_t*)logits, n, top_k, temperature, uniform, seed, \
                                                       counter, out_idx, token_out, pos_inout, (const uint16_t*)table,  \
                                                       n_embd, vocab, (uint16_t*)emb_out, kept_out, (uint16_t*)probs_out)
  if (n <= 1024 * 16) LGA_TOPK(16);
  else if (n <= 1024 * 32) LGA_TOPK(32);
  else LGA_TOPK(64);
#undef LGA_TOPK
  LGA_LAUNCH_RETURN();
}

#ifdef LGA_SAMPLE_TRACE
extern "C" int lga_sample_trace(unsigned long long* out) {  // lab: the last launch's phase timestamps
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(lga::g_sample_trace), sizeof(unsigned long long) * 16);
}
#endif
