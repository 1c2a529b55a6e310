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
    if (pos_inout) *pos_inout += 1;
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

}  // namespace lga

int lga::preload_sample() {
  return lga::preload(lga::argmax_kernel<true>) + lga::preload(lga::argmax_kernel<false>);
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
