// Sparse-MoE routing and combine for LLaMAMoE (Mixtral), lit_gpt/model.py:727-743:
//   router = gate(x); probs, indices = topk(router, k); probs = softmax(probs, fp32).to(bf16)
//   y = 0; for expert e ascending: y[tok] += probs[tok, slot] * expert_e(x[tok])      (bf16 arithmetic)
// The expert GEMVs themselves are lga_q4_gemv(_swiglu)_experts (gemv.hip): slot s of a token streams the weights of
// expert ids[s] only, so a decode step reads k of the E experts and never leaves the device (no host-side
// torch.where as in the reference loop; the step stays inside one HIP graph).
#include <cstdlib>

#include "common.h"
#include "gemv_body.h"

namespace lga {

// ATen's CPU topk comparator for largest=True (aten/src/ATen/native/cpu/SortingKernel.cpp): NaN ranks first
struct KV {
  float v;
  int i;
};
__device__ __forceinline__ bool before(const KV& a, const KV& b) {
  return (a.v != a.v && !(b.v != b.v)) || (a.v > b.v);
}
__device__ __forceinline__ void swp(KV* q, int a, int b) {
  const KV t = q[a];
  q[a] = q[b];
  q[b] = t;
}

// Tie order of torch.topk on the CPU = libstdc++ std::nth_element(begin, begin + k - 1, end) (introselect:
// median-of-3 pivot moved to the front, unguarded Hoare partition while the range is longer than 3, then
// insertion sort) followed by std::sort(begin, begin + k - 1) (insertion sort below 17 elements). For n <= 8 the
// introselect depth limit 2*floor(log2 n) is never reached, so the heap-select fallback is not needed.
// Mirrors the restatement checked against torch.topk in tests/test_host_logic.py.
template <int NMAX>
__device__ void topk_order(KV* q, int n, int k) {
  int first = 0, last = n;
  const int nth = k - 1;
  while (last - first > 3) {
    const int mid = first + (last - first) / 2;
    const int a = first + 1, b = mid, c = last - 1;
    int s;
    if (before(q[a], q[b])) s = before(q[b], q[c]) ? b : (before(q[a], q[c]) ? c : a);
    else s = before(q[a], q[c]) ? a : (before(q[b], q[c]) ? c : b);
    swp(q, first, s);
    int lo = first + 1, hi = last;
    while (true) {
      while (before(q[lo], q[first])) ++lo;
      --hi;
      while (before(q[first], q[hi])) --hi;
      if (!(lo < hi)) break;
      swp(q, lo, hi);
      ++lo;
    }
    if (lo <= nth) first = lo;
    else last = lo;
  }
  auto insertion = [&](int f, int l) {
    for (int i = f + 1; i < l; ++i) {
      const KV v = q[i];
      if (before(v, q[f])) {
        for (int j = i; j > f; --j) q[j] = q[j - 1];
        q[f] = v;
      } else {
        int j = i;
        while (before(v, q[j - 1])) {
          q[j] = q[j - 1];
          --j;
        }
        q[j] = v;
      }
    }
  };
  insertion(first, last);
  insertion(0, k - 1);
}

// top-k of one row of E router logits, fp32 softmax over the k values (ATen's lastdim softmax: exp(v - max), sum,
// multiply by the reciprocal), bf16 probabilities; `row` is global memory or LDS (generic pointer). The selection
// works on q[8] in LDS: its data-dependent indexing would put a register array in scratch (a memory round trip per
// access); each exp is evaluated twice (same input, same bits) instead of being kept in such an array.
__device__ void route_row(const uint16_t* row, int E, int k, int32_t* __restrict__ ids, uint16_t* __restrict__ probs,
                          KV* q) {
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] = {i < E ? bf2f(row[i]) : -INFINITY, i};
  topk_order<8>(q, E, k);
  float mx = q[0].v;
  for (int s = 1; s < k; ++s) mx = fmaxf(mx, q[s].v);
  float sum = 0.0f;
  for (int s = 0; s < k; ++s) sum += expf(q[s].v - mx);
  const float r = 1.0f / sum;
  for (int s = 0; s < k; ++s) {
    ids[s] = q[s].i;
    probs[s] = f2bf(expf(q[s].v - mx) * r);
  }
}

// one thread per token row
__global__ void __launch_bounds__(64) moe_route_kernel(const uint16_t* __restrict__ logits, int T, int E, int k,
                                                       int32_t* __restrict__ ids, uint16_t* __restrict__ probs) {
  __shared__ KV sq[64][8];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  route_row(logits + (size_t)t * E, E, k, ids + (size_t)t * k, probs + (size_t)t * k, sq[threadIdx.x]);
}

// Decode (one token): the router gate GEMV and the routing in ONE single-workgroup launch. The E <= 8 gate rows are
// the decode GEMV body's (lga_q4_gemv's arithmetic for N <= 64, fused RMSNorm included: 4 waves x 2 rows, rows past E
// repeat row E-1), left in LDS as the bf16 logits lga_q4_gemv would store; thread 0 then routes them exactly as
// moe_route_kernel does — the pair lga_q4_gemv + lga_moe_route bit for bit, one launch ramp instead of two.
template <int CPT, int FMT, bool NORM>
__global__ void __launch_bounds__(256) moe_gate_route_kernel(GemvArgs a, int k, int32_t* __restrict__ ids,
                                                             uint16_t* __restrict__ probs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ KV sq[8];
  gemv_q4_body<2, CPT, FMT, false, NORM, false, 4, true>(a, 0, smem);
  __syncthreads();
  if (threadIdx.x == 0) route_row(gemv_out_lds(smem, a.K), a.N, k, ids, probs, sq);
}

// Decode (one token, k = 2, no tensor parallelism): the routed proj GEMVs of both slots — lga_q4_gemv_experts's kernel
// body for the shape, grid (row blocks, 2 slots), rows to LDS — and lga_moe_combine (+ the Block residual) in ONE
// launch, the combine done by the second-arriving workgroup of each row block: the first stores its bf16 rows
// write-through and arrives (MI355X_MICROARCH.md "Valid forms" row 1: sc1 16-B stores, drain, barrier, one agent-scope
// add); the second reads them with sc1 loads, adds both experts in ascending id order with lga_moe_combine's rounding
// points and the residual, and re-arms the block's counter. Bit-identical to lga_q4_gemv_experts + lga_moe_combine.
constexpr int kPairStride = 64;  // per-row-block counters 256 B apart
template <int RPR, int CPT, int FMT, int NW = 4>
__global__ void __launch_bounds__(NW * 64) moe_down_pair_kernel(GemvArgs a, const uint16_t* __restrict__ residual,
                                                            uint16_t* __restrict__ y, uint16_t* __restrict__ scratch,
                                                            unsigned* __restrict__ counters) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ unsigned s_ticket;
  constexpr int ROWS = NW * RPR, PIECES = ROWS / 8;  // the workgroup's rows, their 16-B pieces
  const int b = blockIdx.x, slot = blockIdx.y, t = threadIdx.x;
  const int row0 = b * ROWS;
  // everything the combine needs, read up front: both ids (order), both probabilities, this block's residual rows
  const int id0 = a.eidx[0], id1 = a.eidx[1];
  const float p0 = bf2f(a.probs[0]), p1 = bf2f(a.probs[1]);
  uint4 rv = make_uint4(0, 0, 0, 0);
  if (t < PIECES) rv = ((const uint4*)(residual + row0))[t];
  gemv_q4_body<RPR, CPT, FMT, false, false, false, NW, true>(a, b, smem);
  __syncthreads();
  const uint4* mine = (const uint4*)gemv_out_lds(smem, a.K);
  const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc((void*)scratch, (short)0, 2 * a.N * 2, 0x00020000);
  if (t < PIECES)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, mine[t]), srs,
                                           (slot * a.N + row0 + t * 8) * 2, 0, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned* ctr = counters + (size_t)b * kPairStride;
  if (t == 0) s_ticket = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_ticket == 0) return;  // the other slot's workgroup combines
  if (t < PIECES) {
    const u32x4_t ov = __builtin_amdgcn_raw_buffer_load_b128(srs, ((1 - slot) * a.N + row0 + t * 8) * 2, 0, 16);
    const uint4 e_mine = mine[t], e_other = __builtin_bit_cast(uint4, ov);
    const uint4 e0 = slot == 0 ? e_mine : e_other, e1 = slot == 0 ? e_other : e_mine;  // slot 0's, slot 1's rows
    const bool swap = id1 < id0;  // lga_moe_combine's stable order by expert id
    const uint4 ea = swap ? e1 : e0, eb = swap ? e0 : e1;
    const float pa = swap ? p1 : p0, pb = swap ? p0 : p1;
    const uint32_t da[4] = {ea.x, ea.y, ea.z, ea.w}, db[4] = {eb.x, eb.y, eb.z, eb.w};
    const uint32_t dr[4] = {rv.x, rv.y, rv.z, rv.w};
    uint32_t out[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float lo = 0.0f, hi = 0.0f;
      lo = round_bf(lo + round_bf(pa * bflo(da[q])));
      hi = round_bf(hi + round_bf(pa * bfhi(da[q])));
      lo = round_bf(lo + round_bf(pb * bflo(db[q])));
      hi = round_bf(hi + round_bf(pb * bfhi(db[q])));
      out[q] = pack2(bflo(dr[q]) + lo, bfhi(dr[q]) + hi);
    }
    *(uint4*)(y + row0 + t * 8) = make_uint4(out[0], out[1], out[2], out[3]);
  }
  if (t == 0) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // both arrived: re-arm
}

template <int RPR, int CPT, int FMT, int NW = 4>
static void launch_down_pair(const GemvArgs& a, const uint16_t* residual, uint16_t* y, uint16_t* scratch,
                             unsigned* counters, hipStream_t stream) {
  const dim3 grid(a.N / (NW * RPR), 2);
  moe_down_pair_kernel<RPR, CPT, FMT, NW><<<grid, NW * 64, gemv_lds_bytes(a.K), stream>>>(a, residual, y, scratch,
                                                                                           counters);
}

// gemv.hip dispatch's one-shot tile for an expert GEMV of this K (variant 0)
template <int FMT>
static int dispatch_down_pair(const GemvArgs& a, const uint16_t* residual, uint16_t* y, uint16_t* scratch,
                              unsigned* counters, hipStream_t stream) {
  switch ((a.K / 32 + 63) / 64) {
    case 1: launch_down_pair<4, 1, FMT>(a, residual, y, scratch, counters, stream); break;
    case 2: launch_down_pair<4, 2, FMT>(a, residual, y, scratch, counters, stream); break;
    case 3: launch_down_pair<4, 3, FMT>(a, residual, y, scratch, counters, stream); break;
    case 4: launch_down_pair<2, 4, FMT>(a, residual, y, scratch, counters, stream); break;
    case 5:
    case 6: launch_down_pair<2, 6, FMT>(a, residual, y, scratch, counters, stream); break;
    // K 14,336 (Mixtral): 8 waves x 2 rows, exactly 7 chunks per lane — 15.5 vs 16.1 us for 4 waves x 4 rows
    // (tools/moe_down_ab.py, round 6); the per-row arithmetic is gemv.hip's case 7 (2 rows per wave), bit for bit
    case 7: launch_down_pair<2, 7, FMT, 8>(a, residual, y, scratch, counters, stream); break;
    case 8: launch_down_pair<2, 8, FMT>(a, residual, y, scratch, counters, stream); break;
    default: launch_down_pair<2, 16, FMT>(a, residual, y, scratch, counters, stream); break;
  }
  return 0;
}

template <int CPT, int FMT>
static void launch_gate_route(const GemvArgs& a, int k, int32_t* ids, uint16_t* probs, hipStream_t stream) {
  const size_t lds = gemv_lds_bytes(a.K);
  if (a.norm_w) moe_gate_route_kernel<CPT, FMT, true><<<1, 256, lds, stream>>>(a, k, ids, probs);
  else moe_gate_route_kernel<CPT, FMT, false><<<1, 256, lds, stream>>>(a, k, ids, probs);
}

template <int FMT>
static int dispatch_gate_route(const GemvArgs& a, int k, int32_t* ids, uint16_t* probs, hipStream_t stream) {
  switch ((a.K / 32 + 63) / 64) {  // chunks per lane: the same template lga_q4_gemv picks for these shapes
    case 1: launch_gate_route<1, FMT>(a, k, ids, probs, stream); break;
    case 2: launch_gate_route<2, FMT>(a, k, ids, probs, stream); break;
    case 3: launch_gate_route<3, FMT>(a, k, ids, probs, stream); break;
    default:
      lga_set_error("lga_moe_gate_route: K must be at most 6144");
      return (int)hipErrorInvalidValue;
  }
  return 0;
}

// y[t] = residual[t] + sum over slots in ascending expert order of bf16(p * E_slot[t]), each add rounded to bf16
// (the reference's `y[token_idx] += probs * expert(x)` loop); 8 channels per thread
__global__ void moe_combine_kernel(const uint16_t* __restrict__ eout, const uint16_t* __restrict__ probs,
                                   const int32_t* __restrict__ ids, const uint16_t* __restrict__ residual,
                                   uint16_t* __restrict__ y, int k, int C) {
  const int t = blockIdx.y;
  const int c8 = blockIdx.x * blockDim.x + threadIdx.x;
  if (c8 * 8 >= C) return;
  int order[8];
  for (int s = 0; s < k; ++s) order[s] = s;
  for (int i = 1; i < k; ++i) {  // stable by expert id
    const int v = order[i];
    int j = i;
    while (j > 0 && ids[(size_t)t * k + order[j - 1]] > ids[(size_t)t * k + v]) {
      order[j] = order[j - 1];
      --j;
    }
    order[j] = v;
  }
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.0f;
  for (int j = 0; j < k; ++j) {
    const int s = order[j];
    const float p = bf2f(probs[(size_t)t * k + s]);
    const uint4 ev = *(const uint4*)(eout + ((size_t)t * k + s) * C + c8 * 8);
    const uint32_t d[4] = {ev.x, ev.y, ev.z, ev.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      acc[2 * q] = round_bf(acc[2 * q] + round_bf(p * bflo(d[q])));
      acc[2 * q + 1] = round_bf(acc[2 * q + 1] + round_bf(p * bfhi(d[q])));
    }
  }
  if (residual) {
    const uint4 rv = *(const uint4*)(residual + (size_t)t * C + c8 * 8);
    const uint32_t d[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      acc[2 * q] = bflo(d[q]) + acc[2 * q];
      acc[2 * q + 1] = bfhi(d[q]) + acc[2 * q + 1];
    }
  }
  *(uint4*)(y + (size_t)t * C + c8 * 8) =
      make_uint4(pack2(acc[0], acc[1]), pack2(acc[2], acc[3]), pack2(acc[4], acc[5]), pack2(acc[6], acc[7]));
}

}  // namespace lga

extern "C" int lga_moe_route(const void* logits, int T, int n_expert, int k, int32_t* expert_ids, void* probs,
                             hipStream_t stream) {
  LGA_CHECK_ARG(logits && expert_ids && probs, "lga_moe_route: null pointer");
  LGA_CHECK_ARG(T > 0 && n_expert > 0 && n_expert <= 8 && k > 0 && k <= n_expert,
                "lga_moe_route: needs 1 <= k <= n_expert <= 8");
  lga::moe_route_kernel<<<(T + 63) / 64, 64, 0, stream>>>((const uint16_t*)logits, T, n_expert, k, expert_ids,
                                                          (uint16_t*)probs);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_moe_gate_route(const void* x, const uint8_t* qweight, const void* scales, const void* norm_weight,
                                  float norm_eps, int n_expert, int K, int group, int fmt, int k, int32_t* expert_ids,
                                  void* probs, hipStream_t stream) {
  LGA_CHECK_ARG(x && qweight && scales && expert_ids && probs, "lga_moe_gate_route: null pointer");
  LGA_CHECK_ARG(n_expert > 0 && n_expert <= 8 && k > 0 && k <= n_expert,
                "lga_moe_gate_route: needs 1 <= k <= n_expert <= 8");
  LGA_CHECK_ARG(K > 0 && K % 32 == 0 && K <= 6144, "lga_moe_gate_route: K must be a multiple of 32, at most 6144");
  LGA_CHECK_ARG(group >= 32 && group % 32 == 0 && K % group == 0, "lga_moe_gate_route: bad group");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1 || fmt == 3, "lga_moe_gate_route: fmt must be 0 (int4-g), 1 (nf4) or 3 (fp4)");
  lga::GemvArgs a{(const uint16_t*)x, qweight, scales, nullptr, nullptr, nullptr, nullptr,
                  (const uint16_t*)norm_weight, nullptr, n_expert, K, group, norm_eps};
  a.cb = lga::codebook_of(fmt);
  const int rc = fmt == 0 ? lga::dispatch_gate_route<0>(a, k, expert_ids, (uint16_t*)probs, stream)
                          : lga::dispatch_gate_route<1>(a, k, expert_ids, (uint16_t*)probs, stream);
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_q4_gemv_experts_pair_supported(int N, int K, int group, int fmt) {
  const int cpt = (K / 32 + 63) / 64;
  return N > 0 && N % 16 == 0 && N / 8 <= 65535 && K > 0 && K % 32 == 0 && cpt <= 16 && group >= 32 &&
         group % 32 == 0 && K % group == 0 && (fmt == 0 || fmt == 1 || fmt == 3) && N < 24000;
}

extern "C" size_t lga_q4_gemv_experts_pair_counters(int N) { return (size_t)(N / 8) * lga::kPairStride; }

extern "C" int lga_q4_gemv_experts_pair_combine(const void* x, const uint8_t* qweight, const void* scales,
                                                const int32_t* expert_ids, const void* probs, const void* residual,
                                                int n_expert, long long w_stride, long long s_stride, void* y,
                                                void* scratch, unsigned* counters, int N, int K, int group, int fmt,
                                                hipStream_t stream) {
  LGA_CHECK_ARG(x && qweight && scales && expert_ids && probs && residual && y && scratch && counters,
                "lga_q4_gemv_experts_pair_combine: null pointer");
  LGA_CHECK_ARG(lga_q4_gemv_experts_pair_supported(N, K, group, fmt),
                "lga_q4_gemv_experts_pair_combine: geometry not covered (lga_q4_gemv_experts_pair_supported)");
  LGA_CHECK_ARG(n_expert > 0 && w_stride >= (long long)N * K / 2 && s_stride > 0,
                "lga_q4_gemv_experts_pair_combine: bad expert geometry");
  lga::GemvArgs a{(const uint16_t*)x, qweight, scales, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, N, K, group,
                  0.0f, expert_ids, w_stride, s_stride, K, n_expert, 2};
  a.cb = lga::codebook_of(fmt);
  a.probs = (const uint16_t*)probs;
  const int rc = lga::kernel_fmt(fmt) == 0
                     ? lga::dispatch_down_pair<0>(a, (const uint16_t*)residual, (uint16_t*)y, (uint16_t*)scratch,
                                                  counters, stream)
                     : lga::dispatch_down_pair<1>(a, (const uint16_t*)residual, (uint16_t*)y, (uint16_t*)scratch,
                                                  counters, stream);
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_moe_combine(const void* expert_out, const void* probs, const int32_t* expert_ids,
                               const void* residual, void* y, int T, int k, int C, hipStream_t stream) {
  LGA_CHECK_ARG(expert_out && probs && expert_ids && y, "lga_moe_combine: null pointer");
  LGA_CHECK_ARG(T > 0 && T <= 65535 && k > 0 && k <= 8 && C > 0 && C % 8 == 0, "lga_moe_combine: bad geometry");
  const dim3 grid((C / 8 + 255) / 256, T);
  lga::moe_combine_kernel<<<grid, 256, 0, stream>>>((const uint16_t*)expert_out, (const uint16_t*)probs, expert_ids,
                                                    (const uint16_t*)residual, (uint16_t*)y, k, C);
  LGA_LAUNCH_RETURN();
}

// ---- grouped prefill: the tile table of lga_q4_gemm_grouped -------------------------------------------------------
// One workgroup: a stable counting sort of the T * k (token, slot) pairs by expert (the reference's per-expert token
// groups, lit_gpt/model.py:740-741, in (token, slot) order within each expert), then the m-tiles of bm rows per
// expert. Outputs: tiles = {n_tiles, (expert, first row, rows) x n_tiles}, x_rows[r] = token of permuted row r,
// y_rows[r] = token * k + slot (the row of the (T, k, C) expert-output tensor moe_combine reads).
namespace lga {
__global__ void __launch_bounds__(1024) moe_group_kernel(const int32_t* __restrict__ ids, int n, int k, int E, int bm,
                                                         int32_t* __restrict__ tiles, int32_t* __restrict__ x_rows,
                                                         int32_t* __restrict__ y_rows) {
  __shared__ int cnt[8], base[8], run[8], wtot[16][8];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (tid < 8) cnt[tid] = run[tid] = 0;
  __syncthreads();
  for (int i = tid; i < n; i += 1024) atomicAdd(&cnt[min(max(ids[i], 0), E - 1)], 1);
  __syncthreads();
  if (tid == 0) {
    int b = 0, t = 0;
    for (int e = 0; e < E; ++e) {
      base[e] = b;
      for (int r = 0; r < cnt[e]; r += bm) {
        tiles[1 + 3 * t] = e;
        tiles[2 + 3 * t] = b + r;
        tiles[3 + 3 * t] = min(bm, cnt[e] - r);
        ++t;
      }
      b += cnt[e];
    }
    tiles[0] = t;
  }
  __syncthreads();
  const unsigned long long lt = (1ull << lane) - 1ull;  // lanes below this one
  for (int c0 = 0; c0 < n; c0 += 1024) {
    const int i = c0 + tid;
    const int e = i < n ? min(max(ids[i], 0), E - 1) : -1;
    int rank = 0;
    for (int x = 0; x < E; ++x) {
      const unsigned long long m = __ballot(e == x);
      if (e == x) rank = __popcll(m & lt);
      if (lane == 0) wtot[wave][x] = __popcll(m);
    }
    __syncthreads();
    if (e >= 0) {
      int before = 0;
      for (int w = 0; w < wave; ++w) before += wtot[w][e];
      const int pos = base[e] + run[e] + before + rank;
      x_rows[pos] = i / k;
      y_rows[pos] = i;
    }
    __syncthreads();
    if (tid < E) {
      int tot = 0;
      for (int w = 0; w < 16; ++w) tot += wtot[w][tid];
      run[tid] += tot;
    }
    __syncthreads();
  }
}
}  // namespace lga

extern "C" int lga_moe_group(const int32_t* expert_ids, int T, int k, int n_expert, int bm, int32_t* tiles,
                             int32_t* x_rows, int32_t* y_rows, hipStream_t stream) {
  LGA_CHECK_ARG(expert_ids && tiles && x_rows && y_rows, "lga_moe_group: null pointer");
  LGA_CHECK_ARG(T > 0 && k > 0 && n_expert > 0 && n_expert <= 8 && bm > 0, "lga_moe_group: needs n_expert <= 8");
  lga::moe_group_kernel<<<1, 1024, 0, stream>>>(expert_ids, T * k, k, n_expert, bm, tiles, x_rows, y_rows);
  LGA_LAUNCH_RETURN();
}

int lga::preload_moe() {  // the sparse-MoE prefill's routing, grouping and combine kernels
  return lga::preload(lga::moe_route_kernel) + lga::preload(lga::moe_combine_kernel) +
         lga::preload(lga::moe_group_kernel) + lga::preload(lga::moe_gate_route_kernel<2, 0, true>) +
         lga::preload(lga::moe_gate_route_kernel<2, 1, true>) + lga::preload(lga::moe_down_pair_kernel<2, 7, 0, 8>) + lga::preload(lga::moe_down_pair_kernel<2, 8, 0>);
}
