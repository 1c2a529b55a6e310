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
#include <cstdlib>

#include "decode_ops.h"

namespace lga {

#ifndef LGA_ATTN_PIPE
#define LGA_ATTN_PIPE 1
#endif

#ifdef LGA_ATTN_TRACE  // lab builds only (tools/attn_trace.py): per-block phase timestamps, 100 MHz clock
__device__ unsigned long long g_attn_trace[8192 * 8];
#define LGA_TRACE(i)                                                                            \
  do {                                                                                          \
    if (threadIdx.x == 0) {                                                                     \
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                              \
      g_attn_trace[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                                           \
  } while (0)
#else
#define LGA_TRACE(i) \
  do {               \
  } while (0)
#endif

// per-(t, group) arrival counters sit 256 B apart: same-line device-scope atomics serialize
constexpr int kCounterStride = 64;

// K/V rows are streamed once per step (the next step's re-read comes after ~1 GB of other traffic): nt loads
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_kv(const uint16_t* p) {
  const u32x4_t v = __builtin_nontemporal_load((const u32x4_t*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// FUSED (decode, T = 1): q, k, v come straight from the qkv projection row; every workgroup ropes its group's
// q heads itself, and the workgroup whose split owns the new position p ropes k, appends k and v to the cache
// at p (KVCache.forward, lit_gpt/model.py:788-795) and scores that key from registers — replacing the separate
// lga_rope_kv_append launch of the decode step.
#ifndef LGA_ATTN_SOLO
#define LGA_ATTN_SOLO 1  // lab A/B: 0 = the workgroup-barrier publish for every slice width
#endif

template <int HS, int QPK, int UNR, int NW, bool FUSED, bool PIPE>
__device__ __forceinline__ void attn_body(const uint16_t* __restrict__ q, uint16_t* __restrict__ kc,
                                          uint16_t* __restrict__ vc, const int64_t* __restrict__ input_pos,
                                          uint16_t* __restrict__ y, float* __restrict__ ws,
                                          unsigned* __restrict__ cnt, int n_head, int max_seq, float scale,
                                          const int64_t* __restrict__ rope_pos, const float* __restrict__ cos,
                                          const float* __restrict__ sin, int rope_rows, int hsplit) {
  constexpr int LPR = HS / 8;    // lanes per key row
  constexpr int RGW = 64 / LPR;  // row groups per wave
  constexpr int RG = NW * RGW;   // row groups per workgroup
  constexpr int NT = NW * 64;
  // blockIdx.y = (query group, head slice): with hsplit > 1 the group's QPKT heads are dealt to hsplit workgroups of
  // QPK heads each (few groups per rank: more workgroups per launch, each doing less per key)
  const int split = blockIdx.x, gy = blockIdx.y, t = blockIdx.z;
  const int g = gy / hsplit, hsi = gy % hsplit, QPKT = QPK * hsplit;
  const int n_splits = gridDim.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rg = wave * RGW + lane / LPR;
  const int sub = lane % LPR;
  LGA_TRACE(0);
  // both positions in one scalar round trip (hipcc otherwise waits for input_pos before issuing rope_pos)
  const long p = input_pos[t];
  const long rp_raw = FUSED ? rope_pos[t] : 0;
  const int L = (int)min(p + 1, (long)max_seq);  // keys 0..p (never past the cache)
  const int chunk = (L + n_splits - 1) / n_splits;
  const int k_lo = split * chunk;
  const int k_hi = min(k_lo + chunk, L);
  LGA_TRACE(1);
  const bool owns_new = FUSED && p < max_seq && k_lo <= p && p < k_hi;
  const int k_end = FUSED ? min(k_hi, (int)p) : k_hi;  // fused: key p is scored from registers below
  const float* cr = nullptr;
  const float* sr = nullptr;
  if (FUSED) {
    const long rp = min(max(rp_raw, 0L), (long)rope_rows - 1);
    cr = cos + (size_t)rp * HS + sub * 8;
    sr = sin + (size_t)rp * HS + sub * 8;
  }
  const uint16_t* kbase = kc + (size_t)g * max_seq * HS + sub * 8;
  const uint16_t* vbase = vc + (size_t)g * max_seq * HS + sub * 8;
  // clamped duplicate rows (past k_end) are masked in consume() and hit in cache
  auto fetch = [&](uint4 (&kv)[UNR], uint4 (&vv)[UNR], int j0) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int j = max(min(j0 + u * RG, k_end - 1), 0);
      kv[u] = ld_kv(kbase + (size_t)j * HS);
      vv[u] = ld_kv(vbase + (size_t)j * HS);
    }
  };
  const int j_first = k_lo + rg;

  // the q rows and the RoPE tables, then the first K/V batch (an empty split's batch re-reads row 0 and is never
  // consumed)
  uint4 qraw[QPK];
#pragma unroll
  for (int h = 0; h < QPK; ++h) {
    if (FUSED)  // qkv row layout per group: [q_0 .. q_{QPK-1}, k, v] x HS (scripts/convert_hf_checkpoint.py:181-187)
      qraw[h] = *(const uint4*)(q + ((size_t)g * (QPKT + 2) + hsi * QPK + h) * HS + sub * 8);
    else
      qraw[h] = *(const uint4*)(q + ((size_t)t * n_head + (size_t)g * QPKT + hsi * QPK + h) * HS + sub * 8);
  }
  float cs[FUSED ? 8 : 1], sn[FUSED ? 8 : 1];
  if (FUSED) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      cs[i] = cr[i];
      sn[i] = sr[i];
    }
  }
  // q stays packed bf16 (as the reference's bf16 q): scores are v_dot2_f32_bf16 chains — two exact bf16 products
  // per instruction into an fp32 accumulator, half the VALU of unpack + fma. Interleaved A/B (tools/attn_ab.py,
  // round 5) at p = 32066, 32 splits: Mixtral 34.8 -> 33.8 us, its TP = 2 rank 24.8 -> 23.5; Llama-2-7B neutral
  uint4 qp[QPK];
#pragma unroll
  for (int h = 0; h < QPK; ++h) qp[h] = FUSED ? rope8(qraw[h], cs, sn, sub) : qraw[h];
  // the online softmax runs in log2 units (as the prefill's flash attention): scores scaled by scale * log2(e), every
  // exponential one v_exp_f32 (exp2) instead of expf's 12-instruction range reduction — the long-context launches are
  // VALU-bound (tools/attn_pmc.py: Mixtral at p = 32066, the waves VALU-active 40 % of their cycles, 2 per SIMD);
  // the partials' m is in log2 units too (only this kernel's combine reads it)
  const float sl2 = scale * 1.4426950408889634f;
  auto dot8 = [](const uint4 a, const uint4 b) {
    typedef short s2 __attribute__((ext_vector_type(2)));
    float d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(s2, a.x), __builtin_bit_cast(s2, b.x), 0.0f, false);
    d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(s2, a.y), __builtin_bit_cast(s2, b.y), d, false);
    d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(s2, a.z), __builtin_bit_cast(s2, b.z), d, false);
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(s2, a.w), __builtin_bit_cast(s2, b.w), d, false);
  };
  // the first K/V batch AFTER the RoPE: issued beside q (ahead of the RoPE's wait) every split's first loads leave
  // in one burst at kernel start, measured 0.25-0.3 us slower per launch (tools/attn_ab.py, round 5)
  __builtin_amdgcn_sched_barrier(0);
  uint4 ka[UNR], va[UNR], kb[UNR], vb[UNR];
  if (PIPE) fetch(ka, va, j_first);
  LGA_TRACE(2);
  // m starts at a finite floor, not -inf: every row group runs the split's step count, so one whose keys are all
  // past k_end sees only masked (-inf) scores, and exp(floor - floor) = 1 keeps its (l, o) = 0 instead of NaN; a
  // real first score s gives exp(kMFloor - s) = 0 exactly as exp(-inf) did
  constexpr float kMFloor = -1e30f;
  float m[QPK], l[QPK], o[QPK][8];
#pragma unroll
  for (int h = 0; h < QPK; ++h) {
    m[h] = kMFloor;
    l[h] = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[h][i] = 0.0f;
  }
  // one step = UNR keys per row group: scores, online-softmax rescale, P.V (masked keys score -inf)
  auto consume = [&](const uint4 (&kv)[UNR], const uint4 (&vv)[UNR], int j0) {
#pragma unroll
    for (int h = 0; h < QPK; ++h) {
      float s[UNR];
      float mx = m[h];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const float sd = row_group_sum<LPR>(dot8(qp[h], kv[u])) * sl2;  // whole row group active: DPP inside it
        s[u] = (j0 + u * RG < k_end) ? sd : -INFINITY;
        mx = fmaxf(mx, s[u]);
      }
      const float c = __builtin_amdgcn_exp2f(m[h] - mx);  // m = kMFloor (first step) -> 0
      l[h] *= c;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[h][i] *= c;
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const float e = __builtin_amdgcn_exp2f(s[u] - mx);  // masked keys: exp(-inf) = 0
        l[h] += e;
        float vf[8];
        unpack8(vv[u], vf);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[h][i] = fmaf(e, vf[i], o[h][i]);
      }
      m[h] = mx;
    }
  };
  if (PIPE) {
    // software pipeline: step i + 1's 2*UNR loads are issued before step i's math, so every row group keeps 2-4
    // steps of K/V in flight and a split costs one load round trip plus its streaming time (the first batch was
    // issued above, next to q)
    const int stp = RG * UNR;
    const int nst = k_end > k_lo ? (k_end - k_lo + stp - 1) / stp : 0;
    int i = 0;
    for (; i + 1 < nst; i += 2) {
      fetch(kb, vb, j_first + (i + 1) * stp);
      consume(ka, va, j_first + i * stp);
      if (i + 2 < nst) fetch(ka, va, j_first + (i + 2) * stp);
      consume(kb, vb, j_first + (i + 1) * stp);
    }
    if (i < nst) consume(ka, va, j_first + i * stp);
  } else {
    for (int j0 = j_first; j0 < k_end; j0 += RG * UNR) {
      fetch(ka, va, j0);
      consume(ka, va, j0);
    }
  }
  LGA_TRACE(3);
  if (FUSED && owns_new && rg == 0) {  // the new key/value: rope k, append both to the cache, score from registers
    const uint16_t* kvrow = q + ((size_t)g * (QPKT + 2) + QPKT) * HS + sub * 8;
    const uint4 kr = rope8(*(const uint4*)kvrow, cs, sn, sub);
    const uint4 vr = *(const uint4*)(kvrow + HS);
    if (hsi == 0) {  // one head slice appends; the others score the same key from their registers
      *(uint4*)(kc + ((size_t)g * max_seq + p) * HS + sub * 8) = kr;
      *(uint4*)(vc + ((size_t)g * max_seq + p) * HS + sub * 8) = vr;
    }
    float vf[8];
    unpack8(vr, vf);
#pragma unroll
    for (int h = 0; h < QPK; ++h) {
      const float s = row_group_sum<LPR>(dot8(qp[h], kr)) * sl2;
      const float mx = fmaxf(m[h], s);
      const float c = __builtin_amdgcn_exp2f(m[h] - mx);
      const float e = __builtin_amdgcn_exp2f(s - mx);
      l[h] = l[h] * c + e;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[h][i] = fmaf(e, vf[i], o[h][i] * c);
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
      const float ca = __builtin_amdgcn_exp2f(m[h] - mn);  // m >= kMFloor: finite, never exp(-inf - -inf)
      const float cb = __builtin_amdgcn_exp2f(mo - mn);
      l[h] = l[h] * ca + lo * cb;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[h][i] = o[h][i] * ca + __shfl_xor(o[h][i], off) * cb;
      m[h] = mn;
    }
  }
  __shared__ float sm[NW][QPK], sl[NW][QPK];
  __shared__ __attribute__((aligned(16))) float so[NW][QPK][HS];
  __shared__ unsigned s_ticket;
  if (lane < LPR) {
#pragma unroll
    for (int h = 0; h < QPK; ++h) {
      if (lane == 0) {
        sm[wave][h] = m[h];
        sl[wave][h] = l[h];
      }
      *(float4*)&so[wave][h][sub * 8] = make_float4(o[h][0], o[h][1], o[h][2], o[h][3]);
      *(float4*)&so[wave][h][sub * 8 + 4] = make_float4(o[h][4], o[h][5], o[h][6], o[h][7]);
    }
  }
  __syncthreads();
  // block merge: a thread owns 4 consecutive output columns (h, 4 dq .. 4 dq + 3) of one head of the slice
  constexpr int NQ = QPK * HS / 4;
  static_assert(NQ <= NT, "one 4-column item per thread");
  const bool has_item = threadIdx.x < NQ;
  const int hq = threadIdx.x / (HS / 4), dq = threadIdx.x % (HS / 4);
  float bm = -INFINITY, bl = 0.0f, bo[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (has_item) {
#pragma unroll
    for (int w = 0; w < NW; ++w) bm = fmaxf(bm, sm[w][hq]);
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float c = __builtin_amdgcn_exp2f(sm[w][hq] - bm);
      bl += sl[w][hq] * c;
      const float4 ov = *(const float4*)&so[w][hq][dq * 4];
      bo[0] += ov.x * c;
      bo[1] += ov.y * c;
      bo[2] += ov.z * c;
      bo[3] += ov.w * c;
    }
  }
  const size_t row0 = (size_t)t * n_head + (size_t)g * QPKT + hsi * QPK;  // first head row of this slice
  if (n_splits == 1) {
    if (has_item) {
      uint16_t* yr = y + (row0 + hq) * HS + dq * 4;
      *(uint2*)yr = make_uint2(pack2(bo[0] / bl, bo[1] / bl), pack2(bo[2] / bl, bo[3] / bl));
    }
    return;
  }
  LGA_TRACE(4);
  // ---- publish (m, l, o), then the last-arriving split of this (t, group) merges all splits (MI355X_MICROARCH.md
  // "Valid forms" row 1: 16-B sc1 stores, every storing wave drains, a workgroup barrier, one lane's agent-scope
  // add; the last arriver's loads are sc1 too). Per (head row, split): {m, l, 0, 0, o[HS]} fp32 ----
  // SOLO: every output quad sits in wave 0 (QPK * HS / 4 <= 64), so wave 0 alone stores, drains, counts and, when
  // last, combines: the same row-1 form with one storing wave, no workgroup barrier or LDS ticket on the tail
  constexpr bool SOLO = LGA_ATTN_SOLO && NQ <= 64;
  if (SOLO && wave != 0) return;
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(ws + row0 * n_splits * (HS + 4)), (short)0, QPK * n_splits * (HS + 4) * 4, 0x00020000);
  if (has_item) {
    const unsigned off = (unsigned)((hq * n_splits + split) * (HS + 4)) * 4;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, make_float4(bo[0], bo[1], bo[2], bo[3])), wrs,
                                           off + 16 + dq * 16, 0, 16);
    if (dq == 0)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, make_float4(bm, bl, 0.0f, 0.0f)), wrs, off,
                                             0, 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned* ctr = cnt + ((size_t)t * gridDim.y + gy) * kCounterStride;
  unsigned ticket;
  if constexpr (SOLO) {
    unsigned tk = 0;
    if (lane == 0) tk = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ticket = __builtin_amdgcn_readfirstlane(tk);  // lane 0's
  } else {
    __syncthreads();
    if (threadIdx.x == 0) s_ticket = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    ticket = s_ticket;
  }
  LGA_TRACE(5);
  if (ticket != (unsigned)(n_splits - 1)) return;
  // one output column quad per thread, 8 splits per round with every load of the round in flight at once and an
  // online rescale across rounds. Split 0 always holds key 0, so the running max is finite after round 0; empty
  // splits carry m = kMFloor, l = 0, o = 0 and clamped out-of-range slots are forced to m = -inf: both weigh 0.
  if (has_item) {
    const unsigned hoff = (unsigned)(hq * n_splits * (HS + 4)) * 4;
    float mx = -INFINITY, lt = 0.0f, ot[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int s0 = 0; s0 < n_splits; s0 += 8) {
      float4 ml[8], o4[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const unsigned off = hoff + (unsigned)(min(s0 + u, n_splits - 1) * (HS + 4)) * 4;
        ml[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wrs, off, 0, 16));
        o4[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(wrs, off + 16 + dq * 16, 0, 16));
      }
      float nm = mx;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (s0 + u >= n_splits) ml[u].x = -INFINITY;
        nm = fmaxf(nm, ml[u].x);
      }
      const float c = __builtin_amdgcn_exp2f(mx - nm);  // round 0: exp(-inf) = 0
      lt *= c;
#pragma unroll
      for (int i = 0; i < 4; ++i) ot[i] *= c;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float e = __builtin_amdgcn_exp2f(ml[u].x - nm);
        lt = fmaf(ml[u].y, e, lt);
        ot[0] = fmaf(o4[u].x, e, ot[0]);
        ot[1] = fmaf(o4[u].y, e, ot[1]);
        ot[2] = fmaf(o4[u].z, e, ot[2]);
        ot[3] = fmaf(o4[u].w, e, ot[3]);
      }
      mx = nm;
    }
    uint16_t* yr = y + (row0 + hq) * HS + dq * 4;
    const uint2 yv = make_uint2(pack2(ot[0] / lt, ot[1] / lt), pack2(ot[2] / lt, ot[3] / lt));
    *(uint2*)yr = yv;
  }
  if (threadIdx.x == 0) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  LGA_TRACE(6);
}

template <int HS, int QPK, int UNR, int NW, bool FUSED, bool PIPE>
__global__ void __launch_bounds__(NW * 64) attn_kernel(const uint16_t* __restrict__ q, uint16_t* __restrict__ kc,
                                                   uint16_t* __restrict__ vc, const int64_t* __restrict__ input_pos,
                                                   uint16_t* __restrict__ y, float* __restrict__ ws,
                                                   unsigned* __restrict__ cnt, int n_head, int max_seq, float scale,
                                                   const int64_t* __restrict__ rope_pos, const float* __restrict__ cos,
                                                   const float* __restrict__ sin, int rope_rows, int hsplit) {
  attn_body<HS, QPK, UNR, NW, FUSED, PIPE>(q, kc, vc, input_pos, y, ws, cnt, n_head, max_seq, scale, rope_pos, cos,
                                           sin, rope_rows, hsplit);
}

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

// ---------------------------------------------------------------------------------------------------------------
// Prefill (T >= 16): flash attention on MFMA, swapped form. A workgroup = 4 waves x 32 query rows of one head;
// key tiles of 64 rows stream through a double-buffered LDS image (register-staged: the next tile's global loads are issued
// before this tile's MFMAs and written after them). Per 32-key half-tile, S^T = K . Q^T on v_mfma_f32_32x32x16_bf16
// (A = K rows from LDS, B = this wave's Q^T held in registers), so lane l holds the scores of ONE query (l % 32)
// for 16 keys and its partner lane l ^ 32 the other 16: the online-softmax max / sum are in-lane chains plus one
// exchange. P goes to bf16 in registers and two v_permlane32_swap per 16 keys regroup it into the B operand of
// O^T += V^T . P^T, whose A operand comes straight from the row-major V image by ds_read_b64_tr_b16 (transposed
// LDS read) — no P or V^T round trip through LDS. O^T's lane also owns one query, so the rescale by
// exp(m_old - m_new) is a per-lane scalar, skipped when no row max of the wave moved. Causal masking only on the
// tiles that cross a row's position (a 32-bit compare + select per element, on those tiles only); the scores stay
// raw — the max runs on them and one fma(s, scale log2 e, -m) per element feeds v_exp_f32 (max(s) c == max(s c) for
// c > 0). K / V tiles are staged by buffer loads (the whole row offset in the per-thread voffset; rows past the
// cache read as zeros by the range check) and every LDS address is a per-lane base plus a compile-time offset (the
// tile loop is unrolled by the two buffers). Grid: 1-D, `order` 1 pairs the two workgroups a CU holds — the first
// half walks query blocks nblk-1 .. nblk/2, the second half blocks 0 .. nblk/2-1, so workgroups i and i + half sum
// to a constant number of key tiles and share a head (its K / V in one XCD's L2).
// Llama-2-7B, T = 2048: 64-65 us per layer = 529-540 TFLOP/s causal, 652-667 TFLOP/s with every row seeing all
// keys (tools/prefill_attn_bench.py; round 2's kernel: 88-90 us). PMC (profiles/r03c_prefill_fa_pmc.txt): MFMA busy
// 0.24, SQ_WAIT_ANY 30 % / SQ_WAIT_INST_ANY 35 % of wave cycles, L2 hit 85 % — latency inside each wave (K read ->
// S MFMA -> max -> exp -> P -> PV chains), not bandwidth; one workgroup per CU is only 19 % slower.
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef short i16x4_t __attribute__((ext_vector_type(4)));
typedef short i16x8_t __attribute__((ext_vector_type(8)));

// LDS image of a [64 keys][HS] bf16 tile: 16-B chunk ch of row r at byte r * 2HS + 16 (ch ^ sw(r)). For HS = 128
// this is cdna_hip_programming.md T10 image (b): conflict-free for both the 32x32x16 row reads (K) and the
// transposed reads (V).
template <int HS>
__device__ __forceinline__ int kv_off(int row, int ch) {
  constexpr int CH = HS / 8;
  const int sw = CH == 16 ? (((row & 3) << 2) | ((row >> 2) & 3)) : (((row & 3) << 1) | ((row >> 2) & 1));
  return row * (HS * 2) + 16 * (ch ^ sw);
}

template <int HS>
__global__ void __launch_bounds__(256, 2) attn_prefill_kernel(const uint16_t* __restrict__ q,
                                                                const uint16_t* __restrict__ kc,
                                                                const uint16_t* __restrict__ vc,
                                                                const int64_t* __restrict__ input_pos,
                                                                uint16_t* __restrict__ y, int T, int n_head, int G,
                                                                int max_seq, float scale, int order) {
  constexpr int KT = 64;              // keys per tile
  constexpr int CH = HS / 8;          // 16-B chunks per key row
  constexpr int DK = HS / 16;         // 32x32x16 k-steps over the head dim (S^T)
  constexpr int DT = HS / 32;         // 32-row tiles of O^T
  constexpr int TB = KT * HS * 2;     // bytes of one K or V tile image
  constexpr int LPT = KT * CH / 256;  // 16-B chunks per thread per tile (K and V each)
  constexpr int RPI = 256 / CH;       // key rows between a thread's consecutive chunks
  __shared__ __attribute__((aligned(16))) unsigned char lds[2][2][TB];  // [buffer][K | V]
  __shared__ int s_pos[2][4];                                           // per wave: max / min row position

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hh = lane >> 5, lq = lane & 31;
  const int nblk = (T + 127) / 128;
  // order 0: longest first; order 1: the first half of the grid walks blocks nblk-1 .. nblk/2, the second half
  // blocks 0 .. nblk/2-1, so workgroups i and i + half hold key-tile counts summing to a constant and the same head
  // (its K / V stays in one XCD's L2 when half is a multiple of 8)
  const int nhi = (nblk - nblk / 2) * n_head;
  const int i = blockIdx.x;
  const bool lo_half = order == 1 && i >= nhi;
  const int jj = lo_half ? i - nhi : i;
  const int head = jj % n_head, g = head / (n_head / G);
  const int blk = lo_half ? jj / n_head : nblk - 1 - jj / n_head;
  const int q0 = blk * 128 + wave * 32;
  const int t = q0 + lq;
  const int mypos = t < T ? (int)input_pos[t] : -1;
  {
    int mx = mypos, mn = t < T ? mypos : INT_MAX;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mx = max(mx, __shfl_xor(mx, o));
      mn = min(mn, __shfl_xor(mn, o));
    }
    if (lane == 0) {
      s_pos[0][wave] = mx;
      s_pos[1][wave] = mn;
    }
  }
  bf16x8_t qb[DK];  // Q^T fragments (B operand): lane l holds Q[t][ks*16 + 8*hh .. +8]
  {
    const uint16_t* qr = q + ((size_t)min(t, T - 1) * n_head + head) * HS + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < DK; ++ks) qb[ks] = *(const bf16x8_t*)(qr + ks * 16);
  }
  __syncthreads();
  const int wmax = s_pos[0][wave], wmin = s_pos[1][wave];
  const int bmax = min(max(max(s_pos[0][0], s_pos[0][1]), max(s_pos[0][2], s_pos[0][3])), max_seq - 1);
  const int ntiles = (bmax + 1 + KT - 1) / KT;

  // K / V staging: thread tid moves chunk tid % CH of rows tid / CH + RPI i of every tile
  const __amdgpu_buffer_rsrc_t krs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(kc + (size_t)g * max_seq * HS), (short)0, max_seq * HS * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(vc + (size_t)g * max_seq * HS), (short)0, max_seq * HS * 2, 0x00020000);
  const int gvoff = ((tid / CH) * HS + (tid % CH) * 8) * 2;
  u32x4_t kr[LPT], vr[LPT];  // tile t + 1 in flight under tile t
  int soff[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) soff[i] = kv_off<HS>(tid / CH + RPI * i, tid % CH);
  // the whole byte offset rides in voffset: the buffer range check covers voffset only (soffset is added after
  // it), so rows past max_seq — the last partial tile and the one-tile-ahead prefetch — read as zeros instead of
  // past the group's cache
#ifndef LGA_FA_EXP
#define LGA_FA_EXP 0  // lab only (tools/prefill_attn_bench.py): 1 no tile math, 2 no global loads, 3 neither
#endif
  auto gload = [&](int k0) {
    if (LGA_FA_EXP & 2) return;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int off = gvoff + (k0 + RPI * i) * HS * 2;
      kr[i] = __builtin_amdgcn_raw_buffer_load_b128(krs, off, 0, 0);
      vr[i] = __builtin_amdgcn_raw_buffer_load_b128(vrs, off, 0, 0);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      *(u32x4_t*)(lds[buf][0] + soff[i]) = kr[i];
      *(u32x4_t*)(lds[buf][1] + soff[i]) = vr[i];
    }
  };
  // LDS read bases: K row lq (+ 32 st), chunk 2 ks + hh; V^T transposed reads (16-lane group grp, quad qq, pair pp)
  int koff[DK];
#pragma unroll
  for (int ks = 0; ks < DK; ++ks) koff[ks] = kv_off<HS>(lq, 2 * ks + hh);
  const int gi = lane & 15, qq = gi >> 2, pp = gi & 3, grp = lane >> 4;
  int voff0[DT], voff1[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    const int ch = ((dt * 32 + 16 * (grp & 1)) >> 3) + (pp >> 1);
    voff0[dt] = kv_off<HS>(8 * (grp >> 1) + qq, ch) + 8 * (pp & 1);
    voff1[dt] = kv_off<HS>(8 * (grp >> 1) + 4 + qq, ch) + 8 * (pp & 1);
  }

  f32x16_t o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.0f;
  float m = -INFINITY, l = 0.0f;  // m in the scaled log2 domain; l = this lane's 16-key half of the row sum
  const float sl2 = scale * 1.4426950408889634f;

  auto tile = [&](const unsigned char* K, const unsigned char* V, int k0) {
    if (LGA_FA_EXP & 1) return;
    // S^T of the two 32-key halves as two interleaved accumulation chains
    f32x16_t sacc[2];
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[st][r] = 0.0f;
#pragma unroll
    for (int ks = 0; ks < DK; ++ks)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8_t ka = *(const bf16x8_t*)(K + st * 32 * HS * 2 + koff[ks]);
        sacc[st] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qb[ks], sacc[st], 0, 0, 0);
      }
    if (__builtin_amdgcn_readfirstlane(k0 + KT - 1 > wmin)) {  // a row of this wave ends inside the tile
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (k0 + st * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh > mypos) sacc[st][r] = -INFINITY;
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, sacc[st][r]);
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(tmax), __float_as_uint(tmax), false, false);
      tmax = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));  // both halves of the row
    }
    const float mnew = fmaxf(m, tmax * sl2);
    const float mref = mnew == -INFINITY ? 0.0f : mnew;  // rows with no visible key yet: p = 0, o stays 0
    if (!__all(mnew == m)) {                              // some row max moved: rescale (exactly; no threshold)
      const float c = __builtin_amdgcn_exp2f(m - mref);
      l *= c;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= c;
    }
    m = mnew;
    // P^T . V per 16-key k-step kk: its 8 exponentials (half-tile kk / 2, registers 8 (kk & 1) .. +7) become the
    // B operand just before its DT MFMAs, so the next k-step's exponentials can issue under them
    float rs = 0.0f;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int st = kk >> 1, r0 = 8 * (kk & 1);
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        x[e] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[st][r0 + e], sl2, -mref));
        rs += x[e];
      }
      const uint32_t w0 = pack2(x[0], x[1]), w1 = pack2(x[2], x[3]);
      const uint32_t w2 = pack2(x[4], x[5]), w3 = pack2(x[6], x[7]);
      const auto a = __builtin_amdgcn_permlane32_swap(w0, w2, false, false);
      const auto b = __builtin_amdgcn_permlane32_swap(w1, w3, false, false);
      const u32x4_t f = {a[0], b[0], a[1], b[1]};
      const bf16x8_t pb = __builtin_bit_cast(bf16x8_t, f);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        typedef __attribute__((address_space(3))) i16x4_t lds_i16x4;
        const i16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(V + kk * 16 * HS * 2 + voff0[dt]));
        const i16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(V + kk * 16 * HS * 2 + voff1[dt]));
        const i16x8_t vf = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, vf), pb, o[dt], 0, 0, 0);
      }
    }
    l += rs;
  };

  // unrolled by the two buffers so every LDS address is base + constant; tile t + 1's loads are in flight under
  // tile t's MFMAs (past the cache: zeros, unused) and written to the other buffer after them (a second register
  // set, two tiles ahead, measured no faster: the loop is latency-bound inside the wave, not on the loads)
  if (ntiles > 0) {
    gload(0);
    lstore(0);
  }
  __syncthreads();
  for (int it = 0; it < ntiles; it += 2) {
    const int k0 = it * KT;
    gload(k0 + KT);
    if (k0 <= wmax) tile(lds[0][0], lds[0][1], k0);
    lstore(1);
    __syncthreads();
    if (it + 1 >= ntiles) break;
    gload(k0 + 2 * KT);
    if (k0 + KT <= wmax) tile(lds[1][0], lds[1][1], k0 + KT);
    lstore(0);
    __syncthreads();
  }
  l += __shfl_xor(l, 32);
  // y[t][head * HS + d] = O^T[d][t] / l, d = dt * 32 + crow(r): pairs (r, r + 1) are adjacent columns
  if (t < T) {
    const float inv = 1.0f / l;
    uint16_t* yr = y + ((size_t)t * n_head + head) * HS;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const int d = dt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        *(uint32_t*)(yr + d) = pack2(o[dt][r] * inv, o[dt][r + 1] * inv);
      }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Prefill, paired form (default): one 512-thread workgroup per (head, block pair) holds query blocks hi = nblk-1-p
// (waves 0-3) and lo = p (waves 4-7) of 128 rows and streams the head's K / V ONCE for both — key tile t serves
// every wave whose rows reach it (26 % fewer L2 -> LDS bytes than a workgroup per block at T = 2048, and every SIMD
// holds one hi and one lo wave: 2 (nblk + 1) key tiles per SIMD whatever p). K / V tiles reach LDS by LDS-DMA
// (`buffer_load_dwordx4 ... lds`, range-checked: rows past the cache land as zeros) into a 4-stage ring, three tiles
// ahead of the math, with no staging registers; a raw s_barrier per tile after a counted vmcnt. The LDS reads are
// inline asm with counted lgkmcnt waits (hipcc would wait for every DMA in flight before a compiler-visible LDS
// read, not telling the stages apart). Per wave the arithmetic is attn_prefill_kernel's, op for op.
// an LDS read at a compile-time offset (after unrolling) in inline asm; the host pass, which only type-checks the
// kernel body, cannot take the "i" operand of a non-constant expression
#ifdef __HIP_DEVICE_COMPILE__
#define LGA_DS_READ(op, dst, addr, off) \
  asm volatile(op " %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(off) : "memory")
#else
#define LGA_DS_READ(op, dst, addr, off) ((dst) = {}, (void)(addr), (void)(off))
#endif

template <int HS>
__global__ void __launch_bounds__(512, 1) attn_prefill_pair_kernel(const uint16_t* __restrict__ q,
                                                                   const uint16_t* __restrict__ kc,
                                                                   const uint16_t* __restrict__ vc,
                                                                   const int64_t* __restrict__ input_pos,
                                                                   uint16_t* __restrict__ y, int T, int n_head, int G,
                                                                   int max_seq, float scale) {
  constexpr int KT = 64;           // keys per tile
  constexpr int CH = HS / 8;       // 16-B chunks per key row
  constexpr int DK = HS / 16;      // 32x32x16 k-steps over the head dim (S^T)
  constexpr int DT = HS / 32;      // 32-row tiles of O^T
  constexpr int TB = KT * HS * 2;  // bytes of one K or V tile image
  constexpr int NS = 4;            // ring stages
  constexpr int PIECES = 2 * TB / 1024 / 8;  // 1-KB DMA pieces per wave per tile (K and V)
  static_assert(PIECES * 8 * 1024 == 2 * TB, "pieces");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NS][2][TB];  // [stage][K | V]
  __shared__ int s_pos[2][8];

  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, lq = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nblk = (T + 127) / 128;
  const int head = blockIdx.x % n_head, pr = blockIdx.x / n_head, g = head / (n_head / G);
  const int hi = nblk - 1 - pr, lo = pr;
  const int blk = wave < 4 ? hi : (lo < hi ? lo : -1);  // odd nblk: the middle block has no partner
  const int q0 = blk * 128 + (wave & 3) * 32;
  const int t = q0 + lq;
  const bool valid = blk >= 0 && t < T;
  const int mypos = valid ? (int)input_pos[t] : -1;
  {
    int mx = mypos, mn = valid ? mypos : INT_MAX;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mx = max(mx, __shfl_xor(mx, o));
      mn = min(mn, __shfl_xor(mn, o));
    }
    if (lane == 0) {
      s_pos[0][wave] = mx;
      s_pos[1][wave] = mn;
    }
  }
  bf16x8_t qb[DK];  // Q^T fragments (B operand): lane l holds Q[t][ks*16 + 8*hh .. +8]
  {
    const uint16_t* qr = q + ((size_t)min(max(t, 0), T - 1) * n_head + head) * HS + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < DK; ++ks) qb[ks] = *(const bf16x8_t*)(qr + ks * 16);
  }
  // the Q fragments and positions are in before any DMA is counted; redefining them through an asm tells hipcc so
  // (it would otherwise wait for "their" loads — i.e. for every DMA in flight — at each use inside the loop)
#pragma unroll
  for (int ks = 0; ks < DK; ++ks) asm volatile("" : "+v"(qb[ks]));
  int mpos = mypos;
  asm volatile("" : "+v"(mpos));
  __syncthreads();
  const int wmax = s_pos[0][wave], wmin = s_pos[1][wave];
  int bmax = s_pos[0][0];
#pragma unroll
  for (int w = 1; w < 8; ++w) bmax = max(bmax, s_pos[0][w]);
  bmax = min(bmax, max_seq - 1);
  const int ntiles = (bmax + 1 + KT - 1) / KT;

  // DMA: wave w moves pieces w * PIECES .. +PIECES of the tile (K pieces first, then V); lane L of a piece lands at
  // +16 L = row r0 + L / CH, physical chunk L % CH, so it fetches logical chunk (L % CH) ^ sw(row) (kv_off's swizzle)
  const __amdgpu_buffer_rsrc_t krs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(kc + (size_t)g * max_seq * HS), (short)0, max_seq * HS * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(vc + (size_t)g * max_seq * HS), (short)0, max_seq * HS * 2, 0x00020000);
  constexpr int RPP = 1024 / (HS * 2);  // key rows per piece
  // (recomputed per issue: a few VALU per tile instead of PIECES live registers)
  auto dvoff = [&](int i) -> int {
    const int piece = (wave * PIECES + i) % (TB / 1024);
    const int r = piece * RPP + lane / CH;
    const int phys = lane % CH;
    const int sw = CH == 16 ? (((r & 3) << 2) | ((r >> 2) & 3)) : (((r & 3) << 1) | ((r >> 2) & 1));
    return (r * HS + (phys ^ sw) * 8) * 2;
  };
  auto issue = [&](int tt) {  // tile tt into stage tt % NS (every wave, every tile: the vmcnt counts stay uniform)
    unsigned char* st = &lds[tt % NS][0][0];
    const int kb = tt * KT * HS * 2;
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const int gp = wave * PIECES + i;
      const bool isv = gp >= TB / 1024;
      unsigned char* dst = st + (isv ? TB : 0) + (gp % (TB / 1024)) * 1024;
#ifdef __HIP_DEVICE_COMPILE__  // (a device builtin: the host pass only type-checks the body)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(isv ? vrs : krs, (__attribute__((address_space(3))) void*)dst, 16,
                                               kb + dvoff(i), 0, 0, 0);
#else
      (void)dst, (void)kb, (void)isv, (void)dvoff;
#endif
    }
  };

  // LDS read addresses: K row lq (+ 32 st), chunk 2 ks + hh; V^T transposed reads (16-lane group grp, quad qq, pair pp)
  const unsigned lbase = (unsigned)(uintptr_t)&lds[0][0][0];
  unsigned koff[DK];
#pragma unroll
  for (int ks = 0; ks < DK; ++ks) koff[ks] = lbase + kv_off<HS>(lq, 2 * ks + hh);
  const int gi = lane & 15, qq = gi >> 2, pp = gi & 3, grp = lane >> 4;
  unsigned voff0[DT], voff1[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    const int ch = ((dt * 32 + 16 * (grp & 1)) >> 3) + (pp >> 1);
    voff0[dt] = lbase + TB + kv_off<HS>(8 * (grp >> 1) + qq, ch) + 8 * (pp & 1);
    voff1[dt] = lbase + TB + kv_off<HS>(8 * (grp >> 1) + 4 + qq, ch) + 8 * (pp & 1);
  }

  f32x16_t o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.0f;
  float m = -INFINITY, l = 0.0f;
  const float sl2 = scale * 1.4426950408889634f;

  typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
  // K fragments of batch b (2 k-steps x 2 halves) of the stage at byte offset sb
  auto kread = [&](unsigned sb, int b, u32x4_t (&f)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ks = 2 * b + (j >> 1), st = j & 1;
      LGA_DS_READ("ds_read_b128", f[j], koff[ks] + sb, st * 32 * HS * 2);
    }
  };
  auto kmfma = [&](int b, const u32x4_t (&f)[4], f32x16_t (&acc)[2]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ks = 2 * b + (j >> 1), st = j & 1;
      acc[st] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, f[j]), qb[ks], acc[st], 0, 0, 0);
    }
  };
  auto vread = [&](unsigned sb, int kk, u32x2_t (&f)[DT][2]) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      LGA_DS_READ("ds_read_b64_tr_b16", f[dt][0], voff0[dt] + sb, kk * 16 * HS * 2);
      LGA_DS_READ("ds_read_b64_tr_b16", f[dt][1], voff1[dt] + sb, kk * 16 * HS * 2);
    }
  };
  // tie the fragments to a counted wait so no use moves above it
#define LGA_KW(N, f) asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]))
#define LGA_VW4(N, f)                                                                                             \
  asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(f[0][0]), "+v"(f[0][1]), "+v"(f[1][0]), "+v"(f[1][1]), "+v"(f[2][0]), \
               "+v"(f[2][1]), "+v"(f[3][0]), "+v"(f[3][1]))
#define LGA_VW2(N, f) asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(f[0][0]), "+v"(f[0][1]), "+v"(f[1][0]), "+v"(f[1][1]))

  // S^T = K . Q^T of the tile at sb: 16 K fragments in 4 batches of 4, one batch read ahead
  auto s_tile = [&](unsigned sb, f32x16_t (&sacc)[2]) {
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[st][r] = 0.0f;
    u32x4_t kf[2][4];
    kread(sb, 0, kf[0]);
#pragma unroll
    for (int b = 0; b < DK / 2; ++b) {
      if (b + 1 < DK / 2) {
        kread(sb, b + 1, kf[(b + 1) & 1]);
        LGA_KW(4, kf[b & 1]);
      } else {
        LGA_KW(0, kf[b & 1]);
      }
      kmfma(b, kf[b & 1], sacc);
    }
  };
  // the online softmax of S(t) (sacc) and O += P . V(t) from the stage at sbv
  auto pv_tile = [&](unsigned sbv, int k0, f32x16_t (&sacc)[2]) {
    u32x2_t vf[2][DT][2];
    vread(sbv, 0, vf[0]);
    if (__builtin_amdgcn_readfirstlane(k0 + KT - 1 > wmin)) {  // a row of this wave ends inside the tile
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (k0 + st * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh > mpos) sacc[st][r] = -INFINITY;
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, sacc[st][r]);
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(tmax), __float_as_uint(tmax), false, false);
      tmax = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    const float mnew = fmaxf(m, tmax * sl2);
    const float mref = mnew == -INFINITY ? 0.0f : mnew;
    if (!__all(mnew == m)) {
      const float c = __builtin_amdgcn_exp2f(m - mref);
      l *= c;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= c;
    }
    m = mnew;
    float rs = 0.0f;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int st = kk >> 1, r0 = 8 * (kk & 1);
      if (kk + 1 < 4) vread(sbv, kk + 1, vf[(kk + 1) & 1]);
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        x[e] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[st][r0 + e], sl2, -mref));
        rs += x[e];
      }
      const uint32_t w0 = pack2(x[0], x[1]), w1 = pack2(x[2], x[3]);
      const uint32_t w2 = pack2(x[4], x[5]), w3 = pack2(x[6], x[7]);
      const auto a = __builtin_amdgcn_permlane32_swap(w0, w2, false, false);
      const auto b = __builtin_amdgcn_permlane32_swap(w1, w3, false, false);
      const u32x4_t f = {a[0], b[0], a[1], b[1]};
      const bf16x8_t pb = __builtin_bit_cast(bf16x8_t, f);
      auto& cur = vf[kk & 1];
      if (kk + 1 < 4) {  // V(kk+1)'s 2 DT reads are newer than V(kk)
        if constexpr (DT == 4) LGA_VW4(8, cur); else LGA_VW2(4, cur);
      } else {
        if constexpr (DT == 4) LGA_VW4(0, cur); else LGA_VW2(0, cur);
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const u32x4_t vv = {cur[dt][0][0], cur[dt][0][1], cur[dt][1][0], cur[dt][1][1]};
        o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, vv), pb, o[dt], 0, 0, 0);
      }
    }
    l += rs;
  };

  // Ring: tiles 0 .. NS-2 in flight, then per tile: wait for it (the tiles issued after it may stay in flight),
  // barrier (every wave's pieces landed; every wave done with the stage the next issue overwrites), issue tile
  // + NS - 1, math. (Round 4 also measured the lo waves half a tile behind the hi waves, so the two waves of a SIMD
  // sit in opposite phases, and a software-pipelined form with S(t + 1)'s MFMAs under tile t's softmax and P.V:
  // both slower)
#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < ntiles) issue(i);
  for (int tt = 0; tt < ntiles; ++tt) {
    const int after = min(NS - 2, ntiles - 1 - tt);  // tiles issued after tt
    if (after >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PIECES) : "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PIECES) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (tt + NS - 1 < ntiles) issue(tt + NS - 1);
    const int k0 = tt * KT;
    if (k0 <= wmax) {
      f32x16_t sacc[2];
      const unsigned sb = (unsigned)((tt % NS) * 2 * TB);
      s_tile(sb, sacc);
      pv_tile(sb, k0, sacc);
    }
  }
#undef LGA_KW
#undef LGA_VW4
#undef LGA_VW2
  l += __shfl_xor(l, 32);
  if (valid) {
    const float inv = 1.0f / l;
    uint16_t* yr = y + ((size_t)t * n_head + head) * HS;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const int d = dt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        *(uint32_t*)(yr + d) = pack2(o[dt][r] * inv, o[dt][r + 1] * inv);
      }
  }
}

// (keys in flight per row group, waves per workgroup) by q_per_kv; -D overrides are for tools/attn_sweep.py
#ifndef LGA_ATTN_Q1
#define LGA_ATTN_Q1 4, 4
#endif
#ifndef LGA_ATTN_Q1_FEW
#define LGA_ATTN_Q1_FEW 2, 8
#endif
#ifndef LGA_ATTN_Q2
#define LGA_ATTN_Q2 4, 4
#endif
#ifndef LGA_ATTN_Q4  // 8 waves (round 4, tools/attn_sweep.py 32 8 128: Mixtral at 16 splits 12.5-12.9 vs 13.7-14.1 us)
#define LGA_ATTN_Q4 2, 8
#endif
#ifndef LGA_ATTN_Q8
#define LGA_ATTN_Q8 2, 4
#endif

template <int HS, int QPK, int UNR, int NW, bool FUSED>
static void launch_one(dim3 grid, hipStream_t stream, const void* q, void* kc, void* vc, const int64_t* pos, void* y,
                       float* ws, unsigned* cnt, int H, int max_seq, float scale, const int64_t* rope_pos,
                       const float* cos, const float* sin, int rope_rows, int hsplit) {
  attn_kernel<HS, QPK, UNR, NW, FUSED, LGA_ATTN_PIPE != 0><<<grid, NW * 64, 0, stream>>>((const uint16_t*)q, (uint16_t*)kc, (uint16_t*)vc,
                                                                     pos, (uint16_t*)y, ws, cnt, H, max_seq, scale,
                                                                     rope_pos, cos, sin, rope_rows, hsplit);
}

// head slices per query group: split a group's heads over more workgroups while the launch would fill at most half
// the CUs (tools/attn_sweep.py, p = 2303, 16 splits: Llama-2-70B at TP = 8 — one group of 8 heads per rank — 22.5 ->
// 7.8 us with 8 slices; 70B TP = 1 23.6 -> 13.4 with 2; Mixtral 12.9 -> 10.3 with 2, Mixtral TP = 2 12.6 -> 8.3
// with 4; profiles/r04u_attn_head_slices.txt)
static int attn_hsplit(int T, int G, int qpk, int n_splits) {
  int h = 1;
  if (T == 1 && n_splits > 1)
    while (h < qpk && G * h * n_splits <= 128) h *= 2;
  if (const char* e = getenv("LGA_ATTN_HSPLIT")) {  // lab A/B
    const int v = atoi(e);
    if (v >= 1 && v <= qpk && qpk % v == 0) h = v;
  }
  return h;
}

template <int HS, bool FUSED>
static int launch_hs(const void* q, void* kc, void* vc, const int64_t* pos, void* y, float* ws, unsigned* cnt, int T,
                     int H, int G, int max_seq, int n_splits, float scale, const int64_t* rope_pos, const float* cos,
                     const float* sin, int rope_rows, hipStream_t stream) {
  const int hsplit = attn_hsplit(T, G, H / G, n_splits);
  const dim3 grid(n_splits, G * hsplit, T);
#define LGA_ATTN(QPK, CFG)                                                                                        \
  launch_one<HS, QPK, CFG, FUSED>(grid, stream, q, kc, vc, pos, y, ws, cnt, H, max_seq, scale, rope_pos, cos, sin, \
                                  rope_rows, hsplit)
  switch (H / G / hsplit) {
    case 1:  // one head per group: 8 waves x 2 keys in flight when the groups are few (TP ranks: G = 4 7.9 vs 8.2 us,
             // G = 8 8.0 vs 8.7 at 16 splits; profiles/r04u_attn_head_slices.txt), else 4 x 4 (Llama-2-7B, G = 32)
      if (G * hsplit <= 16) LGA_ATTN(1, LGA_ATTN_Q1_FEW);
      else LGA_ATTN(1, LGA_ATTN_Q1);
      break;
    case 2: LGA_ATTN(2, LGA_ATTN_Q2); break;
    case 4: LGA_ATTN(4, LGA_ATTN_Q4); break;
    case 8: LGA_ATTN(8, LGA_ATTN_Q8); break;
    default: lga_set_error("lga_attention: q_per_kv must be 1, 2, 4 or 8"); return (int)hipErrorInvalidValue;
  }
#undef LGA_ATTN
  return 0;
}

}  // namespace lga

int lga::preload_attention() {
  return lga::preload(lga::attn_prefill_kernel<128>) + lga::preload(lga::attn_prefill_kernel<64>) +
         lga::preload(lga::attn_prefill_pair_kernel<128>) + lga::preload(lga::attn_prefill_pair_kernel<64>);
}

extern "C" int lga_attention(const void* q, const void* k_cache, const void* v_cache, const int64_t* input_pos,
                             void* y, float* workspace, unsigned* counters, int T, int n_head, int n_query_groups,
                             int head_size, int max_seq, int n_splits, float scale, hipStream_t stream) {
  LGA_CHECK_ARG(q && k_cache && v_cache && input_pos && y, "lga_attention: null pointer");
  LGA_CHECK_ARG(T > 0 && n_query_groups > 0 && n_head % n_query_groups == 0, "lga_attention: bad head geometry");
  LGA_CHECK_ARG(n_splits >= 1 && n_splits <= 256, "lga_attention: n_splits must be in [1, 256]");
  LGA_CHECK_ARG(n_splits == 1 || (workspace && counters), "lga_attention: split attention needs workspace + counters");
  if (T >= 16 && n_splits == 1 && (head_size == 128 || head_size == 64)) {  // prefill: flash attention on MFMA
#ifndef LGA_FA_PAIR
#define LGA_FA_PAIR 1
#endif
    if (LGA_FA_PAIR) {
      const dim3 grid((((T + 127) / 128 + 1) / 2) * n_head);
      if (head_size == 128)
        lga::attn_prefill_pair_kernel<128><<<grid, 512, 0, stream>>>((const uint16_t*)q, (const uint16_t*)k_cache,
                                                                     (const uint16_t*)v_cache, input_pos, (uint16_t*)y,
                                                                     T, n_head, n_query_groups, max_seq, scale);
      else
        lga::attn_prefill_pair_kernel<64><<<grid, 512, 0, stream>>>((const uint16_t*)q, (const uint16_t*)k_cache,
                                                                    (const uint16_t*)v_cache, input_pos, (uint16_t*)y,
                                                                    T, n_head, n_query_groups, max_seq, scale);
      LGA_LAUNCH_RETURN();
    }
    const dim3 grid(((T + 127) / 128) * n_head);
    if (head_size == 128)
      lga::attn_prefill_kernel<128><<<grid, 256, 0, stream>>>((const uint16_t*)q, (const uint16_t*)k_cache,
                                                              (const uint16_t*)v_cache, input_pos, (uint16_t*)y, T,
                                                              n_head, n_query_groups, max_seq, scale, 1);
    else
      lga::attn_prefill_kernel<64><<<grid, 256, 0, stream>>>((const uint16_t*)q, (const uint16_t*)k_cache,
                                                             (const uint16_t*)v_cache, input_pos, (uint16_t*)y, T,
                                                             n_head, n_query_groups, max_seq, scale, 1);
    LGA_LAUNCH_RETURN();
  }
  int rc;
  if (head_size == 128)
    rc = lga::launch_hs<128, false>((const void*)q, (void*)k_cache, (void*)v_cache, input_pos, y, workspace, counters,
                                    T, n_head, n_query_groups, max_seq, n_splits, scale, nullptr, nullptr, nullptr, 0,
                                    stream);
  else if (head_size == 64)
    rc = lga::launch_hs<64, false>((const void*)q, (void*)k_cache, (void*)v_cache, input_pos, y, workspace, counters,
                                   T, n_head, n_query_groups, max_seq, n_splits, scale, nullptr, nullptr, nullptr, 0,
                                   stream);
  else {
    lga_set_error("lga_attention: head_size must be 64 or 128");
    return (int)hipErrorInvalidValue;
  }
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}

// Decode step (T = 1) with RoPE + KV-append fused in: qkv is the fused projection row ([G][q_per_kv + 2][hs]
// bf16); q and k are roped with cos/sin row rope_pos[0], k and v are written to the caches at cache_pos[0] and
// the attention output over keys 0..cache_pos[0] lands in y ([n_head][hs]). Replaces lga_rope_kv_append +
// lga_attention for a token step; full rotary only (rope_n_elem == head_size == 128).
extern "C" int lga_attention_decode_fused(const void* qkv, void* k_cache, void* v_cache, const int64_t* cache_pos,
                                          const int64_t* rope_pos, const float* cos, const float* sin, int rope_rows,
                                          void* y, float* workspace, unsigned* counters, int n_head,
                                          int n_query_groups, int head_size, int rope_n_elem, int max_seq,
                                          int n_splits, float scale, hipStream_t stream) {
  LGA_CHECK_ARG(qkv && k_cache && v_cache && cache_pos && rope_pos && cos && sin && y,
                "lga_attention_decode_fused: null pointer");
  LGA_CHECK_ARG(n_query_groups > 0 && n_head % n_query_groups == 0, "lga_attention_decode_fused: bad head geometry");
  LGA_CHECK_ARG(head_size == 128 && rope_n_elem == 128,
                "lga_attention_decode_fused: needs head_size == rope_n_elem == 128 (use rope_kv_append + attention)");
  LGA_CHECK_ARG(rope_rows > 0 && max_seq > 0, "lga_attention_decode_fused: empty rope cache or kv cache");
  LGA_CHECK_ARG(n_splits >= 1 && n_splits <= 256, "lga_attention_decode_fused: n_splits must be in [1, 256]");
  LGA_CHECK_ARG(n_splits == 1 || (workspace && counters),
                "lga_attention_decode_fused: split attention needs workspace + counters");
  const int rc = lga::launch_hs<128, true>(qkv, k_cache, v_cache, cache_pos, y, workspace, counters, 1, n_head,
                                           n_query_groups, max_seq, n_splits, scale, rope_pos, cos, sin, rope_rows,
                                           stream);
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}

#ifdef LGA_ATTN_TRACE
extern "C" int lga_attn_trace_read(unsigned long long* host, int n) {
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(lga::g_attn_trace), (size_t)n * sizeof(unsigned long long));
  void* dptr = nullptr;
  if (e == hipSuccess) e = hipGetSymbolAddress(&dptr, HIP_SYMBOL(lga::g_attn_trace));
  if (e == hipSuccess) e = hipMemset(dptr, 0, sizeof(lga::g_attn_trace));  // read-and-clear
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}
#endif

// fp32 partials (T * H * n_splits * (hs + 4)); the counters (T * n_head * 64 uint32: one per (row, query group, head
// slice) at a 256-B stride) must be zeroed once at allocation
extern "C" size_t lga_attention_workspace_bytes(int T, int n_head, int head_size, int n_splits) {
  return (size_t)T * n_head * (n_splits < 1 ? 1 : n_splits) * (head_size + 4) * sizeof(float);
}
