// Decode step: fused RMSNorm + qkv GEMV + RoPE + KV append + split attention in ONE launch, the attention's K/V
// stream issued right behind the qkv weight stream.
//
// STATUS (round 5): correct (bit-identical q/k/v, tests/test_gpu_kernels.py) but NOT the default: opt in with
// LGA_FUSE_QKV=1. Measured with tools/qkv_attn_ab.py (32 blocks, one graph): 28.1-28.5 us per block against
// 19.2-19.6 us for lga_q4_gemv + lga_attention_decode_fused. tools/qkv_attn_trace.py shows why: once the first
// workgroups issue their K/V, the qkv weights of the others return late (rows done 5.5 .. 19 us), and the group
// exchange waits for the slowest member. Variants measured and dropped: K/V waves issuing at kernel start (roles
// split, 27.6 us), K/V after all 48 rows of the workgroup (29.5 us), x staged by one wave (31.9 us).
//
// Replaces, for one token, the pair "norm_1 + self.attn(x) (the fused qkv Linear, reference lit_gpt/model.py:619,
// bnb gemv_4bit)" then "RoPE + KVCache.forward + SDPA (model.py:620-651, 788-795, 658-665)" that lga_q4_gemv +
// lga_attention_decode_fused run as two launches. The K/V rows of the positions before p do not depend on this
// token, so the only thing the attention waits for is its query: every workgroup issues its share of the qkv weights
// AND of the K/V cache into registers at once, computes its qkv rows while both stream, exchanges the rows inside
// its query group, and scores the already-resident keys. The HBM stream of both ops runs back to back inside one
// launch instead of two, and the attention's ramp hides under the GEMV.
//
// Geometry (the Llama-2-7B decode step at TP = 1, lga_qkv_attention_supported): MHA (n_head == n_query_groups,
// q_per_kv 1), hs 128, C = 4096, 8 splits: grid (8, G), 768 threads = 12 waves per workgroup; a group's 384 qkv rows
// ([q, k, v] x 128, scripts/convert_hf_checkpoint.py:181-187) are split 48 per workgroup = 4 rows per wave.
//  * qkv rows: exactly lga_q4_gemv's arithmetic for this shape (RMSNorm on threads 0..255 as its 4-wave workgroup
//    does, 4 rows x 2 chunks per lane, butterfly<4>), so q, k, v are bit-identical to the two-launch path.
//  * waves 0..10 hold the split's keys: row group rg = wave * 4 + lane / 16 (44 of them), key k_lo + rg + 44 u for
//    u < NKV in registers (NKV = 7: 308 keys per split, p <= 2463 with 8 splits); keys past that stream afterwards.
//    They are issued right after the wave's qkv rows, so the K/V stream queues behind the qkv weights; the waves
//    meet through LDS words, not barriers, until the attention math (a barrier would wait for every wave to have
//    issued all its K/V loads, which stalls while the CU's memory queue is full).
//  * wave 11 (no K/V loads: its vmcnt drains only its own stores) publishes the workgroup's 48 rows write-through,
//    arrives on the group's counter, polls it, and loads + ropes the group's q (and k, v for the split that owns p).
//  * the attention math per key is attn_kernel's; the online-softmax grouping differs (44 row groups, not 16), so y
//    agrees with lga_attention_decode_fused within fp32 summation order. Split publish / last-arriver combine as
//    attn_kernel (MI355X_MICROARCH.md "Valid forms" row 1).
#include "decode_ops.h"

namespace lga {

namespace qa {

#ifdef LGA_QA_TRACE  // lab builds only (tools/qkv_attn_trace.py): per-workgroup phase stamps, 100 MHz clock
__device__ unsigned long long g_qa_trace[4096 * 8];
#define QA_TRACE_T(i, tid)                                                                              \
  do {                                                                                                  \
    if (threadIdx.x == (tid))                                                                           \
      g_qa_trace[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define QA_TRACE(i) QA_TRACE_T(i, 0)
#else
#define QA_TRACE_T(i, tid) \
  do {                     \
  } while (0)
#define QA_TRACE(i) QA_TRACE_T(i, 0)
#endif

constexpr int HS = 128, C = 4096, SPLITS = 8, ROWS = 48, NT = 12 * 64;
// every wave computes 4 of the workgroup's 48 qkv rows; waves 0..10 then hold the keys, wave 11 publishes the rows
constexpr int PASSES = 1, NKW = 11, RGK = NKW * 4, PUB = 11;
constexpr int NC = C / 32, N8 = C / 8, KCH = 2;  // 32-element chunks, uint4 of x, chunks per lane
constexpr int kCounterStride = 64;



struct Args {
  const uint16_t* x;       // [C] the Block input (norm_1 fused)
  const uint16_t* norm_w;  // [C]
  float eps;
  const uint8_t* qw;  // [G * 384][C / 2]
  const void* sc;     // scales
  const uint16_t* bias;  // [G * 384] or null
  int group, cb;
  uint16_t* qkv;  // [G * 384] scratch: the rows, handed between the workgroups of a group (sc1)
  uint16_t* kc;
  uint16_t* vc;
  const int64_t* cache_pos;
  const int64_t* rope_pos;
  const float* cos;
  const float* sin;
  int rope_rows, max_seq;
  float scale;
  uint16_t* y;   // [H * HS]
  float* ws;     // [H][SPLITS][HS + 4] partials
  unsigned* cnt;   // [H] * 64 split arrival counters (re-armed)
  unsigned* gsync;  // [2 G] * 64: group row counters (monotonic) and their per-launch bases
};

template <int FMT, int NKV>
__global__ void __launch_bounds__(NT) qkv_attn_kernel(Args a) {
  constexpr int LPR = 16, NGW = 12;
  __shared__ __attribute__((aligned(16))) uint4 xl[N8];  // x pairs (stage_x8 layout)
  __shared__ float xsum[NC];
  __shared__ float nf4s[16];
  __shared__ __attribute__((aligned(16))) uint16_t rows[ROWS];
  __shared__ __attribute__((aligned(16))) float qs[HS], ks[HS], vs[HS];  // roped q; roped k and v of key p
  __shared__ float sm[NKW], sl[NKW];
  __shared__ __attribute__((aligned(16))) float so[NKW][HS];
  __shared__ unsigned s_last, s_rows, s_q;
  __shared__ float red[4];

  const int split = blockIdx.x, g = blockIdx.y, G = gridDim.y;
  const int t = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;  // wave: scalar
  QA_TRACE(0);
  // scalar state first: positions and the group counter's base for this launch
  const long p = a.cache_pos[0];
  const long rp = min(max(a.rope_pos[0], 0L), (long)a.rope_rows - 1);
  const unsigned gbase = a.gsync[(G + g) * kCounterStride];
  const int L = (int)min(p + 1, (long)a.max_seq);
  const int chunk = (L + SPLITS - 1) / SPLITS;
  const int k_lo = split * chunk;
  const int k_hi = min(k_lo + chunk, L);
  const bool owns_new = p < a.max_seq && k_lo <= p && p < k_hi;
  const int k_end = min(k_hi, (int)p);  // key p is scored from LDS below
  if (t == 0) {
    s_rows = s_q = 0;
  }
  if (FMT == 1 && t < 16) nf4s[t] = kCode4[a.cb][t];  // (both are read after the RMSNorm barriers below)

  const int kw = wave, rg = kw * 4 + lane / LPR, sub = lane % LPR;  // K/V waves' row group
  const bool kv_wave = wave < NKW;
  const uint16_t* kbase = a.kc + (size_t)g * a.max_seq * HS + sub * 8;
  const uint16_t* vbase = a.vc + (size_t)g * a.max_seq * HS + sub * 8;
  uint4 kr[NKV], vr[NKV];
  auto lds_wait = [](unsigned* w, unsigned target) {
    while (__hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
  };
  auto lds_arrive = [&](unsigned* w) {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes are done
    if (lane == 0) __hip_atomic_fetch_add(w, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  };

  // ---- loads: x + norm weight first (threads 0..255 in lga_q4_gemv's 4-wave layout; the other waves load the same
  // pieces so every wave's vmcnt accounting is the same), then the wave's 4 qkv rows x 2 chunks ----
  uint4 xr[2], nr[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    xr[i] = ((const uint4*)a.x)[(t & 255) + 256 * i];
    nr[i] = ((const uint4*)a.norm_w)[(t & 255) + 256 * i];
  }
  __builtin_amdgcn_sched_barrier(0);  // x and the norm weight issue before the weights
  uint4 w[PASSES][4][KCH];
  uint32_t sc[PASSES][4][KCH], bias_bits[PASSES];
  const int rbase = g * 3 * HS + split * ROWS + wave * 4;  // pass k: rows rbase + 4 NGW k .. + 3
#pragma unroll
  for (int k = 0; k < PASSES; ++k) {
#pragma unroll
    for (int j = 0; j < KCH; ++j) {
      const int c = lane + 64 * j;
      const int gi = (c * 32) / a.group;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const size_t n = (size_t)(rbase + 4 * NGW * k + i);
        w[k][i][j] = ld_nt16(a.qw + n * (C / 2) + (size_t)c * 16);
        sc[k][i][j] = load_scale_bits<FMT>(a.sc, n * (C / a.group) + gi);
      }
    }
  }
  // bias without a branch: a null bias is a zero-sized buffer (out-of-range buffer loads return 0)
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
      a.bias ? (void*)a.bias : (void*)a.qw, (short)0, a.bias ? (3 * HS) * G * 2 : 0, 0x00020000);
#pragma unroll
  for (int k = 0; k < PASSES; ++k)
    bias_bits[k] = __builtin_amdgcn_raw_buffer_load_b16(brs, (rbase + 4 * NGW * k + bfly_index<4>(lane)) * 2, 0, 0);
  // RMSNorm: lga_q4_gemv's order (per-wave sums, then ((r0 + r1) + (r2 + r3)))
  {
    float ss = 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float lo = bflo(d[q]), hi = bfhi(d[q]);
        ss = fmaf(lo, lo, ss);
        ss = fmaf(hi, hi, ss);
      }
    }
    ss = wave_sum_uniform(ss);
    if (wave < 4 && lane == 0) red[wave] = ss;
  }
  __syncthreads();
  if (wave < 4) {
    const float tot = (red[0] + red[1]) + (red[2] + red[3]);
    const float rs = 1.0f / sqrtf(tot / (float)C + a.eps);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int u = t + 256 * i;
      uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
      const uint32_t nw[4] = {nr[i].x, nr[i].y, nr[i].z, nr[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        d[q] = pack2(__fmul_rn(bflo(nw[q]), __fmul_rn(bflo(d[q]), rs)),
                     __fmul_rn(bfhi(nw[q]), __fmul_rn(bfhi(d[q]), rs)));
      uint4 xv;
      float cs = stage_x8<FMT>(d, xv);
      cs += __shfl_xor(cs, 1);
      cs += __shfl_xor(cs, 2);
      xl[u] = xv;
      if ((u & 3) == 0) xsum[u >> 2] = cs;
    }
  }
  __syncthreads();
  QA_TRACE(1);  // x staged
  {
    // the rows: gemv_q4_body's dot + butterfly per pass of 4 rows (each row's arithmetic as lga_q4_gemv's)
    const uint32_t nmask = nibble_mask(), nmagic = f16_magic(), nmask_hi = nibble_mask_hi();
#pragma unroll
    for (int k = 0; k < PASSES; ++k) {
      float part[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int j = 0; j < KCH; ++j) {
        const int c = lane + 64 * j;
        uint4 wj[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) wj[i] = w[k][i][j];
        float d[4];
        chunk_dot_rows<FMT, 4>(wj, xl + c * 4, xsum[c], nf4s, nmask, nmagic, nmask_hi, d);
#pragma unroll
        for (int i = 0; i < 4; ++i) part[i] = fmaf(scale_of<FMT>(sc[k][i][j]), d[i], part[i]);
      }
      const float tt = butterfly<4>(part, lane);
      const int vi = bfly_index<4>(lane);
      float o = tt;
      if (a.bias) o += bf2f((uint16_t)bias_bits[k]);  // (a zero-sized buffer read 0 when there is none)
      if ((lane & 15) == 0) rows[4 * NGW * k + wave * 4 + vi] = f2bf(o);
    }
    lds_arrive(&s_rows);
    if (wave == 0) QA_TRACE(2);  // this wave's qkv rows computed
  }
  if (kv_wave) {
    // ---- K/V waves: the split's keys into registers, queued behind the wave's (consumed) qkv weights ----
#pragma unroll
    for (int u = 0; u < NKV; ++u) {
      const int j = max(min(k_lo + rg + RGK * u, k_end - 1), 0);  // clamped rows are masked below
      kr[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load((const u32x4_t*)(kbase + (size_t)j * HS)));
      vr[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load((const u32x4_t*)(vbase + (size_t)j * HS)));
    }
  }
  if (wave == PUB) {
    // ---- wave 11 (no K/V loads in flight: its vmcnt drains only its own stores): publish the 48 rows to the group,
    // wait for the group, q (k, v) roped ----
    lds_wait(&s_rows, 12);
    const int base_row = g * 3 * HS + split * ROWS;
    if (lane < ROWS / 4) {  // 12 lanes x 8 B, write-through
      const uint2 v2 = *(const uint2*)&rows[lane * 4];
      __hip_atomic_store((unsigned long long*)(a.qkv + base_row + lane * 4),
                         ((unsigned long long)v2.y << 32) | v2.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // only this wave's stores drain
    unsigned* gc = a.gsync + g * kCounterStride;
    if (lane == 0) {
      const unsigned prev = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == gbase + SPLITS - 1)  // every workgroup of the group has read the base (it arrived here)
        __hip_atomic_store(a.gsync + (G + g) * kCounterStride, gbase + SPLITS, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while ((int)(__hip_atomic_load(gc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - (gbase + SPLITS)) < 0 &&
             __builtin_amdgcn_s_memrealtime() - t0 < 100000000ull)  // bounded (1 s): never hangs the GPU
        __builtin_amdgcn_s_sleep(1);
    }
    // every lane: its 16-B pieces of q (and k, v) by sc1 loads — issued by the polling wave after its poll matched
    const __amdgpu_buffer_rsrc_t grs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.qkv + (size_t)g * 3 * HS), (short)0, 3 * HS * 2, 0x00020000);
    if (lane < 16) {
      const float* cr = a.cos + (size_t)rp * HS + lane * 8;
      const float* sr = a.sin + (size_t)rp * HS + lane * 8;
      const u32x4_t qv = __builtin_amdgcn_raw_buffer_load_b128(grs, lane * 16, 0, 16);  // sc1
      float f[8];
      unpack8(rope8(__builtin_bit_cast(uint4, qv), cr, sr, lane), f);
#pragma unroll
      for (int i = 0; i < 8; ++i) qs[lane * 8 + i] = f[i];
      if (owns_new) {
        const u32x4_t kv = __builtin_amdgcn_raw_buffer_load_b128(grs, (HS + lane * 8) * 2, 0, 16);
        const u32x4_t vv = __builtin_amdgcn_raw_buffer_load_b128(grs, (2 * HS + lane * 8) * 2, 0, 16);
        const uint4 kro = rope8(__builtin_bit_cast(uint4, kv), cr, sr, lane);
        const uint4 vro = __builtin_bit_cast(uint4, vv);
        *(uint4*)(a.kc + ((size_t)g * a.max_seq + p) * HS + lane * 8) = kro;  // KVCache.forward at p
        *(uint4*)(a.vc + ((size_t)g * a.max_seq + p) * HS + lane * 8) = vro;
        unpack8(kro, f);
#pragma unroll
        for (int i = 0; i < 8; ++i) ks[lane * 8 + i] = f[i];
        unpack8(vro, f);
#pragma unroll
        for (int i = 0; i < 8; ++i) vs[lane * 8 + i] = f[i];
      }
    }
    lds_arrive(&s_q);
    QA_TRACE_T(3, PUB * 64);  // group rows exchanged, q roped
  }

  // ---- attention over the resident keys (K/V waves), then the keys past the register window ----
  if (kv_wave) {
    lds_wait(&s_q, 1);
    float m = -INFINITY, l = 0.0f, o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = 0.0f;
    float qf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) qf[i] = qs[sub * 8 + i];
    auto score = [&](const uint4 kv) {
      float kf[8];
      unpack8(kv, kf);
      float d = 0.0f;
#pragma unroll
      for (int i = 0; i < 8; ++i) d = fmaf(qf[i], kf[i], d);
      return row_group_sum<LPR>(d) * a.scale;
    };
    // a row group whose first key is past the split scores nothing (keeps m = -inf, l = 0, o = 0)
    if (k_lo + rg < k_end) {
      float scv[NKV];
      float mx = m;
#pragma unroll
      for (int u = 0; u < NKV; ++u) {
        const float sd = score(kr[u]);
        scv[u] = (k_lo + rg + RGK * u < k_end) ? sd : -INFINITY;
        mx = fmaxf(mx, scv[u]);
      }
      // m = -inf: the first update (no rescale needed, o and l are 0)
#pragma unroll
      for (int u = 0; u < NKV; ++u) {
        const float e = expf(scv[u] - mx);
        l += e;
        float vf[8];
        unpack8(vr[u], vf);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = fmaf(e, vf[i], o[i]);
      }
      m = mx;
      // keys past the register window (long contexts): streamed two per row group at a time
      for (int j0 = k_lo + rg + RGK * NKV; j0 < k_end; j0 += RGK * 2) {
        uint4 kk[2], vv[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int j = min(j0 + RGK * u, k_end - 1);
          kk[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load((const u32x4_t*)(kbase + (size_t)j * HS)));
          vv[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load((const u32x4_t*)(vbase + (size_t)j * HS)));
        }
        float s2[2];
        float mx2 = m;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const float sd = score(kk[u]);
          s2[u] = (j0 + RGK * u < k_end) ? sd : -INFINITY;
          mx2 = fmaxf(mx2, s2[u]);
        }
        const float c = expf(m - mx2);
        l *= c;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] *= c;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const float e = expf(s2[u] - mx2);
          l += e;
          float vf[8];
          unpack8(vv[u], vf);
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = fmaf(e, vf[i], o[i]);
        }
        m = mx2;
      }
    }
    if (owns_new && rg == 0) {  // the new key / value, scored from LDS
      float kf[8], vf[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        kf[i] = ks[sub * 8 + i];
        vf[i] = vs[sub * 8 + i];
      }
      float d = 0.0f;
#pragma unroll
      for (int i = 0; i < 8; ++i) d = fmaf(qf[i], kf[i], d);
      const float sn = row_group_sum<LPR>(d) * a.scale;
      const float mx = fmaxf(m, sn);
      const float c = expf(m - mx);  // m = -inf (no earlier key in this row group) -> 0
      const float e = expf(sn - mx);
      l = l * c + e;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = fmaf(e, vf[i], o[i] * c);
      m = mx;
    }
    // merge the 4 row groups of this wave
#pragma unroll
    for (int off = LPR; off < 64; off <<= 1) {
      const float mo = __shfl_xor(m, off), lo = __shfl_xor(l, off);
      const float mn = fmaxf(m, mo);
      const float ca = mn == -INFINITY ? 0.0f : expf(m - mn);
      const float cb = mn == -INFINITY ? 0.0f : expf(mo - mn);
      l = l * ca + lo * cb;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = o[i] * ca + __shfl_xor(o[i], off) * cb;
      m = mn;
    }
    if (lane < LPR) {
      if (lane == 0) {
        sm[kw] = m;
        sl[kw] = l;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) so[kw][sub * 8 + i] = o[i];
    }
  }
  __syncthreads();
  QA_TRACE(4);  // keys scored (the K/V landed)
  // ---- 6. block merge (one output column per thread), publish, last-arriving split combines ----
  const size_t hrow = (size_t)g;  // MHA: head g
  if (t < HS) {
    float mx = -INFINITY;
#pragma unroll
    for (int w2 = 0; w2 < NKW; ++w2) mx = fmaxf(mx, sm[w2]);
    float lt = 0.0f, ot = 0.0f;
#pragma unroll
    for (int w2 = 0; w2 < NKW; ++w2) {
      const float c = mx == -INFINITY ? 0.0f : expf(sm[w2] - mx);
      lt += sl[w2] * c;
      ot += so[w2][t] * c;
    }
    float* wsr = a.ws + (hrow * SPLITS + split) * (HS + 4);
    st_sc1(wsr + 4 + t, ot);
    if (t == 0) {
      st_sc1(wsr, mx);
      st_sc1(wsr + 1, lt);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  unsigned* ctr = a.cnt + hrow * kCounterStride;
  if (t == 0) s_last = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  QA_TRACE(5);  // published + arrival returned
  if (s_last != (unsigned)(SPLITS - 1)) return;
  if (t < HS) {
    const float* base = a.ws + hrow * SPLITS * (HS + 4);
    float mv[SPLITS], lv[SPLITS], ov[SPLITS];
#pragma unroll
    for (int u = 0; u < SPLITS; ++u) {
      const float* r = base + u * (HS + 4);
      mv[u] = ld_sc1(r);
      lv[u] = ld_sc1(r + 1);
      ov[u] = ld_sc1(r + 4 + t);
    }
    float nm = -INFINITY;
#pragma unroll
    for (int u = 0; u < SPLITS; ++u) nm = fmaxf(nm, mv[u]);
    float lt = 0.0f, ot = 0.0f;
#pragma unroll
    for (int u = 0; u < SPLITS; ++u) {
      const float e = expf(mv[u] - nm);  // empty splits: m = -inf -> 0
      lt = fmaf(lv[u], e, lt);
      ot = fmaf(ov[u], e, ot);
    }
    a.y[hrow * HS + t] = f2bf(ot / lt);
  }
  if (t == 0) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  QA_TRACE(6);  // combined (last split)
}

}  // namespace qa
}  // namespace lga

extern "C" int lga_qkv_attention_supported(int n_embd, int n_head, int n_query_groups, int head_size, int n_splits,
                                           int group, int fmt) {
  return n_embd == lga::qa::C && n_head == n_query_groups && head_size == lga::qa::HS &&
         n_splits == lga::qa::SPLITS && group >= 32 && group % 32 == 0 && lga::qa::C % group == 0 &&
         (fmt == 0 || fmt == 1 || fmt == 3);
}

extern "C" int lga_qkv_attention_decode(const void* x, const void* norm_weight, float norm_eps, const uint8_t* qweight,
                                        const void* scales, const void* bias, int group, int fmt, void* qkv_scratch,
                                        void* k_cache, void* v_cache, const int64_t* cache_pos, const int64_t* rope_pos,
                                        const float* cos, const float* sin, int rope_rows, void* y, float* workspace,
                                        unsigned* counters, unsigned* group_sync, int n_head, int n_query_groups,
                                        int head_size, int max_seq, int n_splits, float scale, hipStream_t stream) {
  LGA_CHECK_ARG(x && norm_weight && qweight && scales && qkv_scratch && k_cache && v_cache && cache_pos && rope_pos &&
                    cos && sin && y && workspace && counters && group_sync,
                "lga_qkv_attention_decode: null pointer");
  LGA_CHECK_ARG(lga_qkv_attention_supported(lga::qa::C, n_head, n_query_groups, head_size, n_splits, group, fmt),
                "lga_qkv_attention_decode: geometry not covered (lga_qkv_attention_supported)");
  LGA_CHECK_ARG(rope_rows > 0 && max_seq > 0, "lga_qkv_attention_decode: empty rope cache or kv cache");
  lga::qa::Args a{(const uint16_t*)x, (const uint16_t*)norm_weight, norm_eps, qweight, scales, (const uint16_t*)bias,
                  group, lga::codebook_of(fmt), (uint16_t*)qkv_scratch, (uint16_t*)k_cache, (uint16_t*)v_cache,
                  cache_pos, rope_pos, cos, sin, rope_rows, max_seq, scale, (uint16_t*)y, workspace, counters,
                  group_sync};
  const dim3 grid(lga::qa::SPLITS, n_query_groups);
  if (lga::kernel_fmt(fmt) == 0)
    lga::qa::qkv_attn_kernel<0, 7><<<grid, lga::qa::NT, 0, stream>>>(a);
  else
    lga::qa::qkv_attn_kernel<1, 7><<<grid, lga::qa::NT, 0, stream>>>(a);
  LGA_LAUNCH_RETURN();
}

#ifdef LGA_QA_TRACE
extern "C" int lga_qa_trace_read(unsigned long long* host, int n) {
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(lga::qa::g_qa_trace), (size_t)n * sizeof(unsigned long long));
  void* dptr = nullptr;
  if (e == hipSuccess) e = hipGetSymbolAddress(&dptr, HIP_SYMBOL(lga::qa::g_qa_trace));
  if (e == hipSuccess) e = hipMemset(dptr, 0, sizeof(lga::qa::g_qa_trace));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}
#endif
