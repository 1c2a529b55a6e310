// One Llama decode block (lit_gpt/model.py Block.forward :572-593 for T = 1) as ONE persistent launch.
//
// Why: the per-op path launches 5 kernels per block (rmsnorm+qkv GEMV, fused rope/KV/attention, proj GEMV +
// residual, rmsnorm+fc_1/fc_2 SwiGLU GEMV, mlp.proj GEMV + residual). Each pays a launch ramp and a tail in which
// HBM idles while the last waves finish, and the next op cannot start streaming its weights until the boundary.
// Here every stage's weights (and the attention's K/V rows) are loaded BEFORE the stage waits for its input, so
// the weight stream of stage s+1 runs during stage s's tail and the dependency hand-off.
//
// Grid: exactly one 1024-thread workgroup per CU (NB = #CUs, > 80 KB of LDS forces one per CU, so every
// workgroup is resident and the spin-waits below cannot deadlock; every spin is also bounded and reports a
// timeout through *err instead of hanging). Workgroup b owns:
//   S1 qkv rows      [b*R1*16, ...)      (RMSNorm(norm_1) of h_in fused)        -> qkv scratch, counter qkv[g]
//   S2 attention     query group g = b / (NB/G), sequence split b % (NB/G)      -> y scratch (last-arriver merge)
//   S3 attn.proj     rows [b*R3*16, ...) + residual h_in                         -> h_mid
//   S4 fc_1 || fc_2  rows [b*R4*16, ...) (RMSNorm(norm_2) of h_mid fused), SwiGLU -> act
//   S5 mlp.proj      rows [b*R5*16, ...) + residual h_mid (kept in LDS: the same rows as S3) -> h_out
// Hand-offs between workgroups follow MI355X_MICROARCH.md "Valid forms" row 1: every stored byte is an sc1
// (write-through) store, the storing wave drains them (s_waitcnt vmcnt(0)) before ONE lane's agent-scope atomic
// add; consumers poll that counter with sc1 loads and read the bytes with sc1 loads after a workgroup barrier.
// The storing wave is always wave 0 (outputs gathered in LDS), so the other waves' weight prefetches are never
// drained by the publish wait (vmcnt is per wave).
#include "decode_ops.h"

namespace lga {

struct LayerArgs {
  const uint16_t* h_in;
  uint16_t* h_mid;
  uint16_t* h_out;
  const uint16_t* norm1;
  const uint16_t* norm2;
  float eps;
  const uint8_t* wq;  // [Nq][C/2], scales [Nq][C/128] (Nq = (H + 2G) * hs)
  const uint16_t* sq;
  const uint8_t* wo;  // [C][C/2]
  const uint16_t* so;
  const uint8_t* w1;  // [I][C/2]
  const uint16_t* s1;
  const uint8_t* w2;
  const uint16_t* s2;
  const uint8_t* wd;  // [C][I/2], scales [C][I/128]
  const uint16_t* sd;
  uint16_t* kc;  // [G][S][hs]
  uint16_t* vc;
  const float* cos;  // [rope_rows][hs]
  const float* sin;
  int rope_rows;
  const int64_t* pos;  // the token's position (cache row and rope row)
  uint16_t* qkv;       // scratch [Nq]
  uint16_t* yatt;      // scratch [H*hs]
  uint16_t* act;       // scratch [I]
  float* ws;           // attention partials [H][splits][hs + 4]
  unsigned* cnt;       // counters, 64 uint32 apart: qkv[G], split[G], attn, o, gu, exit
  unsigned* err;       // bit 0: a spin-wait timed out
  int C, I, H, G, S;
  float scale;
};

constexpr int LNW = 8;            // waves per workgroup (one workgroup per CU: ~240 VGPRs -> 2 waves per SIMD)
constexpr int LNT = LNW * 64;     // threads
constexpr int LCS = 64;           // counter stride (uint32)
constexpr int kGroupQ4 = 128;     // int4 group size this kernel is built for

#ifdef LGA_LAYER_TRACE  // lab builds only (tools/layer_trace.py): per-workgroup phase stamps, 100 MHz clock
__device__ unsigned long long g_layer_trace[1024 * 16];
#define LGA_LTRACE(i)                                                                                 \
  do {                                                                                                \
    if (threadIdx.x == 0) g_layer_trace[(size_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define LGA_LTRACE(i) \
  do {                \
  } while (0)
#endif

__device__ __forceinline__ unsigned* ctr(const LayerArgs& a, int i) { return a.cnt + (size_t)i * LCS; }

__device__ __forceinline__ uint32_t ld_sc1_u32(const void* p) {
  return __hip_atomic_load((const uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_u32(void* p, uint32_t v) {
  __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint4 ld_sc1_u4(const void* p) {
  const uint32_t* q = (const uint32_t*)p;
  return make_uint4(ld_sc1_u32(q), ld_sc1_u32(q + 1), ld_sc1_u32(q + 2), ld_sc1_u32(q + 3));
}

// thread 0 polls until *c >= target (bounded: ~20 ms, then flags *err and continues), then the workgroup syncs
__device__ __forceinline__ void wait_count(const LayerArgs& a, unsigned* c, unsigned target) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (ld_sc1_u32(c) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) {
        __hip_atomic_fetch_or(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

// wave 0 only: after its sc1 stores, drain them and bump the counter
__device__ __forceinline__ void publish(unsigned* c) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------------ weight tiles
template <int RPR, int CPT, bool DUAL>
struct Tile {
  uint4 w[RPR][CPT];
  uint4 w2[DUAL ? RPR : 1][DUAL ? CPT : 1];
  uint32_t s[RPR][CPT];
  uint32_t s2[DUAL ? RPR : 1][DUAL ? CPT : 1];
};

// rows row0 .. row0 + nrows - 1 of an int4-g128 matrix [N][K/2] (rows past nrows re-read the wave's last valid
// row, or row N-1 when the wave has none: never stored)
template <int RPR, int CPT, bool DUAL>
__device__ __forceinline__ void tile_load(Tile<RPR, CPT, DUAL>& T, const uint8_t* w, const uint16_t* s,
                                          const uint8_t* w2, const uint16_t* s2, int row0, int nrows, int N, int K,
                                          int lane) {
  const int NC = K / 32, groups = K / kGroupQ4;
#pragma unroll
  for (int i = 0; i < RPR; ++i) {
    const int r = nrows > 0 ? row0 + min(i, nrows - 1) : N - 1;
    const size_t rb = (size_t)r * (K / 2);
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int c = min(lane + 64 * j, NC - 1);
      T.w[i][j] = ld_nt16(w + rb + (size_t)c * 16);
      if (DUAL) T.w2[i][j] = ld_nt16(w2 + rb + (size_t)c * 16);
    }
  }
#pragma unroll
  for (int i = 0; i < RPR; ++i) {
    const int r = nrows > 0 ? row0 + min(i, nrows - 1) : N - 1;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int g = (min(lane + 64 * j, NC - 1) * 32) / kGroupQ4;
      T.s[i][j] = s[(size_t)r * groups + g];
      if (DUAL) T.s2[i][j] = s2[(size_t)r * groups + g];
    }
  }
}

// dequant-dot of the tile against x in LDS; returns per-lane butterfly total; value index of this lane via vi
template <int RPR, int CPT, bool DUAL>
__device__ __forceinline__ float tile_dot(const Tile<RPR, CPT, DUAL>& T, const uint4* xl, const float* xsum, int K,
                                          int lane, uint32_t nmask, int& vi) {
  constexpr int R = DUAL ? 2 * RPR : RPR;
  constexpr int RP = R <= 1 ? 2 : (R <= 2 ? 2 : (R <= 4 ? 4 : 8));  // butterfly width (zero padded)
  const int NC = K / 32;
  float part[RP];
#pragma unroll
  for (int i = 0; i < RP; ++i) part[i] = 0.0f;
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    if (CPT > 2) __builtin_amdgcn_sched_barrier(0);  // long rows: keep one x chunk (16 VGPRs) live at a time
    const int c = lane + 64 * j;
    const bool ok = c < NC;
    const int cc = min(c, NC - 1);
    const uint4* xc = xl + cc * 4;
    const float xs = xsum[cc];
#pragma unroll
    for (int i = 0; i < RPR; ++i) {
      const float d = chunk_dot<0>(T.w[i][j], xc, xs, nullptr, nmask);
      if (DUAL) {
        part[2 * i] = fmaf(ok ? scale_of<0>(T.s[i][j]) : 0.0f, d, part[2 * i]);
        const float d2 = chunk_dot<0>(T.w2[i][j], xc, xs, nullptr, nmask);
        part[2 * i + 1] = fmaf(ok ? scale_of<0>(T.s2[i][j]) : 0.0f, d2, part[2 * i + 1]);
      } else {
        part[i] = fmaf(ok ? scale_of<0>(T.s[i][j]) : 0.0f, d, part[i]);
      }
    }
  }
  vi = bfly_index<RP>(lane);
  return butterfly<RP>(part, lane);
}

// Stage x (K bf16, global) into LDS as (x_k, x_k+4) pairs + per-32 chunk sums; optional RMSNorm with weight nw.
// Split in two so weight prefetches can be issued between the x loads and the first wait on them (vmcnt is in
// order: a wait for x must not also wait for loads issued after it). SC1: x was written by other workgroups of
// this launch. stage_x_finish ends with a workgroup barrier.
constexpr int XMAX = 3;  // uint4 of x per thread: K <= 8 * 3 * LNT = 12288
template <bool SC1, bool NORM>
__device__ __forceinline__ void stage_x_load(const uint16_t* x, const uint16_t* nw, int K, uint4* xr, uint4* nr) {
  const int t = threadIdx.x, n8 = K / 8;
#pragma unroll
  for (int i = 0; i < XMAX; ++i) {
    const int u = min(t + LNT * i, n8 - 1);
    xr[i] = SC1 ? ld_sc1_u4(x + (size_t)u * 8) : *(const uint4*)(x + (size_t)u * 8);
    if (NORM) nr[i] = *(const uint4*)(nw + (size_t)u * 8);
  }
}
template <bool NORM>
__device__ __forceinline__ void stage_x_finish(const uint4* xr, const uint4* nr, int K, float eps, uint4* xl,
                                               float* xsum, float* red) {
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int n8 = K / 8;
  float rs = 1.0f;
  if (NORM) {
    float ss = 0.0f;
#pragma unroll
    for (int i = 0; i < XMAX; ++i) {
      const bool ok = t + LNT * i < n8;
      const uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float lo = ok ? bflo(d[q]) : 0.0f, hi = ok ? bfhi(d[q]) : 0.0f;
        ss = fmaf(lo, lo, ss);
        ss = fmaf(hi, hi, ss);
      }
    }
    ss = wave_sum_uniform(ss);
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    float tot = 0.0f;
#pragma unroll
    for (int w = 0; w < LNW; w += 4) tot += (red[w] + red[w + 1]) + (red[w + 2] + red[w + 3]);
    rs = 1.0f / sqrtf(tot / (float)K + eps);
  }
#pragma unroll
  for (int i = 0; i < XMAX; ++i) {
    const int u = t + LNT * i;
    uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
    if (NORM) {
      const uint32_t w4[4] = {nr[i].x, nr[i].y, nr[i].z, nr[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        d[q] = pack2(__fmul_rn(bflo(w4[q]), __fmul_rn(bflo(d[q]), rs)), __fmul_rn(bfhi(w4[q]), __fmul_rn(bfhi(d[q]), rs)));
    }
    float cs = ((bflo(d[0]) + bfhi(d[0])) + (bflo(d[1]) + bfhi(d[1]))) +
               ((bflo(d[2]) + bfhi(d[2])) + (bflo(d[3]) + bfhi(d[3])));
    cs += __shfl_xor(cs, 1);
    cs += __shfl_xor(cs, 2);
    if (u < n8) {
      xl[u] = make_uint4(__builtin_amdgcn_perm(d[2], d[0], 0x05040100u), __builtin_amdgcn_perm(d[2], d[0], 0x07060302u),
                         __builtin_amdgcn_perm(d[3], d[1], 0x05040100u), __builtin_amdgcn_perm(d[3], d[1], 0x07060302u));
      if ((u & 3) == 0) xsum[u >> 2] = cs;
    }
  }
  __syncthreads();
}

// the (value index -> row) owner lanes of a butterfly write their row results to LDS out[]
template <int RPR, bool DUAL>
__device__ __forceinline__ void rows_to_lds(float tot, int vi, int lane, int wave, int nrows, float* out,
                                            int stride = RPR, int base = 0) {
  constexpr int R = DUAL ? 2 * RPR : RPR;
  constexpr int RP = R <= 2 ? 2 : (R <= 4 ? 4 : 8);
  constexpr int GROUP = 64 / RP;
  if (DUAL) {
    constexpr int PD = RP == 8 ? 8 : (RP == 4 ? 16 : 32);
    const float other = PD == 8 ? LGA_DPP(tot, 0x128) : __shfl_xor(tot, PD);
    const int i = vi >> 1;
    if ((lane & (GROUP - 1)) == 0 && (vi & 1) == 0 && i < nrows) {
      const float g = round_bf(silu_f(round_bf(tot)));   // silu(bf16(fc_1 x)) -> bf16 (model.py:715)
      out[wave * stride + base + i] = __fmul_rn(g, round_bf(other));  // * bf16(fc_2 x)
    }
  } else {
    if ((lane & (GROUP - 1)) == 0 && vi < nrows) out[wave * stride + base + vi] = tot;
  }
}

// Rolling two-buffer GEMV over NP parts of PR rows (rows row0 .. row0 + nrows - 1): part p computes from buffer
// p % 2 while part p + 1 is in flight, then the buffer is refilled with part p + 2. The caller has issued parts 0
// (A) and 1 (B). Loads stay unconditional (a part past nrows re-reads the wave's last row, an L2 hit), so the
// in-order vmcnt waits stay exact. Two parts of 2 rows keep ~8 KB per wave in flight, enough for the per-CU share
// of HBM bandwidth, at half the registers of a whole-tile prefetch.
template <int PR, int CPT, bool DUAL>
__device__ __forceinline__ void part_load(Tile<PR, CPT, DUAL>& T, const uint8_t* w, const uint16_t* s,
                                          const uint8_t* w2, const uint16_t* s2, int row0, int nrows, int p, int N,
                                          int K, int lane) {
  const int nr = nrows - p * PR;
  tile_load(T, w, s, w2, s2, nr > 0 ? row0 + p * PR : row0 + max(nrows - 1, 0), nr > 0 ? nr : 1, N, K, lane);
}

template <int PR, int CPT, bool DUAL, int NP>
__device__ __forceinline__ void gemv_parts(Tile<PR, CPT, DUAL>& A, Tile<PR, CPT, DUAL>& B, const uint8_t* w,
                                           const uint16_t* s, const uint8_t* w2, const uint16_t* s2, int row0,
                                           int nrows, int N, int K, int lane, int cw, const uint4* xl,
                                           const float* xsum, uint32_t nmask, float* out, int stride) {
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    Tile<PR, CPT, DUAL>& cur = (p & 1) ? B : A;
    const int pr = min(PR, nrows - p * PR);
    if (pr > 0) {
      int vi;
      const float tot = tile_dot(cur, xl, xsum, K, lane, nmask, vi);
      rows_to_lds<PR, DUAL>(tot, vi, lane, cw, pr, out, stride, p * PR);
    }
    if (p + 2 < NP) {
      __builtin_amdgcn_sched_barrier(0);
      part_load(cur, w, s, w2, s2, row0, nrows, p + 2, N, K, lane);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// ------------------------------------------------------------------------------------------------ the kernel
// LDS: x staging (max(C, I) bf16 + chunk sums), stage outputs, attention merge, h_mid rows; padded past 80 KB
struct LayerLds {
  uint4 xl[16384 / 8];
  float xsum[16384 / 32];
  float red[LNW];
  float out[128];               // stage row results (<= 128 rows per workgroup and stage)
  uint16_t hmid[64];            // this workgroup's h_mid rows (S3 -> S5 residual)
  float am[LNW], al[LNW];       // attention per-wave (m, l)
  float ao[LNW][128];           // attention per-wave o
  unsigned last;
  unsigned char pad[12 * 1024];
};

// Wave 0 is the control wave: it publishes (sc1 stores + vmcnt(0) + counter) and polls; it holds no weight
// prefetches, so neither wait drains a prefetch. Waves 1..15 compute: each issues the NEXT stage's weight loads
// as soon as its current tile is consumed, so they stream during the publish / hand-off / next input load.
template <int R1, int R3, int R4, int R5, int CPTC, int CPTI>
__global__ void __launch_bounds__(LNT) decode_layer_kernel(LayerArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  LayerLds& L = *(LayerLds*)smem_raw;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int cw = wave - 1;  // compute-wave index (-1 = control wave)
  const int b = blockIdx.x, NB = gridDim.x;
  constexpr int HS = 128, LPR = 16, RGW = 4, RG = (LNW - 1) * RGW, UNR = 4;
  const int C = a.C, I = a.I, G = a.G, H = a.H;
  const int Nq = (H + 2 * G) * HS;
  const int qpk = H / G;  // == 1 in the instantiated build
  const uint32_t nmask = nibble_mask();
  LGA_LTRACE(0);
  const long p = a.pos[0];

  // ---- work split: Nq / NB qkv rows, C / NB proj and mlp.proj rows, ceil(I / NB) fc rows per workgroup
  const int q_rows = Nq / NB, o_rows = C / NB;
  const int q_row0 = b * q_rows + cw * R1, q_n = cw < 0 ? 0 : max(0, min(R1, q_rows - cw * R1));
  const int o_row0 = b * o_rows + cw * R3, o_n = cw < 0 ? 0 : max(0, min(R3, o_rows - cw * R3));
  const int g_base = b * ((I + NB - 1) / NB);
  const int g_cnt = max(0, min((I + NB - 1) / NB, I - g_base));
  const int g_row0 = g_base + cw * R4, g_n = cw < 0 ? 0 : max(0, min(R4, g_cnt - cw * R4));
  const int d_row0 = b * o_rows + cw * R5, d_n = cw < 0 ? 0 : max(0, min(R5, o_rows - cw * R5));
  const int bpg = NB / G;  // workgroups (sequence splits) per query group
  const int grp = b / bpg, split = b % bpg;

  // ---- S1 input first, then the S1 weights and the first K/V batch of S2 (vmcnt order: x, T1, K/V)
  uint4 xr[XMAX], nr[XMAX];
  stage_x_load<false, true>(a.h_in, a.norm1, C, xr, nr);
  constexpr int P1 = 2, NP1 = (R1 + P1 - 1) / P1;  // qkv rows in parts of 2 (rolling two-buffer GEMV)
  Tile<P1, CPTC, false> T1a, T1b;
  if (q_n > 0) {
    part_load(T1a, a.wq, a.sq, nullptr, nullptr, q_row0, q_n, 0, Nq, C, lane);
    part_load(T1b, a.wq, a.sq, nullptr, nullptr, q_row0, q_n, 1, Nq, C, lane);
  }
  const int rg = cw * RGW + lane / LPR, sub = lane % LPR;
  const int Lk = (int)min(p + 1, (long)a.S);
  const int chunk = (Lk + bpg - 1) / bpg;
  const int k_lo = split * chunk, k_hi = min(k_lo + chunk, Lk);
  const int k_end = min(k_hi, (int)p);  // key p comes from this step's qkv
  const uint16_t* kbase = a.kc + (size_t)grp * a.S * HS + sub * 8;
  const uint16_t* vbase = a.vc + (size_t)grp * a.S * HS + sub * 8;
  uint4 kv[UNR], vv[UNR];
  const int j_last = max(k_end - 1, 0);
  __builtin_amdgcn_sched_barrier(0);

  // ================= S1: qkv = W_qkv . RMSNorm(h_in)
  stage_x_finish<true>(xr, nr, C, a.eps, L.xl, L.xsum, L.red);
  LGA_LTRACE(1);
  if (q_n > 0)
    gemv_parts<P1, CPTC, false, NP1>(T1a, T1b, a.wq, a.sq, nullptr, nullptr, q_row0, q_n, Nq, C, lane, cw, L.xl, L.xsum,
                                     nmask, L.out, R1);
  __builtin_amdgcn_sched_barrier(0);
    if (cw >= 0) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int j = min(k_lo + rg + u * RG, j_last);
      kv[u] = ld_nt16(kbase + (size_t)j * HS);
      vv[u] = ld_nt16(vbase + (size_t)j * HS);
    }
  }
  __syncthreads();
  if (wave == 0) {  // bf16 rows -> qkv scratch (sc1), then count this workgroup for its query group
    for (int i = lane; i < q_rows / 2; i += 64)
      st_sc1_u32(a.qkv + (size_t)b * q_rows + 2 * i, pack2(L.out[2 * i], L.out[2 * i + 1]));
    publish(ctr(a, (b * q_rows) / ((qpk + 2) * HS)));
  }

#if defined(LGA_LAYER_MAXSTAGE) && LGA_LAYER_MAXSTAGE < 2
  return;
#endif
  // ================= S2: attention for (grp, split), RoPE + KV append of key p fused
  LGA_LTRACE(2);
  wait_count(a, ctr(a, grp), (unsigned)(((qpk + 2) * HS) / q_rows));
  LGA_LTRACE(3);
  float qf[8];
  float m_ = -INFINITY, l_ = 0.0f, o_[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o_[i] = 0.0f;
  const long rp = min(max(p, 0L), (long)a.rope_rows - 1);
  const float* cr = a.cos + (size_t)rp * HS + sub * 8;
  const float* sr = a.sin + (size_t)rp * HS + sub * 8;
  constexpr int P4 = 2, NP4 = (R4 + P4 - 1) / P4;  // fc_1 || fc_2 rows in parts of 2
  Tile<P4, CPTC, true> T4a, T4b;
  Tile<R3, CPTC, false> T3;
  if (cw >= 0) {
    {
      const uint16_t* qrow = a.qkv + (size_t)grp * (qpk + 2) * HS + sub * 8;
      unpack8(rope8(ld_sc1_u4(qrow), cr, sr, sub), qf);
    }
    for (int j0 = k_lo + rg, it = 0; j0 < k_end; j0 += RG * UNR, ++it) {
      if (it > 0) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const int j = min(j0 + u * RG, j_last);
          kv[u] = ld_nt16(kbase + (size_t)j * HS);
          vv[u] = ld_nt16(vbase + (size_t)j * HS);
        }
      }
      float s[UNR];
      float mx = m_;
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        float kf[8];
        unpack8(kv[u], kf);
        float d = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) d = fmaf(qf[i], kf[i], d);
        const float sd = row_group_sum<LPR>(d) * a.scale;
        s[u] = (j0 + u * RG < k_end) ? sd : -INFINITY;
        mx = fmaxf(mx, s[u]);
      }
      const float c = expf(m_ - mx);
      l_ *= c;
#pragma unroll
      for (int i = 0; i < 8; ++i) o_[i] *= c;
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const float e = expf(s[u] - mx);
        l_ += e;
        float vf[8];
        unpack8(vv[u], vf);
#pragma unroll
        for (int i = 0; i < 8; ++i) o_[i] = fmaf(e, vf[i], o_[i]);
      }
      m_ = mx;
    }
    const bool owns_new = p < a.S && k_lo <= p && p < k_hi;
    if (owns_new && rg == 0) {  // roped k and v of position p: append to the cache, score from registers
      const uint16_t* kvrow = a.qkv + ((size_t)grp * (qpk + 2) + qpk) * HS + sub * 8;
      const uint4 kr = rope8(ld_sc1_u4(kvrow), cr, sr, sub);
      const uint4 vr = ld_sc1_u4(kvrow + HS);
      *(uint4*)(a.kc + ((size_t)grp * a.S + p) * HS + sub * 8) = kr;
      *(uint4*)(a.vc + ((size_t)grp * a.S + p) * HS + sub * 8) = vr;
      float kf[8], vf[8];
      unpack8(kr, kf);
      unpack8(vr, vf);
      float d = 0.0f;
#pragma unroll
      for (int i = 0; i < 8; ++i) d = fmaf(qf[i], kf[i], d);
      const float sc = row_group_sum<LPR>(d) * a.scale;
      const float mx = fmaxf(m_, sc);
      const float c = expf(m_ - mx), e = expf(sc - mx);
      l_ = l_ * c + e;
#pragma unroll
      for (int i = 0; i < 8; ++i) o_[i] = fmaf(e, vf[i], o_[i] * c);
      m_ = mx;
    }
    // prefetch S3 (attn.proj) now that the K/V registers are free
    __builtin_amdgcn_sched_barrier(0);
    if (o_n > 0) tile_load(T3, a.wo, a.so, nullptr, nullptr, o_row0, o_n, C, C, lane);
    __builtin_amdgcn_sched_barrier(0);
    // merge the wave's 4 row groups (lanes 16 apart)
#pragma unroll
    for (int off = LPR; off < 64; off <<= 1) {
      const float mo = __shfl_xor(m_, off), lo = __shfl_xor(l_, off);
      const float mn = fmaxf(m_, mo);
      const float ca = mn == -INFINITY ? 0.0f : expf(m_ - mn);
      const float cb = mn == -INFINITY ? 0.0f : expf(mo - mn);
      l_ = l_ * ca + lo * cb;
#pragma unroll
      for (int i = 0; i < 8; ++i) o_[i] = o_[i] * ca + __shfl_xor(o_[i], off) * cb;
      m_ = mn;
    }
  }
  if (lane < LPR) {  // control wave contributes an empty state
    if (lane == 0) {
      L.am[wave] = m_;
      L.al[wave] = l_;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) L.ao[wave][sub * 8 + i] = o_[i];
  }
  __syncthreads();
  const size_t hrow = (size_t)grp * qpk;  // the group's head (qpk == 1)
  if (wave == 0) {
    for (int d = lane; d < HS; d += 64) {
      float mx = -INFINITY;
#pragma unroll
      for (int w = 0; w < LNW; ++w) mx = fmaxf(mx, L.am[w]);
      float lt = 0.0f, ot = 0.0f;
#pragma unroll
      for (int w = 0; w < LNW; ++w) {
        const float c = mx == -INFINITY ? 0.0f : expf(L.am[w] - mx);
        lt += L.al[w] * c;
        ot += L.ao[w][d] * c;
      }
      float* wsr = a.ws + (hrow * bpg + split) * (HS + 4);
      st_sc1(wsr + 4 + d, ot);
      if (d == 0) {
        st_sc1(wsr, mx);
        st_sc1(wsr + 1, lt);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) L.last = __hip_atomic_fetch_add(ctr(a, G + grp), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (L.last == (unsigned)(bpg - 1) && wave == 0) {  // last split of the group: merge, write y, count the group
    const float* base = a.ws + hrow * bpg * (HS + 4);
    // split maxima first (one load per lane), then every (l, o) load of a column issued together
    float* wm = L.ao[0];  // the per-wave o tiles are consumed: reuse as [bpg] maxima
    if (lane < bpg) wm[lane] = ld_sc1(base + lane * (HS + 4));
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);
    float mx = -INFINITY;
    for (int sp = 0; sp < bpg; ++sp) mx = fmaxf(mx, wm[sp]);
    for (int d = lane; d < HS; d += 64) {
      float lt = 0.0f, ot = 0.0f;
#pragma unroll 8
      for (int sp = 0; sp < bpg; ++sp) {
        const float c = expf(wm[sp] - mx);
        lt = fmaf(ld_sc1(base + sp * (HS + 4) + 1), c, lt);
        ot = fmaf(ld_sc1(base + sp * (HS + 4) + 4 + d), c, ot);
      }
      L.out[d] = ot / lt;
    }
    for (int i = lane; i < HS / 2; i += 64)
      st_sc1_u32(a.yatt + hrow * HS + 2 * i, pack2(L.out[2 * i], L.out[2 * i + 1]));
    if (lane == 0) __hip_atomic_store(ctr(a, G + grp), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    publish(ctr(a, 2 * G));
  }

#if defined(LGA_LAYER_MAXSTAGE) && LGA_LAYER_MAXSTAGE < 3
  return;
#endif
  // ================= S3: h_mid = h_in + bf16(W_o . y)
  LGA_LTRACE(4);
  wait_count(a, ctr(a, 2 * G), (unsigned)G);
  LGA_LTRACE(5);
  stage_x_load<true, false>(a.yatt, nullptr, C, xr, nr);
  stage_x_finish<false>(xr, nr, C, 0.0f, L.xl, L.xsum, L.red);
  if (o_n > 0) {
    int vi;
    const float tot = tile_dot(T3, L.xl, L.xsum, C, lane, nmask, vi);
    rows_to_lds<R3, false>(tot, vi, lane, cw, o_n, L.out);
  }
  // prefetch the first half of S4 (fc_1 || fc_2) once the proj tile is consumed
  __builtin_amdgcn_sched_barrier(0);
  if (g_n > 0) part_load(T4a, a.w1, a.s1, a.w2, a.s2, g_row0, g_n, 0, I, C, lane);
  __syncthreads();
  if (wave == 0) {
    const int row0 = b * o_rows;
    for (int i = lane; i < o_rows; i += 64) L.hmid[i] = f2bf(round_bf(L.out[i]) + bf2f(a.h_in[row0 + i]));
    for (int i = lane; i < o_rows / 2; i += 64)
      st_sc1_u32(a.h_mid + row0 + 2 * i, (uint32_t)L.hmid[2 * i] | ((uint32_t)L.hmid[2 * i + 1] << 16));
    publish(ctr(a, 2 * G + 1));
  }

#if defined(LGA_LAYER_MAXSTAGE) && LGA_LAYER_MAXSTAGE < 4
  return;
#endif
  // ================= S4: act = bf16(silu(bf16(W1 . n))) * bf16(W2 . n), n = RMSNorm(h_mid)
  LGA_LTRACE(6);
  wait_count(a, ctr(a, 2 * G + 1), (unsigned)NB);
  LGA_LTRACE(7);
  stage_x_load<true, true>(a.h_mid, a.norm2, C, xr, nr);
  __builtin_amdgcn_sched_barrier(0);
  if (g_n > 0) part_load(T4b, a.w1, a.s1, a.w2, a.s2, g_row0, g_n, 1, I, C, lane);
  __builtin_amdgcn_sched_barrier(0);
  stage_x_finish<true>(xr, nr, C, a.eps, L.xl, L.xsum, L.red);
  if (g_n > 0)
    gemv_parts<P4, CPTC, true, NP4>(T4a, T4b, a.w1, a.s1, a.w2, a.s2, g_row0, g_n, I, C, lane, cw, L.xl, L.xsum,
                                    nmask, L.out, R4);
  constexpr int P5 = 1, NP5 = R5;  // mlp.proj rows one at a time (K = I: 6 chunks per lane per row)
  Tile<P5, CPTI, false> T5a, T5b;    // prefetch the first part of S5 (mlp.proj)
  __builtin_amdgcn_sched_barrier(0);
  if (d_n > 0) part_load(T5a, a.wd, a.sd, nullptr, nullptr, d_row0, d_n, 0, C, I, lane);
  __syncthreads();
  if (wave == 0) {
    for (int i = lane; i < g_cnt / 2; i += 64)
      st_sc1_u32(a.act + g_base + 2 * i, pack2(L.out[2 * i], L.out[2 * i + 1]));
    if ((g_cnt & 1) && lane == 0) {
      const int r = g_cnt - 1;
      __hip_atomic_store(a.act + g_base + r, f2bf(L.out[r]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    publish(ctr(a, 2 * G + 2));
  }

#if defined(LGA_LAYER_MAXSTAGE) && LGA_LAYER_MAXSTAGE < 5
  return;
#endif
  // ================= S5: h_out = h_mid + bf16(W_d . act)
  LGA_LTRACE(8);
  wait_count(a, ctr(a, 2 * G + 2), (unsigned)NB);
  LGA_LTRACE(9);
  stage_x_load<true, false>(a.act, nullptr, I, xr, nr);
  __builtin_amdgcn_sched_barrier(0);
  if (d_n > 0) part_load(T5b, a.wd, a.sd, nullptr, nullptr, d_row0, d_n, 1, C, I, lane);
  __builtin_amdgcn_sched_barrier(0);
  stage_x_finish<false>(xr, nr, I, 0.0f, L.xl, L.xsum, L.red);
  if (d_n > 0)
    gemv_parts<P5, CPTI, false, NP5>(T5a, T5b, a.wd, a.sd, nullptr, nullptr, d_row0, d_n, C, I, lane, cw, L.xl,
                                     L.xsum, nmask, L.out, R5);
  __syncthreads();
  if (wave == 0) {
    const int row0 = b * o_rows;
    for (int i = lane; i < o_rows; i += 64) a.h_out[row0 + i] = f2bf(round_bf(L.out[i]) + bf2f(L.hmid[i]));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) L.last = __hip_atomic_fetch_add(ctr(a, 2 * G + 3), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  LGA_LTRACE(10);
  if (L.last == (unsigned)(NB - 1)) {  // every workgroup is past its last wait: re-arm the counters
    for (int i = t; i < 2 * G + 4; i += LNT) __hip_atomic_store(ctr(a, i), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace lga

// Llama decode block for T = 1 in one launch (see the header comment above). Supported geometry (else an error,
// and the caller uses the per-op path): int4-g128 weights, head_size 128, q_per_kv 1, n_embd == 4096 == 16 rows
// per workgroup x #CUs (256), fused qkv rows = 48 per workgroup, intermediate <= 16384 with ceil(I / #CUs) <= 48
// rows per workgroup, #CUs divisible by n_query_groups.
// the qkv rows of one query group (q, k, v: 3 x hs at q_per_kv 1) must be produced by exactly the NB / G
// workgroups that then run that group's attention splits
static bool qpk_rows_ok(int q_rows, int G, int NB, int hs) {
  const int group_rows = 3 * hs;
  return q_rows > 0 && group_rows % q_rows == 0 && group_rows / q_rows == NB / G;
}

extern "C" size_t lga_decode_layer_counters(int n_query_groups) { return (size_t)(2 * n_query_groups + 4) * lga::LCS; }

extern "C" int lga_decode_layer(const void* h_in, void* h_mid, void* h_out, const void* norm1, const void* norm2,
                                float eps, const uint8_t* wq, const void* sq, const uint8_t* wo, const void* so,
                                const uint8_t* w1, const void* s1, const uint8_t* w2, const void* s2,
                                const uint8_t* wd, const void* sd, void* k_cache, void* v_cache, const float* cos,
                                const float* sin, int rope_rows, const int64_t* pos, void* qkv_scratch,
                                void* y_scratch, void* act_scratch, float* attn_ws, unsigned* counters,
                                unsigned* err, int n_embd, int intermediate, int n_head, int n_query_groups,
                                int head_size, int max_seq, float scale, int n_cu, hipStream_t stream) {
  LGA_CHECK_ARG(h_in && h_mid && h_out && norm1 && norm2 && wq && sq && wo && so && w1 && s1 && w2 && s2 && wd &&
                    sd && k_cache && v_cache && cos && sin && pos && qkv_scratch && y_scratch && act_scratch &&
                    attn_ws && counters && err,
                "lga_decode_layer: null pointer");
  const int NB = n_cu;  // one workgroup per CU (VGPR-bound), so all are resident together
  LGA_CHECK_ARG(head_size == 128 && n_head == n_query_groups, "lga_decode_layer: needs head_size 128, q_per_kv 1");
  const int Nq = (n_head + 2 * n_query_groups) * head_size;
  LGA_CHECK_ARG(NB > 0 && NB % n_query_groups == 0 && Nq % NB == 0 && n_embd % NB == 0,
                "lga_decode_layer: 2 x #CUs must divide n_query_groups, the qkv rows and n_embd");
  LGA_CHECK_ARG(qpk_rows_ok(Nq / NB, n_query_groups, NB, head_size),
                "lga_decode_layer: the qkv rows of a query group must map to its attention workgroups");
  LGA_CHECK_ARG(Nq / NB <= 7 * 7 && n_embd / NB <= 3 * 7 && (n_embd / NB) % 2 == 0 && (Nq / NB) % 2 == 0 &&
                    (intermediate + NB - 1) / NB <= 7 * 7,
                "lga_decode_layer: too many rows per workgroup for the built tile sizes");
  LGA_CHECK_ARG(n_embd % 128 == 0 && intermediate % 128 == 0 && intermediate <= 12288 && n_embd <= 12288,
                "lga_decode_layer: dims must be multiples of 128 and <= 16384");
  LGA_CHECK_ARG((n_embd / 32 + 63) / 64 == 2 && (intermediate / 32 + 63) / 64 <= 6,
                "lga_decode_layer: built for n_embd 4096 and intermediate <= 12288");
  lga::LayerArgs a{(const uint16_t*)h_in, (uint16_t*)h_mid, (uint16_t*)h_out, (const uint16_t*)norm1,
                   (const uint16_t*)norm2, eps, wq, (const uint16_t*)sq, wo, (const uint16_t*)so, w1,
                   (const uint16_t*)s1, w2, (const uint16_t*)s2, wd, (const uint16_t*)sd, (uint16_t*)k_cache,
                   (uint16_t*)v_cache, cos, sin, rope_rows, pos, (uint16_t*)qkv_scratch, (uint16_t*)y_scratch,
                   (uint16_t*)act_scratch, attn_ws, counters, err, n_embd, intermediate, n_head, n_query_groups,
                   max_seq, scale};
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)lga::decode_layer_kernel<7, 3, 7, 3, 2, 6>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(lga::LayerLds));
    attr_set = true;
  }
  lga::decode_layer_kernel<7, 3, 7, 3, 2, 6><<<NB, lga::LNT, sizeof(lga::LayerLds), stream>>>(a);
  LGA_LAUNCH_RETURN();
}

#ifdef LGA_LAYER_TRACE
extern "C" int lga_layer_trace_read(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(lga::g_layer_trace), (size_t)n * sizeof(unsigned long long));
}
#endif
