// Decode GEMV body over packed 4-bit weights (gemv.hip launches it; design notes there).
#pragma once
#include "decode_ops.h"

namespace lga {

#ifdef LGA_GEMV_TRACE  // lab builds only (tools/gemv_trace.py): per-wave phase timestamps, 100 MHz clock
__device__ unsigned long long g_gemv_trace[65536 * 8];
#define LGA_GTRACE(i)                                                                                        \
  do {                                                                                                     \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                          \
    if ((threadIdx.x & 63) == 0)                                                                         \
      g_gemv_trace[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define LGA_GTRACE_NOWAIT(i)                                                                                 \
  do {                                                                                                     \
    if ((threadIdx.x & 63) == 0)                                                                         \
      g_gemv_trace[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define LGA_GTRACE(i) \
  do {                \
  } while (0)
#define LGA_GTRACE_NOWAIT(i) \
  do {                       \
  } while (0)
#endif


struct GemvArgs {
  const uint16_t* x;         // [K] bf16
  const uint8_t* qw;         // [N][K/2]
  const void* sc;            // q4g: bf16 [N][K/G]; nf4: f32 [N][K/G]
  const uint8_t* qw2;        // dual: second weight (fc_2)
  const void* sc2;
  const uint16_t* bias;      // [N] or null
  const uint16_t* residual;  // [N] or null
  const uint16_t* norm_w;    // [K] or null (fused RMSNorm)
  uint16_t* y;               // [N]
  int N, K, G;
  float eps;
  // sparse-MoE expert routing (lga_q4_gemv*_experts): grid.y = slots; slot s computes with the weights of expert
  // eidx[s] (qw/qw2 + e * ew bytes, sc/sc2 + e * es bytes), reads x + s * xs and writes y + s * N
  const int32_t* eidx;
  long long ew, es;
  int xs, n_expert, slots;
  int cb = 0;  // codebook row of kCode4 (FMT 1): 0 nf4, 1 fp4
  const uint16_t* probs = nullptr;  // routing probabilities (lga_q4_gemv_experts_pair_combine)
};

// LDS of gemv_q4_body: x pairs (2K B), chunk sums (K/32 floats), norm partials (16), codebook (16), then (LDS_OUT)
// the workgroup's output rows at a 16-B-aligned offset
__host__ __device__ inline size_t gemv_out_offset(int K) { return ((size_t)K * 2 + (K / 32) * 4 + 128 + 15) & ~(size_t)15; }
__host__ __device__ inline size_t gemv_lds_bytes(int K) { return gemv_out_offset(K) + 256; }
__device__ __forceinline__ uint16_t* gemv_out_lds(unsigned char* smem, int K) { return (uint16_t*)(smem + gemv_out_offset(K)); }

// One wave of a decode GEMV (see gemv.hip for the design). NW waves per workgroup (each its own row slot); the
// workgroup stages x once for all of them. LDS_OUT (gemv_ar.hip): the workgroup's NW * RPR bf16 rows go to LDS
// (gemv_out_lds) instead of a.y, for an epilogue that moves them on as 16-B pieces.
template <int RPR, int CPT, int FMT, bool DUAL, bool NORM, bool RES, int NW = 4, bool LDS_OUT = false>
__device__ __forceinline__ void gemv_q4_body(GemvArgs a, int blk, unsigned char* smem) {
  if (a.eidx) {  // wave-uniform: one scalar load of the routed expert id, then plain pointer offsets
    const long long e = min(max(a.eidx[blockIdx.y], 0), a.n_expert - 1);
    a.qw += e * a.ew;
    a.sc = (const unsigned char*)a.sc + e * a.es;
    if (DUAL) {
      a.qw2 += e * a.ew;
      a.sc2 = (const unsigned char*)a.sc2 + e * a.es;
    }
    a.x += (size_t)blockIdx.y * a.xs;
    a.y += (size_t)blockIdx.y * a.N;
  }
  uint4* xl = (uint4*)smem;                        // K/8 uint4 (bf16 pairs)
  float* xsum = (float*)(smem + (size_t)a.K * 2);  // K/32 chunk sums
  float* red = xsum + a.K / 32;                    // NW (<= 16)
  float* nf4 = red + 16;                           // 16
  constexpr int NT = NW * 64;
  constexpr int XI = (CPT * 4 + NW - 1) / NW;      // x uint4 per thread (CPT * 256 >= K / 8)
  static_assert(NW == 4 || NW == 8 || NW == 16, "4, 8 or 16 waves per workgroup");
  constexpr int R = DUAL ? 2 * RPR : RPR;          // values per lane entering the butterfly
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int NC = a.K / 32, n8 = a.K / 8, groups = a.K / a.G;
  const int row0 = (blk * NW + wave) * RPR;
  if (FMT == 1 && t < 16) nf4[t] = kCode4[a.cb][t];
  LGA_GTRACE_NOWAIT(0);

  // 1. activation (and norm weight) share of this thread: uint4 t, t+NT, ... (clamped, branch-free)
  uint4 xr[XI], nr[XI];
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int u = min(t + NT * i, n8 - 1);
#ifdef LGA_LAB_NOX  // lab builds only: cost of the activation fetch
    xr[i] = make_uint4(0x3F803F80u + u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);
    if (NORM) nr[i] = xr[i];
#else
    xr[i] = ((const uint4*)a.x)[u];
    if (NORM) nr[i] = ((const uint4*)a.norm_w)[u];
#endif
  }
  // 2. every weight / scale / residual load of this wave (rows past N re-read row N-1; never stored), issued in
  //    the order step 4 consumes them (chunk-major, each scale right after its weights): vmcnt retires in order,
  //    so the first dots start once their own chunk has landed instead of after the whole wave's stream
  uint4 w[RPR][CPT], w2[DUAL ? RPR : 1][DUAL ? CPT : 1];
  uint32_t s[RPR][CPT], s2[DUAL ? RPR : 1][DUAL ? CPT : 1];
  uint32_t res = 0;
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = min(lane + 64 * j, NC - 1);
    const int g = (c * 32) / a.G;
#pragma unroll
    for (int i = 0; i < RPR; ++i) {
      const size_t n = (size_t)min(row0 + i, a.N - 1);
      w[i][j] = ld_nt16(a.qw + n * (a.K / 2) + (size_t)c * 16);
#ifdef LGA_LAB_NOSCALE  // lab builds only (tools/gemv_variants.py): cost of the scale loads
      s[i][j] = 0x3F80u + (uint32_t)g;
#else
      s[i][j] = load_scale_bits<FMT>(a.sc, n * groups + g);
#endif
      if (DUAL) {
        w2[i][j] = ld_nt16(a.qw2 + n * (a.K / 2) + (size_t)c * 16);
#ifdef LGA_LAB_NOSCALE
        s2[i][j] = 0x3F80u + (uint32_t)g;
#else
        s2[i][j] = load_scale_bits<FMT>(a.sc2, n * groups + g);
#endif
      }
    }
  }
  if (RES) res = a.residual[min(row0 + (lane & (RPR - 1)), a.N - 1)];
  __builtin_amdgcn_sched_barrier(0);  // nothing that waits on x may move above the weight loads
  LGA_GTRACE_NOWAIT(1);

  // 3. stage x into LDS (RMS-normalised when NORM) while the weights stream
  float rs = 1.0f;
  if (NORM) {
    float ss = 0.0f;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const bool ok = t + NT * i < n8;
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
    LGA_GTRACE_NOWAIT(2);
    __syncthreads();
    float r4[NW / 4];  // pairwise tree over the waves (NW = 4: ((r0 + r1) + (r2 + r3)))
#pragma unroll
    for (int i = 0; i < NW / 4; ++i) r4[i] = (red[4 * i] + red[4 * i + 1]) + (red[4 * i + 2] + red[4 * i + 3]);
    float tot = r4[0];
    if (NW == 8) tot = r4[0] + r4[1];
    if (NW == 16) tot = (r4[0] + r4[1]) + (r4[2] + r4[3]);
    rs = 1.0f / sqrtf(tot / (float)a.K + a.eps);
  }
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int u = t + NT * i;
    uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};  // bf16 pairs (x0,x1) (x2,x3) (x4,x5) (x6,x7)
    if (NORM) {  // bf16(w * (x * rs)), rounded in hardware, two elements per instruction
      const uint32_t nw[4] = {nr[i].x, nr[i].y, nr[i].z, nr[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        d[q] = pack2(__fmul_rn(bflo(nw[q]), __fmul_rn(bflo(d[q]), rs)),
                     __fmul_rn(bfhi(nw[q]), __fmul_rn(bfhi(d[q]), rs)));
    }
    uint4 xv;
    float cs = stage_x8<FMT>(d, xv);
    cs += __shfl_xor(cs, 1);  // 4 consecutive threads hold one 32-element chunk
    cs += __shfl_xor(cs, 2);
    if (u < n8) {
      xl[u] = xv;  // (x0,x4) (x1,x5) (x2,x6) (x3,x7) pairs (stage_x8)
      if ((u & 3) == 0) xsum[u >> 2] = cs;
    }
  }
  __syncthreads();
  LGA_GTRACE_NOWAIT(3);
  LGA_GTRACE(4);

  // 4. dequant-dot every row of this wave, then one butterfly for all of them
  const uint32_t nmask = nibble_mask(), nmagic = f16_magic(), nmask_hi = nibble_mask_hi();
  float part[R];
#pragma unroll
  for (int i = 0; i < R; ++i) part[i] = 0.0f;
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = lane + 64 * j;
    const bool ok = c < NC;
    const int cc = min(c, NC - 1);
    const uint4* xc = xl + cc * 4;
    const float xs = xsum[cc];
#ifdef LGA_LAB_NOCOMPUTE  // lab builds only: cost of the dequant-dot (weights folded, not multiplied)
#pragma unroll
    for (int i = 0; i < RPR; ++i) {
      const float d = __uint_as_float((w[i][j].x ^ w[i][j].y ^ w[i][j].z ^ w[i][j].w) & 0x3FFFFFFFu) + xs;
      if (DUAL) {
        part[2 * i] = fmaf(ok ? scale_of<FMT>(s[i][j]) : 0.0f, d, part[2 * i]);
        const float d2 = __uint_as_float((w2[i][j].x ^ w2[i][j].y ^ w2[i][j].z ^ w2[i][j].w) & 0x3FFFFFFFu);
        part[2 * i + 1] = fmaf(ok ? scale_of<FMT>(s2[i][j]) : 0.0f, d2, part[2 * i + 1]);
      } else {
        part[i] = fmaf(ok ? scale_of<FMT>(s[i][j]) : 0.0f, d, part[i]);
      }
    }
#else
    // all rows (and both matrices) of chunk j in one interleaved pass; value index = 2*row + matrix (DUAL)
    uint4 wj[R];
#pragma unroll
    for (int i = 0; i < RPR; ++i) {
      if (DUAL) {
        wj[2 * i] = w[i][j];
        wj[2 * i + 1] = w2[DUAL ? i : 0][DUAL ? j : 0];
      } else {
        wj[i] = w[i][j];
      }
    }
    float d[R];
    chunk_dot_rows<FMT, R>(wj, xc, xs, nf4, nmask, nmagic, nmask_hi, d);
#pragma unroll
    for (int i = 0; i < RPR; ++i) {
      if (DUAL) {
        part[2 * i] = fmaf(ok ? scale_of<FMT>(s[i][j]) : 0.0f, d[2 * i], part[2 * i]);
        part[2 * i + 1] = fmaf(ok ? scale_of<FMT>(s2[DUAL ? i : 0][DUAL ? j : 0]) : 0.0f, d[2 * i + 1],
                               part[2 * i + 1]);
      } else {
        part[i] = fmaf(ok ? scale_of<FMT>(s[i][j]) : 0.0f, d[i], part[i]);
      }
    }
#endif
  }
  const float tot = butterfly<R>(part, lane);
  const int vi = bfly_index<R>(lane);  // value index held by this lane
  constexpr int GROUP = 64 / R;        // lanes per value after the butterfly
  if (DUAL) {
    // partner value (other matrix, same row) sits in the lane whose value index differs in bit 0
    constexpr int PD = R == 8 ? 8 : (R == 4 ? 16 : 32);
    const float other = PD == 8 ? LGA_DPP(tot, 0x128) : __shfl_xor(tot, PD);
    const int row = row0 + (vi >> 1);
    const float g = round_bf(silu_f(round_bf(tot)));  // silu(bf16(fc_1 x)) -> bf16
    const uint16_t ob = f2bf(__fmul_rn(g, round_bf(other)));  // * bf16(fc_2 x)
    if ((lane & (GROUP - 1)) == 0 && (vi & 1) == 0 && row < a.N) {
      a.y[row] = ob;
    }
    LGA_GTRACE(5);
  } else {
    const int row = row0 + vi;
    float o = tot;
    if (RES) {
      // residual of row vi sits in lane vi (loaded up front); fetch it into this lane
      o = round_bf(a.bias ? o + bf2f(a.bias[min(row, a.N - 1)]) : o) +
          __uint_as_float(((uint32_t)__shfl(res, vi)) << 16);
    } else if (a.bias) {
      o += bf2f(a.bias[min(row, a.N - 1)]);
    }
    if (LDS_OUT) {
      if ((lane & (GROUP - 1)) == 0) gemv_out_lds(smem, a.K)[wave * RPR + vi] = f2bf(o);
    } else if ((lane & (GROUP - 1)) == 0 && row < a.N) {
      a.y[row] = f2bf(o);
    }
    LGA_GTRACE(5);
  }
}

}  // namespace lga
