// Batch-1 decode GEMV over packed 4-bit weights: y[n] = sum_k x[k] * dequant(W)[n, k]  (+ fused epilogues)
//
// Replaces the bitsandbytes 4-bit GEMV that `Linear4bit.forward` dispatches for one-token inputs
// (bnb `matmul_4bit` -> `gemv_4bit`, reached via BitsandbytesPrecision at reference generate/base.py:128-136)
// for every Linear of the decode step: qkv (lit_gpt/model.py:619), attn proj (:656), LLaMAMLP fc_1/fc_2/proj
// (:712-716) and lm_head (:519).
//
// MI355X design. A batch-1 GEMV is a pure weight stream (~1 flop/byte) whose launches are only 8-66 MB, so the
// launch ramp and load latency dominate unless the whole kernel's weights are in flight at once
// (tools/bw_probe: a bare 16-B/lane read of 8 / 25 / 46 / 66 MB takes 3.0 / 5.5 / 8.6 / 11.7 us).
// Measured cost split for the 25 MB qkv shape (tools/gemv_lab): streaming 5.0 us, + int4 dequant-dot 0.9 us,
// + per-row wave reductions 1.3-2.0 us, + the butterfly below only 0.4 us.
//  * One wave per row slot: a wave owns RPR consecutive rows; lane l owns 32-element chunk columns
//    l, l+64, ... (CPT of them). Every wave issues ALL its 16-B non-temporal weight loads (RPR*CPT per lane)
//    up front, one round per wave; enough waves (~3 workgroups per CU) hide the latency.
//  * The activation row is fetched BEFORE the weights (vmcnt is in order, so the wait for x leaves the weight
//    loads in flight), then staged once per workgroup in LDS as bf16 pairs (x_k, x_k+4) with per-chunk sums;
//    the fused RMSNorm (lit_gpt/rmsnorm.py:19-25: bf16(w * (x * rsqrt(mean(x^2) + eps))), the reference's
//    rounding point) runs during that staging, while the weights stream.
//  * int4-g: one AND-OR turns two nibbles into the bf16 pair (128+q_k, 128+q_k+4) for v_dot2c_f32_bf16, and
//    sum x*(q-8) = dot - 136*sum(x); nf4: codebook in LDS, fp32 FMAs; one scale/absmax FMA per 32 weights.
//  * Reduction: a transposed butterfly sums R = RPR (x2 for the dual GEMV) row partials across the wave with
//    log2(R) halving exchanges + DPP, instead of R separate wave reductions.
//  * Epilogues: +bias, +residual (Block residual add, model.py:591-592), dual-weight SwiGLU
//    (silu(fc_1 x) * fc_2 x, model.py:715) with the reference's bf16 rounding points.
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
};

template <int RPR, int CPT, int FMT, bool DUAL, bool NORM, bool RES>
__global__ void __launch_bounds__(256) gemv_q4_kernel(GemvArgs a) {
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
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* xl = (uint4*)smem;                        // K/8 uint4 (bf16 pairs)
  float* xsum = (float*)(smem + (size_t)a.K * 2);  // K/32 chunk sums
  float* red = xsum + a.K / 32;                    // 4
  float* nf4 = red + 4;                            // 16
  constexpr int R = DUAL ? 2 * RPR : RPR;          // values per lane entering the butterfly
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int NC = a.K / 32, n8 = a.K / 8, groups = a.K / a.G;
  const int row0 = (blockIdx.x * 4 + wave) * RPR;
  if (FMT == 1 && t < 16) nf4[t] = kNF4v[t];
  LGA_GTRACE_NOWAIT(0);

  // 1. activation (and norm weight) share of this thread: uint4 t, t+256, ... (clamped, branch-free)
  uint4 xr[CPT], nr[CPT];
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int u = min(t + 256 * i, n8 - 1);
    xr[i] = ((const uint4*)a.x)[u];
    if (NORM) nr[i] = ((const uint4*)a.norm_w)[u];
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
      s[i][j] = load_scale_bits<FMT>(a.sc, n * groups + g);
      if (DUAL) {
        w2[i][j] = ld_nt16(a.qw2 + n * (a.K / 2) + (size_t)c * 16);
        s2[i][j] = load_scale_bits<FMT>(a.sc2, n * groups + g);
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
    for (int i = 0; i < CPT; ++i) {
      const bool ok = t + 256 * i < n8;
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
    rs = 1.0f / sqrtf(((red[0] + red[1]) + (red[2] + red[3])) / (float)a.K + a.eps);
  }
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int u = t + 256 * i;
    uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};  // bf16 pairs (x0,x1) (x2,x3) (x4,x5) (x6,x7)
    if (NORM) {  // bf16(w * (x * rs)), rounded in hardware, two elements per instruction
      const uint32_t nw[4] = {nr[i].x, nr[i].y, nr[i].z, nr[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        d[q] = pack2(__fmul_rn(bflo(nw[q]), __fmul_rn(bflo(d[q]), rs)),
                     __fmul_rn(bfhi(nw[q]), __fmul_rn(bfhi(d[q]), rs)));
    }
    float cs = ((bflo(d[0]) + bfhi(d[0])) + (bflo(d[1]) + bfhi(d[1]))) +
               ((bflo(d[2]) + bfhi(d[2])) + (bflo(d[3]) + bfhi(d[3])));
    cs += __shfl_xor(cs, 1);  // 4 consecutive threads hold one 32-element chunk
    cs += __shfl_xor(cs, 2);
    if (u < n8) {
      // (x0,x4) (x1,x5) (x2,x6) (x3,x7): byte permutes of the bf16 pairs
      xl[u] = make_uint4(__builtin_amdgcn_perm(d[2], d[0], 0x05040100u), __builtin_amdgcn_perm(d[2], d[0], 0x07060302u),
                         __builtin_amdgcn_perm(d[3], d[1], 0x05040100u), __builtin_amdgcn_perm(d[3], d[1], 0x07060302u));
      if ((u & 3) == 0) xsum[u >> 2] = cs;
    }
  }
  __syncthreads();
  LGA_GTRACE_NOWAIT(3);
  LGA_GTRACE(4);

  // 4. dequant-dot every row of this wave, then one butterfly for all of them
  const uint32_t nmask = nibble_mask();
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
#pragma unroll
    for (int i = 0; i < RPR; ++i) {
      const float d = chunk_dot<FMT>(w[i][j], xc, xs, nf4, nmask);
      if (DUAL) {  // value index = 2*row + matrix (so the pair of one row lands in lanes l and l^8 / l^16 / l^32)
        part[2 * i] = fmaf(ok ? scale_of<FMT>(s[i][j]) : 0.0f, d, part[2 * i]);
        const float d2 = chunk_dot<FMT>(w2[i][j], xc, xs, nf4, nmask);
        part[2 * i + 1] = fmaf(ok ? scale_of<FMT>(s2[i][j]) : 0.0f, d2, part[2 * i + 1]);
      } else {
        part[i] = fmaf(ok ? scale_of<FMT>(s[i][j]) : 0.0f, d, part[i]);
      }
    }
  }
  const float tot = butterfly<R>(part, lane);
  const int vi = bfly_index<R>(lane);  // value index held by this lane
  constexpr int GROUP = 64 / R;        // lanes per value after the butterfly
  if (DUAL) {
    // partner value (other matrix, same row) sits in the lane whose value index differs in bit 0
    constexpr int PD = R == 8 ? 8 : (R == 4 ? 16 : 32);
    const float other = PD == 8 ? LGA_DPP(tot, 0x128) : __shfl_xor(tot, PD);
    const int row = row0 + (vi >> 1);
    if ((lane & (GROUP - 1)) == 0 && (vi & 1) == 0 && row < a.N) {
      const float g = round_bf(silu_f(round_bf(tot)));  // silu(bf16(fc_1 x)) -> bf16
      a.y[row] = f2bf(__fmul_rn(g, round_bf(other)));   // * bf16(fc_2 x)
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
    if ((lane & (GROUP - 1)) == 0 && row < a.N) a.y[row] = f2bf(o);
    LGA_GTRACE(5);
  }
}

template <int RPR, int CPT, int FMT, bool DUAL>
static void launch(const GemvArgs& a, hipStream_t stream) {
  const int waves = (a.N + RPR - 1) / RPR;
  const dim3 blocks((waves + 3) / 4, a.eidx ? a.slots : 1);
  const size_t lds = (size_t)a.K * 2 + (a.K / 32) * 4 + 4 * 4 + 16 * 4;
  const bool norm = a.norm_w != nullptr, res = a.residual != nullptr;
  if (DUAL) {
    if (norm) gemv_q4_kernel<RPR, CPT, FMT, DUAL, true, false><<<blocks, 256, lds, stream>>>(a);
    else gemv_q4_kernel<RPR, CPT, FMT, DUAL, false, false><<<blocks, 256, lds, stream>>>(a);
  } else if (norm) {
    if (res) gemv_q4_kernel<RPR, CPT, FMT, DUAL, true, true><<<blocks, 256, lds, stream>>>(a);
    else gemv_q4_kernel<RPR, CPT, FMT, DUAL, true, false><<<blocks, 256, lds, stream>>>(a);
  } else {
    if (res) gemv_q4_kernel<RPR, CPT, FMT, DUAL, false, true><<<blocks, 256, lds, stream>>>(a);
    else gemv_q4_kernel<RPR, CPT, FMT, DUAL, false, false><<<blocks, 256, lds, stream>>>(a);
  }
}

// variant: 0 = fewer rows per wave (more waves), 1 = more rows per wave; < 0 = heuristic
template <int FMT, bool DUAL>
static int dispatch(const GemvArgs& a, int variant, hipStream_t stream) {
  const int cpt = (a.K / 32 + 63) / 64;  // chunks per lane (== uint4 of x per thread)
  if (variant < 0) {
    const long rows = DUAL ? 2L * a.N : a.N;
    variant = rows >= 24000 ? 1 : 0;  // tall matrices: more rows per wave keep the grid ~3-4 workgroups per CU
  }
  // A persistent, double-buffered streaming form of this kernel (few workgroups per CU walking row tiles) measured
  // 10-70 % slower on every decode shape (tools/gemv_sweep.py, round 1) and was dropped.
  const bool big = (variant & 1) != 0;
#define LGA_L(RS, RB, CPT)                                                         \
  do {                                                                             \
    if (big) launch<(DUAL ? (RB) / 2 : (RB)), CPT, FMT, DUAL>(a, stream);          \
    else launch<(DUAL ? (RS) / 2 : (RS)), CPT, FMT, DUAL>(a, stream);              \
  } while (0)
  switch (cpt) {
    case 1: LGA_L(4, 8, 1); break;
    case 2: LGA_L(4, 8, 2); break;
    case 3: LGA_L(4, 8, 3); break;
    case 4: LGA_L(2, 4, 4); break;
    case 5:
    case 6: LGA_L(2, 4, 6); break;
    case 7:
    case 8: LGA_L(2, 4, 8); break;
    default:
      if (cpt <= 16) {
        LGA_L(2, 2, 16);
        break;
      }
      lga_set_error("lga_q4_gemv: K > 32768 is not supported");
      return (int)hipErrorInvalidValue;
  }
#undef LGA_L
  return 0;
}

}  // namespace lga

extern "C" int lga_q4_gemv(const void* x, const uint8_t* qweight, const void* scales, const void* bias,
                           const void* residual, const void* norm_weight, float norm_eps, void* y, int N, int K,
                           int group, int fmt, int variant, hipStream_t stream) {
  LGA_CHECK_ARG(x && qweight && scales && y, "lga_q4_gemv: null pointer");
  LGA_CHECK_ARG(N > 0 && K > 0 && K % 32 == 0, "lga_q4_gemv: K must be a positive multiple of 32");
  LGA_CHECK_ARG(group >= 32 && group % 32 == 0 && K % group == 0, "lga_q4_gemv: group must be a multiple of 32 dividing K");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1, "lga_q4_gemv: fmt must be 0 (int4-g) or 1 (nf4)");
  lga::GemvArgs a{(const uint16_t*)x, qweight, scales, nullptr, nullptr, (const uint16_t*)bias,
                  (const uint16_t*)residual, (const uint16_t*)norm_weight, (uint16_t*)y, N, K, group, norm_eps};
  const int rc = fmt == 0 ? lga::dispatch<0, false>(a, variant, stream) : lga::dispatch<1, false>(a, variant, stream);
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_q4_gemv_swiglu(const void* x, const uint8_t* qweight1, const void* scales1,
                                  const uint8_t* qweight2, const void* scales2, const void* norm_weight,
                                  float norm_eps, void* y, int N, int K, int group, int fmt, int variant,
                                  hipStream_t stream) {
  LGA_CHECK_ARG(x && qweight1 && scales1 && qweight2 && scales2 && y, "lga_q4_gemv_swiglu: null pointer");
  LGA_CHECK_ARG(N > 0 && K > 0 && K % 32 == 0, "lga_q4_gemv_swiglu: K must be a positive multiple of 32");
  LGA_CHECK_ARG(group >= 32 && group % 32 == 0 && K % group == 0, "lga_q4_gemv_swiglu: bad group");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1, "lga_q4_gemv_swiglu: fmt must be 0 or 1");
  lga::GemvArgs a{(const uint16_t*)x, qweight1, scales1, qweight2, scales2, nullptr, nullptr,
                  (const uint16_t*)norm_weight, (uint16_t*)y, N, K, group, norm_eps};
  const int rc = fmt == 0 ? lga::dispatch<0, true>(a, variant, stream) : lga::dispatch<1, true>(a, variant, stream);
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_q4_gemv_experts(const void* x, const uint8_t* qweight, const void* scales, const int32_t* expert_ids,
                                   int n_slots, int n_expert, long long w_stride, long long s_stride, int x_stride,
                                   void* y, int N, int K, int group, int fmt, int variant, hipStream_t stream) {
  LGA_CHECK_ARG(x && qweight && scales && expert_ids && y, "lga_q4_gemv_experts: null pointer");
  LGA_CHECK_ARG(N > 0 && K > 0 && K % 32 == 0, "lga_q4_gemv_experts: K must be a positive multiple of 32");
  LGA_CHECK_ARG(group >= 32 && group % 32 == 0 && K % group == 0, "lga_q4_gemv_experts: bad group");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1, "lga_q4_gemv_experts: fmt must be 0 or 1");
  LGA_CHECK_ARG(n_slots > 0 && n_slots <= 65535 && n_expert > 0 && w_stride >= (long long)N * K / 2 && s_stride > 0 &&
                    x_stride >= 0, "lga_q4_gemv_experts: bad routing geometry");
  lga::GemvArgs a{(const uint16_t*)x, qweight, scales, nullptr, nullptr, nullptr, nullptr, nullptr, (uint16_t*)y,
                  N, K, group, 0.0f, expert_ids, w_stride, s_stride, x_stride, n_expert, n_slots};
  const int rc = fmt == 0 ? lga::dispatch<0, false>(a, variant, stream) : lga::dispatch<1, false>(a, variant, stream);
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_q4_gemv_swiglu_experts(const void* x, const uint8_t* qweight1, const void* scales1,
                                          const uint8_t* qweight2, const void* scales2, const int32_t* expert_ids,
                                          int n_slots, int n_expert, long long w_stride, long long s_stride,
                                          const void* norm_weight, float norm_eps, void* y, int N, int K, int group,
                                          int fmt, int variant, hipStream_t stream) {
  LGA_CHECK_ARG(x && qweight1 && scales1 && qweight2 && scales2 && expert_ids && y,
                "lga_q4_gemv_swiglu_experts: null pointer");
  LGA_CHECK_ARG(N > 0 && K > 0 && K % 32 == 0, "lga_q4_gemv_swiglu_experts: K must be a positive multiple of 32");
  LGA_CHECK_ARG(group >= 32 && group % 32 == 0 && K % group == 0, "lga_q4_gemv_swiglu_experts: bad group");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1, "lga_q4_gemv_swiglu_experts: fmt must be 0 or 1");
  LGA_CHECK_ARG(n_slots > 0 && n_slots <= 65535 && n_expert > 0 && w_stride >= (long long)N * K / 2 && s_stride > 0,
                "lga_q4_gemv_swiglu_experts: bad routing geometry");
  LGA_CHECK_ARG(!norm_weight || K / 32 <= 128, "lga_q4_gemv_swiglu_experts: fused RMSNorm needs K <= 4096");
  lga::GemvArgs a{(const uint16_t*)x, qweight1, scales1, qweight2, scales2, nullptr, nullptr,
                  (const uint16_t*)norm_weight, (uint16_t*)y, N, K, group, norm_eps, expert_ids, w_stride, s_stride, 0,
                  n_expert, n_slots};
  const int rc = fmt == 0 ? lga::dispatch<0, true>(a, variant, stream) : lga::dispatch<1, true>(a, variant, stream);
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}

#ifdef LGA_GEMV_TRACE
extern "C" int lga_gemv_trace_read(unsigned long long* host, int n) {
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(lga::g_gemv_trace), (size_t)n * sizeof(unsigned long long));
  void* dptr = nullptr;
  if (e == hipSuccess) e = hipGetSymbolAddress(&dptr, HIP_SYMBOL(lga::g_gemv_trace));
  if (e == hipSuccess) e = hipMemset(dptr, 0, sizeof(lga::g_gemv_trace));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}
#endif
