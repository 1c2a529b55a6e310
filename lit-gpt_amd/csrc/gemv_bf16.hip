// Batch-1 decode GEMV over bf16 weights: y[n] = sum_k x[k] * W[n, k]  (+ the same fused epilogues as gemv.hip)
//
// Serves BASELINE config 2 (Llama-2-7B with unquantized bf16 weights, precision bf16-true): every Linear of the
// decode step stays an nn.Linear (reference generate/base.py:128-136 without --quantize) and its one-token
// forward (`F.linear`, lit_gpt/model.py:619, :656, :712-716, :519) lands here instead of a rocBLAS GEMV.
//
// A bf16 GEMV moves 2 bytes per weight (13.2 GB per Llama-2-7B token) at ~0.5 flop/byte: a pure HBM stream.
// Layout and schedule mirror the 4-bit kernel:
//  * one wave per row slot owns RPR consecutive rows; a "pass" covers 4096 columns of a row: lane l reads the
//    16-B chunks l, l+64, ..., l+448 (8 weights each), so each wave-instruction is 1 KB contiguous of one row;
//  * the activation row (and norm weight) is fetched first, then every weight load of pass 0 is issued, and the
//    fused RMSNorm (lit_gpt/rmsnorm.py:19-25, the reference's rounding points) stages x into LDS while the
//    weights stream; rows longer than 4096 (mlp.proj, K = 11008) run more passes with the next pass's loads
//    issued before the current pass's math (vmcnt retires in order, so only the current pass is waited for);
//  * dot: v_dot2c_f32_bf16 straight on the (w_k, w_k+1) / (x_k, x_k+1) pairs, fp32 accumulation;
//  * one transposed butterfly reduces all row partials of the wave; bias / residual / SwiGLU epilogues with the
//    reference's bf16 rounding points (decode_ops.h, gemv.hip).
#include "decode_ops.h"

namespace lga {

struct GemvBArgs {
  const uint16_t* x;         // [K] bf16
  const uint16_t* w;         // [N][K] bf16
  const uint16_t* w2;        // dual: fc_2 [N][K]
  const uint16_t* bias;      // [N] or null
  const uint16_t* residual;  // [N] or null
  const uint16_t* norm_w;    // [K] or null (fused RMSNorm)
  uint16_t* y;               // [N]
  int N, K;
  float eps;
};

constexpr int BCPT = 8;                 // 16-B chunks per lane per pass
constexpr int BPASS = 64 * BCPT;        // chunks per pass (4096 columns)

template <int RPR, bool DUAL, bool NORM, bool RES, int XPT, bool MULTI>
__global__ void __launch_bounds__(256) gemv_bf16_kernel(GemvBArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* xl = (uint4*)smem;                     // K/8 uint4 (plain bf16 order)
  float* red = (float*)(smem + (size_t)a.K * 2);  // 4
  constexpr int NM = DUAL ? 2 : 1;                // weight matrices
  constexpr int R = NM * RPR;                     // values per lane entering the butterfly
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int n8 = a.K / 8;
  const int passes = MULTI ? (n8 + BPASS - 1) / BPASS : 1;
  const int row0 = (blockIdx.x * 4 + wave) * RPR;
  const uint16_t* wm[2] = {a.w, DUAL ? a.w2 : a.w};

  // 1. activation (and norm weight) share of this thread: uint4 t, t+256, ... (clamped, branch-free)
  uint4 xr[XPT], nr[XPT];
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int u = min(t + 256 * i, n8 - 1);
    xr[i] = ((const uint4*)a.x)[u];
    if (NORM) nr[i] = ((const uint4*)a.norm_w)[u];
  }
  // 2. pass-0 weight loads of every row of this wave (rows past N re-read row N-1; never stored)
  static_assert(R >= 1 && R <= 8, "row partials per lane");
  uint4 wa[NM][RPR][BCPT];
  uint4 wb[NM][MULTI ? RPR : 1][MULTI ? BCPT : 1];
  auto issue = [&](auto& buf, int pass) {
#pragma unroll
    for (int j = 0; j < BCPT; ++j) {
      const int c = min(pass * BPASS + lane + 64 * j, n8 - 1);
#pragma unroll
      for (int i = 0; i < RPR; ++i)
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          const size_t n = (size_t)min(row0 + i, a.N - 1);
          buf[m][i][j] = ld_nt16(wm[m] + n * a.K + (size_t)c * 8);
        }
    }
  };
  issue(wa, 0);
  uint32_t res = 0;
  if (RES) res = a.residual[min(row0 + (lane & (RPR - 1)), a.N - 1)];
  __builtin_amdgcn_sched_barrier(0);  // nothing that waits on x may move above the weight loads

  // 3. stage x into LDS (RMS-normalised when NORM) while the weights stream
  float rs = 1.0f;
  if (NORM) {
    float ss = 0.0f;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
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
    __syncthreads();
    rs = 1.0f / sqrtf(((red[0] + red[1]) + (red[2] + red[3])) / (float)a.K + a.eps);
  }
#pragma unroll
  for (int i = 0; i < XPT; ++i) {
    const int u = t + 256 * i;
    uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
    if (NORM) {  // bf16(w * (x * rs)), two elements per instruction
      const uint32_t nw[4] = {nr[i].x, nr[i].y, nr[i].z, nr[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        d[q] = pack2(__fmul_rn(bflo(nw[q]), __fmul_rn(bflo(d[q]), rs)),
                     __fmul_rn(bfhi(nw[q]), __fmul_rn(bfhi(d[q]), rs)));
    }
    if (u < n8) xl[u] = make_uint4(d[0], d[1], d[2], d[3]);
  }
  __syncthreads();

  // 4. dot every row of this wave pass by pass, then one butterfly for all of them
  float part[R < 2 ? 2 : R];
#pragma unroll
  for (int i = 0; i < (R < 2 ? 2 : R); ++i) part[i] = 0.0f;
  auto consume = [&](const auto& buf, int pass) {
#pragma unroll
    for (int j = 0; j < BCPT; ++j) {
      const int c = pass * BPASS + lane + 64 * j;
      const bool ok = c < n8;
      const uint4 xv = xl[min(c, n8 - 1)];
#pragma unroll
      for (int i = 0; i < RPR; ++i)
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          const uint4 wv = buf[m][i][j];
          float d = dot2_bf16(wv.x, xv.x, 0.0f);
          d = dot2_bf16(wv.y, xv.y, d);
          d = dot2_bf16(wv.z, xv.z, d);
          d = dot2_bf16(wv.w, xv.w, d);
          part[i * NM + m] += ok ? d : 0.0f;
        }
    }
  };
  if constexpr (MULTI) {
    for (int p = 0; p < passes; p += 2) {
      if (p + 1 < passes) issue(wb, p + 1);
      consume(wa, p);
      if (p + 1 < passes) {
        if (p + 2 < passes) issue(wa, p + 2);
        consume(wb, p + 1);
      }
    }
  } else {
    consume(wa, 0);
  }
  constexpr int RB = R < 2 ? 2 : R;
  const float tot = butterfly<RB>(part, lane);
  const int vi = bfly_index<RB>(lane);  // value index held by this lane
  constexpr int GROUP = 64 / RB;        // lanes per value after the butterfly
  if (DUAL) {
    // value index = 2*row + matrix: the fc_2 partner of a row sits in the lane whose value index differs in bit 0
    constexpr int PD = RB == 8 ? 8 : (RB == 4 ? 16 : 32);
    const float other = PD == 8 ? LGA_DPP(tot, 0x128) : __shfl_xor(tot, PD);
    const int row = row0 + (vi >> 1);
    if ((lane & (GROUP - 1)) == 0 && (vi & 1) == 0 && row < a.N) {
      const float g = round_bf(silu_f(round_bf(tot)));  // silu(bf16(fc_1 x)) -> bf16
      a.y[row] = f2bf(__fmul_rn(g, round_bf(other)));   // * bf16(fc_2 x)
    }
  } else {
    const uint32_t rv = RES ? (uint32_t)__shfl(res, vi) : 0u;  // residual of row vi sits in lane vi
    const int row = row0 + vi;
    float o = tot;
    if (RES) {
      o = round_bf(a.bias ? o + bf2f(a.bias[min(row, a.N - 1)]) : o) + __uint_as_float(rv << 16);
    } else if (a.bias) {
      o += bf2f(a.bias[min(row, a.N - 1)]);
    }
    if ((lane & (GROUP - 1)) == 0 && vi < RPR && row < a.N) a.y[row] = f2bf(o);
  }
}

template <int RPR, bool DUAL, int XPT, bool MULTI>
static void launch_b(const GemvBArgs& a, hipStream_t stream) {
  const int waves = (a.N + RPR - 1) / RPR;
  const dim3 blocks((waves + 3) / 4);
  const size_t lds = (size_t)a.K * 2 + 4 * 4;
  const bool norm = a.norm_w != nullptr, res = a.residual != nullptr;
  if (DUAL) {
    if (norm) gemv_bf16_kernel<RPR, DUAL, true, false, XPT, MULTI><<<blocks, 256, lds, stream>>>(a);
    else gemv_bf16_kernel<RPR, DUAL, false, false, XPT, MULTI><<<blocks, 256, lds, stream>>>(a);
  } else if (norm) {
    if (res) gemv_bf16_kernel<RPR, DUAL, true, true, XPT, MULTI><<<blocks, 256, lds, stream>>>(a);
    else gemv_bf16_kernel<RPR, DUAL, true, false, XPT, MULTI><<<blocks, 256, lds, stream>>>(a);
  } else {
    if (res) gemv_bf16_kernel<RPR, DUAL, false, true, XPT, MULTI><<<blocks, 256, lds, stream>>>(a);
    else gemv_bf16_kernel<RPR, DUAL, false, false, XPT, MULTI><<<blocks, 256, lds, stream>>>(a);
  }
}

template <bool DUAL>
static int dispatch_b(const GemvBArgs& a, hipStream_t stream) {
  const int n8 = a.K / 8;
  // one pass (K <= 4096): 2 rows per wave (fc_1 || fc_2: 1 row of each); longer rows double-buffer their
  // passes, 1 row per wave (keeps both buffers within ~64-128 VGPRs)
  if (n8 <= BPASS) {
    if (DUAL) launch_b<1, true, 2, false>(a, stream);
    else launch_b<2, false, 2, false>(a, stream);
  } else if (n8 <= 256 * 6) {  // K <= 12288
    if (DUAL) launch_b<1, true, 6, true>(a, stream);
    else launch_b<1, false, 6, true>(a, stream);
  } else if (n8 <= 256 * 16) {  // K <= 32768
    if (DUAL) launch_b<1, true, 16, true>(a, stream);
    else launch_b<1, false, 16, true>(a, stream);
  } else {
    lga_set_error("lga_bf16_gemv: K > 32768 is not supported");
    return (int)hipErrorInvalidValue;
  }
  return 0;
}

}  // namespace lga

extern "C" int lga_bf16_gemv(const void* x, const void* weight, const void* bias, const void* residual,
                             const void* norm_weight, float norm_eps, void* y, int N, int K, hipStream_t stream) {
  LGA_CHECK_ARG(x && weight && y, "lga_bf16_gemv: null pointer");
  LGA_CHECK_ARG(N > 0 && K > 0 && K % 8 == 0, "lga_bf16_gemv: K must be a positive multiple of 8");
  LGA_CHECK_ARG(((uintptr_t)x | (uintptr_t)weight | (uintptr_t)(norm_weight ? norm_weight : x)) % 16 == 0,
                "lga_bf16_gemv: x, weight and norm_weight must be 16-B aligned");
  lga::GemvBArgs a{(const uint16_t*)x, (const uint16_t*)weight, nullptr, (const uint16_t*)bias,
                   (const uint16_t*)residual, (const uint16_t*)norm_weight, (uint16_t*)y, N, K, norm_eps};
  const int rc = lga::dispatch_b<false>(a, stream);
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_bf16_gemv_swiglu(const void* x, const void* weight1, const void* weight2, const void* norm_weight,
                                    float norm_eps, void* y, int N, int K, hipStream_t stream) {
  LGA_CHECK_ARG(x && weight1 && weight2 && y, "lga_bf16_gemv_swiglu: null pointer");
  LGA_CHECK_ARG(N > 0 && K > 0 && K % 8 == 0, "lga_bf16_gemv_swiglu: K must be a positive multiple of 8");
  LGA_CHECK_ARG(((uintptr_t)x | (uintptr_t)weight1 | (uintptr_t)weight2 |
                 (uintptr_t)(norm_weight ? norm_weight : x)) % 16 == 0,
                "lga_bf16_gemv_swiglu: x, weights and norm_weight must be 16-B aligned");
  lga::GemvBArgs a{(const uint16_t*)x, (const uint16_t*)weight1, (const uint16_t*)weight2, nullptr, nullptr,
                   (const uint16_t*)norm_weight, (uint16_t*)y, N, K, norm_eps};
  const int rc = lga::dispatch_b<true>(a, stream);
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}
