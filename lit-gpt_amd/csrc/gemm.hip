// Prefill GEMM over packed 4-bit weights: Y[M, N] = X[M, K] . dequant(W)[N, K]^T  (+bias / +residual)
//
// Replaces bitsandbytes' M > 1 path of `Linear4bit.forward` (dequantize_4bit -> cuBLAS GEMM; upstream, reached
// through BitsandbytesPrecision, reference generate/base.py:128-136) for the prefill pass over the prompt
// (next_token(model, arange(0, T), prompt), generate/base.py:83-85).
//
// MI355X design: 128x128 output tile per 256-thread workgroup (2x2 waves, 64x64 per wave = 4x4 tiles of
// v_mfma_f32_16x16x32_bf16), K-step 32, double-buffered LDS (X and dequantised W tiles, 16-B chunks XOR-swizzled
// by row so the 16-lane ds_read_b128 groups are conflict-free), next tile's global loads issued before the
// current tile's MFMAs.
//   int4-g: W enters the MFMA as the exact small integers (q - 8) in bf16; per-column group scales are applied
//           to a per-group fp32 partial accumulator (exact dequant semantics, like the decode GEMV);
//   nf4   : W is dequantised to bf16(NF4[c] * absmax) — the same rounding bitsandbytes' dequantize_4bit applies
//           before its GEMM.
#include "common.h"

namespace lga {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 32;

__device__ __forceinline__ int swz(int row, int chunk) { return row * 64 + 16 * (chunk ^ ((row >> 2) & 3)); }

__constant__ float kNF4g[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f, -0.28444138169288635f,
    -0.18477343022823334f, -0.09105003625154495f, 0.0f, 0.07958029955625534f, 0.16093020141124725f,
    0.24611230194568634f, 0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
    0.7229568362236023f, 1.0f};

struct GemmArgs {
  const uint16_t* x;  // [M][K]
  const uint8_t* qw;  // [N][K/2]
  const void* sc;     // [N][K/G]
  const uint16_t* bias;
  const uint16_t* residual;  // [M][N]
  uint16_t* y;               // [M][N]
  int M, N, K, G;
};

template <int FMT>
__global__ void __launch_bounds__(256) gemm_q4_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * 2 * BM * BK * 2];  // [buf][A|B][128 rows][64 B]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int nk = a.K / BK, groups = a.K / a.G;
  const size_t wrow_bytes = (size_t)a.K / 2;

  // global -> register staging
  uint4 xa[2];
  uint2 wq;
  float wscale = 0.0f;  // nf4 absmax for this thread's W row / block
  const int a_row0 = tid >> 2, a_chunk = tid & 3;
  const int w_row = tid >> 1, w_half = tid & 1;
  const int w_n = min(n0 + w_row, a.N - 1);

  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = m0 + a_row0 + 64 * i;
      xa[i] = r < a.M ? *(const uint4*)(a.x + (size_t)r * a.K + kt * BK + a_chunk * 8) : make_uint4(0, 0, 0, 0);
    }
    wq = *(const uint2*)(a.qw + (size_t)w_n * wrow_bytes + (kt * BK + w_half * 16) / 2);
    if (FMT == 1) wscale = ((const float*)a.sc)[(size_t)w_n * groups + (kt * BK) / a.G];
  };
  auto lstore = [&](int buf) {
    unsigned char* A = lds + buf * (2 * BM * BK * 2);
    unsigned char* B = A + BM * BK * 2;
#pragma unroll
    for (int i = 0; i < 2; ++i) *(uint4*)(A + swz(a_row0 + 64 * i, a_chunk)) = xa[i];
    uint32_t out[8];
    const uint32_t wd[2] = {wq.x, wq.y};
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      const uint32_t n_lo = (wd[e / 8] >> (4 * (e % 8))) & 0xF, n_hi = (wd[e / 8] >> (4 * (e % 8) + 4)) & 0xF;
      float lo, hi;
      if (FMT == 0) {
        lo = (float)((int)n_lo - 8);
        hi = (float)((int)n_hi - 8);
      } else {
        lo = __fmul_rn(kNF4g[n_lo], wscale);
        hi = __fmul_rn(kNF4g[n_hi], wscale);
      }
      out[e / 2] = pack2(lo, hi);
    }
    *(uint4*)(B + swz(w_row, 2 * w_half)) = make_uint4(out[0], out[1], out[2], out[3]);
    *(uint4*)(B + swz(w_row, 2 * w_half + 1)) = make_uint4(out[4], out[5], out[6], out[7]);
  };

  f32x4_t acc[4][4], tmp[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      tmp[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }

  gload(0);
  lstore(0);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const unsigned char* A = lds + cur * (2 * BM * BK * 2);
    const unsigned char* B = A + BM * BK * 2;
    bf16x8_t af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i] = *(const bf16x8_t*)(A + swz(wm * 64 + i * 16 + fr, fk));
      bfr[i] = *(const bf16x8_t*)(B + swz(wn * 64 + i * 16 + fr, fk));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (FMT == 0) tmp[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], tmp[i][j], 0, 0, 0);
        else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    if (FMT == 0 && ((kt + 1) * BK) % a.G == 0) {
      const int g = (kt * BK) / a.G;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = min(n0 + wn * 64 + j * 16 + fr, a.N - 1);
        const float s = bf2f(((const uint16_t*)a.sc)[(size_t)n * groups + g]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[i][j] += tmp[i][j] * s;
          tmp[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + fr;
    if (n >= a.N) continue;
    const float b = a.bias ? bf2f(a.bias[n]) : 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + fk * 4 + r;
        if (m >= a.M) continue;
        float out = acc[i][j][r] + b;
        if (a.residual) out = round_bf(out) + bf2f(a.residual[(size_t)m * a.N + n]);
        a.y[(size_t)m * a.N + n] = f2bf(out);
      }
  }
}

}  // namespace lga

extern "C" int lga_q4_gemm(const void* x, const uint8_t* qweight, const void* scales, const void* bias,
                           const void* residual, void* y, int M, int N, int K, int group, int fmt,
                           hipStream_t stream) {
  LGA_CHECK_ARG(x && qweight && scales && y, "lga_q4_gemm: null pointer");
  LGA_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 32 == 0, "lga_q4_gemm: K must be a positive multiple of 32");
  LGA_CHECK_ARG(group >= 32 && group % 32 == 0 && K % group == 0, "lga_q4_gemm: group must be a multiple of 32 dividing K");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1, "lga_q4_gemm: fmt must be 0 or 1");
  lga::GemmArgs a{(const uint16_t*)x, qweight, scales, (const uint16_t*)bias, (const uint16_t*)residual,
                  (uint16_t*)y, M, N, K, group};
  const dim3 grid((N + lga::BN - 1) / lga::BN, (M + lga::BM - 1) / lga::BM);
  if (fmt == 0) lga::gemm_q4_kernel<0><<<grid, 256, 0, stream>>>(a);
  else lga::gemm_q4_kernel<1><<<grid, 256, 0, stream>>>(a);
  LGA_LAUNCH_RETURN();
}
