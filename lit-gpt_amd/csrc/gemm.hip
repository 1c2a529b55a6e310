// Prefill GEMM over packed 4-bit weights: Y[M, N] = X[M, K] . dequant(W)[N, K]^T  (+bias / +residual)
//
// Replaces bitsandbytes' M > 1 path of `Linear4bit.forward` (dequantize_4bit -> cuBLAS GEMM; upstream, reached
// through BitsandbytesPrecision, reference generate/base.py:128-136) for the prefill pass over the prompt
// (next_token(model, arange(0, T), prompt), generate/base.py:83-85).
//
// MI355X design: 128x128 output tile per 256-thread workgroup (2x2 waves, 64x64 per wave = 4x4 tiles of
// v_mfma_f32_16x16x32_bf16), K-step 64 (two MFMA k-slices per LDS tile, half the barriers of a 32-deep step),
// double-buffered LDS (X and dequantised W tiles, 128-B rows of 16-B chunks XOR-swizzled by row so the 16-lane
// ds_read_b128 groups are conflict-free), next tile's global loads issued before the current tile's MFMAs.
// W is dequantised while it is staged, to bf16(value(nibble) * scale) — the rounding the reference's path applies
// (bitsandbytes dequantize_4bit to the bf16 weight, then the GEMM), and exactly the bf16 weights the CPU oracle
// multiplies: int4-g value = nibble - 8 with the bf16 group scale, nf4 value = NF4[nibble] with the fp32 absmax.
// (An exact-integer-B variant with per-group fp32 partial sums needed 324 VGPRs and ran at half the speed; a
// three-stage form — X two K-steps ahead in a ring of 3 LDS tiles, packed W one step ahead in registers, 80 KB LDS —
// ran at 533 vs 644 TFLOP/s per int4 layer, tools/gemm_sweep.py round 2: the two-stage loop is not latency-bound.)
#include "common.h"

namespace lga {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 64;
#ifndef LGA_GEMM_GLDS
#define LGA_GEMM_GLDS 1  // X (and bf16 W) tiles staged global -> LDS directly (global_load_lds_dwordx4)
#endif
#ifndef LGA_GEMM_XCD
#define LGA_GEMM_XCD 0  // XCD-aware tile order (each XCD walks a contiguous run of tiles): measured 1-3 % slower
#endif
constexpr int TILE_BYTES = BM * BK * 2;  // one operand tile in LDS (128 rows x 128 B)

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + 16 * (chunk ^ (row & 7)); }

struct GemmArgs {
  const uint16_t* x;  // [M][K]
  const uint8_t* qw;  // [N][K/2]
  const void* sc;     // [N][K/G]
  const uint16_t* bias;
  const uint16_t* residual;  // [M][N]
  uint16_t* y;               // [M][N]
  int M, N, K, G;
  int cb = 0;  // codebook row of kCode4 (FMT 1): 0 nf4, 1 fp4
};

// X tile rows [r0, r0 + 8) of one 128-B-row tile, one wave instruction: lane L fills LDS bytes base + 16 L (row
// r0 + L/8, physical chunk L%8), so it loads the logical chunk that swz() puts there: (L%8) ^ (row & 7)
__device__ __forceinline__ void glds_rows8(const uint16_t* src, int ld, int row_lo, int row_max, int k0,
                                           unsigned char* lds_rows, int lane) {
  const int r = row_lo + (lane >> 3);
  const int lc = (lane & 7) ^ (r & 7);
  const uint16_t* g = src + (size_t)min(r, row_max) * ld + k0 + lc * 8;
  __builtin_amdgcn_global_load_lds((const void*)g, (__attribute__((address_space(3))) void*)lds_rows, 16, 0, 0);
}

template <int FMT, bool GLDS>
__global__ void __launch_bounds__(256) gemm_q4_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * 2 * TILE_BYTES];  // [buf][A|B]
  __shared__ float wtab[16];  // nibble -> value: nibble - 8 (int4-g) or the NF4 codebook
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  int bx = blockIdx.x, by = blockIdx.y;
  if (LGA_GEMM_XCD) {  // block b runs on XCD b % 8: give each XCD a contiguous run of tiles (x fastest)
    const int nx = gridDim.x, T = nx * gridDim.y, b = by * nx + bx;
    if (T % 8 == 0) {
      const int t = (b % 8) * (T / 8) + b / 8;
      bx = t % nx;
      by = t / nx;
    }
  }
  const int m0 = by * BM, n0 = bx * BN;
  const int nk = (a.K + BK - 1) / BK, groups = FMT == 2 ? 1 : a.K / a.G;
  const size_t wrow_bytes = (size_t)a.K / 2;
  if (tid < 16) wtab[tid] = FMT == 1 ? kCode4[a.cb][tid] : (float)(tid - 8);

  // global -> register staging: X 4 x 16 B per thread (row tid/8 + 32 i, chunk tid%8); W one row-half of 32 k
  uint4 xa[4];
  uint4 wq, wbf[FMT == 2 ? 4 : 1];  // packed nibbles (4-bit formats) / 32 bf16 weights (FMT 2)
  float wscale = 0.0f;  // group scale (int4-g, bf16) / block absmax (nf4, fp32) of this thread's 32 weights
  const int a_row = tid >> 3, a_chunk = tid & 7;
  const int w_row = tid >> 1, w_half = tid & 1;
  const int w_n = min(n0 + w_row, a.N - 1);

  auto gload = [&](int kt) {
    if (GLDS) {  // K % 64 == 0 here (host): X tile (and bf16 W tile) straight into LDS buffer kt & 1
      unsigned char* A = lds + (kt & 1) * (2 * TILE_BYTES);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r0 = (wave * 4 + i) * 8;
        glds_rows8(a.x, a.K, m0 + r0, a.M - 1, kt * BK, A + r0 * 128, lane);
        if (FMT == 2) glds_rows8((const uint16_t*)a.qw, a.K, n0 + r0, a.N - 1, kt * BK, A + TILE_BYTES + r0 * 128, lane);
      }
      if (FMT == 2) return;
      const int wk = kt * BK + w_half * 32;
      wq = *(const uint4*)(a.qw + (size_t)w_n * wrow_bytes + wk / 2);
      const size_t si = (size_t)w_n * groups + wk / a.G;
      wscale = FMT == 0 ? bf2f(((const uint16_t*)a.sc)[si]) : ((const float*)a.sc)[si];
      return;
    }
    // K % 64 == 32 leaves a half tile at the end: its upper X half is zero-filled (so it adds nothing) and its W
    // half re-reads the row start (in bounds, multiplied by those zeros)
    const bool a_in = kt * BK + a_chunk * 8 < a.K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = min(m0 + a_row + 32 * i, a.M - 1);  // rows past M duplicate row M-1 (never stored)
      const uint4 v = *(const uint4*)(a.x + (size_t)r * a.K + (a_in ? kt * BK + a_chunk * 8 : 0));
      xa[i] = a_in ? v : make_uint4(0, 0, 0, 0);
    }
    const int wk = kt * BK + w_half * 32 < a.K ? kt * BK + w_half * 32 : 0;
    if (FMT == 2) {
      const uint4* src = (const uint4*)((const uint16_t*)a.qw + (size_t)w_n * a.K + wk);
#pragma unroll
      for (int c = 0; c < 4; ++c) wbf[c] = src[c];
      return;
    }
    wq = *(const uint4*)(a.qw + (size_t)w_n * wrow_bytes + wk / 2);
    const size_t si = (size_t)w_n * groups + wk / a.G;
    wscale = FMT == 0 ? bf2f(((const uint16_t*)a.sc)[si]) : ((const float*)a.sc)[si];
  };
  auto lstore = [&](int buf) {
    unsigned char* A = lds + buf * (2 * TILE_BYTES);
    unsigned char* B = A + TILE_BYTES;
    if (!GLDS) {
#pragma unroll
      for (int i = 0; i < 4; ++i) *(uint4*)(A + swz(a_row + 32 * i, a_chunk)) = xa[i];
    }
    if (FMT == 2) {
      if (GLDS) return;
#pragma unroll
      for (int c = 0; c < 4; ++c) *(uint4*)(B + swz(w_row, w_half * 4 + c)) = wbf[c];
      return;
    }
    const uint32_t wd[4] = {wq.x, wq.y, wq.z, wq.w};  // 32 nibbles = 4 chunks of 8 k
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      uint32_t o4[4];
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const uint32_t lo = (wd[c] >> (4 * e)) & 0xF, hi = (wd[c] >> (4 * e + 4)) & 0xF;
        if (FMT == 0) {  // int4-g: value = nibble - 8, exact in fp32 (no LDS table read on this path)
          o4[e / 2] = pack2(__fmul_rn((float)((int)lo - 8), wscale), __fmul_rn((float)((int)hi - 8), wscale));
        } else {
          o4[e / 2] = pack2(__fmul_rn(wtab[lo], wscale), __fmul_rn(wtab[hi], wscale));
        }
      }
      *(uint4*)(B + swz(w_row, w_half * 4 + c)) = make_uint4(o4[0], o4[1], o4[2], o4[3]);
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  gload(0);
  __syncthreads();  // nf4 table
  lstore(0);
  if (GLDS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const unsigned char* A = lds + cur * (2 * TILE_BYTES);
    const unsigned char* B = A + TILE_BYTES;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {  // two 32-deep MFMA k-slices per tile
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = *(const bf16x8_t*)(A + swz(wm * 64 + i * 16 + fr, sub * 4 + fk));
        bfr[i] = *(const bf16x8_t*)(B + swz(wn * 64 + i * 16 + fr, sub * 4 + fk));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    if (GLDS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-direct loads have landed
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

// bf16 weights [N][K] (BASELINE config 2, unquantized nn.Linear; reference F.linear in bf16-true): the same tiles
// with W staged as stored.
extern "C" int lga_bf16_gemm(const void* x, const void* weight, const void* bias, const void* residual, void* y,
                             int M, int N, int K, hipStream_t stream) {
  LGA_CHECK_ARG(x && weight && y, "lga_bf16_gemm: null pointer");
  LGA_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 32 == 0, "lga_bf16_gemm: K must be a positive multiple of 32");
  LGA_CHECK_ARG(((uintptr_t)x | (uintptr_t)weight) % 16 == 0, "lga_bf16_gemm: x and weight must be 16-B aligned");
  lga::GemmArgs a{(const uint16_t*)x, (const uint8_t*)weight, nullptr, (const uint16_t*)bias,
                  (const uint16_t*)residual, (uint16_t*)y, M, N, K, 32};
  const dim3 grid((N + lga::BN - 1) / lga::BN, (M + lga::BM - 1) / lga::BM);
  if (LGA_GEMM_GLDS && K % lga::BK == 0) lga::gemm_q4_kernel<2, true><<<grid, 256, 0, stream>>>(a);
  else lga::gemm_q4_kernel<2, false><<<grid, 256, 0, stream>>>(a);
  LGA_LAUNCH_RETURN();
}

extern "C" int lga_q4_gemm(const void* x, const uint8_t* qweight, const void* scales, const void* bias,
                           const void* residual, void* y, int M, int N, int K, int group, int fmt,
                           hipStream_t stream) {
  LGA_CHECK_ARG(x && qweight && scales && y, "lga_q4_gemm: null pointer");
  LGA_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 32 == 0, "lga_q4_gemm: K must be a positive multiple of 32");
  LGA_CHECK_ARG(group >= 32 && group % 32 == 0 && K % group == 0, "lga_q4_gemm: group must be a multiple of 32 dividing K");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1 || fmt == 3, "lga_q4_gemm: fmt must be 0, 1 or 3");
  lga::GemmArgs a{(const uint16_t*)x, qweight, scales, (const uint16_t*)bias, (const uint16_t*)residual,
                  (uint16_t*)y, M, N, K, group, lga::codebook_of(fmt)};
  const dim3 grid((N + lga::BN - 1) / lga::BN, (M + lga::BM - 1) / lga::BM);
  const bool glds = LGA_GEMM_GLDS && K % lga::BK == 0;
  if (fmt == 0) {
    if (glds) lga::gemm_q4_kernel<0, true><<<grid, 256, 0, stream>>>(a);
    else lga::gemm_q4_kernel<0, false><<<grid, 256, 0, stream>>>(a);
  } else {
    if (glds) lga::gemm_q4_kernel<1, true><<<grid, 256, 0, stream>>>(a);
    else lga::gemm_q4_kernel<1, false><<<grid, 256, 0, stream>>>(a);
  }
  LGA_LAUNCH_RETURN();
}
