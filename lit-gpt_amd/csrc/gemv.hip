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
//  * int4-g: one AND-OR turns two nibbles into the fp16 pair (1024 + q, or 1024 + 16 q for the high nibble of a
//    byte) for v_dot2c_f32_f16 against fp16 x pairs (odd slots staged / 16), and sum x*(q-8) = dot - corr
//    (decode_ops.h chunk_dot_rows); nf4: codebook in LDS, fp32 FMAs; one scale/absmax FMA per 32 weights.
//  * Reduction: a transposed butterfly sums R = RPR (x2 for the dual GEMV) row partials across the wave with
//    log2(R) halving exchanges + DPP, instead of R separate wave reductions.
//  * Epilogues: +bias, +residual (Block residual add, model.py:591-592), dual-weight SwiGLU
//    (silu(fc_1 x) * fc_2 x, model.py:715) with the reference's bf16 rounding points.
#include "gemv_body.h"
#include "gemv_stream.h"

namespace lga {

#ifndef LGA_GEMV_NW
#define LGA_GEMV_NW 4  // waves per workgroup
#endif
constexpr int kGemvNW = LGA_GEMV_NW;

template <int RPR, int CPT, int FMT, bool DUAL, bool NORM, bool RES>
__global__ void __launch_bounds__(kGemvNW * 64) gemv_q4_kernel(GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  gemv_q4_body<RPR, CPT, FMT, DUAL, NORM, RES, kGemvNW>(a, blockIdx.x, smem);
}

template <int RPR, int CPT, int FMT, bool DUAL>
static void launch(const GemvArgs& a, hipStream_t stream) {
  const int waves = (a.N + RPR - 1) / RPR;
  const dim3 blocks((waves + kGemvNW - 1) / kGemvNW, a.eidx ? a.slots : 1);
  size_t lds = (size_t)a.K * 2 + (a.K / 32) * 4 + 16 * 4 + 16 * 4;
#ifdef LGA_LAB_WG_PER_CU  // lab builds only: cap resident workgroups per CU through the LDS footprint
  lds = lds > (163840 / LGA_LAB_WG_PER_CU) ? lds : (size_t)(163840 / LGA_LAB_WG_PER_CU);
#endif
  constexpr int NT = kGemvNW * 64;
  const bool norm = a.norm_w != nullptr, res = a.residual != nullptr;
  if (DUAL) {
    if (norm) gemv_q4_kernel<RPR, CPT, FMT, DUAL, true, false><<<blocks, NT, lds, stream>>>(a);
    else gemv_q4_kernel<RPR, CPT, FMT, DUAL, false, false><<<blocks, NT, lds, stream>>>(a);
  } else if (norm) {
    if (res) gemv_q4_kernel<RPR, CPT, FMT, DUAL, true, true><<<blocks, NT, lds, stream>>>(a);
    else gemv_q4_kernel<RPR, CPT, FMT, DUAL, true, false><<<blocks, NT, lds, stream>>>(a);
  } else {
    if (res) gemv_q4_kernel<RPR, CPT, FMT, DUAL, false, true><<<blocks, NT, lds, stream>>>(a);
    else gemv_q4_kernel<RPR, CPT, FMT, DUAL, false, false><<<blocks, NT, lds, stream>>>(a);
  }
}

template <int RT, int CPT, int FMT, bool DUAL, bool NORM, bool RES>
__global__ void __launch_bounds__(256) gemv_q4s_kernel(GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  gemv_q4_stream<RT, CPT, FMT, DUAL, NORM, RES>(a, smem);
}

// greedy decode head: RMSNorm + lm_head GEMV (streaming form) + argmax + next-token embedding in one launch
template <int RT, int CPT, int FMT, bool NORM>
__global__ void __launch_bounds__(256) gemv_q4s_amax_kernel(GemvArgs a, AmaxArgs am) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  gemv_q4_stream<RT, CPT, FMT, false, NORM, false, true>(a, smem, am);
}

static int amax_grid(int N, int K) {  // the streaming form's grid for a plain GEMV (launch_stream, 3 per CU)
  const int tiles = (N + 1) / 2;
  return max(1, min(num_cu() * 3, (tiles + 3) / 4));
}

// streaming form (variant bit 2): RT rows per tile, `wpc` workgroups per CU (variant bits 4..7, default 2)
template <int RT, int CPT, int FMT, bool DUAL>
static void launch_stream(const GemvArgs& a, int wpc, hipStream_t stream) {
  const int tiles = (a.N + RT - 1) / RT;
  const int blocks = max(1, min(num_cu() * wpc, (tiles + 3) / 4));
  const size_t lds = (size_t)a.K * 2 + (a.K / 32) * 4 + 16 * 4 + 16 * 4;
  const bool norm = a.norm_w != nullptr, res = a.residual != nullptr;
  if (DUAL) {
    if (norm) gemv_q4s_kernel<RT, CPT, FMT, true, true, false><<<blocks, 256, lds, stream>>>(a);
    else gemv_q4s_kernel<RT, CPT, FMT, true, false, false><<<blocks, 256, lds, stream>>>(a);
  } else if (norm) {
    if (res) gemv_q4s_kernel<RT, CPT, FMT, false, true, true><<<blocks, 256, lds, stream>>>(a);
    else gemv_q4s_kernel<RT, CPT, FMT, false, true, false><<<blocks, 256, lds, stream>>>(a);
  } else {
    if (res) gemv_q4s_kernel<RT, CPT, FMT, false, false, true><<<blocks, 256, lds, stream>>>(a);
    else gemv_q4s_kernel<RT, CPT, FMT, false, false, false><<<blocks, 256, lds, stream>>>(a);
  }
}

// The streaming form pays off for tall matrices over short rows (tools/gemv_variants.py, Llama-2-7B shapes):
// fc_1 || fc_2 (2 x 11008 x 4096) 10.9 vs 12.2 us, lm_head (32000 x 4096) 14.3 vs 15.9 us at 3 workgroups per
// CU; not for qkv / o_proj / mlp.proj (equal or slower). Instantiated for K <= 4096 only.
template <int FMT, bool DUAL>
static int dispatch_stream(const GemvArgs& a, int variant, hipStream_t stream) {
  const int cpt = (a.K / 32 + 63) / 64;
  const int wpc = (variant >> 4) & 15 ? (variant >> 4) & 15 : (DUAL ? 2 : 3);
  switch (cpt) {
    case 1: launch_stream<(DUAL ? 1 : 2), 1, FMT, DUAL>(a, wpc, stream); break;
    case 2: launch_stream<(DUAL ? 1 : 2), 2, FMT, DUAL>(a, wpc, stream); break;
    default:
      lga_set_error("lga_q4_gemv: the streaming form covers K <= 4096");
      return (int)hipErrorInvalidValue;
  }
  return 0;
}

static bool stream_default(int N, int K, bool dual) {
  return K <= 4096 && (dual ? N >= 8192 : N >= 24000);
}

// variant: 0 = fewer rows per wave (more waves), 1 = more rows per wave; < 0 = heuristic
template <int FMT, bool DUAL>
static int dispatch(const GemvArgs& a, int variant, hipStream_t stream) {
  const int cpt = (a.K / 32 + 63) / 64;  // chunks per lane (== uint4 of x per thread)
  if (!a.eidx && a.K <= 4096 &&
      ((variant >= 0 && (variant & 4)) || (variant < 0 && stream_default(a.N, a.K, DUAL))))
    return dispatch_stream<FMT, DUAL>(a, variant < 0 ? 4 : variant, stream);
  if (variant < 0) {
    const long rows = DUAL ? 2L * a.N : a.N;
    variant = rows >= 24000 ? 1 : 0;  // tall matrices: more rows per wave keep the grid ~3-4 workgroups per CU
    // the out-projection shape (residual epilogue, 2048..4096 rows, K <= 6144): 2 rows per wave, twice the
    // workgroups — attn.proj 4096 x 4096 3.81 vs 4.18 us (tools/gemv_variants.py, round 5); qkv / down unchanged
    if (!DUAL && !a.eidx && a.residual && a.N >= 2048 && a.N <= 4096 && cpt <= 3) variant |= 8;
    // and for the router gate (N <= 64: 4 rows per wave left half the rows as repeats) and the mid-size qkv
    // projections with the RMSNorm fused (N 4096..8192: Mixtral's 6,144 rows) — gate 3.14 -> 2.70 us, Mixtral qkv
    // 5.71 -> 5.48 (tools/gemv_variants.py GEMV_SHAPES=mixtral, round 6). Not for row-parallel projections (no norm):
    // their fused all-reduce form (gemv_ar.hip) keeps the 4-row grouping bit for bit. moe_gate_route_kernel uses the
    // same 2-row body as the gate GEMV.
    if (!DUAL && !a.eidx && !a.residual && cpt <= 3 && (a.N <= 64 || (a.norm_w && a.N >= 4096 && a.N <= 8192)))
      variant |= 8;
  }
  // A persistent, double-buffered streaming form of this kernel (few workgroups per CU walking row tiles) measured
  // 10-70 % slower on every decode shape (tools/gemv_sweep.py, round 1) and was dropped.
  const bool big = (variant & 1) != 0;
  const bool half = (variant & 8) != 0;  // half the small variant's rows per wave (bit 3)
#define LGA_L(RS, RB, CPT)                                                         \
  do {                                                                             \
    if (big) launch<(DUAL ? (RB) / 2 : (RB)), CPT, FMT, DUAL>(a, stream);          \
    else if (half) launch<((RS) >= 4 ? (DUAL ? (RS) / 4 : (RS) / 2) : (DUAL ? (RS) / 2 : (RS))), CPT, FMT, DUAL>(a, stream); \
    else launch<(DUAL ? (RS) / 2 : (RS)), CPT, FMT, DUAL>(a, stream);              \
  } while (0)
  switch (cpt) {
    case 1: LGA_L(4, 8, 1); break;
    case 2: LGA_L(4, 8, 2); break;
    case 3: LGA_L(4, 8, 3); break;
    case 4: LGA_L(2, 4, 4); break;
    case 5:
    case 6: LGA_L(2, 4, 6); break;
    case 7: LGA_L(2, 4, 7); break;  // K 12,320..14,336 (Mixtral experts' proj, Llama-2-13B mlp.proj): exactly 7 chunks
                                    // per lane, 2 rows per wave as moe.hip's paired down-projection (bit-identical)
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

int lga::preload_gemv() {  // the prefill's lm_head row (last_token_only): the streaming form with the norm fused
  return lga::preload(lga::gemv_q4s_kernel<2, 1, 0, false, true, false>) +
         lga::preload(lga::gemv_q4s_kernel<2, 2, 0, false, true, false>) +
         lga::preload(lga::gemv_q4s_kernel<2, 1, 1, false, true, false>) +
         lga::preload(lga::gemv_q4s_kernel<2, 2, 1, false, true, false>);
}

extern "C" int lga_q4_gemv(const void* x, const uint8_t* qweight, const void* scales, const void* bias,
                           const void* residual, const void* norm_weight, float norm_eps, void* y, int N, int K,
                           int group, int fmt, int variant, hipStream_t stream) {
  LGA_CHECK_ARG(x && qweight && scales && y, "lga_q4_gemv: null pointer");
  LGA_CHECK_ARG(N > 0 && K > 0 && K % 32 == 0, "lga_q4_gemv: K must be a positive multiple of 32");
  LGA_CHECK_ARG(group >= 32 && group % 32 == 0 && K % group == 0, "lga_q4_gemv: group must be a multiple of 32 dividing K");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1 || fmt == 3, "lga_q4_gemv: fmt must be 0 (int4-g), 1 (nf4) or 3 (fp4)");
  lga::GemvArgs a{(const uint16_t*)x, qweight, scales, nullptr, nullptr, (const uint16_t*)bias,
                  (const uint16_t*)residual, (const uint16_t*)norm_weight, (uint16_t*)y, N, K, group, norm_eps};
  a.cb = lga::codebook_of(fmt);
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
  LGA_CHECK_ARG(fmt == 0 || fmt == 1 || fmt == 3, "lga_q4_gemv_swiglu: fmt must be 0, 1 or 3");
  lga::GemvArgs a{(const uint16_t*)x, qweight1, scales1, qweight2, scales2, nullptr, nullptr,
                  (const uint16_t*)norm_weight, (uint16_t*)y, N, K, group, norm_eps};
  a.cb = lga::codebook_of(fmt);
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
  LGA_CHECK_ARG(fmt == 0 || fmt == 1 || fmt == 3, "lga_q4_gemv_experts: fmt must be 0, 1 or 3");
  LGA_CHECK_ARG(n_slots > 0 && n_slots <= 65535 && n_expert > 0 && w_stride >= (long long)N * K / 2 && s_stride > 0 &&
                    x_stride >= 0, "lga_q4_gemv_experts: bad routing geometry");
  lga::GemvArgs a{(const uint16_t*)x, qweight, scales, nullptr, nullptr, nullptr, nullptr, nullptr, (uint16_t*)y,
                  N, K, group, 0.0f, expert_ids, w_stride, s_stride, x_stride, n_expert, n_slots};
  a.cb = lga::codebook_of(fmt);
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
  LGA_CHECK_ARG(fmt == 0 || fmt == 1 || fmt == 3, "lga_q4_gemv_swiglu_experts: fmt must be 0, 1 or 3");
  LGA_CHECK_ARG(n_slots > 0 && n_slots <= 65535 && n_expert > 0 && w_stride >= (long long)N * K / 2 && s_stride > 0,
                "lga_q4_gemv_swiglu_experts: bad routing geometry");
  LGA_CHECK_ARG(!norm_weight || K / 32 <= 128, "lga_q4_gemv_swiglu_experts: fused RMSNorm needs K <= 4096");
  lga::GemvArgs a{(const uint16_t*)x, qweight1, scales1, qweight2, scales2, nullptr, nullptr,
                  (const uint16_t*)norm_weight, (uint16_t*)y, N, K, group, norm_eps, expert_ids, w_stride, s_stride, 0,
                  n_expert, n_slots};
  a.cb = lga::codebook_of(fmt);
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

extern "C" size_t lga_q4_gemv_argmax_work_bytes(int N, int K) {
  return (size_t)lga::amax_grid(N, K) * 8 + 9 * 256;
}

extern "C" int lga_q4_gemv_argmax_embed(const void* x, const uint8_t* qweight, const void* scales,
                                        const void* norm_weight, float norm_eps, void* logits, int N, int K, int group,
                                        int fmt, void* work, int64_t* out_idx, int32_t* token_out, int64_t* pos_inout,
                                        const void* table, int C, int V, void* emb_out, hipStream_t stream) {
  LGA_CHECK_ARG(x && qweight && scales && logits && work, "lga_q4_gemv_argmax_embed: null pointer");
  LGA_CHECK_ARG(N > 0 && K > 0 && K % 32 == 0 && K <= 4096, "lga_q4_gemv_argmax_embed: K must be a multiple of 32, <= 4096");
  LGA_CHECK_ARG(group >= 32 && group % 32 == 0 && K % group == 0, "lga_q4_gemv_argmax_embed: bad group");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1 || fmt == 3, "lga_q4_gemv_argmax_embed: fmt must be 0, 1 or 3");
  LGA_CHECK_ARG(!table || (emb_out && C > 0 && C % 8 == 0 && V > 0 && ((uintptr_t)table % 16) == 0 &&
                           ((uintptr_t)emb_out % 16) == 0),
                "lga_q4_gemv_argmax_embed: table and emb_out must be 16-B aligned rows of C % 8 == 0");
  lga::GemvArgs a{(const uint16_t*)x, qweight, scales, nullptr, nullptr, nullptr, nullptr,
                  (const uint16_t*)norm_weight, (uint16_t*)logits, N, K, group, norm_eps};
  a.cb = lga::codebook_of(fmt);
  const int blocks = lga::amax_grid(N, K);
  lga::AmaxArgs am{(unsigned long long*)work, (unsigned*)((char*)work + (size_t)blocks * 8), out_idx, token_out,
                   pos_inout, (const uint16_t*)table, (uint16_t*)emb_out, C, V};
  const size_t lds = (size_t)K * 2 + (K / 32) * 4 + 16 * 4 + 16 * 4;
  const int cpt = (K / 32 + 63) / 64, kf = lga::kernel_fmt(fmt);
  const bool norm = norm_weight != nullptr;
#define LGA_AM(CPT, FMT)                                                                                  \
  do {                                                                                                    \
    if (norm) lga::gemv_q4s_amax_kernel<2, CPT, FMT, true><<<blocks, 256, lds, stream>>>(a, am);          \
    else lga::gemv_q4s_amax_kernel<2, CPT, FMT, false><<<blocks, 256, lds, stream>>>(a, am);              \
  } while (0)
  if (cpt == 1) {
    if (kf == 0) LGA_AM(1, 0);
    else LGA_AM(1, 1);
  } else {
    if (kf == 0) LGA_AM(2, 0);
    else LGA_AM(2, 1);
  }
#undef LGA_AM
  LGA_LAUNCH_RETURN();
}
