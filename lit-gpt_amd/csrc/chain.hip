// Chained decode GEMVs: the tail of one Llama block and the head of the next in ONE launch.
//
//   stage 0  attn.proj + residual        h_mid = x + proj(y_att)                 (lit_gpt/model.py:656, :591)
//   stage 1  RMSNorm(norm_2) + fc_1||fc_2 + SwiGLU   act = silu(fc_1 n) * fc_2 n  (:592, :712-716)
//   stage 2  mlp.proj + residual          h_out = h_mid + proj(act)               (:716, :592)
//   stage 3  RMSNorm + the next GEMV      next block's norm_1 + fused qkv (:619), or ln_f + lm_head (:518-519)
//
// Why: launched one by one, every GEMV pays a kernel boundary (~1.5 us) plus a ramp of ~2.4 us before its first
// weights land, during which HBM idles (tools/gemv_trace.py: 5.5-11 us launches, 35-45 % fixed cost). Here the
// workgroups of stage s+1 are dispatched as soon as stage s's workgroups leave room, issue ALL their weight loads
// at once, and only then wait for stage s's output — so the weight stream runs through every stage boundary.
//
// Correctness of the waits: stages occupy increasing blockIdx ranges and a consumer only ever waits for the
// stage right before its own; workgroups are dispatched in blockIdx order, so every producer is resident or done
// before any of its consumers is dispatched, and producers never wait on later stages (no deadlock). Every wait
// is bounded (~20 ms, then an error bit) so a broken assumption cannot hang the GPU. Hand-off protocol:
// gemv_body.h (MI355X_MICROARCH.md "Valid forms" row 1). The last workgroup of stage 3 (two-level count) re-arms
// all counters for the next launch (graph replays reuse them).
#include "gemv_body.h"
#include "litgpt_amd.h"
#include <cstdlib>

namespace lga {

constexpr int kChainStages = 4;
constexpr int kChainTop = kChainStages * kChainShards;  // counter index of the stage-3 completion count

struct ChainArgs {
  GemvArgs st[kChainStages];
  int wg_begin[kChainStages + 1];
  unsigned* cnt;  // (kChainStages * kChainShards + 1) counters, kChainStride apart, zero between launches
  unsigned* err;
};

template <int CC, int CI, int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, 8))) chain_kernel(ChainArgs c) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int s = (b >= c.wg_begin[1]) + (b >= c.wg_begin[2]) + (b >= c.wg_begin[3]);
  const int blk = b - c.wg_begin[s];
  ChainLink L;
  L.wait_cnt = s == 0 ? nullptr : c.cnt + (size_t)(s - 1) * kChainShards * kChainStride;
  L.wait_wgs = s == 0 ? 0 : c.wg_begin[s] - c.wg_begin[s - 1];
  L.post_cnt = c.cnt + (size_t)s * kChainShards * kChainStride;
  L.err = c.err;
  switch (s) {
    case 0: gemv_q4_body<4, CC, 0, false, false, true, true>(c.st[0], blk, smem, &L); break;
    case 1: gemv_q4_body<2, CC, 0, true, true, false, true>(c.st[1], blk, smem, &L); break;
    case 2: gemv_q4_body<(CI <= 3 ? 4 : 2), CI, 0, false, false, true, true>(c.st[2], blk, smem, &L); break;
    default: {
      const unsigned old = gemv_q4_body<4, CC, 0, false, true, false, true>(c.st[3], blk, smem, &L);
      if (threadIdx.x == 0) {
        const int wgs = c.wg_begin[4] - c.wg_begin[3];
        const int sh = blk % kChainShards;
        const unsigned shard_total = (unsigned)(wgs / kChainShards + (sh < wgs % kChainShards ? 1 : 0));
        if (old + 1 == shard_total) {  // last workgroup of its shard -> count the shard
          unsigned* top = c.cnt + (size_t)kChainTop * kChainStride;
          const unsigned done = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (done + 1 == (unsigned)min(wgs, kChainShards)) {  // every workgroup of every stage is past its wait
            for (int i = 0; i <= kChainTop; ++i)
              __hip_atomic_store(c.cnt + (size_t)i * kChainStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
      break;
    }
  }
}

template <int CC, int CI>
static void launch_chain(const ChainArgs& c, size_t lds, hipStream_t stream) {
  // occupancy floor (waves per SIMD): 6 keeps Llama-2-7B's 1376 gate_up workgroups resident in one round at the
  // price of register spills in the K = 11008 down stage; lab switch LGA_CHAIN_WAVES=4 / 6
  static const int w = [] { const char* e = getenv("LGA_CHAIN_WAVES"); return e ? atoi(e) : 4; }();
  if (w >= 6) chain_kernel<CC, CI, 6><<<c.wg_begin[kChainStages], 256, lds, stream>>>(c);
  else chain_kernel<CC, CI, 1><<<c.wg_begin[kChainStages], 256, lds, stream>>>(c);
}

}  // namespace lga

extern "C" size_t lga_decode_chain_counter_words(void) {
  return (size_t)(lga::kChainTop + 1) * lga::kChainStride;
}

extern "C" int lga_q4_decode_chain(const lga_chain_stage* stages, unsigned* counters, unsigned* err,
                                   hipStream_t stream) {
  using namespace lga;
  LGA_CHECK_ARG(stages && counters && err, "lga_q4_decode_chain: null pointer");
  const lga_chain_stage* s = stages;
  for (int i = 0; i < kChainStages; ++i) {
    LGA_CHECK_ARG(s[i].x && s[i].qweight && s[i].scales && s[i].y, "lga_q4_decode_chain: null stage pointer");
    LGA_CHECK_ARG(s[i].N > 0 && s[i].K > 0 && s[i].K % 32 == 0 && s[i].group >= 32 && s[i].group % 32 == 0 &&
                      s[i].K % s[i].group == 0, "lga_q4_decode_chain: bad stage geometry");
    LGA_CHECK_ARG(s[i].N % 4 == 0, "lga_q4_decode_chain: every stage needs N % 4 == 0");
  }
  // the block pattern and its in-launch data flow (the only hand-offs the waits cover)
  LGA_CHECK_ARG(s[0].residual && !s[0].norm_weight && !s[0].qweight2, "lga_q4_decode_chain: stage 0 is proj+residual");
  LGA_CHECK_ARG(s[1].qweight2 && s[1].scales2 && s[1].norm_weight && !s[1].residual,
                "lga_q4_decode_chain: stage 1 is norm + fc_1||fc_2");
  LGA_CHECK_ARG(s[2].residual && !s[2].norm_weight && !s[2].qweight2, "lga_q4_decode_chain: stage 2 is proj+residual");
  LGA_CHECK_ARG(s[3].norm_weight && !s[3].residual && !s[3].qweight2, "lga_q4_decode_chain: stage 3 is norm + GEMV");
  LGA_CHECK_ARG(s[1].x == s[0].y && s[2].x == s[1].y && s[2].residual == s[0].y && s[3].x == s[2].y,
                "lga_q4_decode_chain: stages must feed each other (x1 = y0, x2 = y1, res2 = y0, x3 = y2)");
  LGA_CHECK_ARG(s[1].K == s[0].N && s[2].K == s[1].N && s[3].K == s[2].N && s[0].N == s[2].N && s[3].K == s[1].K,
                "lga_q4_decode_chain: stage shapes do not chain");
  const int C = s[1].K, I = s[1].N;
  LGA_CHECK_ARG(s[0].K == C && s[3].K == C, "lga_q4_decode_chain: proj / next GEMV must read C = n_embd");
  const int cc = (C / 32 + 63) / 64, ci = (I / 32 + 63) / 64;
  ChainArgs c;
  // rows per wave as the standalone GEMVs pick them for these widths (same reduction order -> same bits)
  const int rpr[kChainStages] = {4, 2, ci <= 3 ? 4 : 2, 4};
  c.wg_begin[0] = 0;
  for (int i = 0; i < kChainStages; ++i) {
    GemvArgs& a = c.st[i];
    a = GemvArgs{};
    a.x = (const uint16_t*)s[i].x;
    a.qw = s[i].qweight;
    a.sc = s[i].scales;
    a.qw2 = s[i].qweight2;
    a.sc2 = s[i].scales2;
    a.residual = (const uint16_t*)s[i].residual;
    a.norm_w = (const uint16_t*)s[i].norm_weight;
    a.y = (uint16_t*)s[i].y;
    a.N = s[i].N;
    a.K = s[i].K;
    a.G = s[i].group;
    a.eps = s[i].norm_eps;
    c.wg_begin[i + 1] = c.wg_begin[i] + (a.N / rpr[i] + 3) / 4;
  }
  c.cnt = counters;
  c.err = err;
  const size_t lds = (size_t)(C > I ? C : I) * 2 + ((C > I ? C : I) / 32) * 4 + 16 * 4 + 16 * 4;
  if (cc == 1 && ci == 1) launch_chain<1, 1>(c, lds, stream);
  else if (cc == 1 && ci == 2) launch_chain<1, 2>(c, lds, stream);
  else if (cc == 2 && ci == 6) launch_chain<2, 6>(c, lds, stream);
  else {
    lga_set_error("lga_q4_decode_chain: no chained instantiation for this (n_embd, intermediate_size)");
    return (int)hipErrorInvalidValue;
  }
  LGA_LAUNCH_RETURN();
}
