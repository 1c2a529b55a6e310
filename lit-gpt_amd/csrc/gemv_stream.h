// Streaming form of the decode GEMV (gemv.hip dispatches it with variant bit 2): a fixed grid of a few workgroups
// per CU whose waves walk row TILES (RT rows, all CPT chunks of each), two tiles in flight per wave: the loads of
// tile k+2 are issued right after tile k's dequant-dot, so a wave's dot work overlaps its own stream instead of
// piling up behind the last load of a one-shot wave (tools/gemv_variants.py: the dequant-dot of the one-shot form
// costs 1.3-2 us per launch on the 7B shapes although the VALU is ~25 % busy). Same x staging, same per-row
// arithmetic and rounding points as gemv_q4_body (bit-identical results), same epilogues.
#pragma once
#include "gemv_body.h"

namespace lga {

template <int RT, int CPT, int FMT, bool DUAL>
struct GemvTile {
  static constexpr int R = DUAL ? 2 * RT : RT;
  uint4 w[R][CPT];      // value index r = 2*row + matrix (DUAL) or row
  uint32_t s[R][CPT];
  uint32_t res;
};

// AMAX (greedy decode: lm_head + argmax in one launch): every row's bf16 logit is also offered to a running
// (value, index) arg-max with torch.argmax's order (NaN first, then larger, ties to the lower index — a strict total
// order, so the reduction order never changes the winner); each workgroup publishes its winner, and the workgroup
// that arrives last reduces them, writes the token / advances input_pos as lga_argmax does and gathers the token's
// embedding row for the next step (lga_argmax_embed).
struct AmaxArgs {
  unsigned long long* cand;  // [gridDim.x] {value bits, index} written sc1
  unsigned* cnt;             // 9 counters, 256 B apart: 8 per-(blockIdx % 8) classes + the top one (re-armed)
  int64_t* out_idx;
  int32_t* token_out;
  int64_t* pos_inout;
  const uint16_t* table;  // [V][C] bf16 or null
  uint16_t* emb_out;
  int C, V;
};

__device__ __forceinline__ bool amax_better(float v, int i, float bv, int bi) {  // = sample.hip better()
  const bool vn = v != v, bn = bv != bv;
  if (vn || bn) return vn && (!bn || i < bi);
  return (v > bv) || (v == bv && i < bi);
}
__device__ __forceinline__ void amax_take(float v, int i, float& bv, int& bi) {
  const bool t = amax_better(v, i, bv, bi);
  bv = t ? v : bv;
  bi = t ? i : bi;
}

template <int RT, int CPT, int FMT, bool DUAL, bool NORM, bool RES, bool AMAX = false>
__device__ __forceinline__ void gemv_q4_stream(GemvArgs a, unsigned char* smem, AmaxArgs am = AmaxArgs{}) {
  static_assert(!AMAX || (!DUAL && !RES), "AMAX: a plain (lm_head) GEMV");
  constexpr int NW = 4, NT = NW * 64;
  constexpr int XI = (CPT * 4 + NW - 1) / NW;
  using Tile = GemvTile<RT, CPT, FMT, DUAL>;
  constexpr int R = Tile::R;
  uint4* xl = (uint4*)smem;
  float* xsum = (float*)(smem + (size_t)a.K * 2);
  float* red = xsum + a.K / 32;
  float* nf4 = red + 16;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int NC = a.K / 32, n8 = a.K / 8, groups = a.K / a.G;
  const int gw = blockIdx.x * NW + wave, W = gridDim.x * NW;
  const int T = (a.N + RT - 1) / RT;
  if (FMT == 1 && t < 16) nf4[t] = kCode4[a.cb][t];
  // AMAX: the position is read up front (only the last workgroup uses it), so its update is a store, not a load
  const int64_t am_p0 = (AMAX && am.pos_inout && t == 0) ? *am.pos_inout : 0;

  // 1. activation (and norm weight) share of this thread, first in the vmcnt order
  uint4 xr[XI], nr[XI];
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int u = min(t + NT * i, n8 - 1);
    xr[i] = ((const uint4*)a.x)[u];
    if (NORM) nr[i] = ((const uint4*)a.norm_w)[u];
  }
  // 2. the first two tiles of this wave. A tile past the end loads row 0's chunks (one cached 1-KB line per
  //    instruction) so every wave issues the same instruction stream and the compiler's counted vmcnt waits stay
  //    exact; its results are never stored.
  auto issue = [&](Tile& b, int tile) {
    const bool live = tile < T;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int c = min(lane + 64 * j, NC - 1);
      const int g = (c * 32) / a.G;
#pragma unroll
      for (int i = 0; i < RT; ++i) {
        const size_t n = live ? (size_t)min(tile * RT + i, a.N - 1) : 0;
        b.w[DUAL ? 2 * i : i][j] = ld_nt16(a.qw + n * (a.K / 2) + (size_t)c * 16);
        b.s[DUAL ? 2 * i : i][j] = load_scale_bits<FMT>(a.sc, n * groups + g);
        if (DUAL) {
          b.w[2 * i + 1][j] = ld_nt16(a.qw2 + n * (a.K / 2) + (size_t)c * 16);
          b.s[2 * i + 1][j] = load_scale_bits<FMT>(a.sc2, n * groups + g);
        }
      }
    }
    if (RES) b.res = a.residual[live ? min(tile * RT + (RT > 1 ? (lane & (RT - 1)) : 0), a.N - 1) : 0];
  };
  Tile A, B;
  issue(A, gw);
  issue(B, gw + W);
  __builtin_amdgcn_sched_barrier(0);

  // 3. stage x (RMS-normalised when NORM) into LDS while the first tiles stream (gemv_q4_body step 3)
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
    __syncthreads();
    const float tot = (red[0] + red[1]) + (red[2] + red[3]);
    rs = 1.0f / sqrtf(tot / (float)a.K + a.eps);
  }
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int u = t + NT * i;
    uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
    if (NORM) {
      const uint32_t nw[4] = {nr[i].x, nr[i].y, nr[i].z, nr[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        d[q] = pack2(__fmul_rn(bflo(nw[q]), __fmul_rn(bflo(d[q]), rs)),
                     __fmul_rn(bfhi(nw[q]), __fmul_rn(bfhi(d[q]), rs)));
    }
    uint4 xv;
    float cs = stage_x8<FMT>(d, xv);
    cs += __shfl_xor(cs, 1);
    cs += __shfl_xor(cs, 2);
    if (u < n8) {
      xl[u] = xv;
      if ((u & 3) == 0) xsum[u >> 2] = cs;
    }
  }
  __syncthreads();

  // 4. tile loop: dot + butterfly + epilogue of tile k, then issue tile k + 2 into the freed buffer
  const uint32_t nmask = nibble_mask(), nmagic = f16_magic(), nmask_hi = nibble_mask_hi();
  float abv = -INFINITY;  // AMAX: this lane's best (value, row)
  int abi = 0x7FFFFFFF;
  auto consume = [&](const Tile& b, int tile) {
    float part[R];
#pragma unroll
    for (int r = 0; r < R; ++r) part[r] = 0.0f;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int c = lane + 64 * j;
      const bool ok = c < NC;
      const int cc = min(c, NC - 1);
      uint4 wj[R];
#pragma unroll
      for (int r = 0; r < R; ++r) wj[r] = b.w[r][j];
      float d[R];
      chunk_dot_rows<FMT, R>(wj, xl + cc * 4, xsum[cc], nf4, nmask, nmagic, nmask_hi, d);
#pragma unroll
      for (int r = 0; r < R; ++r) part[r] = fmaf(ok ? scale_of<FMT>(b.s[r][j]) : 0.0f, d[r], part[r]);
    }
    float tot;
    int vi;
    if constexpr (R == 1) {  // one row per tile: a plain wave sum, every lane holds it
      tot = wave_sum(part[0]);
      vi = 0;
    } else {
      tot = butterfly<R>(part, lane);
      vi = bfly_index<R>(lane);
    }
    constexpr int GROUP = 64 / R;
    const int row0 = tile * RT;
    if (DUAL) {
      constexpr int PD = R == 8 ? 8 : (R == 4 ? 16 : 32);
      const float other = PD == 8 ? LGA_DPP(tot, 0x128) : __shfl_xor(tot, PD);
      const int row = row0 + (vi >> 1);
      const float gs = round_bf(silu_f(round_bf(tot)));
      const uint16_t ob = f2bf(__fmul_rn(gs, round_bf(other)));
      if ((lane & (GROUP - 1)) == 0 && (vi & 1) == 0 && tile < T && row < a.N) a.y[row] = ob;
    } else {
      const int row = row0 + vi;
      float o = tot;
      if (RES) {
        o = round_bf(a.bias ? o + bf2f(a.bias[min(row, a.N - 1)]) : o) +
            __uint_as_float(((uint32_t)__shfl(b.res, vi)) << 16);
      } else if (a.bias) {
        o += bf2f(a.bias[min(row, a.N - 1)]);
      }
      const uint16_t ob = f2bf(o);
      if ((lane & (GROUP - 1)) == 0 && tile < T && row < a.N) {
        a.y[row] = ob;
        if (AMAX) amax_take(bf2f(ob), row, abv, abi);
      }
    }
  };
  for (int tile = gw; tile < T; tile += 2 * W) {  // wave-uniform trip count
    consume(A, tile);
    issue(A, tile + 2 * W);
    if (tile + W >= T) break;
    consume(B, tile + W);
    issue(B, tile + 3 * W);
  }
  if constexpr (AMAX) {
    // workgroup winner: the wave's lanes, then the 4 waves through LDS (the x staging is no longer read)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) amax_take(__shfl_xor(abv, off), __shfl_xor(abi, off), abv, abi);
    __shared__ float s_v[NW];
    __shared__ int s_i[NW];
    __shared__ unsigned s_last;
    if (lane == 0) {
      s_v[wave] = abv;
      s_i[wave] = abi;
    }
    __syncthreads();
    if (t == 0) {
      for (int w = 1; w < NW; ++w) amax_take(s_v[w], s_i[w], abv, abi);
      // publish (MI355X_MICROARCH.md "Valid forms" row 1: an sc1 store, drained, then the agent-scope adds), then
      // arrive on this workgroup's class counter; the last of a class arrives on the top counter
      __hip_atomic_store(am.cand + blockIdx.x, ((unsigned long long)(unsigned)abi << 32) | __float_as_uint(abv),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned cls = blockIdx.x & 7, classes = min(gridDim.x, 8u);
      const unsigned in_cls = (gridDim.x - cls + 7) / 8;
      unsigned last = 0;
      unsigned* cc = am.cnt + cls * 64;
      if (__hip_atomic_fetch_add(cc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_cls - 1) {
        __hip_atomic_store(cc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm: the class is complete
        unsigned* top = am.cnt + 8 * 64;
        last = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == classes - 1;
        if (last) __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    // the last workgroup: every winner is published (each arrival followed its own drained sc1 store; the counter
    // chain carries them here); reduce them with sc1 loads
    float bv = -INFINITY;
    int bi = 0x7FFFFFFF;
    for (int i = t; i < (int)gridDim.x; i += NT) {
      const unsigned long long c = __hip_atomic_load(am.cand + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      amax_take(__uint_as_float((unsigned)c), (int)(c >> 32), bv, bi);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) amax_take(__shfl_xor(bv, off), __shfl_xor(bi, off), bv, bi);
    __shared__ int s_tok;
    if (lane == 0) {
      s_v[wave] = bv;
      s_i[wave] = bi;
    }
    __syncthreads();
    if (t == 0) {
      for (int w = 1; w < NW; ++w) amax_take(s_v[w], s_i[w], bv, bi);
      if (bi >= a.N) bi = 0;
      if (am.out_idx) *am.out_idx = bi;
      if (am.token_out) *am.token_out = bi;
      if (am.pos_inout) *am.pos_inout = am_p0 + 1;
      s_tok = bi;
    }
    if (am.table) {
      __syncthreads();
      const long id = min(max(s_tok, 0), am.V - 1);  // as lga_embedding: the gather stays in bounds
      const uint4* src = (const uint4*)(am.table + (size_t)id * am.C);
      for (int i = t; i < am.C / 8; i += NT) ((uint4*)am.emb_out)[i] = src[i];
    }
  }
}

}  // namespace lga
