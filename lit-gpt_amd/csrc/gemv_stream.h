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

template <int RT, int CPT, int FMT, bool DUAL, bool NORM, bool RES>
__device__ __forceinline__ void gemv_q4_stream(GemvArgs a, unsigned char* smem) {
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
      if ((lane & (GROUP - 1)) == 0 && tile < T && row < a.N) a.y[row] = f2bf(o);
    }
  };
  for (int tile = gw; tile < T; tile += 2 * W) {  // wave-uniform trip count
    consume(A, tile);
    issue(A, tile + 2 * W);
    if (tile + W >= T) break;
    consume(B, tile + W);
    issue(B, tile + 3 * W);
  }
}

}  // namespace lga
