// Persistent decode engine: one launch per greedy decode step (all blocks + ln_f + lm_head + argmax).
//
// Replaces, for one token of generate/base.py's decode loop (next_token -> GPT.forward -> Block.forward x L ->
// ln_f -> lm_head -> sample(T=0), reference generate/base.py:44-47,87-92; lit_gpt/model.py:499-519,572-593,609-656,
// 712-716; lit_gpt/rmsnorm.py:19-25) the chain of 160 launches of the per-op kernels (gemv.hip, attention.hip,
// sample.hip). Why: a batch-1 decode step is a pure HBM stream (weights + K/V, ~4.5 GB per Llama-2-7B token) cut by
// data dependencies into ~5 ops per block; as separate launches every op pays a dispatch gap, a load ramp and a
// tail (~3-4 us of ~8 us), and the memory pipe idles across every boundary. Here the weight / K/V stream never
// depends on activations, so it runs ahead of the compute across op boundaries.
//
// Structure (MI355X_MICROARCH.md "engine-vs-launches", "prefetch-credit", "ldsdma-fill", "gather-pass"):
//  * one 512-thread workgroup per CU (the LDS footprint admits one): wave 0 is the LOADER, waves 1..7 CONSUMERS;
//  * the loader walks this CU's share of every op of the step in order and streams it with LDS-DMA
//    (global_load_lds_dwordx4 nt, 1 KB per wave instruction = one ring LINE) into an LDS ring of NL lines, keeping
//    DEPTH lines in flight, publishing `landed` (lines landed so far) and reclaiming lines behind the slowest
//    consumer; while a consumer gathers an activation vector the loader thins to THIN lines in flight so the
//    gather's loads are not queued behind the stream;
//  * consumer wave 0 is also the GATHERER: at each op boundary it polls the producing op's arrival counters,
//    loads the activation vector (write-through `sc1` loads), applies the fused RMSNorm, stages x into LDS in the
//    GEMV's fp16-pair layout and releases the op to the other consumers;
//  * consumers take the op's UNITS round-robin (a unit = R rows x CPT lines of packed nibbles, or 16 K/V rows),
//    compute exactly as the per-op kernels do (chunk_dot_rows, butterfly<R>, the same epilogues: bit-identical
//    GEMV outputs), store outputs write-through (sc1), drain, and the last wave of the CU bumps the op's counter;
//  * hand-offs follow MI355X_MICROARCH.md "Valid forms" row 1 (sc1 4/8-B stores -> vmcnt(0) -> per-CU LDS count
//    -> one agent-scope atomic add per CU; sc1 poll -> sc1 loads); counters are sharded 8 ways (fan-in) and
//    monotonic across launches: a per-scratch epoch advanced by the launch's last arriver gives each launch its
//    targets, so nothing is re-armed and the launch is graph-capturable;
//  * attention: CU c owns query group c % G and key split c / G (a group's splits share an XCD under round-robin
//    dispatch); the split owning the new position ropes + appends k, v and scores that key from registers; every
//    split publishes (m, l, o) and the last-arriving split of a group merges them (flash-decoding) into y;
//  * lm_head: every CU keeps the argmax of its rows; the last CU merges the candidates (torch.argmax order: NaN
//    first, lowest index on ties), writes the token, advances input_pos and gathers the token's embedding row as
//    the next launch's input.
// Every wait is bounded (TIMEOUT_TICKS of the 100 MHz clock, then the launch sets `err` / `abort` and drains).
#include <string.h>

#include "decode_ops.h"
#include "engine.h"

namespace lga {
namespace eng {

constexpr int LINE = 1024;           // bytes per ring line (one LDS-DMA wave instruction)
constexpr int CSTRIDE = 16;          // uint32 words between counter slots (64 B)
constexpr int NSH = 8;               // counter shards (fan-in relief, MI355X_MICROARCH.md "fanin")
constexpr int OPS_PER_LAYER = 5;     // QKV, ATTN, OPROJ, FC, DOWN
constexpr int NLW = 4;               // loader waves: one LDS-DMA wave issues at most ~11 GB/s (tools/lab/dma_lab.hip:
                                     // 2.8 TB/s chip-wide at any depth; 2 waves 5.8, 4 waves 7.2 TB/s)
constexpr int DU = 1;                // units each loader keeps in flight besides the one being issued (1-2 units =
                                     // 8-24 KB per loader, ~32-48 KB per CU: dma_lab's depth for 7.2 TB/s, and a
                                     // short queue ahead of the gathers' loads)
#ifndef LGA_ENGINE_NCW
#define LGA_ENGINE_NCW 8
#endif
constexpr int NCW = LGA_ENGINE_NCW;  // consumer waves (2-3 per SIMD: a lone wave is latency-bound on its LDS reads and
                                     // reduction chains; 8 -> 768-thread workgroups, <= 168 VGPRs)
constexpr int NTHREADS = (NLW + NCW) * 64;
constexpr int SCALE_BYTES = 8192;    // LDS for the scales of one op's rows of this CU (x 2: op parity)
constexpr int RES_ROWS = 256;        // LDS for the residual rows of one op of this CU
constexpr int ATT_KEYS = 16;         // keys per attention unit (4 K lines + 4 V lines)
constexpr unsigned long long TIMEOUT_TICKS = 2000000ull;  // 20 ms at 100 MHz

#ifdef LGA_ENGINE_TRACE  // lab builds only (tools/engine_trace.py): per-(CU, op) event times, 100 MHz clock
constexpr int TR_OPS = 192, TR_EV = 8;
__device__ unsigned long long g_eng_trace[256 * TR_OPS * TR_EV];
#define ETRACE(k, ev)                                                                                      \
  do {                                                                                                   \
    if ((threadIdx.x & 63) == 0 && (k) < TR_OPS)                                                         \
      g_eng_trace[((size_t)blockIdx.x * TR_OPS + (k)) * TR_EV + (ev)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define ETRACE(k, ev) \
  do {                \
  } while (0)
#endif

enum Kind { K_QKV = 0, K_ATTN = 1, K_O = 2, K_FC = 3, K_DN = 4, K_LM = 5 };

struct Geo {
  int L, C, H, G, hs, I, V, S, grp, rope_rows, P, NL;
  float eps, scale;
  int QN, SP, gC, gI, QPK;
  int ncC, ncI;            // 32-element chunks per row for K = C / K = I
  int n_slots;
  size_t o_x0, o_x, o_qkv, o_y, o_xp, o_g, o_ws, o_cand, total;
  int lds_ring, lds_total;  // dynamic LDS: ring bytes, total bytes
};

__host__ __device__ inline size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }
__host__ __device__ inline int layer_slots(int G) { return G; }  // one split counter per KV group

__host__ inline bool make_geo(const lga_engine_geom& g, Geo& o, int cpt_c, int cpt_i) {
  o.L = g.n_layer;
  o.C = g.n_embd;
  o.H = g.n_head;
  o.G = g.n_query_groups;
  o.hs = g.head_size;
  o.I = g.intermediate;
  o.V = g.vocab;
  o.S = g.max_seq;
  o.grp = g.group;
  o.rope_rows = g.rope_rows;
  o.P = g.n_cu;
  o.eps = g.norm_eps;
  o.scale = g.attn_scale;
  if (o.G <= 0 || o.H % o.G || o.P <= 0) return false;
  o.QPK = o.H / o.G;
  o.QN = (o.H + 2 * o.G) * o.hs;
  o.SP = o.P / o.G;
  o.gC = o.C / o.grp;
  o.gI = o.I / o.grp;
  o.ncC = o.C / 32;
  o.ncI = o.I / 32;
  o.n_slots = 3 + o.L * layer_slots(o.G) + NSH + 1;
  size_t off = al256((size_t)o.n_slots * CSTRIDE * 4);
  // activations between CUs travel as 8-byte granules {2 bf16, tag = launch epoch + 1} (written by one sc1 store:
  // the data is its own flag); the step's input embedding x0 is plain bf16 (written before the launch)
  o.o_x0 = off;
  off += al256((size_t)o.C * 2);
  o.o_x = off;  // x[1..L]
  off += al256((size_t)o.L * (o.C / 2) * 8);
  o.o_qkv = off;
  off += al256((size_t)o.L * (o.QN / 2) * 8);
  o.o_y = off;
  off += al256((size_t)o.L * (o.C / 2) * 8);
  o.o_xp = off;
  off += al256((size_t)o.L * (o.C / 2) * 8);
  o.o_g = off;
  off += al256((size_t)o.L * (o.I / 2) * 8);
  o.o_ws = off;
  off += al256((size_t)o.L * o.H * o.SP * (o.hs + 4) * 4);
  o.o_cand = off;
  off += al256((size_t)o.P * 8);
  o.total = off;
  // dynamic LDS: control words, residual rows, attention staging + merge, scales, x staging, ring
  const int kmax = o.C > o.I ? o.C : o.I;
  const int fixed = 1024 /*ctrl*/ + RES_ROWS * 2 + (o.QPK + 2) * o.hs * 2 + NCW * o.QPK * (o.hs + 4) * 4 +
                    2 * SCALE_BYTES + kmax * 2 + (kmax / 32) * 4 + 64 * 4;
  const int fixed16 = (fixed + 1023) & ~1023;
  o.NL = (163840 - fixed16) / LINE;
  o.lds_ring = o.NL * LINE;
  o.lds_total = o.lds_ring + fixed16;
  (void)cpt_c;
  (void)cpt_i;
  return true;
}

// shard s of a counter fed by `n` producers numbered 0..n-1 (producer i adds to shard i % NSH)
__host__ __device__ inline int shard_count(int n, int s) { return n > s ? (n - s + NSH - 1) / NSH : 0; }

struct Args {
  Geo g;
  const lga_engine_layer* layers;
  const uint8_t* lm_w;
  const void* lm_s;
  const uint16_t* ln_f;
  const uint16_t* wte;
  const float* cos;
  const float* sin;
  int64_t* pos;
  int32_t* token;
  int64_t* out_idx;
  uint16_t* logits;
  unsigned char* scratch;
  int op_limit;
};

// ---- small device helpers ---------------------------------------------------------------------------------
__device__ __forceinline__ unsigned lds_ld(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ unsigned g_ld(const unsigned* p) {  // sc1 (L2-served) poll / payload load
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t g_ld8(const void* p) {
  return __hip_atomic_load((const uint64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_st4(void* p, uint32_t v) {
  __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_st8(void* p, uint64_t v) {
  __hip_atomic_store((uint64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned g_add(unsigned* p, unsigned v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// s_waitcnt vmcnt(n) for a run-time n in [0, 63] (the immediate is an encoding field)
__device__ __forceinline__ void vmcnt_dyn(unsigned n) {
  switch (min(n, 63u)) {
#define LGA_VMC(i) \
  case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
    LGA_VMC(0) LGA_VMC(1) LGA_VMC(2) LGA_VMC(3) LGA_VMC(4) LGA_VMC(5) LGA_VMC(6) LGA_VMC(7) LGA_VMC(8) LGA_VMC(9)
    LGA_VMC(10) LGA_VMC(11) LGA_VMC(12) LGA_VMC(13) LGA_VMC(14) LGA_VMC(15) LGA_VMC(16) LGA_VMC(17) LGA_VMC(18)
    LGA_VMC(19) LGA_VMC(20) LGA_VMC(21) LGA_VMC(22) LGA_VMC(23) LGA_VMC(24) LGA_VMC(25) LGA_VMC(26) LGA_VMC(27)
    LGA_VMC(28) LGA_VMC(29) LGA_VMC(30) LGA_VMC(31) LGA_VMC(32) LGA_VMC(33) LGA_VMC(34) LGA_VMC(35) LGA_VMC(36)
    LGA_VMC(37) LGA_VMC(38) LGA_VMC(39) LGA_VMC(40) LGA_VMC(41) LGA_VMC(42) LGA_VMC(43) LGA_VMC(44) LGA_VMC(45)
    LGA_VMC(46) LGA_VMC(47) LGA_VMC(48) LGA_VMC(49) LGA_VMC(50) LGA_VMC(51) LGA_VMC(52) LGA_VMC(53) LGA_VMC(54)
    LGA_VMC(55) LGA_VMC(56) LGA_VMC(57) LGA_VMC(58) LGA_VMC(59) LGA_VMC(60) LGA_VMC(61) LGA_VMC(62)
    default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
#undef LGA_VMC
  }
}

// one LDS-DMA line: lane l's 16 B from `src` land at lds_dst + 16 l (non-temporal: read once per step)
__device__ __forceinline__ void glds_line(const void* src, unsigned lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds_dst)
      : "memory");
}

// LDS control words
struct Ctl {
  unsigned* w;  // [1] x_ready (op + 1), [2] gathering, [3] done_local, [4] abort, [5] split-last flag,
                // [6] trace op, [7] RMSNorm partials, [8 + cw] consumer position, [24 + lw] lines landed by loader
                // lw, [32 + 2 cw] argmax candidates, [60] gather waves finished, [61] GEMV ops finished (x waves)
  __device__ unsigned* landed(int lw) const { return w + 24 + lw; }
  __device__ unsigned* xready() const { return w + 1; }
  __device__ unsigned* gathering() const { return w + 2; }
  __device__ unsigned* done() const { return w + 3; }
  __device__ unsigned* abort() const { return w + 4; }
  __device__ unsigned* posw(int cw) const { return w + 8 + cw; }
  __device__ unsigned* cand(int cw) const { return w + 32 + 2 * cw; }
};

struct Clock {
  unsigned long long t0;
  __device__ bool expired() const { return __builtin_amdgcn_s_memrealtime() - t0 > TIMEOUT_TICKS; }
};

__device__ __forceinline__ unsigned* counters(const Args& a) { return (unsigned*)a.scratch; }
__device__ __forceinline__ unsigned* slot(const Args& a, int s) { return counters(a) + (size_t)s * CSTRIDE; }
__device__ __forceinline__ int split_slot(const Geo& g, int l, int grp) { return 3 + l * layer_slots(g.G) + grp; }
__device__ __forceinline__ int arg_slot(const Geo& g, int s) { return 3 + g.L * layer_slots(g.G) + s; }

// set the error / abort words (global) and the local abort flag
__device__ void fail(const Args& a, const Ctl& ctl, unsigned code) {
  __hip_atomic_fetch_or(slot(a, 1), code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(slot(a, 2), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  lds_st(ctl.abort(), 1u);
}

// op bookkeeping shared by loader and consumers -----------------------------------------------------------
struct OpInfo {
  int kind, l;
  int n_units;      // units of this CU
  int lines;        // ring lines per unit
  int u0;           // first global unit (GEMV) of this CU
};

template <int CPT_C, int CPT_I>
__device__ inline int op_lines(int kind) {
  switch (kind) {
    case K_QKV: return 4 * CPT_C;   // 4 rows
    case K_O: return 4 * CPT_C;     // 4 rows
    case K_FC: return 4 * CPT_C;    // 2 rows x (fc_1, fc_2)
    case K_DN: return 2 * CPT_I;    // 2 rows
    case K_LM: return 2 * CPT_C;    // 2 rows
    default: return 8;              // attention: 4 K + 4 V lines (16 keys)
  }
}

// LDS scale buffer of a GEMV op. An op prefetches its scales before its input is complete, so the buffer must not
// be one a unit of this CU may still read: the GEMV before it (across the attention for o_proj) reads the other one,
// and the one before that has finished, since this op's gather follows a gather that needed its whole output.
__device__ inline int scale_buf(int kind) { return (kind == K_O || kind == K_DN) ? 1 : 0; }

__device__ inline int op_rows_per_unit(int kind) {
  return (kind == K_QKV || kind == K_O) ? 4 : 2;
}
__device__ inline int op_N(const Geo& g, int kind) {
  switch (kind) {
    case K_QKV: return g.QN;
    case K_O: return g.C;
    case K_FC: return g.I;
    case K_DN: return g.C;
    default: return g.V;  // K_LM
  }
}

struct AttnSplit {
  int grp, split, k_lo, k_hi, k_end, nkeys;
  bool owns_new;
  long p;
};
__device__ inline AttnSplit attn_split(const Geo& g, int c, long p) {
  AttnSplit s;
  s.p = p;
  s.grp = c % g.G;
  s.split = c / g.G;
  const int Lk = (int)min(p + 1, (long)g.S);
  const int chunk = (Lk + g.SP - 1) / g.SP;
  s.k_lo = min(s.split * chunk, Lk);
  s.k_hi = min(s.k_lo + chunk, Lk);
  s.owns_new = p < g.S && s.k_lo <= p && p < s.k_hi;
  s.k_end = s.owns_new ? (int)p : s.k_hi;  // the new key is scored from registers
  s.nkeys = max(0, s.k_end - s.k_lo);
  return s;
}

template <int CPT_C, int CPT_I>
__device__ inline OpInfo op_info(const Geo& g, int k, int c, long p) {
  OpInfo o;
  if (k >= g.L * OPS_PER_LAYER) {
    o.kind = K_LM;
    o.l = g.L;
  } else {
    o.l = k / OPS_PER_LAYER;
    o.kind = k % OPS_PER_LAYER;  // K_QKV .. K_DN in schedule order
  }
  o.lines = op_lines<CPT_C, CPT_I>(o.kind);
  if (o.kind == K_ATTN) {
    const AttnSplit s = attn_split(g, c, p);
    o.n_units = (s.nkeys + ATT_KEYS - 1) / ATT_KEYS;
    o.u0 = 0;
  } else {
    const int nu = op_N(g, o.kind) / op_rows_per_unit(o.kind);
    o.u0 = (int)(((long)c * nu) / g.P);
    o.n_units = (int)(((long)(c + 1) * nu) / g.P) - o.u0;
  }
  return o;
}

// ---- the loader wave ---------------------------------------------------------------------------------------
// Loader wave lw of NLW: issues the lines of every unit whose step-wide index is = lw (mod NLW), in schedule order,
// at most DU of its units in flight; `landed(lw)` = end line of its newest unit whose lines have all landed (so every
// line of that loader below it has landed). While the CU gathers, one unit in flight per loader.
template <int CPT_C, int CPT_I>
__device__ void run_loader(const Args& a, const Ctl& ctl, const Clock& clk, unsigned char* ring, int nops, long p,
                           int lw, bool interleave = false) {
  const Geo& g = a.g;
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x;
  const unsigned ring_base = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)ring);
  const unsigned NL = (unsigned)g.NL;
  unsigned limit = NL;          // lines below limit may be written (consumers' positions + NL)
  unsigned issued = 0;          // this loader's lines issued
  unsigned hist_e[DU + 1], hist_c[DU + 1];  // end line / issued count after each in-flight unit, oldest first
  int nh = 0;
  unsigned line = 0;            // step-wide ring line of the current unit's first line
  unsigned unit_seq = 0;        // step-wide unit index
  bool dead = false;
  auto publish = [&](unsigned e) { __hip_atomic_store(ctl.landed(lw), e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
  auto retire_oldest = [&]() {  // wait for the oldest in-flight unit, publish it
    vmcnt_dyn(issued - hist_c[0]);
    publish(hist_e[0]);
#pragma unroll
    for (int i = 0; i + 1 < DU + 1; ++i) {
      hist_e[i] = hist_e[i + 1];
      hist_c[i] = hist_c[i + 1];
    }
    --nh;
  };
  // may lines [.., e) be written? While waiting (ring full, or the CU gathering: no new issue), keep retiring the
  // in-flight units one by one so the consumers see each as soon as it lands
  auto room = [&](unsigned e) {
    for (unsigned it = 0;; ++it) {
      const bool gathering = __hip_atomic_load(ctl.gathering(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
      if (!gathering && e <= limit) return true;
      if (nh > 0) {
        retire_oldest();
      } else {
        unsigned b = 0xFFFFFFFFu;
#pragma unroll
        for (int w = 0; w < NCW; ++w)
          b = min(b, __hip_atomic_load(ctl.posw(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        limit = b + NL;
        if (!gathering && e <= limit) return true;
        if ((it & 15u) == 15u) {
          if (lds_ld(ctl.abort())) return false;
          if (clk.expired()) {
            if (lane == 0) fail(a, ctl, 4u);
            return false;
          }
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  };
  auto issue = [&](const void* src, unsigned ln) {
    unsigned off = ln % NL;
    glds_line(src, __builtin_amdgcn_readfirstlane(ring_base + off * LINE));
  };
  // after a unit's lines: record it; more than DU in flight -> retire the oldest
  auto unit_done = [&](unsigned e) {
#pragma unroll
    for (int i = 0; i < DU + 1; ++i)
      if (i == nh) {
        hist_e[i] = e;
        hist_c[i] = issued;
      }
    ++nh;
    if (nh > DU) retire_oldest();
  };
  auto drain_all = [&]() {
    while (nh > 0) retire_oldest();
  };
  const AttnSplit as = attn_split(g, c, p);
  for (int k = 0; k < nops && !dead; ++k) {
    const OpInfo o = op_info<CPT_C, CPT_I>(g, k, c, p);
    if (lw == 0) ETRACE(k, 5);
    // first own unit of this op
    const int u_first = (int)((lw - (int)(unit_seq % NLW) + NLW) % NLW);
    if (o.kind == K_ATTN) {
      const lga_engine_layer* L = a.layers + o.l;
      const unsigned char* kb = (const unsigned char*)L->k_cache + ((size_t)as.grp * g.S) * (g.hs * 2) + (lane & 15) * 16;
      const unsigned char* vb = (const unsigned char*)L->v_cache + ((size_t)as.grp * g.S) * (g.hs * 2) + (lane & 15) * 16;
      const int last = max(as.k_end - 1, 0);
      for (int u = u_first; u < o.n_units; u += NLW) {
        const unsigned l0 = line + (unsigned)(u * o.lines);
        if (!room(l0 + (unsigned)o.lines)) { dead = true; break; }
        const int key0 = as.k_lo + u * ATT_KEYS + (lane >> 4);
#pragma unroll
        for (int jl = 0; jl < 4; ++jl) issue(kb + (size_t)min(key0 + 4 * jl, last) * 256, l0 + jl);
#pragma unroll
        for (int jl = 0; jl < 4; ++jl) issue(vb + (size_t)min(key0 + 4 * jl, last) * 256, l0 + 4 + jl);
        issued += 8;
        unit_done(l0 + 8);
      }
    } else {
      const int rpu = op_rows_per_unit(o.kind);
      const bool dn = o.kind == K_DN;
      const int nc = dn ? g.ncI : g.ncC;
      const size_t rowb = (size_t)(dn ? g.I : g.C) / 2;
      const unsigned char* w1;
      const unsigned char* w2 = nullptr;
      if (o.kind == K_LM) {
        w1 = a.lm_w;
      } else {
        const lga_engine_layer* L = a.layers + o.l;
        w1 = (const unsigned char*)(o.kind == K_QKV ? L->qkv_w : o.kind == K_O ? L->o_w : o.kind == K_FC ? L->fc1_w
                                                                                                   : L->dn_w);
        if (o.kind == K_FC) w2 = (const unsigned char*)L->fc2_w;
      }
      constexpr int CM = CPT_I > CPT_C ? CPT_I : CPT_C;
      int coff[CM];  // this lane's byte offset inside line jj of a row (clamped duplicates past the last chunk)
#pragma unroll
      for (int jj = 0; jj < CM; ++jj) coff[jj] = min(64 * jj + lane, nc - 1) * 16;
      for (int u = u_first; u < o.n_units; u += NLW) {
        const unsigned l0 = line + (unsigned)(u * o.lines);
        if (!room(l0 + (unsigned)o.lines)) { dead = true; break; }
        const int gu = interleave ? min(u * g.P + c, op_N(g, o.kind) / rpu - 1) : o.u0 + u;
        const unsigned char* rp = w1 + (size_t)gu * rpu * rowb;
        const unsigned char* rp2 = w2 ? w2 + (size_t)gu * rpu * rowb : nullptr;
        unsigned ln = l0;
        for (int r = 0; r < rpu; ++r) {
          if (dn) {
#pragma unroll
            for (int jj = 0; jj < CPT_I; ++jj) issue(rp + coff[jj], ln++);
          } else {
#pragma unroll
            for (int jj = 0; jj < CPT_C; ++jj) issue(rp + coff[jj], ln++);
            if (w2) {
#pragma unroll
              for (int jj = 0; jj < CPT_C; ++jj) issue(rp2 + coff[jj], ln++);
              rp2 += rowb;
            }
          }
          rp += rowb;
        }
        issued += (unsigned)o.lines;
        unit_done(l0 + (unsigned)o.lines);
      }
    }
    line += (unsigned)(o.n_units * o.lines);
    unit_seq += (unsigned)o.n_units;
    if (lw == 0) ETRACE(k, 6);
    if (lds_ld(ctl.abort())) dead = true;
  }
  if (!dead) drain_all();
}

// ---- consumer side ---------------------------------------------------------------------------------------
struct Lds {
  unsigned char* ring;
  uint16_t* res;     // residual rows of this CU's op
  uint16_t* qst;     // roped q heads, k_new, v_new (bf16)
  float* amrg;       // per consumer wave: QPK x (m, l, -, -, o[hs])
  unsigned char* scl;
  uint4* xl;         // x staging (fp16 / bf16 pairs)
  float* xsum;       // per-chunk corrections
  float* red;        // 16 floats
  float* nf4;        // 16 floats
};

// GEMV x staging (gemv_q4_body steps 1 + 3, bit-identical; gather_gemv below): one wave plays the four waves of
// the per-op kernel (virtual thread t = vw * 64 + lane handles uint4 t, t + 256, ...), so the RMSNorm partial sums,
// their tree and the chunk corrections are computed in the same order.

// one GEMV unit: NB butterfly groups of R values (rows, or row x matrix when DUAL), CPT ring lines each, streamed
// through registers chunk by chunk (the per-op kernels hold a wave's whole row in registers to hide HBM latency; here
// the lines are in LDS). Per value the partial sums accumulate over the chunks in the same order, so the results are
// the per-op kernels' bits.
template <int FMT, int R, int CPT, int NB, bool DUAL, bool RES, bool LMH>
__device__ void gemv_unit(const Args& a, const Lds& s, const unsigned char* scl, unsigned line0, int n0,
                          int local_row0, int nc, int groups, int rows_cu, int gshift, uint16_t* out,
                          unsigned tag, float& best_v, int& best_i) {
  const int lane = threadIdx.x & 63;
  const uint32_t nmask = nibble_mask(), nmagic = f16_magic(), nmask_hi = nibble_mask_hi();
  constexpr int SB = FMT == 0 ? 2 : 4;
  const unsigned NL = (unsigned)a.g.NL;
  const unsigned lb = line0 % NL;
  uint32_t outw[NB * (DUAL ? 1 : R)];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    float part[R];
#pragma unroll
    for (int r = 0; r < R; ++r) part[r] = 0.0f;
#pragma unroll CPT <= 2 ? CPT : 1
    for (int j = 0; j < CPT; ++j) {
      uint4 wj[R];
      uint32_t sv[R];
      const int gidx = (min(lane + 64 * j, nc - 1) * 32) >> gshift;  // the chunk's quant group (group = 2^gshift)
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int v = b * R + r;
        unsigned ln = lb + (unsigned)(v * CPT + j);
        ln = ln >= NL ? ln - NL : ln;
        wj[r] = *(const uint4*)(s.ring + (size_t)ln * LINE + lane * 16);
        const int lrow = DUAL ? (local_row0 + (v >> 1)) : (local_row0 + v);
        const int mat = DUAL ? (v & 1) : 0;
        const int si = (mat * rows_cu + lrow) * groups + gidx;
        sv[r] = SB == 2 ? (uint32_t)((const uint16_t*)scl)[si] : ((const uint32_t*)scl)[si];
      }
      const int cc = lane + 64 * j;
      const bool ok = cc < nc;
      const int c2 = min(cc, nc - 1);
      float d[R];
      chunk_dot_rows<FMT, R>(wj, s.xl + c2 * 4, s.xsum[c2], s.nf4, nmask, nmagic, nmask_hi, d);
#pragma unroll
      for (int r = 0; r < R; ++r) part[r] = fmaf(ok ? scale_of<FMT>(sv[r]) : 0.0f, d[r], part[r]);
      // keep the scheduler from hoisting every chunk's LDS reads to the top (register budget of 3 consumer waves
      // per SIMD); the co-resident waves hide the LDS latency instead
      __builtin_amdgcn_sched_barrier(0);
    }
    const float tot = butterfly<R>(part, lane);
    constexpr int GROUP = 64 / R;
    if (DUAL) {
      constexpr int PD = R == 8 ? 8 : (R == 4 ? 16 : 32);
      const float other = PD == 8 ? LGA_DPP(tot, 0x128) : __shfl_xor(tot, PD);
      const float gs = round_bf(silu_f(round_bf(tot)));
      outw[b] = f2bf(__fmul_rn(gs, round_bf(other)));  // value 0 (row b, fc_1) sits in lane 0
    } else {
      const int vi = bfly_index<R>(lane);
      float o = tot;
      if (RES) o = round_bf(o) + bf2f(s.res[local_row0 + vi]);
      const uint16_t ob = f2bf(o);
      // values vi = 0..R-1 sit in lanes vi * GROUP: collect them in lane 0
#pragma unroll
      for (int r = 0; r < R; ++r) outw[b * R + r] = (uint32_t)__shfl((int)ob, r * GROUP);
    }
  }
  if (lane == 0) {
    constexpr int NO = NB * (DUAL ? 1 : R);
    if (LMH) {
      if (NO == 2) *(uint32_t*)(out + n0) = outw[0] | (outw[1] << 16);
      else *(uint64_t*)(out + n0) = (uint64_t)(outw[0] | (outw[1] << 16)) | ((uint64_t)(outw[2] | (outw[3] << 16)) << 32);
    } else {  // granules {2 bf16, tag}: out is the granule buffer, n0 even
      uint64_t* gr = (uint64_t*)out + n0 / 2;
      g_st8(gr, (uint64_t)(outw[0] | (outw[1] << 16)) | ((uint64_t)tag << 32));
      if (NO == 4) g_st8(gr + 1, (uint64_t)(outw[2] | (outw[3] << 16)) | ((uint64_t)tag << 32));
    }
    if (LMH) {
#pragma unroll
      for (int r = 0; r < NO; ++r) {
        const float v = bf2f((uint16_t)outw[r]);
        const int idx = n0 + r;
        const bool vn = v != v, bn = best_v != best_v;
        const bool t = (vn || bn) ? (vn && (!bn || idx < best_i)) : ((v > best_v) || (v == best_v && idx < best_i));
        best_v = t ? v : best_v;
        best_i = t ? idx : best_i;
      }
    }
  }
}

__device__ __forceinline__ bool better(float v, int i, float bv, int bi) {
  const bool vn = v != v, bn = bv != bv;
  if (vn || bn) return vn && (!bn || i < bi);
  return (v > bv) || (v == bv && i < bi);
}


// ---- gathers: the op's input vector (+ scales, residual rows) into LDS -------------------------------------
// The producers' granules are their own flags: a gather wave loads its slice of granules (write-through `sc1`
// loads) and re-loads the ones whose tag is not yet this launch's until all are (MI355X_MICROARCH.md "Valid forms":
// 8-byte granule, one sc1 store, no ordering). Consumer waves 0-3 gather together, wave w playing virtual wave w of
// the per-op GEMV kernel (uint4 t, t + 256, ... of x with t = 64 w + lane), so the RMSNorm partial sums and their
// tree are the per-op kernel's: the four partials meet in LDS. Scales and residual rows do not depend on the
// producers and are loaded first.
constexpr int NGW = 4;  // gather waves

// spin until every granule of `gp[idx]` (NG per lane) carries `tag`; returns the data words
template <int NG>
__device__ bool poll_granules(const Args& a, const Ctl& ctl, const Clock& clk, const uint64_t* gp, const int (&idx)[NG],
                              unsigned tag, uint32_t (&data)[NG]) {
  bool got[NG];
#pragma unroll
  for (int i = 0; i < NG; ++i) got[i] = false;
  for (unsigned it = 0;; ++it) {
    bool all = true;
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      if (!got[i]) {
        const uint64_t v = g_ld8(gp + idx[i]);
        data[i] = (uint32_t)v;
        got[i] = (uint32_t)(v >> 32) == tag;
      }
      all = all && got[i];
    }
    if (__all(all)) return true;
    if ((it & 15u) == 15u) {
      if (g_ld(slot(a, 2)) || lds_ld(ctl.abort())) {
        lds_st(ctl.abort(), 1u);
        return false;
      }
      if (clk.expired()) {
        if ((threadIdx.x & 63) == 0) fail(a, ctl, 2u);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// one gather wave's part of a GEMV op's staging. x: granules (or plain bf16 when x_plain, the step input x0).
// The wave that completes the staging raises x_ready.
template <int FMT, int CPT, bool NORM, bool RES, bool DUAL>
__device__ __attribute__((noinline)) bool gather_gemv(const Args& a, const Ctl& ctl, const Clock& clk, const Lds& s,
                                                      int cw, int k, unsigned ng, unsigned ngemv, unsigned tag,
                                                      unsigned char* scl,
                                                      const void* sc, const void* sc2, int n0, int rows, int groups,
                                                      const void* x, bool x_plain, const uint16_t* normw,
                                                      const void* res, bool res_plain, int K) {
  constexpr int SB = FMT == 0 ? 2 : 4;
  constexpr int NSC = 4;  // 8-B scale loads per lane per gather wave: 4 waves x 64 lanes x 4 x 8 B = 8 KB
  const int lane = threadIdx.x & 63;
  const int w8 = rows * groups * SB / 8;  // per matrix (rows even, groups even)
  const int tot8 = DUAL ? 2 * w8 : w8;
  {
    uint2 scv[NSC];
#pragma unroll
    for (int i = 0; i < NSC; ++i) {
      const int idx = min(cw * 64 + lane + 256 * i, tot8 - 1);
      const bool second = DUAL && idx >= w8;
      const unsigned char* base = (const unsigned char*)(second ? sc2 : sc) + (size_t)n0 * groups * SB;
      scv[i] = *(const uint2*)(base + (size_t)(second ? idx - w8 : idx) * 8);
    }
#pragma unroll
    for (int i = 0; i < NSC; ++i)
      if (cw * 64 + lane + 256 * i < tot8) ((uint2*)scl)[cw * 64 + lane + 256 * i] = scv[i];
    if (RES && cw == 0) {  // residual rows [n0, n0 + rows): complete since an earlier edge
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int j = min(lane + 64 * i, rows / 2 - 1);
        const uint32_t v = res_plain ? g_ld((const unsigned*)((const uint16_t*)res + n0) + j)
                                     : (uint32_t)g_ld8((const uint64_t*)res + n0 / 2 + j);
        if (lane + 64 * i < rows / 2) ((uint32_t*)s.res)[lane + 64 * i] = v;
      }
    }
  }
  constexpr int XI = (CPT * 4 + 3) / 4;
  const int n8 = K / 8;
  uint4 xr[XI];
  if (x_plain) {
#pragma unroll
    for (int i = 0; i < XI; ++i) xr[i] = *((const uint4*)x + min(cw * 64 + lane + 256 * i, n8 - 1));
  } else {
    int idx[4 * XI];
    uint32_t d[4 * XI];
#pragma unroll
    for (int i = 0; i < XI; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) idx[4 * i + q] = 4 * min(cw * 64 + lane + 256 * i, n8 - 1) + q;
    if (!poll_granules<4 * XI>(a, ctl, clk, (const uint64_t*)x, idx, tag, d)) return false;
#pragma unroll
    for (int i = 0; i < XI; ++i) xr[i] = make_uint4(d[4 * i], d[4 * i + 1], d[4 * i + 2], d[4 * i + 3]);
  }
#ifdef LGA_ENGINE_TRACE
  if (cw == 0 && lane == 0) g_eng_trace[((size_t)blockIdx.x * TR_OPS + (unsigned)k) * TR_EV + 1] = __builtin_amdgcn_s_memrealtime();
#endif
  // this wave's slice being complete says nothing of this CU's own units of the previous GEMV, which read the whole
  // staged vector: wait until every consumer wave has finished them before overwriting it
  while (lds_ld(ctl.w + 61) < NCW * ngemv) {
    if (lds_ld(ctl.abort()) || clk.expired()) return false;
    __builtin_amdgcn_s_sleep(0);
  }
  float rs = 1.0f;
  if (NORM) {
    uint4 nr[XI];
#pragma unroll
    for (int i = 0; i < XI; ++i) nr[i] = ((const uint4*)normw)[min(cw * 64 + lane + 256 * i, n8 - 1)];
    float ss = 0.0f;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const bool ok = cw * 64 + lane + 256 * i < n8;
      const uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float lo = ok ? bflo(d[q]) : 0.0f, hi = ok ? bfhi(d[q]) : 0.0f;
        ss = fmaf(lo, lo, ss);
        ss = fmaf(hi, hi, ss);
      }
    }
    ss = wave_sum_uniform(ss);
    if (lane == 0) {
      s.red[(ng & 1) * 4 + cw] = ss;
      __hip_atomic_fetch_add(ctl.w + 7, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    while (lds_ld(ctl.w + 7) < NGW * ng) {  // the four partials (ng: this op's ordinal among the norm gathers)
      if (lds_ld(ctl.abort()) || clk.expired()) return false;
      __builtin_amdgcn_s_sleep(0);
    }
    const float* r = s.red + (ng & 1) * 4;
    rs = 1.0f / sqrtf(((r[0] + r[1]) + (r[2] + r[3])) / (float)K + a.g.eps);
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
      const uint32_t nw[4] = {nr[i].x, nr[i].y, nr[i].z, nr[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        d[q] = pack2(__fmul_rn(bflo(nw[q]), __fmul_rn(bflo(d[q]), rs)),
                     __fmul_rn(bfhi(nw[q]), __fmul_rn(bfhi(d[q]), rs)));
      xr[i] = make_uint4(d[0], d[1], d[2], d[3]);
    }
  }
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int u = cw * 64 + lane + 256 * i;
    uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
    uint4 xv;
    float cs = stage_x8<FMT>(d, xv);
    cs += __shfl_xor(cs, 1);
    cs += __shfl_xor(cs, 2);
    if (u < n8) {
      s.xl[u] = xv;
      if ((u & 3) == 0) s.xsum[u >> 2] = cs;
    }
  }
  // the wave finishing the staging releases the op
  unsigned old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(ctl.w + 60, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
  old = __shfl(old, 0);
  if (old % NGW == NGW - 1 && lane == 0) lds_st(ctl.xready(), (unsigned)(k + 1));
  return true;
}

template <int FMT, int QPK, int CPT_C, int CPT_I>
__device__ bool gather(const Args& a, const Ctl& ctl, const Clock& clk, const Lds& s, const OpInfo& o, long p,
                       unsigned tag, int k, int cw, unsigned ng, unsigned ngemv) {
  unsigned char* scl = s.scl + scale_buf(o.kind) * SCALE_BYTES;
  const Geo& g = a.g;
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x;
  const lga_engine_layer* Lp = o.kind == K_LM ? nullptr : a.layers + o.l;
  const uint16_t* x0 = (const uint16_t*)(a.scratch + g.o_x0);
  const uint64_t* xg = (const uint64_t*)(a.scratch + g.o_x);  // x[l] of layer l >= 1 at xg + (l - 1) * C / 2
  const uint64_t* qkvg = (const uint64_t*)(a.scratch + g.o_qkv);
  const uint64_t* yg = (const uint64_t*)(a.scratch + g.o_y);
  const uint64_t* xpg = (const uint64_t*)(a.scratch + g.o_xp);
  const uint64_t* gg = (const uint64_t*)(a.scratch + g.o_g);
  const int rpu = op_rows_per_unit(o.kind);
  const int n0 = o.u0 * rpu, rows = o.n_units * rpu;
  const size_t hC = (size_t)g.C / 2;
  const void* xl_in = o.l == 0 ? (const void*)x0 : (const void*)(xg + (o.l - 1) * hC);  // block input x_l
  switch (o.kind) {
    case K_QKV:
      return gather_gemv<FMT, CPT_C, true, false, false>(a, ctl, clk, s, cw, k, ng, ngemv, tag, scl, Lp->qkv_s, nullptr, n0,
                                                         rows, g.gC, xl_in, o.l == 0, (const uint16_t*)Lp->norm1,
                                                         nullptr, false, g.C);
    case K_O:
      return gather_gemv<FMT, CPT_C, false, true, false>(a, ctl, clk, s, cw, k, ng, ngemv, tag, scl, Lp->o_s, nullptr, n0,
                                                         rows, g.gC, yg + o.l * hC, false, nullptr, xl_in, o.l == 0,
                                                         g.C);
    case K_FC:
      return gather_gemv<FMT, CPT_C, true, false, true>(a, ctl, clk, s, cw, k, ng, ngemv, tag, scl, Lp->fc1_s, Lp->fc2_s,
                                                        n0, rows, g.gC, xpg + o.l * hC, false,
                                                        (const uint16_t*)Lp->norm2, nullptr, false, g.C);
    case K_DN:
      return gather_gemv<FMT, CPT_I, false, true, false>(a, ctl, clk, s, cw, k, ng, ngemv, tag, scl, Lp->dn_s, nullptr, n0,
                                                         rows, g.gI, gg + o.l * ((size_t)g.I / 2), false, nullptr,
                                                         xpg + o.l * hC, false, g.I);
    case K_LM:
      return gather_gemv<FMT, CPT_C, true, false, false>(a, ctl, clk, s, cw, k, ng, ngemv, tag, scl, a.lm_s, nullptr, n0,
                                                         rows, g.gC, g.L == 0 ? (const void*)x0 : (const void*)(xg + (g.L - 1) * hC),
                                                         g.L == 0, a.ln_f, nullptr, false, g.C);
    default: {  // attention (wave 0): the group's q heads, k, v granules; RoPE; the new key/value appended
      const AttnSplit as = attn_split(g, c, p);
      const int HS = 128;
      const long rp = min(max(p, 0L), (long)g.rope_rows - 1);
      const int sub = lane & 15;
      const float* cr = a.cos + (size_t)rp * HS + sub * 8;
      const float* sr = a.sin + (size_t)rp * HS + sub * 8;
      const uint64_t* row = qkvg + o.l * ((size_t)g.QN / 2) + (size_t)as.grp * (QPK + 2) * HS / 2;
      // (QPK + 2) heads of 16 lanes x 8 dims (4 granules); four heads per pass of the wave
      for (int h0 = 0; h0 < QPK + 2; h0 += 4) {
        const int h = min(h0 + (lane >> 4), QPK + 1);
        int idx[4];
        uint32_t d[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) idx[q] = (h * HS + sub * 8) / 2 + q;
        if (!poll_granules<4>(a, ctl, clk, row, idx, tag, d)) return false;
        const uint4 raw = make_uint4(d[0], d[1], d[2], d[3]);
        // rope8's DPP partner (row_ror:8) stays inside the 16-lane row of this head; every lane takes part
        const uint4 roped = rope8(raw, cr, sr, sub);
        if (h0 + (lane >> 4) < QPK + 2) {
          const uint4 val = h <= QPK ? roped : raw;  // q heads and k are roped, v is not
          *(uint4*)(s.qst + (size_t)h * HS + sub * 8) = val;
          if (as.owns_new && h >= QPK) {  // KVCache.forward index_copy_ at input_pos (model.py:788-795)
            uint16_t* cache = (uint16_t*)(h == QPK ? Lp->k_cache : Lp->v_cache);
            *(uint4*)(cache + ((size_t)as.grp * g.S + p) * HS + sub * 8) = val;
          }
        }
      }
#ifdef LGA_ENGINE_TRACE
      if (lane == 0) g_eng_trace[((size_t)blockIdx.x * TR_OPS + (unsigned)k) * TR_EV + 1] = __builtin_amdgcn_s_memrealtime();
#endif
      if (lane == 0) lds_st(ctl.xready(), (unsigned)(k + 1));
      return true;
    }
  }
}

// the last consumer wave of the CU (LDS count) publishes the op: one agent-scope add per CU
__device__ bool last_wave(const Ctl& ctl) {
  const int lane = threadIdx.x & 63;
  drain_stores();  // this wave's write-through outputs are complete before the count
  unsigned old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(ctl.done(), 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
  old = __shfl(old, 0);
  if (old != (unsigned)(NCW - 1)) return false;
  if (lane == 0) lds_st(ctl.done(), 0u);
  return true;
}

// ---- attention over this CU's key split --------------------------------------------------------------------
template <int QPK>
__device__ void attn_op(const Args& a, const Ctl& ctl, const Clock& clk, const Lds& s, const OpInfo& o, int cw,
                        unsigned line_base, unsigned useq, long p, unsigned epoch, unsigned tag) {
  constexpr int HS = 128, LPR = 16;
  const Geo& g = a.g;
  const int lane = threadIdx.x & 63, sub = lane & 15, rg = lane >> 4;
  const int c = blockIdx.x;
  const AttnSplit as = attn_split(g, c, p);
  float qf[QPK][8];
#pragma unroll
  for (int h = 0; h < QPK; ++h) unpack8(*(const uint4*)(s.qst + (size_t)h * HS + sub * 8), qf[h]);
  float m[QPK], l[QPK], acc[QPK][8];
#pragma unroll
  for (int h = 0; h < QPK; ++h) {
    m[h] = -INFINITY;
    l[h] = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[h][i] = 0.0f;
  }
  for (int u = cw; u < o.n_units; u += NCW) {
    const unsigned l0 = line_base + (unsigned)u * 8u;
    lds_st(ctl.posw(cw), l0);
    while (lds_ld(ctl.landed((int)((useq + (unsigned)u) % NLW))) < l0 + 8u) {
      if (lds_ld(ctl.abort()) || clk.expired()) {
        lds_st(ctl.abort(), 1u);
        return;
      }
      __builtin_amdgcn_s_sleep(0);
    }
    uint4 kv[4], vv[4];
#pragma unroll
    for (int jl = 0; jl < 4; ++jl) {
      kv[jl] = *(const uint4*)(s.ring + (size_t)((l0 + jl) % (unsigned)g.NL) * LINE + lane * 16);
      vv[jl] = *(const uint4*)(s.ring + (size_t)((l0 + 4 + jl) % (unsigned)g.NL) * LINE + lane * 16);
    }
    const int kbase = as.k_lo + u * ATT_KEYS + rg;
#pragma unroll
    for (int h = 0; h < QPK; ++h) {
      float sc[4];
      float mx = m[h];
#pragma unroll
      for (int jl = 0; jl < 4; ++jl) {
        float kf[8];
        unpack8(kv[jl], kf);
        float d = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) d = fmaf(qf[h][i], kf[i], d);
        const float sd = row_group_sum<LPR>(d) * g.scale;
        sc[jl] = (kbase + 4 * jl < as.k_end) ? sd : -INFINITY;
        mx = fmaxf(mx, sc[jl]);
      }
      // a row group whose keys so far are all masked keeps m = -inf: exp(-inf - -inf) must not make NaN
      const bool none = mx == -INFINITY;
      const float cf = none ? 0.0f : expf(m[h] - mx);
      l[h] *= cf;
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[h][i] *= cf;
#pragma unroll
      for (int jl = 0; jl < 4; ++jl) {
        const float e = none ? 0.0f : expf(sc[jl] - mx);
        l[h] += e;
        float vf[8];
        unpack8(vv[jl], vf);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[h][i] = fmaf(e, vf[i], acc[h][i]);
      }
      m[h] = mx;
    }
  }
  lds_st(ctl.posw(cw), line_base + (unsigned)o.n_units * 8u);
  // merge the four row groups of the wave
#pragma unroll
  for (int off = LPR; off < 64; off <<= 1) {
#pragma unroll
    for (int h = 0; h < QPK; ++h) {
      const float mo = __shfl_xor(m[h], off), lo = __shfl_xor(l[h], off);
      const float mn = fmaxf(m[h], mo);
      const float ca = mn == -INFINITY ? 0.0f : expf(m[h] - mn);
      const float cb = mn == -INFINITY ? 0.0f : expf(mo - mn);
      l[h] = l[h] * ca + lo * cb;
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[h][i] = acc[h][i] * ca + __shfl_xor(acc[h][i], off) * cb;
      m[h] = mn;
    }
  }
  float* mine = s.amrg + (size_t)cw * QPK * (HS + 4);
  if (lane < LPR) {
#pragma unroll
    for (int h = 0; h < QPK; ++h) {
      if (lane == 0) {
        mine[h * (HS + 4)] = m[h];
        mine[h * (HS + 4) + 1] = l[h];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) mine[h * (HS + 4) + 4 + sub * 8 + i] = acc[h][i];
    }
  }
  if (!last_wave(ctl)) return;
  ETRACE(o.l * OPS_PER_LAYER + 1, 4);
  // ---- the CU's split: merge the consumer waves, score the new key, publish (m, l, o), last split combines ----
  float* ws = (float*)(a.scratch + g.o_ws);
  uint64_t* yg = (uint64_t*)(a.scratch + g.o_y) + (size_t)o.l * (g.C / 2);  // granules
  const size_t row0 = (size_t)as.grp * QPK;  // first head of the group
#pragma unroll
  for (int h = 0; h < QPK; ++h) {
    float mx = -INFINITY;
    for (int w = 0; w < NCW; ++w) mx = fmaxf(mx, s.amrg[(size_t)w * QPK * (HS + 4) + h * (HS + 4)]);
    float lt = 0.0f, ot[2] = {0.0f, 0.0f};
    for (int w = 0; w < NCW; ++w) {
      const float* src = s.amrg + (size_t)w * QPK * (HS + 4) + h * (HS + 4);
      const float cf = mx == -INFINITY ? 0.0f : expf(src[0] - mx);
      lt += src[1] * cf;
      ot[0] += src[4 + lane] * cf;
      ot[1] += src[4 + 64 + lane] * cf;
    }
    if (as.owns_new) {  // the key/value at input_pos, from the staged (roped) qkv row
      float kf[8], qh[8];
      unpack8(*(const uint4*)(s.qst + (size_t)QPK * HS + sub * 8), kf);
      unpack8(*(const uint4*)(s.qst + (size_t)h * HS + sub * 8), qh);
      float d = 0.0f;
#pragma unroll
      for (int i = 0; i < 8; ++i) d = fmaf(qh[i], kf[i], d);
      const float sn = __shfl(row_group_sum<LPR>(d) * g.scale, 0);
      const float mn = fmaxf(mx, sn);
      const float cf = mx == -INFINITY ? 0.0f : expf(mx - mn);
      const float e = expf(sn - mn);
      lt = lt * cf + e;
      const uint16_t* vn = s.qst + (size_t)(QPK + 1) * HS;
      ot[0] = fmaf(e, bf2f(vn[lane]), ot[0] * cf);
      ot[1] = fmaf(e, bf2f(vn[64 + lane]), ot[1] * cf);
      mx = mn;
    }
    float* wsr = ws + (((size_t)o.l * g.H + row0 + h) * g.SP + as.split) * (HS + 4);
    __hip_atomic_store(wsr + 4 + lane, ot[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(wsr + 4 + 64 + lane, ot[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane == 0) {
      __hip_atomic_store(wsr, mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(wsr + 1, lt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  drain_stores();
  unsigned old = 0;
  if (lane == 0) old = g_add(slot(a, split_slot(g, o.l, as.grp)), 1u);
  old = __shfl(old, 0);
  if (old - epoch * (unsigned)g.SP != (unsigned)(g.SP - 1)) return;
  // last split of the group: flash-decoding merge of the SP splits (rounds of 8, as attention.hip's combine)
  if (lane == 0) lds_st(ctl.gathering(), 1u);
#pragma unroll
  for (int h = 0; h < QPK; ++h) {
    const float* base = ws + ((size_t)o.l * g.H + row0 + h) * g.SP * (HS + 4);
    float mx = -INFINITY, lt = 0.0f, ot[2] = {0.0f, 0.0f};
    for (int s0 = 0; s0 < g.SP; s0 += 8) {
      float mv[8], lv[8], ov[8][2];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float* r = base + (size_t)min(s0 + u, g.SP - 1) * (HS + 4);
        mv[u] = ld_sc1(r);
        lv[u] = ld_sc1(r + 1);
        ov[u][0] = ld_sc1(r + 4 + 2 * lane);
        ov[u][1] = ld_sc1(r + 4 + 2 * lane + 1);
      }
      float nm = mx;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (s0 + u >= g.SP) mv[u] = -INFINITY;
        nm = fmaxf(nm, mv[u]);
      }
      const float cf = expf(mx - nm);
      lt *= cf;
      ot[0] *= cf;
      ot[1] *= cf;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float e = expf(mv[u] - nm);
        lt = fmaf(lv[u], e, lt);
        ot[0] = fmaf(ov[u][0], e, ot[0]);
        ot[1] = fmaf(ov[u][1], e, ot[1]);
      }
      mx = nm;
    }
    g_st8(yg + (row0 + h) * (HS / 2) + lane, (uint64_t)pack2(ot[0] / lt, ot[1] / lt) | ((uint64_t)tag << 32));
  }
  if (lane == 0) lds_st(ctl.gathering(), 0u);
  ETRACE(o.l * OPS_PER_LAYER + 1, 7);
}

// ---- the consumer waves --------------------------------------------------------------------------------------
template <int FMT, int QPK, int CPT_C, int CPT_I>
__device__ void run_consumer(const Args& a, const Ctl& ctl, const Clock& clk, const Lds& s, int cw, int nops, long p,
                             unsigned epoch) {
  const Geo& g = a.g;
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x;
  unsigned line_base = 0, useq = 0;
  float best_v = -INFINITY;
  int best_i = 0x7FFFFFFF;
  const unsigned tag = epoch + 1u;  // this launch's granule tag
  unsigned ng = 0;                   // RMSNorm gathers so far
  unsigned ngemv = 0;                // GEMV ops finished by this wave
  for (int k = 0; k < nops; ++k) {
    const OpInfo o = op_info<CPT_C, CPT_I>(g, k, c, p);
    const bool norm = o.kind == K_QKV || o.kind == K_FC || o.kind == K_LM;
    ng += norm ? 1u : 0u;
    if (cw == 0) {
      ETRACE(k, 0);
#ifdef LGA_ENGINE_TRACE
      if (lane == 0) ctl.w[6] = (unsigned)min(k, TR_OPS - 1);
#endif
    }
    if (cw < NGW && (o.kind != K_ATTN || cw == 0)) {
      if (!gather<FMT, QPK, CPT_C, CPT_I>(a, ctl, clk, s, o, p, tag, k, cw, ng, ngemv)) {
        lds_st(ctl.abort(), 1u);
        break;
      }
      if (cw == 0) ETRACE(k, 2);
    }
    {
      bool ab = false;
      while (lds_ld(ctl.xready()) < (unsigned)(k + 1)) {
        if (lds_ld(ctl.abort())) { ab = true; break; }
        if (clk.expired()) {
          if (lane == 0) fail(a, ctl, 8u);
          ab = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (ab) break;
    }
    if (o.kind == K_ATTN) {
      attn_op<QPK>(a, ctl, clk, s, o, cw, line_base, useq, p, epoch, tag);
      if (cw == 0) ETRACE(k, 3);
    } else {
      const int rpu = op_rows_per_unit(o.kind);
      uint16_t* out;
      switch (o.kind) {
        // granule buffers (4 u16 per granule): the unit stores at granule n0 / 2
        case K_QKV: out = (uint16_t*)(a.scratch + g.o_qkv) + (size_t)o.l * g.QN * 2; break;
        case K_O: out = (uint16_t*)(a.scratch + g.o_xp) + (size_t)o.l * g.C * 2; break;
        case K_FC: out = (uint16_t*)(a.scratch + g.o_g) + (size_t)o.l * g.I * 2; break;
        case K_DN: out = (uint16_t*)(a.scratch + g.o_x) + (size_t)o.l * g.C * 2; break;
        default: out = a.logits; break;
      }
      const int rows_cu = o.n_units * rpu;
      const unsigned char* scl = s.scl + scale_buf(o.kind) * SCALE_BYTES;
      const int gshift = 31 - __builtin_clz((unsigned)g.grp);
      bool ab = false;
      for (int u = cw; u < o.n_units; u += NCW) {
        const unsigned l0 = line_base + (unsigned)(u * o.lines);
        lds_st(ctl.posw(cw), l0);
        while (lds_ld(ctl.landed((int)((useq + (unsigned)u) % NLW))) < l0 + (unsigned)o.lines) {
          if (lds_ld(ctl.abort()) || clk.expired()) { ab = true; break; }
          __builtin_amdgcn_s_sleep(0);
        }
        if (ab) break;
        const int n0 = (o.u0 + u) * rpu, lr0 = u * rpu;
        switch (o.kind) {
          case K_QKV:
            gemv_unit<FMT, 4, CPT_C, 1, false, false, false>(a, s, scl, l0, n0, lr0, g.ncC, g.gC, rows_cu, gshift, out, tag, best_v, best_i);
            break;
          case K_O:
            gemv_unit<FMT, 4, CPT_C, 1, false, true, false>(a, s, scl, l0, n0, lr0, g.ncC, g.gC, rows_cu, gshift, out, tag, best_v, best_i);
            break;
          case K_FC:
            gemv_unit<FMT, 2, CPT_C, 2, true, false, false>(a, s, scl, l0, n0, lr0, g.ncC, g.gC, rows_cu, gshift, out, tag, best_v, best_i);
            break;
          case K_DN:
            gemv_unit<FMT, 2, CPT_I, 1, false, true, false>(a, s, scl, l0, n0, lr0, g.ncI, g.gI, rows_cu, gshift, out, tag, best_v, best_i);
            break;
          default:
            gemv_unit<FMT, 2, CPT_C, 1, false, false, true>(a, s, scl, l0, n0, lr0, g.ncC, g.gC, rows_cu, gshift, out, tag, best_v, best_i);
            break;
        }
      }
      if (ab) {
        lds_st(ctl.abort(), 1u);
        break;
      }
      lds_st(ctl.posw(cw), line_base + (unsigned)(o.n_units * o.lines));
      // this wave is done reading the op's staged x / scales / residual rows
      if (lane == 0) __hip_atomic_fetch_add(ctl.w + 61, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      ++ngemv;
      if (o.kind == K_LM) {
        if (lane == 0) {
          ctl.cand(cw)[0] = __float_as_uint(best_v);
          ctl.cand(cw)[1] = (unsigned)best_i;
        }
      }
      if (cw == 0) ETRACE(k, 3);
      if (o.kind == K_LM && last_wave(ctl)) {
        ETRACE(k, 4);
        if (lane == 0) {
          // this CU's candidate, then the two-level arrival count; the last CU finishes the step
          float bv = -INFINITY;
          int bi = 0x7FFFFFFF;
          for (int w = 0; w < NCW; ++w) {
            const float v = __uint_as_float(lds_ld(ctl.cand(w)));
            const int i = (int)lds_ld(ctl.cand(w) + 1);
            if (better(v, i, bv, bi)) {
              bv = v;
              bi = i;
            }
          }
          uint64_t* cand = (uint64_t*)(a.scratch + g.o_cand);
          g_st8(cand + c, (uint64_t)(uint32_t)bi | ((uint64_t)__float_as_uint(bv) << 32));
          drain_stores();
          const int sh = c % NSH;
          const unsigned n_sh = (unsigned)shard_count(g.P, sh);
          const unsigned o1 = g_add(slot(a, arg_slot(g, sh)), 1u);
          bool top_last = false;
          if (o1 - epoch * n_sh == n_sh - 1) {
            const unsigned n_top = (unsigned)min(g.P, NSH);
            const unsigned o2 = g_add(slot(a, arg_slot(g, NSH)), 1u);
            top_last = o2 - epoch * n_top == n_top - 1;
          }
          ctl.w[5] = top_last ? 1u : 0u;
        }
        if (o.kind == K_LM && __shfl((int)ctl.w[5], 0)) {
          // the step's final arriver: global argmax (torch.argmax order), token, input_pos, next embedding
          const uint64_t* cand = (const uint64_t*)(a.scratch + g.o_cand);
          float bv = -INFINITY;
          int bi = 0x7FFFFFFF;
          for (int i = lane; i < g.P; i += 64) {
            const uint64_t v = g_ld8(cand + i);
            const float fv = __uint_as_float((uint32_t)(v >> 32));
            const int fi = (int)(uint32_t)v;
            if (better(fv, fi, bv, bi)) {
              bv = fv;
              bi = fi;
            }
          }
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) {
            const float ov = __shfl_xor(bv, off);
            const int oi = __shfl_xor(bi, off);
            if (better(ov, oi, bv, bi)) {
              bv = ov;
              bi = oi;
            }
          }
          if (bi >= g.V || bi < 0) bi = 0;
          const int tok = bi;
          const uint4* src = (const uint4*)(a.wte + (size_t)tok * g.C);
          uint4* dst = (uint4*)(a.scratch + g.o_x0);
          for (int i = lane; i < g.C / 8; i += 64) dst[i] = src[i];
          if (lane == 0) {
            if (a.token) *a.token = tok;
            if (a.out_idx) *a.out_idx = tok;
            *a.pos += 1;
            __hip_atomic_store(slot(a, 0), epoch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
    }
    line_base += (unsigned)(o.n_units * o.lines);
    useq += (unsigned)o.n_units;
    if (lds_ld(ctl.abort())) break;
  }
  lds_st(ctl.posw(cw), 0xFFFFFFFFu);
}

// lab: consumers that only wait for their units' lines and free them (no edges, no compute)
template <int CPT_C, int CPT_I>
__device__ void run_drain(const Args& a, const Ctl& ctl, const Clock& clk, int cw, int nops, long p) {
  unsigned line_base = 0, useq = 0;
  for (int k = 0; k < nops; ++k) {
    const OpInfo o = op_info<CPT_C, CPT_I>(a.g, k, blockIdx.x, p);
    if (cw == 0) ETRACE(k, 0);
    for (int u = cw; u < o.n_units; u += NCW) {
      const unsigned l0 = line_base + (unsigned)(u * o.lines);
      lds_st(ctl.posw(cw), l0);
      while (lds_ld(ctl.landed((int)((useq + (unsigned)u) % NLW))) < l0 + (unsigned)o.lines) {
        if (lds_ld(ctl.abort()) || clk.expired()) return;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    line_base += (unsigned)(o.n_units * o.lines);
    useq += (unsigned)o.n_units;
    lds_st(ctl.posw(cw), line_base);
    if (cw == 0) ETRACE(k, 3);
  }
  lds_st(ctl.posw(cw), 0xFFFFFFFFu);
}

template <int FMT, int QPK, int CPT_C, int CPT_I>
__global__ void __launch_bounds__(NTHREADS) engine_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Geo& g = a.g;
  const int kmax = g.C > g.I ? g.C : g.I;
  Lds s;
  s.ring = smem;
  unsigned char* q = smem + g.lds_ring;
  Ctl ctl{(unsigned*)q};
  q += 1024;
  s.res = (uint16_t*)q;
  q += RES_ROWS * 2;
  s.qst = (uint16_t*)q;
  q += (QPK + 2) * 128 * 2;
  s.amrg = (float*)q;
  q += NCW * QPK * (128 + 4) * 4;
  s.scl = q;
  q += 2 * SCALE_BYTES;
  s.xl = (uint4*)q;
  q += kmax * 2;
  s.xsum = (float*)q;
  q += (kmax / 32) * 4;
  s.red = (float*)q;
  s.nf4 = s.red + 16;
  if (threadIdx.x < 256) ctl.w[threadIdx.x] = 0u;
  if (FMT == 1 && threadIdx.x < 16) s.nf4[threadIdx.x] = kNF4v[threadIdx.x];
  __syncthreads();
  Clock clk{__builtin_amdgcn_s_memrealtime()};
  const long p = *a.pos;
  const unsigned epoch = g_ld(slot(a, 0));
  const int total = g.L * OPS_PER_LAYER + 1;
  const int nops = a.op_limit > 0 ? min(a.op_limit, total) : total;
  const bool stream_only = a.op_limit < 0;  // lab: the ring's raw throughput (tools/engine_trace.py); -2: interleaved
  const int wave = threadIdx.x >> 6;
  if (g_ld(slot(a, 2))) return;  // a previous launch gave up: the state needs lga_engine_reset
  if (wave < NLW) run_loader<CPT_C, CPT_I>(a, ctl, clk, s.ring, nops, p, wave, a.op_limit == -2);
  else if (stream_only) run_drain<CPT_C, CPT_I>(a, ctl, clk, wave - NLW, nops, p);
  else run_consumer<FMT, QPK, CPT_C, CPT_I>(a, ctl, clk, s, wave - NLW, nops, p, epoch);
}

}  // namespace eng
}  // namespace lga

#ifdef LGA_ENGINE_TRACE
extern "C" int lga_engine_trace_read(unsigned long long* host, long n) {
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(lga::eng::g_eng_trace), (size_t)n * sizeof(unsigned long long));
  void* dptr = nullptr;
  if (e == hipSuccess) e = hipGetSymbolAddress(&dptr, HIP_SYMBOL(lga::eng::g_eng_trace));
  if (e == hipSuccess) e = hipMemset(dptr, 0, sizeof(lga::eng::g_eng_trace));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}
#endif

// ---- C ABI ---------------------------------------------------------------------------------------------------
namespace {

// the per-op kernels' launch choices (gemv.hip dispatch / stream_default) the engine reproduces bit for bit
bool stream_default_(int N, int K, bool dual) { return K <= 4096 && (dual ? N >= 8192 : N >= 24000); }

const char* engine_unsupported(const lga_engine_geom* g, lga::eng::Geo& o, int& cpt_c, int& cpt_i) {
  using namespace lga::eng;
  if (!g) return "null geometry";
  if (g->fmt != 0) return "int4-g weights only (nf4 runs the per-op kernels)";
  if (g->head_size != 128) return "head_size must be 128";
  if (g->n_query_groups <= 0 || g->n_head % g->n_query_groups) return "n_head must be a multiple of n_query_groups";
  if (g->n_head / g->n_query_groups != 1) return "q_per_kv must be 1 (the instantiated attention)";
  if (g->n_head * g->head_size != g->n_embd) return "n_head * head_size must equal n_embd";
  if (g->n_cu <= 0 || g->n_cu > 1024 || g->n_cu % g->n_query_groups) return "n_cu must be a multiple of n_query_groups";
  if (g->n_embd % 32 || g->intermediate % 32) return "n_embd and intermediate_size must be multiples of 32";
  if (g->group < 32 || g->group % 32 || g->n_embd % g->group || g->intermediate % g->group) return "bad group";
  if ((g->n_embd / g->group) % 2 || (g->intermediate / g->group) % 2) return "groups per row must be even";
  if (g->group & (g->group - 1)) return "group must be a power of two";
  if (g->max_seq <= 0 || g->rope_rows <= 0 || g->n_layer <= 0 || g->vocab <= 0) return "empty geometry";
  cpt_c = (g->n_embd / 32 + 63) / 64;
  cpt_i = (g->intermediate / 32 + 63) / 64;
  if (cpt_c != 2 || cpt_i != 6) return "instantiated for n_embd in (2048, 4096] and intermediate in (10240, 12288]";
  const int QN = (g->n_head + 2 * g->n_query_groups) * g->head_size;
  // the per-op kernels pick: qkv / o_proj one-shot 4 rows per wave, fc_1||fc_2 streaming 1 row, mlp.proj one-shot
  // 2 rows (cpt 5-6), lm_head streaming 2 rows — the engine computes with the same groupings
  if (QN >= 24000 || g->n_embd >= 24000 || stream_default_(QN, g->n_embd, false) || stream_default_(g->n_embd, g->n_embd, false))
    return "qkv / o_proj shapes outside the one-shot 4-row GEMV";
  if (!stream_default_(g->intermediate, g->n_embd, true)) return "fc_1/fc_2 shape outside the streaming dual GEMV";
  if (!stream_default_(g->vocab, g->n_embd, false)) return "lm_head shape outside the streaming GEMV";
  if (QN % 4 || g->n_embd % 4 || g->intermediate % 2 || g->vocab % 2) return "row counts must be unit multiples";
  if (!make_geo(*g, o, cpt_c, cpt_i)) return "bad geometry";
  auto rows_max = [&](int N, int rpu) { return ((N / rpu + o.P - 1) / o.P) * rpu; };
  if (rows_max(QN, 4) * o.gC * 2 > SCALE_BYTES || rows_max(o.C, 4) * o.gC * 2 > SCALE_BYTES ||
      2 * rows_max(o.I, 2) * o.gC * 2 > SCALE_BYTES || rows_max(o.C, 2) * o.gI * 2 > SCALE_BYTES ||
      rows_max(o.V, 2) * o.gC * 2 > SCALE_BYTES)
    return "an op's scales for one CU exceed the LDS scale area";
  if (rows_max(o.C, 4) > RES_ROWS || rows_max(o.C, 2) > RES_ROWS) return "residual rows exceed the LDS area";
  if (o.NL < NCW * 12 + 12) return "LDS ring too small";
  return nullptr;
}

}  // namespace

extern "C" int lga_engine_check(const lga_engine_geom* g) {
  lga::eng::Geo o;
  int a, b;
  const char* why = engine_unsupported(g, o, a, b);
  if (why) {
    lga_set_error(why);
    return (int)hipErrorInvalidValue;
  }
  return 0;
}

extern "C" size_t lga_engine_scratch_bytes(const lga_engine_geom* g) {
  lga::eng::Geo o;
  int a, b;
  if (engine_unsupported(g, o, a, b)) return 0;
  return o.total;
}

extern "C" void* lga_engine_x0(const lga_engine_geom* g, void* scratch) {
  lga::eng::Geo o;
  int a, b;
  if (!scratch || engine_unsupported(g, o, a, b)) return nullptr;
  return (unsigned char*)scratch + o.o_x0;
}

extern "C" int lga_engine_reset(const lga_engine_geom* g, void* scratch, hipStream_t stream) {
  lga::eng::Geo o;
  int a, b;
  const char* why = engine_unsupported(g, o, a, b);
  LGA_CHECK_ARG(!why && scratch, "lga_engine_reset: unsupported geometry or null scratch");
  // counters, and the granule buffers (their tags restart with the epoch)
  hipError_t e = hipMemsetAsync(scratch, 0, (size_t)o.n_slots * lga::eng::CSTRIDE * 4, stream);
  if (e == hipSuccess) e = hipMemsetAsync((unsigned char*)scratch + o.o_x, 0, o.o_ws - o.o_x, stream);
  if (e != hipSuccess) {
    lga_set_error(hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

extern "C" int lga_engine_error(const lga_engine_geom* g, const void* scratch, unsigned* err_out) {
  LGA_CHECK_ARG(scratch && err_out, "lga_engine_error: null pointer");
  (void)g;
  unsigned w[2] = {0, 0};
  const hipError_t e = hipMemcpy(w, (const unsigned char*)scratch + lga::eng::CSTRIDE * 4, sizeof(unsigned),
                                 hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    lga_set_error(hipGetErrorString(e));
    return (int)e;
  }
  *err_out = w[0];
  return 0;
}

extern "C" int lga_decode_engine(const lga_engine_geom* g, const lga_engine_layer* layers, const void* lm_w,
                                 const void* lm_s, const void* ln_f, const void* wte, const float* cos,
                                 const float* sin, int64_t* pos, int32_t* token, int64_t* out_idx, void* logits,
                                 void* scratch, int op_limit, hipStream_t stream) {
  lga::eng::Geo o;
  int cpt_c = 0, cpt_i = 0;
  const char* why = engine_unsupported(g, o, cpt_c, cpt_i);
  if (why) {
    lga_set_error(why);
    return (int)hipErrorInvalidValue;
  }
  LGA_CHECK_ARG(layers && lm_w && lm_s && ln_f && wte && cos && sin && pos && logits && scratch,
                "lga_decode_engine: null pointer");
  lga::eng::Args a;
  a.g = o;
  a.layers = layers;
  a.lm_w = (const uint8_t*)lm_w;
  a.lm_s = lm_s;
  a.ln_f = (const uint16_t*)ln_f;
  a.wte = (const uint16_t*)wte;
  a.cos = cos;
  a.sin = sin;
  a.pos = pos;
  a.token = token;
  a.out_idx = out_idx;
  a.logits = (uint16_t*)logits;
  a.scratch = (unsigned char*)scratch;
  a.op_limit = op_limit;
  auto kern = lga::eng::engine_kernel<0, 1, 2, 6>;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    if (e != hipSuccess) {
      lga_set_error(hipGetErrorString(e));
      return (int)e;
    }
    attr = true;
  }
  kern<<<o.P, lga::eng::NTHREADS, o.lds_total, stream>>>(a);
  LGA_LAUNCH_RETURN();
}
