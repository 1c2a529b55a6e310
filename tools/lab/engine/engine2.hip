// Persistent decode engine, version 2 ("stream engine"): the whole greedy decode step in ONE launch, with the
// weight / K-V stream held in REGISTERS and run ahead across op boundaries.
//
// Replaces, for one token of generate/base.py's decode loop (next_token -> GPT.forward -> Block.forward x L ->
// ln_f -> lm_head -> sample(T=0); reference generate/base.py:44-47,87-92; lit_gpt/model.py:499-519,572-593,
// 609-656,712-716; lit_gpt/rmsnorm.py:19-25), the chain of 160 per-op launches (gemv.hip, attention.hip,
// sample.hip). Version 1 (engine.hip: an LDS-DMA ring per CU, 4 loader + 8 consumer waves, granule hand-offs)
// measured 2.22 ms/step against 1.33 for the per-op graph; its trace (profiles/r04a_engine_v1_trace.txt) showed
// every op paying 2.6-10 us of wait for the last producer CU plus ~2.3 us of gather, with the ring (113 KB)
// too small to keep HBM busy across them. This version changes the three things that trace points at:
//  * COMPUTE WAVES STREAM THEIR OWN TILES INTO REGISTERS (8 per CU, two tiles of 8 x 16 B + 8 scales per lane in
//    flight each: ~128 KB per CU, loads issued by inline asm so the run-ahead is not cut by hipcc's vmcnt
//    bookkeeping): the tile after next is issued as soon as a tile is consumed, whatever op it belongs to, so the
//    next op's weights (or K/V rows) are already landing while the current edge is still open;
//  * GATHER WAVES NEVER STREAM (4 per CU): they poll the producers' arrival counters, load the finished
//    activation vector (write-through sc1 loads: 16-44 KB), apply the fused RMSNorm, stage it in LDS exactly as
//    the per-op GEMV does and release the op to the compute waves through an LDS word — so the edge's loads do not
//    queue behind this CU's weight stream in one wave's in-order vmcnt;
//  * THE qkv -> ATTENTION EDGE IS LOCAL: the 8 CUs that own a query group's attention splits also compute that
//    group's 384 qkv rows, and wait only for each other (one 8-arrival counter per group).
// Hand-offs follow MI355X_MICROARCH.md "Valid forms" row 1: payload stored write-through (sc1) by every producing
// wave, each wave drains (vmcnt), the CU's last wave (LDS count) adds once to an agent-scope counter (sharded 8 ways
// for the all-to-all edges); consumers poll the counter with sc1 loads and read the payload with sc1 loads. The
// counters are monotonic across launches (targets from the launch epoch the last CU advances), so nothing is re-armed
// and the launch is graph-capturable. GEMV arithmetic is the per-op kernels' bit for bit (same chunk order, x
// staging, RMSNorm tree, butterflies, epilogues); the attention splits keys per CU differently (fp32 online
// softmax, within 2 bf16 ulps). Every wait is bounded (TMO), then the launch sets the error word and drains.
#include <string.h>

#include <unordered_map>
#include <vector>

#include "decode_ops.h"
#include "engine.h"

namespace lga {
namespace e2 {

constexpr int NGW = 4;              // gather waves (never stream)
constexpr int NCW = 8;              // compute waves (stream their tiles)
constexpr int NW = NGW + NCW;
constexpr int NT = NW * 64;
constexpr int CSW = 16;             // uint32 words per counter (one 64-B line each)
constexpr int NSH = 8;              // shards of an all-to-all arrival counter
constexpr int OPS = 5;              // QKV, ATT, OPJ, FC, DN per block
constexpr int KEYS = 16;            // keys per attention tile (4 per 16-lane row group)
constexpr int HS = 128;
constexpr unsigned long long TMO = 2000000ull;  // 20 ms of the 100 MHz clock
constexpr size_t kArgsBytes = 8192;  // the Args block at the start of the scratch (counters follow)
constexpr int LDS_MIN = 84 * 1024;
constexpr int MAXJ = 8;             // output records per compute wave per op (fc_1 || fc_2: <= 6 tiles)  // > 80 KB: one workgroup per CU, all resident

enum Kind { QKV = 0, ATT = 1, OPJ = 2, FC = 3, DN = 4, LM = 5 };

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#ifdef LGA_ENGINE_TRACE  // lab builds only: per-(CU, op) event times, 100 MHz clock
constexpr int TR_OPS = 192, TR_EV = 8;
__device__ unsigned long long g_e2_trace[256 * TR_OPS * TR_EV];
#define E2TRACE(k, ev)                                                                                     \
  do {                                                                                                   \
    if ((threadIdx.x & 63) == 0 && (k) < TR_OPS)                                                         \
      g_e2_trace[((size_t)blockIdx.x * TR_OPS + (k)) * TR_EV + (ev)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define E2TRACE(k, ev) \
  do {                 \
  } while (0)
#endif

struct Geo {
  int L, C, H, G, I, V, S, grp, rope_rows, P, SP, QPK, QN, GQ, QT;
  float eps, scale;
  int gC, gI, ncC, ncI;
  int c_xo, c_qkv, c_split, c_y, c_xp, c_g, c_lm, c_top, c_key, n_ctr;
  size_t o_x0, o_act, act_len, o_ws, o_dummy, total;
  int a_qkv, a_y, a_xp, a_g, a_x;  // element offsets inside one layer's activation block
  int sb;                          // bytes of one LDS staging buffer
  int lds;
};

__host__ __device__ inline size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

__host__ inline bool make_geo(const lga_engine_geom& g, Geo& o) {
  o.L = g.n_layer;
  o.C = g.n_embd;
  o.H = g.n_head;
  o.G = g.n_query_groups;
  o.I = g.intermediate;
  o.V = g.vocab;
  o.S = g.max_seq;
  o.grp = g.group;
  o.rope_rows = g.rope_rows;
  o.P = g.n_cu;
  o.eps = g.norm_eps;
  o.scale = g.attn_scale;
  if (o.G <= 0 || o.H % o.G || o.P % o.G) return false;
  o.SP = o.P / o.G;
  o.QPK = o.H / o.G;
  o.GQ = (o.QPK + 2) * HS;  // qkv rows per query group
  o.QN = o.G * o.GQ;
  o.QT = o.GQ / 4;
  o.gC = o.C / o.grp;
  o.gI = o.I / o.grp;
  o.ncC = o.C / 32;
  o.ncI = o.I / 32;
  int s = 3;
  o.c_xo = s; s += o.L * NSH;
  o.c_qkv = s; s += o.L * o.G;
  o.c_split = s; s += o.L * o.G;
  o.c_y = s; s += o.L * NSH;
  o.c_xp = s; s += o.L * NSH;
  o.c_g = s; s += o.L * NSH;
  o.c_lm = s; s += NSH;
  o.c_top = s; s += 1;
  o.c_key = s; s += 1;
  o.n_ctr = s;
  size_t off = kArgsBytes + al256((size_t)o.n_ctr * CSW * 4);
  o.o_x0 = off;
  off += al256((size_t)o.C * 2);
  o.a_qkv = 0;
  o.a_y = o.a_qkv + o.QN;
  o.a_xp = o.a_y + o.C;
  o.a_g = o.a_xp + o.C;
  o.a_x = o.a_g + o.I;
  o.act_len = al256((size_t)(o.a_x + o.C) * 2);
  o.o_act = off;
  off += o.act_len * o.L;
  o.o_ws = off;
  off += al256((size_t)o.L * o.H * o.SP * (HS + 4) * 4);
  o.o_dummy = off;
  off += al256((size_t)o.P * NCW * 64);
  o.total = off;
  const int kmax = o.C > o.I ? o.C : o.I;
  o.sb = ((kmax * 2 + (kmax / 32) * 4) + 15) & ~15;
  const int need = 1024 + 2 * o.sb + o.C * 2 + 3 * HS * 2 + NCW * (HS + 4) * 4 + 2 * NCW * MAXJ * 16 + 64;
  o.lds = need > LDS_MIN ? need : LDS_MIN;
  return true;
}

// The launch's fixed arguments live in DEVICE memory at the start of the scratch (written once per binding by
// lga_decode_engine, outside any graph capture): read through a const __restrict__ pointer they are scalar loads
// hipcc issues where needed, instead of ~90 kernel-argument SGPRs it must keep (or spill) for the whole launch.
constexpr int kMaxLayers = 64;
struct Args {
  Geo g;
  lga_engine_layer layers[kMaxLayers];
  const uint8_t* lm_w;
  const uint16_t* lm_s;
  const uint16_t* ln_f;
  const uint16_t* wte;
  const float* cos;
  const float* sin;
  unsigned char* scratch;
};
// per-launch arguments (by value)
struct Dyn {
  int64_t* pos;
  int32_t* token;
  int64_t* out_idx;
  uint16_t* logits;
  int op_limit;
};

// ---- global (agent-scope) helpers -----------------------------------------------------------------------------
// Pointers read from the Args block are generic; every global access goes through an address_space(1) cast so it
// is a global_* instruction (a flat_* one counts in vmcnt AND lgkmcnt and makes hipcc wait vmcnt(0), draining the
// compute waves' in-flight tiles).
template <class T>
using gptr = __attribute__((address_space(1))) T*;
template <class T>
__device__ __forceinline__ gptr<T> G(T* p) { return (gptr<T>)p; }
template <class T>
__device__ __forceinline__ gptr<const T> G(const T* p) { return (gptr<const T>)p; }
__device__ __forceinline__ gptr<unsigned> ctr(const Args& a, int i) {
  return G((unsigned*)(a.scratch + kArgsBytes)) + (size_t)i * CSW;
}
__device__ __forceinline__ unsigned g_ld(gptr<unsigned> p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_add_nr(gptr<unsigned> p, unsigned v) {  // no-return form (no wait on the result)
  (void)__hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned g_add(gptr<unsigned> p, unsigned v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint16_t* act(const Args& a, int l) {
  return (uint16_t*)(a.scratch + a.g.o_act + a.g.act_len * (size_t)l);
}
constexpr int kSc1 = 16;  // buffer cache-policy aux bit SC1 (write-through store / L2-bypassing load)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ uint4 gld16(const void* p) {
  const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void gst16(void* p, uint4 v) {
  const u32x4 w = {v.x, v.y, v.z, v.w};
  *(__attribute__((address_space(1))) u32x4*)p = w;
}
__device__ __forceinline__ void st_sc1g(float* p, float v) {
  __hip_atomic_store(G(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1g(const float* p) {
  return __hip_atomic_load((gptr<float>)G(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint4 ld_sc1_16(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSc1));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// ---- LDS ----------------------------------------------------------------------------------------------------------
// Every LDS pointer is derived from this namespace-scope array inside the function that uses it, so hipcc keeps
// LDS address space (ds_* instructions): a generic pointer passed through a struct would become flat_* accesses,
// which count in vmcnt and would make hipcc drain the compute waves' in-flight tiles.
extern __shared__ __attribute__((aligned(16))) unsigned char e2_smem[];
struct Ctl {
  __device__ unsigned* w() const { return (unsigned*)e2_smem; }
  __device__ unsigned* ready() const { return w() + 0; }   // op index + 1 whose input is staged
  __device__ unsigned* abort() const { return w() + 1; }
  __device__ unsigned* gws() const { return w() + 2; }     // gather-wave sync counter
  __device__ unsigned* attc() const { return w() + 3; }    // attention partials posted (monotonic)
  __device__ unsigned* arr(int k) const { return w() + 4 + (k & 3); }  // compute-wave arrivals per op (monotonic)
  __device__ unsigned* prog(int cw) const { return w() + 8 + cw; }     // ops finished by compute wave cw
  __device__ unsigned* best(int cw) const { return w() + 16 + 2 * cw; }
  __device__ float* red(int par) const { return (float*)(w() + 32 + 4 * (par & 1)); }
  __device__ unsigned* last() const { return w() + 40; }
  __device__ unsigned* edge() const { return w() + 41; }                  // op index + 1 whose input edge is complete
  __device__ unsigned* rcnt(int k, int cw) const { return w() + 48 + 8 * (k & 1) + cw; }  // records per wave
};
struct Lds {
  int sb, C;
  __device__ unsigned char* stage(int k) const { return e2_smem + 1024 + (size_t)(k & 1) * sb; }  // x staging
  __device__ uint16_t* raw() const { return (uint16_t*)(e2_smem + 1024 + 2 * (size_t)sb); }  // residual input
  __device__ uint16_t* qst() const { return raw() + C; }  // roped q, roped k_new, v_new (bf16 heads)
  __device__ float* amrg() const { return (float*)(qst() + 3 * HS); }  // per compute wave: m, l, -, -, o[HS]
  // op outputs of this CU for the gather waves to publish: per op parity, per compute wave, MAXJ records of
  // {element offset, count (2 or 4), 4 bf16}; the wave's record count in rcnt
  __device__ uint4* rec(int k, int w, int j) const {
    return (uint4*)(amrg() + NCW * (HS + 4)) + ((size_t)(k & 1) * NCW + w) * MAXJ + j;
  }
};
__device__ __forceinline__ unsigned lds_ld(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ unsigned lds_add(unsigned* p, unsigned v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
}

struct Clock {
  unsigned long long t0;
  __device__ bool expired() const { return __builtin_amdgcn_s_memrealtime() - t0 > TMO; }
};

__device__ __forceinline__ void fail(const Args& a, const Ctl& ctl, unsigned code) {
  __hip_atomic_fetch_or(ctr(a, 1), code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(ctr(a, 2), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  lds_st(ctl.abort(), 1u);
}

// spin until *p >= target (LDS); false on abort / timeout
__device__ __forceinline__ bool lds_wait(const Args& a, const Ctl& ctl, const Clock& clk, const unsigned* p, unsigned target,
                         unsigned code) {
  for (unsigned it = 0; lds_ld(p) < target; ++it) {
    if (lds_ld(ctl.abort())) return false;
    if ((it & 63u) == 63u && clk.expired()) {
      if ((threadIdx.x & 63) == 0) fail(a, ctl, code);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// spin until the n counters at ctr(first + i * stride), i < n <= 64, each reach `target` (one lane per counter)
__device__ __forceinline__ bool poll_ctrs(const Args& a, const Ctl& ctl, const Clock& clk, int first, int n, int stride,
                          unsigned target, unsigned code) {
  const int lane = threadIdx.x & 63;
  const gptr<unsigned> p = ctr(a, first + min(lane, n - 1) * stride);
  for (unsigned it = 0;; ++it) {
    const unsigned v = g_ld(p);
    if (__all((int)(v - target) >= 0)) return true;
    if ((it & 15u) == 15u) {
      if (lds_ld(ctl.abort()) || g_ld(ctr(a, 2))) {
        lds_st(ctl.abort(), 1u);
        return false;
      }
      if (clk.expired()) {
        if (lane == 0) fail(a, ctl, code);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// ---- op schedule --------------------------------------------------------------------------------------------------
__device__ __forceinline__ int kind_of(const Geo& g, int k) { return k >= g.L * OPS ? LM : k % OPS; }

struct Split {
  int grp, split, k_lo, k_end, nkeys, nunits;
  bool owns_new;
};
__device__ __forceinline__ Split make_split(const Geo& g, int c, long p) {
  Split s;
  s.grp = c % g.G;
  s.split = c / g.G;
  const int Lk = (int)min(p + 1, (long)g.S);
  const int chunk = (Lk + g.SP - 1) / g.SP;
  s.k_lo = min(s.split * chunk, Lk);
  const int k_hi = min(s.k_lo + chunk, Lk);
  s.owns_new = p < g.S && s.k_lo <= p && p < k_hi;
  s.k_end = s.owns_new ? (int)p : k_hi;
  s.nkeys = max(0, s.k_end - s.k_lo);
  s.nunits = (s.nkeys + KEYS - 1) / KEYS;
  return s;
}

// tiles of op k owned by compute wave w of CU c (the GEMV ops deal tiles to slots cw-major: slot = w * P + c)
__device__ __forceinline__ int my_tiles(const Geo& g, int k, int c, int w, const Split& sp) {
  const int S = NCW * g.P, slot = w * g.P + c;
  auto cnt = [](int first, int step, int T) { return first < T ? (T - first + step - 1) / step : 0; };
  switch (kind_of(g, k)) {
    case QKV: return cnt(sp.split + g.SP * w, g.SP * NCW, g.QT);
    case ATT: return cnt(w, NCW, sp.nunits);
    case OPJ: return cnt(slot, S, g.C / 4);
    case FC: return cnt(slot, S, g.I / 2);
    case DN: return 2 * cnt(slot, S, g.C / 2);
    default: return cnt(slot, S, g.V / 4);
  }
}

struct Cur {
  int k, j, n;  // op, tile of this wave within the op, this wave's tile count in the op
};

// ---- tiles: 8 x 16 B of weights (or K / V rows) + 8 scales per lane ----------------------------------------------
// Every tile, whatever its op, is issued by the SAME 16 loads (8 x 16-B non-temporal + 8 x 2-B) from per-kind
// addresses computed without memory accesses: hipcc then sees one straight-line issue sequence and its vmcnt waits
// in the two-buffer loop below are exact (a tile's first use waits only for that tile).
struct Tile {
  u32x4 w[8];
  uint32_t s[8];
};
struct TileAddr {
  const unsigned char* b[2];   // weight / K / V base of entries 0-3 and 4-7
  const uint16_t* sb[2];       // scale base of entries 0-3 and 4-7
  uint32_t off[8];             // bytes
  uint32_t soff[8];            // elements
};

struct Ctx {
  int c, w, lane;
  Split sp;
  long p;
  const void* dummy;  // a valid, cached address for the loads of padding tiles
};

__device__ __forceinline__ void addr_of(const Args& a, const Ctx& x, const Cur& cur, TileAddr& t) {
  const Geo& g = a.g;
  const int lane = x.lane;
  const int S = NCW * g.P, slot = x.w * g.P + x.c;
  const int nops = g.L * OPS + 1;
  const int kind = cur.k < nops ? kind_of(g, cur.k) : -1;
  const lga_engine_layer& Ly = a.layers[cur.k < g.L * OPS ? cur.k / OPS : 0];
  switch (kind) {
    case QKV:
    case OPJ:
    case LM: {  // 4 rows x 2 chunks (K = C): entry 2 i + j
      const int t4 = kind == QKV ? (x.sp.split + g.SP * x.w) + g.SP * NCW * cur.j : slot + S * cur.j;
      const int n0 = kind == QKV ? x.sp.grp * g.GQ + 4 * t4 : 4 * t4;
      const int N = kind == QKV ? g.QN : (kind == OPJ ? g.C : g.V);
      t.b[0] = t.b[1] = (const unsigned char*)(kind == LM ? (const void*)a.lm_w : kind == QKV ? Ly.qkv_w : Ly.o_w);
      t.sb[0] = t.sb[1] = (const uint16_t*)(kind == LM ? (const void*)a.lm_s : kind == QKV ? Ly.qkv_s : Ly.o_s);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const unsigned n = (unsigned)min(n0 + i, N - 1);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const unsigned ch = (unsigned)min(lane + 64 * j, g.ncC - 1);
          t.off[i * 2 + j] = n * (unsigned)(g.C / 2) + ch * 16;
          t.soff[i * 2 + j] = n * (unsigned)g.gC + (ch * 32) / (unsigned)g.grp;
        }
      }
      break;
    }
    case FC: {  // rows n0, n0 + 1: entry 4 m + 2 r + j (m 0: fc_1, 1: fc_2)
      const int n0 = 2 * (slot + S * cur.j);
      t.b[0] = (const unsigned char*)Ly.fc1_w;
      t.b[1] = (const unsigned char*)Ly.fc2_w;
      t.sb[0] = (const uint16_t*)Ly.fc1_s;
      t.sb[1] = (const uint16_t*)Ly.fc2_s;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const unsigned n = (unsigned)min(n0 + r, g.I - 1);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const unsigned ch = (unsigned)min(lane + 64 * j, g.ncC - 1);
#pragma unroll
          for (int m = 0; m < 2; ++m) {
            t.off[4 * m + 2 * r + j] = n * (unsigned)(g.C / 2) + ch * 16;
            t.soff[4 * m + 2 * r + j] = n * (unsigned)g.gC + (ch * 32) / (unsigned)g.grp;
          }
        }
      }
      break;
    }
    case DN: {  // rows n0, n0 + 1 (K = I), chunks 4 sub + jj of each lane: entry 4 r + jj
      const int n0 = 2 * (slot + S * (cur.j >> 1));
      const int sub = cur.j & 1;
      t.b[0] = t.b[1] = (const unsigned char*)Ly.dn_w;
      t.sb[0] = t.sb[1] = (const uint16_t*)Ly.dn_s;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const unsigned n = (unsigned)min(n0 + r, g.C - 1);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const unsigned ch = (unsigned)min(lane + 64 * (4 * sub + jj), g.ncI - 1);
          t.off[r * 4 + jj] = n * (unsigned)(g.I / 2) + ch * 16;
          t.soff[r * 4 + jj] = n * (unsigned)g.gI + (ch * 32) / (unsigned)g.grp;
        }
      }
      break;
    }
    case ATT: {  // 16 keys: lane (row group rg = lane / 16, 16-B column sub) reads keys kb + 4 jl + rg; entries 0-3 K, 4-7 V
      const int kb = x.sp.k_lo + KEYS * (x.w + NCW * cur.j);
      const int last = max(x.sp.k_end - 1, 0);
      t.b[0] = (const unsigned char*)Ly.k_cache;
      t.b[1] = (const unsigned char*)Ly.v_cache;
      t.sb[0] = t.sb[1] = (const uint16_t*)x.dummy;
#pragma unroll
      for (int jl = 0; jl < 4; ++jl) {
        const unsigned key = (unsigned)min(kb + 4 * jl + (lane >> 4), last);
        t.off[jl] = t.off[4 + jl] = ((unsigned)x.sp.grp * (unsigned)g.S + key) * (HS * 2) + (lane & 15) * 16;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) t.soff[i] = 0;
      break;
    }
    default: {  // padding past the schedule: a cached line
      t.b[0] = t.b[1] = (const unsigned char*)x.dummy;
      t.sb[0] = t.sb[1] = (const uint16_t*)x.dummy;
#pragma unroll
      for (int i = 0; i < 8; ++i) t.off[i] = t.soff[i] = 0;
      break;
    }
  }
}

__device__ __forceinline__ void issue(const Args& a, const Ctx& x, const Cur& cur, Tile& t) {
  TileAddr ad;
  addr_of(a, x, cur, ad);
  const gptr<const unsigned char> b0 = G(ad.b[0]), b1 = G(ad.b[1]);
  const gptr<const uint16_t> s0 = G(ad.sb[0]), s1 = G(ad.sb[1]);
#pragma unroll
  for (int i = 0; i < 8; ++i)
    t.w[i] = __builtin_nontemporal_load((const gptr<const u32x4>)((i < 4 ? b0 : b1) + ad.off[i]));
#pragma unroll
  for (int i = 0; i < 8; ++i) t.s[i] = (uint32_t)(i < 4 ? s0 : s1)[ad.soff[i]];
}

__device__ __forceinline__ uint4 u4(const u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }

__device__ __forceinline__ bool better(float v, int i, float bv, int bi) {
  const bool vn = v != v, bn = bv != bv;
  if (vn || bn) return vn && (!bn || i < bi);
  return (v > bv) || (v == bv && i < bi);
}

// per-wave state that lives across tiles
struct CwState {
  float part[2];            // down: the row pair's partial sums across its two sub-tiles
  float m, l, o[8];         // attention: online softmax of this wave's keys (q_per_kv 1)
  float qf[8];              // attention: this lane's 8 dims of the roped query
  float best_v;             // lm_head argmax candidate
  int best_i;
};

// consume tile cur: dot + butterfly + epilogue, exactly one store (dummy when the tile has no output)
__device__ __forceinline__ void consume(const Args& a, const Dyn& dy, const Ctx& x, const Lds& s, const Cur& cur,
                                        const Tile& t, CwState& st) {
  const Geo& g = a.g;
  const int lane = x.lane;
  const int S = NCW * g.P, slot = x.w * g.P + x.c;
  const int kind = kind_of(g, cur.k);
  const int l = cur.k / OPS;
  const uint32_t nmask = nibble_mask(), nmagic = f16_magic(), nmask_hi = nibble_mask_hi();
  const uint4* xl = (const uint4*)s.stage(cur.k);
  unsigned char* dst = a.scratch + g.o_dummy + ((size_t)x.c * NCW + x.w) * 64;
  uint64_t val = 0;
  bool st8 = false;
  switch (kind) {
    case QKV:
    case OPJ:
    case LM: {
      const float* xsum = (const float*)(s.stage(cur.k) + (size_t)g.C * 2);
      float part[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = lane + 64 * j;
        const bool ok = c < g.ncC;
        const int cc = min(c, g.ncC - 1);
        uint4 wj[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) wj[r] = u4(t.w[r * 2 + j]);
        float d[4];
        chunk_dot_rows<0, 4>(wj, xl + cc * 4, xsum[cc], nullptr, nmask, nmagic, nmask_hi, d);
#pragma unroll
        for (int r = 0; r < 4; ++r) part[r] = fmaf(ok ? scale_of<0>(t.s[r * 2 + j]) : 0.0f, d[r], part[r]);
      }
      if (kind == LM) {  // the per-op lm_head is the streaming RT = 2 form: two butterflies of 2 rows
        const int t4 = slot + S * cur.j;
        const float tot0 = butterfly<2>(part, lane), tot1 = butterfly<2>(part + 2, lane);
        const int vi = bfly_index<2>(lane);  // lanes 0-31: row 0 (2), lanes 32-63: row 1 (3)
        const uint16_t o0 = f2bf(tot0), o1 = f2bf(tot1);
        const uint32_t a0 = (uint32_t)__shfl((int)o0, 0), a1 = (uint32_t)__shfl((int)o0, 32);
        const uint32_t b0 = (uint32_t)__shfl((int)o1, 0), b1 = (uint32_t)__shfl((int)o1, 32);
        (void)vi;
        val = (uint64_t)(a0 | (a1 << 16)) | ((uint64_t)(b0 | (b1 << 16)) << 32);
        dst = (unsigned char*)(dy.logits + 4 * (size_t)t4);
        st8 = true;
        if (lane == 0) {
          const uint32_t ov[4] = {a0, a1, b0, b1};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = bf2f((uint16_t)ov[r]);
            const int idx = 4 * t4 + r;
            if (idx < g.V && better(v, idx, st.best_v, st.best_i)) {
              st.best_v = v;
              st.best_i = idx;
            }
          }
        }
      } else {
        const float tot = butterfly<4>(part, lane);
        const int vi = bfly_index<4>(lane);
        const int t4 = kind == QKV ? (x.sp.split + g.SP * x.w) + g.SP * NCW * cur.j : slot + S * cur.j;
        const int n0 = kind == QKV ? x.sp.grp * g.GQ + 4 * t4 : 4 * t4;
        float o = tot;
        if (kind == OPJ) o = round_bf(o) + bf2f(s.raw()[n0 + vi]);  // + x (Block residual, model.py:591)
        const uint32_t ob = f2bf(o);
        uint32_t ov[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) ov[r] = (uint32_t)__shfl((int)ob, r * 16);
        val = (uint64_t)(ov[0] | (ov[1] << 16)) | ((uint64_t)(ov[2] | (ov[3] << 16)) << 32);
        dst = (unsigned char*)(act(a, l) + (kind == QKV ? g.a_qkv : g.a_xp) + n0);
        st8 = true;
      }
      break;
    }
    case FC: {
      const float* xsum = (const float*)(s.stage(cur.k) + (size_t)g.C * 2);
      float part[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = lane + 64 * j;
        const bool ok = c < g.ncC;
        const int cc = min(c, g.ncC - 1);
        // value v = 2 r + m (row r, matrix m) is tile entry 4 m + 2 r + j
        uint4 wj[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) wj[v] = u4(t.w[4 * (v & 1) + 2 * (v >> 1) + j]);
        float d[4];
        chunk_dot_rows<0, 4>(wj, xl + cc * 4, xsum[cc], nullptr, nmask, nmagic, nmask_hi, d);
#pragma unroll
        for (int v = 0; v < 4; ++v)
          part[v] = fmaf(ok ? scale_of<0>(t.s[4 * (v & 1) + 2 * (v >> 1) + j]) : 0.0f, d[v], part[v]);
      }
      // the per-op fc_1 || fc_2 is the streaming RT = 1 dual form: one butterfly of (fc_1, fc_2) per row
      uint32_t gv[2];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const float tot = butterfly<2>(part + 2 * r, lane);
        const float other = __shfl_xor(tot, 32);
        const float gs = round_bf(silu_f(round_bf(tot)));  // silu(bf16(fc_1 x)) -> bf16, model.py:715
        gv[r] = (uint32_t)__shfl((int)f2bf(__fmul_rn(gs, round_bf(other))), 0);  // * bf16(fc_2 x); lane 0: fc_1
      }
      const int n0 = 2 * (slot + S * cur.j);
      val = gv[0] | (gv[1] << 16);
      dst = (unsigned char*)(act(a, l) + g.a_g + n0);
      break;
    }
    case DN: {
      const float* xsum = (const float*)(s.stage(cur.k) + (size_t)g.I * 2);
      const int sub = cur.j & 1;
      if (sub == 0) st.part[0] = st.part[1] = 0.0f;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int c = lane + 64 * (4 * sub + jj);
        const bool ok = c < g.ncI;
        const int cc = min(c, g.ncI - 1);
        uint4 wj[2] = {u4(t.w[jj]), u4(t.w[4 + jj])};
        float d[2];
        chunk_dot_rows<0, 2>(wj, xl + cc * 4, xsum[cc], nullptr, nmask, nmagic, nmask_hi, d);
#pragma unroll
        for (int r = 0; r < 2; ++r)
          st.part[r] = fmaf(ok ? scale_of<0>(t.s[r * 4 + jj]) : 0.0f, d[r], st.part[r]);
      }
      if (sub == 1) {
        float pp[2] = {st.part[0], st.part[1]};
        const float tot = butterfly<2>(pp, lane);
        const int vi = bfly_index<2>(lane);
        const int n0 = 2 * (slot + S * (cur.j >> 1));
        const float o = round_bf(tot) + bf2f(s.raw()[n0 + vi]);  // + residual (model.py:592)
        const uint32_t ob = f2bf(o);
        const uint32_t o0 = (uint32_t)__shfl((int)ob, 0), o1 = (uint32_t)__shfl((int)ob, 32);
        val = o0 | (o1 << 16);
        dst = (unsigned char*)(act(a, l) + g.a_x + n0);
      }
      break;
    }
    case ATT: {
      const int kb = x.sp.k_lo + KEYS * (x.w + NCW * cur.j) + (lane >> 4);
      float sc[4];
      float mx = st.m;
#pragma unroll
      for (int jl = 0; jl < 4; ++jl) {
        float kf[8];
        unpack8(u4(t.w[jl]), kf);
        float d = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) d = fmaf(st.qf[i], kf[i], d);
        const float sd = row_group_sum<16>(d) * g.scale;
        sc[jl] = (kb + 4 * jl < x.sp.k_end) ? sd : -INFINITY;
        mx = fmaxf(mx, sc[jl]);
      }
      const bool none = mx == -INFINITY;  // a row group whose keys are all masked so far
      const float cf = none ? 0.0f : expf(st.m - mx);
      st.l *= cf;
#pragma unroll
      for (int i = 0; i < 8; ++i) st.o[i] *= cf;
#pragma unroll
      for (int jl = 0; jl < 4; ++jl) {
        const float e = none ? 0.0f : expf(sc[jl] - mx);
        st.l += e;
        float vf[8];
        unpack8(u4(t.w[4 + jl]), vf);
#pragma unroll
        for (int i = 0; i < 8; ++i) st.o[i] = fmaf(e, vf[i], st.o[i]);
      }
      st.m = mx;
      break;
    }
  }
  // the outputs go to an LDS record the gather waves publish (a compute wave's own stores could only be drained
  // behind its in-flight tile loads: vmcnt is in order); lm_head logits (read by the host only) go out directly
  if (lane == 0 && kind != ATT && !(kind == DN && (cur.j & 1) == 0)) {
    if (kind == LM) {
      __hip_atomic_store((gptr<uint64_t>)G(dst), val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const int jr = kind == DN ? cur.j >> 1 : cur.j;
      const uint32_t eoff = (uint32_t)(((const uint16_t*)dst) - act(a, 0));
      *s.rec(cur.k, x.w, jr) = make_uint4(eoff, st8 ? 4u : 2u, (uint32_t)val, (uint32_t)(val >> 32));
    }
  }
}

// compute wave: op k is complete on this wave (all its stores drained): post to the CU; the CU's last wave
// arrives on the op's agent-scope counter
__device__ __forceinline__ void cw_signal(const Args& a, const Ctx& x, const Lds& s, const Ctl& ctl, int k, CwState& st) {
  const Geo& g = a.g;
  const int kind = kind_of(g, k), l = k / OPS, lane = x.lane;
  if (kind == ATT) {
    // merge the 4 row groups of the wave, post (m, l, o) for the gather waves' split merge
#pragma unroll
    for (int off = 16; off < 64; off <<= 1) {
      const float mo = __shfl_xor(st.m, off), lo = __shfl_xor(st.l, off);
      const float mn = fmaxf(st.m, mo);
      const float ca = mn == -INFINITY ? 0.0f : expf(st.m - mn);
      const float cb = mn == -INFINITY ? 0.0f : expf(mo - mn);
      st.l = st.l * ca + lo * cb;
#pragma unroll
      for (int i = 0; i < 8; ++i) st.o[i] = st.o[i] * ca + __shfl_xor(st.o[i], off) * cb;
      st.m = mn;
    }
    float* mine = s.amrg() + (size_t)x.w * (HS + 4);
    if (lane < 16) {
      if (lane == 0) {
        mine[0] = st.m;
        mine[1] = st.l;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) mine[4 + lane * 8 + i] = st.o[i];
    }
    st.m = -INFINITY;
    st.l = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) st.o[i] = 0.0f;
    if (lane == 0) lds_add(ctl.attc(), 1u);
  } else if (kind == LM) {
    if (lane == 0) {
      ctl.best(x.w)[0] = __float_as_uint(st.best_v);
      ctl.best(x.w)[1] = (unsigned)st.best_i;
    }
  }
  if (kind != ATT && kind != LM && lane == 0) {
    const int n = my_tiles(g, k, x.c, x.w, x.sp);
    *ctl.rcnt(k, x.w) = (unsigned)(kind == DN ? n / 2 : n);
  }
  // every op counts its compute waves in slot k % 4 (so slot k % 4 holds NCW per op k' <= k, k' = k mod 4)
  if (lane == 0) lds_add(ctl.arr(k), 1u);
  if (lane == 0) lds_st(ctl.prog(x.w), (unsigned)(k + 1));
  if (x.w == 0) E2TRACE(k, 7);
}

__device__ __forceinline__ void run_cw(const Args& a, const Dyn& dy, const Lds& s, const Ctl& ctl, const Clock& clk, int w,
                                       long p, int nops) {
  const Geo& g = a.g;
  Ctx x;
  x.c = blockIdx.x;
  x.w = w;
  x.lane = threadIdx.x & 63;
  x.p = p;
  x.sp = make_split(g, x.c, p);
  x.dummy = a.scratch + g.o_dummy + ((size_t)x.c * NCW + w) * 64 + 32;
  CwState st;
  st.m = -INFINITY;
  st.l = 0.0f;
#pragma unroll
  for (int i = 0; i < 8; ++i) st.o[i] = st.qf[i] = 0.0f;
  st.part[0] = st.part[1] = 0.0f;
  st.best_v = -INFINITY;
  st.best_i = 0x7FFFFFFF;
  auto first = [&](int k) {
    Cur c{k, 0, 0};
    while (c.k < nops && (c.n = my_tiles(g, c.k, x.c, w, x.sp)) == 0) ++c.k;
    return c;
  };
  auto next = [&](Cur c) {
    if (c.k >= nops) return c;
    if (++c.j < c.n) return c;
    return first(c.k + 1);
  };
  Cur cur = first(0);
  Cur nx = next(cur);
  Tile A, B;
  issue(a, x, cur, A);
  issue(a, x, nx, B);
  nx = next(nx);
  int done = 0;       // ops signalled
  bool aborted = false;
  // before consuming a tile of op cur.k: every earlier op of this wave is finished (its outputs are LDS records),
  // post them; then wait for op cur.k's input
  auto boundary = [&](const Cur& c) -> bool {
    for (; done < c.k; ++done) cw_signal(a, x, s, ctl, done, st);
    if (!lds_wait(a, ctl, clk, ctl.ready(), (unsigned)(c.k + 1), 8u)) return false;
    if (w == 0 && c.j == 0) E2TRACE(c.k, 6);
    if (kind_of(g, c.k) == ATT && c.j == 0) {  // the roped query, once per attention op
      unpack8(*(const uint4*)(s.qst() + (x.lane & 15) * 8), st.qf);
    }
    return true;
  };
  while (cur.k < nops) {
    if (!boundary(cur)) { aborted = true; break; }
    consume(a, dy, x, s, cur, A, st);
    issue(a, x, nx, A);
    nx = next(nx);
    cur = next(cur);
    if (cur.k >= nops) break;
    if (!boundary(cur)) { aborted = true; break; }
    consume(a, dy, x, s, cur, B, st);
    issue(a, x, nx, B);
    nx = next(nx);
    cur = next(cur);
  }
  drain();
  if (!aborted)
    for (; done < nops; ++done) cw_signal(a, x, s, ctl, done, st);
}

// ---- gather waves ----------------------------------------------------------------------------------------------
// sync of the 4 gather waves (monotonic LDS counter; every gather wave calls it the same number of times)
__device__ __forceinline__ bool gw_sync(const Args& a, const Ctl& ctl, const Clock& clk, unsigned& n) {
  ++n;
  if ((threadIdx.x & 63) == 0) lds_add(ctl.gws(), 1u);
  return lds_wait(a, ctl, clk, ctl.gws(), n * NGW, 16u);
}

// stage the op input x (K bf16 at src: sc1 loads when `handed`, plain otherwise) into stage[k & 1]: fused RMSNorm
// when normw, the raw copy for the residual when raw; gather wave gw plays wave gw of the per-op GEMV kernel
// (uint4 t, t + 256, ... with t = 64 gw + lane), so the norm's partial sums and tree are the per-op kernel's
template <int XI>
__device__ __forceinline__ bool stage_op(const Args& a, const Lds& s, const Ctl& ctl, const Clock& clk, unsigned& ns, int k,
                         const uint16_t* src, bool handed, int K, const uint16_t* normw, bool raw) {
  const int gw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int t = gw * 64 + lane;
  const int n8 = K / 8;
  uint4 xr[XI], nr[XI];
  const __amdgpu_buffer_rsrc_t rs = rsrc(src, K * 2);
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int u = min(t + 256 * i, n8 - 1);
    if (handed) xr[i] = ld_sc1_16(rs, (unsigned)u * 16);
    else xr[i] = gld16((const uint4*)src + u);
    if (normw) nr[i] = gld16((const uint4*)normw + u);
  }
  // the staging buffer of op k - 2 is free once every compute wave finished it
  for (int w = 0; w < NCW; ++w)
    if (!lds_wait(a, ctl, clk, ctl.prog(w), (unsigned)max(k - 1, 0), 32u)) return false;
  unsigned char* sb = s.stage(k);
  uint4* xl = (uint4*)sb;
  float* xsum = (float*)(sb + (size_t)K * 2);
  float rs_ = 1.0f;
  if (normw) {
    float ss = 0.0f;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
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
    if (lane == 0) ctl.red(k)[gw] = ss;
    if (!gw_sync(a, ctl, clk, ns)) return false;
    const float* r = ctl.red(k);
    rs_ = 1.0f / sqrtf(((r[0] + r[1]) + (r[2] + r[3])) / (float)K + a.g.eps);
  }
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int u = t + 256 * i;
    uint32_t d[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
    if (raw && u < n8) ((uint4*)s.raw())[u] = xr[i];
    if (normw) {
      const uint32_t nw[4] = {nr[i].x, nr[i].y, nr[i].z, nr[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        d[q] = pack2(__fmul_rn(bflo(nw[q]), __fmul_rn(bflo(d[q]), rs_)),
                     __fmul_rn(bfhi(nw[q]), __fmul_rn(bfhi(d[q]), rs_)));
    }
    uint4 xv;
    float cs = stage_x8<0>(d, xv);
    cs += __shfl_xor(cs, 1);
    cs += __shfl_xor(cs, 2);
    if (u < n8) {
      xl[u] = xv;
      if ((u & 3) == 0) xsum[u >> 2] = cs;
    }
  }
  if (!gw_sync(a, ctl, clk, ns)) return false;
  if (threadIdx.x == 0) lds_st(ctl.ready(), (unsigned)(k + 1));
  return true;
}

// attention of op k (layer l) on gather wave 0: q / k / v of the group, RoPE, KV append, release the compute
// waves; then merge their partials (+ the new key), publish the split, and the last split of the group combines
__device__ __forceinline__ bool gw_attention(const Args& a, const Lds& s, const Ctl& ctl, const Clock& clk, int k, long p,
                             unsigned epoch) {
  const Geo& g = a.g;
  const int l = k / OPS, lane = threadIdx.x & 63, sub = lane & 15;
  const Split sp = make_split(g, blockIdx.x, p);
  const lga_engine_layer* Lp = &a.layers[l];
  if (!poll_ctrs(a, ctl, clk, g.c_qkv + l * g.G + sp.grp, 1, 1, (epoch + 1) * (unsigned)g.SP, 64u)) return false;
  E2TRACE(k, 1);
  const uint16_t* row = act(a, l) + g.a_qkv + (size_t)sp.grp * g.GQ;
  const int h = min(lane >> 4, 2);  // q, k, v heads (q_per_kv 1)
  const uint4 raw = ld_sc1_16(rsrc(row, g.GQ * 2), (unsigned)((h * HS + sub * 8) * 2));
  const long rp = min(max(p, 0L), (long)g.rope_rows - 1);
  float cr[8], sr[8];  // this lane's 8 rope coefficients (registers; rope8 indexes them with constants)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    cr[i] = G(a.cos)[(size_t)rp * HS + sub * 8 + i];
    sr[i] = G(a.sin)[(size_t)rp * HS + sub * 8 + i];
  }
  const uint4 roped = rope8(raw, cr, sr, sub);
  if (lane < 48) {
    const uint4 val = h <= 1 ? roped : raw;  // q and k are roped, v is not
    *(uint4*)(s.qst() + (size_t)h * HS + sub * 8) = val;
    if (sp.owns_new && h >= 1) {  // KVCache.forward index_copy_ at input_pos (model.py:788-795)
      uint16_t* cache = (uint16_t*)(h == 1 ? Lp->k_cache : Lp->v_cache);
      gst16(cache + ((size_t)sp.grp * g.S + p) * HS + sub * 8, val);
    }
  }
  if (lane == 0) lds_st(ctl.ready(), (unsigned)(k + 1));
  // the compute waves' partials
  if (!lds_wait(a, ctl, clk, ctl.attc(), (unsigned)(NCW * (l + 1)), 128u)) return false;
  E2TRACE(k, 2);
  float* ws = (float*)(a.scratch + g.o_ws);
  const int head = sp.grp;  // q_per_kv 1: head == group
  float mx = -INFINITY;
  for (int w = 0; w < NCW; ++w) mx = fmaxf(mx, s.amrg()[(size_t)w * (HS + 4)]);
  float lt = 0.0f, ot[2] = {0.0f, 0.0f};
  for (int w = 0; w < NCW; ++w) {
    const float* src = s.amrg() + (size_t)w * (HS + 4);
    const float cf = mx == -INFINITY ? 0.0f : expf(src[0] - mx);
    lt += src[1] * cf;
    ot[0] += src[4 + lane] * cf;
    ot[1] += src[4 + 64 + lane] * cf;
  }
  if (sp.owns_new) {  // the key / value at input_pos, from the staged (roped) qkv row
    float kf[8], qh[8];
    unpack8(*(const uint4*)(s.qst() + (size_t)HS + sub * 8), kf);
    unpack8(*(const uint4*)(s.qst() + sub * 8), qh);
    float d = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) d = fmaf(qh[i], kf[i], d);
    const float sn = __shfl(row_group_sum<16>(d) * g.scale, 0);
    const float mn = fmaxf(mx, sn);
    const float cf = mx == -INFINITY ? 0.0f : expf(mx - mn);
    const float e = expf(sn - mn);
    lt = lt * cf + e;
    const uint16_t* vn = s.qst() + (size_t)2 * HS;
    ot[0] = fmaf(e, bf2f(vn[lane]), ot[0] * cf);
    ot[1] = fmaf(e, bf2f(vn[64 + lane]), ot[1] * cf);
    mx = mn;
  }
  float* wsr = ws + (((size_t)l * g.H + head) * g.SP + sp.split) * (HS + 4);
  st_sc1g(wsr + 4 + lane, ot[0]);
  st_sc1g(wsr + 4 + 64 + lane, ot[1]);
  if (lane == 0) {
    st_sc1g(wsr, mx);
    st_sc1g(wsr + 1, lt);
  }
  drain();
  unsigned old = 0;
  if (lane == 0) old = g_add(ctr(a, g.c_split + l * g.G + sp.grp), 1u);
  old = __shfl(old, 0);
  E2TRACE(k, 3);
  if (old - epoch * (unsigned)g.SP != (unsigned)(g.SP - 1)) return true;
  // the group's last split: flash-decoding merge of the SP splits in split order (rounds of 8)
  const float* base = ws + ((size_t)l * g.H + head) * g.SP * (HS + 4);
  mx = -INFINITY;
  lt = 0.0f;
  ot[0] = ot[1] = 0.0f;
  for (int s0 = 0; s0 < g.SP; s0 += 8) {
    float mv[8], lv[8], ov[8][2];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float* r = base + (size_t)min(s0 + u, g.SP - 1) * (HS + 4);
      mv[u] = ld_sc1g(r);
      lv[u] = ld_sc1g(r + 1);
      ov[u][0] = ld_sc1g(r + 4 + 2 * lane);
      ov[u][1] = ld_sc1g(r + 4 + 2 * lane + 1);
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
  uint16_t* y = act(a, l) + g.a_y + (size_t)head * HS;
  __hip_atomic_store(G((unsigned*)(y + 2 * lane)), pack2(ot[0] / lt, ot[1] / lt), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  drain();
  if (lane == 0) g_add_nr(ctr(a, g.c_y + l * NSH + sp.grp % NSH), 1u);
  E2TRACE(k, 4);
  return true;
}

// gather wave 0: once every compute wave finished GEMV op k, store the CU's outputs (the LDS records) write-through,
// drain, and arrive once on the op's agent-scope counter (MI355X_MICROARCH.md "Valid forms" row 1): this wave
// streams nothing, so the drain waits only for these stores
__device__ __forceinline__ bool gw_publish(const Args& a, const Lds& s, const Ctl& ctl, const Clock& clk, int k) {
  const Geo& g = a.g;
  const int kind = kind_of(g, k), l = k / OPS, lane = threadIdx.x & 63, c = blockIdx.x;
  if (!lds_wait(a, ctl, clk, ctl.arr(k), (unsigned)(NCW * (k / 4 + 1)), 4096u)) return false;
  const int w = lane / MAXJ, j = lane % MAXJ;
  if ((unsigned)j < lds_ld(ctl.rcnt(k, w))) {
    const uint4 r = *s.rec(k, w, j);
    uint16_t* dst = act(a, 0) + r.x;
    if (r.y == 4u)
      __hip_atomic_store((gptr<uint64_t>)G((uint64_t*)dst), (uint64_t)r.z | ((uint64_t)r.w << 32), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    else
      __hip_atomic_store((gptr<uint32_t>)G((uint32_t*)dst), r.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  drain();
  if (lane == 0) {
    int slot;
    switch (kind) {
      case QKV: slot = g.c_qkv + l * g.G + c % g.G; break;
      case OPJ: slot = g.c_xp + l * NSH + c % NSH; break;
      case FC: slot = g.c_g + l * NSH + c % NSH; break;
      default: slot = g.c_xo + l * NSH + c % NSH; break;
    }
    g_add_nr(ctr(a, slot), 1u);
  }
  return true;
}

// op k's input edge: gather wave 0 polls the counters, the other gather waves wait for its LDS word
__device__ __forceinline__ bool gw_edge(const Args& a, const Ctl& ctl, const Clock& clk, int k, int first, int n,
                                        unsigned target, unsigned code) {
  const int gw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (gw == 0) {
    if (!poll_ctrs(a, ctl, clk, first, n, 1, target, code)) return false;
    if ((threadIdx.x & 63) == 0) lds_st(ctl.edge(), (unsigned)(k + 1));
    return true;
  }
  return lds_wait(a, ctl, clk, ctl.edge(), (unsigned)(k + 1), code);
}

__device__ __forceinline__ void run_gw(const Args& a, const Dyn& dy, const Lds& s, const Ctl& ctl, const Clock& clk,
                                       long p, int nops, unsigned epoch) {
  const Geo& g = a.g;
  const int gw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int c = blockIdx.x;
  unsigned ns = 0;  // gather-wave syncs so far
  const unsigned all32 = (epoch + 1) * (unsigned)(g.P / NSH);  // an all-to-all shard's arrivals at this launch
  for (int k = 0; k < nops; ++k) {
    const int kind = kind_of(g, k), l = k / OPS;
    E2TRACE(k, 0);
    const lga_engine_layer* Lp = &a.layers[kind == LM ? 0 : l];
    bool ok = true;
    switch (kind) {
      case QKV:
      case LM: {
        const int li = kind == LM ? g.L : l;  // input = output of block li - 1 (or the embedding)
        const uint16_t* src = li == 0 ? (const uint16_t*)(a.scratch + g.o_x0) : act(a, li - 1) + g.a_x;
        if (li > 0) ok = gw_edge(a, ctl, clk, k, g.c_xo + (li - 1) * NSH, NSH, all32, 256u);
        E2TRACE(k, 1);
        if (ok)
          ok = stage_op<2>(a, s, ctl, clk, ns, k, src, li > 0, g.C,
                           kind == LM ? a.ln_f : (const uint16_t*)Lp->norm1, kind == QKV);
        if (ok && kind == QKV && gw == 0) ok = gw_publish(a, s, ctl, clk, k);
        break;
      }
      case ATT:
        if (gw == 0) ok = gw_attention(a, s, ctl, clk, k, p, epoch);
        break;
      case OPJ:
        ok = gw_edge(a, ctl, clk, k, g.c_y + l * NSH, NSH, (epoch + 1) * (unsigned)(g.G / NSH), 512u);
        E2TRACE(k, 1);
        if (ok) ok = stage_op<2>(a, s, ctl, clk, ns, k, act(a, l) + g.a_y, true, g.C, nullptr, false);
        if (ok && gw == 0) ok = gw_publish(a, s, ctl, clk, k);
        break;
      case FC:
        ok = gw_edge(a, ctl, clk, k, g.c_xp + l * NSH, NSH, all32, 1024u);
        E2TRACE(k, 1);
        if (ok)
          ok = stage_op<2>(a, s, ctl, clk, ns, k, act(a, l) + g.a_xp, true, g.C, (const uint16_t*)Lp->norm2, true);
        if (ok && gw == 0) ok = gw_publish(a, s, ctl, clk, k);
        break;
      default:  // DN
        ok = gw_edge(a, ctl, clk, k, g.c_g + l * NSH, NSH, all32, 2048u);
        E2TRACE(k, 1);
        if (ok) ok = stage_op<6>(a, s, ctl, clk, ns, k, act(a, l) + g.a_g, true, g.I, nullptr, false);
        if (ok && gw == 0) ok = gw_publish(a, s, ctl, clk, k);
        break;
    }
    E2TRACE(k, 5);
    if (!ok) {
      lds_st(ctl.abort(), 1u);
      return;
    }
  }
  if (nops <= g.L * OPS || gw != 0) return;
  // ---- lm_head argmax: the compute waves' candidates, one 64-bit atomic max per CU, the last CU finishes ----
  for (int w = 0; w < NCW; ++w)
    if (!lds_wait(a, ctl, clk, ctl.prog(w), (unsigned)nops, 4096u)) return;
  if (lane == 0) {
    float bv = -INFINITY;
    int bi = 0x7FFFFFFF;
    for (int w = 0; w < NCW; ++w) {
      const float v = __uint_as_float(lds_ld(ctl.best(w)));
      const int i = (int)lds_ld(ctl.best(w) + 1);
      if (better(v, i, bv, bi)) {
        bv = v;
        bi = i;
      }
    }
    // key: the value's total order in the high word (NaN highest, -0 == +0), the inverted index in the low one:
    // the max key is torch.argmax's answer (NaN wins, lowest index among equals)
    uint32_t u = bv == 0.0f ? 0u : __float_as_uint(bv);
    uint32_t ord = (bv != bv) ? 0xFFFFFFFFu : ((u & 0x80000000u) ? ~u : (u | 0x80000000u));
    const unsigned long long key = ((unsigned long long)ord << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)bi);
    const gptr<unsigned long long> kp = (gptr<unsigned long long>)ctr(a, g.c_key);
    (void)__hip_atomic_fetch_max(kp, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    drain();
    const int sh = c % NSH;
    const unsigned n_sh = (unsigned)(g.P / NSH);
    bool last = false;
    if (g_add(ctr(a, g.c_lm + sh), 1u) - epoch * n_sh == n_sh - 1)
      last = g_add(ctr(a, g.c_top), 1u) - epoch * NSH == NSH - 1;
    *ctl.last() = last ? 1u : 0u;
  }
  if (!__shfl((int)*ctl.last(), 0)) return;
  // the step's final arriver: token, input_pos, the next step's embedding, re-arm the key, advance the epoch
  const gptr<unsigned long long> kp = (gptr<unsigned long long>)ctr(a, g.c_key);
  const unsigned long long key = __hip_atomic_load(kp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int tok = (int)(0xFFFFFFFFu - (uint32_t)key);
  if (tok < 0 || tok >= g.V) tok = 0;
  const uint4* src = (const uint4*)(a.wte + (size_t)tok * g.C);
  uint4* dst = (uint4*)(a.scratch + g.o_x0);
  for (int i = lane; i < g.C / 8; i += 64) gst16(dst + i, gld16(src + i));
  if (lane == 0) {
    if (dy.token) *G(dy.token) = tok;
    if (dy.out_idx) *G(dy.out_idx) = tok;
    *G(dy.pos) += 1;
    __hip_atomic_store(kp, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ctr(a, 0), epoch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void __launch_bounds__(NT) engine2_kernel(const Args* __restrict__ ap, Dyn dy) {
  const Args& a = *ap;
  const Geo& g = a.g;
  Ctl ctl;
  Lds s{g.sb, g.C};
  if (threadIdx.x < 256) ctl.w()[threadIdx.x] = 0u;
  __syncthreads();
  if (g_ld(ctr(a, 2))) return;  // a previous launch gave up: the state needs lga_engine_reset
  const Clock clk{__builtin_amdgcn_s_memrealtime()};
  const long p = *G(dy.pos);
  const unsigned epoch = g_ld(ctr(a, 0));
  const int total = g.L * OPS + 1;
  const int nops = dy.op_limit > 0 ? min(dy.op_limit, total) : total;
  // the wave index as a provably wave-uniform value: every schedule decision derived from it is a scalar branch
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave < NGW) run_gw(a, dy, s, ctl, clk, p, nops, epoch);
  else run_cw(a, dy, s, ctl, clk, wave - NGW, p, nops);
}

}  // namespace e2
}  // namespace lga

#ifdef LGA_ENGINE_TRACE
extern "C" int lga_engine_trace_read(unsigned long long* host, long n) {
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(lga::e2::g_e2_trace), (size_t)n * sizeof(unsigned long long));
  void* dptr = nullptr;
  if (e == hipSuccess) e = hipGetSymbolAddress(&dptr, HIP_SYMBOL(lga::e2::g_e2_trace));
  if (e == hipSuccess) e = hipMemset(dptr, 0, sizeof(lga::e2::g_e2_trace));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}
#endif

// ---- C ABI (tools/lab/engine/engine.h; the same entry points as version 1) -----------------------------------------
namespace {

const char* unsupported(const lga_engine_geom* g, lga::e2::Geo& o) {
  using namespace lga::e2;
  if (!g) return "null geometry";
  if (g->fmt != 0) return "int4-g weights only (nf4 runs the per-op kernels)";
  if (g->head_size != HS) return "head_size must be 128";
  if (g->n_query_groups <= 0 || g->n_head % g->n_query_groups) return "n_head must be a multiple of n_query_groups";
  if (g->n_head != g->n_query_groups) return "q_per_kv must be 1";
  if (g->n_head * g->head_size != g->n_embd) return "n_head * head_size must equal n_embd";
  if (g->n_cu <= 0 || g->n_cu > 256 || g->n_cu % g->n_query_groups || g->n_cu % NSH)
    return "n_cu must be a multiple of n_query_groups and of 8, at most 256";
  if (g->n_query_groups % NSH) return "n_query_groups must be a multiple of 8";
  if (g->group < 32 || g->group & (g->group - 1) || g->n_embd % g->group || g->intermediate % g->group)
    return "group must be a power of two >= 32 dividing n_embd and intermediate_size";
  if (g->n_embd / 32 > 128 || g->n_embd / 32 <= 64) return "n_embd must be in (2048, 4096] (two chunks per lane)";
  if (g->intermediate / 32 > 512 || g->intermediate / 32 <= 256)
    return "intermediate_size must be in (8192, 16384] (eight chunks per lane over two sub-tiles)";
  if (g->n_embd % 8 || g->intermediate % 8 || g->vocab % 4) return "n_embd / intermediate % 8, vocab % 4";
  if (g->max_seq <= 0 || g->rope_rows <= 0 || g->n_layer <= 0 || g->vocab <= 0) return "empty geometry";
  if (!make_geo(*g, o)) return "bad geometry";
  if (o.QT % 1 || (o.GQ % 4)) return "qkv rows per group must be a multiple of 4";
  if (o.lds > 163840) return "LDS budget exceeded";
  {  // every compute wave's GEMV tiles of one op fit its MAXJ output records
    const int S = NCW * o.P;
    if ((o.I / 2 + S - 1) / S > MAXJ || (o.C / 4 + S - 1) / S > MAXJ || (o.C / 2 + S - 1) / S > MAXJ ||
        (o.QT + o.SP * NCW - 1) / (o.SP * NCW) > MAXJ)
      return "more GEMV tiles per compute wave than output records";
  }
  return nullptr;
}

}  // namespace

extern "C" int lga_engine_check(const lga_engine_geom* g) {
  lga::e2::Geo o;
  const char* why = unsupported(g, o);
  if (why) {
    lga_set_error(why);
    return (int)hipErrorInvalidValue;
  }
  return 0;
}

extern "C" size_t lga_engine_scratch_bytes(const lga_engine_geom* g) {
  lga::e2::Geo o;
  return unsupported(g, o) ? 0 : o.total;
}

extern "C" void* lga_engine_x0(const lga_engine_geom* g, void* scratch) {
  lga::e2::Geo o;
  if (!scratch || unsupported(g, o)) return nullptr;
  return (unsigned char*)scratch + o.o_x0;
}

extern "C" int lga_engine_reset(const lga_engine_geom* g, void* scratch, hipStream_t stream) {
  lga::e2::Geo o;
  const char* why = unsupported(g, o);
  LGA_CHECK_ARG(!why && scratch, "lga_engine_reset: unsupported geometry or null scratch");
  const hipError_t e =
      hipMemsetAsync((unsigned char*)scratch + lga::e2::kArgsBytes, 0, (size_t)o.n_ctr * lga::e2::CSW * 4, stream);
  if (e != hipSuccess) {
    lga_set_error(hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

extern "C" int lga_engine_error(const lga_engine_geom* g, const void* scratch, unsigned* err_out) {
  LGA_CHECK_ARG(scratch && err_out, "lga_engine_error: null pointer");
  (void)g;
  unsigned w = 0;
  const hipError_t e =
      hipMemcpy(&w, (const unsigned char*)scratch + lga::e2::kArgsBytes + lga::e2::CSW * 4, sizeof(unsigned),
                hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    lga_set_error(hipGetErrorString(e));
    return (int)e;
  }
  *err_out = w;
  return 0;
}

extern "C" int lga_decode_engine(const lga_engine_geom* g, const lga_engine_layer* layers, const void* lm_w,
                                 const void* lm_s, const void* ln_f, const void* wte, const float* cos,
                                 const float* sin, int64_t* pos, int32_t* token, int64_t* out_idx, void* logits,
                                 void* scratch, int op_limit, hipStream_t stream) {
  lga::e2::Geo o;
  const char* why = unsupported(g, o);
  if (why) {
    lga_set_error(why);
    return (int)hipErrorInvalidValue;
  }
  LGA_CHECK_ARG(layers && lm_w && lm_s && ln_f && wte && cos && sin && pos && logits && scratch,
                "lga_decode_engine: null pointer");
  LGA_CHECK_ARG(g->n_layer <= lga::e2::kMaxLayers, "lga_decode_engine: at most 64 layers");
  // the fixed arguments (geometry, pointers, and the layer table copied from the device array `layers`) are
  // written into the scratch when they differ from the last binding of this scratch (the first call: eager,
  // before any graph capture; a captured launch replays with the same bytes)
  struct Key {
    lga::e2::Geo g;
    const void *layers, *lm_w, *lm_s, *ln_f, *wte, *cos, *sin;
  } key;
  memset(&key, 0, sizeof(key));
  key.g = o;
  key.layers = layers;
  key.lm_w = lm_w;
  key.lm_s = lm_s;
  key.ln_f = ln_f;
  key.wte = wte;
  key.cos = cos;
  key.sin = sin;
  static std::unordered_map<void*, std::vector<unsigned char>> bound;
  std::vector<unsigned char>& last = bound[scratch];
  if (last.size() != sizeof(key) || memcmp(last.data(), &key, sizeof(key)) != 0) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(stream, &cs);
    LGA_CHECK_ARG(cs == hipStreamCaptureStatusNone, "lga_decode_engine: first launch of a binding inside a graph capture");
    static_assert(sizeof(lga::e2::Args) <= lga::e2::kArgsBytes, "Args block");
    lga::e2::Args* a = new lga::e2::Args;
    memset(a, 0, sizeof(*a));
    a->g = o;
    hipError_t e = hipMemcpy(a->layers, layers, sizeof(lga_engine_layer) * g->n_layer, hipMemcpyDeviceToHost);
    a->lm_w = (const uint8_t*)lm_w;
    a->lm_s = (const uint16_t*)lm_s;
    a->ln_f = (const uint16_t*)ln_f;
    a->wte = (const uint16_t*)wte;
    a->cos = cos;
    a->sin = sin;
    a->scratch = (unsigned char*)scratch;
    if (e == hipSuccess) e = hipMemcpyAsync(scratch, a, sizeof(*a), hipMemcpyHostToDevice, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    delete a;
    if (e != hipSuccess) {
      lga_set_error(hipGetErrorString(e));
      return (int)e;
    }
    last.assign((const unsigned char*)&key, (const unsigned char*)&key + sizeof(key));
  }
  lga::e2::Dyn dy{pos, token, out_idx, (uint16_t*)logits, op_limit};
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)lga::e2::engine2_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    if (e != hipSuccess) {
      lga_set_error(hipGetErrorString(e));
      return (int)e;
    }
    attr = true;
  }
  lga::e2::engine2_kernel<<<o.P, lga::e2::NT, o.lds, stream>>>((const lga::e2::Args*)scratch, dy);
  LGA_LAUNCH_RETURN();
}

// test hook: the scratch layout (bytes: x0, first layer's activations, bytes per layer; elements inside a layer's
// block: qkv, y (attention output), xp (after o_proj + residual), g (SwiGLU output), x (block output))
extern "C" int lga_engine_layout(const lga_engine_geom* g, long long* out) {
  lga::e2::Geo o;
  LGA_CHECK_ARG(out && !unsupported(g, o), "lga_engine_layout: unsupported geometry");
  const long long v[8] = {(long long)o.o_x0, (long long)o.o_act, (long long)o.act_len, o.a_qkv, o.a_y, o.a_xp, o.a_g,
                          o.a_x};
  for (int i = 0; i < 8; ++i) out[i] = v[i];
  return 0;
}
