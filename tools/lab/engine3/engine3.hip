// Persistent decode layer, version 3 (LAB, not the product): VERDICT r5 "Next round" item 1 — the layer as ONE
// launch on the recipe MI355X_MICROARCH.md prices as engine-vs-launches (0.87-0.89x of launches-baseline): per CU one
// LDS-DMA loader wave streaming the weights (and K/V rows) `nt` into an 8 x 17 KiB ring that runs ahead ACROSS op
// edges, consumer waves computing from the ring, and edges handed over through write-through stores + counters.
//
// What is new against engines v1 / v2 (profiles/r04a_engine_v1_trace.txt, r04d_engine_v2_trace.txt):
// their traces put 2.6-10 us per edge into waiting for the SLOWEST CU of the previous op, with every CU's share of
// every op fixed in advance. Here the units of an op are CLAIMED at run time (one claimer wave per CU, atomic heads
// sharded per XCD): a CU whose stream runs faster claims more, so an op ends within about one unit of the same time
// on every CU. The claim runs ahead of the loader (which runs ahead of the consumers) across op edges, so the next
// op's bytes are in the ring when its input arrives.
//
// Roles per workgroup (one per CU, 320 threads): wave 0 claims units, wave 1 loads them (LDS-DMA, nt, 3 fills in
// flight, thinned to 1 while the CU gathers), waves 2-4 consume units round robin from a descriptor ring. An op's
// input vector (the RMS-normalised layer input, the attention row, the post-attention row, the SwiGLU row) is
// gathered into LDS by whichever consumer first needs it once the previous op is complete chip-wide.
//
// Arithmetic: the GEMV units compute each output row as the fp32 sum over 32-element chunks of scale * dot(w, x)
// (x = the bf16 input as staged); the attention units run an fp32 online softmax over 32-key slots with the split
// merge of the per-op kernel (last-arriving split combines). This lab build measures TIME: its arithmetic is not the
// product's bit for bit, and it skips RoPE (the keys are appended un-rotated), so it is checked against torch
// references of the same math (tools/lab/engine3/e3_ab.py --check), not against the product.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

namespace e3 {

extern __shared__ __attribute__((aligned(16))) unsigned char e3_smem[];

#ifndef E3_NS
#define E3_NS 8
#define E3_SLOT 17408
#endif
#ifndef E3_NCONS
#define E3_NCONS 3
#endif
constexpr int NS = E3_NS;         // ring slots
constexpr int SLOT = E3_SLOT;     // bytes per slot
constexpr int NCONS = E3_NCONS;   // consumer waves
constexpr int NWAVE = 2 + NCONS;  // claimer, loader, consumers
constexpr int NT = NWAVE * 64;
constexpr int NDESC = 32;         // descriptor ring
constexpr int NCQ = 4;            // claim queue (entries the claimer may run ahead of the loader)
constexpr int NSH = 8;            // claim / done shards (one per XCD under round-robin placement)
constexpr int KEYS = SLOT >= 16384 ? 32 : 16;  // attention keys per slot (K rows, then V rows)
constexpr int HS = 128;
constexpr int MAXK = 11008;       // largest GEMV K: the input vector staged in LDS as bf16
constexpr int CW = 16;            // uint32 words per counter (64 B)
constexpr int NACC = 64;          // per-op accounting ring in LDS (the loader can run many small ops ahead)
constexpr unsigned FLAG = 1u << 24;
constexpr unsigned long long TMO = 200000000ull;  // 2 s of the 100 MHz clock: every wait is bounded

enum { OQ = 0, OA = 1, OP = 2, OF = 3, OD = 4 };

struct Layer {
  const uint8_t* wq; const uint16_t* sq;    // qkv [Nq][C/2], scales [Nq][C/gq]
  const uint8_t* wp; const uint16_t* sp;    // proj [C][Kp/2]
  const uint8_t* wf1; const uint16_t* sf1;  // fc_1 [I][C/2]
  const uint8_t* wf2; const uint16_t* sf2;  // fc_2
  const uint8_t* wd; const uint16_t* sd;    // down [C][I/2]
  uint16_t* kc; uint16_t* vc;               // [G][S][HS]
  const uint16_t* n1; const uint16_t* n2;   // RMSNorm weights [C]
};

struct Args {
  const Layer* layers;
  int L, C, H, G, I, Kp, S, splits;
  int gq, gp, gi;      // quantization groups for K = C, Kp, I
  int ru[5];           // rows per unit (GEMV ops; F: rows of fc_1, the same of fc_2)
  int units[5];        // units per op (A: G * splits)
  int Nq;
  const int64_t* pos;
  const uint16_t* x0;
  uint16_t* act;       // per layer: qkv [Nq], y [Kp], xp [C], g [I], xo [C]
  long long act_stride;
  int a_qkv, a_y, a_xp, a_g, a_xo;
  float* ws;           // attention partials [L][H][splits][HS + 4]
  unsigned* ctr;       // counters, zeroed before every launch
  unsigned* err;
  float eps, scale;
  int compute;         // bit 0: consumers compute (0: they only wait / release: the transport floor);
                       // bit 1: static unit ranges (each CU its contiguous 1/n of every op, no claim atomics)
  unsigned long long* trace;  // optional per-(op, CU) event times (TR_* below), 16 words each, after 256 start words
};

// trace events (s_memrealtime, 100 MHz), per (op, CU): claimer first claim / op exhausted, loader first / last fill
// issued, edge seen (previous op complete chip-wide), input staged, then per consumer its first unit start and its
// last unit end
enum { TR_CLAIM0 = 0, TR_CLAIM1, TR_LOAD0, TR_LOAD1, TR_EDGE, TR_STAGED, TR_START = 6, TR_END = 6 + NCONS, TR_N = 32 };
static_assert(TR_END + NCONS <= TR_N, "trace record");
__device__ __forceinline__ void tr(const Args& a, int op, int ev, int lane) {
  if (a.trace && lane == 0)
    a.trace[256 + ((size_t)op * gridDim.x + blockIdx.x) * TR_N + ev] = __builtin_amdgcn_s_memrealtime();
}

// counter layout (words of CW uint32): claim heads [5L][NSH], done [5L][NSH], attention arrivals [L][G]
__device__ __forceinline__ unsigned* claim_ctr(const Args& a, int op, int sh) { return a.ctr + ((size_t)op * NSH + sh) * CW; }
__device__ __forceinline__ unsigned* done_ctr(const Args& a, int op, int sh) {
  return a.ctr + ((size_t)5 * a.L * NSH + (size_t)op * NSH + sh) * CW;
}
__device__ __forceinline__ unsigned* arr_ctr(const Args& a, int layer, int g) {
  return a.ctr + ((size_t)10 * a.L * NSH + (size_t)layer * a.G + g) * CW;
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf(uint32_t h) { return __uint_as_float(h << 16); }
__device__ __forceinline__ float bflo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bfhi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }
__device__ __forceinline__ uint16_t f2bf(float f) {  // round to nearest even
  uint32_t u = __float_as_uint(f);
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, bytes, 0x00020000);
}
// write-through (sc1) stores and loads of hand-off data (MI355X_MICROARCH.md "Valid forms" row 1)
__device__ __forceinline__ void st16_wt(void* p, unsigned off, uint16_t v) {
  __builtin_amdgcn_raw_buffer_store_b16(v, rsrc(p, 0x7FFFFFFF), off, 0, 16);
}
__device__ __forceinline__ void st128_wt(void* p, unsigned off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(p, 0x7FFFFFFF), off, 0, 16);
}
__device__ __forceinline__ u32x4 ld128_wt(const void* p, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc(p, 0x7FFFFFFF), off, 0, 16);
}
__device__ __forceinline__ unsigned ld_ctr(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// the chip-wide completion counts: returning system-scope adds (polled from every XCD by ld_ctr); a no-return
// agent-scope add polled this way lost counts (round 6 lab: 477-492 of 512 seen, flushes all made)
__device__ __forceinline__ void add_done(unsigned* p, unsigned v) {
  const unsigned old = __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("" ::"v"(old));
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// LDS-DMA (inline asm: hipcc does not see these as LDS writes, so it inserts no vmcnt(0) before the loader's own
// LDS polls; the loader publishes a fill only after its explicit counted wait)
__device__ __forceinline__ void dma16(const void* src, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}
__device__ __forceinline__ void dma4(const void* src, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}
// s_waitcnt vmcnt(n) for a run-time n (the count is an instruction field): a scalar branch tree
__device__ __forceinline__ void wait_vm(int n) {
#define W(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (n < 0 ? 0 : (n > 63 ? 63 : n)) {
    W(0) W(1) W(2) W(3) W(4) W(5) W(6) W(7) W(8) W(9) W(10) W(11) W(12) W(13) W(14) W(15) W(16) W(17) W(18) W(19)
    W(20) W(21) W(22) W(23) W(24) W(25) W(26) W(27) W(28) W(29) W(30) W(31) W(32) W(33) W(34) W(35) W(36) W(37)
    W(38) W(39) W(40) W(41) W(42) W(43) W(44) W(45) W(46) W(47) W(48) W(49) W(50) W(51) W(52) W(53) W(54) W(55)
    W(56) W(57) W(58) W(59) W(60) W(61) W(62) W(63)
  }
#undef W
}

// ---- LDS map ----
struct Ctl {
  unsigned full[NS];         // fill index + 1 of the data in the slot
  unsigned freed[NS];        // fill index + 1 released by the consumer
  int desc[NDESC][4];        // {op, unit, first fill, fills}
  unsigned desc_seq;         // descriptors published
  int cq[NCQ][3];            // claim queue {op, first unit, units} (units = 0: op exhausted; op = -1: end)
  unsigned cq_push, cq_pop;
  unsigned acc_w[NACC];      // per-op finished-unit count | FLAG once the loader closed the op
  unsigned acc_n[NACC];      // units this CU claimed of the op (valid with FLAG)
  int staged_op;             // op whose input vector sits in xin
  int gather_op;             // op a consumer is gathering (lock)
  int gathering;             // the loader thins its stream while set
  int edge_ok;               // last op known complete chip-wide
  int ru[5], units[5];       // Args::ru / Args::units (indexed at run time)
  int cur_d[NCONS];          // diagnostics: the descriptor each consumer is on
};
constexpr int LDS_RING = 0;
constexpr int LDS_XIN = NS * SLOT;
constexpr int LDS_TOTAL = LDS_XIN + MAXK * 2;  // dynamic LDS: the ring and the staged input (Ctl is static LDS)
// Ctl as a static __shared__ object: every access to it is a DS instruction. Reached through a pointer into the
// dynamic area, hipcc emitted FLAT loads / stores for the volatile control words, which do not complete in order with
// the DS ones — a descriptor's fields could land after its sequence word (round 6 lab: units lost on 8 CUs).
__shared__ Ctl e3_ctl;
typedef __attribute__((address_space(3))) Ctl CtlL;
typedef __attribute__((address_space(3))) unsigned lu32;
typedef __attribute__((address_space(3))) int li32;
static_assert(LDS_TOTAL + sizeof(Ctl) <= 163840, "LDS budget");
// diagnostics on a timeout: the wave's record in err[64 + (cu * 8 + wave) * 32 ...]: code, three context values, then
// a snapshot of the CU's control words
__device__ __forceinline__ void dbg(const Args& a, const CtlL* c, unsigned code, int v0, int v1, int v2) {
  if ((threadIdx.x & 63) != 0) return;
  unsigned* r = a.err + 64 + ((size_t)blockIdx.x * 8 + (threadIdx.x >> 6)) * 128;
  const volatile CtlL* v = (const volatile CtlL*)c;
  r[0] = code; r[1] = (unsigned)v0; r[2] = (unsigned)v1; r[3] = (unsigned)v2;
  r[4] = (unsigned)v->staged_op; r[5] = (unsigned)v->gather_op; r[6] = (unsigned)v->edge_ok; r[7] = v->desc_seq;
  r[8] = v->cq_push; r[9] = v->cq_pop; r[10] = (unsigned)v->gathering;
  for (int i = 0; i < NS; ++i) { r[12 + i] = v->full[i]; r[20 + i] = v->freed[i]; }
  for (int i = 0; i < 8; ++i) { r[28 + i] = v->acc_w[i]; r[36 + i] = v->acc_n[i]; }
  for (int i = 0; i < NCONS && i < 4; ++i) r[44 + i] = (unsigned)v->cur_d[i];
  for (int i = 0; i < NDESC; ++i) { r[48 + i] = (unsigned)v->desc[i][0]; r[80 + i] = (unsigned)v->desc[i][1]; }
}
__device__ __forceinline__ unsigned vload(const lu32* p) {
  return __builtin_amdgcn_readfirstlane(*(const volatile lu32*)p);
}
__device__ __forceinline__ int vloadi(const li32* p) {
  return (int)__builtin_amdgcn_readfirstlane((unsigned)*(const volatile li32*)p);
}
__device__ __forceinline__ void lst(lu32* p, unsigned v) { *(volatile lu32*)p = v; }
__device__ __forceinline__ void lsti(li32* p, int v) { *(volatile li32*)p = v; }
__device__ __forceinline__ int ru_of(const Args&, int k) {
  return vloadi(&((CtlL*)&e3_ctl)->ru[k]);
}
__device__ __forceinline__ int units_of(const Args&, int k) {
  return vloadi(&((CtlL*)&e3_ctl)->units[k]);
}

// LDS control words are the same for every lane: read once, made wave-uniform (scalar registers), so control flow on
// them is scalar and nothing derived from them (layer pointers, offsets) turns into per-lane vector loads


__device__ __forceinline__ int op_kind(int op) { return op % 5; }
// per-kind fields from an LDS copy (a runtime index into the kernel-argument struct would copy the whole struct to
// scratch and turn every field read into a vector memory load)
__device__ __forceinline__ int ru_of(const Args&, int k);
__device__ __forceinline__ int units_of(const Args&, int k);

// units of op in shard sh: [U sh / NSH, U (sh + 1) / NSH)
__device__ __forceinline__ void shard_range(int U, int sh, int& b, int& e) {
  b = (int)((long)U * sh / NSH);
  e = (int)((long)U * (sh + 1) / NSH);
}

// attention unit (g, split): the cache keys [lo, min(hi, p)) stream through the ring; key p comes from the qkv row
__device__ __forceinline__ void split_range(const Args& a, long p, int s, int& lo, int& hi) {
  const int L = (int)min(p + 1, (long)a.S);
  const int chunk = (L + a.splits - 1) / a.splits;
  lo = min(s * chunk, L);
  hi = min(lo + chunk, L);
}

__device__ __forceinline__ int gemv_rows(const Args& a, int kind) { return kind == OQ ? a.Nq : (kind == OF ? a.I : a.C); }
__device__ __forceinline__ int gemv_k(const Args& a, int kind) { return kind == OP ? a.Kp : (kind == OD ? a.I : a.C); }
__device__ __forceinline__ int gemv_g(const Args& a, int kind) { return kind == OP ? a.gp : (kind == OD ? a.gi : a.gq); }

__device__ __forceinline__ int unit_fills(const Args& a, int op, int u, long p) {
  if (op_kind(op) != OA) return 1;
  int lo, hi;
  split_range(a, p, u % a.splits, lo, hi);
  const int ce = min(hi, (int)p);
  return ce > lo ? (ce - lo + KEYS - 1) / KEYS : 0;
}

// ---------------------------------------------------------------------------------------------------------------
// claimer (wave 0): walks the ops in order, claims units from its XCD's head, queues them for the loader
__device__ __forceinline__ void claimer(const Args& a, CtlL* c, int lane) {
  const int sh = blockIdx.x % NSH;
  const int nops = 5 * a.L;
  unsigned push = 0;
  const bool stat = (a.compute & 2) != 0;
  for (int op = 0; op < nops; ++op) {
    int b, e;
    tr(a, op, TR_CLAIM0, lane);
    if (stat) {
      const int U = units_of(a, op_kind(op));
      b = (int)((long)U * blockIdx.x / gridDim.x);
      e = (int)((long)U * (blockIdx.x + 1) / gridDim.x);
    } else {
      shard_range(units_of(a, op_kind(op)), sh, b, e);
    }
    bool once = false;
    while (true) {
      unsigned v = 0;
      if (stat) {
        v = once ? (unsigned)(e - b) : 0u;  // one record with the whole range, then the exhausted record
        once = true;
      } else {
        if (lane == 0 && b < e) v = __hip_atomic_fetch_add(claim_ctr(a, op, sh), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v = __builtin_amdgcn_readfirstlane(v);
      }
      const int u = b + (int)v;
      const bool last = b >= e || u >= e;
      // wait for a free queue entry
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while ((int)(push - vload(&c->cq_pop)) >= NCQ) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > TMO) { if (lane == 0) atomicOr(a.err, 1u); dbg(a, c, 1, op, push, u); return; }
      }
      if (lane == 0) {
        li32* q = c->cq[push % NCQ];
        q[0] = op;
        q[1] = last ? -1 : u;
        q[2] = last ? 0 : (stat ? e - b : 1);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      ++push;
      if (lane == 0) __hip_atomic_store(&c->cq_push, push, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (last) {
        tr(a, op, TR_CLAIM1, lane);
        break;
      }
    }
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while ((int)(push - vload(&c->cq_pop)) >= NCQ) {
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > TMO) { if (lane == 0) atomicOr(a.err, 1u); return; }
  }
  if (lane == 0) {
    li32* q = c->cq[push % NCQ];
    q[0] = -1;
    q[1] = -1;
    q[2] = 0;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  ++push;
  if (lane == 0) __hip_atomic_store(&c->cq_push, push, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ---------------------------------------------------------------------------------------------------------------
// loader (wave 1): for every claimed unit, a descriptor, then its fills by LDS-DMA

// DMA the bytes of one fill: chunk range A (16-B chunks) then dword range B, into slot base `lds`; returns
// the number of DMA instructions issued
__device__ __forceinline__ int dma_fill(const uint8_t* A, int nA16, const uint8_t* B, int nB4, unsigned lds, int lane) {
  int ins = 0;
  for (int i = 0; i < nA16; i += 64) {
    if (i + lane < nA16) dma16(A + (size_t)(i + lane) * 16, lds + (unsigned)i * 16);
    ++ins;
  }
  const unsigned bo = lds + (unsigned)((nA16 * 16 + 15) & ~15);
  for (int i = 0; i < nB4; i += 64) {
    if (i + lane < nB4) dma4(B + (size_t)(i + lane) * 4, bo + (unsigned)i * 4);
    ++ins;
  }
  return ins;
}

__device__ __forceinline__ void loader(const Args& a, CtlL* c, unsigned char* smem, int lane) {
  const long p = a.pos[0];
  const unsigned ring = (unsigned)(uintptr_t)(smem + LDS_RING);
  unsigned pop = 0, dseq = 0;
  int fill = 0;
  int nin = 0;  // fills in flight (issued, not yet published): their indices f0 < f1 < f2, DMA instruction counts n0..n2
  int f0 = 0, f1 = 0, f2 = 0, n1 = 0, n2 = 0;
  int cur_op = -1, claimed = 0;
  // the oldest fill in flight has landed once vmcnt <= the instructions issued after it (vmcnt retires in order)
  auto publish_oldest = [&]() {
    wait_vm(nin == 3 ? n1 + n2 : (nin == 2 ? n1 : 0));
    if (lane == 0) __hip_atomic_store(&c->full[f0 % NS], (unsigned)f0 + 1u, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
    f0 = f1;
    f1 = f2;
    n1 = n2;
    --nin;
  };
  while (true) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (vload(&c->cq_push) == pop) {
      if (nin > 0) publish_oldest();  // nothing to issue: publish what landed
      else __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > TMO) { if (lane == 0) atomicOr(a.err, 2u); dbg(a, c, 2, pop, fill, dseq); return; }
    }
    const li32* q = c->cq[pop % NCQ];
    const int op = vloadi(&q[0]), u0 = vloadi(&q[1]), n = vloadi(&q[2]);
    ++pop;
    if (lane == 0) __hip_atomic_store(&c->cq_pop, pop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (op != cur_op && op >= 0) {  // first claim record of a new op: open its accounting entry
      cur_op = op;
      claimed = 0;
      if (lane == 0) {
        c->acc_w[op % NACC] = 0;
        c->acc_n[op % NACC] = 0;
      }
      asm volatile("" ::: "memory");
    }
    if (op < 0 || n == 0) {  // op exhausted (or the end): close its accounting
      if (op >= 0 && op_kind(op) != OA) {
        unsigned old = 0;
        if (lane == 0) {
          c->acc_n[op % NACC] = (unsigned)claimed;
          // hipcc may sink a plain store below a relaxed atomic: a consumer seeing FLAG would read a stale count
          asm volatile("" ::: "memory");
          old = __hip_atomic_fetch_add(&c->acc_w[op % NACC], FLAG, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        old = __builtin_amdgcn_readfirstlane(old);
        if (old == (unsigned)claimed && claimed > 0 && lane == 0)  // every claimed unit already finished
          add_done(done_ctr(a, op, blockIdx.x % NSH), (unsigned)claimed);
      }
      if (op < 0) break;
      continue;
    }
    for (int u = u0; u < u0 + n; ++u) {
      const int kind = op_kind(op);
      const int nf = unit_fills(a, op, u, p);
      // descriptor (the consumer of dseq % NCONS); the slot ring bounds how far ahead descriptors can get
      if (lane == 0) {
        li32* d = c->desc[dseq % NDESC];
        d[0] = op;
        d[1] = u;
        d[2] = fill;
        d[3] = nf;
      }
      asm volatile("" ::: "memory");  // LDS writes of one wave complete in order: no fence (it would drain the DMAs)
      ++dseq;
      if (lane == 0) __hip_atomic_store(&c->desc_seq, dseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      ++claimed;
      for (int f = 0; f < nf; ++f) {
        // slot of this fill must have been released by the consumer of fill - NS
        const unsigned need = (unsigned)max(fill - NS + 1, 0);
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        while (vload(&c->freed[fill % NS]) < need) {
          if (nin > 0) publish_oldest();
          else __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t1 > TMO) { if (lane == 0) atomicOr(a.err, 4u); dbg(a, c, 4, fill, op, u); return; }
        }
        // keep at most 3 fills in flight (1 while a consumer of this CU gathers an op input)
        const int maxin = vloadi(&c->gathering) ? 1 : 3;
        while (nin >= maxin) publish_oldest();
        const unsigned slot = ring + (unsigned)((fill % NS) * SLOT);
        const Layer& ly = a.layers[op / 5];
        if (u == u0 && f == 0 && claimed == 1) tr(a, op, TR_LOAD0, lane);
        int ins;
        if (kind == OA) {
          const int g = u / a.splits;
          int lo, hi;
          split_range(a, p, u % a.splits, lo, hi);
          const int k0 = lo + f * KEYS, nk = min(KEYS, min(hi, (int)p) - k0);
          const uint8_t* kr = (const uint8_t*)(ly.kc + ((size_t)g * a.S + k0) * HS);
          const uint8_t* vr = (const uint8_t*)(ly.vc + ((size_t)g * a.S + k0) * HS);
          ins = dma_fill(kr, nk * HS * 2 / 16, nullptr, 0, slot, lane);
          ins += dma_fill(vr, nk * HS * 2 / 16, nullptr, 0, slot + KEYS * HS * 2, lane);
        } else {
          const int N = gemv_rows(a, kind), K = gemv_k(a, kind), G = gemv_g(a, kind), R = ru_of(a, kind);
          const int r0 = u * R, nr = min(R, N - r0);
          const uint8_t* W = kind == OQ ? ly.wq : kind == OP ? ly.wp : kind == OF ? ly.wf1 : ly.wd;
          const uint16_t* Sc = kind == OQ ? ly.sq : kind == OP ? ly.sp : kind == OF ? ly.sf1 : ly.sd;
          const int wb = nr * K / 2, sb = nr * (K / G) * 2;
          if (kind == OF) {  // fc_1 rows, fc_2 rows, then both scale blocks (slot offsets as if nr == R)
            const int wbR = R * K / 2, sbR = R * (K / G) * 2;
            ins = dma_fill(W + (size_t)r0 * K / 2, wb / 16, nullptr, 0, slot, lane);
            ins += dma_fill(ly.wf2 + (size_t)r0 * K / 2, wb / 16, nullptr, 0, slot + wbR, lane);
            ins += dma_fill(nullptr, 0, (const uint8_t*)(Sc + (size_t)r0 * (K / G)), sb / 4, slot + 2 * wbR, lane);
            ins += dma_fill(nullptr, 0, (const uint8_t*)(ly.sf2 + (size_t)r0 * (K / G)), sb / 4,
                            slot + 2 * wbR + sbR, lane);
          } else {
            ins = dma_fill(W + (size_t)r0 * K / 2, wb / 16, nullptr, 0, slot, lane);
            ins += dma_fill(nullptr, 0, (const uint8_t*)(Sc + (size_t)r0 * (K / G)), sb / 4,
                            slot + (unsigned)(R * K / 2), lane);
          }
        }
        ins = __builtin_amdgcn_readfirstlane(ins);
        if (nin == 0) f0 = fill;
        else if (nin == 1) { f1 = fill; n1 = ins; }
        else { f2 = fill; n2 = ins; }
        ++nin;
        ++fill;
        tr(a, op, TR_LOAD1, lane);
      }
    }
  }
  while (nin > 0) publish_oldest();
  // one end descriptor per consumer
  for (int k = 0; k < NCONS; ++k) {
    if (lane == 0) {
      li32* d = c->desc[dseq % NDESC];
      d[0] = -1;
      d[1] = d[2] = d[3] = 0;
    }
    asm volatile("" ::: "memory");
    ++dseq;
    if (lane == 0) __hip_atomic_store(&c->desc_seq, dseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// ---------------------------------------------------------------------------------------------------------------
// consumers (waves 2..4)

// chip-wide completion of op (its done counters reach the op's total)
__device__ __forceinline__ bool wait_done(const Args& a, CtlL* c, int op, int lane) {
  if (op < 0 || vloadi(&c->edge_ok) >= op) return true;
  const unsigned total = op_kind(op) == OA ? (unsigned)a.G : (unsigned)units_of(a, op_kind(op));
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (true) {
    unsigned v = lane < NSH ? ld_ctr(done_ctr(a, op, lane)) : 0u;
#pragma unroll
    for (int o = 4; o > 0; o >>= 1) v += __shfl_xor(v, o);
    v = __builtin_amdgcn_readfirstlane(v);
    if (v >= total) break;
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_s_memrealtime() - t0 > TMO) {
      if (lane == 0) atomicOr(a.err, 8u);
      dbg(a, c, 8, op, (int)v, (int)total);
      return false;
    }
  }
  int was = 0;
  if (lane == 0) was = __hip_atomic_fetch_max(&c->edge_ok, op, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  was = __builtin_amdgcn_readfirstlane(was);
  if (was < op && op + 1 < 5 * a.L) tr(a, op + 1, TR_EDGE, lane);
  return true;
}

// the input vector of a GEMV op into LDS (bf16), RMS-normalised for the qkv and fc ops
__device__ __forceinline__ void gather(const Args& a, CtlL* c, unsigned char* smem, int op, int lane) {
  const int kind = op_kind(op), layer = op / 5;
  const uint16_t* src;
  const uint16_t* nw = nullptr;
  int K;
  uint16_t* act = a.act + (size_t)layer * a.act_stride;
  if (kind == OQ) {
    src = layer == 0 ? a.x0 : a.act + (size_t)(layer - 1) * a.act_stride + a.a_xo;
    nw = a.layers[layer].n1;
    K = a.C;
  } else if (kind == OP) {
    src = act + a.a_y;
    K = a.Kp;
  } else if (kind == OF) {
    src = act + a.a_xp;
    nw = a.layers[layer].n2;
    K = a.C;
  } else {
    src = act + a.a_g;
    K = a.I;
  }
  uint16_t* xin = (uint16_t*)(smem + LDS_XIN);
  const int n8 = K / 8;
  // sum of squares first pass (loads issued in groups of 8 per lane)
  float ss = 0.0f;
  for (int i0 = 0; i0 < n8; i0 += 64 * 8) {
    u32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = min(i0 + k * 64 + lane, n8 - 1);
      v[k] = ld128_wt(src, (unsigned)i * 16);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = i0 + k * 64 + lane;
      if (i < n8) {
        uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
        if (nw) {
#pragma unroll
          for (int q = 0; q < 4; ++q) ss = fmaf(bflo(w[q]), bflo(w[q]), fmaf(bfhi(w[q]), bfhi(w[q]), ss));
        }
        *(u32x4*)(xin + (size_t)i * 8) = v[k];
      }
    }
  }
  if (nw) {
    ss = wave_sum(ss);
    const float rs = 1.0f / sqrtf(ss / (float)K + a.eps);
    for (int i = lane; i < n8; i += 64) {
      u32x4 v = *(u32x4*)(xin + (size_t)i * 8);
      const u32x4 wv = *(const u32x4*)(nw + (size_t)i * 8);
      uint32_t w[4] = {v.x, v.y, v.z, v.w}, g[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        w[q] = (uint32_t)f2bf(bflo(g[q]) * (bflo(w[q]) * rs)) | ((uint32_t)f2bf(bfhi(g[q]) * (bfhi(w[q]) * rs)) << 16);
      *(u32x4*)(xin + (size_t)i * 8) = u32x4{w[0], w[1], w[2], w[3]};
    }
  }
}

// make the input of op available in LDS (returns false on a timeout)
__device__ __forceinline__ bool ensure_input(const Args& a, CtlL* c, unsigned char* smem, int op, int lane) {
  const int kind = op_kind(op);
  if (kind == OA) return wait_done(a, c, op - 1, lane);  // q / k / v rows: read per unit
  if (vloadi(&c->staged_op) == op) return true;
  // every consumer that needs op waits for the previous op chip-wide BEFORE it competes for the gather lock: a
  // consumer that took the lock for op + 1 and then waited would block this CU's consumer of op, whose input then is
  // never staged (round 6 lab: the lock went 5 -> 8 past a CU's only P unit, and op 7 never completed)
  if (!wait_done(a, c, op - 1, lane)) return false;
  int got = 0;
  if (lane == 0) {
    const int prev = vloadi(&c->gather_op);
    int expect = prev;
    got = prev < op && __hip_atomic_compare_exchange_strong(&c->gather_op, &expect, op, __ATOMIC_RELAXED,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  got = __builtin_amdgcn_readfirstlane(got);
  if (got) {
    if (lane == 0) lsti(&c->gathering, 1);
    gather(a, c, smem, op, lane);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) {
      lsti(&c->gathering, 0);
      __hip_atomic_store(&c->staged_op, op, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    tr(a, op, TR_STAGED, lane);
    return true;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (vloadi(&c->staged_op) < op) {
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > TMO) {
      if (lane == 0) atomicOr(a.err, 16u);
      dbg(a, c, 16, op, vloadi(&c->staged_op), 0);
      return false;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return true;
}

__device__ __forceinline__ bool wait_full(const CtlL* c, int fill, const Args& a, int lane) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (vload(&c->full[fill % NS]) < (unsigned)fill + 1u) {
    __builtin_amdgcn_s_sleep(0);
    if (__builtin_amdgcn_s_memrealtime() - t0 > TMO) {
      if (lane == 0) atomicOr(a.err, 32u);
      dbg(a, c, 32, fill, (int)vload(&c->full[fill % NS]), 0);
      return false;
    }
  }
  asm volatile("" ::: "memory");  // no slot read may move above the poll
  return true;
}
__device__ __forceinline__ void release(CtlL* c, int fill, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every LDS read of the slot has returned
  if (lane == 0) __hip_atomic_store(&c->freed[fill % NS], (unsigned)fill + 1u, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_WORKGROUP);
}

// n finished units of a GEMV op (their stores drained): this CU's count; the last of the CU's claimed units adds
// them chip-wide
__device__ __forceinline__ void account(const Args& a, CtlL* c, int op, int lane, unsigned n = 1) {
  unsigned old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(&c->acc_w[op % NACC], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  old = __builtin_amdgcn_readfirstlane(old);
  if ((old & FLAG) && (old & (FLAG - 1)) + n == vload(&c->acc_n[op % NACC]) && lane == 0)
    add_done(done_ctr(a, op, blockIdx.x % NSH), vload(&c->acc_n[op % NACC]));
}

// 32 weights (16 B, byte j = elements 2j | 2j+1 << 4) . 32 x (bf16 in LDS) with the nibble offset 8 folded in
__device__ __forceinline__ float chunk_dot(const u32x4 w, const float (&xf)[32], float xsum) {
  const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
  float d = 0.0f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t lo = ww[q] & 0x0F0F0F0Fu, hi = (ww[q] >> 4) & 0x0F0F0F0Fu;
    d = fmaf((float)((lo >> 0) & 0xFFu), xf[8 * q + 0], d);
    d = fmaf((float)((hi >> 0) & 0xFFu), xf[8 * q + 1], d);
    d = fmaf((float)((lo >> 8) & 0xFFu), xf[8 * q + 2], d);
    d = fmaf((float)((hi >> 8) & 0xFFu), xf[8 * q + 3], d);
    d = fmaf((float)((lo >> 16) & 0xFFu), xf[8 * q + 4], d);
    d = fmaf((float)((hi >> 16) & 0xFFu), xf[8 * q + 5], d);
    d = fmaf((float)((lo >> 24) & 0xFFu), xf[8 * q + 6], d);
    d = fmaf((float)((hi >> 24) & 0xFFu), xf[8 * q + 7], d);
  }
  return fmaf(-8.0f, xsum, d);
}

__device__ __forceinline__ void gemv_unit(const Args& a, unsigned char* smem, int op, int u, int fill, int lane) {
  const int kind = op_kind(op), layer = op / 5;
  const int N = gemv_rows(a, kind), K = gemv_k(a, kind), G = gemv_g(a, kind), R = ru_of(a, kind);
  const int r0 = u * R, nr = min(R, N - r0);
  const int NC = K / 32, gpr = K / G;
  const unsigned char* slot = smem + LDS_RING + (fill % NS) * SLOT;
  const uint16_t* xin = (const uint16_t*)(smem + LDS_XIN);
  const bool dual = kind == OF;
  const int nv = dual ? 2 * R : R;  // values: rows (dual: fc_1 rows, then fc_2 rows)
  const unsigned char* sc0 = slot + (dual ? 2 : 1) * R * K / 2;
  uint16_t* act = a.act + (size_t)layer * a.act_stride;
  uint16_t* out = kind == OQ ? act + a.a_qkv : kind == OP ? act + a.a_xp : kind == OF ? act + a.a_g : act + a.a_xo;
  const uint16_t* res = kind == OP ? (layer == 0 ? a.x0 : a.act + (size_t)(layer - 1) * a.act_stride + a.a_xo)
                                   : (kind == OD ? act + a.a_xp : nullptr);
  // the residual row is issued before the dot loop so its latency hides under the arithmetic
  u32x4 rv = {0u, 0u, 0u, 0u};
  if (res && lane < nr) rv = ld128_wt(res, (unsigned)((r0 + lane) & ~7) * 2);
  const int gsh = __builtin_ctz((unsigned)G);
  float part[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) part[i] = 0.0f;
  for (int cc = lane; cc < NC; cc += 64) {
    float xf[32];
    float xs = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32x4 v = *(const u32x4*)(xin + (size_t)cc * 32 + k * 8);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        xf[8 * k + 2 * q] = bflo(w[q]);
        xf[8 * k + 2 * q + 1] = bfhi(w[q]);
        xs += xf[8 * k + 2 * q] + xf[8 * k + 2 * q + 1];
      }
    }
    const int g = (cc * 32) >> gsh;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i < nv && (i >= R ? i - R : i) < nr) {
        const u32x4 w = *(const u32x4*)(slot + (size_t)i * (K / 2) + cc * 16);
        const uint16_t sb = *(const uint16_t*)(sc0 + ((size_t)i * gpr + g) * 2);
        part[i] = fmaf(bf(sb), chunk_dot(w, xf, xs), part[i]);
      }
    }
  }
  float tot[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) tot[i] = i < nv ? wave_sum(part[i]) : 0.0f;
  // lane r stores row r (residual read write-through: produced by other CUs)
  if (lane < nr) {
    float v = 0.0f, v2 = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i == lane) v = tot[i];
      if (dual && i == lane + R) v2 = tot[i];
    }
    float o;
    if (dual) {
      const float a1 = bf(f2bf(v));
      o = bf(f2bf(a1 / (1.0f + __expf(-a1)))) * bf(f2bf(v2));
    } else {
      o = v;
      if (res) {
        const uint32_t rw[4] = {rv.x, rv.y, rv.z, rv.w};
        const int e = (r0 + lane) & 7;
        const uint32_t h = (e & 1) ? (rw[e >> 1] >> 16) : (rw[e >> 1] & 0xFFFFu);
        o = bf(f2bf(o)) + bf(h);
      }
    }
    st16_wt(out, (unsigned)(r0 + lane) * 2, f2bf(o));
  }
}

// attention unit (query group g, split s): online softmax over the split's cache keys in the ring, the new key p
// from the qkv row, then the publish / last-arriver combine of the per-op kernel
__device__ __forceinline__ void attn_unit(const Args& a, unsigned char* smem, int op, int u, int fill0, int nf, int lane) {
  const int layer = op / 5, g = u / a.splits, s = u % a.splits;
  constexpr int QPK = 1;  // lab build: one query head per group (Llama-2-7B and its TP ranks); the host checks
  const long p = a.pos[0];
  int lo, hi;
  split_range(a, p, s, lo, hi);
  const Layer& ly = a.layers[layer];
  uint16_t* act = a.act + (size_t)layer * a.act_stride;
  const uint16_t* qkv = act + a.a_qkv + (size_t)g * (QPK + 2) * HS;
  const float sl2 = a.scale * 1.4426950408889634f;
  const int key = lane >> 1, half = lane & 1;
  float m[4], l[4], o0[4], o1[4];
  uint32_t q[4][32];  // this lane's half (64 dims) of each head's q, bf16 pairs
  for (int h = 0; h < QPK; ++h) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const u32x4 v = ld128_wt(qkv, (unsigned)((h * HS + half * 64 + k * 8) * 2));
      q[h][4 * k] = v.x;
      q[h][4 * k + 1] = v.y;
      q[h][4 * k + 2] = v.z;
      q[h][4 * k + 3] = v.w;
    }
    m[h] = -1e30f;
    l[h] = 0.0f;
    o0[h] = o1[h] = 0.0f;
  }
  typedef short s2 __attribute__((ext_vector_type(2)));
  auto step = [&](const unsigned char* kb, const unsigned char* vb, int nk) {
    for (int h = 0; h < QPK; ++h) {
      float d = 0.0f;
      const unsigned char* kr = kb + (size_t)key * HS * 2 + half * 128;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const u32x4 kv = *(const u32x4*)(kr + k * 16);
        d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(s2, q[h][4 * k]), __builtin_bit_cast(s2, kv.x), d, false);
        d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(s2, q[h][4 * k + 1]), __builtin_bit_cast(s2, kv.y), d, false);
        d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(s2, q[h][4 * k + 2]), __builtin_bit_cast(s2, kv.z), d, false);
        d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(s2, q[h][4 * k + 3]), __builtin_bit_cast(s2, kv.w), d, false);
      }
      d += __shfl_xor(d, 1);
      const float sc = key < nk ? d * sl2 : -INFINITY;
      const float mx = fmaxf(m[h], wave_max(sc));
      const float e = __builtin_amdgcn_exp2f(sc - mx);
      const float cf = __builtin_amdgcn_exp2f(m[h] - mx);
      l[h] = l[h] * cf + wave_sum(e) * 0.5f;  // each key's score sits in two lanes
      o0[h] *= cf;
      o1[h] *= cf;
      for (int k = 0; k < nk; ++k) {
        const float ek = __shfl(e, 2 * k);
        const uint32_t vv = *(const uint32_t*)(vb + (size_t)k * HS * 2 + lane * 4);
        o0[h] = fmaf(ek, bflo(vv), o0[h]);
        o1[h] = fmaf(ek, bfhi(vv), o1[h]);
      }
      m[h] = mx;
    }
  };
  for (int f = 0; f < nf; ++f) {
    const int fill = fill0 + f;
    CtlL* c = (CtlL*)&e3_ctl;
    if (!wait_full(c, fill, a, lane)) return;
    const unsigned char* slot = smem + LDS_RING + (fill % NS) * SLOT;
    const int nk = min(KEYS, min(hi, (int)p) - (lo + f * KEYS));
    if (a.compute & 1) step(slot, slot + KEYS * HS * 2, nk);
    release(c, fill, lane);
  }
  if (lo <= p && p < hi) {  // the new key: appended to the cache (un-rotated in this lab build) and scored
    const uint16_t* kn = qkv + QPK * HS;
    const uint16_t* vn = kn + HS;
    if (lane < 16) {
      const u32x4 kv = ld128_wt(kn, (unsigned)lane * 16), vv = ld128_wt(vn, (unsigned)lane * 16);
      *(u32x4*)(ly.kc + ((size_t)g * a.S + p) * HS + lane * 8) = kv;
      *(u32x4*)(ly.vc + ((size_t)g * a.S + p) * HS + lane * 8) = vv;
    }
    if (a.compute & 1) {
      for (int h = 0; h < QPK; ++h) {
        float d = 0.0f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const u32x4 kv = ld128_wt(kn, (unsigned)((half * 64 + k * 8) * 2));
          d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(s2, q[h][4 * k]), __builtin_bit_cast(s2, kv.x), d, false);
          d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(s2, q[h][4 * k + 1]), __builtin_bit_cast(s2, kv.y), d, false);
          d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(s2, q[h][4 * k + 2]), __builtin_bit_cast(s2, kv.z), d, false);
          d = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(s2, q[h][4 * k + 3]), __builtin_bit_cast(s2, kv.w), d, false);
        }
        d += __shfl_xor(d, 1);
        const float sc = d * sl2;
        const float mx = fmaxf(m[h], sc);
        const float cf = __builtin_amdgcn_exp2f(m[h] - mx), e = __builtin_amdgcn_exp2f(sc - mx);
        const uint32_t vp = __builtin_amdgcn_raw_buffer_load_b32(rsrc(vn, 0x7FFFFFFF), (unsigned)lane * 4, 0, 16);
        l[h] = l[h] * cf + e;
        o0[h] = fmaf(e, bflo(vp), o0[h] * cf);
        o1[h] = fmaf(e, bfhi(vp), o1[h] * cf);
        m[h] = mx;
      }
    }
  }
  // publish this split's (m, l, o) per head: [layer][head][split][HS + 4]
  float* wsl = a.ws + (size_t)layer * a.H * a.splits * (HS + 4);
  for (int h = 0; h < QPK; ++h) {
    float* pr = wsl + ((size_t)(g * QPK + h) * a.splits + s) * (HS + 4);
    const uint32_t oo[2] = {__float_as_uint(o0[h]), __float_as_uint(o1[h])};
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, oo),
                                          rsrc(pr, 0x7FFFFFFF), 16 + lane * 8, 0, 16);
    if (lane == 0) {
      const u32x4 ml = {__float_as_uint(m[h]), __float_as_uint(l[h]), 0u, 0u};
      st128_wt(pr, 0, ml);
    }
  }
  drain();
  unsigned t = 0;
  if (lane == 0) t = __hip_atomic_fetch_add(arr_ctr(a, layer, g), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  t = __builtin_amdgcn_readfirstlane(t);
  if (t != (unsigned)(a.splits - 1)) return;
  // the last split of the group: merge every split (lane owns dims 2 lane, 2 lane + 1) and hand y over
  for (int h = 0; h < QPK; ++h) {
    const float* base = wsl + (size_t)(g * QPK + h) * a.splits * (HS + 4);
    float mx = -INFINITY;
    for (int k = 0; k < a.splits; ++k) {
      const u32x4 ml = ld128_wt(base + (size_t)k * (HS + 4), 0);
      mx = fmaxf(mx, __uint_as_float(ml.x));
    }
    float lt = 0.0f, a0 = 0.0f, a1 = 0.0f;
    for (int k = 0; k < a.splits; ++k) {
      const float* pr = base + (size_t)k * (HS + 4);
      const u32x4 ml = ld128_wt(pr, 0);
      const auto ov = __builtin_amdgcn_raw_buffer_load_b64(rsrc(pr, 0x7FFFFFFF), 16 + lane * 8, 0, 16);
      const float e = __builtin_amdgcn_exp2f(__uint_as_float(ml.x) - mx);
      lt = fmaf(__uint_as_float(ml.y), e, lt);
      a0 = fmaf(__uint_as_float(ov[0]), e, a0);
      a1 = fmaf(__uint_as_float(ov[1]), e, a1);
    }
    const uint32_t yv = (uint32_t)f2bf(a0 / lt) | ((uint32_t)f2bf(a1 / lt) << 16);
    __builtin_amdgcn_raw_buffer_store_b32(yv, rsrc(act + a.a_y, 0x7FFFFFFF),
                                          (unsigned)(((g * QPK + h) * HS + 2 * lane) * 2), 0, 16);
  }
  drain();
  if (lane == 0) add_done(done_ctr(a, op, 0), 1u);
}

__device__ __forceinline__ void consumer(const Args& a, CtlL* c, unsigned char* smem, int ci, int lane) {
  int last_op = -1;
  // units whose output stores are issued but not yet drained / counted (all of op pend): counted in one drain when
  // the consumer moves to another op or would wait for a descriptor (a wait with uncounted units could deadlock:
  // the loader may need the op complete before it can issue the next descriptor)
  int pend = -1;
  unsigned npend = 0;
  auto flush = [&]() {
    if (pend >= 0) {
      drain();
      account(a, c, pend, lane, npend);
      tr(a, pend, TR_END + ci, lane);
      pend = -1;
      npend = 0;
    }
  };
  for (unsigned d = (unsigned)ci;; d += NCONS) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (vload(&c->desc_seq) <= d) flush();
    while (vload(&c->desc_seq) <= d) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > TMO) {
        if (lane == 0) atomicOr(a.err, 64u);
        dbg(a, c, 64, (int)d, (int)vload(&c->desc_seq), 0);
        return;
      }
    }
    asm volatile("" ::: "memory");
    if (lane == 0) lsti(&c->cur_d[ci], (int)d);
    const li32* ds = c->desc[d % NDESC];
    const int op = vloadi(&ds[0]), u = vloadi(&ds[1]), fill = vloadi(&ds[2]), nf = vloadi(&ds[3]);
    if (op != pend) flush();
    if (op < 0) return;
    if (!ensure_input(a, c, smem, op, lane)) return;
    if (op != last_op) tr(a, op, TR_START + ci, lane);
    last_op = op;
    if (op_kind(op) == OA) {
      attn_unit(a, smem, op, u, fill, nf, lane);
    } else {
      if (!wait_full(c, fill, a, lane)) return;
      if (a.compute & 1) gemv_unit(a, smem, op, u, fill, lane);
      release(c, fill, lane);
      pend = op;
      ++npend;
    }
    if (op_kind(op) == OA) tr(a, op, TR_END + ci, lane);
  }
}

__global__ void __launch_bounds__(NT) engine3_kernel(const Args* __restrict__ ap) {
  const Args& a = *ap;  // read through the scalar cache (a by-value struct argument would be copied to scratch)
  unsigned char* smem = e3_smem;
  CtlL* c = (CtlL*)&e3_ctl;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < (int)(sizeof(Ctl) / 4); i += NT) ((unsigned*)c)[i] = 0u;
  __syncthreads();
  if (threadIdx.x == 0) {
    c->staged_op = -1;
    c->gather_op = -1;
    c->edge_ok = -1;
    c->ru[0] = a.ru[0]; c->ru[1] = a.ru[1]; c->ru[2] = a.ru[2]; c->ru[3] = a.ru[3]; c->ru[4] = a.ru[4];
    c->units[0] = a.units[0]; c->units[1] = a.units[1]; c->units[2] = a.units[2]; c->units[3] = a.units[3];
    c->units[4] = a.units[4];
  }
  __syncthreads();
  const int w = __builtin_amdgcn_readfirstlane(wave);
  if (a.trace && threadIdx.x == 0) a.trace[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  if (w == 0) claimer(a, c, lane);
  else if (w == 1) loader(a, c, smem, lane);
  else consumer(a, c, smem, w - 2, lane);
}

}  // namespace e3

extern "C" int lga_e3_lds_bytes() { return e3::LDS_TOTAL; }
extern "C" int lga_e3_slot_bytes() { return e3::SLOT; }
extern "C" int lga_e3_consumers() { return e3::NCONS; }
extern "C" int lga_e3_counter_words(int L, int G) { return (10 * L * e3::NSH + L * G) * e3::CW; }
extern "C" int lga_e3_args_bytes() { return (int)sizeof(e3::Args); }
extern "C" int lga_e3_layer_bytes() { return (int)sizeof(e3::Layer); }

// args_dev: a device copy of e3::Args (the caller fills it through lga_e3_fill_args and copies it); grid = the CU count
extern "C" int lga_e3_launch(const void* args_dev, int n_cu, hipStream_t stream) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)e3::engine3_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, e3::LDS_TOTAL);
    attr = true;
  }
  e3::engine3_kernel<<<n_cu, e3::NT, e3::LDS_TOTAL, stream>>>((const e3::Args*)args_dev);
  return (int)hipGetLastError();
}

// fills an Args block from plain values (Python side: ctypes)
extern "C" int lga_e3_fill_args(void* out, const void* layers_dev, int L, int C, int H, int G, int I, int Kp, int S,
                                int splits, int gq, int gp, int gi, const int* ru, const int* units, int Nq,
                                const int64_t* pos, const void* x0, void* act, long long act_stride, const int* aoff,
                                float* ws, unsigned* ctr, unsigned* err, float eps, float scale, int compute,
                                unsigned long long* trace) {
  e3::Args a{};
  a.layers = (const e3::Layer*)layers_dev;
  a.L = L; a.C = C; a.H = H; a.G = G; a.I = I; a.Kp = Kp; a.S = S; a.splits = splits;
  a.gq = gq; a.gp = gp; a.gi = gi;
  for (int i = 0; i < 5; ++i) { a.ru[i] = ru[i]; a.units[i] = units[i]; }
  a.Nq = Nq; a.pos = pos; a.x0 = (const uint16_t*)x0; a.act = (uint16_t*)act; a.act_stride = act_stride;
  a.a_qkv = aoff[0]; a.a_y = aoff[1]; a.a_xp = aoff[2]; a.a_g = aoff[3]; a.a_xo = aoff[4];
  a.ws = ws; a.ctr = ctr; a.err = err; a.eps = eps; a.scale = scale; a.compute = compute;
  a.trace = trace;
  memcpy(out, &a, sizeof(a));
  return 0;
}
