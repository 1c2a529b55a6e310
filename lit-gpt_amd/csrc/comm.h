// Mailbox layout of the xGMI one-shot all-reduce (comm.hip) and the pieces of its protocol the fused
// GEMV + all-reduce (gemv_ar.hip) shares: a rank's mailbox is flags[8] (uint32, 256 B apart) then
// data[2 slots][8 sources][cap] bf16; a call's slot is its sequence number's parity.
#pragma once
#include "common.h"

namespace lga {

constexpr int kMaxRanks = 8;
constexpr int kFlagStride = 64;  // uint32 per flag (256 B)
constexpr size_t kFlagBytes = kMaxRanks * kFlagStride * 4;

struct Peers {
  unsigned char* mb[kMaxRanks];
  // diagnostics (lga_comm_trace; null = off): one record of kTraceWords uint64 per call, indexed by the call's sequence
  // number: [0] seq | rank << 32 | kind << 40 (1 one-shot, 2 fused GEMV), [1] entry (one-shot) / last arrival (fused)
  // time, [2] flags raised, [3] wait done, [4] timed out, [5] the sequence word read at entry, [6 + r] the flag of
  // rank r in this rank's mailbox when the wait ended; times from s_memrealtime (100 MHz, one clock per device)
  unsigned long long* trace;
  int trace_n;
};
constexpr int kTraceWords = 16;
__device__ __forceinline__ unsigned long long* trace_rec(const Peers& p, unsigned seq) {
  return p.trace ? p.trace + (size_t)((seq - 1u) % (unsigned)p.trace_n) * kTraceWords : nullptr;
}
// host side: the record buffer lga_comm_trace installed (comm.hip)
void comm_trace_get(unsigned long long** buf, int* n);

__device__ __forceinline__ uint16_t* slot_ptr(unsigned char* mb, int slot, int src, int cap) {
  return (uint16_t*)(mb + kFlagBytes) + ((size_t)slot * kMaxRanks + src) * cap;
}

// Mailbox payload traffic is system-coherent (sc0 sc1): the pushes write through every cache level, the reads bypass
// them, so a slot's bytes never depend on which XCD's L2 (or which process's mapping of the IPC buffer) saw them
// last — on top of the flags' release / acquire. (8 ranks sharing one GPU, 64 back-to-back calls, intermittently
// summed a stale slot with plain payload accesses: tests/workers/allreduce_worker.py "burst".) 16-B buffer accesses,
// offsets in voffset; the resource's base is wave-uniform.
typedef uint32_t mb_u32x4 __attribute__((ext_vector_type(4)));
constexpr int kSysCoherent = 1 | 16;  // cache-policy aux bits sc0 | sc1 (gfx940+)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mb_rsrc(const void* base, int bytes) {
  // the base is wave-uniform by construction; readfirstlane makes that visible to hipCC, which would otherwise keep
  // the resource in VGPRs and wrap every access in a waterfall loop
  const uint64_t v = (uint64_t)(uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ void st_sys16(__amdgpu_buffer_rsrc_t r, int off, uint4 v) {
  const mb_u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(w, r, off, 0, kSysCoherent);
}
__device__ __forceinline__ uint4 ld_sys16(__amdgpu_buffer_rsrc_t r, int off) {
  const mb_u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSysCoherent);
  return make_uint4(w.x, w.y, w.z, w.w);
}

// The flag protocol follows the memory model (LGA_COMM_FORMAL=1, default): a system-scope release before each flag,
// an acquire after the wait. Mailboxes are UNCACHED device memory (lga_comm_alloc: hipDeviceMallocUncached), so
// LGA_COMM_FORMAL=0 builds the form that relies on that instead (drains + barriers, no cache maintenance); on one
// GPU shared by the ranks the two measured the same per call (tools/tp_fused_time.py), across GPUs it is unmeasured.
#ifndef LGA_COMM_FORMAL
#define LGA_COMM_FORMAL 1
#endif

// Raise this rank's flag for call `seq` in every peer's mailbox (threads t < world), after the calling workgroup's
// data stores are complete: each storing wave drained (asm vmcnt(0)) and the workgroup barrier ordered them before
// the flag writers, which drain again and store the flag (system scope).
__device__ __forceinline__ void raise_flags(const Peers& peers, int rank, int world, unsigned seq, int t) {
  if (unsigned long long* rec = trace_rec(peers, seq)) {
    if (t == 0) rec[2] = __builtin_amdgcn_s_memrealtime();
  }
  if (t < world && t != rank) {
    unsigned* f = (unsigned*)peers.mb[t] + rank * kFlagStride;
#if LGA_COMM_FORMAL
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(f, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
#else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(f, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#endif
  }
}

// Wait (threads t < 64) until every peer's flag in this rank's own mailbox reached `seq` — bounded: after 5 s of the
// 100 MHz real-time clock the error word is set and the caller finishes with whatever arrived, so a lost peer never
// hangs the GPU. The caller follows with a workgroup barrier.
__device__ __forceinline__ void wait_flags(const Peers& peers, int rank, int world, unsigned seq, unsigned* err,
                                           int t) {
  if (t < 64) {
    const bool mine = t < world && t != rank;
    const unsigned* f = (const unsigned*)peers.mb[rank] + (mine ? t : 0) * kFlagStride;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    unsigned v = seq;
    bool timed_out = false;
    while (true) {
      v = mine ? __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : seq;
      if (__all((int)(v - seq) >= 0)) break;
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 500000000ull) {
        if (t == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        timed_out = true;
        break;
      }
    }
    if (unsigned long long* rec = trace_rec(peers, seq)) {
      if (t == 0) {
        rec[3] = __builtin_amdgcn_s_memrealtime();
        rec[4] = timed_out ? 1ull : 0ull;
      }
      if (t < world) rec[6 + t] = mine ? v : seq;
    }
#if LGA_COMM_FORMAL
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    // the invalidate completes asynchronously: wait for it here, so the caller's barrier releases the other waves'
    // mailbox loads only after it (MI355X_MICROARCH.md "Valid forms", Consumer: acquire -> vmcnt(0) -> barrier)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // compiler ordering; the mailbox reads go to memory
#endif
  }
}

// y[8 i .. 8 i + 8) = bf16(sum over ranks 0..world-1 of src_r) (+ residual: bf16(bf16(sum) + residual)) — the
// ordered fp32 sum every rank computes identically
// rs[r]: rank r's slot in this rank's mailbox (read system-coherent; built by slot_rsrcs), except rank local_rank
// (-1: none), whose partial is read from `x_local`. The rank loop is unrolled to kMaxRanks so the resources stay in
// scalar registers (a runtime-indexed array would put them in VGPRs and wrap every load in a waterfall loop).
__device__ __forceinline__ void slot_rsrcs(const Peers& peers, int rank, int slot, int world, int cap,
                                           __amdgpu_buffer_rsrc_t (&rs)[kMaxRanks]) {
#pragma unroll
  for (int r = 0; r < kMaxRanks; ++r) rs[r] = mb_rsrc(slot_ptr(peers.mb[rank], slot, r < world ? r : 0, cap), cap * 2);
}
__device__ __forceinline__ uint4 ordered_sum8(const __amdgpu_buffer_rsrc_t (&rs)[kMaxRanks], const uint4* x_local,
                                             int local_rank, int world, const uint16_t* residual, int i) {
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.0f;
  // every rank's piece in flight at once (one load round trip), then the sum in rank order
  uint4 vin[kMaxRanks];
#pragma unroll
  for (int r = 0; r < kMaxRanks; ++r)
    vin[r] = r >= world ? make_uint4(0, 0, 0, 0) : (r == local_rank ? x_local[i] : ld_sys16(rs[r], i * 16));
#pragma unroll
  for (int r = 0; r < kMaxRanks; ++r) {
    if (r >= world) break;
    const uint4 v = vin[r];
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[2 * e] += bflo(d[e]);
      acc[2 * e + 1] += bfhi(d[e]);
    }
  }
  uint32_t o[4];
  if (residual) {
    const uint4 rv = ((const uint4*)residual)[i];
    const uint32_t rd[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      o[e] = pack2(round_bf(acc[2 * e]) + bflo(rd[e]), round_bf(acc[2 * e + 1]) + bfhi(rd[e]));
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2(acc[2 * e], acc[2 * e + 1]);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

}  // namespace lga
