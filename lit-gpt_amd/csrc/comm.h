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
};

__device__ __forceinline__ uint16_t* slot_ptr(unsigned char* mb, int slot, int src, int cap) {
  return (uint16_t*)(mb + kFlagBytes) + ((size_t)slot * kMaxRanks + src) * cap;
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
    while (true) {
      const unsigned v = mine ? __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : seq;
      if (__all((int)(v - seq) >= 0)) break;
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 500000000ull) {
        if (t == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
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
__device__ __forceinline__ uint4 ordered_sum8(const uint4* const* src, int world, const uint16_t* residual, int i) {
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.0f;
  for (int r = 0; r < world; ++r) {
    const uint4 v = src[r][i];
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
