// One-shot all-reduce of the tensor-parallel decode activations over xGMI peer memory.
//
// Replaces the collective behind generate/tp.py's forward hook `all_reduce_output` (reference
// generate/tp.py:73-74: `all_reduce(outs, "sum", ranks)`, hooked after every CausalSelfAttention and MLP at
// :53,57,70) for the small messages of a decode step (one token: C bf16 = 8-16 KB). RCCL's ring / tree kernels
// pay a multi-hop latency per call; at 64 calls per Llama-2-7B token that dominates TP decode. Here every rank
// PUSHES its partial straight into a mailbox in every peer's HBM (one xGMI hop; MI355X links are point to point),
// raises a flag there, waits for the flags of all peers in its own mailbox, and sums the W partials in rank order
// 0..W-1 in fp32 — the same order on every rank, so all ranks hold bit-identical results (TP replicates the
// sampling, generate/tp.py). The Block residual add (lit_gpt/model.py:591-592, `x + attn(...)`) is fused in.
//
// Mailbox (per rank, uncached device memory from lga_comm_alloc, IPC-exported): flags[8] (uint32, 256 B apart)
// then data[2 slots][8 sources][cap] bf16. A call's slot is its sequence number's parity: a rank can run at most
// one call ahead of a peer (call s+1 needs the peer's s+1 data, sent after the peer finished call s), so two
// slots never overwrite unread data. Sequence numbers come from a per-rank device counter the kernel advances,
// so the launch is graph-capturable (the replayed arguments never change).
#include <string.h>

#include "common.h"

namespace lga {

constexpr int kMaxRanks = 8;
constexpr int kFlagStride = 64;                        // uint32 per flag (256 B)
constexpr size_t kFlagBytes = kMaxRanks * kFlagStride * 4;
constexpr int kCommThreads = 512;

struct Peers {
  unsigned char* mb[kMaxRanks];
};

__device__ __forceinline__ uint16_t* slot_ptr(unsigned char* mb, int slot, int src, int cap) {
  return (uint16_t*)(mb + kFlagBytes) + ((size_t)slot * kMaxRanks + src) * cap;
}

__global__ void __launch_bounds__(kCommThreads) allreduce_kernel(const uint16_t* __restrict__ x,
                                                                 const uint16_t* __restrict__ residual,
                                                                 uint16_t* __restrict__ y, int n, Peers peers,
                                                                 int rank, int world, int cap,
                                                                 unsigned* __restrict__ seq_ctr,
                                                                 unsigned* __restrict__ err) {
  const int t = threadIdx.x;
  const unsigned seq = *seq_ctr + 1u;
  const int slot = seq & 1;
  const int n8 = n / 8;
  // 1. push this rank's partial into every peer's mailbox (16-B stores over xGMI)
  for (int r = 0; r < world; ++r) {
    if (r == rank) continue;
    uint4* dst = (uint4*)slot_ptr(peers.mb[r], slot, rank, cap);
    for (int i = t; i < n8; i += kCommThreads) dst[i] = ((const uint4*)x)[i];
  }
  // 2. release: every storing thread's writes are complete and visible system-wide before any flag
  //    (each storing wave drains its stores, the workgroup barrier orders them before the flag writers, and each
  //    flag writer publishes with a system-scope RELEASE store behind an explicit drain: MI355X_MICROARCH.md
  //    "Compiler hazard" — the asm wait keeps the release's write-back wait from being dropped)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t < world && t != rank) {
    unsigned* f = (unsigned*)peers.mb[t] + rank * kFlagStride;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(f, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. wait for every peer's flag in this rank's own mailbox (bounded: 5 s of the 100 MHz real-time clock — far
  //    beyond any host-side skew between live ranks — then the error word is set and the kernel finishes with
  //    whatever arrived, so a lost peer never hangs the GPU)
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
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  // 4. ordered fp32 sum over ranks 0..W-1, bf16 once, then the residual add in the reference's rounding
  for (int i = t; i < n8; i += kCommThreads) {
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.0f;
    for (int r = 0; r < world; ++r) {
      const uint4 v = r == rank ? ((const uint4*)x)[i] : ((const uint4*)slot_ptr(peers.mb[rank], slot, r, cap))[i];
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
    ((uint4*)y)[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
  __syncthreads();
  if (t == 0) *seq_ctr = seq;
}

}  // namespace lga

extern "C" size_t lga_comm_mailbox_bytes(int cap) {
  return lga::kFlagBytes + (size_t)2 * lga::kMaxRanks * (size_t)cap * sizeof(uint16_t);
}

// Uncached (coherent across devices) zeroed device allocation + its IPC handle (64 bytes, hipIpcMemHandle_t).
extern "C" int lga_comm_alloc(size_t bytes, void** ptr, void* ipc_handle) {
  LGA_CHECK_ARG(ptr && ipc_handle && bytes > 0, "lga_comm_alloc: bad arguments");
  hipError_t e = hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(*ptr, 0, bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipIpcGetMemHandle((hipIpcMemHandle_t*)ipc_handle, *ptr);
  if (e != hipSuccess) {
    lga_set_error(hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

extern "C" int lga_comm_open(const void* ipc_handle, void** ptr) {
  LGA_CHECK_ARG(ptr && ipc_handle, "lga_comm_open: bad arguments");
  hipIpcMemHandle_t h;
  memcpy(&h, ipc_handle, sizeof(h));
  hipError_t e = hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) {
    lga_set_error(hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

extern "C" int lga_comm_close(void* ptr) {
  const hipError_t e = hipIpcCloseMemHandle(ptr);
  if (e != hipSuccess) lga_set_error(hipGetErrorString(e));
  return (int)e;
}

extern "C" int lga_comm_free(void* ptr) {
  const hipError_t e = hipFree(ptr);
  if (e != hipSuccess) lga_set_error(hipGetErrorString(e));
  return (int)e;
}

extern "C" int lga_allreduce_bf16(const void* x, const void* residual, void* y, int n, void* const* mailboxes,
                                  int rank, int world, int cap, unsigned* seq_counter, unsigned* err,
                                  hipStream_t stream) {
  LGA_CHECK_ARG(x && y && mailboxes && seq_counter && err, "lga_allreduce_bf16: null pointer");
  LGA_CHECK_ARG(world >= 1 && world <= lga::kMaxRanks && rank >= 0 && rank < world,
                "lga_allreduce_bf16: world must be 1..8 and 0 <= rank < world");
  LGA_CHECK_ARG(n > 0 && n % 8 == 0 && n <= cap, "lga_allreduce_bf16: n must be a positive multiple of 8 <= cap");
  lga::Peers p{};
  for (int r = 0; r < world; ++r) {
    LGA_CHECK_ARG(mailboxes[r] != nullptr, "lga_allreduce_bf16: null mailbox");
    p.mb[r] = (unsigned char*)mailboxes[r];
  }
  lga::allreduce_kernel<<<1, lga::kCommThreads, 0, stream>>>((const uint16_t*)x, (const uint16_t*)residual,
                                                             (uint16_t*)y, n, p, rank, world, cap, seq_counter, err);
  LGA_LAUNCH_RETURN();
}
