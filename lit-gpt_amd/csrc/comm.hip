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

#include "comm.h"

namespace lga {

constexpr int kCommThreads = 512;

static unsigned long long* g_trace = nullptr;
static int g_trace_n = 0;
void comm_trace_get(unsigned long long** buf, int* n) {
  *buf = g_trace;
  *n = g_trace_n;
}

__global__ void __launch_bounds__(kCommThreads) allreduce_kernel(const uint16_t* __restrict__ x,
                                                                 const uint16_t* __restrict__ residual,
                                                                 uint16_t* __restrict__ y, int n, Peers peers,
                                                                 int rank, int world, int cap,
                                                                 unsigned* __restrict__ seq_ctr,
                                                                 unsigned* __restrict__ err) {
  const int t = threadIdx.x;
  const unsigned raw = *seq_ctr;
  const unsigned seq = __builtin_amdgcn_readfirstlane(raw + 1u);  // uniform: the mailbox resources stay scalar
  const int slot = seq & 1;
  if (unsigned long long* rec = trace_rec(peers, seq)) {
    if (t == 0) {
      rec[0] = seq | ((unsigned long long)rank << 32) | (1ull << 40);
      rec[1] = __builtin_amdgcn_s_memrealtime();
      rec[5] = raw;
    }
  }
  const int n8 = n / 8;
  // 1. push this rank's partial into every peer's mailbox (16-B stores over xGMI)
  for (int r = 0; r < world; ++r) {
    if (r == rank) continue;
    const __amdgpu_buffer_rsrc_t dst = mb_rsrc(slot_ptr(peers.mb[r], slot, rank, cap), n * 2);
    for (int i = t; i < n8; i += kCommThreads) st_sys16(dst, i * 16, ((const uint4*)x)[i]);
  }
  // 2. release: every storing thread's writes are complete and visible system-wide before any flag (each storing
  //    wave drains its stores, the workgroup barrier orders them before the flag writers: raise_flags in comm.h;
  //    MI355X_MICROARCH.md "Compiler hazard" — the asm wait keeps the release's write-back wait from being dropped)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  raise_flags(peers, rank, world, seq, t);
  // 3. wait for every peer's flag in this rank's own mailbox (bounded at 5 s, then the error word is set and the
  //    kernel finishes with whatever arrived, so a lost peer never hangs the GPU)
  wait_flags(peers, rank, world, seq, err, t);
  __syncthreads();
  // 4. ordered fp32 sum over ranks 0..W-1, bf16 once, then the residual add in the reference's rounding
  __amdgpu_buffer_rsrc_t rs[kMaxRanks];
  slot_rsrcs(peers, rank, slot, world, cap, rs);
  for (int i = t; i < n8; i += kCommThreads)
    ((uint4*)y)[i] = ordered_sum8(rs, (const uint4*)x, rank, world, residual, i);
  __syncthreads();
  if (t == 0) *seq_ctr = seq;
}

}  // namespace lga

// flags, the flag protocol's data [2][8][cap] bf16, then the tagged protocol's granules [2][8][cap / 2] x 8 B
// (gemv_ar.hip granule_ptr)
extern "C" size_t lga_comm_mailbox_bytes(int cap) {
  return lga::kFlagBytes + (size_t)2 * lga::kMaxRanks * (size_t)cap * sizeof(uint16_t) +
         (size_t)2 * lga::kMaxRanks * (size_t)cap * 4;
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
  lga::comm_trace_get(&p.trace, &p.trace_n);
  lga::allreduce_kernel<<<1, lga::kCommThreads, 0, stream>>>((const uint16_t*)x, (const uint16_t*)residual,
                                                             (uint16_t*)y, n, p, rank, world, cap, seq_counter, err);
  LGA_LAUNCH_RETURN();
}

// Diagnostics: every later all-reduce launch of this process (one-shot and fused GEMV, captured ones included — the
// pointer is baked into a graph at capture) records its call in buf (n_records x 16 uint64, indexed by sequence
// number; layout in comm.h Peers). buf = null switches it off.
extern "C" int lga_comm_trace(void* buf, int n_records) {
  LGA_CHECK_ARG(!buf || n_records > 0, "lga_comm_trace: n_records must be positive");
  lga::g_trace = (unsigned long long*)buf;
  lga::g_trace_n = buf ? n_records : 0;
  return 0;
}
