// Row-parallel decode GEMV with the tensor-parallel all-reduce in its epilogue (one launch instead of two).
//
// Replaces, for one-token messages, the pair "row-parallel Linear, then generate/tp.py's forward hook
// all_reduce_output" (reference generate/tp.py:53,57,70 register it on attn.proj / mlp.proj; :73-74 sum the
// partial outputs over the ranks) plus the Block residual add (lit_gpt/model.py:591-592). Today's two-launch form
// is lga_q4_gemv (partial rows, bias included) + lga_allreduce_bf16 (comm.hip); this kernel produces the same bits:
//  1. every workgroup computes its NW * RPR partial rows with gemv_q4_body (identical arithmetic, rows to LDS) and
//     pushes them as 16-B pieces straight into slot[seq & 1][rank] of EVERY rank's mailbox (its own included) —
//     the partial never lands in this rank's HBM, and the pushes of all workgroups overlap the weight stream;
//  2. it drains its stores and bumps an arrival counter; the workgroup that arrives last on this rank knows all of
//     the rank's rows are in every mailbox, re-arms the counter, raises this rank's flag in every peer's mailbox,
//     waits for the peers' flags (comm.h, bounded at 5 s then the error word) and sums slots 0..W-1 in rank order
//     in fp32, bf16 once, + residual (comm.h ordered_sum8) into y, then advances the call sequence.
// The sequence counter and mailboxes are lga_allreduce_bf16's (the two entry points can be mixed in one call
// sequence). Graph-capturable: every argument is fixed and the sequence lives on the device.
#include "comm.h"
#include "gemv_body.h"

namespace lga {

struct ArArgs {
  Peers peers;
  int rank, world, cap;
  unsigned* seq;     // call sequence (shared with lga_allreduce_bf16)
  unsigned* arrive;  // kArriveWords arrival counters, zero between launches (each last arriver re-arms its own)
  unsigned* err;
  const uint16_t* residual;  // [N] or null
  uint16_t* y;               // [N]
};

// Arrivals go through one counter per blockIdx % 8 class (a class shares an XCD under round-robin placement; that is
// speed only, never correctness), each 256 B apart, and the last arriver of each class bumps the top counter: 8 + 32
// serialized device-scope atomics instead of 256 on one word (MI355X_MICROARCH.md "fanin": ≈12 ns each).
constexpr int kArriveStride = 64;  // uint32 (256 B)

template <int RPR, int CPT, int FMT>
__global__ void __launch_bounds__(256) gemv_q4_ar_kernel(GemvArgs a, ArArgs c) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NW = 4, ROWS = NW * RPR, CH = ROWS / 8;  // rows per workgroup, their 16-B pieces
  static_assert(ROWS % 8 == 0, "16-B pieces of whole rows");
  __shared__ unsigned s_last;
  const int t = threadIdx.x;
  // read before arriving (only the last arriver advances it); uniform, so the mailbox resources stay scalar
  const unsigned seq = __builtin_amdgcn_readfirstlane(*c.seq + 1u);
  const int slot = seq & 1;
  gemv_q4_body<RPR, CPT, FMT, false, false, false, NW, true>(a, blockIdx.x, smem);
  __syncthreads();
  const uint4* rows = (const uint4*)gemv_out_lds(smem, a.K);
  const int row0 = blockIdx.x * ROWS;
  // one peer per iteration: the mailbox resource must be wave-uniform (a lane-dependent peer would need a waterfall)
  for (int r = 0; r < c.world; ++r) {
    const __amdgpu_buffer_rsrc_t dst = mb_rsrc(slot_ptr(c.peers.mb[r], slot, c.rank, c.cap), c.cap * 2);
    if (t < CH && row0 + t * 8 < a.N) st_sys16(dst, (row0 + t * 8) * 2, rows[t]);
  }
  // the pushes are complete (uncached mailboxes: acknowledged = visible) before this workgroup arrives
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const unsigned cls = blockIdx.x & 7, classes = min(gridDim.x, 8u);
    const unsigned in_cls = (gridDim.x - cls + 7) / 8;  // workgroups of this class
    unsigned* cc = c.arrive + cls * kArriveStride;
    unsigned last = 0;
#if LGA_COMM_FORMAL
    // memory-model form: every workgroup's arrival is a system-scope release of its pushes (fence, then an asm
    // drain the compiler cannot drop behind a provably empty scoreboard: MI355X_MICROARCH.md "Compiler hazard"),
    // the counters' RMW chain carries them to the last arriver, whose system-scope acquire precedes its flag
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    if (__hip_atomic_fetch_add(cc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == in_cls - 1) {
      __hip_atomic_store(cc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm: the class is complete
      unsigned* top = c.arrive + 8 * kArriveStride;
#if LGA_COMM_FORMAL
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");  // what the class's arrivals released, released on
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
      last = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == classes - 1;
      if (last) __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#if LGA_COMM_FORMAL
    if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // every workgroup's pushes happen-before the flags
#endif
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  // ---- the last arriver: every row of this rank is in every mailbox ----
  if (unsigned long long* rec = trace_rec(c.peers, seq)) {
    if (t == 0) {
      rec[0] = seq | ((unsigned long long)c.rank << 32) | (2ull << 40);
      rec[1] = __builtin_amdgcn_s_memrealtime();
      rec[5] = seq - 1u;
    }
  }
  raise_flags(c.peers, c.rank, c.world, seq, t);
  wait_flags(c.peers, c.rank, c.world, seq, c.err, t);
  __syncthreads();
  __amdgpu_buffer_rsrc_t rs[kMaxRanks];
  slot_rsrcs(c.peers, c.rank, slot, c.world, c.cap, rs);
  for (int i = t; i < a.N / 8; i += NW * 64) ((uint4*)c.y)[i] = ordered_sum8(rs, nullptr, -1, c.world, c.residual, i);
  __syncthreads();
  if (t == 0) *c.seq = seq;
}

template <int RPR, int CPT, int FMT>
static void launch_ar(const GemvArgs& a, const ArArgs& c, hipStream_t stream) {
  const int blocks = (a.N + 4 * RPR - 1) / (4 * RPR);
  gemv_q4_ar_kernel<RPR, CPT, FMT><<<blocks, 256, gemv_lds_bytes(a.K), stream>>>(a, c);
}

// the one-shot GEMV's tile choice for these shapes (gemv.hip dispatch, variant 0: more waves)
template <int FMT>
static int dispatch_ar(const GemvArgs& a, const ArArgs& c, hipStream_t stream) {
  switch ((a.K / 32 + 63) / 64) {
    case 1: launch_ar<4, 1, FMT>(a, c, stream); break;
    case 2: launch_ar<4, 2, FMT>(a, c, stream); break;
    case 3: launch_ar<4, 3, FMT>(a, c, stream); break;
    case 4: launch_ar<2, 4, FMT>(a, c, stream); break;
    case 5:
    case 6: launch_ar<2, 6, FMT>(a, c, stream); break;
    case 7:
    case 8: launch_ar<2, 8, FMT>(a, c, stream); break;
    default:
      if (a.K <= 16 * 2048) {
        launch_ar<2, 16, FMT>(a, c, stream);
        break;
      }
      lga_set_error("lga_q4_gemv_allreduce: K > 32768 is not supported");
      return (int)hipErrorInvalidValue;
  }
  return 0;
}

}  // namespace lga

extern "C" int lga_q4_gemv_allreduce(const void* x, const uint8_t* qweight, const void* scales, const void* bias,
                                     const void* residual, void* y, int N, int K, int group, int fmt,
                                     void* const* mailboxes, int rank, int world, int cap, unsigned* seq_counter,
                                     unsigned* arrive_counter, unsigned* err, hipStream_t stream) {
  LGA_CHECK_ARG(x && qweight && scales && y && mailboxes && seq_counter && arrive_counter && err,
                "lga_q4_gemv_allreduce: null pointer");
  LGA_CHECK_ARG(N > 0 && N % 8 == 0 && N <= cap, "lga_q4_gemv_allreduce: N must be a positive multiple of 8 <= cap");
  LGA_CHECK_ARG(K > 0 && K % 32 == 0 && group >= 32 && group % 32 == 0 && K % group == 0,
                "lga_q4_gemv_allreduce: K must be a multiple of 32 and of the group (a multiple of 32)");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1 || fmt == 3, "lga_q4_gemv_allreduce: fmt must be 0, 1 or 3");
  LGA_CHECK_ARG(world >= 1 && world <= lga::kMaxRanks && rank >= 0 && rank < world,
                "lga_q4_gemv_allreduce: world must be 1..8 and 0 <= rank < world");
  lga::GemvArgs a{(const uint16_t*)x, qweight, scales, nullptr, nullptr, (const uint16_t*)bias, nullptr, nullptr,
                  nullptr, N, K, group, 0.0f};
  a.cb = lga::codebook_of(fmt);
  lga::ArArgs c{};
  for (int r = 0; r < world; ++r) {
    LGA_CHECK_ARG(mailboxes[r] != nullptr, "lga_q4_gemv_allreduce: null mailbox");
    c.peers.mb[r] = (unsigned char*)mailboxes[r];
  }
  lga::comm_trace_get(&c.peers.trace, &c.peers.trace_n);
  c.rank = rank;
  c.world = world;
  c.cap = cap;
  c.seq = seq_counter;
  c.arrive = arrive_counter;
  c.err = err;
  c.residual = (const uint16_t*)residual;
  c.y = (uint16_t*)y;
  const int rc = fmt == 0 ? lga::dispatch_ar<0>(a, c, stream) : lga::dispatch_ar<1>(a, c, stream);
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}
