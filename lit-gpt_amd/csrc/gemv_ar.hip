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

// ---------------------------------------------------------------------------------------------------------------
// Tagged form (lga_q4_gemv_allreduce_tagged): no arrival counters, no flags, no last-arriver sum. Every workgroup
// pushes its rows into every peer's mailbox as 8-byte granules {bf16 pair, call sequence} (one 16-B system-coherent
// store carries two; MI355X_MICROARCH.md "handoff-1to1": the data is its own flag), then polls its OWN rows'
// granules from every rank in its own mailbox and writes those rows of y — the ordered fp32 sum over ranks 0..W-1,
// bf16 once, + residual: ordered_sum8's arithmetic, so the bits equal lga_q4_gemv + lga_allreduce_bf16. The
// row-parallel projection's all-reduce then costs one push and one poll round trip in every workgroup, in parallel,
// instead of the drain + arrival chain + system-scope fences + one workgroup summing all N rows (measured in one
// process with the peers' flags pre-set: 10.9-11.0 us per call at the 7B TP = 8 rank's shapes against 2.6 us for the
// GEMV alone, profiles/r06_allreduce_push_single_process.txt).
// The call sequence: every workgroup reads the rank's launch index at its start (+ 1 = this call's sequence) and,
// once its pushes are out, arrives on a counter; the last arriver re-arms that counter and advances the index. Every
// workgroup of the launch has started (and read the index) before the last one arrives, and launches on one stream
// do not overlap, so all of a launch's workgroups agree on the sequence and graph replays keep counting. (An
// old / grid division of one shared counter breaks as soon as two calls have different grids.) A granule slot is the sequence's parity, as in the flag protocol: a rank is at most
// one call ahead of a peer, because its call s + 1 needed the peer's call-s granules, which the peer pushed only
// after its call s - 1 had finished reading that slot. Every workgroup waits only for OTHER ranks, never for a
// workgroup of its own launch, so the grid need not be co-resident; the poll is bounded (5 s, then the error word).
constexpr int kGranuleOffsetSlots = 2;  // mailbox granule region: [2 slots][8 sources][cap / 2] x 8 B after the data
__device__ __forceinline__ unsigned char* granule_ptr(unsigned char* mb, int slot, int src, int cap) {
  return mb + kFlagBytes + (size_t)kGranuleOffsetSlots * kMaxRanks * cap * 2 + ((size_t)slot * kMaxRanks + src) * cap * 4;
}

struct ArtArgs {
  unsigned char* mb[kMaxRanks];
  int rank, world, cap;
  unsigned* arrive;      // arrivals of this launch (re-armed by the last arriver)
  unsigned* launch_idx;  // calls completed by this rank (monotonic)
  unsigned* err;
  const uint16_t* residual;
  uint16_t* y;
};

template <int RPR, int CPT, int FMT>
__global__ void __launch_bounds__(256) gemv_q4_art_kernel(GemvArgs a, ArtArgs c) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NW = 4, ROWS = NW * RPR, NP = ROWS / 4;  // rows per workgroup, 16-B pieces (4 rows = 2 granules)
  static_assert(ROWS % 4 == 0, "16-B pieces of two granules");
  __shared__ unsigned s_seq;
  __shared__ __attribute__((aligned(16))) uint4 s_in[kMaxRanks][NP];
  const int t = threadIdx.x;
  if (t == 0)  // lands while the weights stream
    s_seq = __hip_atomic_fetch_add(c.launch_idx, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  gemv_q4_body<RPR, CPT, FMT, false, false, false, NW, true>(a, blockIdx.x, smem);
  __syncthreads();
  const unsigned seq = __builtin_amdgcn_readfirstlane(s_seq);
  const int slot = seq & 1;
  const int row0 = blockIdx.x * ROWS;
  const int np = min(NP, (a.N - row0) / 4);  // N % 8 == 0: whole pieces
  const uint16_t* rows = gemv_out_lds(smem, a.K);
  // 1. push: piece p = rows 4p .. 4p + 3 as granules {rows 4p | 4p+1, seq}, {rows 4p+2 | 4p+3, seq}
  if (t < np) {
    const uint2 rv = ((const uint2*)rows)[t];
    const uint4 piece = make_uint4(rv.x, seq, rv.y, seq);
    for (int r = 0; r < c.world; ++r) {  // one peer per iteration: the resource stays wave-uniform
      if (r == c.rank) continue;           // the own rows stay in LDS (no round trip through the own mailbox)
      const __amdgpu_buffer_rsrc_t dst = mb_rsrc(granule_ptr(c.mb[r], slot, c.rank, c.cap), c.cap * 4);
      st_sys16(dst, (row0 / 4 + t) * 16, piece);
    }
    s_in[c.rank][t] = piece;
  }
  // the launch bookkeeping (off the data path: its latency overlaps the poll below)
  if (t == 64) {
    if (__hip_atomic_fetch_add(c.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __hip_atomic_store(c.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(c.launch_idx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // 2. poll this workgroup's pieces from every rank in the own mailbox (lane t: rank t / NP, piece t % NP)
  if (t < 64) {
    const int r = t / NP, p = t % NP;
    const bool mine = r < c.world && r != c.rank && p < np;
    __amdgpu_buffer_rsrc_t src[kMaxRanks];
#pragma unroll
    for (int k = 0; k < kMaxRanks; ++k)
      src[k] = mb_rsrc(granule_ptr(c.mb[c.rank], slot, k < c.world ? k : 0, c.cap), c.cap * 4);
    uint4 v = make_uint4(0, seq, 0, seq);
    bool ok = !mine;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (true) {
      if (!ok) {
        uint4 w = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < kMaxRanks; ++k)  // scalar resources, the lane's own rank selected (no waterfall)
          if (k == r) w = ld_sys16(src[k], (row0 / 4 + p) * 16);
        if ((int)(w.y - seq) >= 0 && (int)(w.w - seq) >= 0) {
          v = w;
          ok = true;
        }
      }
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 500000000ull) {
        if (t == 0) __hip_atomic_fetch_or(c.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    if (mine) s_in[r][p] = v;
  }
  __syncthreads();
  // 3. rows 4p .. 4p + 3 of y: the ordered sum over ranks (ordered_sum8's rounding points) + residual
  if (t < np) {
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int r = 0; r < c.world; ++r) {
      const uint4 v = s_in[r][t];
      acc[0] += bflo(v.x);
      acc[1] += bfhi(v.x);
      acc[2] += bflo(v.z);
      acc[3] += bfhi(v.z);
    }
    uint2 o;
    if (c.residual) {
      const uint2 rv = ((const uint2*)(c.residual + row0))[t];
      o = make_uint2(pack2(round_bf(acc[0]) + bflo(rv.x), round_bf(acc[1]) + bfhi(rv.x)),
                     pack2(round_bf(acc[2]) + bflo(rv.y), round_bf(acc[3]) + bfhi(rv.y)));
    } else {
      o = make_uint2(pack2(acc[0], acc[1]), pack2(acc[2], acc[3]));
    }
    ((uint2*)(c.y + row0))[t] = o;
  }
}

template <int RPR, int CPT, int FMT>
static void launch_art(const GemvArgs& a, const ArtArgs& c, hipStream_t stream) {
  const int blocks = (a.N + 4 * RPR - 1) / (4 * RPR);
  gemv_q4_art_kernel<RPR, CPT, FMT><<<blocks, 256, gemv_lds_bytes(a.K), stream>>>(a, c);
}

template <int FMT>
static int dispatch_art(const GemvArgs& a, const ArtArgs& c, hipStream_t stream) {
  switch ((a.K / 32 + 63) / 64) {  // dispatch_ar's tiles (the same rows per workgroup, bit-identical rows)
    case 1: launch_art<4, 1, FMT>(a, c, stream); break;
    case 2: launch_art<4, 2, FMT>(a, c, stream); break;
    case 3: launch_art<4, 3, FMT>(a, c, stream); break;
    case 4: launch_art<2, 4, FMT>(a, c, stream); break;
    case 5:
    case 6: launch_art<2, 6, FMT>(a, c, stream); break;
    case 7:
    case 8: launch_art<2, 8, FMT>(a, c, stream); break;
    default:
      if (a.K <= 16 * 2048) {
        launch_art<2, 16, FMT>(a, c, stream);
        break;
      }
      lga_set_error("lga_q4_gemv_allreduce_tagged: K > 32768 is not supported");
      return (int)hipErrorInvalidValue;
  }
  return 0;
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

// The tagged form of lga_q4_gemv_allreduce (same arguments and result bits): arrive_counter's words 9 * 64 (this
// launch's arrivals, re-armed) and 9 * 64 + 32 (calls completed, monotonic; zeroed once); seq_counter is not used
// (the tagged protocol has its own mailbox region, so its calls and the flag protocol's may be mixed).
extern "C" int lga_q4_gemv_allreduce_tagged(const void* x, const uint8_t* qweight, const void* scales,
                                            const void* bias, const void* residual, void* y, int N, int K, int group,
                                            int fmt, void* const* mailboxes, int rank, int world, int cap,
                                            unsigned* seq_counter, unsigned* arrive_counter, unsigned* err,
                                            hipStream_t stream) {
  (void)seq_counter;
  LGA_CHECK_ARG(x && qweight && scales && y && mailboxes && arrive_counter && err,
                "lga_q4_gemv_allreduce_tagged: null pointer");
  LGA_CHECK_ARG(N > 0 && N % 8 == 0 && N <= cap, "lga_q4_gemv_allreduce_tagged: N must be a positive multiple of 8 <= cap");
  LGA_CHECK_ARG(K > 0 && K % 32 == 0 && group >= 32 && group % 32 == 0 && K % group == 0,
                "lga_q4_gemv_allreduce_tagged: K must be a multiple of 32 and of the group (a multiple of 32)");
  LGA_CHECK_ARG(fmt == 0 || fmt == 1 || fmt == 3, "lga_q4_gemv_allreduce_tagged: fmt must be 0, 1 or 3");
  LGA_CHECK_ARG(world >= 1 && world <= lga::kMaxRanks && rank >= 0 && rank < world,
                "lga_q4_gemv_allreduce_tagged: world must be 1..8 and 0 <= rank < world");
  lga::GemvArgs a{(const uint16_t*)x, qweight, scales, nullptr, nullptr, (const uint16_t*)bias, nullptr, nullptr,
                  nullptr, N, K, group, 0.0f};
  a.cb = lga::codebook_of(fmt);
  lga::ArtArgs c{};
  for (int r = 0; r < world; ++r) {
    LGA_CHECK_ARG(mailboxes[r] != nullptr, "lga_q4_gemv_allreduce_tagged: null mailbox");
    c.mb[r] = (unsigned char*)mailboxes[r];
  }
  c.rank = rank;
  c.world = world;
  c.cap = cap;
  c.arrive = arrive_counter + 9 * lga::kArriveStride;
  c.launch_idx = arrive_counter + 9 * lga::kArriveStride + 32;
  c.err = err;
  c.residual = (const uint16_t*)residual;
  c.y = (uint16_t*)y;
  const int rc = fmt == 0 ? lga::dispatch_art<0>(a, c, stream) : lga::dispatch_art<1>(a, c, stream);
  if (rc) return rc;
  LGA_LAUNCH_RETURN();
}
