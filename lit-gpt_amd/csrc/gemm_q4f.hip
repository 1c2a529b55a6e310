// Prefill GEMM with the 4-bit dequantization fused in: Y[M, N] = X[M, K] . bf16(dequant(W))[N, K]^T
// (+bias / +residual), and the fc_1 || fc_2 + SwiGLU form g = bf16(silu(bf16(X W1^T))) * bf16(X W2^T).
//
// Replaces bitsandbytes' M > 1 path of `Linear4bit.forward` (dequantize_4bit into a bf16 weight, then the cuBLAS
// GEMM; reached through BitsandbytesPrecision, reference generate/base.py:128-136) for the prefill pass
// (next_token(model, arange(0, T), prompt), generate/base.py:83-85), the bf16 F.linear of unquantized models
// (lit_gpt/model.py:619,656), and LLaMAMLP's fc_1 / fc_2 / silu product (model.py:712-716). The weight is never
// materialised in bf16 in HBM: each workgroup dequantizes its weight tile into LDS once per K-step, to exactly the
// bits bnb's dequantize_4bit writes (bf16(value(nibble) * scale)), and every row of its tile reads it from there.
//
// MI355X design (CDNA4 playbook §5, "Pipelining across barriers"):
//  * 8 waves per workgroup, 64 rows per wave; tiles <BM, BN> = <256, 128> for long prompts (4 (M) x 2 (N) waves,
//    64 x 64 per wave = 4 x 4 `v_mfma_f32_16x16x32_bf16`), <256, 256> (64 x 128 per wave, one K-step of prefetch
//    to fit LDS) where its rounds fill the CUs better (fc_1 || fc_2 at 2048 tokens: 11 % faster), and <64, 128> /
//    <64, 256> for short ones (1 x 8 waves);
//    the weight rows are the A operand, so a lane's accumulators are 4 consecutive output columns of one row
//    (8-byte stores).
//  * X tiles and the packed weight / scale tiles reach LDS by LDS-DMA (`global_load_lds_dwordx4`, source-swizzled so
//    the 128-B rows are XOR-swizzled for conflict-free `ds_read_b128`), X two K-steps ahead in 3 buffers, the packed
//    weights three ahead in 4 (they are dequantized one K-step before use, between the MFMAs); one raw `s_barrier`
//    per K-step after a COUNTED `s_waitcnt vmcnt`, so the DMAs stay in flight across the barrier (never
//    `__syncthreads()`, whose vmcnt(0) would drain them); all LDS in one `__shared__` array; no other global loads
//    inside the loop.
//  * split-K for short prompts (few tiles): the K-slices of a tile write fp32 slabs write-through, the last to
//    arrive on a per-tile counter reads them past the L2 and sums them in slice order — deterministic — and runs
//    the epilogue (no agent fences).
//  * dequantization, int4-g: one `v_cvt_f32_ubyteN` per nibble, fma(n, s, -8 s) (exact: (n - 8) s needs 12
//    significant bits) and `v_cvt_pk_bf16_f32` (round to nearest even) — the reference's bf16((n - 8) * s).
//    nf4: bf16(NF4[n] * absmax) (fp32 product, as bnb's kernel) from an LDS table.
//  * bf16 weights (unquantized Linear, BASELINE config 2): the weight tile is DMA'd like X (no dequantization).
//  * tile order: m-tile fastest, so with 8 m-tiles (M = 2048) the blocks of one XCD (block id mod 8) share one
//    X row panel in their L2 and stream distinct weight tiles.
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace lga {
namespace pf {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 64, NT = 512;

#ifdef LGA_Q4F_TRACE  // lab builds only (tools/gemm_trace.py): per-workgroup phase timestamps, 100 MHz clock
__device__ unsigned long long g_q4f_trace[8192 * 4];
#define LGA_QTRACE(i)                                                                                  \
  do {                                                                                                 \
    if (threadIdx.x == 0 && blockIdx.x < 8192)                                                         \
      g_q4f_trace[(size_t)blockIdx.x * 4 + (i)] = __builtin_amdgcn_s_memrealtime();                    \
  } while (0)
#else
#define LGA_QTRACE(i) \
  do {                \
  } while (0)
#endif
constexpr int MAX_SPLITS = 8;  // K-slices per tile (split-K for short prompts)

// NW_ waves per workgroup: 8 (one workgroup per CU; the product's tiles), or 4 with a 128 x 128 tile in <= 80 KB of
// LDS so two independent workgroups share a CU (one's MFMAs under the other's DMA waits). The 4-wave tile is a lab
// build only (-DLGA_Q4F_W4_LAB, then LGA_Q4F_W4=1; tools/q4f_tile_ab.py): bit-identical, measured slower
template <int BM_, int BN_, int NW_ = 8>
struct Tile {
  static constexpr int BM = BM_, BN = BN_, NW = NW_, NTH = NW * 64;
  static constexpr int WM = BM / 64, WN = NW / WM;  // wave grid
  static constexpr int WC = BN / WN;               // weight rows (output columns) per wave
  static constexpr int FJ = WC / 16;               // 16-row weight fragments per wave
  static constexpr int A_BYTES = BM * BK * 2;      // one X tile (BM rows x 128 B)
  static constexpr int B_BYTES = BN * BK * 2;      // one bf16 weight tile
  static constexpr int RAW_BYTES = BN * BK / 2;    // one packed weight tile (BN rows x 32 B)
  // packed weights move 32 rows per DMA: with BN / 32 == NW every wave issues one packed-weight DMA and one scale
  // DMA; otherwise (8 waves, BN = 128) waves 4-7 the packed rows and waves 0-3 the scales
  static constexpr bool RAW_ALL = BN / 32 == NW;
  static constexpr int SC_BYTES = (RAW_ALL ? NW : 4) * 256;  // one scale stage: a 256-B slot per scale DMA wave
  // prefetch depth: X (and bf16 weight) tiles D K-steps ahead, packed weights D + 1 ahead. The 64-row tiles of
  // short prompts do little MFMA work per K-step, so they hide the DMA latency with depth instead (D = 4; the
  // 64 x 256 SwiGLU tile has no LDS for it)
  static constexpr int D = NW == 4 ? 1 : (BM == 64 && BN == 128 ? 4 : (BM == 256 && BN == 256 ? 1 : 2));
  static constexpr int NA = D + 1, NRAW = D + 2, NWB = 2;
  // LDS, 4-bit weights: A[NA] | RAW[NRAW] | SC[NRAW] | WB[2] | misc ; bf16 weights: A[NA] | B[NA] | misc
  static constexpr int OFF_RAW = NA * A_BYTES;
  static constexpr int OFF_SC = OFF_RAW + NRAW * RAW_BYTES;
  static constexpr int OFF_WB = OFF_SC + NRAW * SC_BYTES;
  static constexpr int END_Q4 = OFF_WB + NWB * B_BYTES;
  static constexpr int END_BF16 = NA * A_BYTES + NA * B_BYTES;
  static constexpr int OFF_MISC = END_Q4 > END_BF16 ? END_Q4 : END_BF16;  // nf4 table (64 B), last-arriver flag
  static constexpr int LDS_BYTES = OFF_MISC + 128;
  static constexpr int RPT = BN * BK / 2 / NTH;    // packed bytes each thread dequantizes (8 or 16)
  static constexpr int TPR = 32 / RPT;             // dequant threads per weight row
  // DMAs per wave per stage: X pieces (8 rows x 128 B); bf16 weight pieces; packed weight + scale DMAs
  static constexpr int APW = BM / (8 * NW), BPW = BN / (8 * NW), RAWPW = RAW_ALL ? 2 : 1;
  static_assert(WM * WN == NW && FJ >= 1 && RPT >= 8 && APW >= 1, "tile shape");
  static_assert(RAW_ALL || (NW == 8 && BN == 128), "packed-weight DMA roles");
  static_assert(LDS_BYTES <= (NW == 4 ? 81920 : 163840), "LDS budget (4 waves: two workgroups per CU)");
};

struct Args {
  const uint16_t* x;   // [M][K]
  const void* w;       // packed [N][K/2] (4-bit) or bf16 [N][K]
  const void* sc;      // [N][K/G]
  const void* w2;      // SwiGLU: fc_2's packed weight / scales
  const void* sc2;
  const uint16_t* bias;
  const uint16_t* residual;  // [M][N]
  uint16_t* y;               // [M][N]
  int M, N, K, G;
  int mt;                    // m-tiles
  int splits;                // K-slices per tile (1: no split)
  unsigned* counters;        // split-K: one per tile, zero between launches (the last arriver re-zeroes it)
  float* slabs;              // split-K: [splits][M][N] fp32 partial products
  int ldy = 0;               // row stride of y / residual (0: N) — a launch over a column range of a wider output
  int cb = 0;                // codebook row of kCode4 (FMT 1): 0 nf4, 1 fp4
  // grouped (sparse-MoE prefill, lga_q4_gemm_grouped): m-tile i of the launch is entry i of the device table grp =
  // {n_tiles, then (expert, first row, rows) per tile} built by lga_moe_group; its weights are expert e's
  // (w / w2 + e * ew bytes, sc / sc2 + e * es bytes); its X rows are gathered through xrow (null: contiguous) and
  // its Y rows scattered through yrow (null: contiguous). M bounds the row indices of the permuted list.
  const int32_t* grp = nullptr;
  const int32_t* xrow = nullptr;
  const int32_t* yrow = nullptr;
  long long ew = 0, es = 0;
};

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + 16 * (chunk ^ (row & 7)); }

// split-K slab traffic at agent coherence: 16-B buffer stores / loads with the sc1 cache-policy bit (write-through,
// past the L2: the form a relaxed agent-scope atomic takes), compiler-visible intrinsics so the vmcnt accounting
// stays exact; no fences are needed around them. Offsets are bytes from the slab base.
constexpr int kSc1 = 16;  // gfx940+ cache-policy aux bit SC1
__device__ __forceinline__ void st_wt16(__amdgpu_buffer_rsrc_t r, unsigned off, f32x4_t v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, kSc1);
}
__device__ __forceinline__ f32x4_t ld_wt16(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSc1));
}

// LDS byte address of a __shared__ pointer (the low 32 bits of its generic address)
__device__ __forceinline__ unsigned lds_addr(const void* p) { return (unsigned)(uintptr_t)p; }

// the four bytes of w as floats, one v_cvt_f32_ubyteN each (hipcc would otherwise extract each nibble first)
__device__ __forceinline__ void cvt_ubytes(uint32_t w, float (&f)[4]) {
  asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(f[0]) : "v"(w));
  asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(f[1]) : "v"(w));
  asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(f[2]) : "v"(w));
  asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(f[3]) : "v"(w));
}

template <int SIZE>
__device__ __forceinline__ void glds(const void* src, unsigned char* lds) {
  // the builtin's size must be a literal; an LDS-DMA lane slot is 4 bytes wide for the sub-dword sizes
  if constexpr (SIZE == 16) __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
  else __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
}

// s_waitcnt vmcnt(N) / vmcnt(N) lgkmcnt(0) for a compile-time N (the count is an encoding field)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 15, "vmcnt");
#define LGA_VM(n) \
  if constexpr (N == n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory");
  LGA_VM(0) LGA_VM(1) LGA_VM(2) LGA_VM(3) LGA_VM(4) LGA_VM(5) LGA_VM(6) LGA_VM(7) LGA_VM(8) LGA_VM(9) LGA_VM(10)
  LGA_VM(11) LGA_VM(12) LGA_VM(13) LGA_VM(14) LGA_VM(15)
#undef LGA_VM
}
template <int N>
__device__ __forceinline__ void wait_vm_lgkm() {
  wait_vm<N>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// 8 rows x 128 B of a row-major bf16 matrix into a swizzled tile: lane L lands at base + 16 L = row r0 + L/8,
// physical chunk L%8, so it fetches the logical chunk swz() maps there, (L%8) ^ (row & 7)
__device__ __forceinline__ void glds_rows8(const uint16_t* src, int ld, int row, int row_max, int k0,
                                           unsigned char* lds_rows, int lane) {
  const int r = row + (lane >> 3);
  const int lc = (lane & 7) ^ (r & 7);
  glds<16>(src + (size_t)min(r, row_max) * ld + k0 + lc * 8, lds_rows);
}

// FMT 0 int4-g (bf16 scales), 1 nf4 (fp32 absmax), 2 bf16 weights. DUAL: fc_1 || fc_2 + SwiGLU (tile = BN / 2
// columns of each; the weight tile's rows [0, BN/2) are fc_1's, [BN/2, BN) fc_2's).
template <int FMT, bool DUAL, int BM_, int BN_, int NW_ = 8>
__global__ void __launch_bounds__(NW_ * 64, NW_ == 4 ? 2 : 1) gemm_q4f_kernel(Args a) {
  if (a.grp) {  // grouped: this m-tile's expert and row range (surplus tiles of the launch's upper bound exit here)
    const int mi = (blockIdx.x / a.splits) % a.mt;
    if (mi >= a.grp[0]) return;
    const long long e = a.grp[1 + 3 * mi];
    a.w = (const unsigned char*)a.w + e * a.ew;
    if (a.sc) a.sc = (const unsigned char*)a.sc + e * a.es;
    if (DUAL) {
      a.w2 = (const unsigned char*)a.w2 + e * a.ew;
      if (a.sc2) a.sc2 = (const unsigned char*)a.sc2 + e * a.es;
    }
  }
  using T = Tile<BM_, BN_, NW_>;
  constexpr int BM = T::BM, BN = T::BN, NA = T::NA, NRAW = T::NRAW, FJ = T::FJ, WC = T::WC;
  constexpr int A_BYTES = T::A_BYTES, B_BYTES = T::B_BYTES, RAW_BYTES = T::RAW_BYTES, SC_BYTES = T::SC_BYTES;
  constexpr int OFF_RAW = T::OFF_RAW, OFF_SC = T::OFF_SC, OFF_WB = T::OFF_WB, OFF_MISC = T::OFF_MISC;
  static_assert(!DUAL || FJ % 2 == 0, "SwiGLU needs fc_1 and fc_2 fragments in pairs");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[T::LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  LGA_QTRACE(0);
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar branches on it)
  const int wm = wave % T::WM, wn = wave / T::WM;
  const int split = blockIdx.x % a.splits;
  const int tile = blockIdx.x / a.splits;
  // rows [m0, mend) of the (permuted) row list
  const int m0 = a.grp ? a.grp[2 + 3 * (tile % a.mt)] : (tile % a.mt) * BM;
  const int mend = a.grp ? m0 + a.grp[3 + 3 * (tile % a.mt)] : a.M;
  constexpr int TN = DUAL ? BN / 2 : BN;  // output columns per tile
  const int n0 = (tile / a.mt) * TN;
  const int nk_all = a.K / BK;
  const int per = (nk_all + a.splits - 1) / a.splits;
  const int kt0 = split * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);  // K-steps of this slice
  const int groups = a.K / (FMT == 2 ? 1 : a.G);
  const int gshift = FMT == 2 ? 0 : 31 - __builtin_clz((unsigned)a.G);
  float* tab = (float*)(lds + OFF_MISC);
  if (FMT == 1 && tid < 16) tab[tid] = kCode4[a.cb][tid];

  // the weight tile's row r -> (matrix, row)
  auto wrow_ptr = [&](int r) -> const unsigned char* {
    const unsigned char* base = (const unsigned char*)a.w;
    int n = n0 + r;
    if (DUAL && r >= BN / 2) {
      base = (const unsigned char*)a.w2;
      n = n0 + r - BN / 2;
    }
    n = min(n, a.N - 1);
    return base + (size_t)n * (FMT == 2 ? (size_t)a.K * 2 : (size_t)a.K / 2);
  };
  // scale index of weight-tile row r at K-step kt (global). The scale DMA moves 4 bytes per lane: a bf16 scale is
  // fetched with its neighbour from the 4-byte-aligned pair holding it (in bounds: N * groups is even) and the
  // reader picks the half by the index's parity.
  auto sc_index = [&](int r, int kt) -> size_t {
    int n = n0 + r;
    if (DUAL && r >= BN / 2) n = n0 + r - BN / 2;
    n = min(n, a.N - 1);
    return (size_t)n * groups + ((kt * BK) >> gshift);
  };

  // ---- stage issue; `lk` is the slice-local K-step (buffer index), kt0 + lk the global one. Every wave issues
  // the same number of DMAs per stage, so one count serves all. The per-lane source rows are fixed for the whole
  // loop: their pointers are computed once, a stage only adds its K offset. ----
  const unsigned char* xsrc[T::APW];  // X: lane L of piece i -> row r0 + L/8, logical chunk (L%8) ^ (row & 7)
#pragma unroll
  for (int i = 0; i < T::APW; ++i) {
    const int r = (wave * T::APW + i) * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ (r & 7);
    const int mr = min(m0 + r, mend - 1);
    xsrc[i] = (const unsigned char*)(a.x + (size_t)(a.xrow ? a.xrow[mr] : mr) * a.K + (size_t)kt0 * BK + lc * 8);
  }
  auto issue_a = [&](int lk) {
    unsigned char* A = lds + (lk % NA) * A_BYTES;
#pragma unroll
    for (int i = 0; i < T::APW; ++i) glds<16>(xsrc[i] + (size_t)lk * BK * 2, A + (wave * T::APW + i) * 8 * 128);
  };
  const unsigned char* bsrc[FMT == 2 ? T::BPW : 1];  // bf16 weights (FMT 2), the same mapping
  if (FMT == 2) {
#pragma unroll
    for (int i = 0; i < T::BPW; ++i) {
      const int r = (wave * T::BPW + i) * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ (r & 7);
      bsrc[i] = wrow_ptr(r) + (size_t)kt0 * BK * 2 + lc * 16;
    }
  }
  auto issue_b16 = [&](int lk) {  // bf16 weight tile (FMT 2)
    unsigned char* B = lds + NA * A_BYTES + (lk % NA) * B_BYTES;
#pragma unroll
    for (int i = 0; i < T::BPW; ++i) glds<16>(bsrc[i] + (size_t)lk * BK * 2, B + (wave * T::BPW + i) * 8 * 128);
  };
  // packed weight tile (1 KB = 32 rows x 32 B per DMA) and its scales (256 B = 64 rows x 4 B per DMA).
  // RAW_ALL (BN = 32 NW): every wave one of each (waves past BN / 64 repeat earlier scale blocks into their own
  // slots); 8 waves, BN = 128: waves 4-7 the packed rows, waves 0-3 the scales (2, 3 repeat 0, 1): one DMA per wave.
  const int raw_wave = T::RAW_ALL ? wave : wave - 4;
  const unsigned char* rsrc =
      wrow_ptr(max(raw_wave, 0) * 32 + (lane >> 1)) + (size_t)kt0 * (BK / 2) + (lane & 1) * 16;
  const int sw = wave & (BN / 64 - 1);  // the 64-row scale block this wave fetches
  const size_t sc_row = sc_index(sw * 64 + lane, 0);  // its scale index at K-step 0
  const unsigned char* sc_base = (const unsigned char*)(DUAL && sw * 64 + lane >= BN / 2 ? a.sc2 : a.sc);
  auto issue_raw = [&](int lk) {
    const int kt = kt0 + lk;
    unsigned char* R = lds + OFF_RAW + (lk % NRAW) * RAW_BYTES;
    unsigned char* S = lds + OFF_SC + (lk % NRAW) * SC_BYTES + wave * 256;
    const size_t si = sc_row + ((kt * BK) >> gshift);
    const unsigned char* sp = sc_base + (FMT == 0 ? (si & ~(size_t)1) * 2 : si * 4);
    if (T::RAW_ALL) {
      glds<16>(rsrc + (size_t)lk * (BK / 2), R + wave * 1024);
      glds<4>(sp, S);
    } else if (wave >= 4) {
      glds<16>(rsrc + (size_t)lk * (BK / 2), R + raw_wave * 1024);
    } else {
      glds<4>(sp, S);
    }
  };

  // ---- dequantization of packed stage lk into bf16 image buffer lk & 1 ----
  // thread -> weight-tile row dq_r, packed bytes [dq_q * RPT, +RPT) of its 32. The LDS reads / writes are inline
  // asm: their data is ordered by the counted vmcnt + barrier of the loop, and hipcc would otherwise drain every
  // LDS-DMA in flight (vmcnt(0)) before them, as it cannot tell the buffers apart. Split in three so the math can
  // sit between the MFMAs: the reads are issued before the K-step's first MFMA group, the image written after.
  constexpr int RPT = T::RPT, NDW = RPT / 4;
  const int dq_r = tid / T::TPR, dq_q = tid % T::TPR;
  const size_t dq_row0 = FMT == 2 ? 0 : sc_index(dq_r, 0);  // the row's scale index at K-step 0 (parity source)
  typedef uint32_t raw_t __attribute__((ext_vector_type(NDW)));
  auto dq_load = [&](int lk, raw_t& wv, uint32_t& sb) {
    const unsigned raw_a = lds_addr(lds + OFF_RAW + (lk % NRAW) * RAW_BYTES + dq_r * 32 + dq_q * RPT);
    // the scale of row r sits in the slot of the wave that fetched its 64-row block (wave r / 64)
    const unsigned sc_a = lds_addr(lds + OFF_SC + (lk % NRAW) * SC_BYTES + (dq_r >> 6) * 256 + (dq_r & 63) * 4 +
                                   (FMT == 0 ? (int)((dq_row0 + (((kt0 + lk) * BK) >> gshift)) & 1) * 2 : 0));
    if constexpr (NDW == 4) {
      if (FMT == 0)
        asm volatile("ds_read_b128 %0, %2\n\tds_read_u16 %1, %3" : "=&v"(wv), "=&v"(sb) : "v"(raw_a), "v"(sc_a) : "memory");
      else
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b32 %1, %3" : "=&v"(wv), "=&v"(sb) : "v"(raw_a), "v"(sc_a) : "memory");
    } else if constexpr (NDW == 2) {
      if (FMT == 0)
        asm volatile("ds_read_b64 %0, %2\n\tds_read_u16 %1, %3" : "=&v"(wv), "=&v"(sb) : "v"(raw_a), "v"(sc_a) : "memory");
      else
        asm volatile("ds_read_b64 %0, %2\n\tds_read_b32 %1, %3" : "=&v"(wv), "=&v"(sb) : "v"(raw_a), "v"(sc_a) : "memory");
    }
  };
  auto dq_wait = [&](raw_t& wv, uint32_t& sb) {  // ties the values to the wait so no use moves above it
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wv), "+v"(sb) :: "memory");
  };
  auto dq_math = [&](const raw_t wv, uint32_t sb, uint32_t (&o)[4 * NDW]) {
    const float s = FMT == 0 ? __uint_as_float(sb << 16) : __uint_as_float(sb);
    const float c = -8.0f * s;
#pragma unroll
    for (int h = 0; h < NDW; ++h) {
      const uint32_t w = wv[h];
      if (FMT == 0) {
        // even elements in the bytes of lo, odd in hi: one v_cvt_f32_ubyteN per weight, fma(n, s, -8 s) exact
        const uint32_t lo = w & 0x0F0F0F0Fu, hi = (w >> 4) & 0x0F0F0F0Fu;
        float fl[4], fh[4];
        cvt_ubytes(lo, fl);
        cvt_ubytes(hi, fh);
#pragma unroll
        for (int e = 0; e < 4; ++e) o[4 * h + e] = pack2(__builtin_fmaf(fl[e], s, c), __builtin_fmaf(fh[e], s, c));
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t nl = (w >> (8 * e)) & 0xFu, nh = (w >> (8 * e + 4)) & 0xFu;
          o[4 * h + e] = pack2(__fmul_rn(tab[nl], s), __fmul_rn(tab[nh], s));
        }
      }
    }
  };
  auto dq_store = [&](int lk, const uint32_t (&o)[4 * NDW]) {
    unsigned char* WB = lds + OFF_WB + (lk & 1) * B_BYTES;
    {
#pragma unroll
      for (int h = 0; h < NDW; ++h) {  // 16-B chunk (dq_q * NDW + h) of the 128-B bf16 row
        const unsigned wa = lds_addr(WB + swz(dq_r, dq_q * NDW + h));
        const u32x4 ov = {o[4 * h], o[4 * h + 1], o[4 * h + 2], o[4 * h + 3]};
        asm volatile("ds_write_b128 %0, %1" :: "v"(wa), "v"(ov) : "memory");
      }
    }
  };
  auto dequant = [&](int lk) {
    raw_t wv;
    uint32_t sb, o[4 * NDW];
    dq_load(lk, wv, sb);
    dq_wait(wv, sb);
    dq_math(wv, sb, o);
    dq_store(lk, o);
  };

  // accumulators: acc[j][i] = weight rows (fragment j) x X rows (fragment i) of this wave
  f32x4_t acc[FJ][4];
#pragma unroll
  for (int j = 0; j < FJ; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fk = lane >> 4;
  // weight-tile row of fragment j (SwiGLU: the first FJ/2 fragments are fc_1 rows, the rest the same fc_2 rows)
  auto brow = [&](int j) {
    return DUAL ? (j / (FJ / 2)) * (BN / 2) + wn * (WC / 2) + (j % (FJ / 2)) * 16 : wn * WC + j * 16;
  };
  // a K-step's fragments, per 32-deep sub: weight rows (A operand) and X rows (B operand) of this wave
  struct Frags {
    bf16x8_t af[4], bfr[FJ];
  };
  auto frag_read = [&](const unsigned char* A, const unsigned char* B, int sub, Frags& f) {
#pragma unroll
    for (int j = 0; j < FJ; ++j) f.bfr[j] = *(const bf16x8_t*)(B + swz(brow(j) + fr, sub * 4 + fk));
#pragma unroll
    for (int i = 0; i < 4; ++i) f.af[i] = *(const bf16x8_t*)(A + swz(wm * 64 + i * 16 + fr, sub * 4 + fk));
  };
  auto frag_mfma = [&](const Frags& f) {
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.bfr[j], f.af[i], acc[j][i], 0, 0, 0);
  };

  constexpr int D = T::D;
  if (nk > 0) {
    if (FMT == 2) {
      // X and W both DMA'd D K-steps ahead into D + 1 buffers: G = APW + BPW DMAs per wave per stage; at the end
      // of step lk the stages lk+2 .. lk+D may stay in flight
      constexpr int G = T::APW + T::BPW;
#pragma unroll
      for (int st = 0; st < D; ++st)
        if (st < nk) {
          issue_a(st);
          issue_b16(st);
        }
      if (nk >= D) wait_vm<(D - 1) * G>();
      else wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      for (int lk = 0; lk < nk; ++lk) {  // the schedule of the 4-bit loop below, without the dequantization
        const bool full = lk + D < nk;
        const unsigned char* A = lds + (lk % NA) * A_BYTES;
        const unsigned char* B = lds + NA * A_BYTES + (lk % NA) * B_BYTES;
        Frags f0, f1;
        frag_read(A, B, 0, f0);
        __builtin_amdgcn_sched_barrier(0);
        if (full) {
          issue_a(lk + D);
          issue_b16(lk + D);
        }
        __builtin_amdgcn_sched_barrier(0);
        frag_read(A, B, 1, f1);
        frag_mfma(f0);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        frag_mfma(f1);
        if (full) wait_vm_lgkm<(D - 1) * G>();
        else wait_vm_lgkm<0>();
        __builtin_amdgcn_s_barrier();
      }
    } else {
      // G = APW + RAWPW DMAs per wave per group; group g = {A(g), raw(g+1)} (raw(0) rides with group 0), issued
      // D groups ahead. Prologue: groups 0 .. D-1; raw(0) -> WB0 once group 0 has landed
      constexpr int G = T::APW + T::RAWPW;
      issue_a(0);
      issue_raw(0);
      if (nk > 1) issue_raw(1);
#pragma unroll
      for (int g = 1; g < D; ++g) {
        if (g < nk) issue_a(g);
        if (g + 1 < nk) issue_raw(g + 1);
      }
      if (D < nk) wait_vm<(D - 1) * G>();  // groups 1 .. D-1 all full
      else wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      dequant(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      LGA_QTRACE(1);
      // iteration lk: the dequant reads of raw(lk+1) and sub 0's 8 fragment reads; group lk+D {A(lk+D),
      // raw(lk+D+1)} issued under their latency (it fills buffers read one step earlier); sub 0's 16 MFMAs with
      // sub 1's 8 reads two per 4 MFMAs; raw(lk+1) dequantized between them and sub 1's MFMAs; WB(lk+1) stored;
      // wait for group lk+1 and the LDS traffic; barrier. Past the last stage the dequantization reads a stale raw
      // buffer into the bf16 buffer nobody reads again (no branch). sched_barrier / sched_group_barrier pin the
      // order: hipcc would otherwise sink the reads next to their MFMAs (one LDS round trip exposed per 4 MFMAs),
      // and with at most 10 LDS reads in flight its counted lgkmcnt stays exact (the inline-asm dequant reads are
      // older than every fragment read they could be confused with).
#ifndef LGA_Q4F_EXP
#define LGA_Q4F_EXP 0  // lab only (tools/gemm_rates.py A/B): 1 no MFMAs, 2 no dequantization, 4 no fragment reads
#endif
      // (lab) the MFMAs' stand-in: an empty asm that keeps the fragment reads alive
      auto use = [&](const Frags& f) {
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(f.af[i]));
#pragma unroll
        for (int j = 0; j < FJ; ++j) asm volatile("" ::"v"(f.bfr[j]));
      };
      for (int lk = 0; lk < nk; ++lk) {
        const bool full = lk + D + 1 < nk;
        const unsigned char* A = lds + (lk % NA) * A_BYTES;
        const unsigned char* B = lds + OFF_WB + (lk & 1) * B_BYTES;
        raw_t wv;
        uint32_t sb, o[4 * NDW];
        Frags f0, f1;
        if (!(LGA_Q4F_EXP & 2)) dq_load(lk + 1, wv, sb);
        __builtin_amdgcn_sched_barrier(0);
        if (!(LGA_Q4F_EXP & 4)) frag_read(A, B, 0, f0);
        else f0 = Frags{};
        __builtin_amdgcn_sched_barrier(0);
        if (lk + D < nk) issue_a(lk + D);
        if (full) issue_raw(lk + D + 1);
        __builtin_amdgcn_sched_barrier(0);
        if (!(LGA_Q4F_EXP & 4)) frag_read(A, B, 1, f1);
        else f1 = Frags{};
        if (LGA_Q4F_EXP & 1) use(f0);
        else frag_mfma(f0);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // 4 MFMAs
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // 2 LDS reads
        }
        __builtin_amdgcn_sched_barrier(0);
        if (!(LGA_Q4F_EXP & 2)) {
          dq_wait(wv, sb);
          dq_math(wv, sb, o);
        }
        if (LGA_Q4F_EXP & 1) use(f1);
        else frag_mfma(f1);
        if (!(LGA_Q4F_EXP & 2)) dq_store(lk + 1, o);
        if (full) wait_vm_lgkm<(D - 1) * G>();  // groups lk+2 .. lk+D, all full
        else wait_vm_lgkm<0>();
        __builtin_amdgcn_s_barrier();
      }
    }
  }

  LGA_QTRACE(2);
  // ---- split-K: slabs, then the tile's last slice sums them in slice order ----
  if (a.splits > 1) {
    constexpr int NJ = FJ;
    const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
        a.slabs, (short)0, (int)((size_t)a.splits * (DUAL ? 2 : 1) * a.M * a.N * 4), 0x00020000);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      // column in the slab's [N] (SwiGLU: fc_1 and fc_2 partials side by side, [2][M][N])
      const int jj = DUAL ? j % (FJ / 2) : j;
      const int n = n0 + (DUAL ? wn * (WC / 2) : wn * WC) + jj * 16 + fk * 4;
      if (n >= a.N) continue;
      const size_t slab = ((size_t)split * (DUAL ? 2 : 1) + (DUAL ? j / (FJ / 2) : 0)) * a.M * a.N;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 64 + i * 16 + fr;
        if (m < a.M) st_wt16(srs, (unsigned)((slab + (size_t)m * a.N + n) * 4), acc[j][i]);
      }
    }
    // the slabs went out write-through (sc1): drained, they are visible to the tile's last slice, which reads them
    // with sc1 loads — no agent release / acquire fences (an L2 write-back per slice and an invalidate per tile).
    // This is the hardware form, not the HIP memory model's: MI355X_MICROARCH.md "Valid forms", Consumer bullet —
    // sc1 buffer loads may replace the acquire when (1) every load of the slab bytes is such a load, (2) every slab
    // byte was stored sc1, (3) every storing wave waited vmcnt(0) and the counter add follows the workgroup barrier
    // behind all of them, (4) the hand-off is agent-scope on one device. All four hold here; the bitwise split-K
    // stress test (tests/test_gpu_gemm_fused.py::test_fused_gemm_split_k_handoff_stress) checks the result.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned* last = (unsigned*)(lds + OFF_MISC + 64);
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(a.counters + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool is_last = old == (unsigned)a.splits - 1;
      if (is_last) __hip_atomic_store(a.counters + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
      *last = is_last ? 1u : 0u;
    }
    __syncthreads();
    if (*last == 0u) return;
    // every slab value of one output fragment is loaded before any is summed (MAX_SPLITS loads in flight, the
    // index clamped and the surplus weighted by zero: no branch around a load), summed in slice order
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int jj = DUAL ? j % (FJ / 2) : j;
      const int n = min(n0 + (DUAL ? wn * (WC / 2) : wn * WC) + jj * 16 + fk * 4, a.N - 4);
      const size_t mat = DUAL ? j / (FJ / 2) : 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = min(m0 + wm * 64 + i * 16 + fr, a.M - 1);
        f32x4_t v[MAX_SPLITS];
#pragma unroll
        for (int s2 = 0; s2 < MAX_SPLITS; ++s2) {
          const int sc = min(s2, a.splits - 1);
          const size_t slab = ((size_t)sc * (DUAL ? 2 : 1) + mat) * a.M * a.N;
          v[s2] = ld_wt16(srs, (unsigned)((slab + (size_t)m * a.N + n) * 4));
        }
        f32x4_t t = v[0];
#pragma unroll
        for (int s2 = 1; s2 < MAX_SPLITS; ++s2) t += s2 < a.splits ? v[s2] : f32x4_t{0.f, 0.f, 0.f, 0.f};
        acc[j][i] = t;
      }
    }
  }

  // ---- epilogue: lane holds columns (fk * 4 + r) of weight fragment j for X row fr of fragment i ----
  const size_t ldy = a.ldy ? a.ldy : a.N;
  if (DUAL) {
#pragma unroll
    for (int j = 0; j < FJ / 2; ++j) {
      const int n = n0 + wn * (WC / 2) + j * 16 + fk * 4;
      if (n >= a.N) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 64 + i * 16 + fr;
        if (m >= mend) continue;
        const size_t my = a.yrow ? (size_t)a.yrow[m] : (size_t)m;
        uint32_t o[2];
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          float g[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const float gate = round_bf(silu_f(round_bf(acc[j][i][r + e])));  // bf16(silu(bf16(fc_1 x)))
            g[e] = __fmul_rn(gate, round_bf(acc[j + FJ / 2][i][r + e]));      // * bf16(fc_2 x)
          }
          o[r / 2] = pack2(g[0], g[1]);
        }
        *(uint2*)(a.y + my * ldy + n) = make_uint2(o[0], o[1]);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int n = n0 + wn * WC + j * 16 + fk * 4;
      if (n >= a.N) continue;
      float b[4] = {0.f, 0.f, 0.f, 0.f};
      if (a.bias) {
        const uint2 bv = *(const uint2*)(a.bias + n);
        b[0] = bflo(bv.x), b[1] = bfhi(bv.x), b[2] = bflo(bv.y), b[3] = bfhi(bv.y);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 64 + i * 16 + fr;
        if (m >= mend) continue;
        const size_t my = a.yrow ? (size_t)a.yrow[m] : (size_t)m;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[j][i][r] + b[r];
        if (a.residual) {  // bf16(bf16(x W^T + b) + residual): Block's `x + attn(...)` after the Linear's rounding
          const uint2 rv = *(const uint2*)(a.residual + my * ldy + n);
          v[0] = round_bf(v[0]) + bflo(rv.x);
          v[1] = round_bf(v[1]) + bfhi(rv.x);
          v[2] = round_bf(v[2]) + bflo(rv.y);
          v[3] = round_bf(v[3]) + bfhi(rv.y);
        }
        *(uint2*)(a.y + my * ldy + n) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
    }
  }
#ifdef LGA_Q4F_TRACE
  if (tid == 0) __builtin_amdgcn_s_waitcnt(0);  // thread 0's epilogue stores retired
#endif
  LGA_QTRACE(3);
}

}  // namespace pf
}  // namespace lga

namespace {
using lga::pf::Args;

// the fused kernel's shape contract (the callers fall back to gemm.hip's 128 x 128 tiles outside it)
bool q4f_fits(int M, int N, int K, int group, int fmt) {
  if (M < 1 || N < 8 || N % 8 || K < lga::pf::BK || K % lga::pf::BK) return false;
  if (fmt == 2) return true;
  return group >= lga::pf::BK && (group & (group - 1)) == 0 && K % group == 0;
}

// the 4-wave 128 x 128 tile for M > 128: lab builds only (make lab-lib LABFLAGS=-DLGA_Q4F_W4_LAB), then LGA_Q4F_W4=1
bool w4_tiles() {
#ifdef LGA_Q4F_W4_LAB
  static const bool on = [] {
    const char* e = getenv("LGA_Q4F_W4");
    return e && atoi(e) == 1;
  }();
  return on;
#else
  return false;
#endif
}

// Launch plan: tile shape by M, then K-slices so the grid covers the CUs (>= 2 waves of tiles is left whole).
struct Plan {
  int bm, bn, mt, tn, tiles, splits;
};
Plan q4f_plan(int M, int N, int K, bool dual) {
  Plan p;
  p.bm = M <= 128 ? 64 : (w4_tiles() ? 128 : 256);
  p.bn = p.bm == 64 ? (dual ? 256 : 128) : 128;
  if (p.bm == 256) {
    // 256 x 256 tiles (64 x 128 outputs per wave: a third less LDS fragment traffic per FLOP) where their rounds
    // fill the CUs: a 256 x 256 tile-round costs ~1.74 256 x 128 tile-rounds (tools/gemm_rates.py: qkv 261 us in
    // 1.5 big rounds vs 237 in 3 small; fc_1 || fc_2 368 in 2.7 big vs 413 in 5.4 small)
    const int mt = (M + 255) / 256;
    const long small = (long)mt * ((N + (dual ? 63 : 127)) / (dual ? 64 : 128));
    const long big = (long)mt * ((N + (dual ? 127 : 255)) / (dual ? 128 : 256));
    if ((big + 255) / 256 * 174 < (small + 255) / 256 * 100) p.bn = 256;
    if (const char* e = getenv("LGA_Q4F_BN")) p.bn = atoi(e) == 256 ? 256 : 128;
  }
  p.mt = (M + p.bm - 1) / p.bm;
  p.tn = dual ? p.bn / 2 : p.bn;
  p.tiles = p.mt * ((N + p.tn - 1) / p.tn);
  const int nk = K / lga::pf::BK;
  int s = 1;
  // each slice keeps >= 4 K-steps; aim at one workgroup per CU
  while (p.tiles * s * 2 <= 256 && nk / (s * 2) >= 4 && s * 2 <= lga::pf::MAX_SPLITS) s *= 2;
  if (const char* e = getenv("LGA_Q4F_SPLITS")) s = std::max(1, std::min({atoi(e), nk, lga::pf::MAX_SPLITS}));
  p.splits = s;
  return p;
}

template <int FMT, bool DUAL, int BM, int BN, int NW = 8>
int launch_tile(Args a, const Plan& p, hipStream_t stream) {
  a.mt = p.mt;
  a.splits = p.splits;
  const unsigned grid = (unsigned)(p.tiles * p.splits);
  lga::pf::gemm_q4f_kernel<FMT, DUAL, BM, BN, NW><<<grid, NW * 64, 0, stream>>>(a);
  LGA_LAUNCH_RETURN();
}

template <int FMT, bool DUAL>
int launch_q4f(Args a, const Plan& p, hipStream_t stream) {
#ifdef LGA_Q4F_W4_LAB
  if (p.bm == 128) return launch_tile<FMT, DUAL, 128, 128, 4>(a, p, stream);
#endif
  if (p.bm == 256 && p.bn == 256) return launch_tile<FMT, DUAL, 256, 256>(a, p, stream);
  if (p.bm == 256) return launch_tile<FMT, DUAL, 256, 128>(a, p, stream);
  if (DUAL || p.bn == 256) return launch_tile<FMT, DUAL, 64, 256>(a, p, stream);
  return launch_tile<FMT, false, 64, 128>(a, p, stream);
}

size_t ws_need(const Plan& p, int M, int N, bool dual) {
  if (p.splits == 1) return 0;
  return 4096 + (size_t)p.splits * (dual ? 2 : 1) * M * N * 4;
}

// Long prompts, one weight matrix: the first columns as whole rounds of 256 x 256 tiles, the rest as 256 x 128 —
// two launches over column ranges of the same output (Llama-2-7B qkv at 2048 tokens: one big round over 8192 columns
// + one small round over 4096, instead of three small rounds). Returns the big-tile column count (0: no split).
int q4f_big_columns(int M, int N, int K) {
  if (M <= 128 || getenv("LGA_Q4F_BN") || w4_tiles()) return 0;
  const int mt = (M + 255) / 256;
  if (256 % mt || K / lga::pf::BK < 8) return 0;
  const int cols_per_round = 256 / mt * 256;
  auto rounds = [](long tiles) { return (tiles + 255) / 256; };
  const long small_only = rounds((long)mt * ((N + 127) / 128)) * 100;
  long best = small_only;
  int best_cols = 0;
  for (int rb = 1; (long)rb * cols_per_round < N; ++rb) {
    const long cost = rb * 174L + rounds((long)mt * ((N - rb * cols_per_round + 127) / 128)) * 100;
    if (cost < best) {
      best = cost;
      best_cols = rb * cols_per_round;
    }
  }
  return best_cols;
}

int run_tiles(Args a, int fmt, bool dual, int bn, hipStream_t stream);

int run(Args a, int fmt, bool dual, void* ws, size_t ws_bytes, hipStream_t stream) {
  if (!dual) {
    const int nb = q4f_big_columns(a.M, a.N, a.K);
    if (nb > 0) {
      const int kf = lga::kernel_fmt(fmt);
      const size_t row_bytes = kf == 2 ? (size_t)a.K * 2 : (size_t)a.K / 2;
      const size_t sc_bytes = kf == 2 ? 0 : (size_t)(a.K / a.G) * (kf == 0 ? 2 : 4);
      Args b = a, c = a;
      b.N = nb;
      b.ldy = a.N;
      c.N = a.N - nb;
      c.ldy = a.N;
      c.w = (const unsigned char*)a.w + (size_t)nb * row_bytes;
      if (sc_bytes) c.sc = (const unsigned char*)a.sc + (size_t)nb * sc_bytes;
      if (a.bias) c.bias = a.bias + nb;
      if (a.residual) c.residual = a.residual + nb;
      c.y = a.y + nb;
      const int rc = run_tiles(b, fmt, false, 256, stream);
      return rc ? rc : run_tiles(c, fmt, false, 128, stream);
    }
  }
  const Plan p = q4f_plan(a.M, a.N, a.K, dual);
  if (p.splits > 1) {
    LGA_CHECK_ARG(ws && ws_bytes >= ws_need(p, a.M, a.N, dual) && p.tiles <= 1024,
                  "lga_q4_gemm_fused: split-K needs the workspace lga_q4f_workspace_bytes reports");
    a.counters = (unsigned*)ws;
    a.slabs = (float*)((unsigned char*)ws + 4096);
  }
  a.cb = lga::codebook_of(fmt);
  switch (lga::kernel_fmt(fmt) * 2 + (dual ? 1 : 0)) {
    case 0: return launch_q4f<0, false>(a, p, stream);
    case 1: return launch_q4f<0, true>(a, p, stream);
    case 2: return launch_q4f<1, false>(a, p, stream);
    case 3: return launch_q4f<1, true>(a, p, stream);
    case 4: return launch_q4f<2, false>(a, p, stream);
    default: return launch_q4f<2, true>(a, p, stream);
  }
}
// one launch over the tiles of a (sub-)problem with a fixed tile width, no split-K (long prompts only)
int run_tiles(Args a, int fmt, bool dual, int bn, hipStream_t stream) {
  Plan p;
  p.bm = 256;
  p.bn = bn;
  p.mt = (a.M + 255) / 256;
  p.tn = dual ? bn / 2 : bn;
  p.tiles = p.mt * ((a.N + p.tn - 1) / p.tn);
  p.splits = 1;
  a.cb = lga::codebook_of(fmt);
  switch (lga::kernel_fmt(fmt) * 2 + (dual ? 1 : 0)) {
    case 0: return launch_q4f<0, false>(a, p, stream);
    case 1: return launch_q4f<0, true>(a, p, stream);
    case 2: return launch_q4f<1, false>(a, p, stream);
    case 3: return launch_q4f<1, true>(a, p, stream);
    case 4: return launch_q4f<2, false>(a, p, stream);
    default: return launch_q4f<2, true>(a, p, stream);
  }
}
}  // namespace

int lga::preload_gemm_q4f() {
  using namespace lga::pf;
  int bad = 0;
#define LGA_PRE(F, D)                                                                                         \
  bad += lga::preload(gemm_q4f_kernel<F, D, 256, 128>) + lga::preload(gemm_q4f_kernel<F, D, 256, 256>) +  \
         lga::preload(gemm_q4f_kernel<F, D, 64, 256>) +                                                  \
         lga::preload(gemm_q4f_kernel<F, false, 64, 128>)
  LGA_PRE(0, false);
  LGA_PRE(0, true);
  LGA_PRE(1, false);
  LGA_PRE(1, true);
  LGA_PRE(2, false);
  LGA_PRE(2, true);
#undef LGA_PRE
  return bad;
}

#ifdef LGA_Q4F_TRACE
extern "C" int lga_q4f_trace_read(unsigned long long* host, int n) {
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(lga::pf::g_q4f_trace), (size_t)n * sizeof(unsigned long long));
  void* dptr = nullptr;
  if (e == hipSuccess) e = hipGetSymbolAddress(&dptr, HIP_SYMBOL(lga::pf::g_q4f_trace));
  if (e == hipSuccess) e = hipMemset(dptr, 0, sizeof(lga::pf::g_q4f_trace));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}
#endif

extern "C" int lga_q4f_fits(int M, int N, int K, int group, int fmt) { return q4f_fits(M, N, K, group, fmt) ? 1 : 0; }

extern "C" size_t lga_q4f_workspace_bytes(int M, int N, int K, int swiglu) {
  if (M < 1 || N < 1 || K < lga::pf::BK) return 0;
  const Plan p = q4f_plan(M, N, K, swiglu != 0);
  return ws_need(p, M, N, swiglu != 0);
}

extern "C" int lga_q4_gemm_fused(const void* x, const void* weight, const void* scales, const void* bias,
                                 const void* residual, void* y, int M, int N, int K, int group, int fmt,
                                 void* workspace, size_t workspace_bytes, hipStream_t stream) {
  LGA_CHECK_ARG(x && weight && y && (fmt == 2 || scales), "lga_q4_gemm_fused: null pointer");
  LGA_CHECK_ARG(fmt >= 0 && fmt <= 3, "lga_q4_gemm_fused: fmt must be 0 (int4-g), 1 (nf4), 2 (bf16) or 3 (fp4)");
  LGA_CHECK_ARG(q4f_fits(M, N, K, group, fmt),
                "lga_q4_gemm_fused: needs N % 8 == 0, K % 64 == 0 and a power-of-two group >= 64 dividing K");
  LGA_CHECK_ARG(((uintptr_t)x | (uintptr_t)weight | (uintptr_t)y | (uintptr_t)residual) % 16 == 0,
                "lga_q4_gemm_fused: x, weight, residual and y must be 16-B aligned");
  Args a{(const uint16_t*)x, weight, scales, nullptr, nullptr, (const uint16_t*)bias, (const uint16_t*)residual,
         (uint16_t*)y, M, N, K, fmt == 2 ? 64 : group, 1, 1, nullptr, nullptr};
  return run(a, fmt, false, workspace, workspace_bytes, stream);
}

extern "C" int lga_q4_gemm_swiglu(const void* x, const void* qw1, const void* sc1, const void* qw2, const void* sc2,
                                  void* y, int M, int N, int K, int group, int fmt, void* workspace,
                                  size_t workspace_bytes, hipStream_t stream) {
  LGA_CHECK_ARG(x && qw1 && qw2 && y && (fmt == 2 || (sc1 && sc2)), "lga_q4_gemm_swiglu: null pointer");
  LGA_CHECK_ARG(fmt >= 0 && fmt <= 3, "lga_q4_gemm_swiglu: fmt must be 0 (int4-g), 1 (nf4), 2 (bf16) or 3 (fp4)");
  LGA_CHECK_ARG(q4f_fits(M, N, K, group, fmt),
                "lga_q4_gemm_swiglu: needs N % 8 == 0, K % 64 == 0 and a power-of-two group >= 64 dividing K");
  LGA_CHECK_ARG(((uintptr_t)x | (uintptr_t)qw1 | (uintptr_t)qw2 | (uintptr_t)y) % 16 == 0,
                "lga_q4_gemm_swiglu: x, weights and y must be 16-B aligned");
  Args a{(const uint16_t*)x, qw1, sc1, qw2, sc2, nullptr, nullptr, (uint16_t*)y, M, N, K, fmt == 2 ? 64 : group, 1,
         1, nullptr, nullptr};
  return run(a, fmt, true, workspace, workspace_bytes, stream);
}

// ---- grouped (sparse-MoE prefill): every active expert's rows in ONE launch ------------------------------------
// Replaces the reference's per-expert loop of LLaMAMoE.forward for T > 1 (lit_gpt/model.py:740-742: for each expert,
// torch.where(indices == e), then expert(x[token_idx]) — fc_1, fc_2, silu * mul, proj — on the gathered rows) by two
// launches over a device-built tile table (lga_moe_group): no host synchronisation, no gathered or scattered copies.
namespace {
int run_grouped(Args a, int fmt, bool dual, int bm, int max_tiles, hipStream_t stream) {
  Plan p;
  p.bm = bm;
  // 256 x 256 tiles once the routed rows are many (one Mixtral block, bit-identical: T = 8192 prefill 9.09 -> 8.52 ms,
  // T = 32000 43.9 -> 38.5 ms; at T = 2048, 8192 rows, 2.70 vs 2.79 ms: 256 x 128 stays; tools/moe_prefill_ab.py)
  p.bn = (bm == 64 && dual) || (bm == 256 && a.M > 8192) ? 256 : 128;
  if (const char* e = getenv("LGA_GROUPED_BN")) {  // lab A/B: force the column width of the bm = 256 tiles
    if (bm == 256 && (atoi(e) == 128 || atoi(e) == 256)) p.bn = atoi(e);
  }
  p.mt = max_tiles;
  p.tn = dual ? p.bn / 2 : p.bn;
  p.tiles = p.mt * ((a.N + p.tn - 1) / p.tn);
  p.splits = 1;
  a.cb = lga::codebook_of(fmt);
  switch (lga::kernel_fmt(fmt) * 2 + (dual ? 1 : 0)) {
    case 0: return launch_q4f<0, false>(a, p, stream);
    case 1: return launch_q4f<0, true>(a, p, stream);
    case 2: return launch_q4f<1, false>(a, p, stream);
    case 3: return launch_q4f<1, true>(a, p, stream);
    case 4: return launch_q4f<2, false>(a, p, stream);
    default: return launch_q4f<2, true>(a, p, stream);
  }
}
}  // namespace

// upper bound on the m-tiles of `rows` permuted rows over n_expert groups (the tile table's capacity)
extern "C" int lga_moe_group_tiles(int rows, int n_expert, int bm) {
  return bm > 0 ? (rows + bm - 1) / bm + n_expert : 0;
}

extern "C" int lga_q4_gemm_grouped(const void* x, const void* weight, const void* scales, long long w_stride,
                                   long long s_stride, const int32_t* tiles, const int32_t* x_rows,
                                   const int32_t* y_rows, void* y, int rows, int N, int K, int group, int fmt, int bm,
                                   int n_expert, hipStream_t stream) {
  LGA_CHECK_ARG(x && weight && y && tiles && (fmt == 2 || scales), "lga_q4_gemm_grouped: null pointer");
  LGA_CHECK_ARG(fmt >= 0 && fmt <= 3 && (bm == 64 || bm == 256) && n_expert > 0 && rows > 0,
                "lga_q4_gemm_grouped: fmt 0-3, bm 64 or 256");
  LGA_CHECK_ARG(q4f_fits(rows, N, K, group, fmt), "lga_q4_gemm_grouped: needs N % 8 == 0, K % 64 == 0, group >= 64");
  Args a{(const uint16_t*)x, weight, scales, nullptr, nullptr, nullptr, nullptr, (uint16_t*)y, rows, N, K,
         fmt == 2 ? 64 : group, 1, 1, nullptr, nullptr};
  a.grp = tiles;
  a.xrow = x_rows;
  a.yrow = y_rows;
  a.ew = w_stride;
  a.es = s_stride;
  return run_grouped(a, fmt, false, bm, lga_moe_group_tiles(rows, n_expert, bm), stream);
}

extern "C" int lga_q4_gemm_swiglu_grouped(const void* x, const void* qw1, const void* sc1, const void* qw2,
                                          const void* sc2, long long w_stride, long long s_stride,
                                          const int32_t* tiles, const int32_t* x_rows, void* y, int rows, int N,
                                          int K, int group, int fmt, int bm, int n_expert, hipStream_t stream) {
  LGA_CHECK_ARG(x && qw1 && qw2 && y && tiles && (fmt == 2 || (sc1 && sc2)), "lga_q4_gemm_swiglu_grouped: null pointer");
  LGA_CHECK_ARG(fmt >= 0 && fmt <= 3 && (bm == 64 || bm == 256) && n_expert > 0 && rows > 0,
                "lga_q4_gemm_swiglu_grouped: fmt 0-3, bm 64 or 256");
  LGA_CHECK_ARG(q4f_fits(rows, N, K, group, fmt),
                "lga_q4_gemm_swiglu_grouped: needs N % 8 == 0, K % 64 == 0, group >= 64");
  Args a{(const uint16_t*)x, qw1, sc1, qw2, sc2, nullptr, nullptr, (uint16_t*)y, rows, N, K, fmt == 2 ? 64 : group, 1,
         1, nullptr, nullptr};
  a.grp = tiles;
  a.xrow = x_rows;
  a.ew = w_stride;
  a.es = s_stride;
  return run_grouped(a, fmt, true, bm, lga_moe_group_tiles(rows, n_expert, bm), stream);
}
