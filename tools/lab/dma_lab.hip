// LDS-DMA streaming micro-benchmark (lab, not product): every CU's loader wave(s) stream a private contiguous region
// into an LDS ring with global_load_lds_dwordx4, keeping DEPTH lines in flight. Prints chip-wide GB/s per variant.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int DEPTH, int AUX>
__device__ __forceinline__ void glds(const void* src, unsigned dst) {
  unsigned keep;
  if (AUX == 2)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
}

// LW loader waves per workgroup, each streams lines w, w+LW, ... of the CU's region
template <int DEPTH, int AUX, int LW>
__global__ void __launch_bounds__(LW * 64) stream_kernel(const unsigned char* buf, size_t per_cu, int nl_ring, unsigned* sink) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned char* base = buf + (size_t)blockIdx.x * per_cu + lane * 16;
  const unsigned ring = (unsigned)(uintptr_t)smem;
  const int lines = (int)(per_cu / 1024);
  for (int i = w; i < lines; i += LW) {
    glds<DEPTH, AUX>(base + (size_t)i * 1024, __builtin_amdgcn_readfirstlane(ring + (unsigned)((i % nl_ring) * 1024)));
    if (i >= DEPTH * LW) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0 && ((unsigned*)smem)[5] == 0xdeadbeefu) sink[0] = 1;
}

// reference: plain register loads, 16 B per lane, all waves of a 256-thread block, 8 loads in flight per lane
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) regload_kernel(const u32x4_t* buf, size_t n16, unsigned* sink) {
  u32x4_t acc = {0, 0, 0, 0};
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += stride * 8) {
    u32x4_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(buf + min(i + u * stride, n16 - 1));
#pragma unroll
    for (int u = 0; u < 8; ++u) { acc.x ^= v[u].x; acc.y ^= v[u].y; }
  }
  if (acc.x == 0x12345 && acc.y == 7) sink[0] = acc.x;
}

template <int DEPTH, int AUX, int LW>
float run(const unsigned char* buf, size_t per_cu, int ncu, unsigned* sink, int lds_bytes) {
  hipFuncSetAttribute((const void*)stream_kernel<DEPTH, AUX, LW>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int r = 0; r < 2; ++r) stream_kernel<DEPTH, AUX, LW><<<ncu, LW * 64, lds_bytes>>>(buf, per_cu, lds_bytes / 1024, sink);
  hipEventRecord(a);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) stream_kernel<DEPTH, AUX, LW><<<ncu, LW * 64, lds_bytes>>>(buf, per_cu, lds_bytes / 1024, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return (float)(per_cu * ncu) * reps / (ms * 1e-3f) / 1e9f;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const size_t per_cu = 16u << 20;  // 16 MB per CU -> 4 GB total
  unsigned char* buf;
  unsigned* sink;
  hipMalloc(&buf, per_cu * ncu);
  hipMalloc(&sink, 64);
  hipMemset(buf, 1, per_cu * ncu);
  hipDeviceSynchronize();
  printf("CUs %d, %zu MB streamed per launch\n", ncu, per_cu * ncu >> 20);
  const int L = 122 * 1024;
  printf("lds-dma nt   1 wave  depth  8: %7.0f GB/s\n", run<8, 2, 1>(buf, per_cu, ncu, sink, L));
  printf("lds-dma nt   1 wave  depth 16: %7.0f GB/s\n", run<16, 2, 1>(buf, per_cu, ncu, sink, L));
  printf("lds-dma nt   1 wave  depth 32: %7.0f GB/s\n", run<32, 2, 1>(buf, per_cu, ncu, sink, L));
  printf("lds-dma nt   1 wave  depth 48: %7.0f GB/s\n", run<48, 2, 1>(buf, per_cu, ncu, sink, L));
  printf("lds-dma def  1 wave  depth 32: %7.0f GB/s\n", run<32, 0, 1>(buf, per_cu, ncu, sink, L));
  printf("lds-dma nt   2 waves depth 16: %7.0f GB/s\n", run<16, 2, 2>(buf, per_cu, ncu, sink, L));
  printf("lds-dma nt   4 waves depth 12: %7.0f GB/s\n", run<12, 2, 4>(buf, per_cu, ncu, sink, L));
  printf("lds-dma nt   4 waves depth  8: %7.0f GB/s\n", run<8, 2, 4>(buf, per_cu, ncu, sink, L));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const size_t n16 = per_cu * ncu / 16;
  regload_kernel<<<ncu * 4, 256>>>((const u32x4_t*)buf, n16, sink);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) regload_kernel<<<ncu * 4, 256>>>((const u32x4_t*)buf, n16, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  printf("register nt loads (4 WG/CU x 256)   : %7.0f GB/s\n", (float)(per_cu * ncu) * 5 / (ms * 1e-3f) / 1e9f);
  return 0;
}
