// Lab kernel (not shipped): stream a byte range through the cache hierarchy so that a later kernel finds it in
// the Infinity Cache (MALL). Grid-stride, UNR 16-B loads in flight per lane, results folded into one xor that is
// stored only if it equals an impossible value (keeps the loads alive).
// build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/prefetch_lab.hip -o tools/_lab/prefetch_lab.so
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

template <int UNR, int POLICY>
__global__ void __launch_bounds__(256) prefetch_kernel(const uint4* __restrict__ p, long n16, uint32_t* sink) {
  const long stride = (long)gridDim.x * 256;
  uint32_t acc = 0;
  for (long base = (long)blockIdx.x * 256 + threadIdx.x; base < n16; base += stride * UNR) {
    uint4 r[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long i = base + u * stride;
      const uint4* q = p + (i < n16 ? i : n16 - 1);
      if (POLICY == 1) {
        const u32x4_t v = __builtin_nontemporal_load((const u32x4_t*)q);
        r[u] = make_uint4(v.x, v.y, v.z, v.w);
      } else
        r[u] = *q;
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc ^= r[u].x ^ r[u].y ^ r[u].z ^ r[u].w;
  }
  if (acc == 0x9E3779B9u && threadIdx.x == 0) *sink = acc;
}

extern "C" int lab_prefetch(const void* p, long bytes, int blocks, int unr, int policy, uint32_t* sink,
                            hipStream_t s) {
  const long n16 = bytes / 16;
  if (policy == 0 && unr == 8) prefetch_kernel<8, 0><<<blocks, 256, 0, s>>>((const uint4*)p, n16, sink);
  else if (policy == 0 && unr == 4) prefetch_kernel<4, 0><<<blocks, 256, 0, s>>>((const uint4*)p, n16, sink);
  else if (policy == 0) prefetch_kernel<16, 0><<<blocks, 256, 0, s>>>((const uint4*)p, n16, sink);
  else prefetch_kernel<8, 1><<<blocks, 256, 0, s>>>((const uint4*)p, n16, sink);
  return (int)hipGetLastError();
}
