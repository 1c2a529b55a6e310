// HBM read-bandwidth probe for decode-sized kernels (8-66 MB): what a pure 16-B/lane streaming read reaches on
// this MI355X for a given grid / block size / loads in flight, launched back to back over rotating buffers
// (total > 1 GiB, so every launch streams from HBM, as the decode step does).
// build: hipcc --offload-arch=gfx950 -O3 -o bw_probe tools/bw_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int UNR, bool NT>
__global__ void read_probe(const u32x4* __restrict__ p, size_t n16, unsigned* out) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned acc = 0;
  size_t i = tid;
  for (; i + (UNR - 1) * stride < n16; i += UNR * stride) {
    u32x4 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) v[u] = NT ? __builtin_nontemporal_load(p + i + u * stride) : p[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n16; i += stride) acc ^= p[i].x;
  if (acc == 0x12345678u) out[0] = acc;  // keep the loads alive
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t err_ = (x);                                                    \
    if (err_ != hipSuccess) {                                                 \
      printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__);      \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

template <int UNR, bool NT>
float run(char* base, size_t bytes, int copies, int blocks, int threads, unsigned* out) {
  const size_t n16 = bytes / 16;
  for (int c = 0; c < copies; ++c)
    read_probe<UNR, NT><<<blocks, threads>>>((const u32x4*)(base + (size_t)c * bytes), n16, out);
  CK(hipDeviceSynchronize());
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  const int reps = 4 * copies;
  CK(hipEventRecord(s));
  for (int r = 0; r < reps; ++r)
    read_probe<UNR, NT><<<blocks, threads>>>((const u32x4*)(base + (size_t)(r % copies) * bytes), n16, out);
  CK(hipEventRecord(e));
  CK(hipEventSynchronize(e));
  float ms;
  CK(hipEventElapsedTime(&ms, s, e));
  return ms * 1e3f / reps;  // us per launch
}

int main() {
  const size_t total = 2ull << 30;
  char* base;
  unsigned* out;
  CK(hipMalloc(&base, total));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(base, 1, total));
  const size_t sizes[] = {8u << 20, 25u << 20, 46u << 20, 66u << 20, 512u << 20};
  const int grids[] = {256, 512, 1024, 2048, 4096, 8192};
  for (size_t bytes : sizes) {
    const int copies = (int)(total / bytes) > 64 ? 64 : (int)(total / bytes);
    for (int threads : {64, 256}) {
      for (int g : grids) {
        const float a = run<4, true>(base, bytes, copies, g, threads, out);
        const float b = run<8, true>(base, bytes, copies, g, threads, out);
        const float c = run<8, false>(base, bytes, copies, g, threads, out);
        printf("size %4zu MB threads %3d blocks %5d | UNR4 nt %7.2f us %6.0f GB/s | UNR8 nt %7.2f us %6.0f GB/s | "
               "UNR8 plain %7.2f us %6.0f GB/s\n",
               bytes >> 20, threads, g, a, bytes / a / 1e3, b, bytes / b / 1e3, c, bytes / c / 1e3);
      }
    }
  }
  return 0;
}
