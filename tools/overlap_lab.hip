// Lab kernels (not shipped): can a decode step overlap the attention's K/V stream with the qkv GEMV that precedes
// it?  (tools/overlap_lab.py)
//  * lab_set / lab_spin: a flag hand-off between two graph branches (is the side branch really concurrent?);
//  * lab_read: bare streaming read of a byte range (the attention's K/V bytes without the math);
//  * lab_prefetch_wait: each workgroup loads its share of a byte range into registers FIRST, then waits for a
//    flag, then folds the registers (the "prefetch K/V, wait for q" attention shape).
// build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/overlap_lab.hip -o tools/_lab/overlap_lab.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ldnt(const uint4* p) {
  const u32x4_t v = __builtin_nontemporal_load((const u32x4_t*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

__global__ void set_kernel(unsigned* flag, unsigned v) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// waits until *flag == 1 (or ~50 ms), then re-arms it to 0; err += 1 on timeout
__global__ void spin_kernel(unsigned* flag, unsigned* err) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 1u) {
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000ull) {
      atomicAdd(err, 1u);
      break;
    }
  }
  __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int UNR, bool NT = true>
__global__ void __launch_bounds__(256) read_kernel(const uint4* __restrict__ p, long n16, uint32_t* sink) {
  const long stride = (long)gridDim.x * 256;
  uint32_t acc = 0;
  for (long base = (long)blockIdx.x * 256 + threadIdx.x; base < n16; base += stride * UNR) {
    uint4 r[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long i = base + u * stride;
      r[u] = NT ? ldnt(p + (i < n16 ? i : n16 - 1)) : p[i < n16 ? i : n16 - 1];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc ^= r[u].x ^ r[u].y ^ r[u].z ^ r[u].w;
  }
  if (acc == 0x9E3779B9u && threadIdx.x == 0) *sink = acc;
}

// one workgroup per CU-sized chunk: NL 16-B loads per lane into registers, then wait for *flag >= 1 (lane 0 polls,
// bounded), then fold; the last workgroup to finish re-arms the flag (counter in done[])
template <int NL>
__global__ void __launch_bounds__(256) prefetch_wait_kernel(const uint4* __restrict__ p, long n16,
                                                            unsigned* flag, unsigned* done, unsigned* err,
                                                            uint32_t* sink) {
  const long base = (long)blockIdx.x * 256 * NL + threadIdx.x;
  uint4 r[NL];
#pragma unroll
  for (int u = 0; u < NL; ++u) {
    const long i = base + (long)u * 256;
    r[u] = ldnt(p + (i < n16 ? i : n16 - 1));
  }
  __shared__ int go;
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000ull) {
        atomicAdd(err, 1u);
        break;
      }
    }
    go = 1;
  }
  __syncthreads();
  uint32_t acc = go;
#pragma unroll
  for (int u = 0; u < NL; ++u) acc ^= r[u].x ^ r[u].y ^ r[u].z ^ r[u].w;
  if (acc == 0x9E3779B9u) *sink = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = atomicAdd(done, 1u);
    if (prev == gridDim.x - 1) {
      *done = 0;
      __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

extern "C" int lab_set(unsigned* flag, unsigned v, hipStream_t s) {
  set_kernel<<<1, 64, 0, s>>>(flag, v);
  return (int)hipGetLastError();
}
extern "C" int lab_spin(unsigned* flag, unsigned* err, hipStream_t s) {
  spin_kernel<<<1, 64, 0, s>>>(flag, err);
  return (int)hipGetLastError();
}
extern "C" int lab_read(const void* p, long bytes, int blocks, int unr, uint32_t* sink, hipStream_t s) {
  const long n16 = bytes / 16;
  if (unr == 4) read_kernel<4><<<blocks, 256, 0, s>>>((const uint4*)p, n16, sink);
  else if (unr == 16) read_kernel<16><<<blocks, 256, 0, s>>>((const uint4*)p, n16, sink);
  else if (unr == -8) read_kernel<8, false><<<blocks, 256, 0, s>>>((const uint4*)p, n16, sink);
  else read_kernel<8><<<blocks, 256, 0, s>>>((const uint4*)p, n16, sink);
  return (int)hipGetLastError();
}
// NL = 16-B loads per lane (a workgroup covers 4 KB * NL); grid = ceil(bytes / (4096 * NL))
extern "C" int lab_prefetch_wait(const void* p, long bytes, int nl, unsigned* flag, unsigned* done, unsigned* err,
                                 uint32_t* sink, hipStream_t s) {
  const long n16 = bytes / 16;
  const int blocks = (int)((n16 + 256L * nl - 1) / (256L * nl));
  if (nl == 32) prefetch_wait_kernel<32><<<blocks, 256, 0, s>>>((const uint4*)p, n16, flag, done, err, sink);
  else if (nl == 64) prefetch_wait_kernel<64><<<blocks, 256, 0, s>>>((const uint4*)p, n16, flag, done, err, sink);
  else prefetch_wait_kernel<16><<<blocks, 256, 0, s>>>((const uint4*)p, n16, flag, done, err, sink);
  return (int)hipGetLastError();
}
