// Lab (not shipped): can consecutive decode kernels overlap their launch ramp / first-byte latency / tail when they
// alternate between two HIP streams and hand off through a device counter instead of a stream barrier?
//
// A chain of N "layer kernels", each streaming its own `bytes` (a bare read standing in for a GEMV's weights).
// Kernel i issues its first batch of loads, then (two-stream mode) waits until kernel i-1 has signalled that all
// its workgroups are done, then streams the rest and signals. One-stream mode: same kernels, no waits, stream order.
// The whole chain is launched from C++ (host launch cost ~3 us per kernel stays off the GPU timeline).
// build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/chain_lab.hip -o tools/_lab/chain_lab.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ldnt(const uint4* p) {
  const u32x4_t v = __builtin_nontemporal_load((const u32x4_t*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

template <int UNR>
__global__ void __launch_bounds__(256) chain_kernel(const uint4* __restrict__ p, long n16, const unsigned* wait_ctr,
                                                    unsigned wait_target, unsigned* sig_ctr, unsigned* err,
                                                    uint32_t* sink) {
  const long stride = (long)gridDim.x * 256;
  uint32_t acc = 0;
  long base = (long)blockIdx.x * 256 + threadIdx.x;
  uint4 r[UNR];
#pragma unroll
  for (int u = 0; u < UNR; ++u) {
    const long i = base + u * stride;
    r[u] = ldnt(p + (i < n16 ? i : n16 - 1));
  }
  if (wait_ctr) {  // the dependency: every workgroup of the previous kernel has signalled
    __shared__ int ok;
    if (threadIdx.x == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      int good = 1;
      while (__hip_atomic_load(wait_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < wait_target) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {  // 0.2 s: report, never hang
          atomicAdd(err, 1u);
          good = 0;
          break;
        }
      }
      ok = good;
    }
    __syncthreads();
    acc ^= ok;
  }
#pragma unroll
  for (int u = 0; u < UNR; ++u) acc ^= r[u].x ^ r[u].y ^ r[u].z ^ r[u].w;
  for (base += stride * UNR; base < n16; base += stride * UNR) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long i = base + u * stride;
      r[u] = ldnt(p + (i < n16 ? i : n16 - 1));
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc ^= r[u].x ^ r[u].y ^ r[u].z ^ r[u].w;
  }
  if (acc == 0x9E3779B9u && threadIdx.x == 0) *sink = acc;
  if (sig_ctr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(sig_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// bufs: n_kernels device pointers of `bytes` each; ctr: n_kernels * 64 uint32 (zeroed by the caller before each
// run: counters grow by `blocks` per run); mode 0 = one stream, 1 = alternate two streams with counter waits.
extern "C" int lab_chain(void* const* bufs, int n_kernels, long bytes, int blocks, int mode, unsigned* ctr,
                         unsigned* err, uint32_t* sink, hipStream_t s0, hipStream_t s1, unsigned run) {
  const long n16 = bytes / 16;
  for (int i = 0; i < n_kernels; ++i) {
    hipStream_t s = (mode == 1 && (i & 1)) ? s1 : s0;
    const unsigned* w = (mode == 1 && i > 0) ? ctr + (size_t)(i - 1) * 64 : nullptr;
    unsigned* sig = mode == 1 ? ctr + (size_t)i * 64 : nullptr;
    chain_kernel<8><<<blocks, 256, 0, s>>>((const uint4*)bufs[i], n16, w, (run + 1) * (unsigned)blocks, sig, err,
                                           sink);
  }
  return (int)hipGetLastError();
}
