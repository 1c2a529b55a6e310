// Which chip-wide address pattern streams fastest for a one-shot decode GEMV? Each wave issues L 1-KB loads
// (64 lanes x 16 B) up front and then consumes them, as lga_q4_gemv does. Modes:
//   0 grid-stride loop (bw_probe reference)
//   1 wave-private: wave w reads L consecutive KB [w*L, w*L+L)            (row-major weights, GEMV today)
//   2 interleaved:  wave w's load j reads KB j*W + w                        (load-order tiled layout)
//   3 dual wave-private: L/2 KB from region A and L/2 KB from region B     (fc_1 || fc_2 today)
//   4 interleaved in groups of 8 waves: wave w's load j reads KB ((w/8)*L + j)*8 + w%8
// build: hipcc --offload-arch=gfx950 -O3 -o tools/layout_probe tools/layout_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t err_ = (x);                                               \
    if (err_ != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); \
      exit(1);                                                           \
    }                                                                    \
  } while (0)

// SC = extra small loads per wave: 0 none, 1 = 8 ushort gathers (16 distinct 2-B values per instruction, as the
// GEMV's scale loads), 2 = 2 dwordx4 loads of the same bytes, 3 = 8 dwordx4 (x-like, L2-resident)
template <int L, int MODE, int SC = 0>
__global__ void __launch_bounds__(256) probe(const u32x4* __restrict__ p, int waves, unsigned* out,
                                             const unsigned short* __restrict__ sc = nullptr) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= waves) return;
  constexpr int KB = 64;  // u32x4 per KB
  u32x4 v[L];
#pragma unroll
  for (int j = 0; j < L; ++j) {
    size_t kb;
    if (MODE == 1) kb = (size_t)w * L + j;
    else if (MODE == 2) kb = (size_t)j * waves + w;
    else if (MODE == 3) kb = (j < L / 2) ? (size_t)w * (L / 2) + j : (size_t)waves * (L / 2) + (size_t)w * (L / 2) + (j - L / 2);
    else kb = ((size_t)(w / 8) * L + j) * 8 + (w % 8);
    v[j] = __builtin_nontemporal_load(p + kb * KB + lane);
  }
  unsigned acc = 0;
  if (SC == 1) {
    unsigned short s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = sc[(size_t)w * 64 + (j & 1) * 32 + (lane + 64 * (j >> 1)) / 16];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += s[j];
  } else if (SC == 2) {
    u32x4 s[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) s[j] = ((const u32x4*)(sc + (size_t)w * 64))[(lane & 3) + 4 * j];
#pragma unroll
    for (int j = 0; j < 2; ++j) acc += s[j].x ^ s[j].w;
  }
#pragma unroll
  for (int j = 0; j < L; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  if (acc == 0x12345678u) out[0] = acc;
}

// persistent streaming: NB blocks, each wave walks tiles t0, t0+W, ... (L KB each) with two register buffers
template <int L>
__global__ void __launch_bounds__(256) stream_probe(const u32x4* __restrict__ p, int tiles, unsigned* out) {
  const int lane = threadIdx.x & 63;
  const int W = gridDim.x * 4;
  const int t0 = blockIdx.x * 4 + (threadIdx.x >> 6);
  u32x4 a[L], b[L];
  auto ld = [&](u32x4* v, int t) {
    const bool ok = t < tiles;
#pragma unroll
    for (int j = 0; j < L; ++j) v[j] = __builtin_nontemporal_load(p + (ok ? ((size_t)t * L + j) * 64 + lane : 0));
  };
  ld(a, t0);
  ld(b, t0 + W);
  unsigned acc = 0;
  for (int t = t0; t < tiles; t += 2 * W) {
#pragma unroll
    for (int j = 0; j < L; ++j) acc ^= a[j].x ^ a[j].y ^ a[j].z ^ a[j].w;
    ld(a, t + 2 * W);
#pragma unroll
    for (int j = 0; j < L; ++j) acc ^= b[j].x ^ b[j].y ^ b[j].z ^ b[j].w;
    ld(b, t + 3 * W);
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int L>
float run_stream(char* base, size_t bytes, int copies, unsigned* out, int nb) {
  const int tiles = (int)(bytes / 1024 / L);
  for (int c = 0; c < copies; ++c) stream_probe<L><<<nb, 256>>>((const u32x4*)(base + (size_t)c * bytes), tiles, out);
  CK(hipDeviceSynchronize());
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  const int reps = 4 * copies;
  CK(hipEventRecord(s));
  for (int r = 0; r < reps; ++r)
    stream_probe<L><<<nb, 256>>>((const u32x4*)(base + (size_t)(r % copies) * bytes), tiles, out);
  CK(hipEventRecord(e));
  CK(hipEventSynchronize(e));
  float ms;
  CK(hipEventElapsedTime(&ms, s, e));
  return ms * 1e3f / reps;
}

__global__ void stride_probe(const u32x4* __restrict__ p, size_t n16, unsigned* out) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned acc = 0;
  size_t i = tid;
  for (; i + 7 * stride < n16; i += 8 * stride) {
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(p + i + u * stride);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n16; i += stride) acc ^= p[i].x;
  if (acc == 0x12345678u) out[0] = acc;
}

template <int L, int MODE, int SC = 0>
float run(char* base, size_t bytes, int copies, unsigned* out, const unsigned short* sc = nullptr) {
  const int waves = (int)(bytes / 1024 / L);
  const int blocks = (waves + 3) / 4;
  auto launch = [&](int c) {
    const u32x4* p = (const u32x4*)(base + (size_t)c * bytes);
    if (MODE == 0) stride_probe<<<2048, 256>>>(p, bytes / 16, out);
    else probe<L, MODE, SC><<<blocks, 256>>>(p, waves, out, sc + (size_t)c * waves * 64);
  };
  for (int c = 0; c < copies; ++c) launch(c);
  CK(hipDeviceSynchronize());
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  const int reps = 4 * copies;
  CK(hipEventRecord(s));
  for (int r = 0; r < reps; ++r) launch(r % copies);
  CK(hipEventRecord(e));
  CK(hipEventSynchronize(e));
  float ms;
  CK(hipEventElapsedTime(&ms, s, e));
  return ms * 1e3f / reps;
}

int main() {
  const size_t total = 2ull << 30;
  char* base;
  unsigned* out;
  CK(hipMalloc(&base, total));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(base, 1, total));
  unsigned short* sc;
  CK(hipMalloc(&sc, 256u << 20));
  CK(hipMemset(sc, 0, 256u << 20));
  const size_t sizes[] = {8u << 20, 24u << 20, 44u << 20, 64u << 20};
  for (size_t bytes : sizes) {
    const int copies = (int)(total / bytes) > 64 ? 64 : (int)(total / bytes);
    printf("size %3zu MB | one-shot L8 %6.2f | stream L8 nb256 %6.2f nb512 %6.2f nb768 %6.2f nb1024 %6.2f | "
           "stream L4 nb512 %6.2f nb1024 %6.2f | L16 nb256 %6.2f nb512 %6.2f\n", bytes >> 20,
           run<8, 1, 0>(base, bytes, copies, out, sc), run_stream<8>(base, bytes, copies, out, 256),
           run_stream<8>(base, bytes, copies, out, 512), run_stream<8>(base, bytes, copies, out, 768),
           run_stream<8>(base, bytes, copies, out, 1024), run_stream<4>(base, bytes, copies, out, 512),
           run_stream<4>(base, bytes, copies, out, 1024), run_stream<16>(base, bytes, copies, out, 256),
           run_stream<16>(base, bytes, copies, out, 512));
  }
  return 0;
  for (size_t bytes : sizes) {
    const int copies = (int)(total / bytes) > 64 ? 64 : (int)(total / bytes);
    printf("size %3zu MB | L8 priv %6.2f | +8 ushort scale loads %6.2f | +2 x4 scale loads %6.2f\n", bytes >> 20,
           run<8, 1, 0>(base, bytes, copies, out, sc), run<8, 1, 1>(base, bytes, copies, out, sc),
           run<8, 1, 2>(base, bytes, copies, out, sc));
  }
  for (size_t bytes : sizes) {
    const int copies = (int)(total / bytes) > 64 ? 64 : (int)(total / bytes);
    printf("size %3zu MB | stride %6.2f us", bytes >> 20, run<8, 0>(base, bytes, copies, out));
    printf(" | L8: priv %6.2f inter %6.2f dual %6.2f grp8 %6.2f", run<8, 1>(base, bytes, copies, out),
           run<8, 2>(base, bytes, copies, out), run<8, 3>(base, bytes, copies, out), run<8, 4>(base, bytes, copies, out));
    printf(" | L4: priv %6.2f inter %6.2f dual %6.2f", run<4, 1>(base, bytes, copies, out),
           run<4, 2>(base, bytes, copies, out), run<4, 3>(base, bytes, copies, out));
    printf(" | L16: priv %6.2f inter %6.2f dual %6.2f\n", run<16, 1>(base, bytes, copies, out),
           run<16, 2>(base, bytes, copies, out), run<16, 3>(base, bytes, copies, out));
  }
  return 0;
}
