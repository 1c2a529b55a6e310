// Lab: does a kernel launched with hipExtAnyOrderLaunch (AQL barrier bit clear) start its workgroups while the
// previous kernel on the same stream is still draining?  Eager launches and a captured graph.
// Kernels only read the wall clock and spin for a bounded time; no inter-kernel waits (cannot hang).
// build: hipcc --offload-arch=gfx950 -O2 tools/anyorder_lab.hip -o tools/_lab/anyorder_lab
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

// Workgroup b spins for ticks[b] (100 MHz wall clock) and records its start / end.
__global__ void producer(const unsigned* ticks, unsigned long long* t) {
  unsigned long long t0 = wall_clock64();
  unsigned n = ticks[blockIdx.x];
  while (wall_clock64() - t0 < n) { __builtin_amdgcn_s_sleep(1); }
  if (threadIdx.x == 0) { t[2 * blockIdx.x] = t0; t[2 * blockIdx.x + 1] = wall_clock64(); }
}

__global__ void consumer(unsigned long long* t) {
  if (threadIdx.x == 0) t[blockIdx.x] = wall_clock64();
}

static int run(const char* name, hipStream_t s, bool graph, unsigned flags, const std::vector<unsigned>& ticks_h,
               int nb) {
  unsigned* ticks; unsigned long long *ta, *tb;
  int na = (int)ticks_h.size();
  CK(hipMalloc(&ticks, na * 4)); CK(hipMalloc(&ta, na * 16)); CK(hipMalloc(&tb, nb * 8));
  CK(hipMemcpy(ticks, ticks_h.data(), na * 4, hipMemcpyHostToDevice));
  hipGraphExec_t exec = nullptr;
  auto launch = [&]() -> hipError_t {
    hipExtLaunchKernelGGL(producer, dim3(na), dim3(256), 0, s, nullptr, nullptr, 0, ticks, ta);
    hipExtLaunchKernelGGL(consumer, dim3(nb), dim3(256), 0, s, nullptr, nullptr, flags, tb);
    return hipGetLastError();
  };
  if (graph) {
    hipGraph_t g;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    CK(launch());
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0));
  }
  for (int rep = 0; rep < 3; ++rep) {
    if (graph) CK(hipGraphLaunch(exec, s)); else CK(launch());
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> a(2 * na), b(nb);
    CK(hipMemcpy(a.data(), ta, na * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), tb, nb * 8, hipMemcpyDeviceToHost));
    unsigned long long a0 = ~0ull, a_end_max = 0, a_end_min = ~0ull;
    for (int i = 0; i < na; ++i) { a0 = std::min(a0, a[2*i]); a_end_max = std::max(a_end_max, a[2*i+1]);
                                   a_end_min = std::min(a_end_min, a[2*i+1]); }
    unsigned long long b_min = *std::min_element(b.begin(), b.end()), b_max = *std::max_element(b.begin(), b.end());
    int early = 0;
    for (int i = 0; i < nb; ++i) early += b[i] < a_end_max;
    printf("%-28s rep %d: A first start 0, A ends %.2f..%.2f us, B starts %.2f..%.2f us, B wgs before A done: %d/%d\n",
           name, rep, (a_end_min - a0) / 100.0, (a_end_max - a0) / 100.0, ((long long)(b_min - a0)) / 100.0,
           ((long long)(b_max - a0)) / 100.0, early, nb);
  }
  if (exec) CK(hipGraphExecDestroy(exec));
  CK(hipFree(ticks)); CK(hipFree(ta)); CK(hipFree(tb));
  return 0;
}

int main() {
  hipStream_t s; if (hipStreamCreate(&s) != hipSuccess) return 1;
  std::vector<unsigned> tail(256, 500);  // 5 us everywhere ...
  tail[0] = 3000;                        // ... one straggler of 30 us
  std::vector<unsigned> even(256, 1000);
  int rc = 0;
  rc |= run("eager barrier", s, false, 0, tail, 256);
  rc |= run("eager anyorder", s, false, hipExtAnyOrderLaunch, tail, 256);
  rc |= run("eager anyorder even", s, false, hipExtAnyOrderLaunch, even, 256);
  rc |= run("graph barrier", s, true, 0, tail, 256);
  rc |= run("graph anyorder", s, true, hipExtAnyOrderLaunch, tail, 256);
  return rc;
}
