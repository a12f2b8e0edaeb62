// Memory latency probe (single thread pointer chase), gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
#include <algorithm>

__global__ void chase(const unsigned* __restrict__ p, int n, unsigned long long* out) {
  unsigned i = 0;
  unsigned long long t0 = wall_clock64();
  long long c0 = clock64();
  for (int s = 0; s < n; ++s) i = p[i];
  long long c1 = clock64();
  unsigned long long t1 = wall_clock64();
  if (out) { out[0] = t1 - t0; out[1] = c1 - c0; out[2] = i; }
}

int main() {
  for (size_t bytes : {size_t(64) << 10, size_t(2) << 20, size_t(64) << 20, size_t(1) << 30}) {
    size_t n = bytes / 4;
    std::vector<unsigned> h(n);
    // random cycle over cache-line-strided slots
    size_t slots = n / 32;
    std::vector<unsigned> perm(slots);
    for (size_t i = 0; i < slots; ++i) perm[i] = (unsigned)i;
    std::mt19937 g(1);
    std::shuffle(perm.begin(), perm.end(), g);
    for (size_t i = 0; i < slots; ++i) h[(size_t)perm[i] * 32] = perm[(i + 1) % slots] * 32;
    unsigned* d; unsigned long long* o;
    hipMalloc(&d, bytes); hipMalloc(&o, 24);
    hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice);
    int steps = 2000;
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(chase, dim3(1), dim3(1), 0, 0, d + perm[0] * 0, steps, o);
      hipDeviceSynchronize();
    }
    unsigned long long r[3];
    hipMemcpy(r, o, 24, hipMemcpyDeviceToHost);
    printf("buffer %8zu KB: %.1f ns/load (wall), %.1f cycles/load\n", bytes >> 10, r[0] * 10.0 / steps,
           (double)r[1] / steps);
    hipFree(d); hipFree(o);
  }
  // empty kernel dispatch timing
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(a);
    for (int i = 0; i < 1000; ++i) hipLaunchKernelGGL(chase, dim3(1), dim3(1), 0, 0, nullptr, 0, nullptr);
    hipEventRecord(b); hipEventSynchronize(b);
  }
  float ms; hipEventElapsedTime(&ms, a, b);
  printf("back-to-back tiny kernels: %.2f us each\n", ms);
  return 0;
}
