// Per-CU streaming probe (gfx950): NB workgroups of 512 threads each read the
// SAME W-byte buffer (L2-resident after the first pass) with 16-byte loads,
// 8 in flight per lane, and reduce it.  Reports the kernel time (HIP events,
// averaged over repeats) -> effective per-CU bytes/s.  Build:
//   hipcc --offload-arch=gfx950 -O3 tools/stream_probe.hip -o tools/stream_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(512) void stream(const float4* __restrict__ w, int n4, float* out) {
  float acc = 0.f;
  for (int i = threadIdx.x; i < n4; i += 512 * 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = i + u * 512;
      v[u] = w[j];      // n4 is a multiple of 512*8: no bounds test (see header)
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 12345.f) out[blockIdx.x] = acc;
}

__global__ void empty_k() {}

int main() {
  float4* w; float* o;
  hipMalloc(&w, 8 << 20); hipMalloc(&o, 4096 * 4);
  hipMemset(w, 0, 8 << 20);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  float ms;
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, 0);
  hipEventRecord(a);
  for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(empty_k, dim3(64), dim3(256), 0, 0);
  hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
  printf("empty kernel (64 blocks): %.2f us per launch\n", ms * 1000 / 200);
  for (int kb : {64, 128, 192, 256, 512}) {
    for (int nb : {1, 20, 63, 128, 256, 512}) {
      const int n4 = kb * 1024 / 16;
      for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(stream, dim3(nb), dim3(512), 0, 0, w, n4, o);
      hipEventRecord(a);
      const int R = 50;
      for (int i = 0; i < R; ++i) hipLaunchKernelGGL(stream, dim3(nb), dim3(512), 0, 0, w, n4, o);
      hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
      const double us = ms * 1000 / R;
      printf("W %4d KB  blocks %4d : %7.2f us/launch  %7.1f GB/s per block  %8.1f GB/s total\n", kb, nb, us,
             kb * 1024.0 / us / 1e3, kb * 1024.0 * nb / us / 1e3);
    }
  }
  return 0;
}
