// Cross-kernel L2 reuse probe: a row-tiled kernel usually reads what the previous kernel just wrote
// (the ViT step is a chain of such launches).  Does the data stay in the writing XCD's L2 across the
// kernel boundary, so that a consumer workgroup placed on the producer's XCD reads it warm?
// Workgroups are dealt to the 8 XCDs round-robin by id, so with equal grids the consumer of chunk k
// is on the producer's XCD when it is workgroup k ("same"), and on the next XCD when it is
// workgroup k - 1 ("shifted").  Reported: the consumer's time per launch for each placement, after a
// producer launch, and after a 1 GiB sweep that evicts L2 and MALL ("cold").
// Build: hipcc --offload-arch=gfx950 -O3 tools/xcd_probe.hip -o tools/bin/xcd_probe
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int WG = 1024, THREADS = 256;
constexpr size_t CHUNK = 40 * 1024;   // bytes per workgroup: 40 MiB in all (an LN-GEMM launch's bytes)

__global__ __launch_bounds__(THREADS) void produce(float4* buf, float v) {
  float4* p = buf + (size_t)blockIdx.x * (CHUNK / 16);
  for (int i = threadIdx.x; i < (int)(CHUNK / 16); i += THREADS) p[i] = make_float4(v, v + i, v - i, v * 2.f);
}

__global__ __launch_bounds__(THREADS) void consume(const float4* buf, float* out, int shift) {
  const int chunk = (blockIdx.x + shift) % WG;
  const float4* p = buf + (size_t)chunk * (CHUNK / 16);
  float s = 0.f;
  for (int i = threadIdx.x; i < (int)(CHUNK / 16); i += THREADS) {
    const float4 x = p[i];
    s += x.x + x.y + x.z + x.w;
  }
  if (s == 1234.5f) out[blockIdx.x] = s;
}

__global__ __launch_bounds__(THREADS) void sweep(const float4* big, size_t n, float* out) {
  float s = 0.f;
  for (size_t i = (size_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += (size_t)gridDim.x * THREADS) {
    const float4 x = big[i];
    s += x.x;
  }
  if (s == 1234.5f) out[0] = s;
}

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e_)); return 1; } \
  } while (0)

int main() {
  float4 *buf, *big;
  float* out;
  const size_t nbig = (size_t)1 << 26;   // 1 GiB of float4
  CK(hipMalloc(&buf, WG * CHUNK));
  CK(hipMalloc(&big, nbig * sizeof(float4)));
  CK(hipMalloc(&out, WG * sizeof(float)));
  CK(hipMemset(big, 0, nbig * sizeof(float4)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[3] = {"after producer, same XCD   ", "after producer, shifted XCD", "cold (L2+MALL swept)       "};
  for (int rep = 0; rep < 2; ++rep) {
    for (int mode = 0; mode < 3; ++mode) {
      float tot = 0.f;
      const int iters = 20;
      for (int it = 0; it < iters + 2; ++it) {
        hipLaunchKernelGGL(produce, dim3(WG), dim3(THREADS), 0, 0, buf, (float)it);
        if (mode == 2) hipLaunchKernelGGL(sweep, dim3(2048), dim3(THREADS), 0, 0, big, nbig, out);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(consume, dim3(WG), dim3(THREADS), 0, 0, buf, out, mode == 1 ? 1 : 0);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 2) tot += ms;
      }
      printf("%s: %7.2f us per 40 MiB read (%.2f TB/s)\n", names[mode], 1e3f * tot / iters,
             (double)WG * CHUNK / (tot / iters * 1e-3) / 1e12);
    }
  }
  return 0;
}
