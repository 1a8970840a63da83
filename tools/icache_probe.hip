// Instruction-fetch probe: does a long straight-line kernel (the fully unrolled short-attention
// kernels are ~14 KB of code executed once per launch) pay for instruction fetch on MI355X?
// Two kernels issue the same VALU instruction count per wave: `straight` as N unrolled FMAs
// (N * 8 B of code), `looped` as a 64-FMA body repeated N / 64 times (512 B of code).  Launched
// like the short attention (256 workgroups x 1024 threads, one per CU) and alternated with each
// other so no launch finds its code in the instruction cache from the previous launch.
// Build: hipcc --offload-arch=gfx950 -O3 tools/icache_probe.hip -o tools/bin/icache_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N>
__global__ __launch_bounds__(1024) void straight(float* out, float a) {
  float x0 = threadIdx.x, x1 = x0 + 1.f, x2 = x0 + 2.f, x3 = x0 + 3.f;
#pragma unroll
  for (int i = 0; i < N / 4; ++i) {
    x0 = fmaf(x0, a, 0.5f);
    x1 = fmaf(x1, a, 0.25f);
    x2 = fmaf(x2, a, 0.125f);
    x3 = fmaf(x3, a, 0.0625f);
    asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
  }
  if (x0 + x1 + x2 + x3 == 1234.5f) out[threadIdx.x] = x0;
}

__global__ __launch_bounds__(1024) void looped(float* out, float a, int reps) {
  float x0 = threadIdx.x, x1 = x0 + 1.f, x2 = x0 + 2.f, x3 = x0 + 3.f;
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      x0 = fmaf(x0, a, 0.5f);
      x1 = fmaf(x1, a, 0.25f);
      x2 = fmaf(x2, a, 0.125f);
      x3 = fmaf(x3, a, 0.0625f);
      asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    }
  }
  if (x0 + x1 + x2 + x3 == 1234.5f) out[threadIdx.x] = x0;
}

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e_)); return 1; } \
  } while (0)

template <int N>
int run(float* out, hipEvent_t* ev, int grid) {
  const int iters = 20;
  float ts = 0.f, tl = 0.f;
  for (int it = 0; it < iters + 2; ++it) {
    CK(hipEventRecord(ev[0]));
    hipLaunchKernelGGL(straight<N>, dim3(grid), dim3(1024), 0, 0, out, 1.0001f);
    CK(hipEventRecord(ev[1]));
    hipLaunchKernelGGL(looped, dim3(grid), dim3(1024), 0, 0, out, 1.0001f, N / 64);
    CK(hipEventRecord(ev[2]));
    CK(hipEventSynchronize(ev[2]));
    float a, b;
    CK(hipEventElapsedTime(&a, ev[0], ev[1]));
    CK(hipEventElapsedTime(&b, ev[1], ev[2]));
    if (it >= 2) { ts += a; tl += b; }
  }
  printf("N=%5d FMAs/wave (straight code %6d B) grid %4d: straight %7.2f us  looped %7.2f us\n", N, N * 8, grid,
         1e3f * ts / iters, 1e3f * tl / iters);
  return 0;
}

int main() {
  float* out;
  CK(hipMalloc(&out, 4096 * sizeof(float)));
  hipEvent_t ev[3];
  for (auto& e : ev) CK(hipEventCreate(&e));
  for (int grid : {256, 1024}) {
    if (run<512>(out, ev, grid) || run<1024>(out, ev, grid) || run<2048>(out, ev, grid) || run<4096>(out, ev, grid))
      return 1;
  }
  CK(hipFree(out));
  return 0;
}
