// Cost of a workgroup barrier on gfx950 (8 waves, nothing outstanding) and of the
// __syncthreads() form (release/acquire fences + s_barrier), cycles per barrier.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_barrier.hip -o /tmp/ubb && /tmp/ubb
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void bar(long long* out, int mode) {
  __shared__ float s[512];
  const int N = 1024;
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  long long t0 = clock64();
  if (mode == 0) {
    for (int i = 0; i < N; ++i) __builtin_amdgcn_s_barrier();
  } else if (mode == 1) {
    for (int i = 0; i < N; ++i) __syncthreads();
  } else {
    float a = 0.f;
    for (int i = 0; i < N; ++i) {   // one LDS write + read per wave per barrier
      s[(threadIdx.x + i) & 511] += 1.f;
      __syncthreads();
      a += s[(threadIdx.x * 7 + i) & 511];
    }
    s[threadIdx.x] = a;
  }
  long long t1 = clock64();
  if (threadIdx.x == 0) out[mode] = (t1 - t0) / N;
}

int main() {
  long long* d;
  hipMalloc(&d, 8 * sizeof(long long));
  for (int m = 0; m < 3; ++m) hipLaunchKernelGGL(bar, dim3(1), dim3(512), 0, 0, d, m);
  for (int m = 0; m < 3; ++m) hipLaunchKernelGGL(bar, dim3(1), dim3(512), 0, 0, d, m);
  hipDeviceSynchronize();
  long long h[8];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("s_barrier %lld cyc, __syncthreads %lld cyc, LDS rmw + __syncthreads %lld cyc\n", h[0], h[1], h[2]);
  return 0;
}
