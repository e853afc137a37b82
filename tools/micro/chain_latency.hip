// Dependent-chain latency probe (one wave): cycles per step of the CV path kernel's
// lasso walk in fp64 vs fp32, and of single dependent ops. Run: ./chain_latency
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T>
__global__ void walk_kernel(T* out, long long* cyc, T thr, int iters) {
  const int lane = threadIdx.x;
  T u = (T)(0.001 * (lane + 1)), a0 = (T)(0.0005 * lane);
  const T c = (T)(-0.01 * ((lane * 7) % 13));
  __syncthreads();
  const long long t0 = clock64();
  for (int r = 0; r < iters; ++r) {
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      const T cl = sizeof(T) == 8 ? (T)fmin(fmax((double)u, -(double)thr), (double)thr) : (T)fminf(fmaxf((float)u, -(float)thr), (float)thr);
      const T dd = (u - a0) - cl;
      T d;
      if constexpr (sizeof(T) == 8) {
        int lo = __builtin_amdgcn_readlane(__double2loint(dd), i);
        int hi = __builtin_amdgcn_readlane(__double2hiint(dd), i);
        d = __hiloint2double(hi, lo);
      } else {
        d = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, dd), i));
      }
      if constexpr (sizeof(T) == 8) u = __builtin_fma(c, d, u);
      else u = __builtin_fmaf(c, d, u);
    }
  }
  const long long t1 = clock64();
  out[lane] = u;
  if (lane == 0) *cyc = t1 - t0;
}

template <typename T>
__global__ void fma_chain(T* out, long long* cyc, int iters) {
  T x = (T)threadIdx.x * (T)1e-3;
  const T a = (T)0.999, b = (T)1e-7;
  const long long t0 = clock64();
  for (int r = 0; r < iters; ++r) {
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      if constexpr (sizeof(T) == 8) x = __builtin_fma(x, a, b);
      else x = __builtin_fmaf(x, a, b);
    }
  }
  const long long t1 = clock64();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  double* od; float* of; long long* cy;
  hipMalloc(&od, 64 * 8); hipMalloc(&of, 64 * 4); hipMalloc(&cy, 8);
  long long h;
  const int it = 200;
  auto rep = [&](const char* name, double steps) {
    hipDeviceSynchronize(); hipMemcpy(&h, cy, 8, hipMemcpyDeviceToHost);
    printf("%-28s %.1f cycles/step\n", name, (double)h / steps);
  };
  for (int w = 0; w < 2; ++w) {
    hipLaunchKernelGGL(walk_kernel<double>, 1, 64, 0, 0, od, cy, 0.05, it); rep("walk step fp64", 64.0 * it);
    hipLaunchKernelGGL(walk_kernel<float>, 1, 64, 0, 0, of, cy, 0.05f, it); rep("walk step fp32", 64.0 * it);
    hipLaunchKernelGGL(fma_chain<double>, 1, 64, 0, 0, od, cy, it); rep("dependent fma fp64", 64.0 * it);
    hipLaunchKernelGGL(fma_chain<float>, 1, 64, 0, 0, of, cy, it); rep("dependent fma fp32", 64.0 * it);
  }
  return 0;
}
