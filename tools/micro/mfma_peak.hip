// Whole-chip matrix / vector throughput probe: FLOP/s of v_mfma_f64_16x16x4_f64,
// v_mfma_f32_16x16x4_f32, v_mfma_f32_16x16x32_bf16 and v_fma_f64, every CU busy (2048
// workgroups of 4 waves, 8 independent accumulator chains per wave). The fp64 Gram
// (csrc/gram.hip gram_small_kernel<double>) is priced against the measured fp64 MFMA rate.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_peak.hip -o tools/micro/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int CH = 8;   // independent chains per wave

__global__ __launch_bounds__(256) void k_f64(double* out, int iters) {
  f64x4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = f64x4{0, 0, 0, 0};
  const double a = 1e-3 * (threadIdx.x + 1), b = 1e-3 * (blockIdx.x + 1);
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  double s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  if (s == 1.2345) out[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_f32(float* out, int iters) {
  f32x4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = f32x4{0, 0, 0, 0};
  const float a = 1e-3f * (threadIdx.x + 1), b = 1e-3f * (blockIdx.x + 1);
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
  float s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  if (s == 1.2345f) out[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_bf16(float* out, int iters) {
  f32x4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = f32x4{0, 0, 0, 0};
  bf16x8 a, b;
  for (int e = 0; e < 8; ++e) {
    a[e] = (__bf16)(1e-3f * (threadIdx.x + e));
    b[e] = (__bf16)(1e-3f * (blockIdx.x + e));
  }
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[c], 0, 0, 0);
  float s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  if (s == 1.2345f) out[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_vfma64(double* out, int iters) {
  double x[CH];
  for (int c = 0; c < CH; ++c) x[c] = 1e-3 * (threadIdx.x + c);
  const double a = 0.999999, b = 1e-9 * (blockIdx.x + 1);
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = __builtin_fma(x[c], a, b);
  double s = 0;
  for (int c = 0; c < CH; ++c) s += x[c];
  if (s == 1.2345) out[threadIdx.x] = s;
}

template <typename K, typename T>
static double run(K kern, T* out, int iters, double flop_per_wave_iter, const char* name) {
  const int nwg = 2048, nth = 256;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(nth), 0, 0, out, 16);   // warm
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(nth), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop = flop_per_wave_iter * (double)iters * nwg * (nth / 64);
  const double tf = flop / (ms * 1e-3) / 1e12;
  printf("%-28s %8.3f ms  %8.1f TFLOP/s\n", name, ms, tf);
  return tf;
}

int main() {
  double* d64;
  float* d32;
  hipMalloc(&d64, 4096);
  hipMalloc(&d32, 4096);
  // one MFMA 16x16xK = 2*16*16*K FLOP
  run(k_f64, d64, 2000, CH * 2.0 * 16 * 16 * 4, "mfma_f64_16x16x4_f64");
  run(k_f32, d32, 4000, CH * 2.0 * 16 * 16 * 4, "mfma_f32_16x16x4_f32");
  run(k_bf16, d32, 8000, CH * 2.0 * 16 * 16 * 32, "mfma_f32_16x16x32_bf16");
  run(k_vfma64, d64, 8000, CH * 2.0 * 64, "v_fma_f64 (vector)");
  hipFree(d64);
  hipFree(d32);
  return 0;
}
