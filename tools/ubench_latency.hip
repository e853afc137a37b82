// Dependent-issue latency of the instructions on the CD recurrence chain (one wave,
// gfx950): cycles per link of a chain of N dependent operations, measured with s_memtime
// (s_memtime runs at the shader clock on gfx9). Build + run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_latency.hip -o /tmp/ubl && /tmp/ubl
#include <hip/hip_runtime.h>
#include <cstdio>

#define N 256

template <int V>
__device__ __forceinline__ double kstep(double x, const float* src, long long* out) {
  const int lane = threadIdx.x;
  double u = x, at = 0.25, thr = 0.001, gt = x * 0.5, gbef = 0, anv = at;
  unsigned sidx = 0;
  float lo_[32], hi_[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    lo_[j] = src[(threadIdx.x + j) & 63];
    hi_[j] = src[(threadIdx.x + j + 32) & 63];
  }
  const long long t0 = clock64();
  for (int it = 0; it < N; ++it) {
    const int i = __builtin_amdgcn_readfirstlane((sidx += 5) & 63);
    const double an = copysign(fmax(fabs(u) - thr, 0.0), u);
    const double dd = an - at;
    const float clo = lo_[i & 31], chi = hi_[i & 31];
    const float ci = i < 32 ? clo : chi;
    int lo = __builtin_amdgcn_readlane(__double2loint(dd), i);
    int hi = __builtin_amdgcn_readlane(__double2hiint(dd), i);
    const double d = __hiloint2double(hi, lo);
    const bool me = lane == i;
    if (V >= 1) gbef = me ? gt : gbef;
    const double cd = (double)ci * d;
    u -= cd;
    if (V >= 2) gt -= cd;
    __builtin_amdgcn_sched_barrier(0);
    if (V >= 1) anv = me ? an : anv;
  }
  const long long t1 = clock64();
  if (threadIdx.x == 0) *out = t1 - t0;
  return u + gt + gbef + anv;
}

__global__ void chains(long long* out, double* sink, float* sinkf) {
  double x = threadIdx.x * 1e-3, y = 1.0000001;
  float xf = threadIdx.x * 1e-3f, yf = 1.0000001f;
  long long t0, t1;
  int k = 0;
  // 0: v_add_f64 chain
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "v"(y));
  t1 = clock64();
  if (threadIdx.x == 0) out[k++] = t1 - t0;
  // 1: v_fma_f64 chain
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x) : "v"(y));
  t1 = clock64();
  if (threadIdx.x == 0) out[k++] = t1 - t0;
  // 2: v_add_f32 chain
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(xf) : "v"(yf));
  t1 = clock64();
  if (threadIdx.x == 0) out[k++] = t1 - t0;
  // 3: v_fma_f32 chain
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(xf) : "v"(yf));
  t1 = clock64();
  if (threadIdx.x == 0) out[k++] = t1 - t0;
  // 4: readlane -> VALU chain (f32): x = x + readlane(x, 5)
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    int s;
    asm volatile("v_readlane_b32 %0, %1, 5\n\ts_nop 4\n\tv_add_f32 %1, %0, %1" : "=s"(s), "+v"(xf));
  }
  t1 = clock64();
  if (threadIdx.x == 0) out[k++] = t1 - t0;
  // 5: v_cmp_f32 -> s_ff1 -> readlane -> v_add_f32 (the ballot hop)
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    asm volatile(
        "v_cmp_gt_f32 vcc, %0, %1\n\t"
        "s_ff1_i32_b64 s40, vcc\n\t"
        "s_and_b32 s40, s40, 63\n\t"
        "v_readlane_b32 s42, %0, s40\n\t"
        "s_nop 4\n\t"
        "v_add_f32 %0, %0, s42"
        : "+v"(xf) : "v"(yf) : "vcc", "s40", "s42");
  }
  t1 = clock64();
  if (threadIdx.x == 0) out[k++] = t1 - t0;
  // 6: the known-order CD step in fp64 (C++ as in csrc/enet.hip), lane 7 moves each step
  {
    double u = x, at = 0.25, thr = 0.001, c = 0.5 + threadIdx.x * 1e-3;
    t0 = clock64();
    for (int i = 0; i < N; ++i) {
      const double an = copysign(fmax(fabs(u) - thr, 0.0), u);
      const double dd = an - at;
      int lo = __builtin_amdgcn_readlane(__double2loint(dd), 7);
      int hi = __builtin_amdgcn_readlane(__double2hiint(dd), 7);
      const double d = __hiloint2double(hi, lo);
      u -= c * d;
    }
    t1 = clock64();
    x += u;
    if (threadIdx.x == 0) out[k++] = t1 - t0;
  }
  // 7: v_max_f64 chain
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("v_max_f64 %0, %0, %1" : "+v"(x) : "v"(y));
  t1 = clock64();
  if (threadIdx.x == 0) out[k++] = t1 - t0;
  // 8: v_mul_f64 chain
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x) : "v"(y));
  t1 = clock64();
  if (threadIdx.x == 0) out[k++] = t1 - t0;
  // 9: independent v_add_f64 (issue rate): 4 interleaved chains
  double x2 = x + 1, x3 = x + 2, x4 = x + 3;
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < N / 4; ++i)
    asm volatile("v_add_f64 %0, %0, %4\n\tv_add_f64 %1, %1, %4\n\tv_add_f64 %2, %2, %4\n\tv_add_f64 %3, %3, %4"
                 : "+v"(x), "+v"(x2), "+v"(x3), "+v"(x4) : "v"(y));
  t1 = clock64();
  if (threadIdx.x == 0) out[k++] = t1 - t0;
  // 10: independent v_add_f32 issue rate
  float f2 = xf + 1, f3 = xf + 2, f4 = xf + 3;
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < N / 4; ++i)
    asm volatile("v_add_f32 %0, %0, %4\n\tv_add_f32 %1, %1, %4\n\tv_add_f32 %2, %2, %4\n\tv_add_f32 %3, %3, %4"
                 : "+v"(xf), "+v"(f2), "+v"(f3), "+v"(f4) : "v"(yf));
  t1 = clock64();
  if (threadIdx.x == 0) out[k++] = t1 - t0;
  // 11: v_readlane alone chain via SALU (s -> v_mov -> readlane)
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    asm volatile("v_readlane_b32 s44, %0, 3\n\ts_nop 4\n\tv_mov_b32 %0, s44" : "+v"(xf) : : "s44");
  }
  t1 = clock64();
  if (threadIdx.x == 0) out[k++] = t1 - t0;
  // 14: the known-order CD step in fp32
  {
    float u = xf, at = 0.25f, thr = 0.001f, c = 0.5f + threadIdx.x * 1e-3f;
    t0 = clock64();
    for (int i = 0; i < N; ++i) {
      const float an = copysignf(fmaxf(fabsf(u) - thr, 0.0f), u);
      const float dd = an - at;
      const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dd), 7));
      u -= c * d;
    }
    t1 = clock64();
    xf += u;
    if (threadIdx.x == 0) out[14] = t1 - t0;
  }
  // 15..17: the csrc/enet.hip known step with its register-indexed diagonal row (0),
  // + the per-lane bookkeeping (1), + gt tracking (2)
  x += kstep<0>(x, sinkf, out + 15);
  x += kstep<1>(x, sinkf, out + 16);
  x += kstep<2>(x, sinkf, out + 17);
  // 12: wall clock ticks over the same loop as 0 (clock ratio)
  long long w0 = wall_clock64();
  t0 = clock64();
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "v"(y));
  t1 = clock64();
  long long w1 = wall_clock64();
  if (threadIdx.x == 0) { out[k++] = t1 - t0; out[k++] = w1 - w0; }
  sink[threadIdx.x] = x + x2 + x3 + x4;
  sinkf[threadIdx.x] = xf + f2 + f3 + f4;
}

int main() {
  long long* d;
  double* s;
  float* sf;
  hipMalloc(&d, 64 * sizeof(long long));
  hipMalloc(&s, 64 * sizeof(double));
  hipMalloc(&sf, 64 * sizeof(float));
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(chains, dim3(1), dim3(64), 0, 0, d, s, sf);
  hipDeviceSynchronize();
  long long h[64];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[] = {"add_f64", "fma_f64", "add_f32", "fma_f32", "readlane->add_f32",
                         "cmp_f32->ff1->readlane->add_f32", "known CD step fp64", "max_f64",
                         "mul_f64", "indep add_f64 (issue)", "indep add_f32 (issue)",
                         "readlane->mov", "add_f64 (again)"};
  printf("%-36s %7.2f cycles/link\n", "known CD step fp32", (double)h[14] / N);
  const char* vn[] = {"kernel step: + indexed diag row", "  + bookkeeping (gbef, anv)",
                      "  + gt tracking"};
  for (int v = 0; v < 3; ++v) printf("%-36s %7.2f cycles/link\n", vn[v], (double)h[15 + v] / N);
  for (int i = 0; i < 13; ++i) printf("%-36s %7.2f cycles/link\n", names[i], (double)h[i] / N);
  printf("wall ticks over %d add_f64: %lld (clock64 %lld) -> shader MHz ~ %.0f\n", N, h[13], h[12],
         100.0 * h[12] / h[13]);
  return 0;
}
