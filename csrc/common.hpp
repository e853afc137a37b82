// Shared device/host helpers for the gfx950 (MI355X / CDNA4) kernel library.
// Wave size is 64 everywhere: lane = threadIdx.x & 63.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

#define ATE_API extern "C" __attribute__((visibility("default")))

namespace ate {

constexpr int WAVE = 64;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef unsigned short bf16_t;   // storage type for bf16 panels

__device__ __forceinline__ float bf16_to_f32(bf16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
__host__ __device__ inline bf16_t f32_to_bf16_rne(float f) {
#ifdef __HIP_DEVICE_COMPILE__
  uint32_t u = __float_as_uint(f);
#else
  uint32_t u; __builtin_memcpy(&u, &f, 4);
#endif
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

// ---------------------------------------------------------------- Philox4x32-10
// Must match ate_replication_causalml_amd/parallel/rng.py bit for bit.
struct u32x4 { uint32_t x, y, z, w; };

__host__ __device__ inline u32x4 philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}

// purposes: keep in sync with rng.py
enum : uint32_t { P_FOLD = 1, P_BOOT = 2, P_RF_BOOT = 3, P_RF_MTRY = 4, P_DGP = 5,
                  P_SUBSAMPLE = 6, P_GBDT = 7, P_SAMPLE_ROWS = 8 };

__host__ __device__ inline u32x4 rand4(uint64_t seed, uint32_t purpose, uint32_t stream,
                                       uint64_t index) {
  return philox4x32((uint32_t)index, (uint32_t)(index >> 32), purpose, stream,
                    (uint32_t)seed, (uint32_t)(seed >> 32));
}
// uniform integer in [0, n): (u * n) >> 32, word 0
__host__ __device__ inline uint32_t rand_below(uint64_t seed, uint32_t purpose, uint32_t stream,
                                               uint64_t index, uint32_t n) {
  u32x4 r = rand4(seed, purpose, stream, index);
  return (uint32_t)(((uint64_t)r.x * (uint64_t)n) >> 32);
}
__host__ __device__ inline float rand_uniform(uint64_t seed, uint32_t purpose, uint32_t stream,
                                              uint64_t index) {
  u32x4 r = rand4(seed, purpose, stream, index);
  return (float)(r.x >> 8) * (1.0f / 16777216.0f);
}

// ---------------------------------------------------------------- reductions
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { T u = __shfl_xor(v, o, 64); v = v > u ? v : u; }
  return v;
}

// Block-wide sum of NV doubles (blockDim multiple of 64, <= 1024). Result valid in thread 0.
template <int NV>
__device__ inline void block_sum(double (&v)[NV], double* smem /* >= 16*NV */) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) smem[wid * NV + k] = v[k];
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double s = 0.0;
      for (int w = 0; w < nw; ++w) s += smem[w * NV + k];
      v[k] = s;
    }
  }
  __syncthreads();
}

inline int grid_for(int64_t n, int block, int cap = 2048) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

}  // namespace ate

// Device bounds checks: compiled in by a debug build (-DATE_DEVICE_ASSERT;
// ATE_DEBUG=1, ate_replication_causalml_amd/_build.py -> _lib/libatehip_debug.so) and out
// of the production library (the condition is not even evaluated). A failed check prints
// its source site and traps, so an index bug is named instead of found by bisection.
#ifdef ATE_DEVICE_ASSERT
#define ATE_DASSERT(cond)                                                          \
  do {                                                                             \
    if (!(cond)) {                                                                 \
      printf("ATE_DASSERT failed %s:%d: %s\n", __FILE__, __LINE__, #cond);         \
      __builtin_trap();                                                            \
    }                                                                              \
  } while (0)
#else
#define ATE_DASSERT(cond) do { } while (0)
#endif

// ---------------------------------------------------------------- launch errors
// Every kernel launch goes through ATE_LAUNCH: hipLaunchKernelGGL between a check of the
// error state BEFORE it and one AFTER it. A failed launch is recorded as "hipErrorName
// (code): description" with its entry point, file and line, and the entry point's next
// ATE_CHECK_LAUNCH returns the HIP error code; ate_last_error (csrc/errors.hip) hands the
// text to the host, where _native.call puts it in its exception. An error left pending by an
// EARLIER HIP call (another library's, or an ignored one) is not this launch's: ATE_LAUNCH
// clears it first and records it separately as stale (ate_last_stale_error), so it cannot
// be reported under this entry point's name (the unexplained "ate_forest_fit_exact failed
// with status 1" of round 5 was such a report: profiles/r05_debug/README.md).
namespace ate {
struct LaunchError {
  int code = 0;
  bool pending = false;        // recorded by a launch, not yet returned by ATE_CHECK_LAUNCH
  char msg[512] = {0};
};
inline thread_local LaunchError g_launch_error, g_stale_error;

inline void record_error(LaunchError& slot, hipError_t e, const char* what, const char* func,
                         const char* file, int line) {
  slot.code = (int)e;
  snprintf(slot.msg, sizeof(slot.msg), "%s (%d): %s; %s in %s at %s:%d", hipGetErrorName(e),
           (int)e, hipGetErrorString(e), what, func, file, line);
}
inline void launch_pre(const char* func, const char* file, int line) {
  const hipError_t e = hipGetLastError();   // returns AND clears the pending error
  if (e != hipSuccess)
    record_error(g_stale_error, e, "pending before a launch (an earlier HIP call's)", func,
                 file, line);
}
inline void launch_post(const char* func, const char* file, int line) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess && !g_launch_error.pending) {
    record_error(g_launch_error, e, "kernel launch failed", func, file, line);
    g_launch_error.pending = true;
  }
}
inline int take_launch_error() {
  if (!g_launch_error.pending) return 0;
  g_launch_error.pending = false;
  return g_launch_error.code;
}
}  // namespace ate

// Launch shapes of the heavy kernels (block size, dynamic LDS), registered next to each
// kernel: the debug build checks them against the compiled kernels' attributes at library
// load (ate_check_kernel_resources, csrc/errors.hip; _native.hip() under ATE_DEBUG=1).
namespace ate {
struct KernelShape {
  const void* fn;
  const char* name;
  int threads, dyn_lds;
};
inline std::vector<KernelShape>& kernel_shapes() {
  static std::vector<KernelShape> v;
  return v;
}
struct KernelShapeReg {
  KernelShapeReg(const void* f, const char* n, int t, int d) { kernel_shapes().push_back({f, n, t, d}); }
};
}  // namespace ate
#define ATE_CAT2(a, b) a##b
#define ATE_CAT(a, b) ATE_CAT2(a, b)
#define ATE_KERNEL_SHAPE(name, threads, dyn_lds, ...)                                   \
  static ate::KernelShapeReg ATE_CAT(ate_kshape_, __LINE__)((const void*)(__VA_ARGS__), \
                                                              name, threads, dyn_lds);

#define ATE_LAUNCH(...)                                   \
  do {                                                    \
    ate::launch_pre(__func__, __FILE__, __LINE__);        \
    hipLaunchKernelGGL(__VA_ARGS__);                      \
    ate::launch_post(__func__, __FILE__, __LINE__);       \
  } while (0)

#define ATE_CHECK_LAUNCH()                                \
  do {                                                    \
    const int e_ = ate::take_launch_error();              \
    if (e_ != 0) return e_;                               \
  } while (0)
