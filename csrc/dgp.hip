// Tutorial-shape synthetic DGP generated directly in HBM.
// Same generative model as ate_replication_causalml_amd/data/dgp.py::raw_columns
// (Philox keyed by (seed, P_DGP, column stream, GLOBAL row id)), so any shard of
// any world size produces identical rows. Writes the panel layout of ops/panel.py:
//   [one, 15 cts, sex, 5 vote-history, extras..., W, Y, W_hi, W_lo, Y_hi, Y_lo]
// rows of a segment are written at [row0, row0 + count) of the panel.
#include "common.hpp"

using namespace ate;

__device__ __forceinline__ float dgp_normal(uint64_t seed, uint32_t stream, uint64_t idx) {
  u32x4 w = rand4(seed, P_DGP, stream, idx);
  float u1 = ((float)(w.x >> 8) + 1.0f) * (1.0f / 16777217.0f);
  float u2 = (float)(w.y >> 8) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}
__device__ __forceinline__ float dgp_uniform(uint64_t seed, uint32_t stream, uint64_t idx) {
  u32x4 w = rand4(seed, P_DGP, stream, idx);
  return (float)(w.x >> 8) * (1.0f / 16777216.0f);
}

// element (c, i) at c*cs + (i/64)*bs + i%64: column-major panels (cs = ld, bs = 64) or
// 64-row blocked panels (cs = 64, bs = 64*P; ops/panel.py DevicePanel.blocked)
__device__ __forceinline__ int64_t pidx(int c, int64_t i, int64_t cs, int64_t bs) {
  return (int64_t)c * cs + (i >> 6) * bs + (i & 63);
}
template <typename T>
__device__ __forceinline__ void put(T* X, int64_t cs, int64_t bs, int c, int64_t i, float v) {
  X[pidx(c, i, cs, bs)] = (T)v;
}
template <>
__device__ __forceinline__ void put<bf16_t>(bf16_t* X, int64_t cs, int64_t bs, int c, int64_t i,
                                            float v) {
  X[pidx(c, i, cs, bs)] = f32_to_bf16_rne(v);
}

template <typename T>
__global__ void dgp_fill_kernel(T* __restrict__ X, int64_t cs, int64_t bs, int64_t row0, int64_t count,
                                int64_t gid0, uint64_t seed, int p_extra, int hi_lo) {
  const float FL = 0.6f, FS = 0.8f;  // factor loading, sqrt(1 - 0.36)
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < count;
       r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t g = (uint64_t)(gid0 + r);
    const int64_t i = row0 + r;
    const float f = dgp_normal(seed, 40, g);
    int c = 0;
    put(X, cs, bs, c++, i, 1.0f);
    float yob = 0.f;
    for (int j = 0; j < 15; ++j) {
      float z = dgp_normal(seed, j, g);
      float v = j < 3 ? z : FL * f + FS * z;
      if (j == 0) yob = v;
      put(X, cs, bs, c++, i, v);
    }
    const float latent = dgp_normal(seed, 41, g) + 0.3f * yob;
    const float sex = dgp_uniform(seed, 60, g) < 0.5f ? 1.f : 0.f;
    put(X, cs, bs, c++, i, sex);
    float hsum = 0.f;
    for (int k = 0; k < 5; ++k) {
      float h = (dgp_normal(seed, 50 + k, g) + 0.5f * latent > 0.6f) ? 1.f : 0.f;
      hsum += h;
      put(X, cs, bs, c++, i, h);
    }
    for (int j = 0; j < p_extra; ++j) {
      float z = dgp_normal(seed, 100 + j, g);
      float v = (j % 4 == 3) ? (z > 0.f ? 1.f : 0.f) : FL * f + FS * z;
      put(X, cs, bs, c++, i, v);
    }
    const float w = dgp_uniform(seed, 61, g) < (1.0f / 6.0f) ? 1.f : 0.f;
    const float eta = -1.4f + 0.3f * hsum + 0.2f * latent + 0.45f * w;
    const float y = dgp_uniform(seed, 62, g) < 1.0f / (1.0f + expf(-eta)) ? 1.f : 0.f;
    put(X, cs, bs, c++, i, w);
    put(X, cs, bs, c++, i, y);
    if (hi_lo) {  // binary -> hi exact, lo 0
      put(X, cs, bs, c++, i, w);
      put(X, cs, bs, c++, i, 0.f);
      put(X, cs, bs, c++, i, y);
      put(X, cs, bs, c++, i, 0.f);
    }
  }
}

// dtype 1 f32, 2 f64, 3 bf16
ATE_API int ate_dgp_fill(int dtype, void* X, int64_t cs, int64_t bs, int64_t row0, int64_t count, int64_t gid0,
                         uint64_t seed, int p_extra, int hi_lo, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(grid_for(count, 256, 8192)), block(256);
  if (dtype == 1)
    hipLaunchKernelGGL(dgp_fill_kernel<float>, grid, block, 0, s, (float*)X, cs, bs, row0, count, gid0,
                       seed, p_extra, hi_lo);
  else if (dtype == 2)
    hipLaunchKernelGGL(dgp_fill_kernel<double>, grid, block, 0, s, (double*)X, cs, bs, row0, count,
                       gid0, seed, p_extra, hi_lo);
  else if (dtype == 3)
    hipLaunchKernelGGL(dgp_fill_kernel<bf16_t>, grid, block, 0, s, (bf16_t*)X, cs, bs, row0, count,
                       gid0, seed, p_extra, hi_lo);
  else
    return -1;
  ATE_CHECK_LAUNCH();
  return 0;
}
