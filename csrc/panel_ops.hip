// Panel GEMV primitives over the column-major HBM panel (rows = observations,
// one contiguous column per covariate), with a per-row group id (e.g. treatment arm):
//
//   ate_panel_xtv: out[a][j] = sum_{i : grp[i] == a} X[xcols[j]][i] * v[i]   (A groups)
//   ate_panel_xv : out[i]    = sum_j X[xcols[j]][i] * V[grp[i]][j]            (0 if grp < 0)
//
// Used by the residual-balancing interior-point solver (estimators/balance.py), whose
// per-iteration O(n) work besides the weighted Gram is exactly these two products.
// xtv: one block per column, fixed-order block reduction -> deterministic.
#include "common.hpp"

namespace {

constexpr int NT = 256;

template <typename T, int A>
__global__ __launch_bounds__(NT) void xtv_kernel(const T* __restrict__ X, int64_t ld,
                                                 const int* __restrict__ xcols,
                                                 const double* __restrict__ v,
                                                 const int8_t* __restrict__ grp, int64_t n,
                                                 double* __restrict__ out, int p) {
  __shared__ double smem[16 * A];
  const int j = blockIdx.x;
  const T* xc = X + (int64_t)xcols[j] * ld;
  double acc[A];
#pragma unroll
  for (int a = 0; a < A; ++a) acc[a] = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += NT) {
    const int g = grp[i];
    const double xv = (double)xc[i] * v[i];
#pragma unroll
    for (int a = 0; a < A; ++a) acc[a] += g == a ? xv : 0.0;
  }
  ate::block_sum<A>(acc, smem);
  if (threadIdx.x == 0)
#pragma unroll
    for (int a = 0; a < A; ++a) out[(int64_t)a * p + j] = acc[a];
}

template <typename T>
__global__ __launch_bounds__(NT) void xv_kernel(const T* __restrict__ X, int64_t ld,
                                                const int* __restrict__ xcols, int p,
                                                const double* __restrict__ V, int A,
                                                const int8_t* __restrict__ grp, int64_t n,
                                                double* __restrict__ out) {
  extern __shared__ double sV[];          // [A][p]
  for (int k = threadIdx.x; k < A * p; k += NT) sV[k] = V[k];
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int g = grp[i];
    double s = 0.0;
    if (g >= 0) {
      const double* vv = sV + g * p;
      for (int j = 0; j < p; ++j) s += (double)X[(int64_t)xcols[j] * ld + i] * vv[j];
    }
    out[i] = s;
  }
}

template <typename T>
int xtv_launch(const void* X, int64_t ld, const int* xcols, int p, const double* v,
               const int8_t* grp, int64_t n, int A, double* out, hipStream_t st) {
  if (A == 1)
    ATE_LAUNCH((xtv_kernel<T, 1>), dim3(p), dim3(NT), 0, st, (const T*)X, ld, xcols, v,
                       grp, n, out, p);
  else if (A == 2)
    ATE_LAUNCH((xtv_kernel<T, 2>), dim3(p), dim3(NT), 0, st, (const T*)X, ld, xcols, v,
                       grp, n, out, p);
  else
    return -1;
  return 0;
}

}  // namespace

// dt: 1 fp32 panel, 2 fp64 panel
ATE_API int ate_panel_xtv(int dt, const void* X, int64_t ld, const void* xcols, int p,
                          const void* v, const void* grp, int64_t n, int A, void* out,
                          void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int rc = dt == 2 ? xtv_launch<double>(X, ld, (const int*)xcols, p, (const double*)v,
                                        (const int8_t*)grp, n, A, (double*)out, st)
                   : xtv_launch<float>(X, ld, (const int*)xcols, p, (const double*)v,
                                       (const int8_t*)grp, n, A, (double*)out, st);
  if (rc) return rc;
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_panel_xv(int dt, const void* X, int64_t ld, const void* xcols, int p,
                         const void* V, int A, const void* grp, int64_t n, void* out,
                         void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const size_t sh = sizeof(double) * (size_t)A * p;
  if (sh > 64 * 1024) return -1;
  dim3 grid(ate::grid_for(n, NT, 2048));
  if (dt == 2)
    ATE_LAUNCH(xv_kernel<double>, grid, dim3(NT), sh, st, (const double*)X, ld,
                       (const int*)xcols, p, (const double*)V, A, (const int8_t*)grp, n,
                       (double*)out);
  else
    ATE_LAUNCH(xv_kernel<float>, grid, dim3(NT), sh, st, (const float*)X, ld,
                       (const int*)xcols, p, (const double*)V, A, (const int8_t*)grp, n,
                       (double*)out);
  ATE_CHECK_LAUNCH();
  return 0;
}
