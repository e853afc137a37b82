// Data-preparation kernels on the column-major fp64 design matrix X[p][ld]:
//
// * K02 col_moments / R scale() (ate_replication.Rmd:72-74, P5): per-column non-NaN
//   count, mean and sample SD (n-1), two passes like R (mean first, then the sum of
//   squared deviations), NaNs ignored as scale() does; fixed-order two-level fp64
//   reductions (per-chunk partials, then one in-order sum per column), so results
//   are bitwise reproducible; then an in-place standardisation of the selected
//   columns (the 6 binary covariates stay 0/1).
// * K21 interaction_expand (belloni, ate_functions.R:290-296, quirk Q10): the design
//   [x_1..x_p, x_c1 * x_c2 for c1, c2 in 1..p] (both orders and squares), written
//   column-major straight into the output panel.
#include "common.hpp"

using namespace ate;

namespace {

constexpr int NT = 256;
constexpr int CHUNKS = 64;          // fixed row chunks per column (deterministic order)

// mode 0: partial (count, sum); mode 1: partial sum (x - mean)^2
__global__ __launch_bounds__(NT) void colmom_partial_kernel(const double* __restrict__ X,
                                                            int64_t ld, int64_t n, int mode,
                                                            const double* __restrict__ mean,
                                                            double* __restrict__ part) {
  __shared__ double smem[16 * 2];
  const int j = blockIdx.y, c = blockIdx.x;
  const int64_t per = (n + CHUNKS - 1) / CHUNKS;
  const int64_t r0 = c * per, r1 = min(n, r0 + per);
  const double* x = X + (int64_t)j * ld;
  const double m = mode ? mean[j] : 0.0;
  double v[2] = {0.0, 0.0};
  for (int64_t i = r0 + threadIdx.x; i < r1; i += NT) {
    const double a = x[i];
    if (a != a) continue;                               // NaN: ignored (scale, na.rm)
    if (mode == 0) { v[0] += 1.0; v[1] += a; }
    else { const double dv = a - m; v[0] += dv * dv; }
  }
  block_sum<2>(v, smem);
  if (threadIdx.x == 0) {
    part[((int64_t)j * CHUNKS + c) * 2] = v[0];
    part[((int64_t)j * CHUNKS + c) * 2 + 1] = v[1];
  }
}

// out[j] = {count, mean, sd}: mode 0 fills count/mean, mode 1 the SD
__global__ void colmom_final_kernel(const double* __restrict__ part, int p, int mode,
                                    double* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= p) return;
  double a = 0.0, b = 0.0;
  for (int c = 0; c < CHUNKS; ++c) {
    a += part[((int64_t)j * CHUNKS + c) * 2];
    b += part[((int64_t)j * CHUNKS + c) * 2 + 1];
  }
  if (mode == 0) {
    out[3 * j] = a;
    out[3 * j + 1] = a > 0 ? b / a : NAN;
  } else {
    const double cnt = out[3 * j];
    out[3 * j + 2] = cnt > 1 ? sqrt(a / (cnt - 1.0)) : NAN;
  }
}

__global__ void colmom_mean_kernel(const double* __restrict__ out, int p, double* __restrict__ mean) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < p) mean[j] = out[3 * j + 1];
}

// X[j][i] = (X[j][i] - mean_j) / sd_j for columns with sel[j] != 0 (NaN stays NaN)
__global__ __launch_bounds__(NT) void standardize_kernel(double* __restrict__ X, int64_t ld,
                                                         int64_t n, const double* __restrict__ mom,
                                                         const uint8_t* __restrict__ sel) {
  const int j = blockIdx.y;
  if (!sel[j]) return;
  const double m = mom[3 * j + 1], s = mom[3 * j + 2];
  double* x = X + (int64_t)j * ld;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
    x[i] = (x[i] - m) / s;
}

// out column q < p: x_q; q = p + c1 * p + c2: x_c1 * x_c2
__global__ __launch_bounds__(NT) void interactions_kernel(const double* __restrict__ X, int64_t ldx,
                                                          int64_t n, int p,
                                                          double* __restrict__ out, int64_t ldo) {
  const int q = blockIdx.y;
  const double* a;
  const double* b = nullptr;
  if (q < p) {
    a = X + (int64_t)q * ldx;
  } else {
    const int c1 = (q - p) / p, c2 = (q - p) - c1 * p;
    a = X + (int64_t)c1 * ldx;
    b = X + (int64_t)c2 * ldx;
  }
  double* o = out + (int64_t)q * ldo;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
    o[i] = b ? a[i] * b[i] : a[i];
}

}  // namespace

// mom[p][3] = {count, mean, sd} of the non-NaN entries; part: p * CHUNKS * 2 doubles,
// mean: p doubles of scratch
ATE_API int ate_col_moments(const void* X, int64_t ld, int64_t n, int p, void* part, void* mean,
                            void* mom, void* stream) {
  if (p < 1 || n < 0 || ld < n) return -1;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(CHUNKS, p), fb((p + 63) / 64);
  for (int mode = 0; mode < 2; ++mode) {
    ATE_LAUNCH(colmom_partial_kernel, g, dim3(NT), 0, st, (const double*)X, ld, n, mode,
                       (const double*)mean, (double*)part);
    ATE_LAUNCH(colmom_final_kernel, fb, dim3(64), 0, st, (const double*)part, p, mode,
                       (double*)mom);
    if (mode == 0)
      ATE_LAUNCH(colmom_mean_kernel, fb, dim3(64), 0, st, (const double*)mom, p,
                         (double*)mean);
  }
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_standardize(void* X, int64_t ld, int64_t n, int p, const void* mom,
                            const void* sel, void* stream) {
  if (p < 1 || ld < n) return -1;
  ATE_LAUNCH(standardize_kernel, dim3(grid_for(n, NT, 256), p), dim3(NT), 0,
                     (hipStream_t)stream, (double*)X, ld, n, (const double*)mom,
                     (const uint8_t*)sel);
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_interactions(const void* X, int64_t ldx, int64_t n, int p, void* out, int64_t ldo,
                             void* stream) {
  if (p < 1 || (int64_t)p * (p + 1) > 65535 || ldx < n || ldo < n) return -1;
  ATE_LAUNCH(interactions_kernel, dim3(grid_for(n, NT, 64), p * (p + 1)), dim3(NT), 0,
                     (hipStream_t)stream, (const double*)X, ldx, n, p, (double*)out, ldo);
  ATE_CHECK_LAUNCH();
  return 0;
}
