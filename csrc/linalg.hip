// K05 small_spd_solve + K06 ols_se + K07 irls_step + GEMV predictors.
//
// Normal equations are solved from the fp64 Gram (K01) with a column-order
// pivoted Cholesky: column j is aliased (R's lm coefficient NA) when its Schur
// complement d_j < tol^2 * G_jj, i.e. when its norm after projecting out the
// accepted earlier columns is below tol * ||x_j|| -- the same rule as LINPACK
// dqrdc2's limited pivoting used by lm (reference ate_functions.R:28,53,74,320,363).
//
// IRLS (glm.fit, ate_functions.R:156,218,231) runs as a fixed-budget sequence of
// launches (gram -> solve -> update -> check) x maxit with a device-side `done`
// flag: every kernel returns immediately once converged, so the loop needs no
// host round trip and can be captured in a hipGraph.
#include "common.hpp"

using namespace ate;

// ------------------------------------------------------------------ K05/K06
// work: >= k*k doubles (L) + k*k (inverse columns). out layout:
// beta[k], invdiag[k], aux[4] = {rank, yty - beta'Xty, yty, 0}
// kdev (optional, device): solve over the first min(k, *kdev) entries of cols only -- a
// graph-captured caller with a data-dependent design size passes a fixed-size column list
// (active columns first) and the active count (estimators/lasso.py _belloni_body).
__global__ __launch_bounds__(1024) void chol_solve_kernel(
    const double* __restrict__ G, int P, const int* __restrict__ cols, int kmax, int rcol,
    const double* __restrict__ rhs_vec, double tol, double* __restrict__ L, double* __restrict__ Linv,
    double* __restrict__ beta, double* __restrict__ invdiag, double* __restrict__ aux,
    const int* __restrict__ done, const int* __restrict__ kdev) {
  if (done && *done) return;
  const int k = kdev ? min(kmax, max(0, *kdev)) : kmax;
  extern __shared__ double sm[];      // b[k], y[k], alias flags as double[k]
  double* b = sm;
  double* y = sm + k;
  double* al = sm + 2 * k;
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int e = tid; e < k * k; e += nt) {
    int i = e / k, j = e % k;
    ATE_DASSERT(cols[i] >= 0 && cols[i] < P && cols[j] >= 0 && cols[j] < P);
    L[e] = G[(int64_t)cols[i] * P + cols[j]];
  }
  ATE_DASSERT(rhs_vec != nullptr || (rcol >= 0 && rcol < P));
  for (int i = tid; i < k; i += nt) {
    b[i] = rhs_vec ? rhs_vec[i] : G[(int64_t)cols[i] * P + rcol];
    al[i] = 0.0;
  }
  __syncthreads();
  // right-looking Cholesky on the lower triangle, column order, with aliasing
  for (int j = 0; j < k; ++j) {
    double d = L[j * k + j];
    double orig = G[(int64_t)cols[j] * P + cols[j]];
    bool alias = !(orig > 0.0) || !(d > tol * tol * orig);
    if (alias) {
      for (int i = j + tid; i < k; i += nt) L[i * k + j] = 0.0;
      if (tid == 0) al[j] = 1.0;
      __syncthreads();
      continue;
    }
    double ljj = sqrt(d);
    __syncthreads();
    for (int i = j + 1 + tid; i < k; i += nt) L[i * k + j] /= ljj;
    if (tid == 0) L[j * k + j] = ljj;
    __syncthreads();
    // trailing update of the lower triangle: rows i>j, cols j<m<=i
    const int rem = k - j - 1;
    const int64_t npair = (int64_t)rem * (rem + 1) / 2;
    for (int64_t e = tid; e < npair; e += nt) {
      // map e -> (ii, mm) with 0<=mm<=ii<rem
      int ii = (int)((sqrt(8.0 * (double)e + 1.0) - 1.0) * 0.5);
      while ((int64_t)ii * (ii + 1) / 2 > e) --ii;
      while ((int64_t)(ii + 1) * (ii + 2) / 2 <= e) ++ii;
      int mm = (int)(e - (int64_t)ii * (ii + 1) / 2);
      int i = j + 1 + ii, m = j + 1 + mm;
      L[i * k + m] -= L[i * k + j] * L[m * k + j];
    }
    __syncthreads();
  }
  // forward solve L y = b
  for (int i = tid; i < k; i += nt) y[i] = b[i];
  __syncthreads();
  for (int j = 0; j < k; ++j) {
    if (al[j] != 0.0) { if (tid == 0) y[j] = 0.0; __syncthreads(); continue; }
    double yj = y[j] / L[j * k + j];
    __syncthreads();
    if (tid == 0) y[j] = yj;
    for (int i = j + 1 + tid; i < k; i += nt) y[i] -= L[i * k + j] * yj;
    __syncthreads();
  }
  // back solve L' beta = y (in place in y)
  for (int j = k - 1; j >= 0; --j) {
    if (al[j] != 0.0) { if (tid == 0) y[j] = 0.0; __syncthreads(); continue; }
    double bj = y[j] / L[j * k + j];
    __syncthreads();
    if (tid == 0) y[j] = bj;
    for (int i = tid; i < j; i += nt) y[i] -= L[j * k + i] * bj;
    __syncthreads();
  }
  // inverse diagonal: column c of L^{-1} by forward substitution, one thread per column
  for (int c = tid; c < k; c += nt) {
    double* x = Linv + (int64_t)c * k;
    double s2 = 0.0;
    if (al[c] == 0.0) {
      for (int i = 0; i < c; ++i) x[i] = 0.0;
      for (int i = c; i < k; ++i) {
        if (al[i] != 0.0) { x[i] = 0.0; continue; }
        double acc = (i == c) ? 1.0 : 0.0;
        for (int m = c; m < i; ++m) acc -= L[i * k + m] * x[m];
        x[i] = acc / L[i * k + i];
        s2 += x[i] * x[i];
      }
    }
    invdiag[c] = al[c] != 0.0 ? NAN : s2;
  }
  __syncthreads();
  for (int i = tid; i < k; i += nt) beta[i] = al[i] != 0.0 ? NAN : y[i];
  if (tid == 0) {
    int rank = 0;
    double bty = 0.0;
    for (int i = 0; i < k; ++i)
      if (al[i] == 0.0) { ++rank; bty += y[i] * b[i]; }
    double yty = rcol >= 0 ? G[(int64_t)rcol * P + rcol] : 0.0;
    aux[0] = rank;
    aux[1] = yty - bty;
    aux[2] = yty;
    aux[3] = 0.0;
  }
}

ATE_API int ate_chol_solve(const void* G, int P, const void* cols, int k, int rcol,
                           const void* rhs_vec, double tol, void* work, void* beta, void* invdiag,
                           void* aux, const void* done, void* stream) {
  if (k <= 0 || k > 4096) return -1;
  double* L = (double*)work;
  double* Linv = L + (int64_t)k * k;
  size_t sh = (size_t)3 * k * sizeof(double);
  ATE_LAUNCH(chol_solve_kernel, dim3(1), dim3(1024), sh, (hipStream_t)stream,
                     (const double*)G, P, (const int*)cols, k, rcol, (const double*)rhs_vec, tol,
                     L, Linv, (double*)beta, (double*)invdiag, (double*)aux, (const int*)done,
                     (const int*)nullptr);
  ATE_CHECK_LAUNCH();
  return 0;
}

// ate_chol_solve over the first *kdev (device int) of the k columns
ATE_API int ate_chol_solve_k(const void* G, int P, const void* cols, int k, const void* kdev,
                             int rcol, double tol, void* work, void* beta, void* invdiag, void* aux,
                             void* stream) {
  if (k <= 0 || k > 4096) return -1;
  double* L = (double*)work;
  double* Linv = L + (int64_t)k * k;
  size_t sh = (size_t)3 * k * sizeof(double);
  ATE_LAUNCH(chol_solve_kernel, dim3(1), dim3(1024), sh, (hipStream_t)stream,
                     (const double*)G, P, (const int*)cols, k, rcol, (const double*)nullptr, tol,
                     L, Linv, (double*)beta, (double*)invdiag, (double*)aux, (const int*)nullptr,
                     (const int*)kdev);
  ATE_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ batched SPD solve
// x[a] = K[a]^-1 r[a] for A small dense SPD systems (the balancing QP's Schur systems,
// estimators/balance.py): one workgroup per system, unpivoted right-looking Cholesky of the
// lower triangle in `work` (A * k * k doubles), then forward / back substitution in LDS. A
// non-positive pivot makes that system's solution NaN (LAPACK's potrf would report info > 0).
// Own kernel (not rocSOLVER) so the solve can be captured in a hipGraph.
__global__ __launch_bounds__(1024) void spd_solve_kernel(const double* __restrict__ K,
                                                         const double* __restrict__ r, int k,
                                                         double* __restrict__ work,
                                                         double* __restrict__ x) {
  extern __shared__ double sy[];          // [k]
  __shared__ int bad;
  const int a = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  ATE_DASSERT(k > 0 && k <= 4096);       // dynamic LDS sy[k]
  const double* Ka = K + (int64_t)a * k * k;
  double* L = work + (int64_t)a * k * k;
  for (int e = tid; e < k * k; e += nt) L[e] = Ka[e];
  for (int i = tid; i < k; i += nt) sy[i] = r[(int64_t)a * k + i];
  if (tid == 0) bad = 0;
  __syncthreads();
  for (int j = 0; j < k; ++j) {
    const double d = L[j * k + j];
    if (!(d > 0.0)) {                     // uniform: every thread reads the same value
      if (tid == 0) bad = 1;
      break;
    }
    const double ljj = sqrt(d);
    __syncthreads();
    for (int i = j + 1 + tid; i < k; i += nt) L[i * k + j] /= ljj;
    if (tid == 0) L[j * k + j] = ljj;
    __syncthreads();
    const int rem = k - j - 1;
    for (int e = tid; e < rem * rem; e += nt) {
      const int ii = e / rem, mm = e - ii * rem;
      if (mm <= ii) {
        const int i = j + 1 + ii, m = j + 1 + mm;
        L[i * k + m] -= L[i * k + j] * L[m * k + j];
      }
    }
    __syncthreads();
  }
  __syncthreads();
  if (bad) {
    for (int i = tid; i < k; i += nt) x[(int64_t)a * k + i] = NAN;
    return;
  }
  for (int j = 0; j < k; ++j) {           // L y = r
    const double yj = sy[j] / L[j * k + j];
    __syncthreads();
    if (tid == 0) sy[j] = yj;
    for (int i = j + 1 + tid; i < k; i += nt) sy[i] -= L[i * k + j] * yj;
    __syncthreads();
  }
  for (int j = k - 1; j >= 0; --j) {      // L' x = y
    const double xj = sy[j] / L[j * k + j];
    __syncthreads();
    if (tid == 0) sy[j] = xj;
    for (int i = tid; i < j; i += nt) sy[i] -= L[j * k + i] * xj;
    __syncthreads();
  }
  for (int i = tid; i < k; i += nt) x[(int64_t)a * k + i] = sy[i];
}

ATE_API int ate_spd_solve_batched(const void* K, const void* r, int A, int k, void* work, void* x,
                                  void* stream) {
  if (A <= 0 || k <= 0 || k > 4096) return -1;
  ATE_LAUNCH(spd_solve_kernel, dim3(A), dim3(256), (size_t)k * sizeof(double),
                     (hipStream_t)stream, (const double*)K, (const double*)r, k, (double*)work,
                     (double*)x);
  ATE_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ GEMV predictors
// eta_i = sum_c beta_c * X[cols_c][i] (NaN beta treated as 0 = aliased), optional
// override of one design column to a constant (counterfactual W=1 / W=0).
template <typename T>
__device__ __forceinline__ double linpred(const T* __restrict__ X, int64_t ld, const int* cols,
                                          const double* beta, int k, int64_t i, int ov_idx,
                                          double ov_val) {
  double eta = 0.0;
  for (int c = 0; c < k; ++c) {
    double bc = beta[c];
    if (bc != bc) continue;
    double x = (c == ov_idx) ? ov_val : (double)X[(int64_t)cols[c] * ld + i];
    eta += bc * x;
  }
  return eta;
}

// link: 0 identity, 1 logistic
template <typename T>
__global__ void predict_kernel(const T* __restrict__ X, int64_t ld, int64_t n, const int* cols,
                               const double* beta, int k, int ov_idx, double ov_val, int link,
                               double* __restrict__ out) {
  ATE_DASSERT(k >= 0 && ov_idx < k && ld >= n);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double eta = linpred(X, ld, cols, beta, k, i, ov_idx, ov_val);
    out[i] = link == 1 ? 1.0 / (1.0 + exp(-eta)) : eta;
  }
}

template <typename T>
static int predict_t(const void* X, int64_t ld, int64_t n, const void* cols, const void* beta, int k,
                     int ov_idx, double ov_val, int link, void* out, void* stream) {
  ATE_LAUNCH(predict_kernel<T>, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream,
                     (const T*)X, ld, n, (const int*)cols, (const double*)beta, k, ov_idx, ov_val,
                     link, (double*)out);
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_predict(int dtype, const void* X, int64_t ld, int64_t n, const void* cols,
                        const void* beta, int k, int ov_idx, double ov_val, int link, void* out,
                        void* stream) {
  if (dtype == 1) return predict_t<float>(X, ld, n, cols, beta, k, ov_idx, ov_val, link, out, stream);
  if (dtype == 2) return predict_t<double>(X, ld, n, cols, beta, k, ov_idx, ov_val, link, out, stream);
  return -1;
}

// ------------------------------------------------------------------ K07 IRLS (binomial, logit)
// init (first): mu = (y+0.5)/2 ; else mu = sigmoid(X beta). Writes eta/mu (fp64),
// working weight w = mu(1-mu) (panel dtype, 0 on padding rows) and working response
// z into panel column zcol; per-block deviance partials. valid = panel ones column.
__device__ __forceinline__ double binom_dev_i(double y, double mu) {
  double d = 0.0;
  if (y > 0.0) d += y * log(y / mu);
  if (y < 1.0) d += (1.0 - y) * log((1.0 - y) / (1.0 - mu));
  return 2.0 * d;
}

template <typename T>
__global__ void irls_update_kernel(T* __restrict__ X, int64_t ld, int64_t n, const int* cols,
                                   const double* beta, int k, int ycol, int vcol, int zcol, int first,
                                   double* __restrict__ eta_out, double* __restrict__ mu_out,
                                   T* __restrict__ wout, double* __restrict__ dev_partial,
                                   const int* __restrict__ done) {
  if (done && *done) return;
  ATE_DASSERT(ycol >= 0 && vcol >= 0 && zcol >= 0 && zcol != ycol && zcol != vcol && ld >= n);
  __shared__ double smem[16];
  double dev[1] = {0.0};
  const double eps10 = 10.0 * 2.220446049250313e-16;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double valid = (double)X[(int64_t)vcol * ld + i];
    double y = (double)X[(int64_t)ycol * ld + i];
    double mu, eta;
    if (first) {
      mu = (y + 0.5) * 0.5;
      eta = log(mu / (1.0 - mu));
    } else {
      eta = linpred(X, ld, cols, beta, k, i, -1, 0.0);
      mu = 1.0 / (1.0 + exp(-eta));
      mu = fmin(fmax(mu, eps10), 1.0 - eps10);
    }
    double me = mu * (1.0 - mu);
    eta_out[i] = eta;
    mu_out[i] = mu;
    wout[i] = (T)(valid * me);
    X[(int64_t)zcol * ld + i] = (T)(valid * (eta + (y - mu) / me));
    if (valid != 0.0) dev[0] += binom_dev_i(y, mu);
  }
  block_sum<1>(dev, smem);
  if (threadIdx.x == 0) dev_partial[blockIdx.x] = dev[0];
}

// state: [0]=dev_old, [1]=dev, [2]=iters, [3]=converged ; done flag separate (int)
__global__ void irls_check_kernel(const double* __restrict__ dev_partial, int nb, int first,
                                  double eps, int maxit, double* __restrict__ state,
                                  int* __restrict__ done) {
  if (*done) return;
  ATE_DASSERT(nb > 0);
  double dev = 0.0;
  for (int b = 0; b < nb; ++b) dev += dev_partial[b];
  if (first) {
    state[0] = dev;
    state[1] = dev;
    state[2] = 0;
    state[3] = 0;
    return;
  }
  state[2] += 1.0;
  state[1] = dev;
  if (fabs(dev - state[0]) / (fabs(dev) + 0.1) < eps) {
    state[3] = 1.0;
    *done = 1;
  } else if (state[2] >= maxit) {
    *done = 1;
  }
  state[0] = dev;
}

template <typename T>
static int irls_update_t(void* X, int64_t ld, int64_t n, const void* cols, const void* beta, int k,
                         int ycol, int vcol, int zcol, int first, void* eta, void* mu, void* w,
                         void* dev_partial, int nb, const void* done, void* stream) {
  ATE_LAUNCH(irls_update_kernel<T>, dim3(nb), dim3(256), 0, (hipStream_t)stream, (T*)X, ld,
                     n, (const int*)cols, (const double*)beta, k, ycol, vcol, zcol, first,
                     (double*)eta, (double*)mu, (T*)w, (double*)dev_partial, (const int*)done);
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_irls_update(int dtype, void* X, int64_t ld, int64_t n, const void* cols,
                            const void* beta, int k, int ycol, int vcol, int zcol, int first,
                            void* eta, void* mu, void* w, void* dev_partial, int nb,
                            const void* done, void* stream) {
  if (dtype == 1)
    return irls_update_t<float>(X, ld, n, cols, beta, k, ycol, vcol, zcol, first, eta, mu, w,
                                dev_partial, nb, done, stream);
  if (dtype == 2)
    return irls_update_t<double>(X, ld, n, cols, beta, k, ycol, vcol, zcol, first, eta, mu, w,
                                 dev_partial, nb, done, stream);
  return -1;
}

ATE_API int ate_irls_check(const void* dev_partial, int nb, int first, double eps, int maxit,
                           void* state, void* done, void* stream) {
  ATE_LAUNCH(irls_check_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream,
                     (const double*)dev_partial, nb, first, eps, maxit, (double*)state, (int*)done);
  ATE_CHECK_LAUNCH();
  return 0;
}
