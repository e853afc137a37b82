// Deterministic fp64 score reductions: K03 group_moments, K18 aipw_score_se,
// DML orthogonal-score moments, propensity clipping, K20 bootstrap replicates.
//
// Every reduction is two-level with a FIXED order (per-block partials written to
// a slab, then one block sums the slab in block order), so results are bitwise
// reproducible for a given launch geometry and are world-size independent once
// the per-rank partial vectors are all-reduced in rank order (parallel/comm.py).
// Inputs are fp64 score vectors or panel columns; rows with valid==0 (panel
// padding) are skipped.
#include "common.hpp"

using namespace ate;

constexpr int RB = 256;          // block size for row reductions
constexpr int RGRID = 1024;      // fixed grid for row reductions (deterministic order)

template <int NV, class F>
__global__ __launch_bounds__(RB) void rowreduce_kernel(F f, int64_t n, double* __restrict__ partial) {
  __shared__ double smem[16 * NV];
  double v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)RB + threadIdx.x; i < n; i += (int64_t)gridDim.x * RB)
    f(i, v);
  block_sum<NV>(v, smem);
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) partial[blockIdx.x * NV + k] = v[k];
}

template <int NV>
__global__ void slab_sum_kernel(const double* __restrict__ partial, int nb, double* __restrict__ out) {
  int k = threadIdx.x;
  if (k >= NV) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += partial[b * NV + k];
  out[k] = s;
}

template <int NV, class F>
static int rowreduce(F f, int64_t n, double* partial, double* out, hipStream_t s) {
  int nb = grid_for(n, RB, RGRID);
  ATE_LAUNCH((rowreduce_kernel<NV, F>), dim3(nb), dim3(RB), 0, s, f, n, partial);
  ATE_CHECK_LAUNCH();
  ATE_LAUNCH(slab_sum_kernel<NV>, dim3(1), dim3(64), 0, s, partial, nb, out);
  ATE_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ K03 group moments
// out[6] = {n0, sum y0, sum y0^2, n1, sum y1, sum y1^2}
template <typename T>
struct GroupMoments {
  const T* y; const T* w; const T* valid;
  __device__ void operator()(int64_t i, double (&v)[6]) const {
    if (valid && valid[i] == T(0)) return;
    double yi = (double)y[i];
    int g = (double)w[i] != 0.0 ? 3 : 0;
    v[g] += 1.0; v[g + 1] += yi; v[g + 2] += yi * yi;
  }
};

// naive_ate finalize (ate_functions.R:3-21): tau = ybar1 - ybar0,
// se = sqrt(var1/(n1-1) + var0/(n0-1)) with var the (n-1) sample variance (Q2).
__global__ void naive_finalize_kernel(const double* __restrict__ m, double* __restrict__ res) {
  double n0 = m[0], n1 = m[3];
  double mu0 = m[1] / n0, mu1 = m[4] / n1;
  double v0 = (m[2] - n0 * mu0 * mu0) / (n0 - 1.0);
  double v1 = (m[5] - n1 * mu1 * mu1) / (n1 - 1.0);
  res[0] = mu1 - mu0;
  res[1] = sqrt(v0 / (n0 - 1.0) + v1 / (n1 - 1.0));
}

template <typename T>
static int naive_t(const void* y, const void* w, const void* valid, int64_t n, void* partial,
                   void* moments, void* res, hipStream_t s) {
  GroupMoments<T> f{(const T*)y, (const T*)w, (const T*)valid};
  int rc = rowreduce<6>(f, n, (double*)partial, (double*)moments, s);
  if (rc) return rc;
  ATE_LAUNCH(naive_finalize_kernel, dim3(1), dim3(1), 0, s, (const double*)moments,
                     (double*)res);
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_naive(int dtype, const void* y, const void* w, const void* valid, int64_t n,
                      void* partial, void* moments, void* res, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 1) return naive_t<float>(y, w, valid, n, partial, moments, res, s);
  if (dtype == 2) return naive_t<double>(y, w, valid, n, partial, moments, res, s);
  return -1;
}

// ------------------------------------------------------------------ propensity clipping
// ate_functions.R:181-182: p==0 -> min positive, p==1 -> max below one.
__global__ __launch_bounds__(RB) void clip_minmax_kernel(const double* __restrict__ p, const double* __restrict__ valid,
                                   int64_t n, double* __restrict__ partial) {
  __shared__ double sm[2][16];
  double mn = INFINITY, mx = -INFINITY;
  for (int64_t i = blockIdx.x * (int64_t)RB + threadIdx.x; i < n; i += (int64_t)gridDim.x * RB) {
    if (valid && valid[i] == 0.0) continue;
    double pi = p[i];
    if (pi > 0.0) mn = fmin(mn, pi);
    if (pi < 1.0) mx = fmax(mx, pi);
  }
  mn = -wave_max(-mn);
  mx = wave_max(mx);
  int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sm[0][wid] = mn; sm[1][wid] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < RB / 64; ++w) { mn = fmin(mn, sm[0][w]); mx = fmax(mx, sm[1][w]); }
    partial[2 * blockIdx.x] = mn;
    partial[2 * blockIdx.x + 1] = mx;
  }
}

__global__ void clip_apply_kernel(double* __restrict__ p, int64_t n, const double* __restrict__ partial,
                                  int nb) {
  __shared__ double lim[2];
  if (threadIdx.x == 0) {
    double mn = INFINITY, mx = -INFINITY;
    for (int b = 0; b < nb; ++b) { mn = fmin(mn, partial[2 * b]); mx = fmax(mx, partial[2 * b + 1]); }
    lim[0] = mn; lim[1] = mx;
  }
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double pi = p[i];
    if (pi == 0.0 && lim[0] < INFINITY) p[i] = lim[0];
    else if (pi == 1.0 && lim[1] > -INFINITY) p[i] = lim[1];
  }
}

ATE_API int ate_clip_propensity(void* p, const void* valid, int64_t n, void* partial, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int nb = grid_for(n, RB, RGRID);
  ATE_LAUNCH(clip_minmax_kernel, dim3(nb), dim3(RB), 0, s, (const double*)p,
                     (const double*)valid, n, (double*)partial);
  ATE_CHECK_LAUNCH();
  ATE_LAUNCH(clip_apply_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, (double*)p, n,
                     (const double*)partial, nb);
  ATE_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ K18 AIPW
// est1 = w(y-mu1)/p + sign*(1-w)(y-mu0)/(1-p)  (sign=+1: reference Q7, -1 textbook)
// est2 = mu1 - mu0 ; a = w y/p - mu1 (w-p)/p - ((1-w)y/(1-p) + mu0 (w-p)/(1-p))
// out[6] = {sum est1 (non-NaN), n_nonNaN, sum est2, n, sum a, sum a^2}
struct AipwMoments {
  const double *w, *y, *p, *mu0, *mu1, *valid; double sign;
  __device__ void operator()(int64_t i, double (&v)[6]) const {
    if (valid && valid[i] == 0.0) return;
    double wi = w[i], yi = y[i], pi = p[i], m0 = mu0[i], m1 = mu1[i];
    double e1 = wi * (yi - m1) / pi + sign * (1.0 - wi) * (yi - m0) / (1.0 - pi);
    if (e1 == e1) { v[0] += e1; v[1] += 1.0; }
    v[2] += m1 - m0;
    v[3] += 1.0;
    double a = wi * yi / pi - m1 * (wi - pi) / pi - ((1.0 - wi) * yi / (1.0 - pi) + m0 * (wi - pi) / (1.0 - pi));
    if (a == a) { v[4] += a; v[5] += a * a; }
  }
};

// tau = mean(est1, na.rm) + mean(est2); se = sqrt(sum (a - tau)^2) / n (ate_functions.R:198-199)
__global__ void aipw_finalize_kernel(const double* __restrict__ m, double* __restrict__ res) {
  double tau = m[0] / m[1] + m[2] / m[3];
  double n = m[3];
  double ss = m[5] - 2.0 * tau * m[4] + n * tau * tau;
  res[0] = tau;
  res[1] = sqrt(fmax(ss, 0.0)) / n;
}

ATE_API int ate_aipw(const void* w, const void* y, const void* p, const void* mu0, const void* mu1,
                     const void* valid, int64_t n, double sign, void* partial, void* moments,
                     void* res, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  AipwMoments f{(const double*)w, (const double*)y, (const double*)p, (const double*)mu0,
                (const double*)mu1, (const double*)valid, sign};
  int rc = rowreduce<6>(f, n, (double*)partial, (double*)moments, s);
  if (rc) return rc;
  ATE_LAUNCH(aipw_finalize_kernel, dim3(1), dim3(1), 0, s, (const double*)moments,
                     (double*)res);
  ATE_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ DML orthogonal score
// residual vectors yr, wr -> {sum wr yr, sum wr^2, sum yr^2 wr^2, sum yr wr^3, sum wr^4, n, sum yr^2}
struct DmlMoments {
  const double *yr, *wr, *valid;
  __device__ void operator()(int64_t i, double (&v)[7]) const {
    if (valid && valid[i] == 0.0) return;
    double y = yr[i], w = wr[i], w2 = w * w;
    v[0] += w * y; v[1] += w2; v[2] += y * y * w2; v[3] += y * w2 * w; v[4] += w2 * w2;
    v[5] += 1.0; v[6] += y * y;
  }
};

// mode 0 (PLR, Neyman score): theta = S_wy/S_ww, psi = (yr - theta wr) wr,
//   se = sqrt(mean(psi^2)/J^2/n), J = S_ww/n.
// mode 1 (reference lm(Y_resid ~ 0 + W_resid), ate_functions.R:363-366):
//   se = sqrt(RSS/(n-1)/S_ww).
__global__ void dml_finalize_kernel(const double* __restrict__ m, int mode, double* __restrict__ res) {
  double n = m[5];
  double theta = m[0] / m[1];
  double se;
  if (mode == 0) {
    double j = m[1] / n;
    double psi2 = (m[2] - 2.0 * theta * m[3] + theta * theta * m[4]) / n;
    se = sqrt(fmax(psi2, 0.0) / (j * j) / n);
  } else {
    double rss = m[6] - 2.0 * theta * m[0] + theta * theta * m[1];
    se = sqrt(fmax(rss, 0.0) / (n - 1.0) / m[1]);
  }
  res[0] = theta;
  res[1] = se;
}

ATE_API int ate_dml_moments(const void* yr, const void* wr, const void* valid, int64_t n,
                            void* partial, void* moments, void* stream) {
  DmlMoments f{(const double*)yr, (const double*)wr, (const double*)valid};
  return rowreduce<7>(f, n, (double*)partial, (double*)moments, (hipStream_t)stream);
}

ATE_API int ate_dml_finalize(const void* moments, int mode, void* res, void* stream) {
  ATE_LAUNCH(dml_finalize_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream,
                     (const double*)moments, mode, (double*)res);
  ATE_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ K20 bootstrap replicates
// Score terms per row: e1 (NaN allowed -> excluded), est2. Replicate b resamples
// n rows with replacement: draw j picks row rand_below(seed, P_BOOT, b0+b, j, n)
// (identical to rng.bootstrap_counts). Gather form: tau_b = sum_j e1[r_j]/#ok + sum_j est2[r_j]/n.
// One workgroup per replicate; for the streaming large-N form see boot_poisson.
__global__ __launch_bounds__(256) void boot_multinomial_kernel(
    const double* __restrict__ e1, const double* __restrict__ e2, int64_t n, uint64_t seed,
    int b0, double* __restrict__ taus) {
  __shared__ double smem[16 * 3];
  const int b = blockIdx.x;
  double v[3] = {0.0, 0.0, 0.0};
  for (int64_t j = threadIdx.x; j < n; j += blockDim.x) {
    uint32_t r = rand_below(seed, P_BOOT, (uint32_t)(b0 + b), (uint64_t)j, (uint32_t)n);
    double a = e1[r];
    if (a == a) { v[0] += a; v[1] += 1.0; }
    v[2] += e2[r];
  }
  block_sum<3>(v, smem);
  if (threadIdx.x == 0) taus[b] = v[0] / v[1] + v[2] / (double)n;
}

// Poisson(1) bootstrap, row-streaming (each row read once; counts generated on the
// fly; partial sums per (replicate, block) -> no B x N storage). Used for large N
// where a gather per draw would be HBM-latency bound. partial: [nb][B][3].
__device__ __forceinline__ int poisson1(float u) {
  // inverse CDF of Poisson(1)
  const float cdf[8] = {0.36787944f, 0.73575888f, 0.91969860f, 0.98101184f,
                        0.99634015f, 0.99940582f, 0.99991676f, 0.99998975f};
  int k = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) k += (u >= cdf[q]) ? 1 : 0;
  return k;
}

__global__ __launch_bounds__(256) void boot_poisson_kernel(
    const double* __restrict__ e1, const double* __restrict__ e2, int64_t n, uint64_t seed, int b0,
    int B, int64_t row_offset, double* __restrict__ partial) {
  // block = (row slice, tile of 64 replicates); lane <-> replicate, waves stride rows.
  // partial: [nb][ceil(B/64)*64][4] = {sum c*e1 (non-NaN), sum c (non-NaN), sum c*e2, sum c}
  __shared__ double red[4][64][4];
  const int nrep_pad = ((B + 63) / 64) * 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int b = blockIdx.y * 64 + lane;
  double s1 = 0.0, sok = 0.0, s2 = 0.0, sc = 0.0;
  if (b < B) {
    for (int64_t i = blockIdx.x * 4 + wid; i < n; i += (int64_t)gridDim.x * 4) {
      // counter index = global row id (bit 62 set: disjoint from multinomial draws)
      u32x4 r = rand4(seed, P_BOOT, (uint32_t)(b0 + b), (uint64_t)(row_offset + i) | (1ull << 62));
      int c = poisson1((float)(r.x >> 8) * (1.0f / 16777216.0f));
      if (c) {
        double a = e1[i];
        if (a == a) { s1 += c * a; sok += c; }
        s2 += c * e2[i];
        sc += c;
      }
    }
  }
  red[wid][lane][0] = s1; red[wid][lane][1] = sok; red[wid][lane][2] = s2; red[wid][lane][3] = sc;
  __syncthreads();
  if (wid == 0) {
    for (int w = 1; w < 4; ++w) {
      s1 += red[w][lane][0]; sok += red[w][lane][1]; s2 += red[w][lane][2]; sc += red[w][lane][3];
    }
    double* out = partial + ((int64_t)blockIdx.x * nrep_pad + blockIdx.y * 64 + lane) * 4;
    out[0] = s1; out[1] = sok; out[2] = s2; out[3] = sc;
  }
}

ATE_API int ate_boot_multinomial(const void* e1, const void* e2, int64_t n, uint64_t seed, int b0,
                                 int B, void* taus, void* stream) {
  if (n > 0xFFFFFFFFll) return -1;
  ATE_LAUNCH(boot_multinomial_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream,
                     (const double*)e1, (const double*)e2, n, seed, b0, (double*)taus);
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_boot_poisson(const void* e1, const void* e2, int64_t n, uint64_t seed, int b0,
                             int B, int64_t row_offset, int nb, void* partial, void* stream) {
  dim3 grid(nb, (B + 63) / 64);
  ATE_LAUNCH(boot_poisson_kernel, grid, dim3(256), 0, (hipStream_t)stream,
                     (const double*)e1, (const double*)e2, n, seed, b0, B, row_offset,
                     (double*)partial);
  ATE_CHECK_LAUNCH();
  return 0;
}
