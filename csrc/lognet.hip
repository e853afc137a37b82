// Binomial elastic net (glmnet ``lognet``) regularisation path + cross-validation loss.
//
// Reference semantics: reference/glmnet.py::lognet / cv_glmnet (family="binomial"),
// i.e. glmnet's outer Newton (IRLS) quadratic approximation per lambda with an
// unpenalised intercept coordinate, working weights q(1-q) clamped at PMIN, threshold
// scaled by the null deviance, covariance-mode coordinate descent, early path stop.
// Call site: ``prop_score_lasso`` (ate_functions.R:133-146, E7).
//
// Layout: ONE workgroup (4 waves) per problem (full fit or one CV fold fit).
//   * per IRLS step, the working-weighted Gram of Z = [1, Xs] is accumulated from row
//     chunks staged in LDS (one row per thread, standardisation fused into the load);
//     each thread owns TPT (a, b) tasks (C_ab = sum v Z_a Z_b, or g_a = sum r Z_a) and
//     keeps their partial sums in registers for the whole pass;
//   * wave 0 then runs the exact glmnet coordinate sweep over that Gram: every lane
//     evaluates its own coordinate's update speculatively; a ballot picks the next
//     coordinate that changes, readlane broadcasts its delta, and all lanes update the
//     gradient from the Gram column in LDS. Exactly the sequential order of cd_solve.
// p <= 96 (template PM = 32 or 96). Fold problems take the full problem's lambda
// sequence (ulam, count read from device memory: no host round trip).
#include "common.hpp"

namespace {

constexpr int NT = 256;
constexpr double PMIN = 1e-5;
constexpr double BIG = 9.9e35;
constexpr double FDEV = 1e-5;
constexpr double DEVMAX = 0.999;
constexpr int MNLAM = 5;
constexpr int MAXSEG = 64;

__device__ __forceinline__ double rl_d(double v, int i) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), i);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), i);
  return __hiloint2double(hi, lo);
}

template <int PM>
struct Cfg {
  static constexpr int Q = PM + 1;                        // Z columns: 1, x_1..x_p
  static constexpr int RB = PM <= 32 ? 128 : 32;          // staged rows per chunk
  static constexpr int NTASK = Q * (Q + 1) / 2 + Q;
  static constexpr int TPT = (NTASK + NT - 1) / NT;
  static constexpr int NCH = (PM + 63) / 64;
};

template <typename T>
__device__ __forceinline__ double ld_x(const T* X, int64_t i) { return (double)X[i]; }

__device__ __forceinline__ double clampq(double eta) {
  double q = 1.0 / (1.0 + exp(-eta));
  return fmin(fmax(q, PMIN), 1.0 - PMIN);
}

template <typename T, int PM>
__global__ __launch_bounds__(NT) void lognet_path_kernel(
    const T* __restrict__ X, int64_t ld, const int* __restrict__ xcols, int p, int ycol,
    const int64_t* __restrict__ segs, int nseg, const uint8_t* __restrict__ masks,
    const double* __restrict__ vp_in, double alpha, double flmin, double thresh, int maxit,
    const double* __restrict__ ulam, const int* __restrict__ nlam_in, int L,
    double* __restrict__ a0_out, double* __restrict__ beta_out, double* __restrict__ lam_out,
    double* __restrict__ dev_out, int* __restrict__ nlam_out, int* __restrict__ npass_out) {
  using C = Cfg<PM>;
  constexpr int Q = C::Q, RB = C::RB, TPT = C::TPT, NCH = C::NCH;
  __shared__ double sC[Q * Q];
  __shared__ double sg[Q];
  __shared__ double sZ[RB * Q];
  __shared__ double sVZ[RB * Q];
  __shared__ double sR[RB];
  __shared__ double sxm[PM], sxs[PM];
  __shared__ double sb[Q];                    // sb[0] = intercept (standardised scale)
  __shared__ int sju[PM];
  __shared__ int64_t sr0[MAXSEG];
  __shared__ int spre[MAXSEG + 1];
  __shared__ double red[16 * 2];
  __shared__ double sctl[4];                  // broadcast doubles (alm, ...)
  __shared__ int sictl[4];                    // broadcast ints (continue flags)

  const int prob = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint8_t* mk = masks + (int64_t)prob * nseg;

  if (tid == 0) {
    int acc = 0, k = 0;
    for (int s = 0; s < nseg; ++s)
      if (mk[s]) {
        sr0[k] = segs[2 * s];
        spre[k] = acc;
        acc += (int)(segs[2 * s + 1] - segs[2 * s]);
        ++k;
      }
    spre[k] = acc;
    sictl[0] = k;
  }
  __syncthreads();
  const int nts = sictl[0];
  const int ntr = spre[nts];
  const double w = 1.0 / (double)ntr;
  auto vrow = [&](int v) -> int64_t {
    int k = 0;
    while (spre[k + 1] <= v) ++k;
    return sr0[k] + (v - spre[k]);
  };
  const T* Yc = X + (int64_t)ycol * ld;

  // ---- standardisation (population SD with weights 1/n) and the null model
  for (int j = wid; j < p; j += NT / 64) {
    const T* xc = X + (int64_t)xcols[j] * ld;
    double s1 = 0.0, s2 = 0.0;
    for (int v = lane; v < ntr; v += 64) {
      double x = ld_x(xc, vrow(v));
      s1 += x;
      s2 += x * x;
    }
    s1 = ate::wave_sum(s1);
    s2 = ate::wave_sum(s2);
    if (lane == 0) {
      double xm = s1 * w;
      double xs = sqrt(fmax(s2 * w - xm * xm, 0.0));
      sxm[j] = xm;
      sju[j] = xs > 0.0;
      sxs[j] = xs > 0.0 ? xs : 1.0;
    }
  }
  {
    double acc[1] = {0.0};
    for (int v = tid; v < ntr; v += NT) acc[0] += ld_x(Yc, vrow(v));
    ate::block_sum<1>(acc, red);
    if (tid == 0) sctl[1] = acc[0] * w;
  }
  for (int j = tid; j < Q; j += NT) sb[j] = 0.0;
  __syncthreads();
  const double q0 = sctl[1];
  const double q0c = fmin(fmax(q0, PMIN), 1.0 - PMIN);
  const double dev0 = -2.0 * (q0 * log(q0c) + (1.0 - q0) * log(1.0 - q0c));
  if (tid == 0) sb[0] = log(q0 / (1.0 - q0));

  // ---- task decode: task t < Q(Q+1)/2 -> (a <= b) Gram entry; else gradient of column a
  int ta[TPT], tb[TPT];
#pragma unroll
  for (int q = 0; q < TPT; ++q) {
    int t = tid + q * NT;
    ta[q] = -1;
    tb[q] = -1;
    const int ng = Q * (Q + 1) / 2;
    if (t < ng) {
      int a = 0, rem = t;
      while (rem >= Q - a) { rem -= Q - a; ++a; }
      ta[q] = a;
      tb[q] = a + rem;
    } else if (t < ng + Q) {
      ta[q] = t - ng;
      tb[q] = -2;
    }
  }
  // ---- wave-0 coordinate state (lane l owns features l + 64c)
  double ga[NCH], aa[NCH], xva[NCH], vpa[NCH], cia[NCH];
  int jua[NCH], act[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int j = lane + 64 * c;
    aa[c] = 0.0;
    act[c] = 0;
    vpa[c] = j < p ? vp_in[j] : 0.0;
    jua[c] = 0;
    ga[c] = xva[c] = cia[c] = 0.0;
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int j = lane + 64 * c;
    jua[c] = j < p ? sju[j] : 0;
  }

  const bool have_ulam = ulam != nullptr;
  const int nlam = have_ulam ? (nlam_in ? *nlam_in : L) : L;
  const double alf = have_ulam ? 1.0 : pow(flmin, 1.0 / (double)(nlam - 1));
  const double shr = thresh * dev0;
  double alm = 0.0, dev_prev = 0.0;
  int npass_tot = 0, nlam_eff = 0;
  const int ldb = p;
  double* bo = beta_out + (int64_t)prob * L * ldb;

  // accumulate C = Z' diag(v) Z, g = Z' r at the current coefficients
  auto accumulate = [&]() {
    double acc[TPT];
#pragma unroll
    for (int q = 0; q < TPT; ++q) acc[q] = 0.0;
    for (int base = 0; base < ntr; base += RB) {
      if (tid < RB) {
        double* z = sZ + tid * Q;
        double* vz = sVZ + tid * Q;
        if (base + tid < ntr) {
          const int64_t row = vrow(base + tid);
          double eta = sb[0];
          z[0] = 1.0;
          for (int j = 0; j < p; ++j) {
            double xv = sju[j] ? (ld_x(X + (int64_t)xcols[j] * ld, row) - sxm[j]) / sxs[j] : 0.0;
            z[1 + j] = xv;
            eta += xv * sb[1 + j];
          }
          const double q = clampq(eta);
          const double vv = w * q * (1.0 - q);
          sR[tid] = w * (ld_x(Yc, row) - q);
          for (int j = 0; j <= p; ++j) vz[j] = vv * z[j];
        } else {
          for (int j = 0; j <= p; ++j) z[j] = vz[j] = 0.0;
          sR[tid] = 0.0;
        }
      }
      __syncthreads();
      for (int r = 0; r < RB; ++r) {
#pragma unroll
        for (int q = 0; q < TPT; ++q) {
          if (ta[q] >= 0 && ta[q] <= p) {
            if (tb[q] >= 0) {
              if (tb[q] <= p) acc[q] += sVZ[r * Q + ta[q]] * sZ[r * Q + tb[q]];
            } else {
              acc[q] += sR[r] * sZ[r * Q + ta[q]];
            }
          }
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < TPT; ++q) {
      if (ta[q] >= 0 && ta[q] <= p) {
        if (tb[q] >= 0) {
          if (tb[q] <= p) {
            sC[ta[q] * Q + tb[q]] = acc[q];
            sC[tb[q] * Q + ta[q]] = acc[q];
          }
        } else {
          sg[ta[q]] = acc[q];
        }
      }
    }
    __syncthreads();
  };

  auto deviance = [&]() -> double {
    double acc[1] = {0.0};
    for (int v = tid; v < ntr; v += NT) {
      const int64_t row = vrow(v);
      double eta = sb[0];
      for (int j = 0; j < p; ++j)
        if (sb[1 + j] != 0.0)
          eta += (ld_x(X + (int64_t)xcols[j] * ld, row) - sxm[j]) / sxs[j] * sb[1 + j];
      const double q = clampq(eta);
      const double y = ld_x(Yc, row);
      acc[0] += y * log(q) + (1.0 - y) * log(1.0 - q);
    }
    ate::block_sum<1>(acc, red);
    return -2.0 * w * acc[0];   // valid in thread 0
  };

  for (int m = 0; m < nlam; ++m) {
    int kind = have_ulam ? 0 : (m == 0 ? 1 : (m == 1 ? 2 : 3));
    if (kind == 0) alm = ulam[m];
    else if (kind == 1) alm = BIG;
    else if (kind == 3) alm *= alf;
    for (int outer = 0; outer < 1000; ++outer) {
      accumulate();
      int stop = 0;
      if (wid == 0) {
        // load the working gradient / Gram diagonal for this IRLS step
        double gint = sg[0];
        const double xmz = sC[0];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int j = lane + 64 * c;
          ga[c] = j < p ? sg[1 + j] : 0.0;
          xva[c] = j < p ? sC[(1 + j) * Q + 1 + j] : 0.0;
          cia[c] = j < p ? sC[1 + j] : 0.0;
        }
        if (kind == 2 && outer == 0) {
          double mx = 0.0;
#pragma unroll
          for (int c = 0; c < NCH; ++c)
            if (jua[c] && vpa[c] > 0.0) mx = fmax(mx, fabs(ga[c]) / vpa[c]);
          mx = ate::wave_max(mx);
          alm = alf * mx / fmax(alpha, 1e-3);
        }
        const double ab = alm * alpha, dem = alm * (1.0 - alpha);
        double bs[NCH];
#pragma unroll
        for (int c = 0; c < NCH; ++c) bs[c] = aa[c];
        const double b0s = sb[0];
        double b0d = 0.0;
        const int mleft = maxit - npass_tot;
        int npass = 0;
        auto one_pass = [&](bool full) -> double {
          double dlx = 0.0;
#pragma unroll
          for (int c = 0; c < NCH; ++c) {
            int pos = 0;
            while (true) {
              const double u = ga[c] + aa[c] * xva[c];
              const double v = fabs(u) - vpa[c] * ab;
              const double an = v > 0.0 ? copysign(v, u) / (xva[c] + vpa[c] * dem) : 0.0;
              const bool inl = full ? jua[c] : act[c];
              const bool cand = inl && lane >= pos && an != aa[c];
              const uint64_t bal = __ballot(cand);
              if (!bal) break;
              const int i = __ffsll((unsigned long long)bal) - 1;
              const double d = rl_d(an - aa[c], i);
              const double xvj = rl_d(xva[c], i);
              if (lane == i) { aa[c] = an; act[c] = 1; }
              dlx = fmax(dlx, xvj * d * d);
              const int jg = i + 64 * c;
#pragma unroll
              for (int cc = 0; cc < NCH; ++cc) {
                const int l = lane + 64 * cc;
                if (l < p) ga[cc] -= sC[(1 + l) * Q + 1 + jg] * d;
              }
              gint -= sC[1 + jg] * d;
              pos = i + 1;
            }
          }
          const double d = gint / xmz;
          if (d != 0.0) {
            b0d += d;
#pragma unroll
            for (int cc = 0; cc < NCH; ++cc) ga[cc] -= cia[cc] * d;
            gint -= xmz * d;
            dlx = fmax(dlx, xmz * d * d);
          }
          return dlx;
        };
        while (npass < mleft) {
          ++npass;
          if (one_pass(true) < shr) break;
          bool conv = false;
          while (npass < mleft) {
            ++npass;
            if (one_pass(false) < shr) { conv = true; break; }
          }
          (void)conv;
        }
        npass_tot += npass;
        const double b0n = b0s + b0d;
        double dl = xmz * (b0n - b0s) * (b0n - b0s);
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int j = lane + 64 * c;
          if (j < p) {
            dl = fmax(dl, xva[c] * (aa[c] - bs[c]) * (aa[c] - bs[c]));
            sb[1 + j] = aa[c];
          }
        }
        dl = ate::wave_max(dl);
        if (lane == 0) {
          sb[0] = b0n;
          sctl[0] = alm;
          sictl[1] = dl < shr;
        }
      }
      __syncthreads();
      alm = sctl[0];
      stop = sictl[1];
      __syncthreads();
      if (stop) break;
    }
    const double dev = deviance();
    if (tid == 0) {
      const double dr = 1.0 - dev / dev0;
      a0_out[(int64_t)prob * L + m] = sb[0];
      lam_out[(int64_t)prob * L + m] = alm;
      dev_out[(int64_t)prob * L + m] = dr;
      int brk = 0;
      if (!have_ulam && m >= MNLAM - 1 && m > 0)
        if (dr - dev_prev < FDEV * dr || dr > DEVMAX) brk = 1;
      dev_prev = dr;
      sictl[2] = brk;
    }
    for (int j = tid; j < p; j += NT) bo[(int64_t)m * ldb + j] = sb[1 + j];
    __syncthreads();
    nlam_eff = m + 1;
    if (sictl[2]) break;
    __syncthreads();
  }
  __syncthreads();
  // ---- back to the original scale; lambda_0 extrapolated as glmnet does
  for (int m = 0; m < nlam_eff; ++m) {
    double part[1] = {0.0};
    for (int j = tid; j < p; j += NT) {
      double bj = sju[j] ? bo[(int64_t)m * ldb + j] / sxs[j] : 0.0;
      bo[(int64_t)m * ldb + j] = bj;
      part[0] += bj * sxm[j];
    }
    ate::block_sum<1>(part, red);
    if (tid == 0) a0_out[(int64_t)prob * L + m] -= part[0];
  }
  if (tid == 0) {
    double* lm = lam_out + (int64_t)prob * L;
    if (!have_ulam && nlam_eff >= 3) lm[0] = exp(2.0 * log(lm[1]) - log(lm[2]));
    for (int m = nlam_eff; m < L; ++m) lm[m] = __builtin_nan("");
    nlam_out[prob] = nlam_eff;
    npass_out[prob] = npass_tot;
  }
}

// held-out binomial deviance: cvraw[k][m] = mean over rows of segment hold[k]
template <typename T>
__global__ __launch_bounds__(NT) void lognet_cvloss_kernel(
    const T* __restrict__ X, int64_t ld, const int* __restrict__ xcols, int p, int ycol,
    const int64_t* __restrict__ segs, const int* __restrict__ hold, const double* __restrict__ a0,
    const double* __restrict__ beta, const int* __restrict__ nlam, int L,
    double* __restrict__ cvraw) {
  __shared__ double red[16];
  const int k = blockIdx.x, m = blockIdx.y;
  if (m >= nlam[k]) {
    if (threadIdx.x == 0) cvraw[(int64_t)k * L + m] = __builtin_nan("");
    return;
  }
  const int s = hold[k];
  const int64_t r0 = segs[2 * s], r1 = segs[2 * s + 1];
  const double* b = beta + ((int64_t)k * L + m) * p;
  const double b0 = a0[(int64_t)k * L + m];
  double acc[1] = {0.0};
  for (int64_t r = r0 + threadIdx.x; r < r1; r += NT) {
    double eta = b0;
    for (int j = 0; j < p; ++j) eta += (double)X[(int64_t)xcols[j] * ld + r] * b[j];
    const double q = clampq(eta);
    const double y = (double)X[(int64_t)ycol * ld + r];
    acc[0] += y * log(q) + (1.0 - y) * log(1.0 - q);
  }
  ate::block_sum<1>(acc, red);
  if (threadIdx.x == 0) cvraw[(int64_t)k * L + m] = -2.0 * acc[0] / (double)(r1 - r0);
}

template <typename T>
int launch_path(const void* X, int64_t ld, const int* xcols, int p, int ycol, const int64_t* segs,
                int nseg, const uint8_t* masks, int nprob, const double* vp, double alpha,
                double flmin, double thresh, int maxit, const double* ulam, const int* nlam_in,
                int L, double* a0, double* beta, double* lam, double* dev, int* nlam_out,
                int* npass, hipStream_t st) {
  if (p <= 32)
    hipLaunchKernelGGL((lognet_path_kernel<T, 32>), dim3(nprob), dim3(NT), 0, st, (const T*)X, ld,
                       xcols, p, ycol, segs, nseg, masks, vp, alpha, flmin, thresh, maxit, ulam,
                       nlam_in, L, a0, beta, lam, dev, nlam_out, npass);
  else
    hipLaunchKernelGGL((lognet_path_kernel<T, 96>), dim3(nprob), dim3(NT), 0, st, (const T*)X, ld,
                       xcols, p, ycol, segs, nseg, masks, vp, alpha, flmin, thresh, maxit, ulam,
                       nlam_in, L, a0, beta, lam, dev, nlam_out, npass);
  return 0;
}

}  // namespace

// dt: 1 = fp32 panel, 2 = fp64 panel. segs: int64 [nseg][2] real-row ranges.
ATE_API int ate_lognet_path(int dt, const void* X, int64_t ld, const void* xcols, int p, int ycol,
                            const void* segs, int nseg, const void* masks, int nprob,
                            const void* vp, double alpha, double flmin, double thresh, int maxit,
                            const void* ulam, const void* nlam_in, int L, void* a0, void* beta,
                            void* lam, void* dev, void* nlam_out, void* npass, void* stream) {
  if (p < 1 || p > 96 || nseg > MAXSEG || (dt != 1 && dt != 2)) return -1;
  hipStream_t st = (hipStream_t)stream;
  auto f = dt == 2 ? launch_path<double> : launch_path<float>;
  f(X, ld, (const int*)xcols, p, ycol, (const int64_t*)segs, nseg, (const uint8_t*)masks, nprob,
    (const double*)vp, alpha, flmin, thresh, maxit, (const double*)ulam, (const int*)nlam_in, L,
    (double*)a0, (double*)beta, (double*)lam, (double*)dev, (int*)nlam_out, (int*)npass, st);
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_lognet_cvloss(int dt, const void* X, int64_t ld, const void* xcols, int p,
                              int ycol, const void* segs, const void* hold, int nprob,
                              const void* a0, const void* beta, const void* nlam, int L,
                              void* cvraw, void* stream) {
  if (dt != 1 && dt != 2) return -1;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(nprob, L);
  if (dt == 2)
    hipLaunchKernelGGL(lognet_cvloss_kernel<double>, grid, dim3(NT), 0, st, (const double*)X, ld,
                       (const int*)xcols, p, ycol, (const int64_t*)segs, (const int*)hold,
                       (const double*)a0, (const double*)beta, (const int*)nlam, L,
                       (double*)cvraw);
  else
    hipLaunchKernelGGL(lognet_cvloss_kernel<float>, grid, dim3(NT), 0, st, (const float*)X, ld,
                       (const int*)xcols, p, ycol, (const int64_t*)segs, (const int*)hold,
                       (const double*)a0, (const double*)beta, (const int*)nlam, L,
                       (double*)cvraw);
  ATE_CHECK_LAUNCH();
  return 0;
}
