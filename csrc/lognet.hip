// Binomial elastic net (glmnet ``lognet``) regularisation path + cross-validation loss.
//
// Reference semantics: reference/glmnet.py::lognet / cv_glmnet (family="binomial"),
// i.e. glmnet's outer Newton (IRLS) quadratic approximation per lambda with an
// unpenalised intercept coordinate, working weights q(1-q) clamped at PMIN, threshold
// scaled by the null deviance, covariance-mode coordinate descent, early path stop.
// Call site: ``prop_score_lasso`` (ate_functions.R:133-146, E7).
//
// Layout: ONE workgroup (4 waves) per problem (full fit or one CV fold fit).
//   * per IRLS step ONE pass over the training rows builds C = Z' diag(v) Z for
//     Z = [1, Xs, r/v]: the Gram, the intercept cross terms and the gradient (last
//     column: sum v z (r/v) = sum r z) in one register-blocked product. Rows are staged
//     in LDS (one row per thread, 16 loads in flight, standardisation fused); each
//     thread owns a 4x4 block of C for one row group, row groups are combined in a
//     fixed order. The deviance of the current fit falls out of the same pass, and is
//     the deviance of lambda_{m-1}'s converged fit at lambda_m's first step;
//   * wave 0 then runs the exact glmnet coordinate sweep over that Gram: every lane
//     evaluates its own coordinate's update speculatively; a ballot picks the next
//     coordinate that changes, readlane broadcasts its delta, and all lanes update the
//     gradient from the Gram column in LDS. Exactly the sequential order of cd_solve.
// p <= 96 (template PM = 32 or 96). Fold problems take the full problem's lambda
// sequence (ulam, count read from device memory: no host round trip).
//
// Concurrent mode (progress != nullptr): ONE launch of 1+K workgroups, problem 0 the full
// fit, problems 1..K the folds, all co-resident (workgroup 0 is dispatched first, so it is
// never waiting behind a spinning fold). The full fit knows its whole lambda sequence
// once lambda_max is known (m = 1): it stores it to lampub (lambda_0 extrapolated as at
// the end of the path) and releases progress[1]; every later lambda it commits to
// (past glmnet's early-stop check) releases progress[0] = m+1, and the path end releases
// progress[0] = FINAL | nlam. A fold waits for the sequence before lambda 0 and, after
// its own first pass at lambda m, for the full fit's decision on m: the fold path then
// ends exactly where the two-launch form (nlam read from the finished full fit) ends, with
// bit-identical outputs, while the two paths run side by side instead of back to back.
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

template <int PM, int NTK>
struct Cfg {
  static constexpr int Q = PM + 1;                        // Gram stride: 1, x_1..x_p
  static constexpr int QA = PM + 2;                       // + r/v column (gradient)
  static constexpr int NB = (QA + 3) / 4;                 // 4-wide column blocks
  static constexpr int QP = NB * 4;                       // LDS row stride (doubles)
  static constexpr int NPAIR = NB * (NB + 1) / 2;
  static constexpr int TPT = (NPAIR + NTK - 1) / NTK;     // block pairs per thread
  // staged rows per chunk: one per thread up to p = 24 (LDS: 512 x 28 doubles)
  static constexpr int RB = PM <= 24 ? NTK : PM <= 32 ? 256 : 64;
  static constexpr int NCH = (PM + 63) / 64;
};

template <typename T>
__device__ __forceinline__ double ld_x(const T* X, int64_t i) { return (double)X[i]; }

__device__ __forceinline__ double clampq(double eta) {
  double q = 1.0 / (1.0 + exp(-eta));
  return fmin(fmax(q, PMIN), 1.0 - PMIN);
}

template <typename T, int PM, int NTK>
__global__ __launch_bounds__(NTK) void lognet_path_kernel(
    const T* __restrict__ X, int64_t ld, const int* __restrict__ xcols, int p, int ycol,
    const int64_t* __restrict__ segs, int nseg, const uint8_t* __restrict__ masks,
    const double* __restrict__ vp_in, double alpha, double flmin, double thresh, int maxit,
    const double* __restrict__ ulam, const int* __restrict__ nlam_in, int L,
    double* __restrict__ a0_out, double* __restrict__ beta_out, double* __restrict__ lam_out,
    double* __restrict__ dev_out, int* __restrict__ nlam_out, int* __restrict__ npass_out,
    int* __restrict__ progress, double* __restrict__ lampub) {
  using C = Cfg<PM, NTK>;
  constexpr int Q = C::Q, QP = C::QP, RB = C::RB, TPT = C::TPT, NCH = C::NCH;
  __shared__ double sC[Q * Q];
  __shared__ double sg[Q];
  __shared__ __attribute__((aligned(16))) double sZ[RB * QP];   // staged rows / reduce scratch
  __shared__ double sV[RB];
  __shared__ double sxm[PM], sxs[PM], sxr[PM];   // sxr: 1 / SD (0: constant column)
  __shared__ double sb[Q];                    // sb[0] = intercept (standardised scale)
  __shared__ int sju[PM], sxc[PM];
  __shared__ int64_t sr0[MAXSEG];
  __shared__ int spre[MAXSEG + 1];
  __shared__ double red[16 * 2];
  __shared__ double sctl[4];
  __shared__ int sictl[4];

  const int prob = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint8_t* mk = masks + (int64_t)prob * nseg;
  ATE_DASSERT(p > 0 && p <= PM && nseg > 0 && nseg <= MAXSEG && ycol >= 0 && L > 0);

  if (tid == 0) {
    int acc = 0, k = 0;
    for (int s = 0; s < nseg; ++s)
      if (mk[s]) {
        ATE_DASSERT(segs[2 * s] >= 0 && segs[2 * s] <= segs[2 * s + 1] && segs[2 * s + 1] <= ld);
        sr0[k] = segs[2 * s];
        spre[k] = acc;
        acc += (int)(segs[2 * s + 1] - segs[2 * s]);
        ++k;
      }
    spre[k] = acc;
    sictl[0] = k;
  }
  for (int j = tid; j < p; j += NTK) sxc[j] = xcols[j];
  __syncthreads();
  const int nts = sictl[0];
  const int ntr = spre[nts];
  const double w = 1.0 / (double)ntr;
  auto vrow = [&](int v) -> int64_t {
    ATE_DASSERT(v >= 0 && v < ntr);
    int k = 0;
    while (k + 1 < nts && spre[k + 1] <= v) ++k;
    return sr0[k] + (v - spre[k]);
  };
  const T* Yc = X + (int64_t)ycol * ld;

  // ---- standardisation (population SD, weights 1/n) and the null model
  for (int j = wid; j < p; j += NTK / 64) {
    const T* xc = X + (int64_t)sxc[j] * ld;
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
      sxr[j] = xs > 0.0 ? 1.0 / xs : 0.0;
    }
  }
  {
    double acc[1] = {0.0};
    for (int v = tid; v < ntr; v += NTK) acc[0] += ld_x(Yc, vrow(v));
    ate::block_sum<1>(acc, red);
    if (tid == 0) sctl[1] = acc[0] * w;
  }
  for (int j = tid; j < Q; j += NTK) sb[j] = 0.0;
  __syncthreads();
  const double q0 = sctl[1];
  const double q0c = fmin(fmax(q0, PMIN), 1.0 - PMIN);
  const double dev0 = -2.0 * (q0 * log(q0c) + (1.0 - q0) * log(1.0 - q0c));
  if (tid == 0) sb[0] = log(q0 / (1.0 - q0));

  // ---- Gram task layout (runtime p): column blocks of 4 over [1, z_1..z_p, r/v]
  const int qa = p + 2, nb = (qa + 3) / 4, npair = nb * (nb + 1) / 2;
  const int ngrp = npair >= NTK ? 1 : NTK / npair;
  const int grp = ngrp == 1 ? 0 : tid / npair;
  int pa[TPT], pb[TPT];
#pragma unroll
  for (int q = 0; q < TPT; ++q) {
    const int t = ngrp == 1 ? tid + q * NTK : (q == 0 && grp < ngrp ? tid % npair : npair);
    pa[q] = pb[q] = -1;
    if (t < npair) {
      int a = 0, rem = t;
      while (rem >= nb - a) { rem -= nb - a; ++a; }
      pa[q] = a;
      pb[q] = a + rem;
    }
  }

  // ---- wave-0 coordinate state (lane l owns features l + 64c)
  double ga[NCH], aa[NCH], xva[NCH], vpa[NCH], cia[NCH];
  int jua[NCH], act[NCH];
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int j = lane + 64 * c;
    aa[c] = 0.0;
    act[c] = 0;
    vpa[c] = j < p ? vp_in[j] : 0.0;
    jua[c] = j < p ? sju[j] : 0;
    ga[c] = xva[c] = cia[c] = 0.0;
  }

  const bool conc = progress != nullptr;
  const bool have_ulam = conc ? prob > 0 : ulam != nullptr;
  const int nlam = have_ulam && !conc ? (nlam_in ? *nlam_in : L) : L;
  const double alf = have_ulam ? 1.0 : pow(flmin, 1.0 / (double)(nlam - 1));
  const double shr = thresh * dev0;
  double alm = 0.0, dev_prev = 0.0;
  int npass_tot = 0, nlam_eff = 0;
  bool timed_out = false;
  double* bo = beta_out + (int64_t)prob * L * p;

  auto publish = [&](int* dst, int v) {   // one thread: agent-scope release of *dst
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // fold side (thread 0): bounded poll of progress[idx] until ready(v); acquire. -1 = timeout
  auto await = [&](int idx, auto ready) -> int {
    int v = 0;
    for (long spin = 0;; ++spin) {
      v = __hip_atomic_load(progress + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ready(v)) break;
      if (spin > (1l << 26)) return -1;
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return v;
  };
  constexpr int FINAL = 1 << 30;
  if (conc && have_ulam) {                 // the full fit's lambda sequence
    if (tid == 0) sictl[2] = await(1, [](int v) { return v != 0; });
    __syncthreads();
    timed_out = sictl[2] < 0;
    ulam = lampub;
    __syncthreads();
  }

  // One pass over the training rows at the current coefficients:
  //   C = Z' diag(v) Z with Z = [1, z, r/v]  ->  Gram, intercept cross terms, gradient;
  //   deviance of the current fit (returned, valid in every thread).
  auto accumulate = [&]() -> double {
    double acc[TPT][16];
#pragma unroll
    for (int q = 0; q < TPT; ++q)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[q][e] = 0.0;
    double devl = 0.0;
    for (int base = 0; base < ntr; base += RB) {
      for (int t = tid; t < RB; t += NTK) {
        double* z = sZ + t * QP;
        if (base + t < ntr) {
          const int64_t row = vrow(base + t);
          double eta = sb[0];
          for (int jb = 0; jb < p; jb += 16) {
            double xr[16];
#pragma unroll
            for (int u = 0; u < 16; ++u)
              xr[u] = jb + u < p ? ld_x(X + (int64_t)sxc[jb + u] * ld, row) : 0.0;
#pragma unroll
            for (int u = 0; u < 16; ++u) {
              const int j = jb + u;
              if (j < p) {
                // multiply by the reciprocal SD: a division per element and pass cost
                // as much as the rest of the row's staging
                const double zv = (xr[u] - sxm[j]) * sxr[j];
                z[1 + j] = zv;
                eta += zv * sb[1 + j];
              }
            }
          }
          const double q = clampq(eta);
          const double vv = w * q * (1.0 - q);
          const double y = ld_x(Yc, row);
          z[0] = 1.0;
          z[p + 1] = (w * (y - q)) / vv;
          for (int j = p + 2; j < QP; ++j) z[j] = 0.0;
          sV[t] = vv;
          devl += y * log(q) + (1.0 - y) * log(1.0 - q);
        } else {
          for (int j = 0; j < QP; ++j) z[j] = 0.0;
          sV[t] = 0.0;
        }
      }
      __syncthreads();
      const int nr = min(RB, ntr - base);
      for (int r = grp; r < nr; r += ngrp) {
        const double v = sV[r];
        const double* zr = sZ + r * QP;
#pragma unroll
        for (int q = 0; q < TPT; ++q) {
          if (pa[q] >= 0) {
            const double4 za = *reinterpret_cast<const double4*>(zr + 4 * pa[q]);
            const double4 zb = *reinterpret_cast<const double4*>(zr + 4 * pb[q]);
            const double va[4] = {v * za.x, v * za.y, v * za.z, v * za.w};
            const double vb[4] = {zb.x, zb.y, zb.z, zb.w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
              for (int j = 0; j < 4; ++j) acc[q][i * 4 + j] += va[i] * vb[j];
          }
        }
      }
      __syncthreads();
    }
    // combine row groups (fixed order) and scatter into sC / sg
    auto emit = [&](int pair, int e, double val) {
      int A = 0, rem = pair;
      while (rem >= nb - A) { rem -= nb - A; ++A; }
      const int B = A + rem;
      const int a = 4 * A + (e >> 2), b = 4 * B + (e & 3);
      // a <= b only: inside a diagonal block (a,b) and (b,a) round differently
      if (a > b || b > p + 1) return;
      if (b <= p) {
        sC[a * Q + b] = val;
        sC[b * Q + a] = val;
      } else if (a <= p) {
        sg[a] = val;
      }
    };
    if (ngrp == 1) {
#pragma unroll
      for (int q = 0; q < TPT; ++q)
        if (pa[q] >= 0) {
          const int pair = tid + q * NTK;
#pragma unroll
          for (int e = 0; e < 16; ++e) emit(pair, e, acc[q][e]);
        }
    } else {
      if (grp < ngrp && pa[0] >= 0)
#pragma unroll
        for (int e = 0; e < 16; ++e) sZ[(grp * npair + tid % npair) * 16 + e] = acc[0][e];
      __syncthreads();
      for (int t = tid; t < npair * 16; t += NTK) {
        double sum = 0.0;
        for (int gq = 0; gq < ngrp; ++gq) sum += sZ[(gq * npair) * 16 + t];
        emit(t >> 4, t & 15, sum);
      }
    }
    double dv[1] = {devl};
    ate::block_sum<1>(dv, red);
    if (tid == 0) sctl[2] = -2.0 * w * dv[0];
    __syncthreads();
    return sctl[2];
  };

  bool stopped = false;
  for (int m = 0; m < nlam && !stopped && !timed_out; ++m) {
    const int kind = have_ulam ? 0 : (m == 0 ? 1 : (m == 1 ? 2 : 3));
    if (kind == 0) alm = ulam[m];
    else if (kind == 1) alm = BIG;
    else if (kind == 3) alm *= alf;
    for (int outer = 0; outer < 1000; ++outer) {
      const double dev_cur = accumulate();
      if (outer == 0 && m > 0) {
        // deviance at the converged fit of lambda_{m-1}; glmnet's early path stop
        const double dr = 1.0 - dev_cur / dev0;
        if (tid == 0) dev_out[(int64_t)prob * L + m - 1] = dr;
        if (!have_ulam && m - 1 >= MNLAM - 1 && (dr - dev_prev < FDEV * dr || dr > DEVMAX)) {
          stopped = true;
          break;
        }
        if (conc && !have_ulam && tid == 0) publish(progress, m + 1);
        if (conc && have_ulam) {
          // does the full fit go on to lambda m? (this pass's deviance is already the
          // final one of lambda m-1 if not)
          if (tid == 0)
            sictl[2] = await(0, [m](int v) { return (v & (FINAL - 1)) > m || (v & FINAL); });
          __syncthreads();
          const int v = sictl[2];
          __syncthreads();
          if (v < 0) timed_out = true;
          if (v < 0 || (v & (FINAL - 1)) <= m) {
            stopped = true;
            break;
          }
        }
        dev_prev = dr;
      }
      int stop = 0;
      if (wid == 0) {
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
          if (conc && lane == 0) {
            // the whole sequence, rounded exactly as the path computes it
            double x = alm;
            lampub[1] = x;
            double l2 = x;
            for (int mm = 2; mm < L; ++mm) {
              x *= alf;
              lampub[mm] = x;
              if (mm == 2) l2 = x;
            }
            lampub[0] = L >= 3 ? exp(2.0 * log(alm) - log(l2)) : BIG;
            publish(progress + 1, 1);
          }
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
          while (npass < mleft) {
            ++npass;
            if (one_pass(false) < shr) break;
          }
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
    if (stopped) break;
    if (tid == 0) {
      a0_out[(int64_t)prob * L + m] = sb[0];
      lam_out[(int64_t)prob * L + m] = alm;
    }
    for (int j = tid; j < p; j += NTK) bo[(int64_t)m * p + j] = sb[1 + j];
    nlam_eff = m + 1;
    __syncthreads();
  }
  if (conc && !have_ulam && tid == 0) publish(progress, FINAL | nlam_eff);
  if (!stopped && !timed_out) {
    const double dev_cur = accumulate();
    if (tid == 0) dev_out[(int64_t)prob * L + nlam_eff - 1] = 1.0 - dev_cur / dev0;
  }
  __syncthreads();
  // ---- back to the original scale; lambda_0 extrapolated as glmnet does
  for (int m = 0; m < nlam_eff; ++m) {
    double part[1] = {0.0};
    for (int j = tid; j < p; j += NTK) {
      double bj = sju[j] ? bo[(int64_t)m * p + j] / sxs[j] : 0.0;
      bo[(int64_t)m * p + j] = bj;
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
    npass_out[prob] = timed_out ? -1 : npass_tot;
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
  ATE_DASSERT(s >= 0 && r0 >= 0 && r0 <= r1 && r1 <= ld && m < L);
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
                int* npass, int* progress, double* lampub, hipStream_t st) {
  if (p <= 24)
    ATE_LAUNCH((lognet_path_kernel<T, 24, 512>), dim3(nprob), dim3(512), 0, st, (const T*)X,
                       ld, xcols, p, ycol, segs, nseg, masks, vp, alpha, flmin, thresh, maxit, ulam,
                       nlam_in, L, a0, beta, lam, dev, nlam_out, npass, progress, lampub);
  else if (p <= 32)
    ATE_LAUNCH((lognet_path_kernel<T, 32, NT>), dim3(nprob), dim3(NT), 0, st, (const T*)X, ld,
                       xcols, p, ycol, segs, nseg, masks, vp, alpha, flmin, thresh, maxit, ulam,
                       nlam_in, L, a0, beta, lam, dev, nlam_out, npass, progress, lampub);
  else
    ATE_LAUNCH((lognet_path_kernel<T, 96, NT>), dim3(nprob), dim3(NT), 0, st, (const T*)X, ld,
                       xcols, p, ycol, segs, nseg, masks, vp, alpha, flmin, thresh, maxit, ulam,
                       nlam_in, L, a0, beta, lam, dev, nlam_out, npass, progress, lampub);
  return 0;
}

}  // namespace

ATE_KERNEL_SHAPE("lognet_path_kernel<double, 24>", 512, 0, lognet_path_kernel<double, 24, 512>)
ATE_KERNEL_SHAPE("lognet_path_kernel<float, 24>", 512, 0, lognet_path_kernel<float, 24, 512>)
ATE_KERNEL_SHAPE("lognet_path_kernel<double, 32>", NT, 0, lognet_path_kernel<double, 32, NT>)
ATE_KERNEL_SHAPE("lognet_path_kernel<double, 96>", NT, 0, lognet_path_kernel<double, 96, NT>)

// dt: 1 = fp32 panel, 2 = fp64 panel. segs: int64 [nseg][2] real-row ranges.
ATE_API int ate_lognet_path(int dt, const void* X, int64_t ld, const void* xcols, int p, int ycol,
                            const void* segs, int nseg, const void* masks, int nprob,
                            const void* vp, double alpha, double flmin, double thresh, int maxit,
                            const void* ulam, const void* nlam_in, int L, void* a0, void* beta,
                            void* lam, void* dev, void* nlam_out, void* npass, void* progress,
                            void* lampub, void* stream) {
  if (p < 1 || p > 96 || nseg > MAXSEG || (dt != 1 && dt != 2)) return -1;
  // concurrent mode: problem 0 = full fit (own lambda sequence), 1.. = folds, co-resident
  if (progress && (ulam || nprob < 2 || nprob > 256 || L < 3)) return -1;
  hipStream_t st = (hipStream_t)stream;
  auto f = dt == 2 ? launch_path<double> : launch_path<float>;
  f(X, ld, (const int*)xcols, p, ycol, (const int64_t*)segs, nseg, (const uint8_t*)masks, nprob,
    (const double*)vp, alpha, flmin, thresh, maxit, (const double*)ulam, (const int*)nlam_in, L,
    (double*)a0, (double*)beta, (double*)lam, (double*)dev, (int*)nlam_out, (int*)npass,
    (int*)progress, (double*)lampub, st);
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
    ATE_LAUNCH(lognet_cvloss_kernel<double>, grid, dim3(NT), 0, st, (const double*)X, ld,
                       (const int*)xcols, p, ycol, (const int64_t*)segs, (const int*)hold,
                       (const double*)a0, (const double*)beta, (const int*)nlam, L,
                       (double*)cvraw);
  else
    ATE_LAUNCH(lognet_cvloss_kernel<float>, grid, dim3(NT), 0, st, (const float*)X, ld,
                       (const int*)xcols, p, ycol, (const int64_t*)segs, (const int*)hold,
                       (const double*)a0, (const double*)beta, (const int*)nlam, L,
                       (double*)cvraw);
  ATE_CHECK_LAUNCH();
  return 0;
}
