// Forest engine specification shared by the host C++ reference (csrc/cpu/forest_cpu.cpp,
// compiled with g++) and the gfx950 kernels (csrc/forest.hip). Everything that decides
// the SHAPE of a tree lives here, so both implementations grow identical trees:
//
//  * rows are pre-binned to uint8 (<= 256 quantile bins per feature, column-major);
//  * every random choice is Philox(seed, purpose, tree, index) (parallel/rng.py);
//  * every split statistic is an exact integer: class/row counts, and responses in
//    2^-32 fixed point (int64 sums) -- no order-dependent float accumulation, so LDS
//    atomics on the GPU and a sequential loop on the CPU give the same bits;
//  * criteria are evaluated in fp64 with explicitly rounded operations (no FMA
//    contraction) and ties are broken by (feature slot, bin) order.
//
// Tree semantics (reference: randomForest classRF for ate_functions.R:169-174,340-349;
// grf regression/causal forests for ate_replication.Rmd:250-265):
//  kind 0 CLASSIFICATION  Gini: maximise (L0^2+L1^2)/nL + (R0^2+R1^2)/nR over bootstrap
//                          counts; leaf = majority vote (Philox coin on ties).
//  kind 1 REGRESSION      maximise SL^2/nL + SR^2/nR (variance reduction); leaf = mean.
//  kind 2 CAUSAL          grf gradient tree: per node W~, Y~ means, tau_P, pseudo-outcome
//                          rho_i = (W~i - Wbar)((Y~i - Ybar) - tau_P (W~i - Wbar)) / Var(W~),
//                          then a regression split on rho. Split balance is grf's
//                          stabilize.splits = TRUE rule (its instrumental splitting rule
//                          with the treatment as instrument): each child must hold at least
//                          minc = max(ceil(alpha * n_node), 1) rows with W~ BELOW the node's
//                          mean W~ and minc rows with W~ >= that mean ("treated" / "control"
//                          sides; alpha = 0.05 -> tens of rows per side in a 1,000-row node).
//  Sampling 0 (randomForest): bootstrap, n draws with replacement -> integer weights.
//  Sampling 1 (grf): trees come in little bags of `group` trees sharing a half-sample
//    (floor(n*sample_fraction*group) rows without replacement); with honesty each tree
//    splits its sample in two random halves: J1 grows the tree, J2 fills the leaves.
//  A node is split only if it has more than `min_node` (weighted) rows, is not pure
//  (classification), and the best admissible split improves the criterion; children
//  must hold >= max(ceil(alpha * n_node), 1) rows (alpha = 0 -> 1).
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define ATE_HD __host__ __device__ inline
#else
#define ATE_HD inline
#endif

namespace atef {

constexpr uint32_t P_RF_BOOT = 3, P_RF_MTRY = 4, P_SUBSAMPLE = 6;
constexpr int NBINS = 256;
constexpr double FIX_SCALE = 4294967296.0;   // 2^32
constexpr int MAX_DEPTH = 64;

struct ForestParams {
  int kind;           // 0 classification, 1 regression, 2 causal
  int sampling;       // 0 bootstrap, 1 grf half-sampling
  int ntree;
  int mtry;           // features tried per node (grf: Poisson(mtry) draw, capped)
  int min_node;       // split only nodes with weighted size > min_node
  int honesty;        // grf: split sample into J1 (grow) / J2 (estimate)
  int group;          // grf little-bag size (ci.group.size)
  int mtry_poisson;   // grf draws the number of candidate variables ~ Poisson(mtry)
  double alpha;       // min child fraction (grf alpha); 0 -> 1 row
  double sample_fraction;
  double pois0;       // exp(-mtry), computed once on the host (identical on both sides)
  uint64_t seed;
  int p;              // features
  int n;              // rows
  int t0;             // global index of this forest's first tree (tree-parallel shards):
                      // every RNG stream / little-bag group is keyed by t0 + t
};

struct u4 { uint32_t x, y, z, w; };

ATE_HD u4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}
ATE_HD uint32_t rand_below(uint64_t seed, uint32_t purpose, uint32_t stream, uint64_t index,
                           uint32_t n) {
  u4 r = philox((uint32_t)index, (uint32_t)(index >> 32), purpose, stream, (uint32_t)seed,
                (uint32_t)(seed >> 32));
  return (uint32_t)(((uint64_t)r.x * (uint64_t)n) >> 32);
}
ATE_HD uint32_t rand_u32(uint64_t seed, uint32_t purpose, uint32_t stream, uint64_t index) {
  return philox((uint32_t)index, (uint32_t)(index >> 32), purpose, stream, (uint32_t)seed,
                (uint32_t)(seed >> 32)).x;
}

// fixed point (2^-32) for responses; round half away from zero
ATE_HD int64_t to_fix(double v) {
  double s = v * FIX_SCALE;
  return (int64_t)(s >= 0 ? s + 0.5 : s - 0.5);
}
ATE_HD double from_fix(int64_t v) { return (double)v / FIX_SCALE; }

// Prediction accumulators (state [10][n2] int64, csrc/forest.hip ate_forest_predict and the
// host twin): every per-tree term (a leaf mean, a leaf moment, a little-bag score) is
// rounded to 2^-32 fixed point ONCE, with the same IEEE operations on both sides, and the
// terms are summed as int64 -- exact and order-free, so tree-parallel ranks all-reduce
// their partial sums to the single-device bits.
ATE_HD int64_t mean_fix(int64_t s, int64_t c) { return to_fix(from_fix(s) / (double)c); }

// Node-level random stream ids: mtry draw k uses index node*4096 + k (p < 4094), the
// Poisson draw 4094 and the leaf-vote coin 4095.
ATE_HD uint64_t node_index(int node, int k) { return (uint64_t)node * 4096u + (uint64_t)k; }

// number of candidate features for a node (grf: Poisson(mtry) capped to [1, p])
ATE_HD int draw_num_features(const ForestParams& fp, int tree, int node) {
  if (!fp.mtry_poisson) return fp.mtry < fp.p ? fp.mtry : fp.p;
  // inverse-CDF Poisson with one uniform (deterministic)
  uint32_t u32 = rand_u32(fp.seed, P_RF_MTRY, (uint32_t)tree, node_index(node, 4094));
  double u = (double)(u32 >> 8) * (1.0 / 16777216.0);
  double lam = (double)fp.mtry;
  double pmf = fp.pois0, cdf = pmf;
  int k = 0;
  while (u > cdf && k < 4 * fp.mtry + 64) {
    ++k;
    pmf = pmf * lam / (double)k;
    cdf += pmf;
  }
  if (k < 1) k = 1;
  if (k > fp.p) k = fp.p;
  return k;
}

// Gini criterion of a split (weighted class counts), explicitly rounded fp64
// Algorithm S (Knuth): decide, in order, whether element i of a population of `pop`
// joins a sample of size k given `taken` already selected; exact integer arithmetic.
ATE_HD bool select_next(uint64_t seed, uint32_t stream, uint64_t i, int64_t pop_left,
                        int64_t need) {
  uint32_t u24 = rand_u32(seed, P_SUBSAMPLE, stream, i) >> 8;
  return (uint64_t)u24 * (uint64_t)pop_left < (uint64_t)need << 24;
}

ATE_HD double gini_crit(double l0, double l1, double r0, double r1) {
  double nl = l0 + l1, nr = r0 + r1;
  double a = (l0 * l0 + l1 * l1) / nl;
  double b = (r0 * r0 + r1 * r1) / nr;
  return a + b;
}
ATE_HD double mse_crit(double sl, double nl, double sr, double nr) {
  return (sl * sl) / nl + (sr * sr) / nr;
}
ATE_HD int min_child(const ForestParams& fp, double n_node) {
  if (fp.alpha <= 0.0) return 1;
  double c = ceil(fp.alpha * n_node);
  return c < 1.0 ? 1 : (int)c;
}

// Exact-split mode (randomForest split semantics, csrc/forest_exact.hip and its host twin):
// bins are the ranks of a feature's distinct values (uint16, <= 65536 distinct values,
// vals = the sorted distinct values); a split between the node's consecutive distinct
// values u[blo] < u[bhi] is placed at their midpoint like randomForest's findbestsplit, and
// stored as the largest global bin whose value is <= the midpoint (clamped to [blo, bhi-1]
// so the node's own partition cannot change when the fp64 midpoint rounds onto u[bhi]).
// Any row whose value is in the table goes left iff value <= midpoint.
ATE_HD int exact_threshold_bin(const double* v, int nv, int blo, int bhi) {
  const double mid = (v[blo] + v[bhi]) / 2.0;
  int lo = 0, hi = nv;                 // first index with v > mid
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (v[m] <= mid) lo = m + 1; else hi = m;
  }
  int t = lo - 1;
  if (t < blo) t = blo;
  if (t > bhi - 1) t = bhi - 1;
  return t;
}

// causal node constants from exact fixed-point sums over the node's J1 rows:
// n, SW = sum W~, SY = sum Y~, SWW, SWY (products in fixed point as well)
struct CausalNode { double wbar, ybar, tau, varw; };
ATE_HD CausalNode causal_node(double n, int64_t sw, int64_t sy, int64_t sww, int64_t swy) {
  CausalNode c;
  c.wbar = from_fix(sw) / n;
  c.ybar = from_fix(sy) / n;
  double cww = from_fix(sww) / n - c.wbar * c.wbar;
  double cwy = from_fix(swy) / n - c.wbar * c.ybar;
  c.varw = cww;
  c.tau = cww > 0.0 ? cwy / cww : 0.0;
  return c;
}
ATE_HD double causal_rho(const CausalNode& c, double w, double y) {
  double dw = w - c.wbar;
  double r = dw * ((y - c.ybar) - c.tau * dw);
  return c.varw > 0.0 ? r / c.varw : 0.0;
}

// ---- little-bag variance debiasing (grf's objective Bayes debiaser)
// The between-group variance of the little-bag scores overstates the forest's variance by
// the within-group noise / (group - 1); grf does not subtract and clamp at zero (which gives
// zero-width intervals whenever the noise estimate wins) but takes the posterior mean of
// the true variance S under V ~ N(S + noise, se^2), S >= 0, a flat prior:
//   est = V - noise, se = max(V, noise) sqrt(2 / groups), r = est / se,
//   S_hat = est + se * phi(r) / Phi(r).
// Host and device must give the same bits, so exp / erfc / sqrt are built here from
// correctly rounded +, -, *, / and exact scalings (no libm: the device and host libms may
// differ by an ulp); both sides compile without FMA contraction.
ATE_HD double det_exp_neg(double y) {          // e^y for y <= 0 (Cody-Waite + Taylor-13)
  if (y < -745.0) return 0.0;
  const double k = floor(y * 1.4426950408889634 + 0.5);
  const double f = (y - k * 6.93147180369123816490e-01) - k * 1.90821492927058770002e-10;
  double s = 1.0 / 6227020800.0;                // 1/13!
  const double inv[13] = {1.0 / 479001600.0, 1.0 / 39916800.0, 1.0 / 3628800.0, 1.0 / 362880.0,
                          1.0 / 40320.0, 1.0 / 5040.0, 1.0 / 720.0, 1.0 / 120.0, 1.0 / 24.0,
                          1.0 / 6.0, 0.5, 1.0, 1.0};
  for (int i = 0; i < 13; ++i) s = s * f + inv[i];
  return ldexp(s, (int)k);
}
ATE_HD double det_sqrt(double v) {             // v > 0: Newton from an exact power-of-2 guess
  int e;
  frexp(v, &e);                                 // v = m 2^e, m in [0.5, 1)
  double s = ldexp(1.0, e / 2);                 // within a factor 2 of sqrt(v)
  for (int i = 0; i < 8; ++i) s = 0.5 * (s + v / s);
  return s;
}
// phi(r) / Phi(r) for the standard normal (x = -r / sqrt 2, Phi(r) = erfc(x) / 2)
ATE_HD double det_mills(double r) {
  const double x = -r * 0.7071067811865476;
  if (x > 2.5) {
    // erfc(x) = e^{-x^2} / (sqrt(pi) D), D = x + (1/2) / (x + 1 / (x + (3/2) / (x + ...)))
    double k = x;
    for (int j = 60; j >= 1; --j) k = x + (0.5 * j) / k;
    return 1.4142135623730951 * k;             // Phi = e^{-x^2} / (2 sqrt(pi) D), D = k
  }
  const double ax = x < 0 ? -x : x;
  const double ex = det_exp_neg(-ax * ax);
  double erf_ax;                                // erf(|x|)
  if (ax > 2.5) {
    double k = ax;
    for (int j = 60; j >= 1; --j) k = ax + (0.5 * j) / k;
    erf_ax = 1.0 - ex * 0.5641895835477563 / k;
  } else {                                      // positive series: e^{-x^2} sum 2^n x^{2n+1} / (2n+1)!!
    double t = ax, s = ax;
    const double x2 = 2.0 * ax * ax;
    for (int n = 1; n < 90; ++n) {
      t = t * x2 / (double)(2 * n + 1);
      s += t;
      if (t < s * 1e-18) break;
    }
    erf_ax = 1.1283791670955126 * ex * s;
  }
  const double erfc_x = x < 0 ? 1.0 + erf_ax : 1.0 - erf_ax;
  return (ex * 0.3989422804014327) / (0.5 * erfc_x);
}
ATE_HD double grf_debias(double between, double noise, double groups) {
  const double est = between - noise;
  const double big = between > noise ? between : noise;
  if (!(big > 0.0) || !(groups > 0.0)) return est > 0.0 ? est : 0.0;
  const double se = big * det_sqrt(2.0 / groups);
  return est + se * det_mills(est / se);
}

}  // namespace atef
