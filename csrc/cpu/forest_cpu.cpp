// Host C++ reference of the forest engine (spec: csrc/forest_common.hpp).
// One tree per OpenMP task; every tree is grown level by level exactly as the gfx950
// kernel does (csrc/forest.hip), so the two produce bit-identical trees.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <vector>

#include "../forest_common.hpp"

using namespace atef;

#define ATECPU_API extern "C" __attribute__((visibility("default")))

namespace {

struct Out {
  int cap;
  int32_t* feat;
  int32_t* thr;
  int32_t* left;
  double* val;
  int32_t* nnodes;
  uint8_t* inbag;   // [ntree][n]
  int64_t* est;     // [ntree*cap][5] (grf): cnt, S1, S2, S11, S12 (fixed point)
};

struct Rng { int lo, hi, id; };

// sample selection (grf): rows of `pop` (ascending) chosen by Algorithm S on `stream`
static std::vector<int> select_rows(const ForestParams& fp, const std::vector<int>& pop,
                                    int64_t k, uint32_t stream) {
  std::vector<int> out;
  out.reserve(k);
  int64_t N = (int64_t)pop.size();
  for (int64_t i = 0; i < N && (int64_t)out.size() < k; ++i)
    if (select_next(fp.seed, stream, (uint64_t)i, N - i, k - (int64_t)out.size()))
      out.push_back(pop[i]);
  return out;
}

// The rows of tree tg: randomForest's bootstrap counts (sampling 0) or grf's samples
// (sampling 1): with little bags (group > 1) the group's half-sample H (its rows are the
// in-bag rows of every tree of the group), then the tree's subsample of
// floor(|H| * sample_fraction * group) rows of H; with group == 1 the tree's subsample of
// floor(n * sample_fraction) rows directly (grf's ci.group.size = 1: no half-sample);
// with honesty the subsample's random half J1 grows the tree (w = 1) and the rest, J2,
// fills the estimation statistics. Same Algorithm S streams as csrc/forest.hip /
// csrc/forest_exact.hip.
static void draw_rows(const ForestParams& fp, int tg, std::vector<int32_t>& w, uint8_t* inb,
                      std::vector<int>& est_rows) {
  const int n = fp.n;
  if (fp.sampling == 0) {
    for (int j = 0; j < n; ++j) w[rand_below(fp.seed, P_RF_BOOT, (uint32_t)tg, (uint64_t)j, (uint32_t)n)]++;
    for (int i = 0; i < n; ++i) inb[i] = w[i] > 0;
    return;
  }
  std::vector<int> all(n);
  std::iota(all.begin(), all.end(), 0);
  std::vector<int> S;
  std::memset(inb, 0, n);
  if (fp.group > 1) {
    const int g = tg / fp.group;
    std::vector<int> H = select_rows(fp, all, n / 2, (uint32_t)g);
    for (int i : H) inb[i] = 1;
    double f = fp.sample_fraction * fp.group;
    if (f > 1.0) f = 1.0;
    S = f >= 1.0 ? H : select_rows(fp, H, (int64_t)std::floor(H.size() * f), 0x10000u + (uint32_t)tg);
  } else {
    S = select_rows(fp, all, (int64_t)std::floor(n * fp.sample_fraction), 0x10000u + (uint32_t)tg);
    for (int i : S) inb[i] = 1;
  }
  std::vector<int> J1 = S;
  if (fp.honesty) {
    J1 = select_rows(fp, S, (int64_t)(S.size() / 2), 0x20000u + (uint32_t)tg);
    std::vector<uint8_t> in1(n, 0);
    for (int i : J1) in1[i] = 1;
    for (int i : S)
      if (!in1[i]) est_rows.push_back(i);
  } else {
    est_rows = S;
  }
  for (int i : J1) w[i] = 1;
}

// grf estimation statistics of every node from the J2 (honest) rows: cnt, S1 (, S2, S11,
// S12 for causal trees), summed along each row's path. BT: uint8 (binned) / uint16 (exact).
template <typename BT>
static void fill_est(const ForestParams& fp, const BT* Xb, const int64_t* r1, const int64_t* r2,
                     const std::vector<int>& est_rows, const int32_t* feat, const int32_t* thr,
                     const int32_t* left, int nnode, int64_t* est) {
  std::memset(est, 0, sizeof(int64_t) * 5 * nnode);
  for (int i : est_rows) {
    int v = 0;
    while (true) {
      int64_t* e = est + (int64_t)v * 5;
      e[0] += 1;
      if (fp.kind == 1) {
        e[1] += r1[i];
      } else {
        e[1] += r1[i];
        e[2] += r2[i];
        e[3] += to_fix(from_fix(r1[i]) * from_fix(r1[i]));
        e[4] += to_fix(from_fix(r1[i]) * from_fix(r2[i]));
      }
      if (feat[v] < 0) break;
      v = Xb[(int64_t)feat[v] * fp.n + i] <= thr[v] ? left[v] : left[v] + 1;
    }
  }
}

static void grow_tree(const ForestParams& fp, int t, const uint8_t* Xb, const uint8_t* ycls,
                      const int64_t* r1, const int64_t* r2, const Out& o) {
  const int n = fp.n, p = fp.p;
  std::vector<int32_t> w(n, 0);
  const int tg = fp.t0 + t;          // global tree id (RNG key)
  std::vector<int> est_rows;
  uint8_t* inb = o.inbag + (int64_t)t * n;
  draw_rows(fp, tg, w, inb, est_rows);
  std::vector<int> idx;
  for (int i = 0; i < n; ++i)
    if (w[i] > 0) idx.push_back(i);
  const int m = (int)idx.size();
  const int64_t base = (int64_t)t * o.cap;
  int32_t* feat = o.feat + base;
  int32_t* thr = o.thr + base;
  int32_t* left = o.left + base;
  double* val = o.val + base;
  std::vector<Rng> cur{{0, m, 0}};
  int next_id = 1;
  std::vector<int> tmp(m);
  std::vector<int64_t> rho(n);
  std::vector<int> perm(p);
  int64_t h0[NBINS], h1[NBINS], hs[NBINS], ht[NBINS];
  for (int depth = 0; !cur.empty(); ++depth) {
    std::vector<Rng> nxt;
    for (const Rng& nd : cur) {
      const int v = nd.id;
      // ---- node statistics (exact integers)
      int64_t nw = 0, n1 = 0, s1 = 0, sw = 0, sy = 0, sww = 0, swy = 0;
      for (int q = nd.lo; q < nd.hi; ++q) {
        int i = idx[q];
        nw += w[i];
        if (fp.kind == 0) n1 += (int64_t)w[i] * ycls[i];
        else if (fp.kind == 1) s1 += (int64_t)w[i] * r1[i];
        else {
          sw += r1[i];
          sy += r2[i];
          sww += to_fix(from_fix(r1[i]) * from_fix(r1[i]));
          swy += to_fix(from_fix(r1[i]) * from_fix(r2[i]));
        }
      }
      const double dn = (double)nw;
      bool terminal = nw <= fp.min_node || depth >= MAX_DEPTH - 1;
      if (fp.kind == 0 && (n1 == 0 || n1 == nw)) terminal = true;
      CausalNode cn{0, 0, 0, 0};
      if (fp.kind == 2) {
        cn = causal_node(dn, sw, sy, sww, swy);
        if (!(cn.varw > 0.0)) terminal = true;
      }
      int bf = -1, bb = -1;
      int64_t bnl_rows = 0;
      if (!terminal) {
        if (fp.kind == 2)
          for (int q = nd.lo; q < nd.hi; ++q) {
            int i = idx[q];
            rho[i] = to_fix(causal_rho(cn, from_fix(r1[i]), from_fix(r2[i])));
          }
        double parent;
        int64_t stot = 0;
        if (fp.kind == 0) {
          double a = (double)(nw - n1), b = (double)n1;
          parent = (a * a + b * b) / dn;
        } else {
          if (fp.kind == 1) stot = s1;
          else
            for (int q = nd.lo; q < nd.hi; ++q) stot += rho[idx[q]];
          double sd = from_fix(stot);
          parent = (sd * sd) / dn;
        }
        const int minc = min_child(fp, dn);
        const int nf = draw_num_features(fp, tg, v);
        std::iota(perm.begin(), perm.end(), 0);
        for (int k = 0; k < nf; ++k) {
          uint32_t r = rand_below(fp.seed, P_RF_MTRY, (uint32_t)tg, node_index(v, k), (uint32_t)(p - k));
          std::swap(perm[k], perm[k + r]);
        }
        double best = -INFINITY;
        for (int k = 0; k < nf; ++k) {
          const int f = perm[k];
          const uint8_t* xf = Xb + (int64_t)f * n;
          std::memset(h0, 0, sizeof h0);
          std::memset(h1, 0, sizeof h1);
          std::memset(hs, 0, sizeof hs);
          std::memset(ht, 0, sizeof ht);
          for (int q = nd.lo; q < nd.hi; ++q) {
            int i = idx[q];
            int b = xf[i];
            if (fp.kind == 0) {
              h0[b] += (int64_t)w[i] * (1 - ycls[i]);
              h1[b] += (int64_t)w[i] * ycls[i];
            } else if (fp.kind == 1) {
              h0[b] += w[i];
              hs[b] += (int64_t)w[i] * r1[i];
            } else {
              h0[b] += 1;
              hs[b] += rho[i];
              ht[b] += from_fix(r1[i]) >= cn.wbar ? 1 : 0;
            }
          }
          int64_t c0 = 0, c1 = 0, cs = 0, ct = 0;
          int64_t ntreat = 0;
          if (fp.kind == 2)
            for (int b = 0; b < NBINS; ++b) ntreat += ht[b];
          for (int b = 0; b < NBINS - 1; ++b) {
            c0 += h0[b];
            c1 += h1[b];
            cs += hs[b];
            ct += ht[b];
            int64_t nl = fp.kind == 0 ? c0 + c1 : c0;
            int64_t nr = nw - nl;
            if (nl < minc || nr < minc) continue;
            double crit;
            if (fp.kind == 0) {
              crit = gini_crit((double)c0, (double)c1, (double)(nw - n1 - c0), (double)(n1 - c1));
            } else {
              if (fp.kind == 2) {
                int64_t tr = ntreat - ct;
                if (ct < minc || nl - ct < minc || tr < minc || nr - tr < minc) continue;
              }
              crit = mse_crit(from_fix(cs), (double)nl, from_fix(stot - cs), (double)nr);
            }
            if (crit > best) {
              best = crit;
              bf = f;
              bb = b;
            }
          }
        }
        if (!(bf >= 0 && best > parent + 1e-12 * std::max(1.0, std::fabs(parent)))) bf = -1;
      }
      if (bf < 0) {
        feat[v] = -1;
        thr[v] = -1;
        left[v] = -1;
        if (fp.kind == 0) {
          int vote;
          if (2 * n1 > nw) vote = 1;
          else if (2 * n1 < nw) vote = 0;
          else vote = (int)(rand_u32(fp.seed, P_RF_MTRY, (uint32_t)tg, node_index(v, 4095)) & 1u);
          val[v] = vote;
        } else if (fp.kind == 1) {
          val[v] = from_fix(s1) / dn;
        } else {
          val[v] = 0.0;
        }
        continue;
      }
      // ---- stable partition of [lo, hi) by bin <= bb
      const uint8_t* xf = Xb + (int64_t)bf * n;
      int nl = 0;
      for (int q = nd.lo; q < nd.hi; ++q)
        if (xf[idx[q]] <= bb) tmp[nd.lo + nl++] = idx[q];
      int nr = 0;
      for (int q = nd.lo; q < nd.hi; ++q)
        if (xf[idx[q]] > bb) tmp[nd.lo + nl + nr++] = idx[q];
      for (int q = nd.lo; q < nd.hi; ++q) idx[q] = tmp[q];
      (void)bnl_rows;
      feat[v] = bf;
      thr[v] = bb;
      left[v] = next_id;
      val[v] = 0.0;
      nxt.push_back({nd.lo, nd.lo + nl, next_id});
      nxt.push_back({nd.lo + nl, nd.hi, next_id + 1});
      next_id += 2;
    }
    cur.swap(nxt);
  }
  o.nnodes[t] = next_id;
  // ---- grf: estimation statistics of every node from the J2 (honest) rows
  if (fp.sampling == 1 && o.est)
    fill_est(fp, Xb, r1, r2, est_rows, feat, thr, left, next_id, o.est + base * 5);
}

// Exact-split mode (GPU twin csrc/forest_exact.hip): uint16 value-rank bins. A node's
// candidate feature is scanned over its rows sorted by (bin, row); the criterion is
// evaluated at every boundary between two consecutive DISTINCT in-node values, in
// ascending order, with the same integer statistics, formulas and (feature slot,
// position) tie-break as the binned engine. randomForest sampling (0): kinds 0/1, the
// threshold is the value midpoint (forest_common.hpp::exact_threshold_bin). grf sampling
// (1): kinds 1/2 with half-samples, honesty and J2 estimation statistics; the threshold is
// the left value itself (x <= v goes left). Kind 2 (causal) scans the node's pseudo-
// outcomes rho with the per-position statistic 1 + treated * 2^32 (count and treated count
// in one int64 prefix sum) so each child keeps >= 1 treated and >= 1 control row.
static void grow_tree_exact(const ForestParams& fp, int t, const uint16_t* Xb, const double* vals,
                            int ldv, const int32_t* nval, const uint8_t* ycls, const int64_t* r1,
                            const int64_t* r2, const Out& o) {
  const int n = fp.n, p = fp.p;
  std::vector<int32_t> w(n, 0);
  const int tg = fp.t0 + t;
  uint8_t* inb = o.inbag + (int64_t)t * n;
  std::vector<int> est_rows;
  draw_rows(fp, tg, w, inb, est_rows);
  std::vector<int> idx;
  for (int i = 0; i < n; ++i)
    if (w[i] > 0) idx.push_back(i);
  const int m = (int)idx.size();
  const int64_t base = (int64_t)t * o.cap;
  int32_t* feat = o.feat + base;
  int32_t* thr = o.thr + base;
  int32_t* left = o.left + base;
  double* val = o.val + base;
  std::vector<Rng> cur{{0, m, 0}};
  int next_id = 1;
  std::vector<int> tmp(m);
  std::vector<uint64_t> keys(m);
  std::vector<int> perm(p);
  std::vector<int64_t> rho(fp.kind == 2 ? n : 0);
  const int64_t LO32 = 0xffffffffll;
  for (int depth = 0; !cur.empty(); ++depth) {
    std::vector<Rng> nxt;
    for (const Rng& nd : cur) {
      const int v = nd.id;
      int64_t nw = 0, n1 = 0, s1 = 0, sw = 0, sy = 0, sww = 0, swy = 0;
      for (int q = nd.lo; q < nd.hi; ++q) {
        const int i = idx[q];
        nw += w[i];
        if (fp.kind == 0) n1 += (int64_t)w[i] * ycls[i];
        else if (fp.kind == 1) s1 += (int64_t)w[i] * r1[i];
        else {
          sw += r1[i];
          sy += r2[i];
          sww += to_fix(from_fix(r1[i]) * from_fix(r1[i]));
          swy += to_fix(from_fix(r1[i]) * from_fix(r2[i]));
        }
      }
      const double dn = (double)nw;
      bool terminal = nw <= fp.min_node || depth >= MAX_DEPTH - 1;
      if (fp.kind == 0 && (n1 == 0 || n1 == nw)) terminal = true;
      CausalNode cn{0, 0, 0, 0};
      if (fp.kind == 2) {
        cn = causal_node(dn, sw, sy, sww, swy);
        if (!(cn.varw > 0.0)) terminal = true;
      }
      int bf = -1, blo = -1, bhi = -1;
      if (!terminal) {
        int64_t stot = s1;
        if (fp.kind == 2) {
          stot = 0;
          for (int q = nd.lo; q < nd.hi; ++q) {
            const int i = idx[q];
            rho[i] = to_fix(causal_rho(cn, from_fix(r1[i]), from_fix(r2[i])));
            stot += rho[i];
          }
        }
        double parent;
        if (fp.kind == 0) {
          double a = (double)(nw - n1), b = (double)n1;
          parent = (a * a + b * b) / dn;
        } else {
          double sd = from_fix(stot);
          parent = (sd * sd) / dn;
        }
        const int minc = min_child(fp, dn);
        const int nf = draw_num_features(fp, tg, v);
        std::iota(perm.begin(), perm.end(), 0);
        for (int k = 0; k < nf; ++k) {
          uint32_t r = rand_below(fp.seed, P_RF_MTRY, (uint32_t)tg, node_index(v, k), (uint32_t)(p - k));
          std::swap(perm[k], perm[k + r]);
        }
        int64_t ntreat = 0;
        if (fp.kind == 2)
          for (int q = nd.lo; q < nd.hi; ++q) ntreat += from_fix(r1[idx[q]]) >= cn.wbar ? 1 : 0;
        double best = -INFINITY;
        const int cnt = nd.hi - nd.lo;
        for (int k = 0; k < nf; ++k) {
          const int f = perm[k];
          const uint16_t* xf = Xb + (int64_t)f * n;
          for (int q = 0; q < cnt; ++q)
            keys[q] = ((uint64_t)xf[idx[nd.lo + q]] << 32) | (uint32_t)idx[nd.lo + q];
          std::sort(keys.begin(), keys.begin() + cnt);
          int64_t c0 = 0, c1 = 0;
          for (int s = 0; s + 1 < cnt; ++s) {
            const int i = (int)(uint32_t)keys[s];
            if (fp.kind == 0) {
              c0 += (int64_t)w[i] * (1 - ycls[i]);
              c1 += (int64_t)w[i] * ycls[i];
            } else if (fp.kind == 1) {
              c0 += w[i];
              c1 += (int64_t)w[i] * r1[i];
            } else {
              c0 += 1 + ((from_fix(r1[i]) >= cn.wbar ? 1ll : 0ll) << 32);
              c1 += rho[i];
            }
            const int b = (int)(keys[s] >> 32), bn = (int)(keys[s + 1] >> 32);
            if (b == bn) continue;
            const int64_t nl = fp.kind == 0 ? c0 + c1 : (c0 & LO32);
            const int64_t nr = nw - nl;
            if (nl < minc || nr < minc) continue;
            if (fp.kind == 2) {
              const int64_t ct = c0 >> 32, tr = ntreat - ct;
              if (ct < minc || nl - ct < minc || tr < minc || nr - tr < minc) continue;
            }
            const double crit = fp.kind == 0
                ? gini_crit((double)c0, (double)c1, (double)(nw - n1 - c0), (double)(n1 - c1))
                : mse_crit(from_fix(c1), (double)nl, from_fix(stot - c1), (double)nr);
            if (crit > best) {
              best = crit;
              bf = f;
              blo = b;
              bhi = bn;
            }
          }
        }
        if (!(bf >= 0 && best > parent + 1e-12 * std::max(1.0, std::fabs(parent)))) bf = -1;
      }
      if (bf < 0) {
        feat[v] = -1;
        thr[v] = -1;
        left[v] = -1;
        if (fp.kind == 0) {
          int vote;
          if (2 * n1 > nw) vote = 1;
          else if (2 * n1 < nw) vote = 0;
          else vote = (int)(rand_u32(fp.seed, P_RF_MTRY, (uint32_t)tg, node_index(v, 4095)) & 1u);
          val[v] = vote;
        } else if (fp.kind == 1) {
          val[v] = from_fix(s1) / dn;
        } else {
          val[v] = 0.0;
        }
        continue;
      }
      const int tb = fp.sampling == 1 ? blo
                                      : exact_threshold_bin(vals + (int64_t)bf * ldv, nval[bf], blo, bhi);
      const uint16_t* xf = Xb + (int64_t)bf * n;
      int nl = 0;
      for (int q = nd.lo; q < nd.hi; ++q)
        if (xf[idx[q]] <= tb) tmp[nd.lo + nl++] = idx[q];
      int nr = 0;
      for (int q = nd.lo; q < nd.hi; ++q)
        if (xf[idx[q]] > tb) tmp[nd.lo + nl + nr++] = idx[q];
      for (int q = nd.lo; q < nd.hi; ++q) idx[q] = tmp[q];
      feat[v] = bf;
      thr[v] = tb;
      left[v] = next_id;
      val[v] = 0.0;
      nxt.push_back({nd.lo, nd.lo + nl, next_id});
      nxt.push_back({nd.lo + nl, nd.hi, next_id + 1});
      next_id += 2;
    }
    cur.swap(nxt);
  }
  o.nnodes[t] = next_id;
  if (fp.sampling == 1 && o.est)
    fill_est(fp, Xb, r1, r2, est_rows, feat, thr, left, next_id, o.est + base * 5);
}

}  // namespace

ATECPU_API int atecpu_forest_fit_exact(const ForestParams* fpp, const uint16_t* Xb, const double* vals,
                                       int ldv, const int32_t* nval, const uint8_t* ycls,
                                       const int64_t* r1, const int64_t* r2, int cap, int32_t* feat,
                                       int32_t* thr, int32_t* left, double* val, int32_t* nnodes,
                                       uint8_t* inbag, int64_t* est, int nthreads) {
  const ForestParams fp = *fpp;
  if (fp.p >= 4094 || fp.n <= 0) return -1;
  if (fp.sampling == 0 ? fp.kind == 2 : (fp.kind == 0 || !est)) return -1;
  Out o{cap, feat, thr, left, val, nnodes, inbag, est};
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
  for (int t = 0; t < fp.ntree; ++t) grow_tree_exact(fp, t, Xb, vals, ldv, nval, ycls, r1, r2, o);
  return 0;
}

ATECPU_API int atecpu_forest_fit(const ForestParams* fpp, const uint8_t* Xb, const uint8_t* ycls,
                                 const int64_t* r1, const int64_t* r2, int cap, int32_t* feat,
                                 int32_t* thr, int32_t* left, double* val, int32_t* nnodes,
                                 uint8_t* inbag, int64_t* est, int nthreads) {
  const ForestParams fp = *fpp;
  if (fp.p >= 4094 || fp.n <= 0) return -1;
  Out o{cap, feat, thr, left, val, nnodes, inbag, est};
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
  for (int t = 0; t < fp.ntree; ++t) grow_tree(fp, t, Xb, ycls, r1, r2, o);
  return 0;
}

// Forest predictions on a binned matrix Xb [p][n2].
//  oob: use tree t for row i only if inbag[t][i] == 0 (requires n2 == fp.n).
//  out (kind 0): [n2] vote share (NaN if no tree used); (kind 1): [n2] mean of tree
//  predictions; (kind 2): [n2][4] = tau, var (little bags), trees used, groups used.
// Regression/causal grf trees predict from the deepest node on the path with J2 rows.
template <typename BT>
static int predict_impl(const ForestParams* fpp, const BT* Xb, int n2, int oob, int cap,
                        const int32_t* feat, const int32_t* thr, const int32_t* left,
                        const double* val, const uint8_t* inbag, const int64_t* est, int64_t* state,
                        int phases, double* out, int nthreads) {
  // state: [10][n2] int64 accumulators (2^-32 fixed point, forest_common.hpp mean_fix),
  // same protocol as csrc/forest.hip ate_forest_predict
  // (1 = per-tree sums, 2 = kind-2 little-bag group sums, 4 = finalise).
  const ForestParams fp = *fpp;
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
  for (int i = 0; i < n2; ++i) {
    // the node whose statistics predict for row i in tree t (-1 if the tree is excluded)
    auto leaf_of = [&](int t) -> int64_t {
      if (oob && inbag[(int64_t)t * fp.n + i]) return -1;
      const int64_t base = (int64_t)t * cap;
      int v = 0, last_ok = 0;
      while (true) {
        if (fp.sampling == 1 && est && est[(base + v) * 5] > 0) last_ok = v;
        if (feat[base + v] < 0) break;
        v = Xb[(int64_t)feat[base + v] * n2 + i] <= thr[base + v] ? left[base + v] : left[base + v] + 1;
      }
      return base + (fp.sampling == 1 && est ? last_ok : v);
    };
    int64_t* st = state;
    if (phases & 1) {
      if (fp.kind != 2) {
        int64_t acc = st[i], used = st[n2 + i];
        for (int t = 0; t < fp.ntree; ++t) {
          const int64_t nd = leaf_of(t);
          if (nd < 0) continue;
          used += 1;
          if (fp.kind == 0 || fp.sampling == 0) acc += to_fix(val[nd]);
          else acc += mean_fix(est[nd * 5 + 1], est[nd * 5]);
        }
        st[i] = acc;
        st[n2 + i] = used;
      } else {
        int64_t a1 = st[i], aw = st[n2 + i], ay = st[2 * n2 + i], aww = st[3 * n2 + i],
                awy = st[4 * n2 + i];
        for (int t = 0; t < fp.ntree; ++t) {
          const int64_t nd = leaf_of(t);
          if (nd < 0) continue;
          const int64_t* e = est + nd * 5;
          a1 += 1; aw += mean_fix(e[1], e[0]); ay += mean_fix(e[2], e[0]);
          aww += mean_fix(e[3], e[0]); awy += mean_fix(e[4], e[0]);
        }
        st[i] = a1; st[n2 + i] = aw; st[2 * n2 + i] = ay; st[3 * n2 + i] = aww;
        st[4 * n2 + i] = awy;
      }
    }
    if ((phases & 2) && fp.kind == 2 && st[i] > 0) {
      // little bags: linearised score psi = (w - Wbar)(y - Ybar - tau (w - Wbar)) per
      // group at the full-forest tau
      const double a1 = (double)st[i];
      const double wb = from_fix(st[n2 + i]) / a1, yb = from_fix(st[2 * n2 + i]) / a1;
      const double H = from_fix(st[3 * n2 + i]) / a1 - wb * wb;
      if (H > 0) {
        const double tau = (from_fix(st[4 * n2 + i]) / a1 - wb * yb) / H;
        int64_t gs = st[5 * n2 + i], gss = st[6 * n2 + i], within = st[7 * n2 + i];
        int64_t nwithin = st[8 * n2 + i], ng = st[9 * n2 + i];
        for (int g0 = 0; g0 < fp.ntree; g0 += fp.group) {
          double ps = 0, pss = 0;
          int nb = 0;
          const int gsz = g0 + fp.group <= fp.ntree ? fp.group : fp.ntree - g0;
          for (int t = g0; t < g0 + fp.group && t < fp.ntree; ++t) {
            const int64_t nd = leaf_of(t);
            if (nd < 0) continue;
            const int64_t* e = est + nd * 5;
            const double w_ = from_fix(mean_fix(e[1], e[0])), y_ = from_fix(mean_fix(e[2], e[0]));
            const double ww = from_fix(mean_fix(e[3], e[0])), wy = from_fix(mean_fix(e[4], e[0]));
            const double psi = wy - wb * y_ - yb * w_ + wb * yb - tau * (ww - 2.0 * wb * w_ + wb * wb);
            ps += psi; pss += psi * psi; ++nb;
          }
          if (nb == 0 || nb < gsz) continue;   // grf: complete groups only
          const double pg = ps / nb;
          gs += to_fix(pg); gss += to_fix(pg * pg); ng += 1;
          if (nb >= 2) { within += to_fix(pss / nb - pg * pg); nwithin += 1; }
        }
        st[5 * n2 + i] = gs; st[6 * n2 + i] = gss; st[7 * n2 + i] = within;
        st[8 * n2 + i] = nwithin; st[9 * n2 + i] = ng;
      }
    }
    if (phases & 4) {
      if (fp.kind != 2) {
        out[i] = st[n2 + i] > 0 ? from_fix(st[i]) / (double)st[n2 + i] : NAN;
        continue;
      }
      const double a1 = (double)st[i];
      double tau = NAN, var = NAN;
      const double ng = (double)st[9 * n2 + i];
      if (a1 > 0) {
        const double wb = from_fix(st[n2 + i]) / a1, yb = from_fix(st[2 * n2 + i]) / a1;
        const double H = from_fix(st[3 * n2 + i]) / a1 - wb * wb;
        if (H > 0) {
          tau = (from_fix(st[4 * n2 + i]) / a1 - wb * yb) / H;
          if (ng >= 2) {
            const double mean = from_fix(st[5 * n2 + i]) / ng;
            const double between = from_fix(st[6 * n2 + i]) / ng - mean * mean;
            const double nw = (double)st[8 * n2 + i];
            const double wc = nw > 0 ? from_fix(st[7 * n2 + i]) / nw / (double)(fp.group > 1 ? fp.group - 1 : 1) : 0.0;
            var = grf_debias(between, wc, ng) / (H * H);
          }
        }
      }
      out[4 * i + 0] = tau;
      out[4 * i + 1] = var;
      out[4 * i + 2] = a1;
      out[4 * i + 3] = ng;
    }
  }
  return 0;
}

ATECPU_API int atecpu_forest_predict(const ForestParams* fpp, const uint8_t* Xb, int n2, int oob,
                                     int cap, const int32_t* feat, const int32_t* thr,
                                     const int32_t* left, const double* val,
                                     const uint8_t* inbag, const int64_t* est, int64_t* state,
                                     int phases, double* out, int nthreads) {
  return predict_impl(fpp, Xb, n2, oob, cap, feat, thr, left, val, inbag, est, state, phases, out,
                      nthreads);
}

// exact-split forests: uint16 value-rank bins
ATECPU_API int atecpu_forest_predict16(const ForestParams* fpp, const uint16_t* Xb, int n2, int oob,
                                       int cap, const int32_t* feat, const int32_t* thr,
                                       const int32_t* left, const double* val,
                                       const uint8_t* inbag, const int64_t* est, int64_t* state,
                                       int phases, double* out, int nthreads) {
  return predict_impl(fpp, Xb, n2, oob, cap, feat, thr, left, val, inbag, est, state, phases, out,
                      nthreads);
}

// the little-bag variance debiaser alone (forest_common.hpp grf_debias; tests check it
// against scipy's normal density / CDF)
ATECPU_API double atecpu_grf_debias(double between, double noise, double groups) {
  return grf_debias(between, noise, groups);
}
