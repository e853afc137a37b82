// Level-synchronous forest engine for LARGE training sets (BASELINE config 3: 8e6-row
// bootstrap trees), randomForest semantics (kind 0 classification / kind 1 regression,
// bootstrap sampling). Spec: forest_common.hpp; same trees, bit for bit, as the
// one-workgroup-per-tree kernel (forest.hip) and the host twin (cpu/forest_cpu.cpp).
//
// Why: one workgroup per tree puts a whole 8e6-row tree on ONE CU; its top levels stream
// millions of dependent idx -> bin gathers through 16 waves and its middle levels walk
// thousands of nodes a wave at a time (the per-GPU shard of config 3 took 37 s). Here the
// GPU grows ALL trees of a forest together, one tree level per step, and every node is
// sized to its own decomposition:
//
//  * BIG nodes (> LV_BIG rows): many workgroups per node. Work items = (node, chunk of
//    LV_CH positions) x (group of LV_FG drawn features); each item stages the group's
//    histograms in LDS (int64, exact) and adds them to the node's global histogram with
//    int64 atomics (exact, any order). A workgroup per node then scans every drawn feature
//    (one wave per feature, 4 bins per lane) and picks the split.
//  * MID nodes (65 .. LV_BIG rows): one workgroup per node; per feature group all rows'
//    bins are gathered at once (LV_FG independent loads per row) into LDS histograms.
//  * SMALL nodes (<= 64 rows): one wave per node, rows in registers: <= 16 rows compare
//    every present bin directly, 17-64 rows use a per-wave LDS histogram.
//  * partition: stable (ascending positions, like the host), ping-pong position buffers;
//    big nodes by chunk counts + scan + scatter, the others one wave per node (ballot).
//  * node ids: level order per tree (an exclusive scan of the split flags over the level
//    list, which is grouped by tree), exactly the host's numbering.
// Decisions use the same exact integer sums and explicitly rounded fp64 criteria (this file
// is compiled with -ffp-contract=off) and the same tie-breaks: per feature the max
// criterion at the lowest bin, across features strict improvement in draw order.
#include <stdint.h>

#include <algorithm>

#include "common.hpp"
#include "forest_common.hpp"

using namespace atef;

namespace {

constexpr int LV_FG = 8;          // drawn features per histogram pass
constexpr int LV_PMAX = 512;      // max features (per-wave permutation buffer)
constexpr int LV_MAXF = 64;       // max drawn features per node (kinds 0/1: nf = mtry)

struct LNode { int tree, lo, hi, id; };

__device__ __forceinline__ int64_t lv_wsum(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// criterion of "bin <= b goes left" from the left sums; -inf when not admissible
__device__ __forceinline__ double lv_crit(int kind, int64_t L0, int64_t L1, int64_t nw, int64_t n1,
                                          int64_t s1, int minc) {
  const int64_t nl = kind == 0 ? L0 + L1 : L0;
  const int64_t nr = nw - nl;
  if (nl < minc || nr < minc) return -INFINITY;
  if (kind == 0)
    return gini_crit((double)L0, (double)L1, (double)(nw - n1 - L0), (double)(n1 - L1));
  return mse_crit(from_fix(L1), (double)nl, from_fix(s1 - L1), (double)nr);
}

// one wave scans a feature's two-channel histogram (h0, h1: 256 bins each, any memory):
// max criterion, lowest bin on ties (bin NBINS when nothing is admissible)
template <typename HT>
__device__ __forceinline__ void lv_scan(const HT* h0, const HT* h1, int kind, int64_t nw,
                                        int64_t n1, int64_t s1, int minc, double* best,
                                        int* bin) {
  const int lane = threadIdx.x & 63;
  int64_t c0[4], c1[4];
  int64_t a0 = 0, a1 = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    a0 += (int64_t)h0[4 * lane + e];
    a1 += (int64_t)h1[4 * lane + e];
    c0[e] = a0;
    c1[e] = a1;
  }
  int64_t x0 = a0, x1 = a1;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y0 = __shfl_up(x0, o, 64), y1 = __shfl_up(x1, o, 64);
    if (lane >= o) { x0 += y0; x1 += y1; }
  }
  const int64_t p0 = x0 - a0, p1 = x1 - a1;
  double lbest = -INFINITY;
  int lbin = NBINS;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int b = 4 * lane + e;
    if (b >= NBINS - 1) continue;
    const double c = lv_crit(kind, p0 + c0[e], p1 + c1[e], nw, n1, s1, minc);
    if (c > lbest) { lbest = c; lbin = b; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double oc = __shfl_xor(lbest, o, 64);
    const int ob = __shfl_xor(lbin, o, 64);
    if (oc > lbest || (oc == lbest && ob < lbin)) { lbest = oc; lbin = ob; }
  }
  *best = lbest;
  *bin = lbin;
}

// LDS atomics of few-bin features (binary covariates: 64 lanes on 2 x 2 addresses) serialise
// in the LDS. A feature with nb bins therefore SPREADS its histogram over the same 256 slots:
// slot = bin * S + (lane & (S - 1)), S = the largest power of two <= 64 with nb * S <= 256,
// so lanes of a wave hit different slots; lv_collapse folds the S copies back into bins
// [0, nb) (exact integer sums) before a scan reads them.
__device__ __forceinline__ int lv_spread(int nb) {
  int S = 1;
  while (S < 64 && nb * (S * 2) <= NBINS) S *= 2;
  return S;
}

// one wave folds a spread two-channel histogram in place (slots >= nb end up zero)
template <typename HT>
__device__ void lv_collapse(HT* h0, HT* h1, int S) {
  if (S == 1) return;
  const int lane = threadIdx.x & 63;
  HT a[4], b[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) { a[e] = h0[4 * lane + e]; b[e] = h1[4 * lane + e]; }
  HT p0, p1, q0 = 0, q1 = 0;
  if (S == 2) {                                   // lane holds bins 2L (slots 0,1), 2L+1 (2,3)
    p0 = a[0] + a[1]; q0 = a[2] + a[3];
    p1 = b[0] + b[1]; q1 = b[2] + b[3];
  } else {                                        // lane holds part of bin 4L / S
    p0 = a[0] + a[1] + a[2] + a[3];
    p1 = b[0] + b[1] + b[2] + b[3];
    for (int o = 1; o < S / 4; o <<= 1) {
      p0 += __shfl_xor(p0, o, 64);
      p1 += __shfl_xor(p1, o, 64);
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int e = 0; e < 4; ++e) { h0[4 * lane + e] = 0; h1[4 * lane + e] = 0; }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_wave_barrier();
  if (S == 2) {
    h0[2 * lane] = p0; h0[2 * lane + 1] = q0;
    h1[2 * lane] = p1; h1[2 * lane + 1] = q1;
  } else if ((lane & (S / 4 - 1)) == 0) {
    const int bin = lane / (S / 4);
    h0[bin] = p0;
    h1[bin] = p1;
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_wave_barrier();
}

// the partial Fisher-Yates draw of a node's candidate features (forest.hip / host order):
// perm[0..nf) in a per-wave LDS buffer of p int16
__device__ void lv_draw(const ForestParams& fp, int tg, int v, int nf, int16_t* perm) {
  const int lane = threadIdx.x & 63;
  for (int k = lane; k < fp.p; k += 64) perm[k] = (int16_t)k;
  const uint32_t rk = lane < nf ? rand_below(fp.seed, P_RF_MTRY, (uint32_t)tg, node_index(v, lane),
                                             (uint32_t)(fp.p - lane)) : 0u;
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    for (int k = 0; k < nf; ++k) {
      const uint32_t r = k < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)rk, k)
                                : rand_below(fp.seed, P_RF_MTRY, (uint32_t)tg, node_index(v, k),
                                             (uint32_t)(fp.p - k));
      const int16_t t = perm[k];
      perm[k] = perm[k + r];
      perm[k + r] = t;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_wave_barrier();
}

// leaf value / decision record (lane 0 of the deciding wave)
__device__ void lv_record(const ForestParams& fp, int tg, int v, int bf, int bb, int64_t nw,
                          int64_t n1, int64_t s1, int32_t* feat, int32_t* thr, int32_t* left,
                          double* val, int4* dec) {
  if (bf >= 0) {
    feat[v] = bf;
    thr[v] = bb;
    val[v] = 0.0;
  } else {
    feat[v] = -1;
    thr[v] = -1;
    left[v] = -1;
    if (fp.kind == 0) {
      int vote;
      if (2 * n1 > nw) vote = 1;
      else if (2 * n1 < nw) vote = 0;
      else vote = (int)(rand_u32(fp.seed, P_RF_MTRY, (uint32_t)tg, node_index(v, 4095)) & 1u);
      val[v] = vote;
    } else {
      val[v] = from_fix(s1) / (double)nw;
    }
  }
  *dec = make_int4(bf >= 0 ? 1 : 0, bf, bb, 0);
}

// terminal test + parent criterion from the node totals
__device__ __forceinline__ bool lv_terminal(const ForestParams& fp, int64_t nw, int64_t n1,
                                            int depth) {
  bool t = nw <= fp.min_node || depth >= MAX_DEPTH - 1;
  if (fp.kind == 0 && (n1 == 0 || n1 == nw)) t = true;
  return t;
}
__device__ __forceinline__ double lv_parent(int kind, int64_t nw, int64_t n1, int64_t s1) {
  const double dn = (double)nw;
  if (kind == 0) {
    const double a = (double)(nw - n1), b = (double)n1;
    return __ddiv_rn(__dadd_rn(__dmul_rn(a, a), __dmul_rn(b, b)), dn);
  }
  const double sd = from_fix(s1);
  return __ddiv_rn(__dmul_rn(sd, sd), dn);
}
__device__ __forceinline__ bool lv_accept(double best, double parent) {
  return best > parent + 1e-12 * fmax(1.0, fabs(parent));
}

struct LvArgs {
  ForestParams fp;
  const uint8_t* Xb;      // bins: element (feature f, row i) at f * fst + i * rst
  const uint8_t* Xc;      // the same bins column-major [p][n] (dense big-node streams)
  const int16_t* nbin;    // [p] bins per feature (edges + 1)
  const uint8_t* ycls;    // kind 0: [n] class
  const int64_t* r1;      // kind 1: [n] response, 2^-32 fixed point
  const int32_t* w;       // [T][n] bootstrap counts
  const int32_t* idx;     // [T * n] positions of this level (ping)
  int32_t* idx2;          // [T * n] next level positions (pong)
  const LNode* cur;       // [ncur] level list (grouped by tree, level order)
  int4* dec;              // [ncur] (split, feat, bin, -)
  int32_t* nl;            // [ncur] left rows of split nodes
  int cap;                // node capacity per tree
  int32_t* feat;
  int32_t* thr;
  int32_t* left;
  double* val;
  int depth;
  int64_t fst, rst;       // column-major [p][n]: (n, 1); row-major [n][p]: (1, p)
};


// accumulate rows [q0, q1) (stride 256 per thread, 4 rows per thread in flight: the idx
// loads, then every row's weight / label / LV_FG bins, then the LDS atomics) into the LDS
// histograms sh[k][c][bin] of the nk features xf[0..nk)
// HT: LDS histogram element (uint32 for kind 0: integer weights; int64 for kind 1),
// FG: features per pass, U: rows in flight per thread
template <typename HT, int FG, int U>
__device__ __forceinline__ void lv_accumulate(const LvArgs& a, const int32_t* __restrict__ wt,
                                              const uint8_t* X, const int* fi, int64_t fst,
                                              const int* sp, int64_t rst, int nk, int q0, int q1,
                                              HT (*sh)[2][NBINS]) {
  const int kind = a.fp.kind;
  const int lane = threadIdx.x & 63;
  for (int base = q0 + threadIdx.x; base < q1; base += 256 * U) {
    int ii[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = base + u * 256;
      ii[u] = q < q1 ? a.idx[q] : -1;
    }
    int64_t wv[U], rv[U];
    int yv[U];
    int bins[U][FG];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = ii[u] < 0 ? 0 : ii[u];
      wv[u] = ii[u] < 0 ? 0 : wt[i];
      yv[u] = kind == 0 ? a.ycls[i] : 0;
      rv[u] = kind == 0 ? 0 : a.r1[i];
#pragma unroll
      for (int k = 0; k < FG; ++k) bins[u][k] = X[(int64_t)fi[k] * fst + (int64_t)i * rst];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (ii[u] < 0) continue;
#pragma unroll
      for (int k = 0; k < FG; ++k) {
        if (k >= nk) break;
        const int slot = bins[u][k] * sp[k] + (lane & (sp[k] - 1));
        if constexpr (sizeof(HT) == 4) {                    // kind 0: class weights
          atomicAdd((unsigned int*)&sh[k][yv[u]][slot], (unsigned int)wv[u]);
        } else if (kind == 0) {
          atomicAdd((unsigned long long*)&sh[k][yv[u]][slot], (unsigned long long)wv[u]);
        } else {
          atomicAdd((unsigned long long*)&sh[k][0][slot], (unsigned long long)wv[u]);
          atomicAdd((unsigned long long*)&sh[k][1][slot], (unsigned long long)(wv[u] * rv[u]));
        }
      }
    }
  }
}

#ifndef LV_MID_RK
#define LV_MID_RK 1
#endif
// Kind-0 mid nodes, lanes = (row, feature): lane l of a wave takes drawn feature l & 31 of
// row l >> 5, so one wave instruction gathers the drawn bins of TWO rows (their few cache
// lines, coalesced) instead of one bin of 64 rows (64 lines, one byte each); the row's
// index, weight and class are one broadcast load per 32 lanes. Same integer sums as
// lv_accumulate, in any order. U rows per lane in flight.
template <int FG, int U>
__device__ __forceinline__ void lv_accumulate_rk(const LvArgs& a, const int32_t* __restrict__ wt,
                                                 const uint8_t* X, int fik, int64_t fst,
                                                 int spk, int64_t rst, int nk, int q0, int q1,
                                                 uint32_t (*sh)[2][NBINS]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane >> 5, k = lane & 31;
  const bool kon = k < nk;
  const int kk = kon ? k : 0;
  const int64_t fo = (int64_t)fik * fst;
  const int spread = lane & (spk - 1);
  // rows of step s: q0 + ((s * U + u) * 4 + wid) * 2 + r
  for (int base = q0 + wid * 2 + r; base < q1; base += 8 * U) {
    int ii[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = base + u * 8;
      ii[u] = q < q1 ? a.idx[q] : -1;
    }
    uint32_t wv[U];
    int yv[U], bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = ii[u] < 0 ? 0 : ii[u];
      wv[u] = ii[u] < 0 ? 0u : (uint32_t)wt[i];
      yv[u] = a.ycls[i];
      bv[u] = X[fo + (int64_t)i * rst];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (ii[u] >= 0 && kon)
        atomicAdd(&sh[kk][yv[u]][bv[u] * spk + spread], wv[u]);
  }
}

// ------------------------------------------------------------------ sampling (K10)
__global__ __launch_bounds__(256) void lv_boot_kernel(ForestParams fp, int32_t* __restrict__ w) {
  const int t = blockIdx.y;
  const int n = fp.n;
  int32_t* wt = w + (int64_t)t * n;
  for (int j = blockIdx.x * 256 + threadIdx.x; j < n; j += gridDim.x * 256)
    atomicAdd(&wt[rand_below(fp.seed, P_RF_BOOT, (uint32_t)(fp.t0 + t), (uint64_t)j, (uint32_t)n)], 1);
}

// ------------------------------------------------------------------ node classes
// classes: 0 small (<= 64 rows: wave decide, wave partition), 1 mid (<= t2 rows: workgroup
// decide, wave partition), 2 mid-large (<= t3: workgroup decide, chunked partition), 3 big
// (> t3: multi-workgroup decide, chunked partition). One atomic per wave and class.
// The level length is 2 * nsplit[0] (the previous level's split count, still on the device:
// the host learns it with the class counts, counts[4], in ONE read per level) or, with no
// nsplit, ncur_ub; the grid and the class lists' stride are sized for ncur_ub.
__global__ __launch_bounds__(256) void lv_classify_kernel(const LNode* __restrict__ cur,
                                                          int ncur_ub,
                                                          const int32_t* __restrict__ nsplit,
                                                          int t2, int t3, int32_t* __restrict__ lists,
                                                          int32_t* __restrict__ counts) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int ncur = nsplit ? 2 * nsplit[0] : ncur_ub;
  ATE_DASSERT(ncur <= ncur_ub);
  if (j == 0) counts[4] = ncur;
  int c = -1;
  if (j < ncur) {
    const int m = cur[j].hi - cur[j].lo;
    c = m <= 64 ? 0 : (m <= t2 ? 1 : (m <= t3 ? 2 : 3));
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint64_t mk = __ballot(c == k);
    if (!mk) continue;
    const int leader = __ffsll((long long)mk) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(&counts[k], __popcll(mk));
    base = __shfl(base, leader, 64);
    if (c == k) {
      const int pos = base + __popcll(mk & ((1ull << lane) - 1ull));
      ATE_DASSERT(pos < ncur);
      lists[(int64_t)k * ncur_ub + pos] = j;
    }
  }
}

// ------------------------------------------------------------------ BIG nodes
// drawn features of each big node: [nbig][LV_MAXF] int16, nf[nbig]
__global__ __launch_bounds__(256) void lv_big_draw_kernel(LvArgs a, const int32_t* __restrict__ blist,
                                                          int nbig, int16_t* __restrict__ drawn,
                                                          int32_t* __restrict__ nfo) {
  __shared__ int16_t perm[4][LV_PMAX];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + wid;
  if (b >= nbig) return;                                    // uniform per wave
  const LNode nd = a.cur[blist[b]];
  const int tg = a.fp.t0 + nd.tree;
  const int nf = draw_num_features(a.fp, tg, nd.id);
  lv_draw(a.fp, tg, nd.id, nf, perm[wid]);
  for (int k = lane; k < nf; k += 64) drawn[(int64_t)b * LV_MAXF + k] = perm[wid][k];
  if (lane == 0) nfo[b] = nf;
}

// work item = (big slot, [q0, q1) positions) x feature group blockIdx.y: LDS histograms of
// the group's features, added to hist[slot][k][c][bin] with int64 atomics
__global__ __launch_bounds__(256) void lv_big_hist_kernel(LvArgs a, const int32_t* __restrict__ item_slot,
                                                          const int32_t* __restrict__ item_q0,
                                                          const int32_t* __restrict__ item_q1,
                                                          const int32_t* __restrict__ blist,
                                                          const int16_t* __restrict__ drawn,
                                                          const int32_t* __restrict__ nfo,
                                                          int64_t* __restrict__ hist, int fs) {
  __shared__ int64_t sh[LV_FG][2][NBINS];
  const int it = blockIdx.x, g = blockIdx.y;
  const int slot = item_slot[it];
  const int nf = nfo[slot];
  const int k0 = g * LV_FG;
  if (k0 >= nf) return;                                     // uniform
  const int nk = min(LV_FG, nf - k0);
  const LNode nd = a.cur[blist[slot]];
  const int n = a.fp.n;
  // positions are global over the forest's trees (tree t's in-bag rows after tree t-1's),
  // so a node's range is bounded by ntree * n, not by n
  ATE_DASSERT(nd.lo <= item_q0[it] && item_q0[it] <= item_q1[it] && item_q1[it] <= nd.hi &&
              (int64_t)nd.hi <= (int64_t)a.fp.ntree * n && nk <= LV_FG && k0 + nk <= LV_MAXF);
  const int32_t* wt = a.w + (int64_t)nd.tree * n;
  for (int e = threadIdx.x; e < LV_FG * 2 * NBINS; e += 256) (&sh[0][0][0])[e] = 0;
  int fi[LV_FG], sp[LV_FG];
#pragma unroll
  for (int k = 0; k < LV_FG; ++k) {
    fi[k] = drawn[(int64_t)slot * LV_MAXF + k0 + min(k, nk - 1)];
    sp[k] = lv_spread(a.nbin[fi[k]]);
  }
  __syncthreads();
  // big nodes hold dense runs of ascending positions: the column-major bins stream
  lv_accumulate<int64_t, LV_FG, 4>(a, wt, a.Xc, fi, n, sp, 1, nk, item_q0[it], item_q1[it], sh);
  __syncthreads();
  for (int k = threadIdx.x >> 6; k < nk; k += 4) lv_collapse(sh[k][0], sh[k][1], sp[k]);
  __syncthreads();
  int64_t* hs = hist + ((int64_t)slot * fs + k0) * 2 * NBINS;
  for (int e = threadIdx.x; e < nk * 2 * NBINS; e += 256) {
    const int64_t v = (&sh[0][0][0])[e];
    if (v != 0) atomicAdd((unsigned long long*)&hs[e], (unsigned long long)v);
  }
}

// one workgroup (4 waves) per big node: totals from the first drawn feature's histogram,
// every drawn feature scanned (wave per feature), strict best in draw order
__global__ __launch_bounds__(256) void lv_big_split_kernel(LvArgs a, const int32_t* __restrict__ blist,
                                                           int nbig, const int16_t* __restrict__ drawn,
                                                           const int32_t* __restrict__ nfo,
                                                           const int64_t* __restrict__ hist,
                                                           int fs) {
  __shared__ double rbest[LV_MAXF];
  __shared__ int rbin[LV_MAXF];
  __shared__ int64_t stot[3];
  const int b = blockIdx.x;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j = blist[b];
  const LNode nd = a.cur[j];
  const int tg = a.fp.t0 + nd.tree;
  const int nf = nfo[b];
  const int kind = a.fp.kind;
  const int64_t* hb = hist + (int64_t)b * fs * 2 * NBINS;
  if (wid == 0) {
    int64_t s0 = 0, s1v = 0;
    for (int e = lane; e < NBINS; e += 64) { s0 += hb[e]; s1v += hb[NBINS + e]; }
    s0 = lv_wsum(s0);
    s1v = lv_wsum(s1v);
    if (lane == 0) {
      // kind 0: channel c = class c weight; kind 1: channel 0 = weight, 1 = sum w r1
      stot[0] = kind == 0 ? s0 + s1v : s0;         // nw
      stot[1] = kind == 0 ? s1v : 0;               // n1
      stot[2] = kind == 0 ? 0 : s1v;               // s1
    }
  }
  __syncthreads();
  const int64_t nw = stot[0], n1 = stot[1], s1 = stot[2];
  const int64_t base = (int64_t)nd.tree * a.cap;
  if (lv_terminal(a.fp, nw, n1, a.depth)) {
    if (threadIdx.x == 0)
      lv_record(a.fp, tg, nd.id, -1, -1, nw, n1, s1, a.feat + base, a.thr + base, a.left + base,
                a.val + base, &a.dec[j]);
    return;
  }
  const int minc = min_child(a.fp, (double)nw);
  for (int k = wid; k < nf; k += 4) {
    double bc;
    int bn;
    lv_scan(hb + (int64_t)k * 2 * NBINS, hb + (int64_t)k * 2 * NBINS + NBINS, kind, nw, n1, s1,
            minc, &bc, &bn);
    if (lane == 0) { rbest[k] = bc; rbin[k] = bn; }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double best = -INFINITY;
    int bf = -1, bb = -1;
    for (int k = 0; k < nf; ++k)
      if (rbin[k] < NBINS && rbest[k] > best) {
        best = rbest[k];
        bf = drawn[(int64_t)b * LV_MAXF + k];
        bb = rbin[k];
      }
    if (!(bf >= 0 && lv_accept(best, lv_parent(kind, nw, n1, s1)))) bf = -1;
    lv_record(a.fp, tg, nd.id, bf, bb, nw, n1, s1, a.feat + base, a.thr + base, a.left + base,
              a.val + base, &a.dec[j]);
  }
}

// ------------------------------------------------------------------ MID nodes
// one workgroup (4 waves) per node with 65 .. t3 rows. Kind 0 (class weights) keeps
// uint32 histograms of 24 features in LDS (48 KB), so mtry <= 24 candidates take ONE pass
// over the node's rows: a row's drawn bins (row-major: its few cache lines) are fetched
// once, not once per feature group (the groups' re-reads were the HBM traffic of the
// deep levels). Kind 1 (int64 sums) takes groups of 8.
template <typename HT, int FG, int U>
__global__ __launch_bounds__(256) void lv_mid_kernel(LvArgs a, const int32_t* __restrict__ mlist) {
  __shared__ HT sh[FG][2][NBINS];
  __shared__ int16_t perm[LV_PMAX];
  __shared__ double rbest[LV_MAXF];
  __shared__ int rbin[LV_MAXF];
  __shared__ int64_t stot[3];
  __shared__ int snf;
  const int j = mlist[blockIdx.x];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const LNode nd = a.cur[j];
  const int tg = a.fp.t0 + nd.tree;
  const int n = a.fp.n, kind = a.fp.kind;
  const int32_t* wt = a.w + (int64_t)nd.tree * n;
  const int64_t base = (int64_t)nd.tree * a.cap;
  if (wid == 0) {
    const int nf = draw_num_features(a.fp, tg, nd.id);
    lv_draw(a.fp, tg, nd.id, nf, perm);
    if (lane == 0) snf = nf;
  }
  __syncthreads();
  const int nf = snf;
  int64_t nw = 0, n1 = 0, s1 = 0;
  int minc = 1;
  for (int k0 = 0; k0 < nf; k0 += FG) {
    const int nk = min(FG, nf - k0);
    for (int e = threadIdx.x; e < FG * 2 * NBINS; e += 256) (&sh[0][0][0])[e] = 0;
    int fi[FG], sp[FG];
#pragma unroll
    for (int k = 0; k < FG; ++k) {
      fi[k] = perm[k0 + min(k, nk - 1)];
      sp[k] = lv_spread(a.nbin[fi[k]]);
    }
    __syncthreads();
    if constexpr (LV_MID_RK && sizeof(HT) == 4 && FG <= 32) {
      const int k = threadIdx.x & 31;
      const int fik = perm[k0 + min(k, nk - 1)];
      lv_accumulate_rk<FG, 8>(a, wt, a.Xb, fik, a.fst, lv_spread(a.nbin[fik]), a.rst, nk,
                              nd.lo, nd.hi, reinterpret_cast<uint32_t (*)[2][NBINS]>(sh));
    } else {
      lv_accumulate<HT, FG, U>(a, wt, a.Xb, fi, a.fst, sp, a.rst, nk, nd.lo, nd.hi, sh);
    }
    __syncthreads();
    for (int k = wid; k < nk; k += 4) lv_collapse(sh[k][0], sh[k][1], sp[k]);
    __syncthreads();
    if (k0 == 0) {
      if (wid == 0) {
        int64_t c0 = 0, c1 = 0;
        for (int e = lane; e < NBINS; e += 64) { c0 += (int64_t)sh[0][0][e]; c1 += (int64_t)sh[0][1][e]; }
        c0 = lv_wsum(c0);
        c1 = lv_wsum(c1);
        if (lane == 0) {
          stot[0] = kind == 0 ? c0 + c1 : c0;
          stot[1] = kind == 0 ? c1 : 0;
          stot[2] = kind == 0 ? 0 : c1;
        }
      }
      __syncthreads();
      nw = stot[0];
      n1 = stot[1];
      s1 = stot[2];
      if (lv_terminal(a.fp, nw, n1, a.depth)) {
        if (threadIdx.x == 0)
          lv_record(a.fp, tg, nd.id, -1, -1, nw, n1, s1, a.feat + base, a.thr + base,
                    a.left + base, a.val + base, &a.dec[j]);
        return;                                             // uniform
      }
      minc = min_child(a.fp, (double)nw);
    }
    for (int k = wid; k < nk; k += 4) {
      double bc;
      int bn;
      lv_scan(&sh[k][0][0], &sh[k][1][0], kind, nw, n1, s1, minc, &bc, &bn);
      if (lane == 0) { rbest[k0 + k] = bc; rbin[k0 + k] = bn; }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double best = -INFINITY;
    int bf = -1, bb = -1;
    for (int k = 0; k < nf; ++k)
      if (rbin[k] < NBINS && rbest[k] > best) { best = rbest[k]; bf = perm[k]; bb = rbin[k]; }
    if (!(bf >= 0 && lv_accept(best, lv_parent(kind, nw, n1, s1)))) bf = -1;
    lv_record(a.fp, tg, nd.id, bf, bb, nw, n1, s1, a.feat + base, a.thr + base, a.left + base,
              a.val + base, &a.dec[j]);
  }
}

// ------------------------------------------------------------------ SMALL nodes
// one wave per node with <= 64 rows: a row per lane, bins of 16 drawn features per batch
// (one memory round trip), <= 16 rows: every present bin is a candidate threshold (same
// sums as a histogram: an absent bin splits like the present bin below it, which wins the
// lowest-bin tie), 17..64 rows: per-wave LDS histogram per feature.
__global__ __launch_bounds__(256) void lv_small_kernel(LvArgs a, const int32_t* __restrict__ slist,
                                                       int nsmall) {
  __shared__ int16_t perm[4][LV_PMAX];
  __shared__ int64_t hist[4][2][NBINS];
  __shared__ uint8_t sbin[4][16][64];                       // [wave][drawn feature][row]
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int s = blockIdx.x * 4 + wid;
  if (s >= nsmall) return;                                  // uniform per wave
  const int j = slist[s];
  const LNode nd = a.cur[j];
  const int tg = a.fp.t0 + nd.tree;
  const int n = a.fp.n, kind = a.fp.kind;
  const int32_t* wt = a.w + (int64_t)nd.tree * n;
  const int64_t base = (int64_t)nd.tree * a.cap;
  const int m = nd.hi - nd.lo;
  const bool valid = lane < m;
  int ci = 0, cy = 0;
  int64_t cw = 0, cr = 0;
  if (valid) {
    ci = a.idx[nd.lo + lane];
    cw = wt[ci];
    if (kind == 0) cy = a.ycls[ci]; else cr = a.r1[ci];
  }
  // channel values of this lane's row: kind 0 -> (class c gets w), kind 1 -> (w, w r1)
  const int64_t v0 = kind == 0 ? (cy ? 0 : cw) : cw;
  const int64_t v1 = kind == 0 ? (cy ? cw : 0) : cw * cr;
  const int64_t t0 = lv_wsum(v0), t1 = lv_wsum(v1);
  const int64_t nw = kind == 0 ? t0 + t1 : t0;
  const int64_t n1 = kind == 0 ? t1 : 0;
  const int64_t s1 = kind == 0 ? 0 : t1;
  if (lv_terminal(a.fp, nw, n1, a.depth)) {
    if (lane == 0)
      lv_record(a.fp, tg, nd.id, -1, -1, nw, n1, s1, a.feat + base, a.thr + base, a.left + base,
                a.val + base, &a.dec[j]);
    return;
  }
  const int minc = min_child(a.fp, (double)nw);
  const int nf = draw_num_features(a.fp, tg, nd.id);
  lv_draw(a.fp, tg, nd.id, nf, perm[wid]);
  double best = -INFINITY;
  int bf = -1, bb = -1;
  for (int k0 = 0; k0 < nf; k0 += 16) {
    // Gather the batch's bins with lanes = (row, feature): one wave instruction covers 4
    // rows x 16 drawn features (those rows' few lines) instead of one feature of 64 rows
    // (64 lines, a byte each), and ceil(m / 4) instructions instead of 16 for m rows; the
    // bins pass through LDS back to a row per lane.
    {
      const int kq = lane & 15, kf = k0 + kq;
      const int64_t fo = kf < nf ? (int64_t)perm[wid][kf] * a.fst : 0;
      for (int r0 = 0; r0 < m; r0 += 4) {                   // uniform: m is the node's
        const int r = r0 + (lane >> 4);
        const int cir = __shfl(ci, r & 63, 64);
        if (r < m && kf < nf) sbin[wid][kq][r] = a.Xb[fo + (int64_t)cir * a.rst];
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);                   // lgkmcnt(0): LDS stores done
      __builtin_amdgcn_wave_barrier();
    }
    int bins[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int k = k0 + u;
      bins[u] = (valid && k < nf) ? (int)sbin[wid][u][lane] : 0;
    }
    __builtin_amdgcn_wave_barrier();                        // reads done before the next batch
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int k = k0 + u;
      if (k >= nf) break;
      const int f = perm[wid][k];
      double lbest = -INFINITY;
      int lbin = NBINS;
      if (m <= 16) {
        const int bme = bins[u];
        int64_t L0 = 0, L1 = 0;
        for (int r = 0; r < m; ++r) {
          const int br = __builtin_amdgcn_readlane(bins[u], r);
          const int64_t a0 = ((int64_t)__builtin_amdgcn_readlane((int)(v0 >> 32), r) << 32) |
                             (uint32_t)__builtin_amdgcn_readlane((int)v0, r);
          const int64_t a1 = ((int64_t)__builtin_amdgcn_readlane((int)(v1 >> 32), r) << 32) |
                             (uint32_t)__builtin_amdgcn_readlane((int)v1, r);
          if (br <= bme) { L0 += a0; L1 += a1; }
        }
        if (valid && bme < NBINS - 1) {
          const double c = lv_crit(kind, L0, L1, nw, n1, s1, minc);
          if (c > lbest) { lbest = c; lbin = bme; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const double oc = __shfl_xor(lbest, o, 64);
          const int ob = __shfl_xor(lbin, o, 64);
          if (oc > lbest || (oc == lbest && ob < lbin)) { lbest = oc; lbin = ob; }
        }
      } else {
        for (int b = lane; b < NBINS; b += 64) { hist[wid][0][b] = 0; hist[wid][1][b] = 0; }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        const int S = lv_spread(a.nbin[f]);
        if (valid) {
          const int slot = bins[u] * S + (lane & (S - 1));
          atomicAdd((unsigned long long*)&hist[wid][0][slot], (unsigned long long)v0);
          atomicAdd((unsigned long long*)&hist[wid][1][slot], (unsigned long long)v1);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        lv_collapse(hist[wid][0], hist[wid][1], S);
        lv_scan(hist[wid][0], hist[wid][1], kind, nw, n1, s1, minc, &lbest, &lbin);
        __builtin_amdgcn_wave_barrier();
      }
      if (lbin < NBINS && lbest > best) { best = lbest; bf = f; bb = lbin; }
    }
  }
  if (!(bf >= 0 && lv_accept(best, lv_parent(kind, nw, n1, s1)))) bf = -1;
  if (lane == 0)
    lv_record(a.fp, tg, nd.id, bf, bb, nw, n1, s1, a.feat + base, a.thr + base, a.left + base,
              a.val + base, &a.dec[j]);
}

// ------------------------------------------------------------------ partition
// one wave per split node of a list (small / mid): stable ballot compaction into idx2.
// Pass 1 gathers the split feature's bins (4 x 64 rows in flight) and keeps each 64-row
// block's left mask in LDS; pass 2 re-reads only the positions and writes both sides.
constexpr int LV_PART_BLK = 8192 / 64;      // mask blocks per wave (mid nodes <= 8192 rows)

__global__ __launch_bounds__(256) void lv_part_wave_kernel(LvArgs a, const int32_t* __restrict__ list,
                                                           int cnt) {
  __shared__ uint64_t masks[4][LV_PART_BLK];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int s = blockIdx.x * 4 + wid;
  if (s >= cnt) return;
  const int j = list[s];
  const int4 d = a.dec[j];
  if (!d.x) return;
  const LNode nd = a.cur[j];
  const uint8_t* xf = a.Xb + (int64_t)d.y * a.fst;
  const int m = nd.hi - nd.lo;
  const int nblk = (m + 63) / 64;
  if (nblk > LV_PART_BLK) {                                 // (not reached: mid <= LV_BIG)
    if (lane == 0) a.nl[j] = -1;
    return;
  }
  const uint64_t below = (1ull << lane) - 1ull;
  int cl = 0;
  for (int b0 = 0; b0 < nblk; b0 += 4) {
    int ii[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = nd.lo + (b0 + u) * 64 + lane;
      ii[u] = q < nd.hi ? a.idx[q] : -1;
    }
    int bv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) bv[u] = ii[u] < 0 ? 0 : xf[(int64_t)ii[u] * a.rst];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (b0 + u >= nblk) break;
      const uint64_t bl = __ballot(ii[u] >= 0 && bv[u] <= d.z);
      if (lane == 0) masks[wid][b0 + u] = bl;
      cl += __popcll(bl);
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_wave_barrier();
  int lb = 0;                                               // lefts before this block
  for (int b = 0; b < nblk; ++b) {
    const int q = nd.lo + b * 64 + lane;
    const uint64_t bl = masks[wid][b];
    if (q < nd.hi) {
      const int i = a.idx[q];
      const bool gl = (bl >> lane) & 1ull;
      const int l = lb + __popcll(bl & below);
      ATE_DASSERT(gl ? l < cl : cl + (b * 64 + lane - l) < m);
      if (gl) a.idx2[nd.lo + l] = i;
      else a.idx2[nd.lo + cl + (b * 64 + lane - l)] = i;
    }
    lb += __popcll(bl);
  }
  if (lane == 0) a.nl[j] = cl;
}

// big split nodes: left count per work item
__global__ __launch_bounds__(256) void lv_part_count_kernel(LvArgs a, const int32_t* __restrict__ item_slot,
                                                            const int32_t* __restrict__ item_q0,
                                                            const int32_t* __restrict__ item_q1,
                                                            const int32_t* __restrict__ blist,
                                                            int32_t* __restrict__ icnt) {
  __shared__ int ws[4];
  const int it = blockIdx.x;
  const int j = blist[item_slot[it]];
  const int4 d = a.dec[j];
  if (!d.x) {
    if (threadIdx.x == 0) icnt[it] = 0;
    return;
  }
  const uint8_t* xf = a.Xc + (int64_t)d.y * a.fp.n;
  int c = 0;
  for (int q = item_q0[it] + threadIdx.x; q < item_q1[it]; q += 256) c += xf[a.idx[q]] <= d.z;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) icnt[it] = ws[0] + ws[1] + ws[2] + ws[3];
}

// big split nodes: stable scatter; ipre = lefts before the item within its node,
// nlb = the node's left total (per big slot)
__global__ __launch_bounds__(256) void lv_part_scatter_kernel(LvArgs a, const int32_t* __restrict__ item_slot,
                                                              const int32_t* __restrict__ item_q0,
                                                              const int32_t* __restrict__ item_q1,
                                                              const int32_t* __restrict__ blist,
                                                              const int32_t* __restrict__ ipre,
                                                              const int32_t* __restrict__ nlb) {
  __shared__ int ws[4];
  const int it = blockIdx.x;
  const int slot = item_slot[it];
  const int j = blist[slot];
  const int4 d = a.dec[j];
  if (!d.x) return;
  const LNode nd = a.cur[j];
  const uint8_t* xf = a.Xc + (int64_t)d.y * a.fp.n;
  const int nlt = nlb[slot];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int run = ipre[it];                                       // lefts before this tile
  const int q1 = item_q1[it];
  for (int t0 = item_q0[it]; t0 < q1; t0 += 256) {
    const int q = t0 + threadIdx.x;
    int i = 0;
    bool gl = false;
    if (q < q1) {
      i = a.idx[q];
      gl = xf[i] <= d.z;
    }
    const uint64_t bl = __ballot(gl);
    const int wl = __popcll(bl);
    if (lane == 0) ws[wid] = wl;
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w2 = 0; w2 < 4; ++w2) {
      if (w2 < wid) off += ws[w2];
      tot += ws[w2];
    }
    const int lb = run + off + __popcll(bl & ((1ull << lane) - 1ull));   // lefts before q
    if (q < q1) {
      ATE_DASSERT(gl ? lb < nlt : nlt + (q - nd.lo - lb) < nd.hi - nd.lo);
      if (gl) a.idx2[nd.lo + lb] = i;
      else a.idx2[nd.lo + nlt + (q - nd.lo - lb)] = i;
    }
    run += tot;
    __syncthreads();
  }
}

// ------------------------------------------------------------------ ids + next level
// first list entry of each tree present in the level: base rank (exclusive split count)
__global__ __launch_bounds__(256) void lv_tree_base_kernel(const LNode* __restrict__ cur, int ncur,
                                                           const int32_t* __restrict__ excl,
                                                           int32_t* __restrict__ brank) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= ncur) return;
  if (j == 0 || cur[j - 1].tree != cur[j].tree) brank[cur[j].tree] = excl[j];
}

__global__ __launch_bounds__(256) void lv_children_kernel(LvArgs a, int ncur,
                                                          const int32_t* __restrict__ excl,
                                                          const int32_t* __restrict__ brank,
                                                          int32_t* __restrict__ next_id,
                                                          LNode* __restrict__ nxt) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= ncur) return;
  const LNode nd = a.cur[j];
  const int4 d = a.dec[j];
  const int t = nd.tree;
  const int r = excl[j] - brank[t];
  const int nid = next_id[t];
  if (d.x) {
    const int lid = nid + 2 * r;
    a.left[(int64_t)t * a.cap + nd.id] = lid;
    const int nlft = a.nl[j];
    ATE_DASSERT(nd.id < a.cap && lid + 1 < a.cap && nlft >= 0 && nlft <= nd.hi - nd.lo);
    nxt[2 * excl[j]] = {t, nd.lo, nd.lo + nlft, lid};
    nxt[2 * excl[j] + 1] = {t, nd.lo + nlft, nd.hi, lid + 1};
  }
}

__global__ __launch_bounds__(256) void lv_next_id_kernel(const LNode* __restrict__ cur, int ncur,
                                                         const int32_t* __restrict__ excl,
                                                         const int4* __restrict__ dec,
                                                         const int32_t* __restrict__ brank,
                                                         int32_t* __restrict__ next_id) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= ncur) return;
  const int t = cur[j].tree;
  if (j == ncur - 1 || cur[j + 1].tree != t) next_id[t] += 2 * (excl[j] + dec[j].x - brank[t]);
}

// ------------------------------------------------------------------ layout copy
// column-major bins [p][n] -> row-major [n][ldr] (ldr % 16 == 0): a workgroup moves a
// 64-feature x 256-row tile through LDS, reading 4-byte words along the rows and writing
// each row's 64 bytes as four aligned 16-byte stores
__global__ __launch_bounds__(256) void lv_transpose_kernel(const uint8_t* __restrict__ src, int p,
                                                           int n, uint8_t* __restrict__ dst,
                                                           int ldr) {
  __shared__ uint8_t tile[64][256 + 4];
  const int f0 = blockIdx.y * 64;
  const int r0 = blockIdx.x * 256;
  const int t = threadIdx.x;
  const bool full = r0 + 256 <= n && (n & 3) == 0;
  for (int fl = t >> 6; fl < 64; fl += 4) {
    const int f = f0 + fl;
    const int c = (t & 63) * 4;                             // row offset within the tile
    uint32_t v = 0;
    if (f < p) {
      const uint8_t* row = src + (int64_t)f * n + r0 + c;
      if (full) {
        v = *reinterpret_cast<const uint32_t*>(row);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (r0 + c + e < n) v |= (uint32_t)row[e] << (8 * e);
      }
    }
    *reinterpret_cast<uint32_t*>(&tile[fl][c]) = v;
  }
  __syncthreads();
  const int r = r0 + t;
  if (r >= n) return;
  uint8_t* out = dst + (int64_t)r * ldr + f0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (f0 + 16 * q >= ldr) break;
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int fl = 16 * q + 4 * e;
      w[e] = (uint32_t)tile[fl][t] | ((uint32_t)tile[fl + 1][t] << 8) |
             ((uint32_t)tile[fl + 2][t] << 16) | ((uint32_t)tile[fl + 3][t] << 24);
    }
    *reinterpret_cast<uint4*>(out + 16 * q) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

}  // namespace

// --------------------------------------------------------------------- host entry points
// The level loop is driven from Python (models/forest_level.py): these entry points launch
// one phase each on `stream`; the host reads the few counts it needs to size the next
// launches (node classes, big-node ranges, the next level's length).
struct LvHost {
  ForestParams fp;
  const void *Xb, *ycls, *r1, *w;
  const void *idx;
  void *idx2, *cur, *dec, *nl;
  int cap;
  void *feat, *thr, *left, *val;
  int depth;
  int64_t fst, rst;
  const void* Xc;
  const void* nbin;
};

static LvArgs lv_args(const LvHost& h) {
  LvArgs a;
  a.fp = h.fp;
  a.Xb = (const uint8_t*)h.Xb;
  a.ycls = (const uint8_t*)h.ycls;
  a.r1 = (const int64_t*)h.r1;
  a.w = (const int32_t*)h.w;
  a.idx = (const int32_t*)h.idx;
  a.idx2 = (int32_t*)h.idx2;
  a.cur = (const LNode*)h.cur;
  a.dec = (int4*)h.dec;
  a.nl = (int32_t*)h.nl;
  a.cap = h.cap;
  a.feat = (int32_t*)h.feat;
  a.thr = (int32_t*)h.thr;
  a.left = (int32_t*)h.left;
  a.val = (double*)h.val;
  a.depth = h.depth;
  a.fst = h.fst;
  a.rst = h.rst;
  a.Xc = (const uint8_t*)h.Xc;
  a.nbin = (const int16_t*)h.nbin;
  return a;
}

ATE_API int ate_lv_boot(const void* fpp, void* w, void* stream) {
  const ForestParams fp = *(const ForestParams*)fpp;
  const int gx = std::min(4096, (fp.n + 255) / 256);
  ATE_LAUNCH(lv_boot_kernel, dim3(gx, fp.ntree), dim3(256), 0, (hipStream_t)stream, fp,
                     (int32_t*)w);
  ATE_CHECK_LAUNCH();
  return 0;
}

// counts[0..3]: class sizes (zeroed by the caller), counts[4]: the level length
ATE_API int ate_lv_classify(const void* cur, int ncur_ub, const void* nsplit, int t2, int t3,
                            void* lists, void* counts, void* stream) {
  if (ncur_ub <= 0) return 0;
  ATE_LAUNCH(lv_classify_kernel, dim3((ncur_ub + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, (const LNode*)cur, ncur_ub, (const int32_t*)nsplit, t2,
                     t3, (int32_t*)lists, (int32_t*)counts);
  ATE_CHECK_LAUNCH();
  return 0;
}

// phase 1: decisions of every node of the level (class lists from ate_lv_classify)
ATE_API int ate_lv_decide(const void* hp, const void* small, int nsmall, const void* mid, int nmid,
                          const void* mid2, int nmid2, const void* big, int nbig, void* drawn,
                          void* nfo, const void* item_slot, const void* item_q0,
                          const void* item_q1, int nitems, int ngroups, void* hist, int fs,
                          void* stream) {
  const LvHost& h = *(const LvHost*)hp;
  if (h.fp.kind > 1 || h.fp.sampling != 0 || h.fp.mtry_poisson || h.fp.p > LV_PMAX ||
      h.fp.mtry > LV_MAXF || fs < h.fp.mtry || ngroups * LV_FG < h.fp.mtry)
    return -1;
  const LvArgs a = lv_args(h);
  hipStream_t st = (hipStream_t)stream;
  if (nsmall)
    ATE_LAUNCH(lv_small_kernel, dim3((nsmall + 3) / 4), dim3(256), 0, st, a,
                       (const int32_t*)small, nsmall);
  for (int c = 0; c < 2; ++c) {
    const int cnt = c == 0 ? nmid : nmid2;
    const int32_t* L = (const int32_t*)(c == 0 ? mid : mid2);
    if (!cnt) continue;
    if (h.fp.kind == 0)
      ATE_LAUNCH((lv_mid_kernel<uint32_t, 24, 1>), dim3(cnt), dim3(256), 0, st, a, L);
    else
      ATE_LAUNCH((lv_mid_kernel<int64_t, LV_FG, 4>), dim3(cnt), dim3(256), 0, st, a, L);
  }
  if (nbig) {
    const int32_t* B = (const int32_t*)big;
    ATE_LAUNCH(lv_big_draw_kernel, dim3((nbig + 3) / 4), dim3(256), 0, st, a, B, nbig,
                       (int16_t*)drawn, (int32_t*)nfo);
    ATE_LAUNCH(lv_big_hist_kernel, dim3(nitems, ngroups), dim3(256), 0, st, a,
                       (const int32_t*)item_slot, (const int32_t*)item_q0,
                       (const int32_t*)item_q1, B, (const int16_t*)drawn, (const int32_t*)nfo,
                       (int64_t*)hist, fs);
    ATE_LAUNCH(lv_big_split_kernel, dim3(nbig), dim3(256), 0, st, a, B, nbig,
                       (const int16_t*)drawn, (const int32_t*)nfo, (const int64_t*)hist, fs);
  }
  ATE_CHECK_LAUNCH();
  return 0;
}

// phase 2a: partition of the wave-partitioned split nodes (two lists), left counts of the
// chunked list's items
ATE_API int ate_lv_partition(const void* hp, const void* l1, int n1, const void* l2, int n2,
                             const void* plist, const void* item_slot, const void* item_q0,
                             const void* item_q1, int nitems, void* icnt, void* stream) {
  const LvHost& h = *(const LvHost*)hp;
  const LvArgs a = lv_args(h);
  hipStream_t st = (hipStream_t)stream;
  if (n1)
    ATE_LAUNCH(lv_part_wave_kernel, dim3((n1 + 3) / 4), dim3(256), 0, st, a,
                       (const int32_t*)l1, n1);
  if (n2)
    ATE_LAUNCH(lv_part_wave_kernel, dim3((n2 + 3) / 4), dim3(256), 0, st, a,
                       (const int32_t*)l2, n2);
  if (nitems)
    ATE_LAUNCH(lv_part_count_kernel, dim3(nitems), dim3(256), 0, st, a,
                       (const int32_t*)item_slot, (const int32_t*)item_q0,
                       (const int32_t*)item_q1, (const int32_t*)plist, (int32_t*)icnt);
  ATE_CHECK_LAUNCH();
  return 0;
}

// phase 2b: stable scatter of the chunked list (ipre / nlb from the item counts)
ATE_API int ate_lv_scatter(const void* hp, const void* plist, const void* item_slot,
                           const void* item_q0, const void* item_q1, int nitems, const void* ipre,
                           const void* nlb, void* stream) {
  const LvHost& h = *(const LvHost*)hp;
  const LvArgs a = lv_args(h);
  if (nitems)
    ATE_LAUNCH(lv_part_scatter_kernel, dim3(nitems), dim3(256), 0, (hipStream_t)stream, a,
                       (const int32_t*)item_slot, (const int32_t*)item_q0,
                       (const int32_t*)item_q1, (const int32_t*)plist, (const int32_t*)ipre,
                       (const int32_t*)nlb);
  ATE_CHECK_LAUNCH();
  return 0;
}

// phase 3: node ids (level order per tree) and the next level's list
ATE_API int ate_lv_children(const void* hp, int ncur, const void* excl, void* brank,
                            void* next_id, void* nxt, void* stream) {
  const LvHost& h = *(const LvHost*)hp;
  const LvArgs a = lv_args(h);
  hipStream_t st = (hipStream_t)stream;
  const int g = (ncur + 255) / 256;
  ATE_LAUNCH(lv_tree_base_kernel, dim3(g), dim3(256), 0, st, a.cur, ncur,
                     (const int32_t*)excl, (int32_t*)brank);
  ATE_LAUNCH(lv_children_kernel, dim3(g), dim3(256), 0, st, a, ncur, (const int32_t*)excl,
                     (const int32_t*)brank, (int32_t*)next_id, (LNode*)nxt);
  ATE_LAUNCH(lv_next_id_kernel, dim3(g), dim3(256), 0, st, a.cur, ncur,
                     (const int32_t*)excl, a.dec, (const int32_t*)brank, (int32_t*)next_id);
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_lv_transpose(const void* src, int p, int n, void* dst, int ldr, void* stream) {
  if (ldr % 16 || ldr < p) return -1;
  dim3 grid((n + 255) / 256, (p + 63) / 64);
  ATE_LAUNCH(lv_transpose_kernel, grid, dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)src, p, n, (uint8_t*)dst, ldr);
  ATE_CHECK_LAUNCH();
  return 0;
}
