// Exact-split forest growth on gfx950 (randomForest split semantics).
// Spec: forest_common.hpp (exact_threshold_bin); host twin: cpu/forest_cpu.cpp
// grow_tree_exact -- both grow the same trees bit for bit.
//
// Bins are uint16 ranks of each feature's distinct values, so a split can fall between ANY
// two consecutive distinct in-node values (the binned engine, csrc/forest.hip, quantises
// to <= 256 bins). Split search walks each candidate feature's rows of the node in value
// order, prefix-summing the integer statistics; the criterion is evaluated at every
// boundary between two distinct values, ties broken by (feature slot, position) as on the
// host.
//
// No node is sorted. The forest's rows are sorted once per feature (host: a stable argsort
// of the value ranks, `order` [p][n]); a tree's root list of feature f is that order
// filtered to its in-bag rows (one wave per feature), and every split stable-partitions each
// feature's list segment into its children's segments of the next level's lists (double-
// buffered [p][mc] entries (value rank, position)), so every node's rows are in value order for every feature
// at all times. Ties between equal values never matter (the criterion is only evaluated
// between distinct values, at the same positions for any order of ties): the trees are the
// same bits as a sort per node and as the host twin.
//
// Decomposition: ONE workgroup (8 waves) per tree, level by level.
//  * nodes of <= WCAP (256) rows are decided and partitioned by ONE WAVE each, without
//    workgroup barriers (node j goes to wave j mod 8): lane l owns list positions
//    [l ch, l ch + ch), ch <= 4; the rows' statistics are gathered by row id, summed by a
//    wave scan, and the partition moves four features' segments per batch; in forests of
//    mtry <= 8, nodes of <= 64 rows hold a row per lane and rank values by lane compares,
//    and lists are not partitioned into children of <= 64 rows (no node reads them);
//  * larger nodes are decided by the whole workgroup, one at a time: per feature a chunk of
//    list positions per thread, a workgroup scan of the chunk sums, an argmax reduction; their
//    partitions run one wave per feature, the rows' sides in an LDS bit per row;
//  * child ids are assigned after the level in list order (a workgroup scan of the split
//    flags), so numbering equals the host engine's.
// randomForest sampling (bootstrap; kinds 0/1, midpoint thresholds) and grf sampling (half-
// samples, honesty, J2 estimation statistics; kinds 1/2, the left value as threshold):
// grf's causal_forest / regression_forest split on exact values (ate_replication.Rmd:250).
// Kind 2 scans the node's pseudo-outcomes rho with the per-position statistic 1 + treated
// * 2^32 (count and treated count in one int64 prefix sum).
#include "common.hpp"
#include "forest_common.hpp"

using namespace atef;

#ifdef EXACT_PROF
// per-phase wall_clock64 ticks of tree 0 (tools/exact_forest_prof.py): [0] setup, [1] big-node
// list, [2] workgroup decisions, [3] wave decisions, [4] ids, [5] workgroup partitions,
// [6] wave partitions, [7] levels, [8..15] per-wave busy ticks in the wave decisions,
// workgroup decisions split: [16] statistics + draws, [17] key fill, [18] sort, [19] walk +
// argmax, [20] threshold, [21] workgroup-level nodes decided
__device__ unsigned long long exact_prof[24];
#define XPROF_T(v) const unsigned long long v = wall_clock64()
#define XPROF_ADD(k, d) do { if (blockIdx.x == 0 && threadIdx.x == 0) exact_prof[k] += (d); } while (0)
#else
#define XPROF_T(v)
#define XPROF_ADD(k, d) do { } while (0)
#endif

namespace {

constexpr int XT = 512;            // threads per tree
constexpr int XW = XT / 64;        // waves per tree
// Two trees per CU: 58 KB of LDS and <= 128 VGPRs per lane (__launch_bounds__ minimum of 4
// waves per SIMD; the compiler spills ~60 VGPRs to scratch) instead of one tree per CU at
// 99 KB / 228 VGPRs. On the tutorial's forests (df_mod, 2500 / 4 x 2000 trees) the many
// trees in flight outweigh the spills and the smaller per-wave node cap: aipw_rf 188 -> 125
// ms, double_ml 294 -> 177 ms, the same trees (profiles/r03_forest_exact/occupancy_ab.txt).
#ifndef EXACT_WCAP
#define EXACT_WCAP 256
#endif
#ifndef EXACT_MINWG
#define EXACT_MINWG 4          // __launch_bounds__ minimum waves per SIMD
#endif
constexpr int WCAP = EXACT_WCAP;   // nodes up to this many rows: one wave each
// Nodes of <= SMALL rows hold a row per lane and rank each candidate feature's values by lane
// compares (no list reads); their children are as small, so the lists of a split whose
// children both have <= SMALL rows are never partitioned (most nodes of a deep tree).
constexpr int SMALL = 64;
// ... for forests of few candidate features per node (randomForest's mtry 4 / 7 at p = 21):
// at grf's mtry (all 21 features) 21 lane-compare rankings per node cost more than reading
// the node's list segments (config 4: 0.70 -> 0.76 s), so grf forests keep the lists
constexpr int SMALL_MTRY = 8;
// one LDS arena: per wave, a wave-level node's partition staging (WCAP row ids); or
// (large-node phases) a bit per row: in-bag rows / rows going left
constexpr int WSLICE = WCAP * 4;   // a wave-level node's partition staging (row ids)
constexpr int XBIG = 65536 / WCAP + 1;     // > WCAP-row nodes of one level (n <= 65536)
constexpr int ARENA = (65536 / 8 > XW * WSLICE) ? 65536 / 8 : XW * WSLICE;
constexpr int XPMAX = 512;         // max features

struct XRng { int lo, hi, id; };
struct XDec { int split, feat, thr, nl; double val; };

// Per-tree scratch. mc = the tree's in-bag (J1) row count bound (host: exact_mcap): every
// per-position array is mc long, so a grf tree (mc = n / 4) needs a quarter of the memory.
struct XScratch {
  int64_t* sx0;     // [mc] per-position statistics of the nodes being decided
  int64_t* sx1;     // [mc]
  int32_t* w;       // [n] bootstrap weights
  int32_t* idx;     // [mc] rows of the growing nodes by position (node = contiguous range)
  uint32_t* keys;   // [max(n, mc)] sampling scratch / partition staging
  XRng* cur;        // [mc + 1]
  XRng* nxt;        // [mc + 1]
  XDec* dec;        // [mc + 1]
  int32_t* est;     // [n] grf J2 (estimation) rows
  uint32_t* La;     // [p][mc] per-feature lists of every node: (value rank << 16) | position,
  uint32_t* Lb;     // [p][mc] in value order; current level's and next level's
  uint8_t* side;    // [mc] by position: 1 = goes left (splitting wave-level nodes)
  uint16_t* npos;   // [mc] by position: the position after the level's partition
};

__host__ __device__ inline int np2(int n) {
  int v = 1;
  while (v < n) v <<= 1;
  return v;
}

__host__ __device__ inline int64_t align16(int64_t b) { return (b + 15) & ~(int64_t)15; }

__host__ __device__ inline int64_t tree_bytes(int n, int p, int mc) {
  return align16(8ll * mc) * 2 + align16(4ll * n) + align16(4ll * mc) +
         align16(4ll * (n > mc ? n : mc)) + align16(12ll * (mc + 1)) * 2 +
         align16((int64_t)sizeof(XDec) * (mc + 1)) + align16(4ll * n) +
         align16(4ll * p * mc) * 2 + align16(mc) + align16(2ll * mc);
}

__device__ XScratch scratch_at(char* base, int n, int np_, int mc) {
  XScratch s;
  char* p = base;
  s.sx0 = (int64_t*)p; p += align16(8ll * mc);
  s.sx1 = (int64_t*)p; p += align16(8ll * mc);
  s.w = (int32_t*)p; p += align16(4ll * n);
  s.idx = (int32_t*)p; p += align16(4ll * mc);
  s.keys = (uint32_t*)p; p += align16(4ll * (n > mc ? n : mc));
  s.cur = (XRng*)p; p += align16(12ll * (mc + 1));
  s.nxt = (XRng*)p; p += align16(12ll * (mc + 1));
  s.dec = (XDec*)p; p += align16((int64_t)sizeof(XDec) * (mc + 1));
  s.est = (int32_t*)p; p += align16(4ll * n);
  s.La = (uint32_t*)p; p += align16(4ll * np_ * mc);
  s.Lb = (uint32_t*)p; p += align16(4ll * np_ * mc);
  s.side = (uint8_t*)p; p += align16(mc);
  s.npos = (uint16_t*)p;
  return s;
}

__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// (crit, pos) argmax with the host's tie-break: larger crit, then smaller position
__device__ __forceinline__ void better(double& c, int& s, double c2, int s2) {
  if (c2 > c || (c2 == c && s2 < s)) { c = c2; s = s2; }
}

__device__ __forceinline__ void wave_argmax(double& c, int& s) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double c2 = __shfl_xor(c, o, 64);
    const int s2 = __shfl_xor(s, o, 64);
    better(c, s, c2, s2);
  }
}

// nw rows (weighted), n1 class-1 weight (kind 0), s1 response / pseudo-outcome sum (kinds 1/2);
// kind 2: ntreat rows above the node's mean treatment, cn the node's causal constants
struct NodeStats { int64_t nw, n1, s1, ntreat; CausalNode cn; };

// leaf value (forest_cpu.cpp grow_tree_exact): majority vote with a Philox coin on ties /
// the node mean of the response
__device__ double leaf_value(const ForestParams& fp, int tg, int v, const NodeStats& st) {
  if (fp.kind == 0) {
    if (2 * st.n1 > st.nw) return 1.0;
    if (2 * st.n1 < st.nw) return 0.0;
    return (double)(rand_u32(fp.seed, P_RF_MTRY, (uint32_t)tg, node_index(v, 4095)) & 1u);
  }
  if (fp.kind == 2) return 0.0;
  return from_fix(st.s1) / (double)st.nw;
}

__device__ bool is_terminal(const ForestParams& fp, const NodeStats& st, int depth) {
  bool terminal = st.nw <= fp.min_node || depth >= MAX_DEPTH - 1;
  if (fp.kind == 0 && (st.n1 == 0 || st.n1 == st.nw)) terminal = true;
  if (fp.kind == 2 && !(st.cn.varw > 0.0)) terminal = true;
  return terminal;
}

// kind-2 node sums of one row (cpu/forest_cpu.cpp grow_tree_exact): W~, Y~, W~^2, W~ Y~
__device__ __forceinline__ void causal_row(const int64_t* r1, const int64_t* r2, int i, int64_t& a,
                                           int64_t& b, int64_t& c, int64_t& d) {
  a = r1[i];
  b = r2[i];
  c = to_fix(from_fix(r1[i]) * from_fix(r1[i]));
  d = to_fix(from_fix(r1[i]) * from_fix(r2[i]));
}

__device__ double parent_crit(const ForestParams& fp, const NodeStats& st) {
  const double dn = (double)st.nw;
  if (fp.kind == 0) {
    const double a = (double)(st.nw - st.n1), b = (double)st.n1;
    return (a * a + b * b) / dn;
  }
  const double sd = from_fix(st.s1);
  return (sd * sd) / dn;
}

// criterion at a boundary with left sums (c0, c1); -inf when a child is too small
__device__ __forceinline__ double boundary_crit(const ForestParams& fp, const NodeStats& st, int minc,
                                                int64_t c0, int64_t c1) {
  const int64_t nl = fp.kind == 0 ? c0 + c1 : (fp.kind == 2 ? (c0 & 0xffffffffll) : c0);
  const int64_t nr = st.nw - nl;
  if (nl < minc || nr < minc) return -INFINITY;
  if (fp.kind == 2) {                  // each child keeps >= 1 treated and >= 1 control row
    const int64_t ct = c0 >> 32, tr = st.ntreat - ct;
    if (ct < minc || nl - ct < minc || tr < minc || nr - tr < minc) return -INFINITY;
  }
  return fp.kind == 0
      ? gini_crit((double)c0, (double)c1, (double)(st.nw - st.n1 - c0), (double)(st.n1 - c1))
      : mse_crit(from_fix(c1), (double)nl, from_fix(st.s1 - c1), (double)nr);
}

// per-row statistics in scan order: kind 0 (w (1-y), w y), kind 1 (w, w r1), kind 2
// (1 + treated 2^32, rho)
__device__ __forceinline__ void row_stats(const ForestParams& fp, const int32_t* w, const uint8_t* ycls,
                                          const int64_t* r1, const int64_t* r2, const CausalNode& cn,
                                          int i, int64_t& a0, int64_t& a1) {
  const int64_t wi = w[i];
  if (fp.kind == 2) {
    a0 = 1 + ((from_fix(r1[i]) >= cn.wbar ? 1ll : 0ll) << 32);
    a1 = to_fix(causal_rho(cn, from_fix(r1[i]), from_fix(r2[i])));
  } else if (fp.kind == 0) {
    const int64_t y = ycls[i];
    a0 = wi * (1 - y);
    a1 = wi * y;
  } else {
    a0 = wi;
    a1 = wi * r1[i];
  }
}

// the node's candidate features: perm[0..nf) after the host's Fisher-Yates draws
__device__ int draw_features(const ForestParams& fp, int tg, int v, int* perm) {
  const int nf = draw_num_features(fp, tg, v);
  for (int k = 0; k < fp.p; ++k) perm[k] = k;
  for (int k = 0; k < nf; ++k) {
    const uint32_t r = rand_below(fp.seed, P_RF_MTRY, (uint32_t)tg, node_index(v, k), (uint32_t)(fp.p - k));
    const int a = perm[k];
    perm[k] = perm[k + r];
    perm[k + r] = a;
  }
  return nf;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// lane dst_lane receives v (ds_permute: a push, a bijection when the lanes' targets are)
__device__ __forceinline__ uint32_t permute_u32(int dst_lane, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_permute(dst_lane << 2, (int)v);
}
__device__ __forceinline__ int64_t permute_i64(int dst_lane, int64_t v) {
  const uint32_t lo = permute_u32(dst_lane, (uint32_t)(uint64_t)v);
  const uint32_t hi = permute_u32(dst_lane, (uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int64_t wave_excl_scan64(int64_t v, int lane) {
  int64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t u = __shfl_up(x, o, 64);
    if (lane >= o) x += u;
  }
  return x - v;
}

// Workgroup exclusive count of `f` over threads (thread order); returns the total.
// scnt: XW ints of LDS. Two barriers.
__device__ __forceinline__ int block_flag_scan(bool f, int* scnt, int& before) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t b = __ballot(f);
  if (lane == 0) scnt[wid] = __popcll(b);
  __syncthreads();
  int off = 0, tot = 0;
  for (int w = 0; w < XW; ++w) {
    if (w < wid) off += scnt[w];
    tot += scnt[w];
  }
  before = off + __popcll(b & ((1ull << lane) - 1ull));
  __syncthreads();
  return tot;
}

// forest_common.hpp::exact_threshold_bin by a whole wave (uniform arguments): the largest
// index t in [blo, bhi) with v[t] <= (v[blo] + v[bhi]) / 2, by a 64-ary search (one memory
// latency per 64x narrowing instead of one per halving).
__device__ int wave_threshold(const double* __restrict__ v, int blo, int bhi, int lane) {
  const double mid = (v[blo] + v[bhi]) / 2.0;
  int lo = blo, hi = bhi;                     // answer in [lo, hi); v[lo] <= mid
  while (hi - lo > 1) {
    const int step = (hi - lo + 63) / 64;
    const int x = lo + lane * step;
    const bool ok = x < hi && v[x] <= mid;
    const uint64_t b = __ballot(ok);           // a prefix of lanes (v is sorted)
    const int L = 63 - __clzll(b);
    lo = lo + L * step;
    hi = min(hi, lo + step);
  }
  return lo;
}

// LANES: the lane-per-row path for nodes of <= SMALL rows (forests of mtry <= SMALL_MTRY); a
// separate instantiation, so the list-only kernel keeps its register allocation
template <bool LANES>
__global__ __launch_bounds__(XT, EXACT_MINWG) void forest_exact_kernel(
    ForestParams fp, int tbeg, int mc, const uint16_t* __restrict__ Xb,
    const uint32_t* __restrict__ order,
    const double* __restrict__ vals,
    int ldv, const int32_t* __restrict__ nval, const uint8_t* __restrict__ ycls,
    const int64_t* __restrict__ r1, const int64_t* __restrict__ r2, int cap,
    int32_t* __restrict__ feat, int32_t* __restrict__ thr, int32_t* __restrict__ left,
    double* __restrict__ val, int32_t* __restrict__ nnodes, uint8_t* __restrict__ inbag,
    int64_t* __restrict__ est_o, char* __restrict__ scratch) {
  // one LDS arena: a slice (WCAP keys + statistics) per wave for the wave-level nodes, or a
  // bit per row in the large-node phases (the phases never overlap)
  __shared__ __attribute__((aligned(16))) char sarena[ARENA];
  __shared__ int64_t sw0[XW], sw1[XW];
  __shared__ int sperm[XW][XPMAX];
  __shared__ double sredc[XW];
  __shared__ int sreds[XW];
  __shared__ int64_t sred64[5][XW];
  __shared__ int scnt[XW + 1];
  __shared__ int sncur, snext_id, sm, snbig, sestn;
  __shared__ int sbig[XBIG];                  // this level's workgroup-level nodes
  __shared__ int swpre[65536 / 32];           // root lists: in-bag rows before each 32-row word
  const int t = tbeg + blockIdx.x;            // tree within this forest
  const int tg = fp.t0 + t;                   // global tree id (RNG key)
  const int n = fp.n, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  XScratch S = scratch_at(scratch + (int64_t)blockIdx.x * tree_bytes(n, fp.p, mc), n, fp.p, mc);
  const int64_t base = (int64_t)t * cap;
  int32_t* tfeat = feat + base;
  int32_t* tthr = thr + base;
  int32_t* tleft = left + base;
  double* tval = val + base;
  uint8_t* inb = inbag + (int64_t)t * n;
  uint32_t* sbits = (uint32_t*)sarena;        // root: a bit per row; large partitions: per position
  const uint64_t below = (1ull << lane) - 1ull;
  auto bit = [&](int i) -> bool { return (sbits[i >> 5] >> (i & 31)) & 1u; };
  char* wsl = sarena + wid * WSLICE;          // this wave's slice: keys, then statistics
  uint32_t* Kw = (uint32_t*)wsl;

  // ---- weights: bootstrap counts (integer atomics: order-free), or grf's samples (Algorithm
  // S, sequential by definition, thread 0; cpu/forest_cpu.cpp draw_rows): the group's
  // half-sample (its rows are the in-bag rows), the tree's subsample, J1 (w = 1) / J2 (est)
  for (int i = tid; i < n; i += XT) S.w[i] = 0;
  __syncthreads();
  if (fp.sampling == 0) {
    for (int j = tid; j < n; j += XT)
      atomicAdd(&S.w[rand_below(fp.seed, P_RF_BOOT, (uint32_t)tg, (uint64_t)j, (uint32_t)n)], 1);
    if (tid == 0) sestn = 0;
  } else if (tid == 0) {
    int32_t* tmp = (int32_t*)S.keys;            // >= n entries, free until the first level
    for (int i = 0; i < n; ++i) inb[i] = 0;
    int ns;
    if (fp.group > 1) {
      const int g = tg / fp.group;
      int nh = 0;
      const int64_t kh = n / 2;
      for (int i = 0; i < n && nh < kh; ++i)
        if (select_next(fp.seed, (uint32_t)g, (uint64_t)i, (int64_t)(n - i), kh - nh)) tmp[nh++] = i;
      for (int q = 0; q < nh; ++q) inb[tmp[q]] = 1;
      double f = fp.sample_fraction * fp.group;
      if (f > 1.0) f = 1.0;
      ns = nh;
      if (f < 1.0) {
        const int64_t ks = (int64_t)floor(nh * f);
        int c = 0;
        for (int q = 0; q < nh && c < ks; ++q)
          if (select_next(fp.seed, 0x10000u + (uint32_t)tg, (uint64_t)q, (int64_t)(nh - q), ks - c))
            tmp[c++] = tmp[q];
        ns = c;
      }
    } else {
      const int64_t ks = (int64_t)floor(n * fp.sample_fraction);
      int c = 0;
      for (int i = 0; i < n && c < ks; ++i)
        if (select_next(fp.seed, 0x10000u + (uint32_t)tg, (uint64_t)i, (int64_t)(n - i), ks - c))
          tmp[c++] = i;
      ns = c;
      for (int q = 0; q < ns; ++q) inb[tmp[q]] = 1;
    }
    int ne = 0;
    if (fp.honesty) {
      const int64_t k1 = ns / 2;
      int c = 0;
      for (int q = 0; q < ns; ++q) {
        const int i = tmp[q];
        if (c < k1 && select_next(fp.seed, 0x20000u + (uint32_t)tg, (uint64_t)q, (int64_t)(ns - q), k1 - c)) {
          S.w[i] = 1;
          ++c;
        } else {
          S.est[ne++] = i;
        }
      }
    } else {
      for (int q = 0; q < ns; ++q) {
        S.w[tmp[q]] = 1;
        S.est[ne++] = tmp[q];
      }
    }
    sestn = ne;
  }
  __syncthreads();
  int m = 0;                                  // uniform running count
  for (int c0 = 0; c0 < n; c0 += XT) {
    const int i = c0 + tid;
    const bool in = i < n && S.w[i] > 0;
    if (i < n && fp.sampling == 0) inb[i] = in;
    const uint64_t b = __ballot(in);
    if (lane == 0) scnt[wid] = __popcll(b);
    __syncthreads();
    int off = m;
    for (int q = 0; q < wid; ++q) off += scnt[q];
    const int at = off + __popcll(b & ((1ull << lane) - 1ull));
    ATE_DASSERT(!in || at < mc);
    if (in && at < mc) S.idx[at] = i;
    int tot = 0;
    for (int q = 0; q < XW; ++q) tot += scnt[q];
    m += tot;
    __syncthreads();
  }
  if (m > mc) {                               // the host's bound is exact; never taken
    if (tid == 0) nnodes[t] = -1;
    return;
  }
  if (tid == 0) {
    S.cur[0] = XRng{0, m, 0};
    sncur = 1;
    snext_id = 1;
  }
  // ---- presorted root lists: feature f's entries (value rank, row) in value order, the
  // forest-wide order filtered to this tree's in-bag rows (a bit per row in LDS) with the row
  // replaced by its position: the rank of the row among the in-bag rows (S.idx is in row
  // order at the root), from per-word prefix popcounts. One wave per feature.
  {
    const int nw32 = (n + 31) / 32;
    for (int e = tid; e < nw32; e += XT) sbits[e] = 0u;
    __syncthreads();
    for (int i = tid; i < n; i += XT)
      if (S.w[i] > 0) atomicOr(&sbits[i >> 5], 1u << (i & 31));
    __syncthreads();
    {                                         // swpre = exclusive prefix of the word counts
      constexpr int WPT = (65536 / 32) / XT;  // words per thread (4)
      int c = 0;
#pragma unroll
      for (int u = 0; u < WPT; ++u) {
        const int e = tid * WPT + u;
        c += e < nw32 ? __popc(sbits[e]) : 0;
      }
      int64_t ex = wave_excl_scan64(c, lane);
      if (lane == 63) sw0[wid] = ex + c;
      __syncthreads();
      for (int q = 0; q < wid; ++q) ex += sw0[q];
      int run = (int)ex;
#pragma unroll
      for (int u = 0; u < WPT; ++u) {
        const int e = tid * WPT + u;
        if (e < nw32) { swpre[e] = run; run += __popc(sbits[e]); }
      }
    }
    __syncthreads();
    for (int f = wid; f < fp.p; f += XW) {
      const uint32_t* of = order + (int64_t)f * n;
      uint32_t* Lf = S.La + (int64_t)f * mc;
      int c = 0;
      for (int c0 = 0; c0 < n; c0 += 64 * 8) {
        uint32_t ev[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int q = c0 + u * 64 + lane;
          ev[u] = q < n ? of[q] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int r = (int)(ev[u] & 0xFFFFu);
          const bool keep = c0 + u * 64 + lane < n && bit(r);
          const uint64_t b = __ballot(keep);
          if (keep) {
            const int pos = swpre[r >> 5] + __popc(sbits[r >> 5] & ((1u << (r & 31)) - 1u));
            Lf[c + __popcll(b & below)] = (ev[u] & 0xFFFF0000u) | (uint32_t)pos;
          }
          c += __popcll(b);
        }
      }
      ATE_DASSERT(c == m);
    }
  }
  __syncthreads();
#ifdef EXACT_PROF
  unsigned long long tp = wall_clock64();
  XPROF_ADD(0, 0ull);
#define XPHASE(k) do { __syncthreads(); const unsigned long long tn_ = wall_clock64(); \
    XPROF_ADD(k, tn_ - tp); tp = tn_; } while (0)
#else
#define XPHASE(k) do { } while (0)
#endif

  for (int depth = 0;; ++depth) {
    const int ncur = sncur;
    if (ncur == 0) break;
    // this level's workgroup-level nodes, in list order
    {
      int nb = 0;
      for (int c0 = 0; c0 < ncur; c0 += XT) {
        const int j = c0 + tid;
        bool big = false;
        if (j < ncur) {
          const XRng nd = S.cur[j];
          big = nd.hi - nd.lo > WCAP;
        }
        int before;
        const int tot = block_flag_scan(big, scnt, before);
        ATE_DASSERT(!big || nb + before < XBIG);
        if (big) sbig[nb + before] = j;
        nb += tot;
      }
      if (tid == 0) snbig = nb;
      __syncthreads();
    }
    const int nbig = snbig;
    XPHASE(1);
    XPROF_ADD(7, 1ull);

    // ================= decisions: nodes > WCAP rows, whole workgroup, one at a time
    for (int jb = 0; jb < nbig; ++jb) {
      const int j = sbig[jb];
      const XRng nd = S.cur[j];
      const int cnt = nd.hi - nd.lo;
      // node statistics (kind 2: n, SW, SY, SWW, SWY -> the node's causal constants)
      int64_t a = 0, b1 = 0, c = 0, d2 = 0, e2 = 0;
      for (int q = nd.lo + tid; q < nd.hi; q += XT) {
        const int i = S.idx[q];
        a += S.w[i];
        if (fp.kind == 0) b1 += (int64_t)S.w[i] * ycls[i];
        else if (fp.kind == 1) c += (int64_t)S.w[i] * r1[i];
        else {
          int64_t x, y, z, u;
          causal_row(r1, r2, i, x, y, z, u);
          b1 += x; c += y; d2 += z; e2 += u;
        }
      }
      a = wave_sum64(a); b1 = wave_sum64(b1); c = wave_sum64(c);
      d2 = wave_sum64(d2); e2 = wave_sum64(e2);
      if (lane == 0) {
        sred64[0][wid] = a; sred64[1][wid] = b1; sred64[2][wid] = c;
        sred64[3][wid] = d2; sred64[4][wid] = e2;
      }
      __syncthreads();
      NodeStats st{0, 0, 0, 0, CausalNode{0, 0, 0, 0}};
      int64_t tot[5] = {0, 0, 0, 0, 0};
      for (int q = 0; q < XW; ++q)
        for (int r = 0; r < 5; ++r) tot[r] += sred64[r][q];
      __syncthreads();                        // sred64 reused below / by the next node
      st.nw = tot[0];
      if (fp.kind == 0) st.n1 = tot[1];
      else if (fp.kind == 1) st.s1 = tot[2];
      else st.cn = causal_node((double)tot[0], tot[1], tot[2], tot[3], tot[4]);
      if (is_terminal(fp, st, depth)) {
        if (tid == 0) S.dec[j] = XDec{0, -1, -1, 0, leaf_value(fp, tg, nd.id, st)};
        continue;
      }
      if (tid == 0) scnt[XW] = draw_features(fp, tg, nd.id, sperm[0]);
      __syncthreads();
#ifdef EXACT_PROF
      unsigned long long tq = wall_clock64();
#define XSUB(k) do { __syncthreads(); const unsigned long long tn_ = wall_clock64(); \
    XPROF_ADD(k, tn_ - tq); tq = tn_; } while (0)
      XPROF_ADD(21, 1ull);
#else
#define XSUB(k) do { } while (0)
#endif
      const int nf = scnt[XW];
      const int minc = min_child(fp, (double)st.nw);
      // per-row statistics once per node (the feature loop gathers them in list order)
      int64_t srho = 0, stre = 0;
      for (int qb = tid; qb < cnt; qb += XT * 8) {
        int iv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) iv[u] = qb + u * XT < cnt ? S.idx[nd.lo + qb + u * XT] : 0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (qb + u * XT < cnt) {
            int64_t x0, x1;
            row_stats(fp, S.w, ycls, r1, r2, st.cn, iv[u], x0, x1);
            S.sx0[nd.lo + qb + u * XT] = x0;      // by position (the list entries carry it)
            S.sx1[nd.lo + qb + u * XT] = x1;
            srho += x1;
            stre += x0 >> 32;
          }
      }
      if (fp.kind == 2) {                     // rho sum and treated count of the node
        srho = wave_sum64(srho); stre = wave_sum64(stre);
        if (lane == 0) { sred64[0][wid] = srho; sred64[1][wid] = stre; }
        __syncthreads();
        st.s1 = 0; st.ntreat = 0;
        for (int q = 0; q < XW; ++q) { st.s1 += sred64[0][q]; st.ntreat += sred64[1][q]; }
      }
      __syncthreads();                        // the statistics are read by other threads
      XSUB(17);
      double best = -INFINITY;                // thread 0's running best over features
      int bf = -1, blo = -1, bhi = -1, bnl = 0;
      // thread tid owns list positions [s0, s1) of the node's segment
      const int ch = (cnt + XT - 1) / XT;
      const int s0 = min(cnt, tid * ch), s1 = min(cnt, s0 + ch);
      for (int k = 0; k < nf; ++k) {
        const int f = sperm[0][k];
        const uint32_t* Lf = S.La + (int64_t)f * mc + nd.lo;   // (rank, position), value order
        int64_t l0 = 0, l1 = 0;
        for (int sb = s0; sb < s1; sb += 8) {
          uint32_t ev[8];
          int64_t a0[8], a1[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) ev[u] = sb + u < s1 ? Lf[sb + u] : 0u;
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            a0[u] = sb + u < s1 ? S.sx0[ev[u] & 0xFFFFu] : 0;
            a1[u] = sb + u < s1 ? S.sx1[ev[u] & 0xFFFFu] : 0;
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) { l0 += a0[u]; l1 += a1[u]; }
        }
        // workgroup exclusive scan of the chunk sums: wave scan + wave totals
        int64_t p0 = wave_excl_scan64(l0, lane), p1 = wave_excl_scan64(l1, lane);
        if (lane == 63) { sw0[wid] = p0 + l0; sw1[wid] = p1 + l1; }
        __syncthreads();
        for (int q = 0; q < wid; ++q) { p0 += sw0[q]; p1 += sw1[q]; }
        double bc = -INFINITY;
        int bs = 0x7FFFFFFF;
        for (int sb = s0; sb < s1; sb += 8) {
          uint32_t ev[9], bv[9];
          int64_t a0[8], a1[8];
#pragma unroll
          for (int u = 0; u < 9; ++u) ev[u] = sb + u < cnt ? Lf[sb + u] : 0u;
#pragma unroll
          for (int u = 0; u < 9; ++u) bv[u] = sb + u < cnt ? ev[u] >> 16 : 0xFFFFFFFFu;
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            a0[u] = sb + u < s1 ? S.sx0[ev[u] & 0xFFFFu] : 0;
            a1[u] = sb + u < s1 ? S.sx1[ev[u] & 0xFFFFu] : 0;
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int s_ = sb + u;
            if (s_ >= s1) break;
            p0 += a0[u]; p1 += a1[u];
            if (s_ + 1 < cnt && bv[u] != bv[u + 1]) {
              const double cr = boundary_crit(fp, st, minc, p0, p1);
              if (cr > bc) { bc = cr; bs = s_; }
            }
          }
        }
        wave_argmax(bc, bs);
        if (lane == 0) { sredc[wid] = bc; sreds[wid] = bs; }
        __syncthreads();
        if (tid == 0) {
          double c2 = sredc[0];
          int s2 = sreds[0];
          for (int q = 1; q < XW; ++q) better(c2, s2, sredc[q], sreds[q]);
          if (c2 > best) {
            best = c2;
            bf = f;
            ATE_DASSERT(s2 >= 0 && s2 + 1 < cnt);
            blo = (int)(Lf[s2] >> 16);
            bhi = (int)(Lf[s2 + 1] >> 16);
            bnl = s2 + 1;
          }
        }
        __syncthreads();                      // sw*, sred* reused by the next feature
        XSUB(19);
      }
      if (tid == 0) {
        const double parent = parent_crit(fp, st);
        if (bf >= 0 && best > parent + 1e-12 * fmax(1.0, fabs(parent)))
          S.dec[j] = XDec{1, bf, fp.sampling == 1 ? blo
                                 : exact_threshold_bin(vals + (int64_t)bf * ldv, nval[bf], blo, bhi),
                          bnl, 0.0};
        else
          S.dec[j] = XDec{0, -1, -1, 0, leaf_value(fp, tg, nd.id, st)};
      }
    }
    __syncthreads();                          // the LDS key buffer changes owners
    XPHASE(2);
#ifdef EXACT_PROF
    const unsigned long long tw0_ = wall_clock64();
#endif

    // ================= decisions: nodes <= WCAP rows, one wave each (round-robin)
    // Lane l owns list positions [l ch, l ch + ch) (ch = ceil(cnt / 64) <= 4) of every
    // feature's value-ordered segment: its rows' statistics are gathered by row id, prefix-
    // summed by a wave scan, and the boundaries between distinct values evaluated in order.
    {
      int* perm = sperm[wid];
      XRng ndn = wid < ncur ? S.cur[wid] : XRng{0, 0, 0};
      for (int j = wid; j < ncur; j += XW) {   // node j -> wave j % XW
        const XRng nd = ndn;
        if (j + XW < ncur) ndn = S.cur[j + XW];   // next node's range, in flight meanwhile
        const int cnt = nd.hi - nd.lo;
        if (cnt > WCAP) continue;
        static_assert(WCAP <= 64 * 4, "four rows per lane");
        int iv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) iv[u] = lane + 64 * u < cnt ? S.idx[nd.lo + lane + 64 * u] : 0;
        NodeStats st{0, 0, 0, 0, CausalNode{0, 0, 0, 0}};
        if (fp.kind == 2) {                   // the node's causal constants first
          int64_t ca = 0, cb = 0, cc = 0, cd = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (lane + 64 * u < cnt) {
              int64_t x, y, z, v2;
              causal_row(r1, r2, iv[u], x, y, z, v2);
              ca += x; cb += y; cc += z; cd += v2;
            }
          st.cn = causal_node((double)cnt, wave_sum64(ca), wave_sum64(cb), wave_sum64(cc),
                              wave_sum64(cd));
        }
        const bool small = LANES && cnt <= SMALL;
        int64_t a = 0, b1 = 0, y0 = 0, y1 = 0;  // y*: the lane's first row (small nodes)
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (lane + 64 * u < cnt) {
            int64_t x0, x1;
            row_stats(fp, S.w, ycls, r1, r2, st.cn, iv[u], x0, x1);
            if (!small) {
              S.sx0[nd.lo + lane + 64 * u] = x0;  // by position (the list entries carry it)
              S.sx1[nd.lo + lane + 64 * u] = x1;
            }
            if (u == 0) { y0 = x0; y1 = x1; }
            a += x0; b1 += x1;
          }
        a = wave_sum64(a); b1 = wave_sum64(b1);
        if (fp.kind == 0) { st.nw = a + b1; st.n1 = b1; st.s1 = 0; }
        else if (fp.kind == 1) { st.nw = a; st.n1 = 0; st.s1 = b1; }
        else { st.nw = a & 0xffffffffll; st.ntreat = a >> 32; st.s1 = b1; }
        if (is_terminal(fp, st, depth)) {
          if (lane == 0) S.dec[j] = XDec{0, -1, -1, 0, leaf_value(fp, tg, nd.id, st)};
          continue;
        }
        int nf = 0;
        if (lane == 0) nf = draw_features(fp, tg, nd.id, perm);
        nf = __shfl(nf, 0, 64);
        // the statistics stores (global) and perm (LDS) before any lane's gathers
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int minc = min_child(fp, (double)st.nw);
        const int ch = (cnt + 63) / 64;
        const int s0 = min(cnt, lane * ch), s1 = min(cnt, s0 + ch);
        double best = -INFINITY;
        int bf = -1, blo = -1, bhi = -1, bnl = 0;
        // a row per lane: each feature's value ranks by lane compares, the rows' statistics
        // moved to their ranks (ds_permute) and prefix-summed; the boundaries between distinct
        // values are the list positions' boundaries, so the decision is the same
        const bool live = lane < cnt;
        constexpr int PF = 4;                  // bins of up to 4 features fetched together
        uint32_t bins[PF];
        for (int k = 0; LANES && small && k < nf; ++k) {
          const int f = perm[k];
          if ((k % PF) == 0) {
#pragma unroll
            for (int u = 0; u < PF; ++u)
              bins[u] = (live && k + u < nf) ? (uint32_t)Xb[(int64_t)perm[k + u] * n + iv[0]] : 0u;
          }
          uint32_t bk = bins[0];
#pragma unroll
          for (int u = 1; u < PF; ++u) bk = (k % PF) == u ? bins[u] : bk;
          // idle lanes rank last with distinct keys (ranks cnt..63: the permute is a bijection)
          const uint32_t key = live ? ((bk << 16) | (uint32_t)lane) : (0xFFFF0000u | (uint32_t)lane);
          int rank = 0;
          for (int q = 0; q < 64; ++q) rank += (uint32_t)__builtin_amdgcn_readlane((int)key, q) < key;
          const uint32_t ks = permute_u32(rank, key);
          int64_t c0 = permute_i64(rank, y0), c1 = permute_i64(rank, y1);
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            const int64_t u0 = __shfl_up(c0, o, 64), u1 = __shfl_up(c1, o, 64);
            if (lane >= o) { c0 += u0; c1 += u1; }
          }
          const uint32_t kn = __shfl_down(ks, 1, 64);
          double cr = -INFINITY;
          int s = 0x7FFFFFFF;
          if (lane + 1 < cnt && (ks >> 16) != (kn >> 16)) {
            cr = boundary_crit(fp, st, minc, c0, c1);
            s = lane;
          }
          wave_argmax(cr, s);
          if (cr > best) {                      // uniform
            best = cr;
            bf = f;
            blo = (int)(__shfl(ks, s, 64) >> 16);
            bhi = (int)(__shfl(kn, s, 64) >> 16);
            bnl = s + 1;
          }
        }
        for (int k = 0; !small && k < nf; ++k) {
          const int f = perm[k];
          const uint32_t* Lf = S.La + (int64_t)f * mc + nd.lo;
          uint32_t ev[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) ev[u] = s0 + u < s1 ? Lf[s0 + u] : 0u;
          uint32_t bv[4];
          int64_t a0[4], a1[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const bool in = s0 + u < s1;
            bv[u] = in ? ev[u] >> 16 : 0xFFFFFFFFu;
            a0[u] = in ? S.sx0[ev[u] & 0xFFFFu] : 0;
            a1[u] = in ? S.sx1[ev[u] & 0xFFFFu] : 0;
          }
          int64_t l0 = 0, l1 = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u) { l0 += a0[u]; l1 += a1[u]; }
          int64_t p0 = wave_excl_scan64(l0, lane), p1 = wave_excl_scan64(l1, lane);
          // the value after this lane's last position: the next lane's first (lane 63 ends
          // at cnt, where no boundary is evaluated)
          const uint32_t bnext = (uint32_t)__shfl_down((int)bv[0], 1, 64);
          double bc = -INFINITY;
          int bs = 0x7FFFFFFF;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int s_ = s0 + u;
            if (s_ >= s1) break;
            p0 += a0[u]; p1 += a1[u];
            const uint32_t bn = s_ + 1 < s1 ? bv[u + 1 < 4 ? u + 1 : 3] : bnext;
            if (s_ + 1 < cnt && bv[u] != bn) {
              const double cr = boundary_crit(fp, st, minc, p0, p1);
              if (cr > bc) { bc = cr; bs = s_; }
            }
          }
          wave_argmax(bc, bs);
          if (bc > best) {                    // uniform
            best = bc;
            bf = f;
            // the bins at positions bs and bs + 1, from the lanes that hold them
            const int o0 = bs / ch, u0 = bs - o0 * ch;
            const int o1 = (bs + 1) / ch, u1 = bs + 1 - o1 * ch;
            uint32_t m0 = bv[0], m1 = bv[0];
#pragma unroll
            for (int u = 1; u < 4; ++u) { if (u == u0) m0 = bv[u]; if (u == u1) m1 = bv[u]; }
            blo = __builtin_amdgcn_readlane((int)m0, o0);
            bhi = __builtin_amdgcn_readlane((int)m1, o1);
            bnl = bs + 1;
          }
        }
        const double parent = parent_crit(fp, st);
        const bool split = bf >= 0 && best > parent + 1e-12 * fmax(1.0, fabs(parent));
        const int tb = !split ? -1 : fp.sampling == 1 ? blo
                              : wave_threshold(vals + (int64_t)bf * ldv, blo, bhi, lane);
        if (lane == 0)
          S.dec[j] = split ? XDec{1, bf, tb, bnl, 0.0}
                           : XDec{0, -1, -1, 0, leaf_value(fp, tg, nd.id, st)};
      }
    }
#ifdef EXACT_PROF
    if (blockIdx.x == 0 && lane == 0) exact_prof[8 + wid] += wall_clock64() - tw0_;
#endif
    __syncthreads();
    XPHASE(3);

    // ================= child ids in list order (host numbering), node arrays
    {
      const int nid0 = snext_id;
      int ns = 0;                             // split nodes before this chunk (uniform)
      for (int c0 = 0; c0 < ncur; c0 += XT) {
        const int j = c0 + tid;
        XRng nd{0, 0, 0};
        XDec d{0, -1, -1, 0, 0.0};
        if (j < ncur) { nd = S.cur[j]; d = S.dec[j]; }
        int before;
        const int tot = block_flag_scan(j < ncur && d.split, scnt, before);
        if (j < ncur) {
          if (!d.split) {
            tfeat[nd.id] = -1; tthr[nd.id] = -1; tleft[nd.id] = -1; tval[nd.id] = d.val;
          } else {
            const int k = ns + before, nid = nid0 + 2 * k;
            ATE_DASSERT(nd.id < 2 * n + 1 && nid + 1 < 2 * n + 1 && d.nl >= 0 &&
                        d.nl <= nd.hi - nd.lo && 2 * k + 1 <= n);
            tfeat[nd.id] = d.feat; tthr[nd.id] = d.thr; tleft[nd.id] = nid; tval[nd.id] = 0.0;
            S.nxt[2 * k] = XRng{nd.lo, nd.lo + d.nl, nid};
            S.nxt[2 * k + 1] = XRng{nd.lo + d.nl, nd.hi, nid + 1};
          }
        }
        ns += tot;
      }
      if (tid == 0) {
        snext_id = nid0 + 2 * ns;
        sm = 2 * ns;
      }
      __syncthreads();
    }
    XPHASE(4);

    // ================= stable partitions by bin <= thr
    // S.idx (rows by position) is partitioned in place per node; every position's side and
    // new position are recorded, then each feature's entries (rank, position) move to their
    // children's segments of the next level's lists with the position renumbered.
    for (int jb = 0; jb < nbig; ++jb) {       // large nodes: whole workgroup
      const int j = sbig[jb];
      const XRng nd = S.cur[j];
      const int cnt = nd.hi - nd.lo;
      const XDec d = S.dec[j];
      if (!d.split) continue;
      const uint16_t* xf = Xb + (int64_t)d.feat * n;
      int lo_l = 0, lo_r = d.nl;              // uniform running offsets
      for (int c0 = 0; c0 < cnt; c0 += XT) {
        const int q = c0 + tid;
        const bool in = q < cnt;
        const int i = in ? S.idx[nd.lo + q] : 0;
        const bool l = in && xf[i] <= d.thr;
        const uint64_t bl = __ballot(l), br = __ballot(in && !l);
        if (lane == 0) { scnt[wid] = __popcll(bl); sreds[wid] = __popcll(br); }
        __syncthreads();
        int ol = lo_l, orr = lo_r, tl = 0, tr = 0;
        for (int w = 0; w < XW; ++w) {
          if (w < wid) { ol += scnt[w]; orr += sreds[w]; }
          tl += scnt[w]; tr += sreds[w];
        }
        ATE_DASSERT(!in || (l ? ol + __popcll(bl & below) < d.nl
                             : orr + __popcll(br & below) < cnt));
        if (in) {
          const int dest = nd.lo + (l ? ol + __popcll(bl & below) : orr + __popcll(br & below));
          S.keys[dest] = (uint32_t)i;
          S.npos[nd.lo + q] = (uint16_t)dest;
          // the position's side (a bit per position of this node in LDS)
          const int pq = nd.lo + q;
          if (l) atomicOr(&sbits[pq >> 5], 1u << (pq & 31));
          else atomicAnd(&sbits[pq >> 5], ~(1u << (pq & 31)));
        }
        lo_l += tl; lo_r += tr;
        __syncthreads();
      }
      for (int q = tid; q < cnt; q += XT) S.idx[nd.lo + q] = (int32_t)S.keys[nd.lo + q];
      __syncthreads();
      // every feature's value-ordered entries, stable-partitioned into the children's segments
      // of the next level's lists (one wave per feature)
      for (int f = wid; f < fp.p; f += XW) {
        const uint32_t* src = S.La + (int64_t)f * mc + nd.lo;
        uint32_t* dst = S.Lb + (int64_t)f * mc + nd.lo;
        int ol = 0, orr = d.nl;
        for (int c0 = 0; c0 < cnt; c0 += 64 * 8) {
          uint32_t ev[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int q = c0 + u * 64 + lane;
            ev[u] = q < cnt ? src[q] : 0u;
          }
          uint16_t np[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) np[u] = c0 + u * 64 + lane < cnt ? S.npos[ev[u] & 0xFFFFu] : 0;
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const bool in = c0 + u * 64 + lane < cnt;
            const bool l = in && bit((int)(ev[u] & 0xFFFFu));
            const uint64_t bl = __ballot(l), br = __ballot(in && !l);
            if (in)
              dst[l ? ol + __popcll(bl & below) : orr + __popcll(br & below)] =
                  (ev[u] & 0xFFFF0000u) | (uint32_t)np[u];
            ol += __popcll(bl);
            orr += __popcll(br);
          }
        }
        ATE_DASSERT(ol == d.nl && orr == cnt);
      }
      __syncthreads();
    }
    XPHASE(5);
    {                                          // wave-level nodes, staged in the wave's LDS
      for (int j = wid; j < ncur; j += XW) {
        const XRng nd = S.cur[j];
        const int cnt = nd.hi - nd.lo;
        if (cnt > WCAP) continue;
        const XDec d = S.dec[j];
        if (!d.split) continue;
        const uint16_t* xf = Xb + (int64_t)d.feat * n;
        // children of <= SMALL rows never read their lists
        const bool lists = !LANES || d.nl > SMALL || cnt - d.nl > SMALL;
        int lo_l = 0, lo_r = d.nl;
        for (int c0 = 0; c0 < cnt; c0 += 64) {
          const int q = c0 + lane;
          const bool in = q < cnt;
          const int i = in ? S.idx[nd.lo + q] : 0;
          const bool l = in && xf[i] <= d.thr;
          const uint64_t bl = __ballot(l), br = __ballot(in && !l);
          if (in) {
            const int dl = l ? lo_l + __popcll(bl & below) : lo_r + __popcll(br & below);
            Kw[dl] = (uint32_t)i;
            if (lists) {
              S.side[nd.lo + q] = l ? 1 : 0;
              S.npos[nd.lo + q] = (uint16_t)(nd.lo + dl);
            }
          }
          lo_l += __popcll(bl);
          lo_r += __popcll(br);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        for (int q = lane; q < cnt; q += 64) S.idx[nd.lo + q] = (int32_t)Kw[q];
        if (!lists) {
          wave_sync();
          continue;
        }
        // every feature's value-ordered segment into its children's segments of the next
        // level's lists (four features per batch: their loads in flight together)
        for (int f0 = 0; f0 < fp.p; f0 += 4) {
          uint32_t ev[4][4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int q = u * 64 + lane;
              ev[e][u] = (f0 + e < fp.p && q < cnt) ? S.La[(int64_t)(f0 + e) * mc + nd.lo + q] : 0u;
            }
          uint8_t sv[4][4];
          uint16_t np[4][4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const bool ok = f0 + e < fp.p && u * 64 + lane < cnt;
              sv[e][u] = ok ? S.side[ev[e][u] & 0xFFFFu] : 0;
              np[e][u] = ok ? S.npos[ev[e][u] & 0xFFFFu] : 0;
            }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (f0 + e >= fp.p) break;
            uint32_t* dst = S.Lb + (int64_t)(f0 + e) * mc + nd.lo;
            int ol = 0, orr = d.nl;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const bool in = u * 64 + lane < cnt;
              const bool l = in && sv[e][u];
              const uint64_t bl = __ballot(l), br = __ballot(in && !l);
              if (in)
                dst[l ? ol + __popcll(bl & below) : orr + __popcll(br & below)] =
                    (ev[e][u] & 0xFFFF0000u) | (uint32_t)np[e][u];
              ol += __popcll(bl);
              orr += __popcll(br);
            }
            ATE_DASSERT(ol == d.nl && orr == cnt);
          }
        }
        wave_sync();
      }
    }
    __syncthreads();
    XPHASE(6);
    if (tid == 0) sncur = sm;
    {                                         // the children list becomes the current list
      XRng* tmp = S.cur;
      S.cur = S.nxt;
      S.nxt = tmp;
      uint32_t* tl = S.La;                    // ... and the partitioned lists the current
      S.La = S.Lb;
      S.Lb = tl;
    }
    __syncthreads();
  }
  if (tid == 0) nnodes[t] = snext_id;
  // ---- grf: estimation statistics of every node from the J2 (honest) rows (order-free
  // int64 atomics; cpu/forest_cpu.cpp fill_est)
  if (fp.sampling == 1 && est_o) {
    __syncthreads();
    const int nn = snext_id;
    int64_t* est = est_o + base * 5;
    for (int e = tid; e < nn * 5; e += XT) est[e] = 0;
    __syncthreads();
    const int ne = sestn;
    for (int q = tid; q < ne; q += XT) {
      const int i = S.est[q];
      int v = 0;
      while (true) {
        ATE_DASSERT(v >= 0 && v < nn);
        int64_t* e = est + (int64_t)v * 5;
        atomicAdd((unsigned long long*)&e[0], 1ull);
        if (fp.kind == 1) {
          atomicAdd((unsigned long long*)&e[1], (unsigned long long)r1[i]);
        } else {
          int64_t x, y, z, u;
          causal_row(r1, r2, i, x, y, z, u);
          atomicAdd((unsigned long long*)&e[1], (unsigned long long)x);
          atomicAdd((unsigned long long*)&e[2], (unsigned long long)y);
          atomicAdd((unsigned long long*)&e[3], (unsigned long long)z);
          atomicAdd((unsigned long long*)&e[4], (unsigned long long)u);
        }
        if (tfeat[v] < 0) break;
        v = Xb[(int64_t)tfeat[v] * n + i] <= tthr[v] ? tleft[v] : tleft[v] + 1;
      }
    }
  }
}

}  // namespace

ATE_KERNEL_SHAPE("forest_exact_kernel<lane>", XT, 0, forest_exact_kernel<true>)
ATE_KERNEL_SHAPE("forest_exact_kernel<lists>", XT, 0, forest_exact_kernel<false>)

ATE_API int64_t ate_forest_exact_scratch_bytes(int n, int p, int mc, int ntree) {
  return tree_bytes(n, p, mc) * (int64_t)ntree;
}

// Grow trees [tbeg, tbeg + ntree_chunk) of the forest (scratch: ntree_chunk trees).
// grf sampling (fp.sampling == 1, kinds 1/2) needs est ([ntree * cap][5] int64).
ATE_API int ate_forest_fit_exact(const void* fpp, int tbeg, int nchunk, int mc, const void* Xb,
                                 const void* order, const void* vals, int ldv, const void* nval, const void* ycls,
                                 const void* r1, const void* r2, int cap, void* feat, void* thr,
                                 void* left, void* val, void* nnodes, void* inbag, void* est,
                                 void* scratch, void* stream) {
  const ForestParams fp = *(const ForestParams*)fpp;
  if (fp.p > XPMAX || fp.n <= 0 || fp.n > 65536) return -1;
  if (fp.sampling == 0 ? fp.kind == 2 : (fp.kind == 0 || !est || (fp.kind == 2 && !r2))) return -1;
  if (tbeg < 0 || nchunk < 1 || tbeg + nchunk > fp.ntree) return -1;
  if (mc < 1 || mc > fp.n) return -1;
  auto kern = fp.mtry <= SMALL_MTRY ? forest_exact_kernel<true> : forest_exact_kernel<false>;
  ATE_LAUNCH(kern, dim3(nchunk), dim3(XT), 0, (hipStream_t)stream, fp, tbeg,
                     mc, (const uint16_t*)Xb, (const uint32_t*)order, (const double*)vals, ldv, (const int32_t*)nval,
                     (const uint8_t*)ycls, (const int64_t*)r1, (const int64_t*)r2, cap,
                     (int32_t*)feat, (int32_t*)thr, (int32_t*)left, (double*)val, (int32_t*)nnodes,
                     (uint8_t*)inbag, (int64_t*)est, (char*)scratch);
  ATE_CHECK_LAUNCH();
  return 0;
}

#ifdef EXACT_PROF
extern "C" __attribute__((visibility("default"))) int ate_exact_prof_read(void* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(exact_prof), sizeof(exact_prof));
}
extern "C" __attribute__((visibility("default"))) int ate_exact_prof_reset() {
  static unsigned long long z[24];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(exact_prof), z, sizeof(z));
}
#endif
