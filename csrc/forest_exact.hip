// Exact-split forest growth on gfx950 (randomForest split semantics).
// Spec: forest_common.hpp (exact_threshold_bin); host twin: cpu/forest_cpu.cpp
// grow_tree_exact -- both grow the same trees bit for bit.
//
// Bins are uint16 ranks of each feature's distinct values, so a split can fall between ANY
// two consecutive distinct in-node values (the binned engine, csrc/forest.hip, quantises
// to <= 256 bins). Split search is sort-based instead of histogram-based: a node's rows
// are sorted by (bin, position) for each candidate feature and the integer statistics are
// prefix-summed in that order; the criterion is evaluated at every boundary between two
// distinct values, ties broken by (feature slot, position) as on the host.
//
// Decomposition: ONE workgroup (4 waves) per tree, level by level.
//  * nodes of <= 64 rows are decided and partitioned by ONE WAVE each (the 4 waves take
//    them round-robin): a row per lane, ranks by 64 lane compares, the sorted order built
//    with ds_permute (no LDS round trip), prefix sums by lane shuffles;
//  * larger nodes are decided by the whole workgroup, one at a time: a bitonic sort of the
//    32-bit keys in LDS (<= 8192 rows) or in the tree's global scratch (larger nodes),
//    chunked prefix sums with a workgroup scan, an argmax reduction;
//  * child ids are assigned after the level in list order (thread 0), so numbering
//    equals the host engine's.
// Only randomForest sampling (bootstrap) and kinds 0/1 (classification, regression).
#include "common.hpp"
#include "forest_common.hpp"

using namespace atef;

namespace {

constexpr int XT = 256;            // threads per tree
constexpr int XW = XT / 64;        // waves per tree
constexpr int XLDS = 8192;         // node keys sorted in LDS up to this many rows
constexpr int XPMAX = 512;         // max features

struct XRng { int lo, hi, id; };
struct XDec { int split, feat, thr, nl; double val; };

struct XScratch {
  int32_t* w;       // [n] bootstrap weights
  int32_t* idx;     // [n] rows of the growing nodes (node = contiguous range)
  uint32_t* keys;   // [np2] global sort keys / partition staging
  XRng* cur;        // [n + 1]
  XRng* nxt;        // [n + 1]
  XDec* dec;        // [n + 1]
};

__host__ __device__ inline int np2(int n) {
  int v = 1;
  while (v < n) v <<= 1;
  return v;
}

__host__ __device__ inline int64_t align16(int64_t b) { return (b + 15) & ~(int64_t)15; }

__host__ __device__ inline int64_t tree_bytes(int n) {
  return align16(4ll * n) * 2 + align16(4ll * np2(n)) + align16(12ll * (n + 1)) * 2 +
         align16((int64_t)sizeof(XDec) * (n + 1));
}

__device__ XScratch scratch_at(char* base, int n) {
  XScratch s;
  char* p = base;
  s.w = (int32_t*)p; p += align16(4ll * n);
  s.idx = (int32_t*)p; p += align16(4ll * n);
  s.keys = (uint32_t*)p; p += align16(4ll * np2(n));
  s.cur = (XRng*)p; p += align16(12ll * (n + 1));
  s.nxt = (XRng*)p; p += align16(12ll * (n + 1));
  s.dec = (XDec*)p;
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

__device__ __forceinline__ uint32_t permute_u32(int dst_lane, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_permute(dst_lane << 2, (int)v);
}
__device__ __forceinline__ int64_t permute_i64(int dst_lane, int64_t v) {
  const uint32_t lo = permute_u32(dst_lane, (uint32_t)(uint64_t)v);
  const uint32_t hi = permute_u32(dst_lane, (uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

struct NodeStats { int64_t nw, n1, s1; };

// leaf value (forest_cpu.cpp grow_tree_exact): majority vote with a Philox coin on ties /
// the node mean of the response
__device__ double leaf_value(const ForestParams& fp, int tg, int v, const NodeStats& st) {
  if (fp.kind == 0) {
    if (2 * st.n1 > st.nw) return 1.0;
    if (2 * st.n1 < st.nw) return 0.0;
    return (double)(rand_u32(fp.seed, P_RF_MTRY, (uint32_t)tg, node_index(v, 4095)) & 1u);
  }
  return from_fix(st.s1) / (double)st.nw;
}

__device__ bool is_terminal(const ForestParams& fp, const NodeStats& st, int depth) {
  bool terminal = st.nw <= fp.min_node || depth >= MAX_DEPTH - 1;
  if (fp.kind == 0 && (st.n1 == 0 || st.n1 == st.nw)) terminal = true;
  return terminal;
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
  const int64_t nl = fp.kind == 0 ? c0 + c1 : c0;
  const int64_t nr = st.nw - nl;
  if (nl < minc || nr < minc) return -INFINITY;
  return fp.kind == 0
      ? gini_crit((double)c0, (double)c1, (double)(st.nw - st.n1 - c0), (double)(st.n1 - c1))
      : mse_crit(from_fix(c1), (double)nl, from_fix(st.s1 - c1), (double)nr);
}

// per-row statistics in scan order: kind 0 (w (1-y), w y), kind 1 (w, w r1)
__device__ __forceinline__ void row_stats(const ForestParams& fp, const int32_t* w, const uint8_t* ycls,
                                          const int64_t* r1, int i, int64_t& a0, int64_t& a1) {
  const int64_t wi = w[i];
  if (fp.kind == 0) {
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

__global__ __launch_bounds__(XT) void forest_exact_kernel(
    ForestParams fp, int tbeg, const uint16_t* __restrict__ Xb, const double* __restrict__ vals,
    int ldv, const int32_t* __restrict__ nval, const uint8_t* __restrict__ ycls,
    const int64_t* __restrict__ r1, int cap, int32_t* __restrict__ feat, int32_t* __restrict__ thr,
    int32_t* __restrict__ left, double* __restrict__ val, int32_t* __restrict__ nnodes,
    uint8_t* __restrict__ inbag, char* __restrict__ scratch) {
  __shared__ uint32_t skeys[XLDS];
  __shared__ int64_t sc0[XT], sc1[XT];
  __shared__ int sperm[XW][XPMAX];
  __shared__ double sredc[XW];
  __shared__ int sreds[XW];
  __shared__ int64_t sred64[3][XW];
  __shared__ int scnt[XW + 1];
  __shared__ int sncur, snext_id, sm;
  const int t = tbeg + blockIdx.x;            // tree within this forest
  const int tg = fp.t0 + t;                   // global tree id (RNG key)
  const int n = fp.n, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  XScratch S = scratch_at(scratch + (int64_t)blockIdx.x * tree_bytes(n), n);
  const int64_t base = (int64_t)t * cap;
  int32_t* tfeat = feat + base;
  int32_t* tthr = thr + base;
  int32_t* tleft = left + base;
  double* tval = val + base;
  uint8_t* inb = inbag + (int64_t)t * n;

  // ---- bootstrap weights (integer atomics: order-free), in-bag mask, row list
  for (int i = tid; i < n; i += XT) S.w[i] = 0;
  __syncthreads();
  for (int j = tid; j < n; j += XT)
    atomicAdd(&S.w[rand_below(fp.seed, P_RF_BOOT, (uint32_t)tg, (uint64_t)j, (uint32_t)n)], 1);
  __syncthreads();
  int m = 0;                                  // uniform running count
  for (int c0 = 0; c0 < n; c0 += XT) {
    const int i = c0 + tid;
    const bool in = i < n && S.w[i] > 0;
    if (i < n) inb[i] = in;
    const uint64_t b = __ballot(in);
    if (lane == 0) scnt[wid] = __popcll(b);
    __syncthreads();
    int off = m;
    for (int q = 0; q < wid; ++q) off += scnt[q];
    if (in) S.idx[off + __popcll(b & ((1ull << lane) - 1ull))] = i;
    int tot = 0;
    for (int q = 0; q < XW; ++q) tot += scnt[q];
    m += tot;
    __syncthreads();
  }
  if (tid == 0) {
    S.cur[0] = XRng{0, m, 0};
    sncur = 1;
    snext_id = 1;
  }
  __syncthreads();

  for (int depth = 0;; ++depth) {
    const int ncur = sncur;
    if (ncur == 0) break;

    // ================= decisions: nodes > 64 rows, whole workgroup, one at a time
    for (int j = 0; j < ncur; ++j) {
      const XRng nd = S.cur[j];
      const int cnt = nd.hi - nd.lo;
      if (cnt <= 64) continue;
      // node statistics
      int64_t a = 0, b1 = 0, c = 0;
      for (int q = nd.lo + tid; q < nd.hi; q += XT) {
        const int i = S.idx[q];
        a += S.w[i];
        if (fp.kind == 0) b1 += (int64_t)S.w[i] * ycls[i];
        else c += (int64_t)S.w[i] * r1[i];
      }
      a = wave_sum64(a); b1 = wave_sum64(b1); c = wave_sum64(c);
      if (lane == 0) { sred64[0][wid] = a; sred64[1][wid] = b1; sred64[2][wid] = c; }
      __syncthreads();
      NodeStats st{0, 0, 0};
      for (int q = 0; q < XW; ++q) {
        st.nw += sred64[0][q]; st.n1 += sred64[1][q]; st.s1 += sred64[2][q];
      }
      __syncthreads();                        // sred64 reused by the next node
      if (is_terminal(fp, st, depth)) {
        if (tid == 0) S.dec[j] = XDec{0, -1, -1, 0, leaf_value(fp, tg, nd.id, st)};
        continue;
      }
      if (tid == 0) scnt[XW] = draw_features(fp, tg, nd.id, sperm[0]);
      __syncthreads();
      const int nf = scnt[XW];
      const int minc = min_child(fp, (double)st.nw);
      const int N2 = np2(cnt);
      uint32_t* K = N2 <= XLDS ? skeys : S.keys;
      double best = -INFINITY;                // thread 0's running best over features
      int bf = -1, blo = -1, bhi = -1, bnl = 0;
      for (int k = 0; k < nf; ++k) {
        const int f = sperm[0][k];
        const uint16_t* xf = Xb + (int64_t)f * n;
        for (int s = tid; s < N2; s += XT)
          K[s] = s < cnt ? (((uint32_t)xf[S.idx[nd.lo + s]] << 16) | (uint32_t)s) : 0xFFFFFFFFu;
        __syncthreads();
        // bitonic sort, ascending
        for (int kk = 2; kk <= N2; kk <<= 1)
          for (int jj = kk >> 1; jj > 0; jj >>= 1) {
            for (int s = tid; s < N2; s += XT) {
              const int o = s ^ jj;
              if (o > s) {
                const uint32_t x = K[s], y = K[o];
                const bool up = (s & kk) == 0;
                if ((x > y) == up) { K[s] = y; K[o] = x; }
              }
            }
            __syncthreads();
          }
        // chunked prefix sums: thread tid owns positions [s0, s1)
        const int ch = (cnt + XT - 1) / XT;
        const int s0 = min(cnt, tid * ch), s1 = min(cnt, s0 + ch);
        int64_t l0 = 0, l1 = 0;
        for (int s = s0; s < s1; ++s) {
          int64_t x0, x1;
          row_stats(fp, S.w, ycls, r1, S.idx[nd.lo + (int)(K[s] & 0xFFFFu)], x0, x1);
          l0 += x0; l1 += x1;
        }
        sc0[tid] = l0; sc1[tid] = l1;
        __syncthreads();
        int64_t p0 = 0, p1 = 0;
        for (int q = 0; q < tid; ++q) { p0 += sc0[q]; p1 += sc1[q]; }
        double bc = -INFINITY;
        int bs = 0x7FFFFFFF;
        for (int s = s0; s < s1; ++s) {
          int64_t x0, x1;
          row_stats(fp, S.w, ycls, r1, S.idx[nd.lo + (int)(K[s] & 0xFFFFu)], x0, x1);
          p0 += x0; p1 += x1;
          if (s + 1 < cnt && (K[s] >> 16) != (K[s + 1] >> 16)) {
            const double cr = boundary_crit(fp, st, minc, p0, p1);
            if (cr > bc) { bc = cr; bs = s; }
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
            blo = (int)(K[s2] >> 16);
            bhi = (int)(K[s2 + 1] >> 16);
            bnl = s2 + 1;
          }
        }
        __syncthreads();                      // K, sc*, sred* reused by the next feature
      }
      if (tid == 0) {
        const double parent = parent_crit(fp, st);
        if (bf >= 0 && best > parent + 1e-12 * fmax(1.0, fabs(parent)))
          S.dec[j] = XDec{1, bf, exact_threshold_bin(vals + (int64_t)bf * ldv, nval[bf], blo, bhi),
                          bnl, 0.0};
        else
          S.dec[j] = XDec{0, -1, -1, 0, leaf_value(fp, tg, nd.id, st)};
      }
    }

    // ================= decisions: nodes <= 64 rows, one wave each
    {
      int r = 0;                              // rank among small nodes (uniform)
      int* perm = sperm[wid];
      for (int j = 0; j < ncur; ++j) {
        const XRng nd = S.cur[j];
        const int cnt = nd.hi - nd.lo;
        if (cnt > 64) continue;
        if ((r++ % XW) != wid) continue;
        const bool live = lane < cnt;
        const int i = live ? S.idx[nd.lo + lane] : 0;
        int64_t x0 = 0, x1 = 0;
        if (live) row_stats(fp, S.w, ycls, r1, i, x0, x1);
        NodeStats st;
        if (fp.kind == 0) {
          st.nw = wave_sum64(x0 + x1);
          st.n1 = wave_sum64(x1);
          st.s1 = 0;
        } else {
          st.nw = wave_sum64(x0);
          st.n1 = 0;
          st.s1 = wave_sum64(x1);
        }
        if (is_terminal(fp, st, depth)) {
          if (lane == 0) S.dec[j] = XDec{0, -1, -1, 0, leaf_value(fp, tg, nd.id, st)};
          continue;
        }
        int nf = 0;
        if (lane == 0) nf = draw_features(fp, tg, nd.id, perm);
        nf = __shfl(nf, 0, 64);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int minc = min_child(fp, (double)st.nw);
        double best = -INFINITY;
        int bf = -1, blo = -1, bhi = -1, bnl = 0;
        for (int k = 0; k < nf; ++k) {
          const int f = perm[k];
          // idle lanes sort last with distinct keys (ranks cnt..63, so ds_permute is a bijection)
          const uint32_t key = live ? (((uint32_t)Xb[(int64_t)f * n + i] << 16) | (uint32_t)lane)
                                    : (0xFFFF0000u | (uint32_t)lane);
          int rank = 0;
          for (int q = 0; q < 64; ++q) rank += (uint32_t)__builtin_amdgcn_readlane((int)key, q) < key;
          // lane s receives the key and statistics of the row ranked s
          const uint32_t ks = permute_u32(rank, key);
          int64_t c0 = permute_i64(rank, x0), c1 = permute_i64(rank, x1);
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
          if (cr > best) {                    // uniform
            best = cr;
            bf = f;
            blo = (int)(__shfl(ks, s, 64) >> 16);
            bhi = (int)(__shfl(kn, s, 64) >> 16);
            bnl = s + 1;
          }
        }
        const double parent = parent_crit(fp, st);
        if (lane == 0) {
          if (bf >= 0 && best > parent + 1e-12 * fmax(1.0, fabs(parent)))
            S.dec[j] = XDec{1, bf, exact_threshold_bin(vals + (int64_t)bf * ldv, nval[bf], blo, bhi),
                            bnl, 0.0};
          else
            S.dec[j] = XDec{0, -1, -1, 0, leaf_value(fp, tg, nd.id, st)};
        }
      }
    }
    __syncthreads();

    // ================= child ids in list order (host numbering), node arrays
    if (tid == 0) {
      int nid = snext_id, nn = 0;
      for (int j = 0; j < ncur; ++j) {
        const XRng nd = S.cur[j];
        const XDec d = S.dec[j];
        if (!d.split) {
          tfeat[nd.id] = -1; tthr[nd.id] = -1; tleft[nd.id] = -1; tval[nd.id] = d.val;
          continue;
        }
        tfeat[nd.id] = d.feat; tthr[nd.id] = d.thr; tleft[nd.id] = nid; tval[nd.id] = 0.0;
        S.nxt[nn++] = XRng{nd.lo, nd.lo + d.nl, nid};
        S.nxt[nn++] = XRng{nd.lo + d.nl, nd.hi, nid + 1};
        nid += 2;
      }
      snext_id = nid;
      sm = nn;
    }
    __syncthreads();

    // ================= stable partitions by bin <= thr
    for (int j = 0; j < ncur; ++j) {          // large nodes: whole workgroup
      const XRng nd = S.cur[j];
      const int cnt = nd.hi - nd.lo;
      if (cnt <= 64) continue;
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
        const uint64_t below = (1ull << lane) - 1ull;
        if (in) S.keys[nd.lo + (l ? ol + __popcll(bl & below) : orr + __popcll(br & below))] = (uint32_t)i;
        lo_l += tl; lo_r += tr;
        __syncthreads();
      }
      for (int q = tid; q < cnt; q += XT) S.idx[nd.lo + q] = (int32_t)S.keys[nd.lo + q];
      __syncthreads();
    }
    {                                          // small nodes: one wave each, in registers
      int r = 0;
      for (int j = 0; j < ncur; ++j) {
        const XRng nd = S.cur[j];
        const int cnt = nd.hi - nd.lo;
        if (cnt > 64) continue;
        if ((r++ % XW) != wid) continue;
        const XDec d = S.dec[j];
        if (!d.split) continue;
        const bool in = lane < cnt;
        const int i = in ? S.idx[nd.lo + lane] : 0;
        const bool l = in && Xb[(int64_t)d.feat * n + i] <= d.thr;
        const uint64_t bl = __ballot(l), br = __ballot(in && !l);
        const uint64_t below = (1ull << lane) - 1ull;
        if (in) S.idx[nd.lo + (l ? __popcll(bl & below) : d.nl + __popcll(br & below))] = i;
      }
    }
    __syncthreads();
    if (tid == 0) sncur = sm;
    // next level reads the children list: swap the roles of cur / nxt
    {
      XRng* tmp = S.cur;
      S.cur = S.nxt;
      S.nxt = tmp;
    }
    __syncthreads();
  }
  if (tid == 0) nnodes[t] = snext_id;
}

}  // namespace

ATE_API int64_t ate_forest_exact_scratch_bytes(int n, int ntree) {
  return tree_bytes(n) * (int64_t)ntree;
}

// Grow trees [tbeg, tbeg + ntree_chunk) of the forest (scratch: ntree_chunk trees).
ATE_API int ate_forest_fit_exact(const void* fpp, int tbeg, int nchunk, const void* Xb,
                                 const void* vals, int ldv, const void* nval, const void* ycls,
                                 const void* r1, int cap, void* feat, void* thr, void* left,
                                 void* val, void* nnodes, void* inbag, void* scratch, void* stream) {
  const ForestParams fp = *(const ForestParams*)fpp;
  if (fp.p > XPMAX || fp.n <= 0 || fp.n > 65536 || fp.sampling != 0 || fp.kind == 2) return -1;
  if (tbeg < 0 || nchunk < 1 || tbeg + nchunk > fp.ntree) return -1;
  hipLaunchKernelGGL(forest_exact_kernel, dim3(nchunk), dim3(XT), 0, (hipStream_t)stream, fp, tbeg,
                     (const uint16_t*)Xb, (const double*)vals, ldv, (const int32_t*)nval,
                     (const uint8_t*)ycls, (const int64_t*)r1, cap, (int32_t*)feat, (int32_t*)thr,
                     (int32_t*)left, (double*)val, (int32_t*)nnodes, (uint8_t*)inbag,
                     (char*)scratch);
  ATE_CHECK_LAUNCH();
  return 0;
}
