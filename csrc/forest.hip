// K10-K15 forest engine on gfx950 (spec and CPU twin: forest_common.hpp, cpu/forest_cpu.cpp).
//
// K10 bootstrap_counts / grf half-sampling, K11 (binning is done by bin_kernel below),
// K12 hist_build (LDS int64 histograms, ds_add_u64), K13 split_search (wave prefix scan +
// argmax with (feature slot, bin) tie-break), K14 partition (stable ballot compaction),
// K15 forest_predict (row x tree traversal, OOB masks), K16/K17 causal pseudo-outcomes
// and leaf sufficient statistics.
//
// Decomposition: ONE workgroup of NW waves grows ONE tree level by level (trees are
// independent: tree parallelism across CUs; NW = 4..16 so that a launch of few trees still
// keeps ~16 waves per CU busy, see ate_forest_fit). Within a level the NW waves take nodes
// round-robin; a node's decision is made by one wave. Child ids are assigned after the
// level by a scan in list order, so node numbering equals the CPU reference.
#include "common.hpp"
#include "forest_common.hpp"

using namespace atef;

constexpr int PMAX_F = 512;   // max features for the per-wave permutation buffer
// nodes above 256 * NW rows are decided by all NW waves together (COOP_CAP per chunk of
// candidates; the rest by one wave per node)
constexpr int COOP_CAP = 256;
// bins gathered per batch in the 17-64-row histogram path (register pressure: 16 -> ~60
// more VGPRs and one wave fewer per SIMD)
constexpr int SMALL_B = 4;

#ifdef FOREST_PROF
// per tree (debug builds, tools/forest_profile.py): [0] decisions, [1] child ids,
// [2] partition (wall_clock64 ticks, thread 0 at the level barriers), [3] levels,
// [4] nodes, [5] nodes <= 16 rows, [6] nodes <= 64 rows, [7] setup (sampling, rows)
__device__ unsigned long long forest_prof[1024][8];
#define FPROF_T(var) const unsigned long long var = wall_clock64()
#define FPROF_ADD(k, v) do { if (threadIdx.x == 0) atomicAdd(&forest_prof[t & 1023][k], (unsigned long long)(v)); } while (0)
#else
#define FPROF_T(var)
#define FPROF_ADD(k, v) do { } while (0)
#endif

namespace {

struct Rng3 { int lo, hi, id; };

__device__ __forceinline__ int64_t wsum64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

struct Scratch {
  int32_t* w;       // [n] weights of growing rows
  int32_t* idx;     // [n]
  int32_t* tmp;     // [n]
  int64_t* rho;     // [n] causal pseudo-outcomes (fixed point)
  Rng3* cur;        // [n+1]
  Rng3* nxt;        // [n+1]
  int4* dec;        // [n+1] per level node: (split flag, feat, bin, left rows)
  int32_t* est_rows;// [n]
};

__device__ Scratch scratch_for(char* base, int n, int t) {
  // per-tree region; layout must match forest_scratch_bytes()
  const int64_t nn = n + 1;
  const int64_t bytes = nn * (4 + 4 + 4 + 8 + 12 + 12 + 16 + 4) + 64;
  char* p = base + (int64_t)t * ((bytes + 255) / 256 * 256);
  Scratch s;
  s.rho = (int64_t*)p;            p += nn * 8;
  s.dec = (int4*)p;               p += nn * 16;
  s.w = (int32_t*)p;              p += nn * 4;
  s.idx = (int32_t*)p;            p += nn * 4;
  s.tmp = (int32_t*)p;            p += nn * 4;
  s.cur = (Rng3*)p;               p += nn * 12;
  s.nxt = (Rng3*)p;               p += nn * 12;
  s.est_rows = (int32_t*)p;
  return s;
}

}  // namespace

ATE_API int64_t ate_forest_scratch_bytes(int n, int ntree) {
  const int64_t nn = n + 1;
  const int64_t bytes = nn * (4 + 4 + 4 + 8 + 12 + 12 + 16 + 4) + 64;
  return (bytes + 255) / 256 * 256 * (int64_t)ntree;
}

// block-wide exclusive scan of one int per thread (NW waves); returns total via *tot
template <int NW>
__device__ int block_scan_excl(int v, int* sh /*>= NW*/, int* tot) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[wid] = x;
  __syncthreads();
  int off = 0;
  for (int k = 0; k < wid; ++k) off += sh[k];
  int total = 0;
#pragma unroll
  for (int k = 0; k < NW; ++k) total += sh[k];
  __syncthreads();
  *tot = total;
  return off + x - v;
}

// NW waves per workgroup (one tree); MINW = waves per SIMD the register allocation must
// allow (4: <= 128 VGPRs with some scratch spill, 3: <= 168)
template <int NW, int MINW>
__global__ __launch_bounds__(64 * NW, MINW) void forest_grow_kernel(
    ForestParams fp, const uint8_t* __restrict__ Xb, const uint8_t* __restrict__ ycls,
    const int64_t* __restrict__ r1, const int64_t* __restrict__ r2, int cap,
    int32_t* __restrict__ feat_o, int32_t* __restrict__ thr_o, int32_t* __restrict__ left_o,
    double* __restrict__ val_o, int32_t* __restrict__ nnodes, uint8_t* __restrict__ inbag,
    int64_t* __restrict__ est_o, char* __restrict__ scratch_base) {
  // LDS: per wave histogram (256 bins x 4 int64 = 8 KB) + feature permutation
  constexpr int NT = 64 * NW;
  constexpr int COOP_ROWS = 256 * NW;
  __shared__ int64_t hist[NW][4][NBINS];
  __shared__ int16_t perm[NW][PMAX_F];
  __shared__ int shi[NW];
  __shared__ int64_t sred[NW][8];         // cooperative nodes: per-wave partial sums
  __shared__ int sbig[COOP_CAP];          // this chunk's nodes with > COOP_ROWS rows
  __shared__ int sncur, snext_id, sm, sestn;
  const int t = blockIdx.x;
  const int tg = fp.t0 + t;          // global tree id (RNG key)
  const int n = fp.n, p = fp.p;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  Scratch S = scratch_for(scratch_base, n, t);
  uint8_t* inb = inbag + (int64_t)t * n;
  FPROF_T(tstart_);
  // ------------------------------------------------------------ sampling (K10)
  for (int i = tid; i < n; i += NT) S.w[i] = 0;
  __syncthreads();
  if (fp.sampling == 0) {
    for (int j = tid; j < n; j += NT)
      atomicAdd(&S.w[rand_below(fp.seed, P_RF_BOOT, (uint32_t)tg, (uint64_t)j, (uint32_t)n)], 1);
    __syncthreads();
    for (int i = tid; i < n; i += NT) inb[i] = S.w[i] > 0;
    if (tid == 0) sestn = 0;
  } else if (tid == 0) {
    // Algorithm S (sequential by definition): group half-sample H (group > 1), tree
    // subsample S, honesty split J1 (grow) / J2 (estimate). tmp holds H, then S; est_rows
    // holds J2. group == 1 (grf ci.group.size = 1): S drawn from all rows directly.
    // Spec: cpu/forest_cpu.cpp draw_rows.
    for (int i = 0; i < n; ++i) inb[i] = 0;
    int ns;
    if (fp.group > 1) {
      const int g = tg / fp.group;
      int nh = 0;
      const int64_t kh = n / 2;
      for (int i = 0; i < n && nh < kh; ++i)
        if (select_next(fp.seed, (uint32_t)g, (uint64_t)i, (int64_t)(n - i), kh - nh)) S.tmp[nh++] = i;
      for (int q = 0; q < nh; ++q) inb[S.tmp[q]] = 1;
      double f = fp.sample_fraction * fp.group;
      if (f > 1.0) f = 1.0;
      ns = nh;
      if (f < 1.0) {
        const int64_t ks = (int64_t)floor(nh * f);
        int c = 0;
        for (int q = 0; q < nh && c < ks; ++q)
          if (select_next(fp.seed, 0x10000u + (uint32_t)tg, (uint64_t)q, (int64_t)(nh - q), ks - c))
            S.tmp[c++] = S.tmp[q];
        ns = c;
      }
    } else {
      const int64_t ks = (int64_t)floor(n * fp.sample_fraction);
      int c = 0;
      for (int i = 0; i < n && c < ks; ++i)
        if (select_next(fp.seed, 0x10000u + (uint32_t)tg, (uint64_t)i, (int64_t)(n - i), ks - c))
          S.tmp[c++] = i;
      ns = c;
      for (int q = 0; q < ns; ++q) inb[S.tmp[q]] = 1;
    }
    int ne = 0;
    if (fp.honesty) {
      const int64_t k1 = ns / 2;
      int c = 0;
      for (int q = 0; q < ns; ++q) {
        const int i = S.tmp[q];
        if (c < k1 && select_next(fp.seed, 0x20000u + (uint32_t)tg, (uint64_t)q, (int64_t)(ns - q), k1 - c)) {
          S.w[i] = 1;
          ++c;
        } else {
          S.est_rows[ne++] = i;
        }
      }
    } else {
      for (int q = 0; q < ns; ++q) {
        S.w[S.tmp[q]] = 1;
        S.est_rows[ne++] = S.tmp[q];
      }
    }
    sestn = ne;
  }
  __syncthreads();
  // ------------------------------------------------------------ in-bag rows, ascending
  int m = 0;
  for (int base = 0; base < n; base += NT) {
    const int i = base + tid;
    const int f = (i < n && S.w[i] > 0) ? 1 : 0;
    int tot;
    const int pos = block_scan_excl<NW>(f, shi, &tot);
    ATE_DASSERT(!f || m + pos < n);
    if (f) S.idx[m + pos] = i;
    m += tot;
  }
  const int64_t obase = (int64_t)t * cap;
  int32_t* feat = feat_o + obase;
  int32_t* thr = thr_o + obase;
  int32_t* left = left_o + obase;
  double* val = val_o + obase;
  if (tid == 0) {
    S.cur[0] = {0, m, 0};
    sncur = 1;
    snext_id = 1;
  }
  __syncthreads();
  // ------------------------------------------------------------ levels
  FPROF_T(tsetup_);
  FPROF_ADD(7, tsetup_ - tstart_);
  for (int depth = 0;; ++depth) {
    const int ncur = sncur;
    if (ncur == 0) break;
    FPROF_T(tl0_);
    FPROF_ADD(3, 1);
    FPROF_ADD(4, ncur);
    // ---- decisions: one wave per node
    // Nodes with <= 64 rows (most nodes of a fully grown tree) keep their rows' index,
    // weight, label / outcome and pseudo-outcome in registers (one row per lane) and
    // fetch the bins of all drawn features in batches of 16 independent loads, so a node
    // costs a few memory round trips instead of two per feature. Larger nodes stream
    // their rows per feature. Both paths add the same values to the same histograms.
    // Nodes with more than COOP_ROWS rows (the top levels) are decided by all four waves
    // together: rows split over the waves, integer sums combined through LDS in wave
    // order, every wave evaluates the same combined histogram (identical decisions).
    auto decide = [&](int j, bool coop) {
      const Rng3 nd = S.cur[j];
      const int v = nd.id;
      const bool small = !coop && nd.hi - nd.lo <= 64;
      const int q0 = nd.lo + lane + (coop ? wid * 64 : 0);
      const int qstep = coop ? NT : 64;
      // sum over the node's rows: one wave, or all four (fixed wave order)
      auto red = [&](int64_t x, int slot) -> int64_t {
        x = wsum64(x);
        if (!coop) return x;
        if (lane == 0) sred[wid][slot] = x;
        __syncthreads();
        int64_t r = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) r += sred[w][slot];
        __syncthreads();
        return r;
      };
      const int qs = nd.lo + lane;
      const bool cvalid = small && qs < nd.hi;
      int ci = 0, cy = 0;
      int64_t cw = 0, cr1 = 0, cr2 = 0, crho = 0;
      if (cvalid) {
        ci = S.idx[qs];
        cw = S.w[ci];
        if (fp.kind == 0) cy = ycls[ci];
        else { cr1 = r1[ci]; if (fp.kind == 2) cr2 = r2[ci]; }
      }
      int64_t nw = 0, n1 = 0, s1 = 0, sw = 0, sy = 0, sww = 0, swy = 0;
      for (int q = q0; q < nd.hi; q += qstep) {   // small: one pass, cached values
        int64_t wi, a1 = 0, a2 = 0;
        int yi = 0;
        if (small) {
          wi = cw; yi = cy; a1 = cr1; a2 = cr2;
        } else {
          const int i = S.idx[q];
          wi = S.w[i];
          if (fp.kind == 0) yi = ycls[i];
          else { a1 = r1[i]; if (fp.kind == 2) a2 = r2[i]; }
        }
        nw += wi;
        if (fp.kind == 0) n1 += wi * yi;
        else if (fp.kind == 1) s1 += wi * a1;
        else {
          sw += a1;
          sy += a2;
          sww += to_fix(__dmul_rn(from_fix(a1), from_fix(a1)));
          swy += to_fix(__dmul_rn(from_fix(a1), from_fix(a2)));
        }
      }
      nw = red(nw, 0); n1 = red(n1, 1); s1 = red(s1, 2);
      sw = red(sw, 3); sy = red(sy, 4); sww = red(sww, 5); swy = red(swy, 6);
      const double dn = (double)nw;
      bool terminal = nw <= fp.min_node || depth >= MAX_DEPTH - 1;
      if (fp.kind == 0 && (n1 == 0 || n1 == nw)) terminal = true;
      CausalNode cn{0, 0, 0, 0};
      if (fp.kind == 2) {
        cn = causal_node(dn, sw, sy, sww, swy);
        if (!(cn.varw > 0.0)) terminal = true;
      }
      int bf = -1, bb = -1;
      if (!terminal) {
        int64_t stot = 0;
        if (fp.kind == 2) {
          if (small) {
            if (cvalid) crho = to_fix(causal_rho(cn, from_fix(cr1), from_fix(cr2)));
            stot = crho;
          } else {
            for (int q = q0; q < nd.hi; q += qstep) {
              const int i = S.idx[q];
              const int64_t rv = to_fix(causal_rho(cn, from_fix(r1[i]), from_fix(r2[i])));
              S.rho[i] = rv;
              stot += rv;
            }
          }
          stot = small ? wsum64(stot) : red(stot, 7);
        } else if (fp.kind == 1) {
          stot = s1;
        }
        double parent;
        if (fp.kind == 0) {
          const double a = (double)(nw - n1), b = (double)n1;
          parent = __ddiv_rn(__dadd_rn(__dmul_rn(a, a), __dmul_rn(b, b)), dn);
        } else {
          const double sd = from_fix(stot);
          parent = __ddiv_rn(__dmul_rn(sd, sd), dn);
        }
        const int minc = min_child(fp, dn);
        const int nf = draw_num_features(fp, tg, v);
        // partial Fisher-Yates: draws k < 64 in parallel (lane k), swaps in order by lane 0
        for (int k = lane; k < p; k += 64) perm[wid][k] = (int16_t)k;
        const uint32_t rk = lane < nf ? rand_below(fp.seed, P_RF_MTRY, (uint32_t)tg,
                                                   node_index(v, lane), (uint32_t)(p - lane)) : 0u;
        __builtin_amdgcn_s_waitcnt(0xC07F);
        if (lane == 0) {
          for (int k = 0; k < nf; ++k) {
            const uint32_t r = k < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)rk, k)
                                      : rand_below(fp.seed, P_RF_MTRY, (uint32_t)tg,
                                                   node_index(v, k), (uint32_t)(p - k));
            const int16_t tmpv = perm[wid][k];
            perm[wid][k] = perm[wid][k + r];
            perm[wid][k + r] = tmpv;
          }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        double best = -INFINITY;
        int64_t ntreat = 0;
        auto hist_row = [&](int b, int64_t wi, int yi, int64_t a1, int64_t rho) {
          ATE_DASSERT(b >= 0 && b < NBINS);          // LDS histogram slot
          if (fp.kind == 0) {
            if (yi) atomicAdd((unsigned long long*)&hist[wid][1][b], (unsigned long long)wi);
            else atomicAdd((unsigned long long*)&hist[wid][0][b], (unsigned long long)wi);
          } else if (fp.kind == 1) {
            atomicAdd((unsigned long long*)&hist[wid][0][b], (unsigned long long)wi);
            atomicAdd((unsigned long long*)&hist[wid][2][b], (unsigned long long)(wi * a1));
          } else {
            atomicAdd((unsigned long long*)&hist[wid][0][b], 1ull);
            atomicAdd((unsigned long long*)&hist[wid][2][b], (unsigned long long)rho);
            if (from_fix(a1) >= cn.wbar) atomicAdd((unsigned long long*)&hist[wid][3][b], 1ull);
          }
        };
        // per feature: clear, accumulate (by the caller), scan, evaluate, argmax
        auto clear_hist = [&]() {
          for (int b = lane; b < NBINS; b += 64) {
            hist[wid][0][b] = 0; hist[wid][1][b] = 0; hist[wid][2][b] = 0; hist[wid][3][b] = 0;
          }
          __builtin_amdgcn_s_waitcnt(0xC07F);
        };
        // split criterion of "bin <= b" from the left-side sums; -inf when not admissible
        auto crit_at = [&](int64_t L0, int64_t L1, int64_t LS, int64_t LT) -> double {
          const int64_t nl = fp.kind == 0 ? L0 + L1 : L0;
          const int64_t nr = nw - nl;
          if (nl < minc || nr < minc) return -INFINITY;
          if (fp.kind == 0)
            return gini_crit((double)L0, (double)L1, (double)(nw - n1 - L0), (double)(n1 - L1));
          if (fp.kind == 2) {
            const int64_t tr = ntreat - LT;
            if (LT < minc || nl - LT < minc || tr < minc || nr - tr < minc) return -INFINITY;
          }
          return mse_crit(from_fix(LS), (double)nl, from_fix(stot - LS), (double)nr);
        };
        // wave argmax (max crit, then lowest bin), then the strict cross-feature update
        auto take_best = [&](double lbest, int lbin, int f) {
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) {
            const double oc = __shfl_xor(lbest, o, 64);
            const int ob = __shfl_xor(lbin, o, 64);
            if (oc > lbest || (oc == lbest && ob < lbin)) { lbest = oc; lbin = ob; }
          }
          if (lbin < NBINS && lbest > best) { best = lbest; bf = f; bb = lbin; }
        };
        auto scan_eval = [&](int f) {
          __builtin_amdgcn_s_waitcnt(0xC07F);
          // wave prefix scan: lane owns bins 4*lane .. 4*lane+3
          int64_t c0[4], c1[4], cs[4], ct[4];
          int64_t a0 = 0, a1 = 0, as = 0, at_ = 0;
          const int hw = coop ? 0 : wid;   // cooperative nodes: combined into hist[0]
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int b = 4 * lane + e;
            a0 += hist[hw][0][b]; a1 += hist[hw][1][b]; as += hist[hw][2][b]; at_ += hist[hw][3][b];
            c0[e] = a0; c1[e] = a1; cs[e] = as; ct[e] = at_;
          }
          int64_t x0 = a0, x1 = a1, xs = as, xt = at_;
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            const int64_t y0 = __shfl_up(x0, o, 64), y1 = __shfl_up(x1, o, 64);
            const int64_t ys_ = __shfl_up(xs, o, 64), yt = __shfl_up(xt, o, 64);
            if (lane >= o) { x0 += y0; x1 += y1; xs += ys_; xt += yt; }
          }
          const int64_t p0 = x0 - a0, p1 = x1 - a1, ps = xs - as, pt = xt - at_;   // exclusive
          if (fp.kind == 2) ntreat = __shfl(xt, 63, 64);
          double lbest = -INFINITY;
          int lbin = NBINS;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int b = 4 * lane + e;
            if (b >= NBINS - 1) continue;
            const double crit = crit_at(p0 + c0[e], p1 + c1[e], ps + cs[e], pt + ct[e]);
            if (crit > lbest) { lbest = crit; lbin = b; }
          }
          take_best(lbest, lbin, f);
        };
        const int mrows = nd.hi - nd.lo;
#ifdef FOREST_PROF
        if (lane == 0 && small) atomicAdd(&forest_prof[t & 1023][mrows <= 16 ? 5 : 6], 1ull);
#endif
        if (small && mrows <= 16) {
          // Tiny node: every row is a lane; the candidate thresholds are the bins present
          // (an absent bin splits like the present bin below it, which wins the lowest-bin
          // tie-break), and each lane sums its own threshold's left side over the node's
          // rows. Same integer sums and criteria as the histogram path.
          if (fp.kind == 2) {
            int64_t t = 0;
            for (int j = 0; j < mrows; ++j) {
              const int64_t r1j = ((int64_t)__builtin_amdgcn_readlane((int)(cr1 >> 32), j) << 32) |
                                  (uint32_t)__builtin_amdgcn_readlane((int)cr1, j);
              t += from_fix(r1j) >= cn.wbar ? 1 : 0;
            }
            ntreat = t;
          }
          for (int k0 = 0; k0 < nf; k0 += 16) {
            int bins[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
              const int k = k0 + u;
              bins[u] = (cvalid && k < nf) ? (int)Xb[(int64_t)perm[wid][k] * n + ci] : 0;
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) {
              const int k = k0 + u;
              if (k >= nf) break;
              const int f = perm[wid][k];
              const int bme = bins[u];
              int64_t L0 = 0, L1 = 0, LS = 0, LT = 0;
              for (int j = 0; j < mrows; ++j) {
                const int bj = __builtin_amdgcn_readlane(bins[u], j);
                const bool in = bj <= bme;
                const int64_t wj = ((int64_t)__builtin_amdgcn_readlane((int)(cw >> 32), j) << 32) |
                                   (uint32_t)__builtin_amdgcn_readlane((int)cw, j);
                if (fp.kind == 0) {
                  const int yj = __builtin_amdgcn_readlane(cy, j);
                  if (in) { if (yj) L1 += wj; else L0 += wj; }
                } else {
                  const int64_t r1j =
                      ((int64_t)__builtin_amdgcn_readlane((int)(cr1 >> 32), j) << 32) |
                      (uint32_t)__builtin_amdgcn_readlane((int)cr1, j);
                  if (fp.kind == 1) {
                    if (in) { L0 += wj; LS += wj * r1j; }
                  } else {
                    const int64_t rhoj =
                        ((int64_t)__builtin_amdgcn_readlane((int)(crho >> 32), j) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)crho, j);
                    if (in) {
                      L0 += 1;
                      LS += rhoj;
                      LT += from_fix(r1j) >= cn.wbar ? 1 : 0;
                    }
                  }
                }
              }
              double lbest = -INFINITY;
              int lbin = NBINS;
              if (cvalid && bme < NBINS - 1) {
                const double crit = crit_at(L0, L1, LS, LT);
                if (crit > lbest) { lbest = crit; lbin = bme; }
              }
              take_best(lbest, lbin, f);
            }
          }
        } else if (small) {
          for (int k0 = 0; k0 < nf; k0 += SMALL_B) {
            int bins[SMALL_B];
#pragma unroll
            for (int u = 0; u < SMALL_B; ++u) {
              const int k = k0 + u;
              bins[u] = (cvalid && k < nf) ? (int)Xb[(int64_t)perm[wid][k] * n + ci] : 0;
            }
#pragma unroll
            for (int u = 0; u < SMALL_B; ++u) {
              const int k = k0 + u;
              if (k >= nf) break;
              const int f = perm[wid][k];
              clear_hist();
              if (cvalid) hist_row(bins[u], cw, cy, cr1, crho);
              scan_eval(f);
            }
          }
        } else {
          for (int k = 0; k < nf; ++k) {
            const int f = perm[wid][k];
            const uint8_t* xf = Xb + (int64_t)f * n;
            clear_hist();
            // 4 rows per lane per iteration: all gathers issued before the (integer,
            // order-independent) LDS atomics, so 4x more loads are in flight
            int q = q0;
            for (; q + 3 * qstep < nd.hi; q += 4 * qstep) {
              int ii[4], bb[4], yy[4];
              int64_t ww[4], aa[4], rr[4];
#pragma unroll
              for (int u = 0; u < 4; ++u) ii[u] = S.idx[q + qstep * u];
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                const int i = ii[u];
                bb[u] = xf[i];
                ww[u] = S.w[i];
                yy[u] = fp.kind == 0 ? ycls[i] : 0;
                aa[u] = fp.kind != 0 ? r1[i] : 0;
                rr[u] = fp.kind == 2 ? S.rho[i] : 0;
              }
#pragma unroll
              for (int u = 0; u < 4; ++u) hist_row(bb[u], ww[u], yy[u], aa[u], rr[u]);
            }
            for (; q < nd.hi; q += qstep) {
              const int i = S.idx[q];
              hist_row(xf[i], S.w[i], fp.kind == 0 ? ycls[i] : 0, fp.kind != 0 ? r1[i] : 0,
                       fp.kind == 2 ? S.rho[i] : 0);
            }
            if (coop) {
              __syncthreads();              // every wave's rows are in
              // combine the per-wave histograms into hist[0] (integer sums: exact)
              for (int e = tid; e < 4 * NBINS; e += NT) {
                const int c = e / NBINS, b = e % NBINS;
                int64_t acc = 0;
                for (int w = 1; w < NW; ++w) acc += hist[w][c][b];
                hist[0][c][b] += acc;
              }
              __syncthreads();
            }
            scan_eval(f);
            if (coop) __syncthreads();      // histograms read before the next clear
          }
        }
        if (!(bf >= 0 && best > parent + 1e-12 * fmax(1.0, fabs(parent)))) bf = -1;
      }
      // ---- record the decision (lane 0; wave 0 for a cooperative node)
      if (lane == 0 && (!coop || wid == 0)) {
        int nl_rows = 0;
        ATE_DASSERT(v >= 0 && v < cap && (bf < 0 || (bf < p && bb >= 0 && bb < NBINS - 1)));
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
          } else if (fp.kind == 1) {
            val[v] = from_fix(s1) / dn;
          } else {
            val[v] = 0.0;
          }
        }
        S.dec[j] = make_int4(bf >= 0 ? 1 : 0, bf, bb, nl_rows);
      }
    };
    // big nodes in level order, in chunks of COOP_CAP candidates (block compaction), each
    // decided by the whole workgroup; then every other node by one wave
    for (int base = 0; base < ncur; base += COOP_CAP) {
      const int j = base + tid;
      const bool big = tid < COOP_CAP && j < ncur && S.cur[j].hi - S.cur[j].lo > COOP_ROWS;
      int tot;
      const int pos = block_scan_excl<NW>(big ? 1 : 0, shi, &tot);
      if (big) sbig[pos] = j;
      __syncthreads();
      for (int e = 0; e < tot; ++e) decide(sbig[e], true);
      __syncthreads();
    }
    for (int j = wid; j < ncur; j += NW) {
      const Rng3 nd = S.cur[j];
      if (nd.hi - nd.lo > COOP_ROWS) continue;
      decide(j, false);
    }
    __syncthreads();
    FPROF_T(tl1_);
    FPROF_ADD(0, tl1_ - tl0_);
    // ---- child ids in level order (block scan over split flags)
    int id_base = snext_id;
    int nsplit_total = 0;
    for (int base = 0; base < ncur; base += NT) {
      const int j = base + tid;
      const int f = j < ncur ? S.dec[j].x : 0;
      int tot;
      const int pos = block_scan_excl<NW>(f, shi, &tot);
      if (f) {
        const int v = S.cur[j].id;
        ATE_DASSERT(v >= 0 && v < cap && id_base + 2 * (nsplit_total + pos) + 1 < cap);
        left[v] = id_base + 2 * (nsplit_total + pos);
        S.dec[j].w = nsplit_total + pos;   // split rank
      }
      nsplit_total += tot;
    }
    __syncthreads();
    FPROF_T(tl2_);
    FPROF_ADD(1, tl2_ - tl1_);
    // ---- stable partition of each split node (one wave per node) + next level list
    for (int j = wid; j < ncur; j += NW) {
      const int4 d = S.dec[j];
      if (!d.x) continue;
      const Rng3 nd = S.cur[j];
      const uint8_t* xf = Xb + (int64_t)d.y * n;
      int cnt_l = 0;
      for (int q0 = nd.lo; q0 < nd.hi; q0 += 64) {
        const int q = q0 + lane;
        const bool gl = q < nd.hi && xf[S.idx[q]] <= d.z;
        const uint64_t bl = __ballot(gl);
        if (gl) S.tmp[nd.lo + cnt_l + __popcll(bl & ((1ull << lane) - 1ull))] = S.idx[q];
        cnt_l += __popcll(bl);
      }
      int cnt_r = 0;
      for (int q0 = nd.lo; q0 < nd.hi; q0 += 64) {
        const int q = q0 + lane;
        const bool gr = q < nd.hi && xf[S.idx[q]] > d.z;
        const uint64_t br = __ballot(gr);
        if (gr) S.tmp[nd.lo + cnt_l + cnt_r + __popcll(br & ((1ull << lane) - 1ull))] = S.idx[q];
        cnt_r += __popcll(br);
      }
      for (int q = nd.lo + lane; q < nd.hi; q += 64) S.idx[q] = S.tmp[q];
      if (lane == 0) {
        const int r = d.w;
        const int lid = id_base + 2 * r;
        ATE_DASSERT(nd.lo <= nd.lo + cnt_l && nd.lo + cnt_l <= nd.hi && nd.hi <= n);
        S.nxt[2 * r] = {nd.lo, nd.lo + cnt_l, lid};
        S.nxt[2 * r + 1] = {nd.lo + cnt_l, nd.hi, lid + 1};
      }
    }
    __syncthreads();
    if (tid == 0) {
      sncur = 2 * nsplit_total;
      snext_id = id_base + 2 * nsplit_total;
    }
    FPROF_T(tl3_);
    FPROF_ADD(2, tl3_ - tl2_);
    // swap lists
    Rng3* tswap = S.cur; S.cur = S.nxt; S.nxt = tswap;
    __syncthreads();
  }
  const int nn = snext_id;
  if (tid == 0) nnodes[t] = nn;
  // ------------------------------------------------------------ grf leaf statistics (J2)
  if (fp.sampling == 1 && est_o) {
    int64_t* est = est_o + obase * 5;
    for (int e = tid; e < nn * 5; e += NT) est[e] = 0;
    __syncthreads();
    const int ne = sestn;
    for (int q = tid; q < ne; q += NT) {
      const int i = S.est_rows[q];
      int v = 0;
      while (true) {
        int64_t* e = est + (int64_t)v * 5;
        atomicAdd((unsigned long long*)&e[0], 1ull);
        if (fp.kind == 1) {
          atomicAdd((unsigned long long*)&e[1], (unsigned long long)r1[i]);
        } else {
          atomicAdd((unsigned long long*)&e[1], (unsigned long long)r1[i]);
          atomicAdd((unsigned long long*)&e[2], (unsigned long long)r2[i]);
          atomicAdd((unsigned long long*)&e[3],
                    (unsigned long long)to_fix(__dmul_rn(from_fix(r1[i]), from_fix(r1[i]))));
          atomicAdd((unsigned long long*)&e[4],
                    (unsigned long long)to_fix(__dmul_rn(from_fix(r1[i]), from_fix(r2[i]))));
        }
        if (feat[v] < 0) break;
        v = Xb[(int64_t)feat[v] * n + i] <= thr[v] ? left[v] : left[v] + 1;
      }
    }
  }
}

#ifndef FOREST_W4_MINW
#define FOREST_W4_MINW 4   // 4 waves/SIMD: 4 trees per CU, ~48 VGPRs spilled; vs 3: config 4
#endif                     // 0.616 -> 0.597 s, tutorial causal forest 124 -> 114 ms, same trees
ATE_KERNEL_SHAPE("forest_grow_kernel<4>", 256, 0, forest_grow_kernel<4, FOREST_W4_MINW>)
ATE_KERNEL_SHAPE("forest_grow_kernel<8>", 512, 0, forest_grow_kernel<8, 4>)
ATE_KERNEL_SHAPE("forest_grow_kernel<16>", 1024, 0, forest_grow_kernel<16, 4>)

ATE_API int ate_forest_fit(const void* fpp, const void* Xb, const void* ycls, const void* r1,
                           const void* r2, int cap, void* feat, void* thr, void* left, void* val,
                           void* nnodes, void* inbag, void* est, void* scratch, int nw,
                           void* stream) {
  const ForestParams fp = *(const ForestParams*)fpp;
  if (fp.p > PMAX_F || fp.n <= 0) return -1;
  // waves per tree and register budget (tools/forest_occ.sh, growth alone on MI355X):
  // <= 256 trees: 16 waves at 4 per SIMD (64 trees, n = 1e6: 1.01 s; 4 waves at 2 per
  // SIMD 1.83 s); <= 1024 trees: 8 waves at 4 per SIMD (300 trees: 2.11 s vs 2.35 s);
  // more: 4-wave workgroups at 3 per SIMD (2500 trees, n = 1e4: 33 ms vs 42 ms), round 3:
  // at 4 per SIMD (profiles/r03_forest_exact/w4_minw4_ab.txt).
  // nw: 0 = auto, or 4 / 8 / 16 (A/B).
  int w = nw;
  if (w == 0) w = fp.ntree <= 256 ? 16 : fp.ntree <= 1024 ? 8 : 4;
  hipStream_t s = (hipStream_t)stream;
#define ATE_FOREST_LAUNCH(NWV, MINW)                                                              \
  ATE_LAUNCH((forest_grow_kernel<NWV, MINW>), dim3(fp.ntree), dim3(64 * NWV), 0, s, fp,   \
                     (const uint8_t*)Xb, (const uint8_t*)ycls, (const int64_t*)r1,                 \
                     (const int64_t*)r2, cap, (int32_t*)feat, (int32_t*)thr, (int32_t*)left,      \
                     (double*)val, (int32_t*)nnodes, (uint8_t*)inbag, (int64_t*)est,              \
                     (char*)scratch)
  if (w == 4) ATE_FOREST_LAUNCH(4, FOREST_W4_MINW);
  else if (w == 8) ATE_FOREST_LAUNCH(8, 4);
  else if (w == 16) ATE_FOREST_LAUNCH(16, 4);
  else return -1;
#undef ATE_FOREST_LAUNCH
  ATE_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------ K15 prediction
// One thread per row, all trees (tree arrays are L2-resident). Same formulas and
// summation order as the CPU twin (atecpu_forest_predict).
// ---------------------------------------------------------------- K15/K17 prediction
// Node packing: one 8-byte load per tree level. code = (feat+1) << 9 | estok << 8 | thr,
// code >> 9 == 0 marks a leaf; estok = honest estimation count of the node > 0.
__global__ __launch_bounds__(256) void forest_pack_kernel(ForestParams fp, int cap,
                                                          const int32_t* __restrict__ feat,
                                                          const int32_t* __restrict__ thr,
                                                          const int32_t* __restrict__ left,
                                                          const int32_t* __restrict__ nnodes,
                                                          const int64_t* __restrict__ est,
                                                          int2* __restrict__ packed) {
  const int64_t total = (int64_t)fp.ntree * cap;
  for (int64_t k = blockIdx.x * (int64_t)256 + threadIdx.x; k < total;
       k += (int64_t)gridDim.x * 256) {
    const int t = (int)(k / cap), v = (int)(k % cap);
    if (v >= nnodes[t]) continue;
    const int f = feat[k];
    const int estok = (fp.sampling == 1 && est) ? (est[k * 5] > 0) : 1;
    const int code = f < 0 ? (estok << 8) : (((f + 1) << 9) | (estok << 8) | (thr[k] & 255));
    packed[k] = make_int2(f < 0 ? 0 : left[k], code);
  }
}

// leaves[tt][i] = leaf (node id within tree t0+tt) reached by row i, -1 if excluded (OOB)
__global__ __launch_bounds__(256) void forest_leaf_kernel(ForestParams fp,
                                                          const uint8_t* __restrict__ Xb, int n2,
                                                          int oob, int cap, int t0,
                                                          const int2* __restrict__ packed,
                                                          const uint8_t* __restrict__ inbag,
                                                          int32_t* __restrict__ leaves) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int t = t0 + blockIdx.y;
  if (i >= n2) return;
  int32_t* out = leaves + (int64_t)blockIdx.y * n2 + i;
  if (oob && inbag[(int64_t)t * fp.n + i]) { *out = -1; return; }
  const int2* tree = packed + (int64_t)t * cap;
  const bool honest = fp.sampling == 1;
  int v = 0, last_ok = 0;
  while (true) {
    ATE_DASSERT(v >= 0 && v < cap);
    const int2 nd = tree[v];
    if (honest && ((nd.y >> 8) & 1)) last_ok = v;
    const int f1 = nd.y >> 9;
    if (f1 == 0) break;
    v = Xb[(int64_t)(f1 - 1) * n2 + i] <= (nd.y & 255) ? nd.x : nd.x + 1;
  }
  *out = honest ? last_ok : v;
}

// exact-split forests (csrc/forest_exact.hip): uint16 value-rank bins, unpacked node arrays
__global__ __launch_bounds__(256) void forest_leaf16_kernel(ForestParams fp,
                                                            const uint16_t* __restrict__ Xb, int n2,
                                                            int oob, int cap, int t0,
                                                            const int32_t* __restrict__ feat,
                                                            const int32_t* __restrict__ thr,
                                                            const int32_t* __restrict__ left,
                                                            const uint8_t* __restrict__ inbag,
                                                            const int64_t* __restrict__ est,
                                                            int32_t* __restrict__ leaves) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int t = t0 + blockIdx.y;
  if (i >= n2) return;
  int32_t* out = leaves + (int64_t)blockIdx.y * n2 + i;
  if (oob && inbag[(int64_t)t * fp.n + i]) { *out = -1; return; }
  const int64_t b = (int64_t)t * cap;
  // grf (honest) trees predict from the deepest node on the path with J2 rows
  const bool honest = fp.sampling == 1 && est;
  int v = 0, last_ok = 0;
  while (true) {
    ATE_DASSERT(v >= 0 && v < cap);
    if (honest && est[(b + v) * 5] > 0) last_ok = v;
    if (feat[b + v] < 0) break;
    ATE_DASSERT(feat[b + v] < fp.p);
    v = Xb[(int64_t)feat[b + v] * n2 + i] <= thr[b + v] ? left[b + v] : left[b + v] + 1;
  }
  *out = honest ? last_ok : v;
}

// kind 0/1: running (sum, count) per row over trees in ascending order; per-tree values
// in 2^-32 fixed point, int64 sums (forest_common.hpp mean_fix)
__global__ __launch_bounds__(256) void forest_vote_kernel(ForestParams fp, int n2, int cap, int t0,
                                                          int nt, const int32_t* __restrict__ leaves,
                                                          const double* __restrict__ val,
                                                          const int64_t* __restrict__ est,
                                                          int64_t* __restrict__ state) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n2) return;
  int64_t acc = state[i], used = state[n2 + i];
  const bool leafmean = fp.kind == 0 || fp.sampling == 0;
#pragma unroll 4
  for (int tt = 0; tt < nt; ++tt) {
    const int lf = leaves[(int64_t)tt * n2 + i];
    if (lf < 0) continue;
    ATE_DASSERT(lf < cap);
    const int64_t nd = (int64_t)(t0 + tt) * cap + lf;
    used += 1;
    acc += leafmean ? to_fix(val[nd]) : mean_fix(est[nd * 5 + 1], est[nd * 5]);
  }
  state[i] = acc;
  state[n2 + i] = used;
}

// kind 2, pass 1: forest-weighted leaf moments (1, W, Y, WW, WY), fixed-point terms
__global__ __launch_bounds__(256) void forest_cate1_kernel(int n2, int cap, int t0, int nt,
                                                           const int32_t* __restrict__ leaves,
                                                           const int64_t* __restrict__ est,
                                                           int64_t* __restrict__ st) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n2) return;
  int64_t a1 = st[i], aw = st[n2 + i], ay = st[2 * n2 + i], aww = st[3 * n2 + i],
          awy = st[4 * n2 + i];
  for (int tt = 0; tt < nt; ++tt) {
    const int lf = leaves[(int64_t)tt * n2 + i];
    if (lf < 0) continue;
    ATE_DASSERT(lf < cap);
    const int64_t* e = est + ((int64_t)(t0 + tt) * cap + lf) * 5;
    a1 += 1; aw += mean_fix(e[1], e[0]); ay += mean_fix(e[2], e[0]);
    aww += mean_fix(e[3], e[0]); awy += mean_fix(e[4], e[0]);
  }
  st[i] = a1; st[n2 + i] = aw; st[2 * n2 + i] = ay; st[3 * n2 + i] = aww; st[4 * n2 + i] = awy;
}

// kind 2, pass 2: little-bag groups of the linearised score psi at the full-forest tau
// (chunks hold whole groups). st[5..9]: gs, gss, within (fixed point), nwithin, ng.
__global__ __launch_bounds__(256) void forest_cate2_kernel(ForestParams fp, int n2, int cap, int t0,
                                                           int nt, const int32_t* __restrict__ leaves,
                                                           const int64_t* __restrict__ est,
                                                           int64_t* __restrict__ st) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n2) return;
  const double a1 = (double)st[i];
  if (!(a1 > 0)) return;
  const double wb = from_fix(st[n2 + i]) / a1, yb = from_fix(st[2 * n2 + i]) / a1;
  const double H = from_fix(st[3 * n2 + i]) / a1 - wb * wb;
  if (!(H > 0)) return;
  const double tau = (from_fix(st[4 * n2 + i]) / a1 - wb * yb) / H;
  int64_t gs = st[5 * n2 + i], gss = st[6 * n2 + i], within = st[7 * n2 + i];
  int64_t nwithin = st[8 * n2 + i], ng = st[9 * n2 + i];
  ATE_DASSERT(fp.group >= 1 && t0 % fp.group == 0);   // chunks hold whole little bags
  for (int g0 = 0; g0 < nt; g0 += fp.group) {
    double ps = 0, pss = 0;
    int nb = 0;
    const int gsz = g0 + fp.group <= nt ? fp.group : nt - g0;
    for (int tt = g0; tt < g0 + fp.group && tt < nt; ++tt) {
      const int lf = leaves[(int64_t)tt * n2 + i];
      if (lf < 0) continue;
      const int64_t* e = est + ((int64_t)(t0 + tt) * cap + lf) * 5;
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

__global__ __launch_bounds__(256) void forest_final_kernel(ForestParams fp, int n2,
                                                           const int64_t* __restrict__ st,
                                                           double* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n2) return;
  if (fp.kind != 2) {
    out[i] = st[n2 + i] > 0 ? from_fix(st[i]) / (double)st[n2 + i] : NAN;
    return;
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
        const double wc = nw > 0 ? from_fix(st[7 * n2 + i]) / nw / (double)(fp.group > 1 ? fp.group - 1 : 1)
                                 : 0.0;
        var = grf_debias(between, wc, ng) / (H * H);
      }
    }
  }
  out[4 * i + 0] = tau;
  out[4 * i + 1] = var;
  out[4 * i + 2] = a1;
  out[4 * i + 3] = ng;
}

ATE_API int ate_forest_pack(const void* fpp, int cap, const void* feat, const void* thr,
                            const void* left, const void* nnodes, const void* est, void* packed,
                            void* stream) {
  const ForestParams fp = *(const ForestParams*)fpp;
  ATE_LAUNCH(forest_pack_kernel, dim3(ate::grid_for((int64_t)fp.ntree * cap, 256, 4096)),
                     dim3(256), 0, (hipStream_t)stream, fp, cap, (const int32_t*)feat,
                     (const int32_t*)thr, (const int32_t*)left, (const int32_t*)nnodes,
                     (const int64_t*)est, (int2*)packed);
  ATE_CHECK_LAUNCH();
  return 0;
}

// state: [10][n2] int64 accumulators (zeroed by the caller before phase 1); leaves:
// [tchunk][n2] int32 scratch, tchunk a multiple of the little-bag group size. Trees are
// visited in ascending order, so the sums match the host engine's sequential loop.
// phases (bitmask): 1 = per-tree sums (kind 0/1 votes, kind 2 leaf moments),
// 2 = kind-2 little-bag group sums (needs the COMPLETE phase-1 sums in state),
// 4 = finalise state -> out. A tree-parallel forest runs 1, all-reduce(state[0:5n2]),
// 2, all-reduce(state[5n2:10n2]), 4 (models/forest.py::predict_tree_parallel).
template <typename LeafFn>
static int forest_predict_impl(const ForestParams& fp, int n2, int cap, const void* val,
                               const void* est, void* leaves, int tchunk, void* state, void* out,
                               int phases, hipStream_t st, LeafFn leaf) {
  if (tchunk < 1 || (fp.kind == 2 && tchunk % fp.group)) return -1;
  const int rb = (n2 + 255) / 256;
  for (int pass = 0; pass < 2; ++pass) {
    if (!(phases & (1 << pass)) || (pass == 1 && fp.kind != 2)) continue;
    for (int t0 = 0; t0 < fp.ntree; t0 += tchunk) {
      const int nt = min(tchunk, fp.ntree - t0);
      leaf(dim3(rb, nt), t0);
      if (fp.kind != 2)
        ATE_LAUNCH(forest_vote_kernel, dim3(rb), dim3(256), 0, st, fp, n2, cap, t0, nt,
                           (const int32_t*)leaves, (const double*)val, (const int64_t*)est,
                           (int64_t*)state);
      else if (pass == 0)
        ATE_LAUNCH(forest_cate1_kernel, dim3(rb), dim3(256), 0, st, n2, cap, t0, nt,
                           (const int32_t*)leaves, (const int64_t*)est, (int64_t*)state);
      else
        ATE_LAUNCH(forest_cate2_kernel, dim3(rb), dim3(256), 0, st, fp, n2, cap, t0, nt,
                           (const int32_t*)leaves, (const int64_t*)est, (int64_t*)state);
    }
  }
  if (phases & 4)
    ATE_LAUNCH(forest_final_kernel, dim3(rb), dim3(256), 0, st, fp, n2,
                       (const int64_t*)state, (double*)out);
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_forest_predict(const void* fpp, const void* Xb, int n2, int oob, int cap,
                               const void* packed, const void* val, const void* inbag,
                               const void* est, void* leaves, int tchunk, void* state, void* out,
                               int phases, void* stream) {
  const ForestParams fp = *(const ForestParams*)fpp;
  hipStream_t st = (hipStream_t)stream;
  return forest_predict_impl(fp, n2, cap, val, est, leaves, tchunk, state, out, phases, st,
                             [&](dim3 g, int t0) {
    ATE_LAUNCH(forest_leaf_kernel, g, dim3(256), 0, st, fp, (const uint8_t*)Xb, n2, oob,
                       cap, t0, (const int2*)packed, (const uint8_t*)inbag, (int32_t*)leaves);
  });
}

// exact-split forests: uint16 bins and the unpacked (feat, thr, left) arrays
// est: grf estimation statistics (sampling 1), else null
ATE_API int ate_forest_predict16(const void* fpp, const void* Xb, int n2, int oob, int cap,
                                 const void* feat, const void* thr, const void* left,
                                 const void* val, const void* inbag, const void* est, void* leaves,
                                 int tchunk, void* state, void* out, int phases, void* stream) {
  const ForestParams fp = *(const ForestParams*)fpp;
  if (fp.sampling == 1 && !est) return -1;
  hipStream_t st = (hipStream_t)stream;
  return forest_predict_impl(fp, n2, cap, val, est, leaves, tchunk, state, out, phases, st,
                             [&](dim3 g, int t0) {
    ATE_LAUNCH(forest_leaf16_kernel, g, dim3(256), 0, st, fp, (const uint16_t*)Xb, n2, oob,
                       cap, t0, (const int32_t*)feat, (const int32_t*)thr, (const int32_t*)left,
                       (const uint8_t*)inbag, (const int64_t*)est, (int32_t*)leaves);
  });
}

// ------------------------------------------------------------ K11 binning
// bin(x) = #{edges < x} with per-feature sorted edges (<= 255), binary search in LDS.
// X: [p][n] column-major (float64), edges: [p][255] (unused slots = +inf), out uint8 [p][n].
__global__ __launch_bounds__(256) void bin_kernel(const double* __restrict__ X, int64_t n, int p,
                                                  const double* __restrict__ edges,
                                                  const int* __restrict__ nedges,
                                                  uint8_t* __restrict__ out) {
  __shared__ double e[255];
  const int f = blockIdx.y;
  const int ne = nedges[f];
  for (int k = threadIdx.x; k < 255; k += 256) e[k] = edges[(int64_t)f * 255 + k];
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double x = X[(int64_t)f * n + i];
    int lo = 0, hi = ne;   // first edge >= x
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (e[mid] < x) lo = mid + 1; else hi = mid;
    }
    out[(int64_t)f * n + i] = (uint8_t)lo;
  }
}

ATE_API int ate_bin_matrix(const void* X, int64_t n, int p, const void* edges, const void* nedges,
                           void* out, void* stream) {
  dim3 grid(ate::grid_for(n, 256, 512), p);
  ATE_LAUNCH(bin_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const double*)X, n, p,
                     (const double*)edges, (const int*)nedges, (uint8_t*)out);
  ATE_CHECK_LAUNCH();
  return 0;
}

#ifdef FOREST_PROF
extern "C" __attribute__((visibility("default"))) int ate_forest_prof_read(void* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(forest_prof), sizeof(forest_prof));
}
extern "C" __attribute__((visibility("default"))) int ate_forest_prof_reset() {
  static unsigned long long z[1024][8];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(forest_prof), z, sizeof(z));
}
#endif
