// K08 enet_cd_gram + K09 cv_loss (gaussian): glmnet-equivalent LASSO / elastic-net
// paths and cv.glmnet selection computed entirely from per-fold Gram matrices (K01).
// Reference call sites: ate_functions.R:101,123,304,305 (cv.glmnet gaussian).
//
//  prepare:  for each training set s (a subset of fold segments) sum the raw
//            augmented fold Grams and standardise (glmnet `standard`: population
//            SD, centred): C_s = D^-1 (G/n - m m') D^-1, g_{s,y} = D^-1 (G_xy/n - m ym)/ys.
//  path:     ONE WAVE per problem (training set, response). The gradient g, the
//            coefficients a, xv, vp live in registers, lane l owning coordinates
//            l, l+64, ...; a pass walks coordinates in order and uses a ballot to
//            jump to the next coordinate that can move (nonzero, or |u| > vp*lambda),
//            re-evaluated after every update -- exactly glmnet's sequential semantics
//            (full pass, then active-set passes until max xv*d^2 < thresh). Gram rows
//            are read from L2 (the Gram stack is a few MB).
//  cv loss:  held-out MSE of every (fold problem, lambda) from the held-out fold's
//            Gram: sum (y - a0 - x b)^2 = y'y - 2 a0 S_y - 2 b'X'y + n a0^2 + 2 a0 b'S_x
//            + b'X'X b -- no pass over the data.
//  select:   cvm, cvsd, lambda.min, lambda.1se with glmnet's rules.
#include <cstdlib>

#include <utility>

#include "common.hpp"

#include <type_traits>

using namespace ate;

// ------------------------------------------------------------------ prepare
// G: [nseg][P][P] raw Gram stack (panel columns). masks: [ntrain][nseg] (1 = in training set).
// xcols[p], ones_col, ycols[ny]. Outputs per training set s:
//   C[s][p][p], g[s][ny][p], xm[s][p], xs[s][p] (1 where constant), ju[s][p],
//   ym[s][ny], ys[s][ny], nobs[s]
// Two launches: per-set column statistics (means, SDs, constant flags, n), then the
// standardised Gram / gradient entries, each reading only its own masked segment sum.
__device__ __forceinline__ double seg_sum(const double* __restrict__ G, int nseg, int P,
                                          const unsigned char* __restrict__ mk, int a, int b) {
  double acc = 0.0;
  for (int q = 0; q < nseg; ++q)
    if (mk[q]) acc += G[((int64_t)q * P + a) * P + b];
  return acc;
}

__global__ __launch_bounds__(256) void enet_prep_stats_kernel(
    const double* __restrict__ G, int nseg, int P, const unsigned char* __restrict__ masks,
    const int* __restrict__ xcols, int p, int ones_col, const int* __restrict__ ycols, int ny,
    double* __restrict__ xm, double* __restrict__ xs, unsigned char* __restrict__ ju,
    double* __restrict__ ym, double* __restrict__ ys, double* __restrict__ nobs) {
  const int s = blockIdx.y;
  const unsigned char* mk = masks + (int64_t)s * nseg;
  const double n = seg_sum(G, nseg, P, mk, ones_col, ones_col);
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < p) {
    const int j = e;
    const double mj = seg_sum(G, nseg, P, mk, ones_col, xcols[j]) / n;
    const double vj = seg_sum(G, nseg, P, mk, xcols[j], xcols[j]) / n - mj * mj;
    xm[(int64_t)s * p + j] = mj;
    xs[(int64_t)s * p + j] = vj > 0 ? sqrt(vj) : 1.0;
    ju[(int64_t)s * p + j] = vj > 0 ? 1 : 0;
    if (j == 0) nobs[s] = n;
  } else if (e < p + ny) {
    const int y = e - p;
    const double my = seg_sum(G, nseg, P, mk, ones_col, ycols[y]) / n;
    const double vy = seg_sum(G, nseg, P, mk, ycols[y], ycols[y]) / n - my * my;
    ym[(int64_t)s * ny + y] = my;
    ys[(int64_t)s * ny + y] = vy > 0 ? sqrt(vy) : 1.0;
  }
}

// G: [nseg][P][P] raw Gram stack (panel columns). masks: [ntrain][nseg] (1 = in training set).
// Outputs per training set s: C[s][p][ldc] = D^-1 (G/n - m m') D^-1 (glmnet `standard`:
// population SD, centred; identity row/col for constant columns), g[s][ny][p].
template <typename CT>
__global__ __launch_bounds__(256) void enet_prepare_kernel(
    const double* __restrict__ G, int nseg, int P, const unsigned char* __restrict__ masks,
    const int* __restrict__ xcols, int p, int ldc, const int* __restrict__ ycols, int ny,
    const double* __restrict__ xm, const double* __restrict__ xs,
    const unsigned char* __restrict__ ju, const double* __restrict__ ym,
    const double* __restrict__ ys, const double* __restrict__ nobs, CT* __restrict__ C,
    double* __restrict__ g) {
  const int s = blockIdx.y;
  const unsigned char* mk = masks + (int64_t)s * nseg;
  const double n = nobs[s];
  const int64_t total = (int64_t)p * p + (int64_t)ny * p;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    if (e < (int64_t)p * p) {
      const int j = (int)(e / p), k = (int)(e % p);
      const bool okj = ju[(int64_t)s * p + j], okk = ju[(int64_t)s * p + k];
      double cjk;
      if (!okj || !okk) {
        cjk = (j == k) ? 1.0 : 0.0;
      } else {
        const double mj = xm[(int64_t)s * p + j], mk2 = xm[(int64_t)s * p + k];
        cjk = (seg_sum(G, nseg, P, mk, xcols[j], xcols[k]) / n - mj * mk2) /
              (xs[(int64_t)s * p + j] * xs[(int64_t)s * p + k]);
      }
      C[((int64_t)s * p + j) * ldc + k] = (CT)cjk;
    } else {
      const int64_t r = e - (int64_t)p * p;
      const int y = (int)(r / p), j = (int)(r % p);
      double gj = 0.0;
      if (ju[(int64_t)s * p + j]) {
        const double mj = xm[(int64_t)s * p + j], my = ym[(int64_t)s * ny + y];
        gj = (seg_sum(G, nseg, P, mk, xcols[j], ycols[y]) / n - mj * my) /
             (xs[(int64_t)s * p + j] * ys[(int64_t)s * ny + y]);
      }
      g[((int64_t)s * ny + y) * p + j] = gj;
    }
  }
}

ATE_API int ate_enet_prepare(const void* G, int nseg, int P, const void* masks, int ntrain,
                             const void* xcols, int p, int ones_col, const void* ycols, int ny,
                             void* C, int c_f32, void* g, void* xm, void* xs, void* ju, void* ym,
                             void* ys, void* nobs, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  ATE_LAUNCH(enet_prep_stats_kernel, dim3((p + ny + 255) / 256, ntrain), dim3(256), 0, st,
                     (const double*)G, nseg, P, (const unsigned char*)masks, (const int*)xcols,
                     p, ones_col, (const int*)ycols, ny, (double*)xm, (double*)xs,
                     (unsigned char*)ju, (double*)ym, (double*)ys, (double*)nobs);
  ATE_CHECK_LAUNCH();
  const int64_t total = (int64_t)p * p + (int64_t)ny * p;
  dim3 grid(grid_for(total, 256, 512), ntrain);
  const int ldc = (p + 63) / 64 * 64;   // padded row stride (C buffer must be zeroed)
  if (c_f32)
    ATE_LAUNCH(enet_prepare_kernel<float>, grid, dim3(256), 0, st, (const double*)G, nseg,
                       P, (const unsigned char*)masks, (const int*)xcols, p, ldc,
                       (const int*)ycols, ny, (const double*)xm, (const double*)xs,
                       (const unsigned char*)ju, (const double*)ym, (const double*)ys,
                       (const double*)nobs, (float*)C, (double*)g);
  else
    ATE_LAUNCH(enet_prepare_kernel<double>, grid, dim3(256), 0, st, (const double*)G, nseg,
                       P, (const unsigned char*)masks, (const int*)xcols, p, ldc,
                       (const int*)ycols, ny, (const double*)xm, (const double*)xs,
                       (const unsigned char*)ju, (const double*)ym, (const double*)ys,
                       (const double*)nobs, (double*)C, (double*)g);
  ATE_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ path (one wave / problem)
struct EnetProblem {
  int train;        // training set index (C, xm, xs, ju)
  int y;            // response index within the training set's g/ym/ys
  int ulam_src;     // -1: computed path; >=0: problem whose (original-scale) lambdas to use;
                    // < -1: placeholder slot (skipped)
  int nlam_req;
};

constexpr double BIGL = 9.9e35;
constexpr int PMAX = 512;

#ifdef ENET_PROF
// cycle accounting per problem (debug builds): [0] pull, [1] recurrence, [2] other,
// [3] block visits, [4] coordinate updates, [5] pending columns pulled, [6] passes
__device__ unsigned long long enet_prof[256][32];
#define PROF_T(var) const unsigned long long var = wall_clock64()
#define PROF_ADD(k, v) do { if (tid == 0) sprof[0][k] += (unsigned long long)(v); } while (0)
#else
#define PROF_T(var)
#define PROF_ADD(k, v) do { } while (0)
#endif

template <typename CT> struct VecT;
template <> struct VecT<float> { typedef float4 type; };
template <> struct VecT<double> { typedef double2 type; };
__device__ __forceinline__ float vdot(float4 a, float4 b) {
  return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}
__device__ __forceinline__ double vdot(double2 a, double2 b) { return a.x * b.x + a.y * b.y; }

// LDS-DMA: each lane copies 16 B from its own global address to dst + 16 * lane
__device__ __forceinline__ void glds16f(const float* src, float* dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}
__device__ __forceinline__ void glds16f(const double*, float*) {}   // fp64 C: unused

__device__ __forceinline__ double readlane_d(double v, int i) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), i);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), i);
  return __hiloint2double(hi, lo);
}

// a = (lane == i) ? b : a and c = (lane == i) ? d : c for a compile-time lane i
__device__ __forceinline__ void select_lane(int i, int lane, double& a, double b, double& c, double d) {
  int a0 = __double2loint(a), a1 = __double2hiint(a), c0 = __double2loint(c), c1 = __double2hiint(c);
  asm volatile(
      "v_cmp_eq_u32_e32 vcc, %4, %5\n\t"
      "v_cndmask_b32_e32 %0, %0, %6, vcc\n\t"
      "v_cndmask_b32_e32 %1, %1, %7, vcc\n\t"
      "v_cndmask_b32_e32 %2, %2, %8, vcc\n\t"
      "v_cndmask_b32_e32 %3, %3, %9, vcc"
      : "+v"(a0), "+v"(a1), "+v"(c0), "+v"(c1)
      : "i"(i), "v"(lane), "v"(__double2loint(b)), "v"(__double2hiint(b)), "v"(__double2loint(d)),
        "v"(__double2hiint(d))
      : "vcc");
  a = __hiloint2double(a1, a0);
  c = __hiloint2double(c1, c0);
}

// a = (lane == i) ? b : a for a compile-time lane i (one compare + two selects)
__device__ __forceinline__ void select_lane1(int i, int lane, double& a, double b) {
  int a0 = __double2loint(a), a1 = __double2hiint(a);
  asm volatile(
      "v_cmp_eq_u32_e32 vcc, %2, %3\n\t"
      "v_cndmask_b32_e32 %0, %0, %4, vcc\n\t"
      "v_cndmask_b32_e32 %1, %1, %5, vcc"
      : "+v"(a0), "+v"(a1)
      : "i"(i), "v"(lane), "v"(__double2loint(b)), "v"(__double2hiint(b))
      : "vcc");
  a = __hiloint2double(a1, a0);
}

// ---- row-blocked broadcast (the lasso dense walk, ENET_ROWWALK)
// u += bcast(d) * nc, bcast = lane C of each 16-lane row (DPP64 row_newbcast: v_fmac_f64
// takes the broadcast as an operand, no readlane -> SGPR -> VALU hop on the chain). The
// s_nop covers the VALU-write -> DPP-read hazard on d.
template <int C>
__device__ __forceinline__ void fmac_bcast(double& u, double d, double nc) {
  asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(u)
               : "v"(d), "v"(nc), "i"(C));
}
// every 16-lane row <- row R of x (gfx950 v_permlane32_swap: rows (0,1) <-> (2,3) of the
// two operands, then v_permlane16_swap: odd <-> even rows)
template <int R>
__device__ __forceinline__ double row_replicate(double x) {
  unsigned w[2] = {(unsigned)__double2loint(x), (unsigned)__double2hiint(x)};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const auto p = __builtin_amdgcn_permlane32_swap(w[h], w[h], false, false);
    const unsigned a = R < 2 ? p[0] : p[1];            // (Ra, Rb, Ra, Rb), a = R & ~1
    const auto q = __builtin_amdgcn_permlane16_swap(a, a, false, false);
    w[h] = (R & 1) ? q[1] : q[0];
  }
  return __hiloint2double((int)w[1], (int)w[0]);
}

// min(max(u, lo), hi) as the two hardware ops fmin(fmax(...)) compiles to, without the
// canonicalising max(u, u) the compiler puts in front of a value produced by inline asm
// (u is never NaN here, so the result is the same bits)
__device__ __forceinline__ double clamp_hw(double u, double lo, double hi) {
  double r;
  asm("v_max_f64 %0, %1, %2\n\tv_min_f64 %0, %0, %3" : "=&v"(r) : "v"(u), "v"(lo), "v"(hi));
  return r;
}

// (u - a) - min(max(u, lo), hi): the lasso step of the dense walk, with u - a issued first
// (it only waits for u) so the clamp chain is max -> min -> sub
__device__ __forceinline__ double lasso_step_hw(double u, double a, double lo, double hi) {
  double t, c;
  asm("v_add_f64 %0, %2, -%3\n\t"
      "v_max_f64 %1, %2, %4\n\t"
      "v_min_f64 %1, %1, %5\n\t"
      "v_add_f64 %1, %0, -%1"
      : "=&v"(t), "=&v"(c)
      : "v"(u), "v"(a), "v"(lo), "v"(hi));
  return c;
}

template <class F, int... C>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, C...>) {
  (f(std::integral_constant<int, C>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {   // f(integral_constant<int, 0..N-1>)
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// Self-test of the two cross-lane primitives above (tests/test_gpu.py): out[r * 64 + l] =
// row_replicate<r>(x)[l] for x = lane id, out[256 + l] = u after fmac_bcast<5> with
// u = 1, d = lane, nc = 2 (= 1 + 2 * (16 * (l >> 4) + 5)).
__global__ void enet_isa_selftest_kernel(double* out) {
  const int l = threadIdx.x;
  const double x = (double)l;
  out[l] = row_replicate<0>(x);
  out[64 + l] = row_replicate<1>(x);
  out[128 + l] = row_replicate<2>(x);
  out[192 + l] = row_replicate<3>(x);
  double u = 1.0;
  fmac_bcast<5>(u, x, 2.0);
  out[256 + l] = u;
}

ATE_API int ate_enet_isa_selftest(void* out, void* stream) {
  ATE_LAUNCH(enet_isa_selftest_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     (double*)out);
  ATE_CHECK_LAUNCH();
  return 0;
}

// Blocked covariance-mode coordinate descent, ONE WAVE per problem.
//
// glmnet's pass visits coordinates j = 0..p-1 in order and processes j iff it is nonzero
// or |u_j| > vp_j*lambda (u = g + a). We walk the coordinates in blocks of 64:
//   * gradient / coefficients / flags of all p coordinates live in LDS (fp64);
//   * inside block t the recurrence only involves the 64x64 diagonal Gram block, staged
//     in LDS: lane l keeps g of coordinate t*64+l in a register, the next coordinate to
//     process is found with a ballot re-evaluated after every update (so zero coordinates
//     are tested against the current gradient exactly as in the sequential pass), and an
//     update costs one LDS read + one FMA per lane;
//   * after block t its deltas are propagated to every other block with bulk, coalesced
//     row-segment loads  g[t2*64+l] -= sum_i C[t2*64+l][t*64+i] d_i  -- no serial memory
//     latency on the coordinate chain.
// Same sequence of coordinate updates as glmnet's pass; only the order of floating-point
// additions into far gradients differs.
// PULL formulation. Each coordinate's cumulative change is kept in Dcum; each block t keeps
// a snapshot Dsnap_t of Dcum taken when its gradient was last brought up to date. Before
// block t is processed, one bandwidth-bound pass over its 64 Gram rows applies every
// pending change:   g_t -= C[t rows, :] (Dcum - Dsnap_t)
// (4 waves split the columns; partial sums reduced through LDS), and the same loads
// deposit the 64x64 diagonal block in LDS for the sequential in-block recurrence (wave 0).
// Active passes skip blocks without active coordinates (no pull needed: nothing in them
// can move); full passes pull every block, so every KKT check uses the current gradient.
#ifndef ENET_NW
#define ENET_NW 8   // waves per problem: wave 0 = recurrence, waves 1.. = pulls
#endif
constexpr int NW = ENET_NW, NTH = NW * 64, NP = NW - 1;
static_assert(NW >= 3, "phase B uses wave 1 for block tn and waves 2.. for snapshots");
// the fp32 pulls give ONE 64-column block to each pull wave (jb = wid + (wid >= t)), so
// every block of a PMAX-column problem needs its own wave
static_assert(NW >= PMAX / 64, "one pull wave per 64-column block: NW >= PMAX / 64");
#ifndef ENET_SETPRIO
#define ENET_SETPRIO 0       // A/B: 1 = recurrence wave at issue priority 3, 2 = every wave
#endif
#ifndef ENET_BALLOT_ONLY
#define ENET_BALLOT_ONLY 0   // 1: every pass uses the ballot recurrence (A/B timing)
#endif
#ifndef ENET_PULL_DENSE      // pull a whole 64-row column block when at least this many of
#define ENET_PULL_DENSE 12   //   its coordinates are pending, else a compacted row list
#endif                       //   (sweep 4..48: 12 best, CV stage 3.12 -> 2.98 ms, same bits;
                             //   profiles/r03_enet/pull_dense_sweep.txt)
#ifndef ENET_ROWWALK          // 1: lasso dense walk in 16-lane rows (DPP64 broadcasts inside
#define ENET_ROWWALK 0       //   a row, permlane replicate + 16 DPP64 fmas to catch the other
#endif                       //   rows up). Same bits, but the CV stage took 3.37-3.46 ms vs
                             //   2.84 for the readlane walk (profiles/r04_enet/rowwalk_ab.txt)
#ifndef ENET_MODE_S          // small-active-set mode (fp32 C): while at most ENET_S_ENTER
#define ENET_MODE_S 1        //   coordinates have ever moved, passes run in wave 0 over all p
#endif                       //   coordinates with the movers' Gram columns cached in LDS
#ifndef ENET_S_ENTER
#define ENET_S_ENTER 40
#endif
#ifndef ENET_S_FETCH         // ... and while a lambda fetched at most this many new columns:
#define ENET_S_FETCH 8       //   a fetch is an L2/HBM round trip on the mode-S chain, so a
#endif                       //   problem whose active set grows fast (dense W fits) leaves early
constexpr int S_UNION = 112 * 1024;          // LDS shared by mode L's blocks and mode S's cache
constexpr int S_CAP = S_UNION / (PMAX * 4);  // cached columns (56)
#ifndef ENET_DENSE_MIN       // dense (all 64 lanes, static) walk of a block when at least
#define ENET_DENSE_MIN 28    //   this many lanes move: nonzero lanes (full pass) /
#endif                       //   eligible lanes (active pass)

#define LDS_AS __attribute__((address_space(3)))
struct PassS {
  double dlx, rsq;
};
// ---- mode S: small active set (glmnet covariance mode's own design: the Gram columns
// of the coordinates that have moved are kept on chip). While few coordinates have ever
// moved, a pass runs in wave 0 alone over ALL p coordinates, lane l holding g, a, vp of
// coordinates k = s * 64 + l (s = 0..7) in registers: the next coordinate that can move
// (eligible, and nonzero or |g| > vp * lambda; in index order past the last one) comes
// from eight ballots, and a move updates all p gradients from the mover's cached column
// (fetched from C's row j -- C is symmetric -- on its first move). Exactly glmnet's
// sequential pass (full: every coordinate; active: the ever-moved ones), with every
// gradient exact at all times: nothing is pending when the problem switches to mode L.
// fp32 C only; the gradients accumulate in fp64. Returns max d^2 (wave-uniform).
// A separate (not inlined) function: its SGPR-heavy walk would otherwise push the path
// kernel's own SGPRs into spills (8 -> 91) inside the mode-L walks. LDS operands arrive as
// address-space-3 pointers, so they stay ds_* accesses.
__device__ __noinline__ PassS enet_pass_s(bool full, int T, int ldc, double ab, double dem,
                                          const float* __restrict__ Cf, LDS_AS double* sg,
                                          LDS_AS double* sa, const LDS_AS double* svp,
                                          LDS_AS int* sflag, LDS_AS int* sslot,
                                          LDS_AS float* sccache, LDS_AS int* sever_n,
                                          LDS_AS int* sncache,
                                          LDS_AS unsigned long long* sprof_row) {
  const int lane = threadIdx.x & 63;
#ifdef ENET_PROF
  const long long tps0_ = clock64();
  unsigned long long nit_ = 0, nfetch_ = 0;
#endif
  double gS[8], aS[8], tS[8];
  int slS[8];
  // per-lane flag bits (VGPR, not 24 SGPR masks): bit s = coordinate s*64+lane is visited
  // by this pass (eligible; in an active pass also ever moved), bit 8+s = ever moved
  int flb = 0;
#pragma unroll
  for (int s8 = 0; s8 < 8; ++s8) {   // sets past the padded width ldc: never eligible
    const int k = s8 * 64 + lane;
    const bool in = s8 < T;          // (their LDS entries are not initialised)
    gS[s8] = in ? sg[k] : 0.0;
    aS[s8] = in ? sa[k] : 0.0;
    tS[s8] = in ? svp[k] * ab : 0.0;
    slS[s8] = in ? sslot[k] : -1;
    const int f = in ? sflag[k] : 0;
    if ((f & 1) && (full || (f & 2))) flb |= 1 << s8;
    if (f & 2) flb |= 1 << (8 + s8);
  }
  int ncache = __builtin_amdgcn_readfirstlane(*sncache);   // uniform (SGPR) counters
  int ever_n = __builtin_amdgcn_readfirstlane(*sever_n);
  double dlx = 0.0, rsq_add = 0.0;
#ifdef ENET_PROF
  const long long tpl0_ = clock64();
#endif
  // The pass walks the sets in order (static: every register array is indexed with a
  // compile-time set, no 8-way selects); inside set s the candidates are re-evaluated after
  // every move, for the lanes past the mover only (the sets after s are evaluated when the
  // walk reaches them, with their gradients as they are then: glmnet's order exactly).
  static_for<8>([&](auto s_tag) __attribute__((always_inline)) {
    constexpr int SJ = decltype(s_tag)::value;
    if (SJ >= T) return;
    uint64_t live = ~0ull;   // lanes of this set not yet passed
    for (;;) {
      const bool c = ((flb >> SJ) & 1) & ((aS[SJ] != 0.0) | (fabs(gS[SJ] + aS[SJ]) > tS[SJ]));
      const uint64_t cm = __builtin_amdgcn_ballot_w64(c) & live;
      if (!cm) break;
      const int lj = __ffsll((unsigned long long)cm) - 1;
      live = lj == 63 ? 0ull : (~0ull << (lj + 1));
#ifdef ENET_PROF
      ++nit_;
#endif
      const int j = SJ * 64 + lj;
      const double gj = readlane_d(gS[SJ], lj);
      const double aj = readlane_d(aS[SJ], lj);
      const double tj = readlane_d(tS[SJ], lj);
      int slj = __builtin_amdgcn_readlane(slS[SJ], lj);
      const double uj = gj + aj;
      double an = copysign(fmax(fabs(uj) - tj, 0.0), uj);
      if (dem != 0.0) an = an / (1.0 + svp[j] * dem);
      const double d = an - aj;
      if (__builtin_amdgcn_readfirstlane((int)(d == 0.0))) continue;
      // the mover's column: cached, newly cached, or (cache full) read from C directly
      float cv[8];
      if (slj < 0 && ncache < S_CAP) {
#ifdef ENET_PROF
        ++nfetch_;
#endif
        slj = ncache++;
        const float* Cj = Cf + (int64_t)j * ldc;
        LDS_AS float* dst = sccache + slj * PMAX;
#pragma unroll
        for (int s8 = 0; s8 < 8; ++s8) {
          const int k = s8 * 64 + lane;
          const float v = k < ldc ? Cj[k] : 0.f;
          cv[s8] = v;
          dst[(s8 >> 2) * 256 + lane * 4 + (s8 & 3)] = v;
        }
        if (lane == 0) sslot[j] = slj;
        if (lane == lj) slS[SJ] = slj;
      } else if (slj >= 0) {
        const LDS_AS float* src = sccache + slj * PMAX + lane * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {   // two 16-byte LDS reads
          cv[e] = src[e];
          cv[4 + e] = src[256 + e];
        }
      } else {
        const float* Cj = Cf + (int64_t)j * ldc;
#pragma unroll
        for (int s8 = 0; s8 < 8; ++s8) cv[s8] = s8 * 64 + lane < ldc ? Cj[s8 * 64 + lane] : 0.f;
      }
#pragma unroll
      for (int s8 = 0; s8 < 8; ++s8) gS[s8] = __builtin_fma(-(double)cv[s8], d, gS[s8]);
      // bookkeeping of j (glmnet: the gradient BEFORE the move enters rsq)
      const int evj = __builtin_amdgcn_readlane(flb, lj);
      if (!((evj >> (8 + SJ)) & 1)) ++ever_n;
      if (lane == lj) {
        flb |= 1 << (8 + SJ);
        aS[SJ] = an;
      }
      rsq_add += d * (2.0 * gj - d);
      dlx = fmax(dlx, d * d);
    }
  });
#ifdef ENET_PROF
  if (lane == 0) sprof_row[23] += (unsigned long long)(clock64() - tpl0_);   // [23] loop only
#endif
#pragma unroll
  for (int s8 = 0; s8 < 8; ++s8) {
    if (s8 < T) {
      const int k = s8 * 64 + lane;
      sg[k] = gS[s8];
      sa[k] = aS[s8];
      if ((flb >> (8 + s8)) & 1) sflag[k] |= 2;
    }
  }
  if (lane == 0) {
    *sever_n = ever_n;
    *sncache = ncache;
  }
#ifdef ENET_PROF
  if (lane == 0) {   // mode S: [19] passes, [20] candidates visited, [21] cycles, [22] fetches
    sprof_row[19] += 1ull;
    sprof_row[20] += nit_;
    sprof_row[21] += (unsigned long long)(clock64() - tps0_);
    sprof_row[22] += nfetch_;
  }
#endif
  return PassS{dlx, rsq_add};
}

// LASSO: alpha == 1 (dem == 0 at every lambda): the elastic-net walk and scaling are not
// compiled into that instantiation (the kernel's code is ~60 KB against a 64 KB instruction
// cache shared by two CUs; every unused walk variant is cache pressure on the hot one).
// how many lambdas a fold problem may run ahead of its source (enet_path_kernel)
constexpr int FOLD_LEAD = 2;

// glmnet's lambda_0, extrapolated from lambda_1 and lambda_2 (one definition: the source's
// published sequence and its own lams[] must be the same bits)
__device__ __noinline__ double lambda0_extrap(double l1, double l2) {
#pragma clang fp contract(off)
  return exp(2.0 * log(l1) - log(l2));
}

template <typename CT, bool LASSO>
__global__ __launch_bounds__(NTH) void enet_path_kernel(
    const CT* __restrict__ C, const double* __restrict__ gin, int p, int ny,
    const unsigned char* __restrict__ ju_s, const double* __restrict__ ys_s,
    const double* __restrict__ vp_in, const EnetProblem* __restrict__ probs, int nprob,
    double alpha, double flmin, double thr, int maxit,
    double* __restrict__ apath, double* __restrict__ lams, double* __restrict__ rsqs,
    int* __restrict__ nlam_out, int* __restrict__ npass_out, int L, int* __restrict__ progress,
    long spin_max, double* __restrict__ lampub) {
  constexpr int TMAX = PMAX / 64;
  __shared__ double sg[PMAX], sa[PMAX], svp[PMAX], sdc[PMAX];
  // Mode L's snapshots and staged blocks share one LDS region with mode S's column cache
  // (mode S only runs before the first mode-L pass and never again; the switch re-zeroes the
  // snapshots). sds: per-block snapshots of Dcum (32 KB); sCn2 / sCorr: see below.
  __shared__ __attribute__((aligned(16))) unsigned char s_union[S_UNION];
  double(&sds)[TMAX][PMAX] = *reinterpret_cast<double(*)[TMAX][PMAX]>(s_union);
  float(&sCn2)[2][64 * 64] = *reinterpret_cast<float(*)[2][64 * 64]>(s_union + 32768);
  float(&sCorr)[64 * 64] = *reinterpret_cast<float(*)[64 * 64]>(s_union + 65536);
  // mode S: column slot c holds C[k][j] for every k at (c * PMAX + (k >> 8) * 256 + (k & 63) * 4
  // + ((k >> 6) & 3)) floats: lane l's 8 coordinates k = s * 64 + l are two 16-byte reads
  float* const sccache = reinterpret_cast<float*>(s_union);
  __shared__ int sslot[PMAX];             // mode S: cache slot of coordinate k (-1: none)
  __shared__ int sever_n;                 // mode S: coordinates that have ever moved
  __shared__ int sncache;                 // mode S: cached columns
  // phase-B hand-offs without a second barrier: wave 0's publication count (visits whose
  // block t it has published) and the pull waves' phase-B arrival count (NP per visit
  // with a prefetch block)
  __shared__ int spub, sarr;
  __shared__ int sfetch0;                 // mode S: cached columns at the lambda's start
  __shared__ int sflag[PMAX];             // bit0 ju, bit1 active
  __shared__ double spart2[2][NW][64];    // pull partials (and fp64 own-delta corr, slot 0),
                                          // double-buffered by visit parity
  __shared__ __attribute__((aligned(16))) float sred[NW][256];   // group reduction per wave
  __shared__ __attribute__((aligned(16))) float sdw[NW][64];     // pull_block deltas per wave
  __shared__ int srow[NW][64];                                   // pull_block row lists
  __shared__ float scorr2[2][NP][64];     // phase B: own-delta correction partials (fp32 C)
  __shared__ int scorr_ok[2];             // ... and whether they were computed
#ifdef ENET_PROF
  // per-wave cycle accumulators in LDS (lane 0 of a wave adds to its own row), flushed to
  // enet_prof once at kernel end: no global atomics (and their vmcnt waits at barriers)
  // inside the visit loop
  __shared__ unsigned long long sprof[NW][32];
  for (int e = threadIdx.x; e < NW * 32; e += blockDim.x) (&sprof[0][0])[e] = 0ull;
#endif
  __shared__ __attribute__((aligned(16))) CT sdelta[PMAX];
  __shared__ int slist[PMAX];             // compacted pending columns (per-wave quarters)
  constexpr int PER = (PMAX + NP - 1) / NP + 1;   // pending entries per pull wave
  __shared__ int slist2[NP * PER];        // pipelined pull: waves 1.., PER entries each
  __shared__ __attribute__((aligned(16))) CT sdelta2[NP * PER];
  __shared__ int scl[64];                 // wave 0: changed coordinates of the block
  __shared__ CT scd[64];
  // diagonal blocks, double-buffered: sCn2[cpar] holds the block of the visit in progress
  // (wave 0 loads it into registers at the start of its recurrence), the pull waves DMA the
  // next visited block's into sCn2[cpar ^ 1]. Keeping the recurrence's registers out of the
  // loop-carried state leaves the pull waves' code the whole register budget (no spills).
  // sCn2[2][64 * 64], sCorr[64 * 64] (C[t rows][tn cols], fp32 C): in s_union above
  __shared__ __attribute__((aligned(16))) float sdall[64];         // wave 0: block t's deltas
  __shared__ int svis[8], snv, sblk_any[8], svis_id[8];
  __shared__ double sdl;
  __shared__ double srsq;                 // a lambda's R^2 (apart from sdl: fewer barriers)
  __shared__ int snl_final;               // fold: the source's final count
  __shared__ int sany;
  __shared__ int schg;                    // wave 0: some coordinate of block t moved
  __shared__ double slam;
  __shared__ int savail;
  __shared__ int snpass_ring[4];          // npass after lambda m, at m & 3 (fold truncation)
  int q;
  {
    int bid = blockIdx.x, nwg = gridDim.x;
    int xcd = bid & 7, qq = nwg >> 3, r = nwg & 7;
    q = ((xcd < r) ? xcd * (qq + 1) : r * (qq + 1) + (xcd - r) * qq) + (bid >> 3);
  }
  if (q >= nprob) return;
  const EnetProblem pr = probs[q];
  if (pr.ulam_src < -1) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
#if ENET_SETPRIO
  // issue priority of the recurrence wave (or all waves) over co-resident Gram waves
  if (ENET_SETPRIO == 2 || wid == 0) __builtin_amdgcn_s_setprio(3);
#endif
  const int T = (p + 63) >> 6;
  const int ldc = T * 64;
  const int cw = ldc / NW;                 // columns per wave in the pull (multiple of 8)
  const CT* Cq = C + (int64_t)pr.train * p * ldc;
  const double ysq = ys_s[(int64_t)pr.train * ny + pr.y];
  for (int k = tid; k < T * 64; k += NTH) {
    bool in = k < p;
    sg[k] = in ? gin[((int64_t)pr.train * ny + pr.y) * p + k] : 0.0;
    sa[k] = 0.0;
    svp[k] = in ? vp_in[k] : 0.0;
    sdc[k] = 0.0;
    sflag[k] = (in && ju_s[(int64_t)pr.train * p + k]) ? 1 : 0;
  }
  for (int e = tid; e < TMAX * PMAX; e += NTH) (&sds[0][0])[e] = 0.0;
  for (int k = tid; k < PMAX; k += NTH) sslot[k] = -1;
  if (tid < 8) svis_id[tid] = tid;
  if (tid == 0) { sever_n = 0; sncache = 0; spub = 0; sarr = 0; sfetch0 = 0; }
  __syncthreads();
  const int nlam = pr.ulam_src >= 0 ? L : pr.nlam_req;
  const double alf = pr.ulam_src >= 0 ? 1.0 : pow(flmin, 1.0 / (double)(nlam - 1));
  double alm = 0.0, rsq = 0.0, rsq_prev = 0.0;
  int npass = 0, m_out = 0;
  double ab = 0.0, dem = 0.0;
  double rsq_l = 0.0;
  typedef typename VecT<CT>::type V;
  constexpr int W = sizeof(V) / sizeof(CT);
  float dg_lo[32], dg_hi[32];
  int cpar = 0;                            // sCn2 buffer of the current visit's block

  // bring block t's gradient up to date (all waves); stage its diagonal block.
  // By symmetry coordinate j's contribution is the contiguous row segment C[j][t*64 .. +63].
  // fp32 C: dense pull, one column block per wave (pull_block). fp64 C: sparse pull, each
  // wave compacts the nonzero pending deltas of its share of the columns (ordered ballot)
  // and streams those segments. Wave 0 then loads its row of the 64x64 diagonal block.
  // Pull of column block jb into block tb (fp32 C):  sum_j C[j][tb*64 + r] * D_j over the
  // 64 coordinates j of block jb, D_j = Dcum_j - Dsnap_tb,j (zero for unchanged j). The
  // pull is bound by the CU's vector-memory bandwidth, so only rows with D_j != 0 are
  // fetched: none (block skipped), a compacted list (< ENET_PULL_DENSE of them), or the
  // whole 64-row block. 16-byte loads: one wave instruction fetches 4 row segments (lane
  // group g = lane/16, 4 columns per lane). Returns the sum for row r = lane (the 4 lane
  // groups combined through the wave's `sred` area).
  auto pull_block = [&](int jb, int tb) __attribute__((always_inline)) -> float {
    ATE_DASSERT(jb >= 0 && jb < T && tb >= 0 && tb < T && jb != tb);
    const int grp = lane >> 4, c4 = (lane & 15) * 4;
    const int j = jb * 64 + lane;
    const double ddj = sdc[j] - sds[tb][j];
    const uint64_t nzb = __builtin_amdgcn_ballot_w64(ddj != 0.0);
    if (!nzb) return 0.f;
    const int n = __popcll(nzb);
    const float* Cf = reinterpret_cast<const float*>(Cq) + tb * 64 + c4;
    float* dw = sdw[wid];
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    auto fma4 = [&](float4 w, float d) __attribute__((always_inline)) {
      a.x += w.x * d;
      a.y += w.y * d;
      a.z += w.z * d;
      a.w += w.w * d;
    };
    if (n >= ENET_PULL_DENSE) {
      const int r0 = jb * 64 + grp * 16;
      float4 v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int r = min(r0 + u, p - 1);  // rows >= p: finite data, zero delta
        v[u] = *reinterpret_cast<const float4*>(Cf + (int64_t)r * ldc);
      }
      dw[lane] = (float)ddj;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4 d4 = *reinterpret_cast<const float4*>(dw + grp * 16 + 4 * k);
        fma4(v[4 * k + 0], d4.x);
        fma4(v[4 * k + 1], d4.y);
        fma4(v[4 * k + 2], d4.z);
        fma4(v[4 * k + 3], d4.w);
      }
    } else {
      int* rw = srow[wid];
      const int pos = __popcll(nzb & ((1ull << lane) - 1ull));
      if (ddj != 0.0) {
        rw[pos] = j;
        dw[pos] = (float)ddj;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      constexpr int NS = (ENET_PULL_DENSE + 3) / 4;
      float4 v[NS];
      float dv[NS];
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        if (4 * u < n) {                     // uniform
          const int idx = 4 * u + grp;
          const bool ok = idx < n;
          const int ix = ok ? idx : 0;
          v[u] = *reinterpret_cast<const float4*>(Cf + (int64_t)rw[ix] * ldc);
          dv[u] = ok ? dw[ix] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < NS; ++u)
        if (4 * u < n) fma4(v[u], dv[u]);
    }
    float* red = sred[wid];
    *reinterpret_cast<float4*>(red + grp * 64 + c4) = a;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return (red[lane] + red[64 + lane]) + (red[128 + lane] + red[192 + lane]);
  };

  auto pull = [&](int t) __attribute__((always_inline)) {
    const int c0 = wid * cw;
    int cnt = 0;
    if constexpr (sizeof(CT) != 4) {
      for (int base = c0; base < c0 + cw; base += 64) {
        const int j = base + lane;
        const bool inq = j < c0 + cw;     // cw < 64 when p is small
        const double dj = inq ? sdc[j] - sds[t][j] : 0.0;
        const bool nz = dj != 0.0;
        const uint64_t bal = __ballot(nz);
        const int pos = cnt + __popcll(bal & ((1ull << lane) - 1ull));
        if (nz) { slist[c0 + pos] = j; sdelta[c0 + pos] = (CT)dj; }
        cnt += __popcll(bal);
      }
    }
    CT acc = 0;
    if constexpr (sizeof(CT) == 4) {
      // every column block but t itself (its own changes are already in g_t): wave w
      // takes the w-th of them
      const int jb = wid + (wid >= t ? 1 : 0);
      if (jb < T) acc = pull_block(jb, t);
    } else {
      const CT* colt = Cq + t * 64 + lane;
      int e = 0;
      for (; e + 16 <= cnt; e += 16) {
        CT v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = colt[(int64_t)slist[c0 + e + u] * ldc];
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += v[u] * sdelta[c0 + e + u];
      }
      for (; e < cnt; ++e) acc += colt[(int64_t)slist[c0 + e] * ldc] * sdelta[c0 + e];
    }
#ifdef ENET_PROF
    if (sizeof(CT) != 4 && lane == 0) sprof[wid][5] += (unsigned long long)cnt;
#endif
    // block t's 64x64 diagonal block -> sCn2[cpar] (wave 0 moves it into registers at the
    // start of the visit): sCn2[i * 64 + c] = C[t*64 + i][t*64 + c]. Rows >= p are clamped
    // (fp32, finite) or zero (fp64): they only ever multiply the step of a coordinate >= p,
    // which is 0.
    if constexpr (sizeof(CT) == 4) {
      for (int pc = wid; pc < 16; pc += NW) {
        const int i = pc * 4 + (lane >> 4);
        const int r = min(t * 64 + i, p - 1);
        glds16f(Cq + (int64_t)r * ldc + t * 64 + (lane & 15) * 4, &sCn2[cpar][0] + pc * 256);
      }
    } else {
      for (int i = wid; i < 64; i += NW) {
        const int r = t * 64 + i;
        sCn2[cpar][i * 64 + lane] = r < p ? (float)Cq[(int64_t)r * ldc + t * 64 + lane] : 0.f;
      }
    }
    spart2[0][wid][lane] = (double)acc;
    __syncthreads();
    if (tid < 64) {
      const int k = t * 64 + tid;
      double sp = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) sp += spart2[0][w][tid];
      sg[k] -= sp;
    }
    for (int j = tid; j < ldc; j += NTH) sds[t][j] = sdc[j];
    __syncthreads();
  };

  // Pipelined pass. Wave 0 runs the sequential recurrence of block t (diagonal block in
  // registers) and then applies block t's own deltas to block tn = next visited block
  // (contiguous row segments C[k][tn*64..]); meanwhile the pull waves (1..NW-1) pull every OTHER change
  // pending for block tn (sdc is frozen until the first barrier) and stage tn's diagonal
  // block in LDS. After the barrier wave 0 publishes block t, completes block tn's
  // gradient and snapshot, and moves tn's diagonal block into registers.
  auto pull_rest = [&](int t, int tn, int vpar) __attribute__((always_inline)) {     // waves 1..NW-1
    ATE_DASSERT(t >= 0 && t < T && tn >= 0 && tn < T);
    const int my = wid - 1;
    CT acc = 0;
    if constexpr (sizeof(CT) == 4) {
      // fp32 C: tn's diagonal block and the (t rows x tn cols) block that wave 0 needs
      // for block t's own deltas go global -> LDS by DMA (16 B per lane = 4 row segments
      // of 64 floats per wave instruction). Rows >= p are clamped (finite) and masked
      // where used.
      for (int pc = my; pc < 32; pc += NP) {
        const int blk = pc < 16 ? tn : t;
        const int i = (pc & 15) * 4 + (lane >> 4);
        const int r = min(blk * 64 + i, p - 1);
        const CT* src = Cq + (int64_t)r * ldc + tn * 64 + (lane & 15) * 4;
        float* dst = (pc < 16 ? &sCn2[cpar ^ 1][0] : sCorr) + (pc & 15) * 256;
        glds16f(src, dst);
      }
      // every column block but tn (its own changes are in g_tn already); block t's changes
      // up to this visit are pulled here (sdc is frozen until the barrier), this visit's
      // arrive through wave 0's correction. Pull wave my takes the my-th such block.
      const int jb = my + (my >= tn ? 1 : 0);
      if (jb < T) acc = pull_block(jb, tn);
    } else {
      // fp64 C: sparse pull. The pending columns of block tn (ordered ballots over all
      // column blocks) are split into NP contiguous ranges, one per pull wave.
      const int base0 = my * PER;           // private slist/sdelta region
      double dvv[TMAX];
#pragma unroll
      for (int c = 0; c < TMAX; ++c) {
        const int j = c * 64 + lane;
        dvv[c] = c < T ? sdc[j] - sds[tn][j] : 0.0;
      }
      uint64_t bals[TMAX];
      int pref[TMAX];
      int tot = 0;
#pragma unroll
      for (int c = 0; c < TMAX; ++c) {
        bals[c] = __builtin_amdgcn_ballot_w64(dvv[c] != 0.0);
        pref[c] = tot;
        tot += __popcll(bals[c]);
      }
      const int share = (tot + NP - 1) / NP;
      const int lo = my * share, hi = min(tot, lo + share);
      ATE_DASSERT(hi - lo <= PER);                       // the wave's slist2 region
      const uint64_t ltmask = (1ull << lane) - 1ull;
#pragma unroll
      for (int c = 0; c < TMAX; ++c) {
        const int pos = pref[c] + __popcll(bals[c] & ltmask);
        if (((bals[c] >> lane) & 1ull) && pos >= lo && pos < hi) {
          slist2[base0 + pos - lo] = c * 64 + lane;
          sdelta2[base0 + pos - lo] = (CT)dvv[c];
        }
      }
      const int cnt = max(0, hi - lo);
      const CT* colt = Cq + tn * 64 + lane;
      int e = 0;
      for (; e + 16 <= cnt; e += 16) {
        CT v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = colt[(int64_t)slist2[base0 + e + u] * ldc];
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += v[u] * sdelta2[base0 + e + u];
      }
      for (; e < cnt; ++e) acc += colt[(int64_t)slist2[base0 + e] * ldc] * sdelta2[base0 + e];
    }
    spart2[vpar][wid][lane] = (double)acc;
    if constexpr (sizeof(CT) == 4) return;
    // fp64 C: tn's diagonal block -> LDS (fp32) through registers, rows i = my (mod NP)
    constexpr int NR = (64 + NP - 1) / NP;
    float dr[NR];
#pragma unroll
    for (int ii = 0; ii < NR; ++ii) {
      const int i = my + NP * ii;
      const int r = tn * 64 + i;
      dr[ii] = (i < 64 && r < p) ? (float)Cq[(int64_t)r * ldc + tn * 64 + lane] : 0.f;
    }
#pragma unroll
    for (int ii = 0; ii < NR; ++ii) {
      const int i = my + NP * ii;
      if (i < 64) sCn2[cpar ^ 1][i * 64 + lane] = dr[ii];
    }
  };

  int ready = -1;   // block whose gradient and diagonal registers a pass end left current
  int nvis = 0;     // visits so far (all waves, uniform)
  int narr = 0;     // ... of them with a prefetch block (phase-B arrivals expected: NP each)
  // LDS hand-off waits (workgroup scope): spin with s_sleep until *c >= target, then acquire
  auto wait_ge = [&](int* c, int target) __attribute__((always_inline)) {
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target)
      __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };
  // Block tn's gradient is completed lazily: the visit that pulls for tn leaves the pull
  // partials (spart2[par]) and the own-delta correction partials (scorr2[par], or slot 0
  // of spart2 with fp64 C) in LDS, and the next visit's recurrence wave folds them into
  // g_tn as it loads it (one LDS round trip on wave 0 instead of a second phase-B
  // barrier). Same additions in the same order as an eager update.
  auto pending_sum = [&](int par) __attribute__((always_inline)) -> double {
    double c0 = spart2[par][0][lane];
    if constexpr (sizeof(CT) == 4) {
      float cs = 0.f;
      if (scorr_ok[par]) {
#pragma unroll
        for (int w = 0; w < NP; ++w) cs += scorr2[par][w][lane];
      }
      c0 = (double)cs;
    }
    double sp = c0;
#pragma unroll
    for (int w = 1; w < NW; ++w) sp += spart2[par][w][lane];
    return sp;
  };
  bool modeS = sizeof(CT) == 4 && ENET_MODE_S != 0;
  auto pass = [&](bool full) __attribute__((always_inline)) -> double {
    if (modeS) {
      if (wid == 0) {
        const PassS r = enet_pass_s(
            full, T, ldc, ab, dem, reinterpret_cast<const float*>(Cq), (LDS_AS double*)sg,
            (LDS_AS double*)sa, (const LDS_AS double*)svp, (LDS_AS int*)sflag,
            (LDS_AS int*)sslot, (LDS_AS float*)sccache, (LDS_AS int*)&sever_n,
            (LDS_AS int*)&sncache,
#ifdef ENET_PROF
            (LDS_AS unsigned long long*)&sprof[0][0]
#else
            nullptr
#endif
        );
        if (lane == 0) {
          sdl = r.dlx;
          rsq_l += r.rsq;
        }
      }
      __syncthreads();
      const double r = sdl;
      __syncthreads();
      return r;
    }
    double dlx_l = 0.0;
    // a full pass visits every block (no list, no barriers); an active pass the blocks
    // holding an active coordinate
    int nv = T;
    if (!full) {
      for (int t = wid; t < T; t += NW) {
        const bool a = (sflag[t * 64 + lane] & 3) == 3;
        const uint64_t b = __builtin_amdgcn_ballot_w64(a);
        if (lane == 0) sblk_any[t] = b != 0;
      }
      __syncthreads();
      if (tid == 0) {
        int c = 0;
        for (int t = 0; t < T; ++t)
          if (sblk_any[t]) svis[c++] = t;
        snv = c;
      }
      __syncthreads();
      nv = snv;
    }
    const int* vl = full ? svis_id : svis;          // identity list: written at kernel start
    if (nv == 0) {
      PROF_ADD(13, 1ull);                  // [12]: mode-L passes with visits, [13]: empty
      return 0.0;
    }
    PROF_T(tp0_);
    PROF_ADD(12, 1ull);
    if (ready != vl[0]) pull(vl[0]);       // else: brought up to date by the last visit
    ready = -1;
    PROF_T(tp1_);
    PROF_ADD(0, tp1_ - tp0_);
    PROF_ADD(8, tp1_ - tp0_);
    for (int v = 0; v < nv; ++v) {
      const int t = vl[v];
      const int vpar = v & 1;
      // the last visit prefetches block 0, the first block of the next pass whenever
      // that pass is a full pass or block 0 holds an active coordinate (checked there)
      const int tn = v + 1 < nv ? vl[v + 1] : (t != 0 ? 0 : -1);
      if (v + 1 == nv) ready = tn;
      const int k = t * 64 + lane;
      PROF_T(ta_);
      double gt = 0.0, at = 0.0, dblk = 0.0;
      CT corr = 0;                          // wave 0: block t's own deltas applied to tn
      int nc = 0;                           // wave 0: coordinates of block t that changed
      uint64_t chm = 0;                     // wave 0: their lane mask
      int fl = 0;
      // wave 0: phase-B operands that nothing changes during phase A, read now so their
      // LDS latency hides under the recurrence
      double dc0 = 0.0, ds0 = 0.0;
      if (wid == 0) {
#ifdef ENET_PROF
        const long long tv0_ = clock64();
#endif
        // this block's diagonal row into registers (deposited by the last visit's DMA or
        // by pull()): dg_lo[i] / dg_hi[i-32] = C[t*64+lane][t*64+i]
#pragma unroll
        for (int i = 0; i < 32; ++i) {
          dg_lo[i] = sCn2[cpar][i * 64 + lane];
          dg_hi[i] = sCn2[cpar][(i + 32) * 64 + lane];
        }
        dc0 = sdc[k];
        gt = sg[k];
        // Everything that does not come from the pull waves' phase B is read BEFORE the
        // arrival wait: block t's own coefficient, flag and penalty (wave 0 wrote them),
        // and the pull partials of block t (written in phase A, before the barrier), so
        // that only the phase-B correction partials and the snapshot remain after it.
        // pending_sum's additions, in its order, run after the wait.
        at = sa[k];
        const double vpt = svp[k];
        fl = sflag[k];
        const int par = vpar ^ 1;
        double pend[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) pend[w] = spart2[par][w][lane];
        const bool cok = sizeof(CT) == 4 && scorr_ok[par];
        const bool elig = (fl & 1) && (full || (fl & 2));
        const double thr_l = vpt * ab;
        const double rden = (LASSO || dem == 0.0) ? 1.0 : 1.0 / (1.0 + vpt * dem);
        // block t was the last visit's tn: its phase-B own-delta partials and snapshot come
        // from the pull waves' arrivals (no second barrier per visit)
#ifdef ENET_PROF
        const long long tw0_ = clock64();
#endif
        if (v > 0) wait_ge(&sarr, NP * narr);
#ifdef ENET_PROF
        const long long tw1_ = clock64();
        if (lane == 0) {   // prologue split: [24] before the arrival wait, [25] the wait
          sprof[wid][24] += (unsigned long long)(tw0_ - tv0_);
          sprof[wid][25] += (unsigned long long)(tw1_ - tw0_);
        }
#endif
        ds0 = sds[t][k];
        if (v > 0) {                          // == gt - pending_sum(par), same operations
          double c0 = pend[0];
          if constexpr (sizeof(CT) == 4) {
            float cs = 0.f;
            if (cok) {
#pragma unroll
              for (int w = 0; w < NP; ++w) cs += scorr2[par][w][lane];
            }
            c0 = (double)cs;
          }
          double sp = c0;
#pragma unroll
          for (int w = 1; w < NW; ++w) sp += pend[w];
          gt = gt - sp;
        }
        // Each lane changes at most once per visit (lane > last): its bookkeeping is
        // deferred (delta + the gradient it was computed from), so the loop body is the
        // bare coordinate recurrence.
        double gbef = 0.0;
        // Candidate test folded into ONE compare: a lane > last moves iff it is eligible
        // and (nonzero, or |u| > vp*lambda). `at` of a lane > last is constant during the
        // visit, so the nonzero case becomes threshold -1 (always passes) and ineligible
        // lanes get +inf; lanes <= last are cut with a scalar mask. The proposed step
        // an - at of every lane is computed alongside the ballot, so the serial chain is
        // mul -> sub -> compare/ballot -> ff1 -> readlane -> mul. Per update the loop only
        // records the new coefficient and the gradient it came from for the moving lane;
        // the delta (an - at, the same operation on the same operands as the broadcast
        // step) and the new coefficient are applied after the loop. Unrolled twice: one
        // taken branch per two updates.
        const double thr0 = elig ? (at != 0.0 ? -1.0 : thr_l) : __builtin_inf();
        uint64_t live = ~0ull, moved = 0ull;
        double anv = at;
        // u = g + a is carried instead of recomputed: a lane's a is constant while it can
        // still move (lanes <= last are cut), and u receives the same "- c*d" as g, so the
        // add drops off the serial chain. For a == 0 lanes u == g bit for bit (same ops on
        // the same values): every zero-coefficient entry test sees glmnet's gradient.
        double u = gt + at;
#ifdef ENET_PROF
        unsigned long long nupd_ = 0;
#endif
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): dg_* landed; no waits in the loop
#ifdef ENET_PROF
        const long long tloop0_ = clock64();
        if (lane == 0) sprof[wid][17] += (unsigned long long)(tloop0_ - tv0_);   // prologue cycles
        if (lane == 0) sprof[wid][26] += (unsigned long long)(tloop0_ - tw1_);   // [26] after the wait
#endif
        auto step = [&]() __attribute__((always_inline)) -> bool {
#pragma clang fp contract(off)
          const double au = fabs(u);
          const uint64_t msk = __builtin_amdgcn_ballot_w64(au > thr0) & live;
          const double an = __dmul_rn(copysign(fmax(au - thr_l, 0.0), u), rden);   // no fma: d == an - at
          const double dd = an - at;
          asm volatile("" : : "v"(dd));    // keep the step computation ahead of the branch
          if (!msk) return false;
          const int i = __ffsll((unsigned long long)msk) - 1;
          const float clo = dg_lo[i & 31], chi = dg_hi[i & 31];   // masked: stays in VGPRs
          const float ci = i < 32 ? clo : chi;
          const double d = readlane_d(dd, i);
          const bool me = lane == i;
          gbef = me ? gt : gbef;
          const double cd = (double)ci * d;
          u -= cd;
          gt -= cd;
          __builtin_amdgcn_sched_barrier(0);   // bookkeeping below stays off the chain
          live = i == 63 ? 0ull : (~0ull << (i + 1));
          moved |= 1ull << i;
          anv = me ? an : anv;
#ifdef ENET_PROF
          if (lane == 0) ++nupd_;
#endif
          return true;
        };
        // Active-set passes: every eligible lane of the block is visited in lane order,
        // unconditionally. An eligible lane the ballot form would skip (a == 0 and
        // |u| <= vp*lambda) gets an = +-0, d = +-0, and u - c*(+-0) == u: the same sequence
        // of updates, bit for bit, but the visiting order is known before the loop, so
        // the compare -> ballot -> branch -> ff1 hop leaves the serial chain (the scalar
        // unit walks the mask ahead of the vector recurrence).
        auto step_known = [&](int i) __attribute__((always_inline)) {
#pragma clang fp contract(off)
          const double au = fabs(u);
          const double an = __dmul_rn(copysign(fmax(au - thr_l, 0.0), u), rden);
          const double dd = an - at;
          const float clo = dg_lo[i & 31], chi = dg_hi[i & 31];
          const float ci = i < 32 ? clo : chi;
          const double d = readlane_d(dd, i);
          const bool me = lane == i;
          gbef = me ? gt : gbef;
          const double cd = (double)ci * d;
          u -= cd;
          gt -= cd;
          __builtin_amdgcn_sched_barrier(0);
          anv = me ? an : anv;
#ifdef ENET_PROF
          if (lane == 0) ++nupd_;
#endif
        };
        // Dense walk: when enough lanes of the block will (or may) move, visit all 64 lanes
        // in order with STATIC lane indices (fully unrolled): no mask walk, no register-
        // indexed diagonal row, readlane with an immediate lane. Ineligible lanes get
        // threshold +inf, so an = +-0 and d = +-0 - 0 (a == 0 there): a no-op, bit for bit.
        // A wave issues one instruction per ~4 cycles, so the step cost is its instruction
        // count: ~15 here against ~33 for a dynamic step (profiles/r02_enet).
        const uint64_t em = __builtin_amdgcn_ballot_w64(elig);
        const uint64_t nzm = __builtin_amdgcn_ballot_w64(elig && at != 0.0);
        const int ncand = full ? __popcll(nzm) : __popcll(em);
        auto dense_walk = [&](auto lasso_tag) __attribute__((always_inline)) {
          constexpr bool LW = decltype(lasso_tag)::value;   // lasso walk
          const double thr_e = elig ? thr_l : __builtin_inf();
          if constexpr (LW) {
            // lasso: an = u - clamp(u, -thr, thr) and d = (u - a) - clamp(u), so the serial
            // chain is max -> min -> sub -> sub -> readlane -> fma (u), and the gradient is
            // not carried per step (g = u - a_visit_start after the walk). Lane i's own
            // bookkeeping (the gradient it moved from, its new coefficient) is a function of
            // its u at step i alone, so the loop only snapshots that u (one compare + two
            // selects) and both are formed after the walk by the same operations on the
            // same value: 11 instructions per step instead of 15 (profiles/r03_enet).
            const double a0v = at;
            double usnap = u;
#if ENET_ROWWALK
            // Row-blocked order of the SAME fmas: lane k still applies d_0, d_1, ..., d_63
            // in coordinate order (fma(nc, d, u) == fma(-c, d, u) bit for bit). Row r's 16
            // coordinates are walked with exec = row r only, each step broadcasting d_i
            // inside the row by DPP64 (chain max -> min -> sub -> fmac: no readlane hop);
            // then every other row catches up on d_16r..d_16r+15 (row r replicated to all
            // rows by two permlane swaps, 16 DPP64 fmas). d_i is re-derived from lane i's
            // snapshot by the same operations as in the walk, so it is the same value.
            const int row = lane >> 4;
            auto row_pass = [&](auto r_tag) __attribute__((always_inline)) {
              constexpr int R = decltype(r_tag)::value;
              if (row == R) {
                asm volatile("s_nop 4");                 // exec write -> DPP
                static_for<16>([&](auto c_tag) __attribute__((always_inline)) {
                  constexpr int C = decltype(c_tag)::value, I = R * 16 + C;
                  const double dd = lasso_step_hw(u, a0v, -thr_e, thr_e);
                  const float ci = I < 32 ? dg_lo[I] : dg_hi[I - 32];
                  select_lane1(I, lane, usnap, u);
                  fmac_bcast<C>(u, dd, -(double)ci);
                });
              }
              const double cls = fmin(fmax(usnap, -thr_e), thr_e);
              const double rep = row_replicate<R>((usnap - a0v) - cls);
              if (row != R) {
                asm volatile("s_nop 4");
                static_for<16>([&](auto c_tag) __attribute__((always_inline)) {
                  constexpr int C = decltype(c_tag)::value, I = R * 16 + C;
                  const float ci = I < 32 ? dg_lo[I] : dg_hi[I - 32];
                  fmac_bcast<C>(u, rep, -(double)ci);
                });
              }
            };
            row_pass(std::integral_constant<int, 0>{});
            row_pass(std::integral_constant<int, 1>{});
            row_pass(std::integral_constant<int, 2>{});
            row_pass(std::integral_constant<int, 3>{});
#else
#pragma unroll
            for (int i = 0; i < 64; ++i) {
              const double cl = fmin(fmax(u, -thr_e), thr_e);
              const double dd = (u - a0v) - cl;
              const float ci = i < 32 ? dg_lo[i] : dg_hi[i - 32];
              const double d = readlane_d(dd, i);
              // in asm: left to itself the compiler materialises 64 constant lane masks in
              // SGPRs and spills them (an exec-masked v_mov_b64 instead measured 2 % slower:
              // profiles/r04_enet/snap_exec_ab.txt)
              select_lane1(i, lane, usnap, u);
              u = __builtin_fma(-(double)ci, d, u);
            }
#endif
            {
              const double cl = fmin(fmax(usnap, -thr_e), thr_e);
              gbef = usnap - a0v;
              anv = usnap - cl;
            }
            gt = u - a0v;
          } else {
#pragma unroll
            for (int i = 0; i < 64; ++i) {
#pragma clang fp contract(off)
              const double au = fabs(u);
              const double sv = copysign(fmax(au - thr_e, 0.0), u);
              const double an = __dmul_rn(sv, rden);
              const double dd = an - at;
              const float ci = i < 32 ? dg_lo[i] : dg_hi[i - 32];
              const double d = readlane_d(dd, i);
              select_lane(i, lane, gbef, gt, anv, an);
              const double cd = (double)ci * d;
              u -= cd;
              gt -= cd;
            }
          }
#ifdef ENET_PROF
          if (lane == 0) nupd_ += 64;
#endif
        };
        if (!ENET_BALLOT_ONLY && ncand >= ENET_DENSE_MIN) {
          moved = ~0ull;
          if (LASSO || dem == 0.0) dense_walk(std::true_type{});
          else if constexpr (!LASSO) dense_walk(std::false_type{});
        } else if (full || ENET_BALLOT_ONLY) {
          while (step() && step()) {
          }
        } else {
          uint64_t rem = em;
          moved = rem;
          while (rem) {
            const int i = __ffsll((unsigned long long)rem) - 1;
            rem &= rem - 1ull;
            step_known(i);
            if (!rem) break;
            const int i2 = __ffsll((unsigned long long)rem) - 1;
            rem &= rem - 1ull;
            step_known(i2);
          }
        }
#ifdef ENET_PROF
        if (lane == 0) sprof[wid][15] += (unsigned long long)(clock64() - tloop0_);
        const long long tpost0_ = clock64();
#endif
        if ((moved >> lane) & 1ull) {
          const double dn = anv - at;      // == the broadcast step d of this lane
          if (dn != 0.0) {                 // visited but not moved (active pass): keep a
            dblk = dn;
            at = anv;
          }
        }
#ifdef ENET_PROF
        if (lane == 0) {
          const unsigned long long tl_ = wall_clock64() - ta_;
          sprof[wid][6] += tl_;
          sprof[wid][7] += nupd_;

          sprof[wid][14] += 1ull;    // wave-0 visits (full + active)
        }
#endif
        if (dblk != 0.0) {
          rsq_l += dblk * (2.0 * gbef - dblk);
          dlx_l = fmax(dlx_l, dblk * dblk);
          fl |= 2;
        }
        // fp64 C: block t's own deltas -> block tn (wave-private list, contiguous segments);
        // fp32 C: wave 1 applies them from the DMA'd block in phase B
        if (sizeof(CT) != 4 && tn >= 0) {
          const bool ch = dblk != 0.0;
          const uint64_t bal = __builtin_amdgcn_ballot_w64(ch);
          const int pos = __popcll(bal & ((1ull << lane) - 1ull));
          if (ch) { scl[pos] = k; scd[pos] = (CT)dblk; }
          nc = __popcll(bal);
          chm = bal;
          const CT* colt = Cq + tn * 64 + lane;
          int e = 0;
          for (; e + 16 <= nc; e += 16) {
            CT w[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) w[u] = colt[(int64_t)scl[e + u] * ldc];
#pragma unroll
            for (int u = 0; u < 16; ++u) corr += w[u] * scd[e + u];
          }
          for (; e < nc; ++e) corr += colt[(int64_t)scl[e] * ldc] * scd[e];
        }
        if constexpr (sizeof(CT) != 4) {
          spart2[vpar][0][lane] = (double)corr;
        } else if (tn >= 0) {                  // wave 1 applies them in phase B
          sdall[lane] = (float)dblk;
          const uint64_t chg = __builtin_amdgcn_ballot_w64(dblk != 0.0);
          if (lane == 0) schg = chg != 0ull;
        }
#ifdef ENET_PROF
        if (lane == 0) sprof[wid][2] += (unsigned long long)(wall_clock64() - ta_);
        if (lane == 0) sprof[wid][28] += (unsigned long long)(clock64() - tpost0_);   // [28] post-walk
#endif
      } else if (tn >= 0) {
        // wave 0's publication of every earlier visit (Dcum of its blocks) and every pull
        // wave's last phase B (sCorr is re-filled below) must be complete
        wait_ge(&spub, nvis);
        wait_ge(&sarr, NP * narr);
        pull_rest(t, tn, vpar);
#ifdef ENET_PROF
        if (wid == 1 && lane == 0)
          sprof[wid][4] += (unsigned long long)(wall_clock64() - ta_);
        if (wid == NW - 1 && lane == 0)
          sprof[wid][18] += (unsigned long long)(wall_clock64() - ta_);
#endif
      }
#ifdef ENET_PROF
      const long long tsb_ = clock64();
#endif
      __syncthreads();
#ifdef ENET_PROF
      if (wid == 0 && lane == 0) sprof[0][27] += (unsigned long long)(clock64() - tsb_);   // [27] barrier
#endif
      PROF_T(tb_);
      PROF_ADD(1, tb_ - ta_);
      PROF_ADD(3, 1);
      // phase B: wave 0 publishes block t and moves tn's diagonal block into registers;
      // the pull waves split block t's own deltas of this visit over the rows of the DMA'd
      // (t rows x tn cols) block (fp32 C) and copy tn's snapshot. Block tn's gradient is
      // folded in by the next visit (pending_sum).
      const double dnew = dc0 + dblk;
      if (wid == 0) {
        sg[k] = gt;
        sa[k] = at;
        sflag[k] = fl;
        sdc[k] = dnew;
        sds[t][k] = ds0 + dblk;  // own changes are already in g_t
        if (tn >= 0) {
          sds[tn][k] = dnew;     // block t's columns; the pull waves copy the others
          if constexpr (sizeof(CT) == 4) {
            if (lane == 0) scorr_ok[vpar] = schg;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&spub, nvis + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef ENET_PROF
        if (lane == 0) sprof[wid][9] += (unsigned long long)(wall_clock64() - tb_);
#endif
      } else if (tn >= 0) {
        const int my = wid - 1;
        if (sizeof(CT) == 4 && schg) {
          constexpr int RPW = (64 + NP - 1) / NP;   // rows per pull wave
          float cv[RPW], dv[RPW];
#pragma unroll
          for (int j = 0; j < RPW; ++j) {
            const int r = my + NP * j;
            cv[j] = r < 64 ? sCorr[r * 64 + lane] : 0.f;
            dv[j] = r < 64 ? sdall[r] : 0.f;
          }
          float a = 0.f;
#pragma unroll
          for (int j = 0; j < RPW; ++j) a = __builtin_fmaf(cv[j], dv[j], a);
          scorr2[vpar][my][lane] = a;
        }
        // snapshot of block tn for every column block except t (unchanged this phase)
        for (int j = my * 64 + lane; j < ldc; j += NP * 64)
          if ((j >> 6) != t) sds[tn][j] = sdc[j];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_fetch_add(&sarr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef ENET_PROF
        if (wid == 1 && lane == 0) sprof[wid][16] += (unsigned long long)(wall_clock64() - tb_);
#endif
      }
      if (tn >= 0) {
        cpar ^= 1;                         // tn's diagonal block is in the other buffer
        ++narr;
      }
      ++nvis;
      PROF_T(tc_);
      PROF_ADD(0, tc_ - tb_);
    }
    if (ready >= 0) {   // the prefetched block's gradient: fold its pending partials now
      if (wid == 0) {
        wait_ge(&sarr, NP * narr);
        const int kr = ready * 64 + lane;
        sg[kr] = sg[kr] - pending_sum((nv - 1) & 1);
      }
    }
    __syncthreads();   // every phase B of the pass is complete past here
    const double dlx = wave_max(dlx_l);
    if (tid == 0) sdl = dlx;
    __syncthreads();
    // sdl's next writer is a later mode-L pass, after its own barriers (mode S never
    // follows mode L, and the lambda's R^2 goes through srsq)
    return sdl;
  };

  auto publish = [&](int v) {   // thread 0 only: agent-scope release of progress[q]
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(progress + q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // Fold problems run CONCURRENTLY with the full-data problem that defines their lambda
  // sequence: it publishes the whole sequence once lambda_max is known (lampub, release of
  // progress[q] = 2) and progress[q] = m+1 after each lambda m >= 2; a fold polls that
  // counter (relaxed, bounded spin) and acquires before reading, running up to FOLD_LEAD
  // lambdas ahead of the source, and drops what it computed past the source's final count.
  // All problems of a launch are co-resident (one workgroup per problem, grid <= #CUs); a
  // timed-out spin ends the fold path (npass_out = -1 flags it).
#ifdef ENET_PROF
  const long long kc0_ = clock64();
  const unsigned long long kw0_ = wall_clock64();
#endif
  const bool is_fold = pr.ulam_src >= 0;
  bool timed_out = false;
  int vseen = 0;            // fold, wave 0 (uniform): the source's progress last acquired
  // fold, wave 0: the source's published sequence in registers once it is out (lane l:
  // lambdas l and 64 + l; L <= 128), so a lambda needs no global load
  double lam_lo = 0.0, lam_hi = 0.0;
  bool lam_reg = false;
  for (int m = 0; m < nlam; ++m) {
#ifdef ENET_PROF
    const unsigned long long tlam0_ = wall_clock64();
#endif
    if (is_fold) {
      if (wid == 0) {
        // The source publishes its whole lambda sequence at its lambda 1 (progress 2,
        // lampub) and progress m+1 after each lambda m >= 2. A fold runs lambda m once the
        // source has finished lambda m - FOLD_LEAD (any m <= FOLD_LEAD + 1 as soon as the
        // sequence is out): it does not trail the source by a lambda, and the lambdas it
        // computes past the end of the source's path (at most FOLD_LEAD + 1) are
        // discarded after the loop. Where the source has ended (FINAL) the committed
        // lams[] values are read (the same bits as lampub).
        const int need = m <= FOLD_LEAD + 1 ? 2 : m - FOLD_LEAD + 1;
        // a value already acquired that satisfies this lambda needs no new load (the
        // source only moves forward, and what it published before it is visible)
        int v = vseen;
        if (v < need) {
          if (lane == 0) {
            for (long spin = 0;; ++spin) {
              v = __hip_atomic_load(progress + pr.ulam_src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if (v >= need) break;
              if (spin > spin_max) { v = -1; break; }
              __builtin_amdgcn_s_sleep(2);
            }
          }
          v = __builtin_amdgcn_readfirstlane(v);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (v > 0) vseen = v;
          if (v >= 2 && v < (1 << 30) && !lam_reg && L <= 128) {
            const double* lp = lampub + (int64_t)pr.ulam_src * L;
            lam_lo = lane < L ? lp[lane] : 0.0;
            lam_hi = 64 + lane < L ? lp[64 + lane] : 0.0;
            lam_reg = true;
          }
        }
        int avail = 0;
        double lv = 0.0;
        if (v < 0) {
          timed_out = true;
        } else if (v >= (1 << 30)) {
          if (lane == 0) {
            int nl = __hip_atomic_load(nlam_out + pr.ulam_src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            avail = m < nl;
            if (avail) lv = __hip_atomic_load(lams + (int64_t)pr.ulam_src * L + m, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
          }
        } else if (lam_reg) {
          avail = 1;
          lv = readlane_d(m < 64 ? lam_lo : lam_hi, m & 63);
        } else {
          avail = 1;
          if (lane == 0)
            lv = __hip_atomic_load(lampub + (int64_t)pr.ulam_src * L + m, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
          savail = avail;
          slam = lv;
        }
      }
      __syncthreads();
      const int avail = savail;
      alm = slam / ysq;     // savail / slam are next written after this lambda's barriers
      if (!avail) break;
    } else if (m == 0) {
      alm = BIGL;
    } else if (m == 1) {
      // lambda_max needs the exact current gradient of every coordinate (mode S keeps
      // every gradient exact)
      if (!modeS) {
        for (int t = 0; t < T; ++t) pull(t);
        ready = -1;
      }
      double mx = 0.0;
      for (int k = lane; k < p; k += 64)
        if ((sflag[k] & 1) && svp[k] > 0.0) mx = fmax(mx, fabs(sg[k]) / svp[k]);
      mx = wave_max(mx);      // every wave computes the same value
      alm = alf * mx / fmax(alpha, 1e-3);
      if (tid == 0 && L >= 3) {
        // the whole sequence for the fold problems, by the operations the path itself
        // uses (lams[] below): alm_m = alm_{m-1} * alf, lambda_0 extrapolated
        double* lp = lampub + (int64_t)q * L;
        double x = alm, x2 = alm;
        lp[1] = x * ysq;
        for (int mm = 2; mm < L; ++mm) {
          x *= alf;
          lp[mm] = x * ysq;
          if (mm == 2) x2 = x;
        }
        lp[0] = lambda0_extrap(lp[1], x2 * ysq);
        publish(2);
      }
    } else {
      alm *= alf;
    }
    ab = alm * alpha;
    dem = LASSO ? 0.0 : alm * (1.0 - alpha);
    // leave mode S for good once many coordinates have moved or the last lambda fetched
    // many new columns (cheap in mode L, where a new mover's row is pulled by the helpers)
    const int fetched = sncache - sfetch0;
    __syncthreads();
    if (tid == 0) sfetch0 = sncache;
    if (modeS && (sever_n > ENET_S_ENTER || fetched > ENET_S_FETCH)) {
      // to mode L for the rest of the path: every gradient is exact (Dcum = 0), so the
      // snapshots the column cache overwrote restart at zero and every block is pulled anew
      modeS = false;
      for (int e = tid; e < TMAX * PMAX; e += NTH) (&sds[0][0])[e] = 0.0;
      ready = -1;
      __syncthreads();
    }
#ifdef ENET_PROF
    const unsigned long long tpass0_ = wall_clock64();
    if (tid == 0) sprof[0][29] += tpass0_ - tlam0_;   // [29]: lambda start -> first pass
#endif
    while (npass < maxit) {
      ++npass;
      double dl = pass(true);
      if (dl < thr) break;
      while (npass < maxit) {
        ++npass;
        dl = pass(false);
        if (dl < thr) break;
      }
    }
#ifdef ENET_PROF
    const unsigned long long tpend_ = wall_clock64();
    if (tid == 0) sprof[0][5] += tpend_ - tpass0_;   // [5]: wall ticks inside passes
#endif
    double* ap = apath + ((int64_t)q * L + m) * p;
    for (int k = tid; k < p; k += NTH) ap[k] = sa[k];
    rsq = wave_sum(rsq_l);
    if (tid == 0) srsq = rsq;
    __syncthreads();
    const double rsq_all = srsq;   // srsq is next written after the next lambda's barriers
    if (tid == 0) {
      lams[(int64_t)q * L + m] = alm * ysq;
      rsqs[(int64_t)q * L + m] = rsq_all;
      if (!is_fold && m == 2)   // glmnet reports lambda_0 extrapolated from lambda_1, lambda_2
        lams[(int64_t)q * L] = lambda0_extrap(lams[(int64_t)q * L + 1], alm * ysq);
      // a count only (the folds read the sequence published at lambda 1, and lams[] only
      // after the releasing FINAL): no wait for this lambda's stores
      if (!is_fold && m >= 2)
        __hip_atomic_store(progress + q, m + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    m_out = m + 1;
    if (tid == 0) snpass_ring[m & 3] = npass;
    if (pr.ulam_src < 0 && m >= 4 && m > 0) {
      if (rsq_all - rsq_prev < 1e-5 * rsq_all || rsq_all > 0.999) break;
    }
    rsq_prev = rsq_all;
#ifdef ENET_PROF
    if (tid == 0) sprof[0][30] += wall_clock64() - tpend_;   // [30]: last pass -> lambda end
#endif
  }
  if (is_fold) {
    // lambdas computed past the end of the source's path: back to their launch state
    if (tid == 0) {
      int v = 0;
      for (long spin = 0;; ++spin) {
        v = __hip_atomic_load(progress + pr.ulam_src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v >= (1 << 30)) break;
        if (spin > spin_max) { v = -1; break; }
        __builtin_amdgcn_s_sleep(2);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (v < 0) timed_out = true;
      snl_final = v < 0 ? m_out
                     : __hip_atomic_load(nlam_out + pr.ulam_src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const int nl = snl_final;
    if (m_out > nl) {
      ATE_DASSERT(m_out - nl <= FOLD_LEAD + 1);
      for (int mm = nl; mm < m_out; ++mm) {
        double* ap = apath + ((int64_t)q * L + mm) * p;
        for (int k = tid; k < p; k += NTH) ap[k] = 0.0;
        if (tid == 0) {
          lams[(int64_t)q * L + mm] = __builtin_nan("");
          rsqs[(int64_t)q * L + mm] = 0.0;
        }
      }
      npass = nl > 0 ? snpass_ring[(nl - 1) & 3] : 0;
      m_out = nl;
    }
  }
#ifdef ENET_PROF
  __syncthreads();
  if (tid < 32) {
    unsigned long long acc = 0;
    for (int w = 0; w < NW; ++w) acc += sprof[w][tid];
    // [10] / [11]: shader clock cycles and 100 MHz wall ticks of the whole path (clock rate)
    if (tid == 10) acc = (unsigned long long)(clock64() - kc0_);
    if (tid == 11) acc = wall_clock64() - kw0_;
    atomicAdd(&enet_prof[q][tid], acc);
  }
#endif
  if (tid == 0) {
    nlam_out[q] = m_out;
    npass_out[q] = timed_out ? -1 : npass;
    if (!is_fold) publish(1 << 30);
  }
}

#ifdef ENET_PROF
extern "C" __attribute__((visibility("default"))) int ate_enet_prof_read(void* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(enet_prof), sizeof(enet_prof));
}
extern "C" __attribute__((visibility("default"))) int ate_enet_prof_reset() {
  static unsigned long long z[256][32];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(enet_prof), z, sizeof(z));
}
#endif

ATE_KERNEL_SHAPE("enet_path_kernel<float, lasso>", NTH, 0, enet_path_kernel<float, true>)
ATE_KERNEL_SHAPE("enet_path_kernel<float, enet>", NTH, 0, enet_path_kernel<float, false>)
ATE_KERNEL_SHAPE("enet_path_kernel<double, lasso>", NTH, 0, enet_path_kernel<double, true>)
ATE_KERNEL_SHAPE("enet_path_kernel<double, enet>", NTH, 0, enet_path_kernel<double, false>)

ATE_API int ate_enet_path(const void* C, int c_f32, const void* g, int p, int ny, const void* ju,
                          const void* ys, const void* vp, const void* probs, int nprob,
                          double alpha, double flmin, double thr, int maxit, void* apath,
                          void* lams, void* rsqs, void* nlam_out, void* npass_out, int L,
                          void* progress, void* lampub, void* stream) {
  if (p > PMAX) return -2;
  if (nprob > 256) return -3;   // co-residency of fold problems and their sources
  hipStream_t s = (hipStream_t)stream;
  // grid rounded up to a multiple of 8 so the XCD remap is a bijection onto [0, nwg)
  const int nwg = (nprob + 7) / 8 * 8;
  // bound of a fold problem's wait for its source's next lambda (polls of ~2 s_sleep);
  // ATE_ENET_SPIN_MAX overrides it (tests force the timeout path with 0)
  const char* sm = getenv("ATE_ENET_SPIN_MAX");
  const long spin_max = sm ? atol(sm) : (1l << 26);
#define LAUNCH_C(CTT, LS)                                                                      \
  ATE_LAUNCH((enet_path_kernel<CTT, LS>), dim3(nwg), dim3(NTH), 0, s, (const CTT*)C,   \
                     (const double*)g, p, ny, (const unsigned char*)ju, (const double*)ys,     \
                     (const double*)vp, (const EnetProblem*)probs, nprob, alpha, flmin, thr,   \
                     maxit, (double*)apath, (double*)lams, (double*)rsqs, (int*)nlam_out,     \
                     (int*)npass_out, L, (int*)progress, spin_max, (double*)lampub)
  const bool lasso = alpha == 1.0;
  if (c_f32 && lasso) LAUNCH_C(float, true);
  else if (c_f32) LAUNCH_C(float, false);
  else if (lasso) LAUNCH_C(double, true);
  else LAUNCH_C(double, false);
#undef LAUNCH_C
  ATE_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ coefficients (original scale)
// coef[q][m][0] = intercept, coef[q][m][1+j] = beta_j = a_j * ys / xs_j (0 if !ju)
__global__ void enet_coef_kernel(const double* __restrict__ apath, const EnetProblem* __restrict__ probs,
                                 int nprob, int p, int ny, int L, const int* __restrict__ nlam_out,
                                 const double* __restrict__ xm, const double* __restrict__ xs,
                                 const unsigned char* __restrict__ ju, const double* __restrict__ ym,
                                 const double* __restrict__ ys, double* __restrict__ coef) {
  const int q = blockIdx.y, m = blockIdx.x;
  if (q >= nprob || m >= L) return;
  const EnetProblem pr = probs[q];
  double* out = coef + ((int64_t)q * L + m) * (p + 1);
  if (m >= nlam_out[q]) {
    for (int j = threadIdx.x; j <= p; j += blockDim.x) out[j] = NAN;
    return;
  }
  const double* a = apath + ((int64_t)q * L + m) * p;
  const double ysq = ys[(int64_t)pr.train * ny + pr.y], ymq = ym[(int64_t)pr.train * ny + pr.y];
  __shared__ double smem[16];
  double acc[1] = {0.0};
  for (int j = threadIdx.x; j < p; j += blockDim.x) {
    int64_t sj = (int64_t)pr.train * p + j;
    double b = ju[sj] ? a[j] * ysq / xs[sj] : 0.0;
    out[1 + j] = b;
    acc[0] += b * xm[sj];
  }
  block_sum<1>(acc, smem);
  if (threadIdx.x == 0) out[0] = ymq - acc[0];
}

ATE_API int ate_enet_coef(const void* apath, const void* probs, int nprob, int p, int ny, int L,
                          const void* nlam_out, const void* xm, const void* xs, const void* ju,
                          const void* ym, const void* ys, void* coef, void* stream) {
  ATE_LAUNCH(enet_coef_kernel, dim3(L, nprob), dim3(128), 0, (hipStream_t)stream,
                     (const double*)apath, (const EnetProblem*)probs, nprob, p, ny, L,
                     (const int*)nlam_out, (const double*)xm, (const double*)xs,
                     (const unsigned char*)ju, (const double*)ym, (const double*)ys,
                     (double*)coef);
  ATE_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ K09 CV loss from held-out Gram
// For fold problem q (trained without segment hold[q]) and every lambda m:
// cvraw[q][m] = SSE / n_hold using the raw held-out Gram G[hold] (panel columns).
// Rows of the held-out Gram outside every support of the chunk are skipped (LASSO paths
// are sparse over most lambdas); a wave's next row is in flight while it applies the
// current one.
// One workgroup per (fold problem, chunk of CVL lambdas), densest chunks dispatched first:
// every entry of the held-out
// Gram is read ONCE per chunk and applied to all CVL coefficient vectors, which each lane
// keeps in registers for its own columns j = lane + 64 k (dense: zeros off the support).
// quad_m = b_m' Gxx b_m accumulates per lane as sum_a b_m[a] * sum_{j in lane} G[a][j] b_m[j];
// lin_m = b_m' Gxy, sx_m = b_m' Sx come from the same lane-owned columns.
constexpr int CVL = 8;
constexpr int CVK = PMAX / 64;

__global__ __launch_bounds__(256) void enet_cvloss_gauss_kernel(
    const double* __restrict__ G, int P, const int* __restrict__ hold,
    const int* __restrict__ xcols, int p, int ones_col, const int* __restrict__ ycol_of_prob,
    const double* __restrict__ coef, const int* __restrict__ nlam_out, int L, int q0,
    double* __restrict__ cvraw) {
  // grid (problem, chunk), chunks dispatched densest first: the last lambdas (largest
  // supports) start in the first round, so the workgroups past one round of the chip are
  // the sparse early-lambda chunks that skip most rows
  const int q = q0 + blockIdx.x, m0 = (gridDim.y - 1 - blockIdx.y) * CVL;
  const int nl = nlam_out[q];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (m0 >= nl) {
    if (tid < CVL && m0 + tid < L) cvraw[(int64_t)q * L + m0 + tid] = NAN;
    return;
  }
  const double* Gh = G + (int64_t)hold[q] * P * P;
  const int yc = ycol_of_prob[q];
  __shared__ double sbeta[CVL][PMAX];
  __shared__ int sxc[PMAX];
  __shared__ unsigned char snz[PMAX];
  __shared__ double sred[4][3 * CVL];
  for (int e = tid; e < CVL * PMAX; e += 256) {
    const int m = e / PMAX, j = e % PMAX;
    const bool ok = j < p && m0 + m < nl;
    sbeta[m][j] = ok ? coef[((int64_t)q * L + m0 + m) * (p + 1) + 1 + j] : 0.0;
  }
  for (int j = tid; j < PMAX; j += 256) sxc[j] = j < p ? xcols[j] : xcols[0];
  __syncthreads();
  for (int j = tid; j < PMAX; j += 256) {
    bool any = false;
#pragma unroll
    for (int m = 0; m < CVL; ++m) any |= sbeta[m][j] != 0.0;
    snz[j] = any;                                   // row j inside some support
  }
  __syncthreads();
  double bl[CVK][CVL];          // this lane's columns
#pragma unroll
  for (int k = 0; k < CVK; ++k)
#pragma unroll
    for (int m = 0; m < CVL; ++m) bl[k][m] = sbeta[m][k * 64 + lane];
  int cl[CVK];
#pragma unroll
  for (int k = 0; k < CVK; ++k) cl[k] = sxc[k * 64 + lane];
  double quad[CVL], lin[CVL], sx[CVL];
#pragma unroll
  for (int m = 0; m < CVL; ++m) { quad[m] = 0.0; lin[m] = 0.0; sx[m] = 0.0; }
  if (wid == 0) {
    // linear terms: b' Gxy and b' Sx over this lane's columns
#pragma unroll
    for (int k = 0; k < CVK; ++k) {
      if (k * 64 + lane >= p) continue;
      const double gy = Gh[(int64_t)cl[k] * P + yc], g1 = Gh[(int64_t)cl[k] * P + ones_col];
#pragma unroll
      for (int m = 0; m < CVL; ++m) {
        lin[m] = fma(bl[k][m], gy, lin[m]);
        sx[m] = fma(bl[k][m], g1, sx[m]);
      }
    }
  }
  // rows a = wid, wid + 4, ... inside some support of the chunk, in order; the next such
  // row's Gram entries are loaded while the current row is applied (same arithmetic)
  auto next_row = [&](int a) {
    while (a < p && !snz[a]) a += 4;
    return a;
  };
  auto load_row = [&](int a, double* g) {
    const double* Gr = Gh + (int64_t)sxc[a] * P;
#pragma unroll
    for (int k = 0; k < CVK; ++k) g[k] = (k * 64 + lane < p) ? Gr[cl[k]] : 0.0;
  };
  double gn[CVK];
  int a = next_row(wid);
  if (a < p) load_row(a, gn);
  while (a < p) {
    double g[CVK];
#pragma unroll
    for (int k = 0; k < CVK; ++k) g[k] = gn[k];
    const int an = next_row(a + 4);
    if (an < p) load_row(an, gn);
#pragma unroll
    for (int m = 0; m < CVL; ++m) {
      double t = 0.0;
#pragma unroll
      for (int k = 0; k < CVK; ++k) t = fma(g[k], bl[k][m], t);
      quad[m] = fma(sbeta[m][a], t, quad[m]);
    }
    a = an;
  }
#pragma unroll
  for (int m = 0; m < CVL; ++m) {
    quad[m] = wave_sum(quad[m]);
    lin[m] = wave_sum(lin[m]);
    sx[m] = wave_sum(sx[m]);
  }
  if (lane == 0)
#pragma unroll
    for (int m = 0; m < CVL; ++m) {
      sred[wid][m] = quad[m];
      sred[wid][CVL + m] = lin[m];
      sred[wid][2 * CVL + m] = sx[m];
    }
  __syncthreads();
  if (tid < CVL && m0 + tid < L) {
    const int m = tid;
    if (m0 + m >= nl) {
      cvraw[(int64_t)q * L + m0 + m] = NAN;
    } else {
      const double qd = sred[0][m] + sred[1][m] + sred[2][m] + sred[3][m];
      const double ln = sred[0][CVL + m], s1 = sred[0][2 * CVL + m];
      const double a0 = coef[((int64_t)q * L + m0 + m) * (p + 1)];
      const double n = Gh[(int64_t)ones_col * P + ones_col];
      const double yy = Gh[(int64_t)yc * P + yc], sy = Gh[(int64_t)ones_col * P + yc];
      const double sse = yy - 2.0 * a0 * sy - 2.0 * ln + n * a0 * a0 + 2.0 * a0 * s1 + qd;
      cvraw[(int64_t)q * L + m0 + m] = sse / n;
    }
  }
}

// q0: first problem to score (problems before it -- the full-data fits -- have no
// held-out fold); nprob: number of problems from q0.
ATE_API int ate_enet_cvloss_gauss(const void* G, int P, const void* hold, const void* xcols, int p,
                                  int ones_col, const void* ycol_of_prob, const void* coef,
                                  const void* nlam_out, int L, int q0, int nprob, void* cvraw,
                                  void* stream) {
  if (p > PMAX) return -1;
  if (nprob <= 0) return 0;
  ATE_LAUNCH(enet_cvloss_gauss_kernel, dim3(nprob, (L + CVL - 1) / CVL), dim3(256), 0,
                     (hipStream_t)stream, (const double*)G, P, (const int*)hold,
                     (const int*)xcols, p, ones_col, (const int*)ycol_of_prob,
                     (const double*)coef, (const int*)nlam_out, L, q0, (double*)cvraw);
  ATE_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ selection (cv.glmnet rules)
// For full problem f with K fold problems fold_probs[f*K + k] and fold sizes nfold[f*K+k]:
// cvm = weighted mean, cvsd = sqrt(weighted var/(K-1)); idx_min = first (largest lambda)
// attaining min cvm; idx_1se = first with cvm <= cvm[min] + cvsd[min].
// One wave per full problem; lanes own lambdas m = lane + 64 c (c < 4, L <= 256) with the
// per-lambda arithmetic of a serial scan, then wave reductions pick the first indices.
// fnp[0 .. nfp): the launch's fold-problem pass counts; any < 0 (a fold path that timed out
// waiting for its source's lambdas, enet_path_kernel) NaN-poisons cvm / cvsd (and, in
// enet_pick_kernel, the picked coefficients): device-side, capturable, no extra launches.
__device__ __forceinline__ bool any_truncated(const int* fnp, int nfp) {
  bool bad = false;
  if (fnp)
    for (int i = threadIdx.x; i < nfp; i += blockDim.x) bad |= fnp[i] < 0;
  return __syncthreads_or(bad) != 0;
}

__global__ __launch_bounds__(64) void cv_select_kernel(
    const double* __restrict__ cvraw, const int* __restrict__ fold_probs,
    const double* __restrict__ nfold, int K, int nfull, const int* __restrict__ nlam_full, int L,
    double* __restrict__ cvm, double* __restrict__ cvsd, int* __restrict__ sel,
    const int* __restrict__ fnp, int nfp) {
  const int f = blockIdx.x;
  const int lane = threadIdx.x;
  if (f >= nfull) return;
  if (any_truncated(fnp, nfp)) {
    for (int m = lane; m < L; m += 64) {
      cvm[(int64_t)f * L + m] = NAN;
      cvsd[(int64_t)f * L + m] = NAN;
    }
    if (lane == 0) { sel[2 * f] = 0; sel[2 * f + 1] = 0; }
    return;
  }
  const int nl = nlam_full[f];
  double wsum = 0.0;
  for (int k = 0; k < K; ++k) wsum += nfold[f * K + k];
  double mus[4], sds[4];
  double best = INFINITY;
  int imin = 0x7fffffff;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int m = c * 64 + lane;
    mus[c] = INFINITY;
    sds[c] = 0.0;
    if (m >= nl) continue;
    double mu = 0.0;
    for (int k = 0; k < K; ++k) mu += nfold[f * K + k] * cvraw[(int64_t)fold_probs[f * K + k] * L + m];
    mu /= wsum;
    double var = 0.0;
    for (int k = 0; k < K; ++k) {
      double d = cvraw[(int64_t)fold_probs[f * K + k] * L + m] - mu;
      var += nfold[f * K + k] * d * d;
    }
    const double sd = sqrt(var / wsum / (double)(K - 1));
    cvm[(int64_t)f * L + m] = mu;
    cvsd[(int64_t)f * L + m] = sd;
    mus[c] = mu;
    sds[c] = sd;
    if (mu < best) { best = mu; imin = m; }     // per lane: first of its own minima
  }
  // lambda.min = largest lambda attaining min(cvm) -> first index attaining the minimum
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(imin, o, 64);
    if (ob < best || (ob == best && oi < imin)) { best = ob; imin = oi; }
  }
  if (imin == 0x7fffffff) imin = 0;
  // thr1 = cvm[imin] + cvsd[imin], read from the owning lane's registers
  const int oc = imin >> 6, ol = imin & 63;
  double mine = 0.0;
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (c == oc) mine = mus[c] + sds[c];
  const double thr1 = __shfl(mine, ol, 64);
  int i1 = imin;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint64_t b = __ballot(c * 64 + lane < nl && mus[c] <= thr1);
    if (b) { i1 = c * 64 + __ffsll((unsigned long long)b) - 1; break; }
  }
  if (lane == 0) {
    sel[2 * f] = imin;
    sel[2 * f + 1] = i1;
  }
}

ATE_API int ate_cv_select(const void* cvraw, const void* fold_probs, const void* nfold, int K,
                          int nfull, const void* nlam_full, int L, void* cvm, void* cvsd, void* sel,
                          const void* fold_npass, int nfp, void* stream) {
  if (L > 256) return -1;
  ATE_LAUNCH(cv_select_kernel, dim3(nfull), dim3(64), 0, (hipStream_t)stream,
                     (const double*)cvraw, (const int*)fold_probs, (const double*)nfold, K, nfull,
                     (const int*)nlam_full, L, (double*)cvm, (double*)cvsd, (int*)sel,
                     (const int*)fold_npass, nfp);
  ATE_CHECK_LAUNCH();
  return 0;
}

// gather the selected coefficient vectors of each full problem: out_min[f][p+1] (lambda.min,
// blockIdx.y 0) and out_1se[f][p+1] (lambda.1se, blockIdx.y 1); NaN when a fold path of the
// launch was truncated (any_truncated)
__global__ void enet_pick_kernel(const double* __restrict__ coef, const int* __restrict__ sel,
                                 int p, int L, int nfull, double* __restrict__ out_min,
                                 double* __restrict__ out_1se, const int* __restrict__ fnp,
                                 int nfp) {
  const int f = blockIdx.x, which = blockIdx.y;
  double* out = which ? out_1se : out_min;
  const bool bad = any_truncated(fnp, nfp);
  const int m = sel[2 * f + which];
  for (int j = threadIdx.x; j <= p; j += blockDim.x)
    out[(int64_t)f * (p + 1) + j] = bad ? NAN : coef[((int64_t)f * L + m) * (p + 1) + j];
}

ATE_API int ate_enet_pick(const void* coef, const void* sel, int p, int L, int nfull,
                          void* out_min, void* out_1se, const void* fold_npass, int nfp,
                          void* stream) {
  ATE_LAUNCH(enet_pick_kernel, dim3(nfull, 2), dim3(128), 0, (hipStream_t)stream,
                     (const double*)coef, (const int*)sel, p, L, nfull, (double*)out_min,
                     (double*)out_1se, (const int*)fold_npass, nfp);
  ATE_CHECK_LAUNCH();
  return 0;
}
