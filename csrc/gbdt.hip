// Histogram gradient-boosted trees (extension nuisance learner, BASELINE config 5).
// Spec and numpy reference: ate_replication_causalml_amd/reference/gbdt.py.
//
// Numerics: gradients/hessians are int64 fixed point (2^-28), so every histogram sum is
// an exact integer — LDS/global atomics in any order, row shards + RCCL all-reduce (C04),
// histogram subtraction and the host reference all give the same bits. Split gains are
// compiled with -ffp-contract=off so they round exactly like numpy's.
//
// Data layout (MI355X-first, LightGBM-style):
// * bins are ROW-major uint8 [n][ldr], ldr % 32 == 0: one 128-B line holds a row's bins
//   for p <= 128, and a workgroup reading a 16-feature block reads 16 aligned bytes;
// * training rows are kept in a position array `idx` sorted by tree node (the
//   "segments"), with the fixed-point gradient pair (packed into one int64) stored in
//   the same order. After each level's split a three-kernel partition (count / scan /
//   scatter) moves (idx, gh) into child buckets — 12 B per row, bins never move;
// * a histogram workgroup = (node segment chunk, 32-feature block): 32 features x 256
//   bins x (G, H) int64 live in 128 KB of LDS (one 1024-thread workgroup per CU; GBDT_FB=16
//   builds two 64-KB workgroups per CU), feature-minor so the int64 LDS atomics are
//   bank-conflict-free; chunk c runs on XCD c % 8 with its feature blocks back to back;
//   partial images go to slabs (plain stores) and a reduce kernel
//   sums each node's slabs into H[node][c][bin][feature] — no global atomics. Only the
//   SMALLER child of each split parent is histogrammed — the sibling is parent - child
//   (histogram subtraction), so levels >= 1 touch at most half of the rows;
// * split search: workgroup = (node, 8-feature block) staged in LDS, wave = feature,
//   lane = 4 bins; a one-wave finalize picks each node's best block candidate;
// * the reduce kernel writes only the histogrammed nodes, COMPACTED: level 0 -> slot 0,
//   level d >= 1 -> slot m = the histogrammed child of parent m (Hs, nn/2 slots), so a
//   row-sharded fit all-reduces (C04) half a level's histogram bytes; an expand kernel
//   then writes the level in node order (histogrammed child = Hs[m], sibling = parent -
//   Hs[m]);
// * the whole boosting loop (grad -> per level: hist / reduce / [all-reduce] / expand /
//   split / partition -> apply) is issued from C++ on one stream by a resumable stepper
//   (ate_gbdt_run): a row-sharded fit (rule 1) returns to the caller after each level's
//   compact histogram with the element count to all-reduce; the caller enqueues the
//   collective on the same stream (torch.distributed / RCCL, no host sync) and calls
//   again. A single-device fit runs to completion in one call. Root totals come from
//   the (reduced) level-0 histogram;
// * feature-sliced C04 (world W > 1): the compact histograms are written rank-block-major
//   ([W][slot][c][bin][pw], pw = ceil(p / W) features per rank), the caller REDUCE-
//   SCATTERS them (each rank receives the sums of its own feature slice: half the ring
//   bytes of an all-reduce), expand + split search run on the slice only, and the stepper
//   pauses once more for an all-gather of the per-(node, block) candidates (32 B each);
//   the final reduction over all ranks' candidates picks the same (gain, feature, bin) as
//   a single device, so the trees stay bit-identical at every world size (the
//   data-parallel scheme of LightGBM's voting-free mode).
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "common.hpp"

namespace {

constexpr int NT = 256;
#ifndef GBDT_FB
#define GBDT_FB 32
#endif
// features per histogram workgroup: 16 (512 threads, 64-KB LDS image, two workgroups per
// CU) or 32 (1024 threads, one 128-KB image per CU: half the workgroups per row chunk share
// each 128-B bin line, and idx / gh are loaded half as often)
constexpr int FB = GBDT_FB;
static_assert(FB == 16 || FB == 32, "GBDT_FB: 16 or 32");
constexpr int NTH = FB * 32;         // histogram workgroup: FB / 4 lanes per row, 16 waves per CU
constexpr int FQ = FB / 4;           // dwords (lanes) per row
constexpr int SFB = 8;               // features per split-search workgroup (one per wave)
constexpr int HS = 257;              // padded bins per (feature, channel) in LDS
constexpr int MAXD = 8;              // max tree depth (levels 0 .. MAXD - 1 histogrammed)
constexpr int MAXN = 1 << (MAXD - 1);  // max nodes of a histogrammed level (128)
constexpr int MAXM = (1 << (MAXD + 1)) - 1;   // max nodes of a tree (511)
constexpr int MAXB = MAXN + 1;       // partition buckets (partitions follow levels <= MAXD - 2:
                                     // 2 * 64 children) + retired; fits the uint8 bucket ids
constexpr double GFIX = 268435456.0;   // 2^28

typedef unsigned long long u64;

// One int64 per row carries the fixed-point pair: squared loss -> G (H is exactly 2^28);
// logistic -> (int32 G, int32 H) since |g| < 1 and h <= 1/4 (|G| <= 2^28, H <= 2^26).
__device__ __forceinline__ int64_t gbdt_pack(int loss, int64_t G, int64_t H) {
  return loss == 0 ? G : (int64_t)(((uint64_t)(uint32_t)H << 32) | (uint32_t)(int32_t)G);
}
__device__ __forceinline__ void gbdt_unpack(int loss, int64_t v, u64& g, u64& h) {
  if (loss == 0) {
    g = (u64)v;
    h = (u64)268435456;                                      // 2^28
  } else {
    g = (u64)(int64_t)(int32_t)(uint32_t)v;
    h = (u64)((uint64_t)v >> 32);
  }
}

// g, h of the loss at the current raw score for the training positions [0, n_train)
// (4 positions per thread, loads batched); level-0 segment = [0, n_train). The root
// totals are taken from the level-0 histogram (gbdt_root_kernel).
__global__ __launch_bounds__(NT) void gbdt_grad_kernel(int loss, const double* __restrict__ f,
                                                       const double* __restrict__ y,
                                                       const int32_t* __restrict__ idx,
                                                       int64_t n_train, int64_t* __restrict__ gh,
                                                       int32_t* __restrict__ seg,
                                                       int64_t* __restrict__ gh2 = nullptr) {
  if (blockIdx.x == 0 && threadIdx.x == 0) { seg[0] = 0; seg[1] = (int32_t)n_train; }
  const int64_t q0 = (blockIdx.x * (int64_t)NT * 4) + threadIdx.x;
  int32_t ii[4];
  double fv[4], yv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) ii[u] = idx[min(q0 + u * NT, n_train - 1)];
#pragma unroll
  for (int u = 0; u < 4; ++u) { fv[u] = f[ii[u]]; yv[u] = y[ii[u]]; }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t q = q0 + u * NT;
    if (q >= n_train) continue;
    double g, h;
    if (loss == 0) {
      g = fv[u] - yv[u];
      h = 1.0;
    } else {
      const double s = 1.0 / (1.0 + exp(-fv[u]));
      g = s - yv[u];
      h = fmax(s * (1.0 - s), 1e-16);
    }
    const int64_t v = gbdt_pack(loss, llrint(g * GFIX), llrint(h * GFIX));
    gh[q] = v;
    if (gh2) gh2[2 * q] = v;      // the fused root pass's interleaved (fit A, fit B) pairs
  }
}

// root totals = the level-0 histogram of feature 0 summed over its bins (every training
// row is in exactly one bin), exact and already reduced over row shards
__global__ __launch_bounds__(NT) void gbdt_root_kernel(const int64_t* __restrict__ H, int p,
                                                       int64_t* __restrict__ tot) {
  __shared__ int64_t red[2][NT / 64];
  int64_t a = H[(int64_t)threadIdx.x * p], b = H[(int64_t)(256 + threadIdx.x) * p];
  a = ate::wave_sum(a);
  b = ate::wave_sum(b);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { red[0][wid] = a; red[1][wid] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t sa = 0, sb = 0;
    for (int w = 0; w < NT / 64; ++w) { sa += red[0][w]; sb += red[1][w]; }
    tot[0] = sa;
    tot[1] = sb;
  }
}

// Which nodes of level d get a histogram of their own: the root, and for every split
// parent the child with fewer rows (rule 0, single rank: segment lengths) or with the
// smaller hessian total (rule 1, row shards: tot[] is identical on every rank, so all
// ranks histogram the same child). Ties -> left child.
__device__ __forceinline__ bool gbdt_computed(int k, int d, const int32_t* seg,
                                              const int64_t* tot, int rule) {
  if (d == 0) return true;
  const int sib = k ^ 1;
  int64_t a, b;
  if (rule == 0) {
    a = seg[k + 1] - seg[k];
    b = seg[sib + 1] - seg[sib];
  } else {
    const int hk = (1 << d) - 1;
    a = tot[2 * (hk + k) + 1];
    b = tot[2 * (hk + sib) + 1];
  }
  return a < b || (a == b && !(k & 1));
}

// Work plan of a level's histogram: computed nodes are cut into chunks of CH positions;
// chunk i of node k is global chunk acc[k] + i. Filled by thread 0 into LDS.
__device__ void gbdt_plan(const int* sseg, const int64_t* tot, int rule, int nn, int d,
                          int64_t CH, int* acc, int* nch) {
  int a = 0;
  for (int k = 0; k < nn; ++k) {
    const int64_t len = sseg[k + 1] - sseg[k];
    const int c = (len > 0 && gbdt_computed(k, d, sseg, tot, rule)) ? (int)((len + CH - 1) / CH)
                                                                     : 0;
    acc[k] = a;
    nch[k] = c;
    a += c;
  }
  acc[nn] = a;
}

constexpr int SLAB = 2 * 256 * FB;   // one workgroup's histogram image, u64 entries

// Partial histograms: workgroup = (chunk of a computed node's segment, 32-feature block),
// LDS image [bin][c][slot(f)] (feature-minor, see the lane map below: the int64 LDS
// atomics are bank-conflict-free whatever the bins are). The image goes to slab
// `logical` with plain 16-B stores; gbdt_hist_reduce_kernel sums a node's slabs.
// 1-D grid, chunk-to-XCD mapped (below) so the feature blocks of one chunk share an XCD's L2.
// ABL: the profiling ablation build (ATE_GBDT_HIST_MODE != 0); the production
// instantiation compiles the mode tests out of the atomic loop (they were uniform branches
// plus scalar bookkeeping around every LDS atomic).
template <bool ABL>
__global__ __launch_bounds__(NTH) void gbdt_hist_kernel(
    const uint8_t* __restrict__ Xr, int64_t ldr, const int32_t* __restrict__ idx,
    const int64_t* __restrict__ gh, const int32_t* __restrict__ seg, const int64_t* tot,
    int rule, int nn, int p, int d, int64_t CH, int ydim, u64* __restrict__ slab, int mode_in,
    int loss) {
  const int mode = ABL ? mode_in : 0;
  __shared__ u64 sh[SLAB];
  __shared__ int sseg[MAXN + 1], sacc[MAXN + 1], snch[MAXN];
  __shared__ int64_t wk[3];
  const int bid = blockIdx.x;
  // Chunk c runs on XCD c % 8 (dispatch sends block b to XCD b % 8), its ydim feature
  // blocks back to back there (they share the chunk's bin lines through that XCD's L2).
  // Chunks are numbered over the level's histogrammed nodes only, so the spare
  // workgroups of an upper-bound grid are the highest chunks of EVERY XCD: a level that
  // histograms half of the rows keeps all 8 XCDs busy (a chunk-major order put all the
  // spare workgroups, half the grid below the root, on XCDs 4-7).
  // G == 8 * ceil(chunks / 8) * ydim (gbdt_hist_geom).
  const int xq = bid >> 3;
  const int chunk = (xq / ydim) * 8 + (bid & 7), yb = xq % ydim;
  const int logical = chunk * ydim + yb;
  if (threadIdx.x <= nn) sseg[threadIdx.x] = seg[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    gbdt_plan(sseg, tot, rule, nn, d, CH, sacc, snch);
    wk[0] = -1;
    for (int k = 0; k < nn; ++k)
      if (chunk >= sacc[k] && chunk < sacc[k] + snch[k]) {
        wk[0] = k;
        wk[1] = sseg[k] + (int64_t)(chunk - sacc[k]) * CH;
        wk[2] = min((int64_t)sseg[k + 1], wk[1] + CH);
      }
  }
  __syncthreads();
  if (wk[0] < 0) return;                                    // uniform: spare workgroup
  const int64_t s = wk[1], e = wk[2];
  const int j0 = yb * FB, nf = min(FB, p - j0);
  ATE_DASSERT(wk[0] < nn && sseg[wk[0]] <= s && s <= e && e <= sseg[wk[0] + 1] && nf > 0);
  {
    ulonglong2* z = reinterpret_cast<ulonglong2*>(sh);
    for (int t = threadIdx.x; t < SLAB / 2; t += NTH) z[t] = make_ulonglong2(0, 0);
  }
  __syncthreads();
  // lane = (row r16 of 64 / FQ, word l4 of FQ): the lane reads the dword of features
  // 4*l4..+3 of its row. LDS slot of local feature f: (f & 3) * FQ + (f >> 2), so feature
  // 4*l4 + q sits on bank pair FQ*q + l4; row r walks q in the order rotated by r & 3, so
  // the four consecutive rows of a lane group use distinct bank pairs: the int64 atomics
  // are conflict-free whatever the bins are.
  const int l4 = threadIdx.x % FQ, r16 = (threadIdx.x / FQ) % (64 / FQ), w = threadIdx.x >> 6;
  const int rot = r16 & 3;
  const uint32_t* xw = reinterpret_cast<const uint32_t*>(Xr + j0) + l4;   // in the row
  const int64_t ldw = ldr >> 2;
  // rows of iteration `base`: base + (u*8 + w)*16 + r16; software pipeline: positions of
  // iteration i+2 and (g, h, bins) of iteration i+1 are in flight while iteration i's
  // atomics run. Loads are unconditional (positions past the segment are clamped to its
  // last row; words past p read row padding), so no branch forces a vmcnt(0) per row.
#ifndef GBDT_U
#define GBDT_U 8
#endif
  constexpr int U = GBDT_U, RPI = U * (NTH / FQ);
  // (g, h) stay packed (one int64 per row) until the atomics: half the VGPRs of two
  // unpacked u64 per row (U = 12 fits without spills but was not faster)
  int32_t iiA[U], iiB[U];
  int64_t gA[U];
  uint32_t bA[U];
  // positions are int32 (a fit holds < 2^31 training rows): half the address VALU of int64
  const int s32 = (int)s, e32 = (int)e, last = e32 - 1;
  const bool wok = 4 * l4 < nf;
  auto pos = [&](int base, int u) { return base + (u * (NTH / 64) + w) * (64 / FQ) + r16; };
#pragma unroll
  for (int u = 0; u < U; ++u) iiA[u] = idx[min(pos(s32, u), last)];
#pragma unroll
  for (int u = 0; u < U; ++u) iiB[u] = idx[min(pos(s32 + RPI, u), last)];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    gA[u] = gh[min(pos(s32, u), last)];
    bA[u] = (mode & 2) ? (uint32_t)iiA[u] * 0x9E3779B1u : xw[(int64_t)iiA[u] * ldw];
  }
  u64 dummy = 0;
  // One pipelined iteration. TAIL: positions may pass the segment end (clamped loads, rows
  // past it skipped); the main loop runs only while iterations i .. i+2 lie inside it, so it
  // carries no clamps and no per-row range test.
  auto step = [&](int base, auto tail_tag) __attribute__((always_inline)) {
    constexpr bool TAIL = decltype(tail_tag)::value;
    auto at = [&](int q) { return TAIL ? min(q, last) : q; };
    int64_t gB[U];
    uint32_t bB[U];
    int32_t iiC[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      gB[u] = gh[at(pos(base + RPI, u))];
      bB[u] = (mode & 2) ? (uint32_t)iiB[u] * 0x9E3779B1u : xw[(int64_t)iiB[u] * ldw];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) iiC[u] = idx[at(pos(base + 2 * RPI, u))];
    if (mode & 1) {
#pragma unroll
      for (int u = 0; u < U; ++u) dummy += (u64)gA[u] * bA[u];
    } else if (wok) {                                       // padding words add nothing
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (TAIL && pos(base, u) > last) continue;          // rows past the segment
        u64 gu, hu;
        gbdt_unpack(loss, gA[u], gu, hu);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int q = (k + rot) & 3;
          // bit-field extract + shift-or: 2 VALU per byte for the address (was 3)
          const uint32_t bin = __builtin_amdgcn_ubfe(bA[u], 8 * q, 8);
          // image [bin][G, H][slot]: H sits 8 * FB bytes after G, inside the DS offset field
          u64* e0 = sh + ((bin * 2 * FB) | (q * FQ + l4));
          atomicAdd(e0, gu);
          if (mode & 8) continue;                             // ablation: G only
          if (mode & 16)                                      // ablation: H as a u32 add
            atomicAdd(reinterpret_cast<unsigned*>(e0 + FB), (unsigned)hu);
          else
            atomicAdd(e0 + FB, hu);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      iiA[u] = iiB[u];
      gA[u] = gB[u];
      bA[u] = bB[u];
      iiB[u] = iiC[u];
    }
  };
  int base = s32;
  for (; base + 3 * RPI <= e32; base += RPI) step(base, std::false_type{});
  for (; base < e32; base += RPI) step(base, std::true_type{});
  if (dummy == 0x123456789ull) sh[0] = dummy;
  __syncthreads();
  if (mode & 4) return;
  ulonglong2* dst = reinterpret_cast<ulonglong2*>(slab + (int64_t)logical * SLAB);
  const ulonglong2* src = reinterpret_cast<const ulonglong2*>(sh);
  for (int t = threadIdx.x; t < SLAB / 2; t += NTH) dst[t] = src[t];
}

// Hs[slot][c][b][j] (feature-minor) = sum of the slabs of histogrammed node k, slot 0 at
// the root, slot k >> 1 below (the histogrammed child of parent k >> 1; gbdt_expand_kernel
// puts the level in node order). Nodes without a histogram of their own write nothing.
// Feature-sliced layout (nr > 1 rank blocks of pw features, nr * pw >= p): entry (slot, c,
// bin, j) goes to block r = j / pw at ((r * nsl + slot) * 512 + cb) * pw + j - r * pw
// (nsl = slots of this level), the padding features past p are written as zeros; nr = 1,
// pw = p is the plain [slot][c][b][j] image.
__global__ __launch_bounds__(NT) void gbdt_hist_reduce_kernel(
    const u64* __restrict__ slab, const int32_t* __restrict__ seg, const int64_t* tot, int rule,
    int nn, int p, int d, int64_t CH, int ydim, int64_t* __restrict__ Hs, int nr, int pw) {
  __shared__ int sseg[MAXN + 1], sacc[MAXN + 1], snch[MAXN];
  const int k = blockIdx.y;
  if (threadIdx.x <= nn) sseg[threadIdx.x] = seg[threadIdx.x];
  __syncthreads();
  if (d > 0 && !gbdt_computed(k, d, sseg, tot, rule)) return;   // uniform per workgroup
  if (threadIdx.x == 0) gbdt_plan(sseg, tot, rule, nn, d, CH, sacc, snch);
  __syncthreads();
  const int a = sacc[k], c = snch[k];
  const int P = nr * pw;                                    // padded feature count
  const int64_t per = 512LL * P;
  const int slot = d == 0 ? 0 : (k >> 1), nsl = d == 0 ? 1 : nn >> 1;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < per; t += (int64_t)gridDim.x * NT) {
    const int cb = (int)(t / P), j = (int)(t - (int64_t)cb * P);
    const int r = j / pw;
    int64_t* dst = Hs + ((int64_t)(r * nsl + slot) * 512 + cb) * pw + (j - r * pw);
    if (j >= p) {
      *dst = 0;
      continue;
    }
    const int yb = j / FB, fl = j - yb * FB;
    // slab image [bin][channel][slot] (gbdt_hist_kernel); Hs is [channel][bin][feature]
    const int bc = ((cb & 255) << 1) | (cb >> 8);
    const u64* sp = slab + ((int64_t)a * ydim + yb) * SLAB + bc * FB + ((fl & 3) * FQ + (fl >> 2));
    const int64_t stride = (int64_t)ydim * SLAB;
    u64 v0 = 0, v1 = 0, v2 = 0, v3 = 0;
    int i = 0;
    for (; i + 4 <= c; i += 4) {
      v0 += sp[i * stride];
      v1 += sp[(i + 1) * stride];
      v2 += sp[(i + 2) * stride];
      v3 += sp[(i + 3) * stride];
    }
    for (; i < c; ++i) v0 += sp[i * stride];
    *dst = (int64_t)(v0 + v1 + v2 + v3);
  }
}

// ---- fused root histogram of two fits on the same training rows (ate_gbdt_pair_root) ----
// A fold's E[Y|X] and E[W|X] fits (config 5) histogram the same rows at level 0; trained in
// lockstep, tree by tree, one pass reads each row's bins once for both and accumulates four
// channels (G_A, H_A, G_B, H_B). 16 features per workgroup keep the four-channel image at
// 128 KB of LDS: [bin][channel][slot(f)], slot(f) = (f & 3) * FQ2 + (f >> 2). Lane = (row r16
// of 16, dword l4 of 4). A u64 atomic lands on banks 2 (16 ch + 4 q + l4) mod 64 = 32 (ch & 1)
// + 8 q + 2 l4: in a 32-lane group (8 rows) the rotation rot = r16 & 3 separates 4 rows
// through q, and the other 4 (bsw = (r16 >> 2) & 1) add the channel of the opposite parity
// first (H before G), so every atomic instruction is conflict-free whatever the bins. The
// integer sums are the two separate passes' bits (profiles/r06_cfg5: the separate pass is
// latency-bound between its bin gathers and the LDS atomic queue, LDS array 52 % busy).
constexpr int FB2 = 16, FQ2 = FB2 / 4, NTH2 = 1024;
constexpr int SLAB2 = 4 * 256 * FB2;   // u64 entries of one workgroup's image (128 KB)
#ifndef GBDT_U2
#define GBDT_U2 4
#endif

// gh2: the two fits' packed (g, h) of position q at gh2[2q], gh2[2q + 1] (one 16-byte load).
// RANGES: the training rows are rows a0 .. a0 + n0 - 1 then a1 .. (a DML fold's complement
// on a fold-segmented panel): the row of a position is computed, no idx load.
template <bool RANGES>
__global__ __launch_bounds__(NTH2) void gbdt_hist2_kernel(
    const uint8_t* __restrict__ Xr, int64_t ldr, const int32_t* __restrict__ idx,
    const longlong2* __restrict__ gh2, int a0, int n0, int a1, int n_train, int p, int CH,
    int nchunk, int ydim2, u64* __restrict__ slab, int lossA, int lossB) {
  __shared__ u64 sh[SLAB2];
  const int bid = blockIdx.x;
  // chunk c on XCD c % 8 with its ydim2 feature blocks back to back (gbdt_hist_kernel)
  const int xq = bid >> 3;
  const int chunk = (xq / ydim2) * 8 + (bid & 7), yb = xq % ydim2;
  if (chunk >= nchunk) return;                               // uniform: spare workgroup
  const int s = chunk * CH, e = min(n_train, s + CH);
  const int j0 = yb * FB2, nf = min(FB2, p - j0);
  ATE_DASSERT(s < e && nf > 0 && yb < ydim2);
  {
    ulonglong2* z = reinterpret_cast<ulonglong2*>(sh);
    for (int t = threadIdx.x; t < SLAB2 / 2; t += NTH2) z[t] = make_ulonglong2(0, 0);
  }
  __syncthreads();
  const int l4 = threadIdx.x % FQ2, r16 = (threadIdx.x / FQ2) % 16, w = threadIdx.x >> 6;
  const int rot = r16 & 3, bsw = (r16 >> 2) & 1;
  const uint32_t* xw = reinterpret_cast<const uint32_t*>(Xr + j0) + l4;
  const int64_t ldw = ldr >> 2;
  constexpr int U = GBDT_U2, RPI = U * (NTH2 / FQ2);
  const int last = e - 1;
  const bool wok = 4 * l4 < nf;
  auto pos = [&](int base, int u) { return base + (u * (NTH2 / 64) + w) * 16 + r16; };
  auto row_of = [&](int q) { return q < n0 ? a0 + q : a1 + (q - n0); };
  // software pipeline as gbdt_hist_kernel: positions two iterations ahead (idx path), (g, h,
  // bins) one
  int32_t iiA[U], iiB[U];
  longlong2 gA[U];
  uint32_t bA[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    iiA[u] = RANGES ? row_of(min(pos(s, u), last)) : idx[min(pos(s, u), last)];
    iiB[u] = RANGES ? row_of(min(pos(s + RPI, u), last)) : idx[min(pos(s + RPI, u), last)];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    gA[u] = gh2[min(pos(s, u), last)];
    bA[u] = xw[(int64_t)iiA[u] * ldw];
  }
  auto step = [&](int base, auto tail_tag) __attribute__((always_inline)) {
    constexpr bool TAIL = decltype(tail_tag)::value;
    auto at = [&](int q) { return TAIL ? min(q, last) : q; };
    longlong2 nA[U];
    uint32_t bB[U];
    int32_t iiC[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      nA[u] = gh2[at(pos(base + RPI, u))];
      bB[u] = xw[(int64_t)iiB[u] * ldw];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      iiC[u] = RANGES ? row_of(at(pos(base + 2 * RPI, u))) : idx[at(pos(base + 2 * RPI, u))];
    if (wok) {                                                // padding words add nothing
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (TAIL && pos(base, u) > last) continue;            // rows past the chunk
        u64 ga, ha, gb, hb;
        gbdt_unpack(lossA, gA[u].x, ga, ha);
        gbdt_unpack(lossB, gA[u].y, gb, hb);
        const u64 x0 = bsw ? ha : ga, x1 = bsw ? ga : ha;
        const u64 x2 = bsw ? hb : gb, x3 = bsw ? gb : hb;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int q = (k + rot) & 3;
          const uint32_t bin = __builtin_amdgcn_ubfe(bA[u], 8 * q, 8);
          u64* e0 = sh + ((bin * 4 * FB2) | (q * FQ2 + l4));
          u64* pa = e0 + bsw * FB2;                           // channel bsw (then 2 + bsw)
          u64* pb = e0 + (bsw ^ 1) * FB2;                     // channel 1 - bsw (then 3 - bsw)
          atomicAdd(pa, x0);
          atomicAdd(pb, x1);
          atomicAdd(pa + 2 * FB2, x2);
          atomicAdd(pb + 2 * FB2, x3);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      iiA[u] = iiB[u];
      gA[u] = nA[u];
      bA[u] = bB[u];
      iiB[u] = iiC[u];
    }
  };
  int base = s;
  for (; base + 3 * RPI <= e; base += RPI) step(base, std::false_type{});
  for (; base < e; base += RPI) step(base, std::true_type{});
  __syncthreads();
  ulonglong2* dst = reinterpret_cast<ulonglong2*>(slab + ((int64_t)chunk * ydim2 + yb) * SLAB2);
  const ulonglong2* src = reinterpret_cast<const ulonglong2*>(sh);
  for (int t = threadIdx.x; t < SLAB2 / 2; t += NTH2) dst[t] = src[t];
}

// Root histograms of both fits from the fused images: fit m (blockIdx.y) gets channels 2m
// (G) and 2m + 1 (H), summed over the chunks, in gbdt_hist_reduce_kernel's compact layout
// (slot 0; rank-block-major [nr][1][512][pw] when feature-sliced).
__global__ __launch_bounds__(NT) void gbdt_hist2_reduce_kernel(
    const u64* __restrict__ slab, int nchunk, int p, int ydim2, int64_t* __restrict__ HsA,
    int64_t* __restrict__ HsB, int nr, int pw) {
  const int m = blockIdx.y;
  int64_t* Hs = m ? HsB : HsA;
  const int P = nr * pw;
  const int64_t per = 512LL * P;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < per; t += (int64_t)gridDim.x * NT) {
    const int cb = (int)(t / P), j = (int)(t - (int64_t)cb * P);
    const int r = j / pw;
    int64_t* dst = Hs + ((int64_t)r * 512 + cb) * pw + (j - r * pw);
    if (j >= p) {
      *dst = 0;
      continue;
    }
    const int yb = j / FB2, fl = j - yb * FB2;
    const int ch = 2 * m + (cb >> 8), bin = cb & 255;
    const u64* sp = slab + (int64_t)yb * SLAB2 + (bin * 4 + ch) * FB2 + ((fl & 3) * FQ2 + (fl >> 2));
    const int64_t stride = (int64_t)ydim2 * SLAB2;
    u64 v0 = 0, v1 = 0, v2 = 0, v3 = 0;
    int i = 0;
    for (; i + 4 <= nchunk; i += 4) {
      v0 += sp[i * stride];
      v1 += sp[(i + 1) * stride];
      v2 += sp[(i + 2) * stride];
      v3 += sp[(i + 3) * stride];
    }
    for (; i < nchunk; ++i) v0 += sp[i * stride];
    *dst = (int64_t)(v0 + v1 + v2 + v3);
  }
}

// level d in node order from the compact (all-reduced) histograms: the root is Hs[0];
// below, for every split parent m the histogrammed child is Hs[m] and its sibling is
// parent - Hs[m] (histogram subtraction, exact in integers)
__global__ __launch_bounds__(NT) void gbdt_expand_kernel(const int64_t* __restrict__ Hs,
                                                         const int64_t* __restrict__ Hp,
                                                         int64_t* __restrict__ Hc,
                                                         const int32_t* __restrict__ seg,
                                                         const int64_t* __restrict__ tot,
                                                         const int32_t* __restrict__ feat,
                                                         int rule, int p, int d) {
  const int m = blockIdx.y;                                 // parent index at level d-1
  const int64_t per = (int64_t)p * 512;
  const int64_t* S = Hs + m * per;
  if (d == 0) {
    for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < per; t += (int64_t)gridDim.x * NT)
      Hc[t] = S[t];
    return;
  }
  if (feat[(1 << (d - 1)) - 1 + m] < 0) return;
  const int small = gbdt_computed(2 * m, d, seg, tot, rule) ? 2 * m : 2 * m + 1;
  const int big = small ^ 1;
  const int64_t* P = Hp + m * per;
  int64_t* Cs = Hc + small * per;
  int64_t* B = Hc + big * per;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < per; t += (int64_t)gridDim.x * NT) {
    const int64_t v = S[t];
    Cs[t] = v;
    B[t] = P[t] - v;
  }
}

struct Best {
  double gain;
  int j, b;
};

__device__ __forceinline__ bool better(double g, int j, int b, const Best& o) {
  if (g > o.gain) return true;
  if (g < o.gain || !(g == g)) return false;
  return j < o.j || (j == o.j && b < o.b);
}

constexpr int NTS = 512;   // split search workgroup: one wave per feature of an 8-feature block

struct Cand {               // best split of one (node, feature block)
  double gain;
  int j, b;
  int64_t gl, hl;
};
static_assert(sizeof(Cand) == 32, "Cand: 32 B (models/gbdt.py sizes cand as 4 int64 each)");

// grid (node, 8-feature block): the block's histograms are staged feature-major in LDS
// ([c][f][bin], so a lane's 4 consecutive bins are two 16-B reads); wave = feature,
// lane = 4 bins: lane totals, in-wave exclusive scan, running prefix and the gains of
// the 4 split points (ascending bins, strict > keeps the lowest on ties), wave argmax
// (gain desc, feature asc, bin asc); the workgroup's best goes to cand[node][block].
// H has row stride p and holds features [joff, joff + pc) (a rank's slice; pc <= p, the
// slice's blocks past pc yield -inf candidates); candidates carry GLOBAL feature indices.
__global__ __launch_bounds__(NTS) void gbdt_split_search_kernel(
    const int64_t* __restrict__ H, int p, int pc, int joff, int d, int depth, double lam,
    int64_t min_child, const int64_t* __restrict__ tot, const int32_t* __restrict__ feat,
    Cand* __restrict__ cand) {
  __shared__ __attribute__((aligned(16))) int64_t sh[2 * SFB * 256];
  __shared__ Cand wb[NTS / 64];
  const int k = blockIdx.x, yb = blockIdx.y, ydim = gridDim.y;
  const int hk = (1 << d) - 1 + k;
  if (d >= depth || (d > 0 && feat[(hk - 1) / 2] < 0)) return;
  const int j0 = yb * SFB, nf = min(SFB, pc - j0);
  const int64_t* Hk = H + (int64_t)k * 512 * p + j0;
  {
    constexpr int PER = 2 * SFB * 256 / NTS;                // entries per thread
    const int fl = threadIdx.x & (SFB - 1), fc = max(0, min(fl, nf - 1));
    int64_t v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int cb = (threadIdx.x + i * NTS) / SFB;
      v[i] = Hk[(int64_t)cb * p + fc];
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int cb = (threadIdx.x + i * NTS) / SFB;
      sh[((cb >> 8) * SFB + fl) * 256 + (cb & 255)] = v[i];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, f = threadIdx.x >> 6;
  const int64_t G = tot[2 * hk], Hh = tot[2 * hk + 1];
  const double gf = (double)G / GFIX, hf = (double)Hh / GFIX;
  const double parent = gf * gf / (hf + lam);
  Cand lb{-INFINITY, joff + j0 + f, 0x7fffffff, 0, 0};
  if (f < nf) {                                             // uniform per wave
    const longlong2* pg = reinterpret_cast<const longlong2*>(sh + f * 256 + 4 * lane);
    const longlong2* ph = reinterpret_cast<const longlong2*>(sh + (SFB + f) * 256 + 4 * lane);
    const longlong2 g01 = pg[0], g23 = pg[1], h01 = ph[0], h23 = ph[1];
    const int64_t gv[4] = {g01.x, g01.y, g23.x, g23.y}, hv[4] = {h01.x, h01.y, h23.x, h23.y};
    const int64_t sg = gv[0] + gv[1] + gv[2] + gv[3], sh2 = hv[0] + hv[1] + hv[2] + hv[3];
    int64_t eg = sg, eh = sh2;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t tg = __shfl_up(eg, o, 64), th = __shfl_up(eh, o, 64);
      if (lane >= o) { eg += tg; eh += th; }
    }
    int64_t GL = eg - sg, HL = eh - sh2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      GL += gv[i];
      HL += hv[i];
      if (HL >= min_child && Hh - HL >= min_child) {
        const double glf = (double)GL / GFIX, hlf = (double)HL / GFIX;
        const double grf = gf - glf, hrf = hf - hlf;
        const double gain = glf * glf / (hlf + lam) + grf * grf / (hrf + lam) - parent;
        if (gain > lb.gain) lb = {gain, joff + j0 + f, 4 * lane + i, GL, HL};
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Cand ob;
    ob.gain = __shfl_xor(lb.gain, o, 64);
    ob.j = __shfl_xor(lb.j, o, 64);
    ob.b = __shfl_xor(lb.b, o, 64);
    ob.gl = __shfl_xor(lb.gl, o, 64);
    ob.hl = __shfl_xor(lb.hl, o, 64);
    if (better(ob.gain, ob.j, ob.b, Best{lb.gain, lb.j, lb.b})) lb = ob;
  }
  if (lane == 0) wb[f] = lb;
  __syncthreads();
  if (threadIdx.x == 0) {
    Cand b = wb[0];
    for (int w = 1; w < NTS / 64; ++w)
      if (better(wb[w].gain, wb[w].j, wb[w].b, Best{b.gain, b.j, b.b})) b = wb[w];
    cand[(int64_t)k * ydim + yb] = b;
  }
}

// one wave per node of level d: best candidate over the feature blocks -> split (and the
// children's totals) or leaf value; children of leaves / absent nodes are marked -2.
// Candidates of node k: cand[r * rstride + k * ydim + y] for nr rank blocks (all-gathered
// feature slices; nr = 1 on a single device)
__global__ __launch_bounds__(64) void gbdt_split_final_kernel(
    const Cand* __restrict__ cand, int ydim, int nr, int64_t rstride, int d, int depth,
    double min_gain, double lam, double lr, int64_t* __restrict__ tot, int32_t* __restrict__ feat,
    int32_t* __restrict__ thr, double* __restrict__ value) {
  const int k = blockIdx.x, lane = threadIdx.x;
  const int hk = (1 << d) - 1 + k;
  if (d > 0 && feat[(hk - 1) / 2] < 0) {
    if (lane == 0) feat[hk] = -2;
    return;
  }
  Cand lb{-INFINITY, 0x7fffffff, 0x7fffffff, 0, 0};
  if (d < depth)
    for (int y = lane; y < nr * ydim; y += 64) {
      const int r = y / ydim;
      const Cand c = cand[r * rstride + (int64_t)k * ydim + (y - r * ydim)];
      if (better(c.gain, c.j, c.b, Best{lb.gain, lb.j, lb.b})) lb = c;
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Cand ob;
    ob.gain = __shfl_xor(lb.gain, o, 64);
    ob.j = __shfl_xor(lb.j, o, 64);
    ob.b = __shfl_xor(lb.b, o, 64);
    ob.gl = __shfl_xor(lb.gl, o, 64);
    ob.hl = __shfl_xor(lb.hl, o, 64);
    if (better(ob.gain, ob.j, ob.b, Best{lb.gain, lb.j, lb.b})) lb = ob;
  }
  if (lane == 0) {
    const int64_t G = tot[2 * hk], Hh = tot[2 * hk + 1];
    if (d < depth && lb.gain > -INFINITY && lb.gain > min_gain) {
      feat[hk] = lb.j;
      thr[hk] = lb.b;
      tot[2 * (2 * hk + 1)] = lb.gl;
      tot[2 * (2 * hk + 1) + 1] = lb.hl;
      tot[2 * (2 * hk + 2)] = G - lb.gl;
      tot[2 * (2 * hk + 2) + 1] = Hh - lb.hl;
    } else {
      const double gf = (double)G / GFIX, hf = (double)Hh / GFIX;
      feat[hk] = -1;
      value[hk] = -lr * gf / (hf + lam);
    }
  }
}

// ---- partition of the training positions into child buckets after a level's split ----
// bucket of position q: 2k + (bin > thr) for a row of split node k, 2nn ("retired")
// for rows of leaves (and rows retired at earlier levels, which sit past seg[nn]).
__global__ __launch_bounds__(NT) void gbdt_part_count_kernel(
    const uint8_t* __restrict__ Xr, int64_t ldr, const int32_t* __restrict__ idx,
    int64_t n_train, const int32_t* __restrict__ seg, int nn, int d,
    const int32_t* __restrict__ feat, const int32_t* __restrict__ thr, int64_t R, int W,
    uint8_t* __restrict__ bkt, int32_t* __restrict__ cnt) {
  __shared__ int sseg[MAXN / 2 + 1], sft[MAXN / 2], sth[MAXN / 2], lc[MAXB];
  if (threadIdx.x <= nn) sseg[threadIdx.x] = seg[threadIdx.x];
  if (threadIdx.x < nn) {
    sft[threadIdx.x] = feat[(1 << d) - 1 + threadIdx.x];
    sth[threadIdx.x] = thr[(1 << d) - 1 + threadIdx.x];
  }
  if (threadIdx.x < MAXB) lc[threadIdx.x] = 0;
  __syncthreads();
  const int wgi = blockIdx.x;
  const int64_t q0 = wgi * R, q1 = min(n_train, q0 + R);
  for (int64_t qb = q0 + threadIdx.x; qb < q1; qb += 4 * NT) {
    int32_t ii[4];
    int kk[4];
    uint8_t bv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t q = min(qb + u * NT, q1 - 1);
      ii[u] = idx[q];
      int lo = 0, hi = nn - 1;                              // largest k with seg[k] <= q
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (sseg[mid] <= q) lo = mid; else hi = mid - 1;
      }
      kk[u] = lo;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) bv[u] = Xr[(int64_t)ii[u] * ldr + max(sft[kk[u]], 0)];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t q = qb + u * NT;
      if (q >= q1) continue;
      int b = 2 * nn;
      if (q < sseg[nn] && sft[kk[u]] >= 0) b = 2 * kk[u] + (bv[u] > sth[kk[u]] ? 1 : 0);
      ATE_DASSERT(b <= 2 * nn && b < MAXB && kk[u] < nn);
      bkt[q] = (uint8_t)b;
      atomicAdd(&lc[b], 1);
    }
  }
  __syncthreads();
  if (threadIdx.x <= 2 * nn) cnt[(int64_t)threadIdx.x * W + wgi] = lc[threadIdx.x];
}

// one workgroup per bucket: exclusive scan of the per-workgroup counts (W <= 4 * NT)
__global__ __launch_bounds__(NT) void gbdt_part_scan_kernel(const int32_t* __restrict__ cnt,
                                                            int W, int32_t* __restrict__ base,
                                                            int32_t* __restrict__ btot) {
  __shared__ int ws[NT / 64];
  const int b = blockIdx.x;
  const int32_t* c = cnt + (int64_t)b * W;
  int v[4], s = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int w = 4 * threadIdx.x + u;
    v[u] = w < W ? c[w] : 0;
    s += v[u];
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) ws[wid] = incl;
  __syncthreads();
  int off = 0;
  for (int w2 = 0; w2 < wid; ++w2) off += ws[w2];
  int run = off + incl - s;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int w = 4 * threadIdx.x + u;
    if (w < W) base[(int64_t)b * W + w] = run;
    run += v[u];
  }
  if (threadIdx.x == NT - 1) {
    int t = 0;
    for (int w2 = 0; w2 < NT / 64; ++w2) t += ws[w2];
    btot[b] = t;
  }
}

__global__ __launch_bounds__(NT) void gbdt_part_scatter_kernel(
    const int32_t* __restrict__ idx, const int64_t* __restrict__ gh,
    const uint8_t* __restrict__ bkt, int64_t n_train, int nb, int64_t R, int W,
    const int32_t* __restrict__ base, const int32_t* __restrict__ btot,
    int32_t* __restrict__ idx2, int64_t* __restrict__ gh2, int32_t* __restrict__ seg2) {
  __shared__ int off[MAXB], lr[MAXB];
  if (threadIdx.x == 0) {
    int a = 0;
    for (int b = 0; b < nb; ++b) { off[b] = a; a += btot[b]; }
  }
  if (threadIdx.x < MAXB) lr[threadIdx.x] = 0;
  __syncthreads();
  const int wgi = blockIdx.x;
  if (wgi == 0 && threadIdx.x < nb) seg2[threadIdx.x] = off[threadIdx.x];
  if (threadIdx.x < nb) off[threadIdx.x] += base[(int64_t)threadIdx.x * W + wgi];
  __syncthreads();
  const int64_t q0 = wgi * R, q1 = min(n_train, q0 + R);
  for (int64_t q = q0 + threadIdx.x; q < q1; q += NT) {
    const int b = bkt[q];
    ATE_DASSERT(b < nb);
    const int64_t dst = off[b] + atomicAdd(&lr[b], 1);
    ATE_DASSERT(dst >= 0 && dst < n_train);
    idx2[dst] = idx[q];
    gh2[dst] = gh[q];
  }
}

// f[i] += value of the leaf row i reaches, for trees [0, ntree) (all rows). A workgroup
// stages RW whole rows in LDS with coalesced 16-B loads (all in flight at once) and the
// trees (M <= MAXM nodes), so a row's walk is LDS-latency only.
__global__ __launch_bounds__(NT) void gbdt_apply_kernel(const uint8_t* __restrict__ Xr, int64_t ldr,
                                                        int64_t n, int RW, int ntree, int M,
                                                        const int32_t* __restrict__ feat,
                                                        const int32_t* __restrict__ thr,
                                                        const double* __restrict__ value,
                                                        double* __restrict__ f) {
  extern __shared__ uint4 srow[];                           // [RW][ldr] bytes
  __shared__ int sft[MAXM], sth[MAXM];
  __shared__ double sv[MAXM];
  const int64_t r0 = blockIdx.x * (int64_t)RW;
  const int rows = (int)min((int64_t)RW, n - r0);
  const int v16 = (int)(ldr >> 4);
  const uint4* src = reinterpret_cast<const uint4*>(Xr + r0 * ldr);
  for (int t = threadIdx.x; t < rows * v16; t += NT) srow[t] = src[t];
  const uint8_t* mine = reinterpret_cast<const uint8_t*>(srow) + (int64_t)threadIdx.x * ldr;
  double acc = threadIdx.x < rows ? f[r0 + threadIdx.x] : 0.0;
  for (int t = 0; t < ntree; ++t) {
    __syncthreads();
    for (int m = threadIdx.x; m < M; m += NT) {
      sft[m] = feat[(int64_t)t * M + m];
      sth[m] = thr[(int64_t)t * M + m];
      sv[m] = value[(int64_t)t * M + m];
    }
    __syncthreads();
    if (threadIdx.x < rows) {
      int k = 0;
      while (sft[k] >= 0) k = 2 * k + 1 + (mine[sft[k]] > sth[k] ? 1 : 0);
      acc += sv[k];
    }
  }
  if (threadIdx.x < rows) f[r0 + threadIdx.x] = acc;
}

// Per-tree score update inside the fit: f[i] += value of the leaf row i reaches, for ONE
// tree and all rows. The walk reads only the <= depth bins on the row's path straight from
// HBM (one line each) instead of staging whole rows (2 KB at p = 2000) in LDS: ~6 lines
// instead of 16 per row. Four rows per thread walk in lockstep (independent chains in
// flight); same additions as gbdt_apply_kernel, so the same bits.
constexpr int WALK_U = 4;
__global__ __launch_bounds__(NT) void gbdt_walk_kernel(const uint8_t* __restrict__ Xr, int64_t ldr,
                                                       int64_t n, int depth, int M,
                                                       const int32_t* __restrict__ feat,
                                                       const int32_t* __restrict__ thr,
                                                       const double* __restrict__ value,
                                                       double* __restrict__ f) {
  __shared__ int sft[MAXM], sth[MAXM];
  __shared__ double sv[MAXM];
  for (int m = threadIdx.x; m < M; m += NT) {
    sft[m] = feat[m];
    sth[m] = thr[m];
    sv[m] = value[m];
  }
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * NT * WALK_U;
  for (int64_t i0 = (int64_t)blockIdx.x * NT * WALK_U + threadIdx.x; i0 < n; i0 += stride) {
    int k[WALK_U];
    double fv[WALK_U];
#pragma unroll
    for (int u = 0; u < WALK_U; ++u) {
      k[u] = 0;
      const int64_t i = i0 + (int64_t)u * NT;
      fv[u] = i < n ? f[i] : 0.0;
    }
    for (int d = 0; d < depth; ++d) {
      uint8_t b[WALK_U];
#pragma unroll
      for (int u = 0; u < WALK_U; ++u) {
        const int64_t i = i0 + (int64_t)u * NT;
        const int ft = sft[k[u]];
        b[u] = (i < n && ft >= 0) ? Xr[i * ldr + ft] : 0;
      }
#pragma unroll
      for (int u = 0; u < WALK_U; ++u)
        if (sft[k[u]] >= 0) k[u] = 2 * k[u] + 1 + (b[u] > sth[k[u]] ? 1 : 0);
    }
#pragma unroll
    for (int u = 0; u < WALK_U; ++u) {
      const int64_t i = i0 + (int64_t)u * NT;
      if (i < n) f[i] = fv[u] + sv[k[u]];
    }
  }
}

static int gbdt_apply_rows(int64_t ldr) {                   // rows staged per workgroup
  return (int)std::max<int64_t>(16, std::min<int64_t>(NT, 65536 / ldr) / 16 * 16);
}

static void gbdt_launch_apply(const uint8_t* Xr, int64_t ldr, int64_t n, int ntree, int M,
                              const int32_t* feat, const int32_t* thr, const double* value,
                              double* f, hipStream_t st) {
  const int RW = gbdt_apply_rows(ldr);
  ATE_LAUNCH(gbdt_apply_kernel, dim3((unsigned)((n + RW - 1) / RW)), dim3(NT),
                     (size_t)RW * ldr, st, Xr, ldr, n, RW, ntree, M, feat, thr, value, f);
}

}  // namespace

// Everything one fit needs; layout mirrored by models/gbdt.py::FitArgs.
struct GbdtFitArgs {
  const uint8_t* Xr;      // [n][ldr] row-major bins
  int64_t ldr, n, n_train;
  int p, depth, n_trees, loss, rule, W;
  double lam, min_gain, lr;
  int64_t min_child, R;
  const double* y;        // [n] (original row order)
  double* f;              // [n] raw scores (in: base, out: final)
  int32_t* idx[2];        // [n_train] positions -> row (idx[0] holds the training rows)
  int64_t* gh[2];         // [n_train] packed fixed-point (g, h) (gbdt_pack)
  uint8_t* bkt;           // [n_train]
  int32_t* cnt;           // [MAXB * W]
  int32_t* base;          // [MAXB * W]
  int32_t* btot;          // [MAXB]
  int32_t* seg[2];        // [MAXB + 1]
  int64_t* tot;           // [2 M]
  int32_t* feat;          // [T][M]
  int32_t* thr;
  double* value;
  int64_t* H[2];          // [2^(depth-1)][2][256][p] levels in node order (ping-pong)
  int64_t* Hs;            // [max(1, 2^(depth-2))][2][256][p] compact histogrammed nodes
  u64* slab;              // [slab_cap] partial histograms
  int64_t slab_cap;
  Cand* cand;             // [2^(depth-1) * ceil(p / 8)] split candidates (32 B each)
  // feature-sliced C04 (nr > 1; rule 1): rank `rk` of nr owns features [rk * pw, rk * pw +
  // pl); Hs is then [nr][slots][2][256][pw], Hl [slots][2][256][pw] receives the reduce-
  // scatter, candg [nr][2^(depth-1) * ceil(pw / 8)] Cands the candidate all-gather.
  // nr = 1: Hl, candg unused.
  int nr, rk, pw, pl;
  int64_t* Hl;
  Cand* candg;
};

// Resumable position of a fit (models/gbdt.py::RunState): tree t, level d, ping-pong
// index cur, resume = 1 when re-entering after the caller all-reduced (nr = 1) or reduce-
// scattered (nr > 1) level d's compact histograms (red_count int64 entries at the start
// of Hs), 2 after the caller all-gathered the level's candidates (red_count int64 entries
// of a.cand per rank, into a.candg).
struct GbdtRunState {
  int t, d, cur, resume;
  int64_t red_count;
  int t_stop;             // > 0: return 0 once tree t_stop - 1 is done (lockstep pair fits)
};

// chunk length and (upper bound of the) workgroup count of level d's histogram
static void gbdt_hist_geom(int64_t n_train, int p, int d, int rule, int64_t* CH, int64_t* nwg) {
  const int ydim = (p + FB - 1) / FB;
  // rows histogrammed: all of them at the root, at most half (count rule) or all
  // (hessian rule) of them below; `target` workgroups of full chunks (two resident per
  // CU; each pays a fixed 64-KB LDS clear + slab store)
  const int64_t rows = (d == 0 || rule == 1) ? n_train : (n_train + 1) / 2;
  // Chunks of ~64k rows: the ydim workgroups of a chunk read 16-byte slices of the same
  // row-major lines, and they only share them through L2 while they run close together --
  // short chunks keep them so (config-5 shard, 3 trees: 512 workgroups 4.46 s, 8192-65536
  // workgroups 2.7-3.2 s, the same bits; profiles/r03_cfg5). ATE_GBDT_HIST_TARGET = fixed
  // workgroup count.
  static const int64_t env_target = [] {
    const char* e = getenv("ATE_GBDT_HIST_TARGET");
    return e ? (int64_t)std::max(64, atoi(e)) : (int64_t)0;
  }();
  // ~R rows per chunk (ATE_GBDT_HIST_ROWS; round 6, config-5 shard with the fused root, 10
  // trees: 16384 3.13-3.58 s, 32768 2.86, 65536 2.77-2.79, 131072 2.81-2.82, 262144
  // 3.07-3.09; tools/r06_fused4.sh)
  static const int64_t env_rows = [] {
    const char* e = getenv("ATE_GBDT_HIST_ROWS");
    return e ? (int64_t)std::max(1024, atoi(e)) : (int64_t)65536;
  }();
  const int64_t target = env_target ? env_target
                                    : std::max<int64_t>(512, (rows * ydim + env_rows - 1) / env_rows);
  int64_t ch = (rows * ydim + target - 1) / target;
  ch = std::max<int64_t>(1024, (ch + 255) / 256 * 256);
  const int64_t wg = (((n_train + ch - 1) / ch + (1 << d)) + 7) / 8 * 8 * ydim;
  *CH = ch;
  *nwg = wg;
}

// fused root pass (gbdt_hist2_kernel): chunk length, chunk count, workgroups
static void gbdt_hist2_geom(int64_t n_train, int p, int64_t* CH, int64_t* nchunk, int64_t* nwg) {
  const int ydim2 = (p + FB2 - 1) / FB2;
  // ~R rows per chunk (ATE_GBDT_HIST2_ROWS; config-5 shard, 10 trees: 16384 3.05-3.46 s,
  // 32768 2.905-2.914, 65536 2.874-2.879, 131072 2.889-2.894; tools/r06_fused3.sh)
  static const int64_t R = [] {
    const char* e = getenv("ATE_GBDT_HIST2_ROWS");
    return e ? (int64_t)std::max(1024, atoi(e)) : (int64_t)65536;
  }();
  const int64_t target = std::max<int64_t>(512, (n_train * ydim2 + R - 1) / R);
  int64_t ch = (n_train * ydim2 + target - 1) / target;
  ch = std::max<int64_t>(1024, (ch + 255) / 256 * 256);
  *CH = ch;
  *nchunk = (n_train + ch - 1) / ch;
  *nwg = (*nchunk + 7) / 8 * 8 * ydim2;
}

ATE_KERNEL_SHAPE("gbdt_hist2_kernel<idx>", NTH2, 0, gbdt_hist2_kernel<false>)
ATE_KERNEL_SHAPE("gbdt_hist2_kernel<ranges>", NTH2, 0, gbdt_hist2_kernel<true>)
ATE_KERNEL_SHAPE("gbdt_hist_kernel<compact>", NTH, 0, gbdt_hist_kernel<true>)
ATE_KERNEL_SHAPE("gbdt_hist_kernel<full>", NTH, 0, gbdt_hist_kernel<false>)

// compile-time limits the host side sizes its buffers with (models/gbdt.py checks them)
ATE_API int ate_gbdt_limits(void* out) {
  int* o = static_cast<int*>(out);
  o[0] = MAXD;
  o[1] = MAXB;
  o[2] = FB;
  return 0;
}

ATE_API int64_t ate_gbdt_slab_entries(int64_t n_train, int p, int depth, int rule) {
  int64_t m = 0;
  for (int d = 0; d < depth; ++d) {
    int64_t ch, wg;
    gbdt_hist_geom(n_train, p, d, rule, &ch, &wg);
    m = std::max(m, wg);
  }
  return m * SLAB;
}

// slab entries the fused root pass of a pair of fits needs (in fit A's slab)
ATE_API int64_t ate_gbdt_slab2_entries(int64_t n_train, int p) {
  int64_t ch, nc, wg;
  gbdt_hist2_geom(n_train, p, &ch, &nc, &wg);
  return wg * SLAB2;
}

// Level 0 of tree t of two fits A, B on the same training rows, in lockstep
// (models/gbdt.fit_gbdt_pair): both fits' positions reset to idx_root (any order gives the
// same trees: every histogram is an exact integer sum), both gradients, ONE fused root
// histogram pass, and the compact root histograms of each fit written to its Hs. The caller
// then (rule 1) all-reduces / reduce-scatters each fit's 512 * nr * pw entries and resumes each
// stepper at (t, d = 0, cur = 0, resume = 1, t_stop = t + 1).
// gh2: [2 n_train] int64 scratch (the interleaved pairs); a0 / n0 / a1: the training rows as
// two ranges (rows a0 .. a0 + n0 - 1, then from a1; idx_root must list them in that order),
// or n0 < 0: read positions -> rows from idx_root.
ATE_API int ate_gbdt_pair_root(const void* args_a, const void* args_b, const void* idx_root,
                               void* gh2, int64_t a0, int64_t n0, int64_t a1, void* stream) {
  const GbdtFitArgs& A = *static_cast<const GbdtFitArgs*>(args_a);
  const GbdtFitArgs& B = *static_cast<const GbdtFitArgs*>(args_b);
  hipStream_t st = (hipStream_t)stream;
  if (A.Xr != B.Xr || A.ldr != B.ldr || A.n != B.n || A.n_train != B.n_train || A.p != B.p ||
      A.rule != B.rule || A.nr != B.nr || A.pw != B.pw || A.depth < 1 || B.depth < 1 ||
      (A.ldr & 31) || A.n_train < 1 || A.n_train >= (1LL << 31))
    return -1;
  if (A.slab_cap < ate_gbdt_slab2_entries(A.n_train, A.p)) return -5;
  const bool sliced = A.nr > 1;
  const int hp = sliced ? A.pw : A.p, nr = sliced ? A.nr : 1;
  const size_t bytes = (size_t)A.n_train * sizeof(int32_t);
  if (hipMemcpyAsync(A.idx[0], idx_root, bytes, hipMemcpyDeviceToDevice, st) != hipSuccess ||
      hipMemcpyAsync(B.idx[0], idx_root, bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return -3;
  const dim3 gg((unsigned)((A.n_train + 4 * NT - 1) / (4 * NT)));
  // (rows are int32 in the kernel: a fit holds < 2^31 rows)
  if (!gh2 || A.n >= (1LL << 31) ||
      (n0 >= 0 && (a0 < 0 || n0 > A.n_train || a1 < a0 + n0 || a1 + (A.n_train - n0) > A.n)))
    return -1;
  int64_t* g2 = static_cast<int64_t*>(gh2);
  ATE_LAUNCH(gbdt_grad_kernel, gg, dim3(NT), 0, st, A.loss, A.f, A.y, A.idx[0], A.n_train,
             A.gh[0], A.seg[0], g2);
  ATE_LAUNCH(gbdt_grad_kernel, gg, dim3(NT), 0, st, B.loss, B.f, B.y, B.idx[0], B.n_train,
             B.gh[0], B.seg[0], g2 + 1);
  int64_t CH, nchunk, nwg;
  gbdt_hist2_geom(A.n_train, A.p, &CH, &nchunk, &nwg);
  const int ydim2 = (A.p + FB2 - 1) / FB2;
  const bool ranges = n0 >= 0;
  ATE_LAUNCH(ranges ? gbdt_hist2_kernel<true> : gbdt_hist2_kernel<false>, dim3((unsigned)nwg),
             dim3(NTH2), 0, st, A.Xr, A.ldr, A.idx[0], reinterpret_cast<const longlong2*>(g2),
             (int)a0, (int)n0, (int)a1, (int)A.n_train, A.p, (int)CH, (int)nchunk, ydim2, A.slab,
             A.loss, B.loss);
  const int64_t perP = 512LL * nr * hp;
  ATE_LAUNCH(gbdt_hist2_reduce_kernel, dim3((unsigned)std::min<int64_t>((perP + NT - 1) / NT, 256), 2),
             dim3(NT), 0, st, A.slab, (int)nchunk, A.p, ydim2, A.Hs, B.Hs, nr, hp);
  ATE_CHECK_LAUNCH();
  return 0;
}

// Runs the fit from the position in *state to completion (returns 0), or until a
// row-sharded fit (rule 1) needs level d's compact histograms all-reduced (nr = 1) or
// reduce-scattered into a.Hl (nr > 1) across ranks (returns 1; state->red_count int64
// entries at a.Hs), or, feature-sliced, the level's split candidates all-gathered into
// a.candg (returns 2; state->red_count int64 entries at a.cand). Call again to continue.
ATE_API int ate_gbdt_run(const void* args, void* state, void* stream) {
  const GbdtFitArgs& a = *static_cast<const GbdtFitArgs*>(args);
  GbdtRunState& s = *static_cast<GbdtRunState*>(state);
  hipStream_t st = (hipStream_t)stream;
  if (a.depth < 1 || a.depth > MAXD || (a.ldr & 31) || a.n_train < 1 || a.W < 1 || a.W > 4 * NT)
    return -1;
  if ((a.n_train + a.R - 1) / a.R > a.W) return -2;
  if (a.slab_cap < ate_gbdt_slab_entries(a.n_train, a.p, a.depth, a.rule)) return -5;
  const bool sliced = a.nr > 1;
  if (sliced && (a.rule != 1 || a.rk < 0 || a.rk >= a.nr || a.pw < 1 || (int64_t)a.nr * a.pw < a.p ||
                 a.pl < 1 || a.pl > a.pw || a.rk * a.pw + a.pl > a.p || !a.Hl || !a.candg))
    return -6;
  const int M = (1 << (a.depth + 1)) - 1;
  const int ydim = (a.p + FB - 1) / FB;
  // histogram image / split search geometry of this rank: all p features, or its slice
  const int hp = sliced ? a.pw : a.p, hc = sliced ? a.pl : a.p, joff = sliced ? a.rk * a.pw : 0;
  const int nr = sliced ? a.nr : 1;
  const int ydim_s = (hp + SFB - 1) / SFB;
  const int64_t per = 512LL * hp;
  int64_t* Hsrc = sliced ? a.Hl : a.Hs;
  // ablation switch (profiling only): 1 no LDS atomics, 2 no bin gather, 4 no slab store,
  // 8 G atomics only, 16 H atomics as u32
  const char* hm = getenv("ATE_GBDT_HIST_MODE");
  const int hmode = hm ? atoi(hm) : 0;
  const int t_end = s.t_stop > 0 ? std::min(s.t_stop, a.n_trees) : a.n_trees;
  for (; s.t < t_end; ++s.t, s.d = 0) {
    int32_t* ft = a.feat + (int64_t)s.t * M;
    int32_t* th = a.thr + (int64_t)s.t * M;
    double* vt = a.value + (int64_t)s.t * M;
    if (s.d == 0 && !s.resume) {
      s.cur = 0;                                          // ping-pong index of idx/gh/seg
      ATE_LAUNCH(gbdt_grad_kernel, dim3((unsigned)((a.n_train + 4 * NT - 1) / (4 * NT))),
                         dim3(NT), 0, st, a.loss, a.f, a.y, a.idx[0], a.n_train, a.gh[0],
                         a.seg[0]);
    }
    for (; s.d <= a.depth; ++s.d) {
      const int d = s.d, cur = s.cur;
      const int nn = 1 << d;
      int64_t* Hc = a.H[d & 1];
      const int64_t* Hp = a.H[(d + 1) & 1];
      const int nsl = d == 0 ? 1 : nn / 2;                 // compact histogram slots
      if (d < a.depth) {
        if (s.resume == 0) {
          int64_t CH, nwg;
          gbdt_hist_geom(a.n_train, a.p, d, a.rule, &CH, &nwg);
          ATE_LAUNCH(hmode ? gbdt_hist_kernel<true> : gbdt_hist_kernel<false>,
                             dim3((unsigned)nwg), dim3(NTH), 0, st, a.Xr,
                             a.ldr, a.idx[cur], a.gh[cur], a.seg[cur], a.tot, a.rule, nn, a.p, d,
                             CH, ydim, a.slab, hmode, a.loss);
          const int64_t perP = 512LL * nr * hp;
          ATE_LAUNCH(gbdt_hist_reduce_kernel,
                             dim3((unsigned)std::min<int64_t>((perP + NT - 1) / NT, 256), nn),
                             dim3(NT), 0, st, a.slab, a.seg[cur], a.tot, a.rule, nn, a.p, d, CH,
                             ydim, a.Hs, nr, hp);
          if (a.rule == 1) {
            ATE_CHECK_LAUNCH();
            s.resume = 1;
            s.red_count = nsl * perP;
            return 1;                       // caller all-reduces / reduce-scatters Hs
          }
        }
        if (s.resume <= 1) {
          if (d == 0) ATE_LAUNCH(gbdt_root_kernel, dim3(1), dim3(NT), 0, st, Hsrc, hp, a.tot);
          ATE_LAUNCH(gbdt_expand_kernel,
                             dim3((unsigned)std::min<int64_t>((per + NT - 1) / NT, 128), nsl),
                             dim3(NT), 0, st, Hsrc, Hp, Hc, a.seg[cur], a.tot, ft, a.rule, hp, d);
          ATE_LAUNCH(gbdt_split_search_kernel, dim3(nn, ydim_s), dim3(NTS), 0, st, Hc,
                             hp, hc, joff, d, a.depth, a.lam, a.min_child, a.tot, ft, a.cand);
          if (sliced) {
            ATE_CHECK_LAUNCH();
            s.resume = 2;
            s.red_count = (int64_t)nn * ydim_s * (sizeof(Cand) / sizeof(int64_t));
            return 2;                                     // caller all-gathers cand
          }
        }
        s.resume = 0;
      }
      ATE_LAUNCH(gbdt_split_final_kernel, dim3(nn), dim3(64), 0, st,
                         sliced ? a.candg : a.cand, ydim_s, nr, (int64_t)nn * ydim_s, d,
                         a.depth, a.min_gain, a.lam, a.lr, a.tot, ft, th, vt);
      if (d + 1 < a.depth) {
        const int nb = 2 * nn + 1;
        const int W = (int)((a.n_train + a.R - 1) / a.R);
        ATE_LAUNCH(gbdt_part_count_kernel, dim3(W), dim3(NT), 0, st, a.Xr, a.ldr,
                           a.idx[cur], a.n_train, a.seg[cur], nn, d, ft, th, a.R, W, a.bkt,
                           a.cnt);
        ATE_LAUNCH(gbdt_part_scan_kernel, dim3(nb), dim3(NT), 0, st, a.cnt, W, a.base,
                           a.btot);
        ATE_LAUNCH(gbdt_part_scatter_kernel, dim3(W), dim3(NT), 0, st, a.idx[cur],
                           a.gh[cur], a.bkt, a.n_train, nb, a.R, W, a.base, a.btot,
                           a.idx[cur ^ 1], a.gh[cur ^ 1], a.seg[cur ^ 1]);
        s.cur ^= 1;
      }
    }
    // the next tree starts from whichever order this one left: keep idx[0] current
    if (s.cur == 1 &&
        hipMemcpyAsync(a.idx[0], a.idx[1], a.n_train * sizeof(int32_t), hipMemcpyDeviceToDevice,
                       st) != hipSuccess)
      return -3;
    {
      const int64_t g = std::min<int64_t>((a.n + NT * WALK_U - 1) / (NT * WALK_U), 256 * 16);
      ATE_LAUNCH(gbdt_walk_kernel, dim3((unsigned)g), dim3(NT), 0, st, a.Xr, a.ldr, a.n,
                         a.depth, M, ft, th, vt, a.f);
    }
  }
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_gbdt_apply(const void* Xr, int64_t ldr, int64_t n, int ntree, int M,
                           const void* feat, const void* thr, const void* value, void* f,
                           void* stream) {
  if (M > MAXM || (ldr & 15)) return -1;
  gbdt_launch_apply((const uint8_t*)Xr, ldr, n, ntree, M, (const int32_t*)feat,
                    (const int32_t*)thr, (const double*)value, (double*)f, (hipStream_t)stream);
  ATE_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ K11 on a device panel
// Bins the feature columns of an HBM-resident column-major panel (bf16 or fp32 storage,
// fold segments with padding) straight into the row-major uint8 layout of the trainer:
// out[i][j] (stride ldr) for compact real row i = seg_c0[s] + (row - seg_r0[s]).
// bin(x) = #{edges < x} (first edge >= x), the rule of csrc/forest.hip::bin_kernel.
// Workgroup = 256 rows x 16 features: reads are row-contiguous per feature, each thread
// writes its row's 16 bins as one 16-byte store; the 16 features' edges sit in LDS.
template <typename T>
__device__ __forceinline__ double panel_val(const T* X, int64_t off);
template <> __device__ __forceinline__ double panel_val<uint16_t>(const uint16_t* X, int64_t off) {
  return (double)__uint_as_float(((uint32_t)X[off]) << 16);
}
template <> __device__ __forceinline__ double panel_val<float>(const float* X, int64_t off) {
  return (double)X[off];
}

template <typename T>
__global__ __launch_bounds__(256) void gbdt_bin_panel_kernel(
    const T* __restrict__ X, int64_t ld, const int* __restrict__ xcols, int p,
    const int64_t* __restrict__ seg_r0, const int64_t* __restrict__ seg_n,
    const int64_t* __restrict__ seg_c0, int nseg, int64_t nreal,
    const double* __restrict__ edges, const int* __restrict__ nedges,
    uint8_t* __restrict__ out, int64_t ldr) {
  __shared__ double se[16][255];
  __shared__ int sne[16];
  const int f0 = blockIdx.y * 16;
  for (int e = threadIdx.x; e < 16 * 255; e += 256) {
    const int k = e / 255, b = e % 255;
    se[k][b] = f0 + k < p ? edges[(int64_t)(f0 + k) * 255 + b] : 0.0;
  }
  if (threadIdx.x < 16) sne[threadIdx.x] = f0 + threadIdx.x < p ? nedges[f0 + threadIdx.x] : 0;
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < nreal;
       i += (int64_t)gridDim.x * 256) {
    int s = 0;
    while (s + 1 < nseg && seg_c0[s + 1] <= i) ++s;
    const int64_t row = seg_r0[s] + (i - seg_c0[s]);
    uint8_t b[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      b[k] = 0;
      if (f0 + k < p) {
        const double x = panel_val<T>(X, (int64_t)xcols[f0 + k] * ld + row);
        int lo = 0, hi = sne[k];
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (se[k][mid] < x) lo = mid + 1; else hi = mid;
        }
        b[k] = (uint8_t)lo;
      }
    }
    uint4 v;
    v.x = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
    v.y = b[4] | (b[5] << 8) | (b[6] << 16) | ((uint32_t)b[7] << 24);
    v.z = b[8] | (b[9] << 8) | (b[10] << 16) | ((uint32_t)b[11] << 24);
    v.w = b[12] | (b[13] << 8) | (b[14] << 16) | ((uint32_t)b[15] << 24);
    *reinterpret_cast<uint4*>(out + i * ldr + f0) = v;
  }
}

// dtype: 0 = bf16 storage, 1 = fp32. ldr must be a multiple of 16 and >= p rounded to 16.
ATE_API int ate_gbdt_bin_panel(const void* X, int dtype, int64_t ld, const void* xcols, int p,
                               const void* seg_r0, const void* seg_n, const void* seg_c0,
                               int nseg, int64_t nreal, const void* edges, const void* nedges,
                               void* out, int64_t ldr, void* stream) {
  if (ldr % 16 || ldr < (p + 15) / 16 * 16) return -1;
  dim3 grid(ate::grid_for(nreal, 256, 4096), (p + 15) / 16);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    ATE_LAUNCH(gbdt_bin_panel_kernel<uint16_t>, grid, dim3(256), 0, st,
                       (const uint16_t*)X, ld, (const int*)xcols, p, (const int64_t*)seg_r0,
                       (const int64_t*)seg_n, (const int64_t*)seg_c0, nseg, nreal,
                       (const double*)edges, (const int*)nedges, (uint8_t*)out, ldr);
  else if (dtype == 1)
    ATE_LAUNCH(gbdt_bin_panel_kernel<float>, grid, dim3(256), 0, st, (const float*)X, ld,
                       (const int*)xcols, p, (const int64_t*)seg_r0, (const int64_t*)seg_n,
                       (const int64_t*)seg_c0, nseg, nreal, (const double*)edges,
                       (const int*)nedges, (uint8_t*)out, ldr);
  else
    return -1;
  ATE_CHECK_LAUNCH();
  return 0;
}
