// K04 select_compact: the selection-bias transform of ate_replication.Rmd:97-121 on the
// device (P7) — per-arm candidate flags, ordered ranks by a three-phase block scan, drop
// of the FIRST round(pt*k_treat) / round(pc*k_control) candidates in row order, and a
// stable compaction of the kept row indices. Matches data/selection.py::drop_indices.
//
// X is the column-major covariate matrix [p][n] (fp64); the caller passes the column
// indices of g2000, g2002, p2000, p2002, p2004, city, yob and the "last" primary
// column the treated rule uses (p2002 under the reference quirk Q17, else p2004).
#include "common.hpp"

namespace {

constexpr int NT = 256;

struct SelCols { int g2000, g2002, p2000, p2002, p2004, city, yob, last; };

__device__ __forceinline__ int flag_of(const double* X, int64_t n, const double* W, int64_t i,
                                       SelCols c) {
  auto v = [&](int col) { return X[(int64_t)col * n + i]; };
  if (W[i] == 1.0) {
    const bool d = v(c.g2000) == 1 || v(c.g2002) == 1 || v(c.p2000) == 1 || v(c.p2002) == 1 ||
                   v(c.last) == 1 || v(c.city) > 2 || v(c.yob) > 2;
    return d ? 1 : 0;
  }
  if (W[i] == 0.0) {
    const bool d = v(c.g2000) == 0 || v(c.g2002) == 0 || v(c.p2000) == 0 || v(c.p2002) == 0 ||
                   v(c.p2004) == 0 || v(c.city) < -2 || v(c.yob) < -2;
    return d ? 2 : 0;
  }
  return 0;
}

// block-exclusive scan of NT ints (returns block total)
__device__ int block_scan(int x, int* ws) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) ws[wid] = incl;
  __syncthreads();
  int off = 0, tot = 0;
  for (int w = 0; w < NT / 64; ++w) {
    if (w < wid) off += ws[w];
    tot += ws[w];
  }
  __syncthreads();
  ws[NT / 64] = tot;
  return off + incl - x;
}

// phase 1: flags + per-block candidate counts (treated, control)
__global__ __launch_bounds__(NT) void sel_count_kernel(const double* X, int64_t n, const double* W,
                                                       SelCols c, uint8_t* flags, int* cnt) {
  __shared__ int ws[2][NT / 64 + 1];
  const int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x;
  const int f = i < n ? flag_of(X, n, W, i, c) : 0;
  if (i < n) flags[i] = (uint8_t)f;
  block_scan(f == 1, ws[0]);
  block_scan(f == 2, ws[1]);
  if (threadIdx.x == 0) {
    cnt[2 * blockIdx.x] = ws[0][NT / 64];
    cnt[2 * blockIdx.x + 1] = ws[1][NT / 64];
  }
}

// phase 2 (one block): exclusive offsets over blocks, per arm; totals -> thresholds
__global__ __launch_bounds__(NT) void sel_offsets_kernel(int* cnt, int nblk, double pt, double pc,
                                                         int* thr) {
  __shared__ int ws[NT / 64 + 1];
  for (int arm = 0; arm < 2; ++arm) {
    int carry = 0;
    for (int b0 = 0; b0 < nblk; b0 += NT) {
      const int b = b0 + threadIdx.x;
      const int x = b < nblk ? cnt[2 * b + arm] : 0;
      const int ex = block_scan(x, ws);
      if (b < nblk) cnt[2 * b + arm] = carry + ex;
      carry += ws[NT / 64];
      __syncthreads();
    }
    if (threadIdx.x == 0) thr[arm] = (int)rint((arm == 0 ? pt : pc) * (double)carry);
  }
}

// phase 3: drop flag from the ordered rank; per-block kept counts
__global__ __launch_bounds__(NT) void sel_drop_kernel(const uint8_t* flags, int64_t n,
                                                      const int* cnt, const int* thr,
                                                      uint8_t* keep, int* kcnt) {
  __shared__ int ws[3][NT / 64 + 1];
  const int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x;
  const int f = i < n ? flags[i] : 0;
  const int r1 = block_scan(f == 1, ws[0]) + cnt[2 * blockIdx.x];
  const int r2 = block_scan(f == 2, ws[1]) + cnt[2 * blockIdx.x + 1];
  ATE_DASSERT(r1 >= 0 && r2 >= 0 && thr[0] >= 0 && thr[1] >= 0);
  const bool drop = (f == 1 && r1 < thr[0]) || (f == 2 && r2 < thr[1]);
  const int k = i < n && !drop;
  if (i < n) keep[i] = (uint8_t)k;
  block_scan(k, ws[2]);
  if (threadIdx.x == 0) kcnt[blockIdx.x] = ws[2][NT / 64];
}

// phase 4 (one block): exclusive offsets of kept counts
__global__ __launch_bounds__(NT) void sel_koff_kernel(int* kcnt, int nblk, int* total) {
  __shared__ int ws[NT / 64 + 1];
  int carry = 0;
  for (int b0 = 0; b0 < nblk; b0 += NT) {
    const int b = b0 + threadIdx.x;
    const int x = b < nblk ? kcnt[b] : 0;
    const int ex = block_scan(x, ws);
    if (b < nblk) kcnt[b] = carry + ex;
    carry += ws[NT / 64];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

// phase 5: stable compaction of kept row indices
__global__ __launch_bounds__(NT) void sel_compact_kernel(const uint8_t* keep, int64_t n,
                                                         const int* koff, int64_t* out) {
  __shared__ int ws[NT / 64 + 1];
  const int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x;
  const int k = i < n ? keep[i] : 0;
  const int pos = block_scan(k, ws) + koff[blockIdx.x];
  ATE_DASSERT(!k || (pos >= 0 && pos <= i));     // a compaction never moves a row forward
  if (k) out[pos] = i;
}

}  // namespace

// cols: int[8] = g2000, g2002, p2000, p2002, p2004, city, yob, last. scratch: int[2*nblk +
// nblk + 4] with nblk = ceil(n/256). out: kept row indices (int64, capacity n);
// n_kept/thresholds land in scratch tail (read back by the caller).
ATE_API int ate_select_compact(const void* X, int64_t n, const void* W, const void* cols,
                               double pt, double pc, void* flags, void* keep, void* scratch,
                               void* out, void* stream) {
  const int* cc = (const int*)cols;
  SelCols c{cc[0], cc[1], cc[2], cc[3], cc[4], cc[5], cc[6], cc[7]};
  hipStream_t st = (hipStream_t)stream;
  const int nblk = (int)((n + NT - 1) / NT);
  int* cnt = (int*)scratch;
  int* kcnt = cnt + 2 * nblk;
  int* tail = kcnt + nblk;        // thr[2], total
  ATE_LAUNCH(sel_count_kernel, dim3(nblk), dim3(NT), 0, st, (const double*)X, n,
                     (const double*)W, c, (uint8_t*)flags, cnt);
  ATE_LAUNCH(sel_offsets_kernel, dim3(1), dim3(NT), 0, st, cnt, nblk, pt, pc, tail);
  ATE_LAUNCH(sel_drop_kernel, dim3(nblk), dim3(NT), 0, st, (const uint8_t*)flags, n, cnt,
                     tail, (uint8_t*)keep, kcnt);
  ATE_LAUNCH(sel_koff_kernel, dim3(1), dim3(NT), 0, st, kcnt, nblk, tail + 2);
  ATE_LAUNCH(sel_compact_kernel, dim3(nblk), dim3(NT), 0, st, (const uint8_t*)keep, n,
                     kcnt, (int64_t*)out);
  ATE_CHECK_LAUNCH();
  return 0;
}
