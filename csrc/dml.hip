// Fused cross-fit residual pass for partially-linear DML with linear nuisances.
//
// For every row i of held-out segment k:
//   yr_i = y_i - (cy[k][0] + x_i . cy[k][1:]) ,  wr_i = w_i - (cw[k][0] + x_i . cw[k][1:])
// and the orthogonal-score moments {S_wy, S_ww, S_yyww, S_yw3, S_w4, n, S_yy} are
// accumulated in fp64 -- the residual vectors are never written to HBM. Only the
// columns in the fold's LASSO support (nonzero Y- or W-coefficient) are read, once
// each (bandwidth-bound: one column-major stream per feature, coalesced across the
// 256 rows of a block). Coefficients for all folds are staged
// in LDS. y/w are reconstructed from their hi+lo bf16 columns on bf16 panels.
#include "common.hpp"

using namespace ate;

template <typename T>
__device__ __forceinline__ double ld_col(const T* X, int64_t ld, int c, int64_t i) {
  return (double)X[(int64_t)c * ld + i];
}
template <>
__device__ __forceinline__ double ld_col<bf16_t>(const bf16_t* X, int64_t ld, int c, int64_t i) {
  return (double)bf16_to_f32(X[(int64_t)c * ld + i]);
}

struct Seg { int64_t r0, r1; };

// Ordered compaction (ascending j, so the dot products keep their summation order and
// the result is bit-identical to the dense loop) of the feature columns whose Y- or
// W-coefficient is nonzero: LASSO nuisances are sparse, so the pass reads only the
// selected columns of the panel. cy/cw/xc: dense staged arrays; outputs in place
// (cy[1+q], cw[1+q], xc[q] for q < *nnz). Whole block must call it.
template <typename C>
__device__ int compact_support(C* cy, C* cw, int* xc, int p, int* wcnt /* [>= 4] */) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int base = 0;
  for (int j0 = 0; j0 < p; j0 += blockDim.x) {
    const int j = j0 + threadIdx.x;
    const bool keep = j < p && (cy[1 + j] != C(0) || cw[1 + j] != C(0));
    C vy = j < p ? cy[1 + j] : C(0), vw = j < p ? cw[1 + j] : C(0);
    const int c = j < p ? xc[j] : 0;
    const uint64_t m = __ballot(keep);
    if (lane == 0) wcnt[wid] = __popcll(m);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wid; ++w) off += wcnt[w];
    int tot = base;
    for (int w = 0; w < nw; ++w) tot += wcnt[w];
    const int pos = off + __popcll(m & ((1ull << lane) - 1ull));
    __syncthreads();                                      // all reads of the dense slots done
    if (keep) { cy[1 + pos] = vy; cw[1 + pos] = vw; xc[pos] = c; }
    __syncthreads();
    base = tot;
  }
  return base;
}

template <typename T, int RPT>
__global__ __launch_bounds__(256) void dml_resid_kernel(
    const T* __restrict__ X, int64_t ld, const int* __restrict__ xcols, int p,
    const Seg* __restrict__ segs, int nseg, const double* __restrict__ coef /*[nseg][2][p+1]*/,
    int y0, int y1, int w0, int w1, int vcol, double* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) double sh[];
  double* cy = sh;                    // [p+1]
  double* cw = sh + (p + 1);          // [p+1]
  int* xc = (int*)(sh + 2 * (p + 1)); // [p]
  __shared__ double red[16 * 7];
  __shared__ int wcnt[16];
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int j = threadIdx.x; j < p; j += blockDim.x) xc[j] = xcols[j];
  // grid: blockIdx.y = segment; blocks stride over that segment's rows
  const int k = blockIdx.y;
  ATE_DASSERT(k < nseg && y0 >= 0 && w0 >= 0 && vcol >= 0);
  for (int j = threadIdx.x; j <= p; j += blockDim.x) {
    cy[j] = coef[((int64_t)k * 2 + 0) * (p + 1) + j];
    cw[j] = coef[((int64_t)k * 2 + 1) * (p + 1) + j];
  }
  __syncthreads();
  p = compact_support(cy, cw, xc, p, wcnt);
  const Seg sg = segs[k];
  ATE_DASSERT(sg.r0 >= 0 && sg.r0 <= sg.r1 && sg.r1 <= ld);
  for (int64_t base = sg.r0 + (int64_t)blockIdx.x * 256 * RPT; base < sg.r1;
       base += (int64_t)gridDim.x * 256 * RPT) {
    double py[RPT], pw[RPT];
    int64_t ii[RPT];
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      ii[r] = base + r * 256 + threadIdx.x;
      py[r] = cy[0];
      pw[r] = cw[0];
    }
    for (int j = 0; j < p; ++j) {
      const double by = cy[1 + j], bw = cw[1 + j];
      const int c = xc[j];
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        double x = ii[r] < sg.r1 ? ld_col(X, ld, c, ii[r]) : 0.0;
        py[r] += by * x;
        pw[r] += bw * x;
      }
    }
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      if (ii[r] >= sg.r1) continue;
      if (ld_col(X, ld, vcol, ii[r]) == 0.0) continue;
      double y = ld_col(X, ld, y0, ii[r]) + (y1 >= 0 ? ld_col(X, ld, y1, ii[r]) : 0.0);
      double w = ld_col(X, ld, w0, ii[r]) + (w1 >= 0 ? ld_col(X, ld, w1, ii[r]) : 0.0);
      double yr = y - py[r], wr = w - pw[r], w2 = wr * wr;
      v[0] += wr * yr; v[1] += w2; v[2] += yr * yr * w2; v[3] += yr * w2 * wr; v[4] += w2 * w2;
      v[5] += 1.0; v[6] += yr * yr;
    }
  }
  block_sum<7>(v, red);
  if (threadIdx.x == 0) {
    double* out = partial + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 7;
#pragma unroll
    for (int q = 0; q < 7; ++q) out[q] = v[q];
  }
}

// one block of 256 threads: thread i sums partials i, i+256, ... (fixed order), then a
// fixed-shape block reduction -> deterministic for a given launch geometry
__global__ __launch_bounds__(256) void sum7_kernel(const double* __restrict__ partial, int nb,
                                                   double* __restrict__ out) {
  __shared__ double red[16 * 7];
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int b = threadIdx.x; b < nb; b += 256)
#pragma unroll
    for (int q = 0; q < 7; ++q) v[q] += partial[(int64_t)b * 7 + q];
  block_sum<7>(v, red);
  if (threadIdx.x == 0)
#pragma unroll
    for (int q = 0; q < 7; ++q) out[q] = v[q];
}

template <typename T>
static int dml_resid_t(const void* X, int64_t ld, const void* xcols, int p, const void* segs,
                       int nseg, const void* coef, int y0, int y1, int w0, int w1, int vcol,
                       int nbx, void* partial, void* moments, hipStream_t s) {
  size_t sh = (size_t)2 * (p + 1) * sizeof(double) + (size_t)p * sizeof(int);
  dim3 grid(nbx, nseg);
  ATE_LAUNCH((dml_resid_kernel<T, 4>), grid, dim3(256), sh, s, (const T*)X, ld,
                     (const int*)xcols, p, (const Seg*)segs, nseg, (const double*)coef, y0, y1,
                     w0, w1, vcol, (double*)partial);
  ATE_CHECK_LAUNCH();
  ATE_LAUNCH(sum7_kernel, dim3(1), dim3(256), 0, s, (const double*)partial, nbx * nseg,
                     (double*)moments);
  ATE_CHECK_LAUNCH();
  return 0;
}

// bf16 panels: each thread owns 8 CONSECUTIVE rows, so every column read is one 16-byte
// load (a wave reads 1 KB contiguous per column -- Guideline 13); dot products in fp32
// (bf16 values are exact in fp32; coefficients rounded to fp32), moments in fp64.
// mode 0: fp64 moments (partial [blocks][7] double); exact mode (world-size-invariant,
// ops/exact.py): 1 = per-term max |t| (partial [blocks][7] double, reduced with max),
// 2 = per-term int64 limb sums at the shifts sh[7] derived from the global max
// (partial [blocks][14] int64: hi limbs, then lo limbs) -- integer sums, so the block and
// the rank that own a row cannot change the result.
__global__ __launch_bounds__(256) void dml_resid_bf16_kernel(
    const bf16_t* __restrict__ X, int64_t cs, int64_t bs, const int* __restrict__ xcols, int p,
    const Seg* __restrict__ segs, int nseg, const double* __restrict__ coef,
    int y0, int y1, int w0, int w1, int vcol, double* __restrict__ partial, int mode,
    const int64_t* __restrict__ sh) {
  extern __shared__ __attribute__((aligned(16))) float shf[];
  float* cy = shf;                 // [p+1]
  float* cw = shf + (p + 1);       // [p+1]
  int* xc = (int*)(shf + 2 * (p + 1));
  __shared__ double red[16 * 7];
  __shared__ int wcnt[16];
  const int k = blockIdx.y;
  for (int j = threadIdx.x; j < p; j += blockDim.x) xc[j] = xcols[j];
  for (int j = threadIdx.x; j <= p; j += blockDim.x) {
    cy[j] = (float)coef[((int64_t)k * 2 + 0) * (p + 1) + j];
    cw[j] = (float)coef[((int64_t)k * 2 + 1) * (p + 1) + j];
  }
  __syncthreads();
  p = compact_support(cy, cw, xc, p, wcnt);
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
  long long lh[7] = {0, 0, 0, 0, 0, 0, 0}, ll[7] = {0, 0, 0, 0, 0, 0, 0};
  double scale[7];
#pragma unroll
  for (int q = 0; q < 7; ++q) scale[q] = mode == 2 ? ldexp(1.0, (int)sh[q]) : 1.0;
  const Seg sg = segs[k];
  ATE_DASSERT(k < nseg && sg.r0 >= 0 && sg.r0 <= sg.r1 && (sg.r0 & 7) == 0 && mode >= 0 &&
              mode <= 2 && y0 >= 0 && w0 >= 0 && vcol >= 0);
  auto ld8 = [&](int c, int64_t i, float (&o)[8]) {
    ATE_DASSERT((i & 7) == 0 && c >= 0);
    // (c, i) at c*cs + (i/64)*bs + i%64: column-major (cs = ld, bs = 64) or 64-row blocked
    // (cs = 64, bs = 64*P); the 8 rows never straddle a block (i % 8 == 0)
    const uint4 u = *reinterpret_cast<const uint4*>(X + (int64_t)c * cs + (i >> 6) * bs + (i & 63));
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      o[2 * q] = __uint_as_float(w[q] << 16);
      o[2 * q + 1] = __uint_as_float(w[q] & 0xFFFF0000u);
    }
  };
  for (int64_t i = sg.r0 + ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8; i < sg.r1;
       i += (int64_t)gridDim.x * 256 * 8) {
    float py[8], pw[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) { py[r] = cy[0]; pw[r] = cw[0]; }
#pragma unroll 4
    for (int j = 0; j < p; ++j) {
      float x[8];
      ld8(xc[j], i, x);
      const float by = cy[1 + j], bw = cw[1 + j];
#pragma unroll
      for (int r = 0; r < 8; ++r) { py[r] += by * x[r]; pw[r] += bw * x[r]; }
    }
    float vv[8], ya[8], yb[8], wa[8], wb[8];
    ld8(vcol, i, vv);
    ld8(y0, i, ya);
    ld8(w0, i, wa);
    if (y1 >= 0) ld8(y1, i, yb); else { for (int r = 0; r < 8; ++r) yb[r] = 0.f; }
    if (w1 >= 0) ld8(w1, i, wb); else { for (int r = 0; r < 8; ++r) wb[r] = 0.f; }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if (vv[r] == 0.f) continue;
      const double yr = ((double)ya[r] + (double)yb[r]) - (double)py[r];
      const double wr = ((double)wa[r] + (double)wb[r]) - (double)pw[r];
      const double w2 = wr * wr;
      if (mode == 0) {
        v[0] += wr * yr; v[1] += w2; v[2] += yr * yr * w2; v[3] += yr * w2 * wr; v[4] += w2 * w2;
        v[5] += 1.0; v[6] += yr * yr;
        continue;
      }
      const double t[7] = {wr * yr, w2, yr * yr * w2, yr * w2 * wr, w2 * w2, 1.0, yr * yr};
#pragma unroll
      for (int q = 0; q < 7; ++q) {
        if (mode == 1) {
          v[q] = fmax(v[q], fabs(t[q]));
        } else {
          const double x = t[q] * scale[q];                 // exact (power of two)
          const double h = floor(x);
          lh[q] += (long long)h;
          ll[q] += (long long)rint((x - h) * 4294967296.0);
        }
      }
    }
  }
  const int64_t blk = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
  if (mode == 0) {
    block_sum<7>(v, red);
    if (threadIdx.x == 0) {
      double* out = partial + blk * 7;
#pragma unroll
      for (int q = 0; q < 7; ++q) out[q] = v[q];
    }
    return;
  }
  // exact modes: wave reduction (max or integer sum, both order-free), then one atomic-free
  // LDS pass over the 4 waves
  __shared__ long long xr[4][14];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 7; ++q) {
    for (int o = 32; o > 0; o >>= 1) {
      if (mode == 1) {
        v[q] = fmax(v[q], __shfl_xor(v[q], o, 64));
      } else {
        lh[q] += __shfl_xor(lh[q], o, 64);
        ll[q] += __shfl_xor(ll[q], o, 64);
      }
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < 7; ++q) {
      xr[wid][q] = mode == 1 ? __double_as_longlong(v[q]) : lh[q];
      xr[wid][7 + q] = ll[q];
    }
  }
  __syncthreads();
  if (threadIdx.x < 14) {
    const int q = threadIdx.x;
    if (mode == 1) {
      if (q < 7) {
        double m = 0.0;
        for (int w = 0; w < 4; ++w) m = fmax(m, __longlong_as_double(xr[w][q]));
        partial[blk * 7 + q] = m;
      }
    } else {
      long long a = 0;
      for (int w = 0; w < 4; ++w) a += xr[w][q];
      reinterpret_cast<long long*>(partial)[blk * 14 + q] = a;
    }
  }
}

// dtype 1 f32, 2 f64, 3 bf16. partial: [nseg*nbx*7]
// (cs, bs): element (c, i) at c*cs + (i/64)*bs + i%64 (fp32/fp64 panels: column-major only)
ATE_API int ate_dml_resid_moments(int dtype, const void* X, int64_t cs, int64_t bs,
                                  const void* xcols, int p,
                                  const void* segs, int nseg, const void* coef, int y0, int y1,
                                  int w0, int w1, int vcol, int nbx, void* partial, void* moments,
                                  void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dtype != 3 && bs != 64) return -1;
  const int64_t ld = cs;
  if (dtype == 1)
    return dml_resid_t<float>(X, ld, xcols, p, segs, nseg, coef, y0, y1, w0, w1, vcol, nbx,
                              partial, moments, s);
  if (dtype == 2)
    return dml_resid_t<double>(X, ld, xcols, p, segs, nseg, coef, y0, y1, w0, w1, vcol, nbx,
                               partial, moments, s);
  if (dtype == 3) {
    size_t sh = (size_t)2 * (p + 1) * sizeof(float) + (size_t)p * sizeof(int);
    dim3 grid(nbx, nseg);
    ATE_LAUNCH(dml_resid_bf16_kernel, grid, dim3(256), sh, s, (const bf16_t*)X, cs, bs,
                       (const int*)xcols, p, (const Seg*)segs, nseg, (const double*)coef, y0, y1,
                       w0, w1, vcol, (double*)partial, 0, (const int64_t*)nullptr);
    ATE_CHECK_LAUNCH();
    ATE_LAUNCH(sum7_kernel, dim3(1), dim3(256), 0, s, (const double*)partial, nbx * nseg,
                       (double*)moments);
    ATE_CHECK_LAUNCH();
    return 0;
  }
  return -1;
}

// exact-mode passes of the bf16 residual kernel (mode 1: per-block max |term| into
// partial [nseg*nbx][7] double; mode 2: per-block int64 limb sums into partial
// [nseg*nbx][14] at the shifts sh[7]); the caller reduces the blocks (max / integer sum)
ATE_API int ate_dml_resid_exact(const void* X, int64_t cs, int64_t bs, const void* xcols, int p,
                                const void* segs, int nseg, const void* coef, int y0, int y1,
                                int w0, int w1, int vcol, int nbx, int mode, const void* sh,
                                void* partial, void* stream) {
  if (mode < 1 || mode > 2) return -1;
  size_t shm = (size_t)2 * (p + 1) * sizeof(float) + (size_t)p * sizeof(int);
  dim3 grid(nbx, nseg);
  ATE_LAUNCH(dml_resid_bf16_kernel, grid, dim3(256), shm, (hipStream_t)stream,
                     (const bf16_t*)X, cs, bs, (const int*)xcols, p, (const Seg*)segs, nseg,
                     (const double*)coef, y0, y1, w0, w1, vcol, (double*)partial, mode,
                     (const int64_t*)sh);
  ATE_CHECK_LAUNCH();
  return 0;
}
