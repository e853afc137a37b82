// K01 gram_syrk_mfma: G_s = X_s' D X_s for every row segment s (cross-fit fold),
// X column-major [P][ld] (bf16 or fp32), D = diag(w) optional (fp32 path).
//
// Work decomposition (tall-skinny SYRK, reduction dim = rows):
//   workgroup = (row chunk c, upper-triangular output tile t). Chunks never cross
//   a segment, so per-fold Grams fall out of the same launch. Each workgroup
//   writes its fp32 tile partial to a slab; a second kernel reduces the slab
//   per segment in a FIXED chunk order in fp64 (bitwise reproducible, no atomics).
//   Block ids are remapped so that all tiles of one row chunk run on the same
//   XCD (they re-read the same rows of X from that XCD's L2).
//
// bf16 path: 128x128 tile / 256 threads (2x2 waves of 64x64), K-step 64 rows,
//   mfma_f32_16x16x32_bf16, A/B tiles staged through LDS with a per-column XOR
//   swizzle of the 16-byte chunks (conflict-reduced ds_read_b128), register
//   double-buffered global loads. Padding rows are all-zero, so they add nothing.
// fp32/fp64 path: 64x64 tile, K-step 16 rows, mfma_f32_16x16x4f32 / mfma_f64_16x16x4f64
//   (fp64 = the parity mode, exact enough for lm-style rank detection), optional
//   row weights fused into the A-tile staging.
#include "common.hpp"

using namespace ate;

struct Chunk { int64_t row0, row1; int seg, pad; };

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // bijective remap: blocks b, b+8, b+16... (same XCD label) get consecutive logical ids
  int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// ------------------------------------------------------------------ bf16 128x128
constexpr int BT = 128;      // tile
constexpr int BK = 64;       // rows per K-step

__global__ __launch_bounds__(256) void gram_bf16_kernel(
    const bf16_t* __restrict__ X, int64_t ld, const int2* __restrict__ tiles, int ntiles,
    const Chunk* __restrict__ chunks, int nchunks, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2][2][BT * BK];   // [buf][A/B][col*64+row]
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int c = L / ntiles, t = L % ntiles;
  const Chunk ch = chunks[c];
  const int2 tl = tiles[t];
  const bool diag = tl.x == tl.y;
  const int a0 = tl.x * BT, b0 = tl.y * BT;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // staging map: 128 cols x 8 chunks of 16B = 1024 loads; thread does 4 (A) + 4 (B)
  uint4 ra[4], rb[4];
  auto gload = [&](int64_t i0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int idx = r * 256 + tid, col = idx >> 3, cc = idx & 7;
      ra[r] = *reinterpret_cast<const uint4*>(X + (int64_t)(a0 + col) * ld + i0 + cc * 8);
      if (!diag) rb[r] = *reinterpret_cast<const uint4*>(X + (int64_t)(b0 + col) * ld + i0 + cc * 8);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int idx = r * 256 + tid, col = idx >> 3, cc = idx & 7;
      int off = col * BK + ((cc ^ (col & 7)) << 3);
      *reinterpret_cast<uint4*>(&lds[buf][0][off]) = ra[r];
      if (!diag) *reinterpret_cast<uint4*>(&lds[buf][1][off]) = rb[r];
    }
  };

  const int64_t nsteps = (ch.row1 - ch.row0) / BK;
  if (nsteps > 0) {
    gload(ch.row0);
    lstore(0);
  }
  __syncthreads();
  for (int64_t s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) gload(ch.row0 + (s + 1) * BK);
    const bf16_t* As = lds[buf][0];
    const bf16_t* Bs = diag ? lds[buf][0] : lds[buf][1];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int cc = kk * 4 + (lane >> 4);
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        int col = wr * 64 + m * 16 + (lane & 15);
        af[m] = *reinterpret_cast<const bf16x8*>(&As[col * BK + ((cc ^ (col & 7)) << 3)]);
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        int col = wc * 64 + n * 16 + (lane & 15);
        bfr[n] = *reinterpret_cast<const bf16x8*>(&Bs[col * BK + ((cc ^ (col & 7)) << 3)]);
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
    }
    if (s + 1 < nsteps) lstore(buf ^ 1);
    __syncthreads();
  }
  // epilogue: acc reg r of lane l = C[row=(l>>4)*4+r][col=l&15]
  float* out = slab + ((int64_t)c * ntiles + t) * (BT * BT);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int row = wr * 64 + m * 16 + (lane >> 4) * 4 + r;
        int col = wc * 64 + n * 16 + (lane & 15);
        out[row * BT + col] = acc[m][n][r];
      }
}

// ------------------------------------------------------------------ bf16 256x256, LDS-DMA staged
// 512 threads = 8 waves as 2 (rows) x 4 (cols); each wave owns a 128x64 output block
// (8x4 tiles of mfma_f32_16x16x32_bf16 -> 128 accumulator registers). Per 64-row
// K-step the A and B panels (256 columns x 64 rows x bf16 = 32 KB each) are copied
// global -> LDS with global_load_lds_dwordx4 (no VGPR round trip), double buffered so
// the copy of step s+1 overlaps the 64 MFMAs/wave of step s. The LDS image is written
// lane-linearly, so the per-column XOR swizzle of the 16-byte chunks is applied on the
// SOURCE address (chunk (l&7)^(col&7) lands at position l&7) and undone on the read.
constexpr int GT = 256;
constexpr int GK = 64;

__device__ __forceinline__ void glds16(const void* src, bf16_t* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(lds_base), 16, 0, 0);
}

__global__ __launch_bounds__(512) void gram_bf16_256_kernel(
    const bf16_t* __restrict__ X, int64_t ld, const int2* __restrict__ tiles, int ntiles,
    const Chunk* __restrict__ chunks, int nchunks, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2][2][GT * GK];   // 128 KB
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int c = L / ntiles, t = L % ntiles;
  const Chunk ch = chunks[c];
  const int2 tl = tiles[t];
  const bool diag = tl.x == tl.y;
  const int a0 = tl.x * GT, b0 = tl.y * GT;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // each wave issues 4 x 1 KB pieces per panel: piece q covers columns q*8 .. q*8+7
  auto stage = [&](int st, int64_t i0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = wid * 4 + r;
      const int col = q * 8 + (lane >> 3);
      const int cc = (lane & 7) ^ (col & 7);
      glds16(X + (int64_t)(a0 + col) * ld + i0 + cc * 8, &lds[st][0][q * 8 * GK]);
      if (!diag) glds16(X + (int64_t)(b0 + col) * ld + i0 + cc * 8, &lds[st][1][q * 8 * GK]);
    }
  };

  const int64_t nsteps = (ch.row1 - ch.row0) / GK;
  if (nsteps > 0) stage(0, ch.row0);
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
  __syncthreads();
  for (int64_t s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    if (s + 1 < nsteps) stage(cur ^ 1, ch.row0 + (s + 1) * GK);
    const bf16_t* As = lds[cur][0];
    const bf16_t* Bs = diag ? lds[cur][0] : lds[cur][1];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int cc = kk * 4 + (lane >> 4);
      bf16x8 af[8], bfr[4];
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int col = wr * 128 + m * 16 + (lane & 15);
        af[m] = *reinterpret_cast<const bf16x8*>(&As[col * GK + ((cc ^ (col & 7)) << 3)]);
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int col = wc * 64 + n * 16 + (lane & 15);
        bfr[n] = *reinterpret_cast<const bf16x8*>(&Bs[col * GK + ((cc ^ (col & 7)) << 3)]);
      }
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): next stage landed
    __syncthreads();
  }
  float* out = slab + ((int64_t)c * ntiles + t) * (GT * GT);
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 128 + m * 16 + (lane >> 4) * 4 + r;
        const int col = wc * 64 + n * 16 + (lane & 15);
        out[row * GT + col] = acc[m][n][r];
      }
}

// ------------------------------------------------------------------ bf16 256x256, 4-stage pipeline
// Same 8-wave 2x4 decomposition as above, but the K-step is ONE MFMA deep (32 rows) and
// the LDS holds NST = 4 stages (4 x (A+B) x 256 cols x 64 B = 128 KB), so three stages of
// LDS-DMA are in flight while a stage is consumed (~3 x 1000 MFMA cycles of prefetch
// distance instead of one step). The barrier is a raw s_barrier preceded by a COUNTED
// vmcnt (stages still allowed in flight x glds per stage), never a vmcnt(0) drain.
// LDS image of a stage: column-major, 64 B (4 chunks of 8 rows) per column; logical
// chunk cc of column c sits at position cc ^ H[(c >> 2) & 3] with H = {0,3,2,1}, which
// makes every 16-lane group of a ds_read_b128 fragment load hit 16 distinct 4-bank
// groups (conflict-free). The swizzle is applied on the DMA source address.
constexpr int PK = 32;
constexpr int NST = 4;

__device__ __forceinline__ int pk_swz(int col) { return (0x1230 >> (((col >> 2) & 3) * 4)) & 3; }

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 16, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt(0x0F70 | N);
}

__device__ __forceinline__ void wait_vm_rt(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<1>(); break;
    case 2: wait_vm<2>(); break;
    case 3: wait_vm<3>(); break;
    case 4: wait_vm<4>(); break;
    case 5: wait_vm<5>(); break;
    case 6: wait_vm<6>(); break;
    case 7: wait_vm<7>(); break;
    default: wait_vm<8>(); break;
  }
}

__global__ __launch_bounds__(512) void gram_bf16_256p_kernel(
    const bf16_t* __restrict__ X, int64_t ld, const int2* __restrict__ tiles, int ntiles,
    const Chunk* __restrict__ chunks, int nchunks, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[NST][2][GT * PK];   // 128 KB
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int c = L / ntiles, t = L % ntiles;
  const Chunk ch = chunks[c];
  const int2 tl = tiles[t];
  const bool diag = tl.x == tl.y;
  const int a0 = tl.x * GT, b0 = tl.y * GT;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // a stage = 16 pieces of 1 KB (16 columns x 64 B) per operand; wave w stages pieces
  // 2w, 2w+1 of A (and of B off the diagonal): 2 or 4 glds per wave per stage
  const int per_stage = diag ? 2 : 4;
  const int scol = lane >> 2;
  auto stage = [&](int st, int64_t i0) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int q = wid * 2 + r;
      const int col = q * 16 + scol;
      const int cc = (lane & 3) ^ pk_swz(col);
      glds16(X + (int64_t)(a0 + col) * ld + i0 + cc * 8, &lds[st][0][q * 16 * PK]);
      if (!diag) glds16(X + (int64_t)(b0 + col) * ld + i0 + cc * 8, &lds[st][1][q * 16 * PK]);
    }
  };

  const int nsteps = (int)((ch.row1 - ch.row0) / PK);
#pragma unroll
  for (int j = 0; j < NST - 1; ++j)
    if (j < nsteps) stage(j, ch.row0 + (int64_t)j * PK);

  const int fc = lane & 15, kc = lane >> 4;
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s % NST;
    // stage s landed (this wave's part) once at most `ahead` later stages are pending
    const int ahead = min(NST - 2, nsteps - 1 - s);
    wait_vm_rt(ahead * per_stage);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();   // ... and every wave's part; also retires reads of s-1
    asm volatile("" ::: "memory");
    if (s + NST - 1 < nsteps) stage((s + NST - 1) % NST, ch.row0 + (int64_t)(s + NST - 1) * PK);
    const bf16_t* As = lds[cur][0];
    const bf16_t* Bs = diag ? lds[cur][0] : lds[cur][1];
    bf16x8 af[8], bfr[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = wc * 64 + n * 16 + fc;
      bfr[n] = *reinterpret_cast<const bf16x8*>(&Bs[col * PK + ((kc ^ pk_swz(col)) << 3)]);
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int col = wr * 128 + m * 16 + fc;
      af[m] = *reinterpret_cast<const bf16x8*>(&As[col * PK + ((kc ^ pk_swz(col)) << 3)]);
    }
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
  }
  float* out = slab + ((int64_t)c * ntiles + t) * (GT * GT);
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 128 + m * 16 + (lane >> 4) * 4 + r;
        const int col = wc * 64 + n * 16 + (lane & 15);
        out[row * GT + col] = acc[m][n][r];
      }
}

// ------------------------------------------------------------------ fp32 / fp64 64x64
constexpr int FT = 64;
constexpr int FK = 16;

typedef __attribute__((ext_vector_type(4))) double f64x4;
template <typename T> struct AccT;
template <> struct AccT<float> { typedef f32x4 type; };
template <> struct AccT<double> { typedef f64x4 type; };

__device__ __forceinline__ f32x4 mfma_16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f64x4 mfma_16x16x4(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
// C/D row of accumulator register r: f32 16x16x4 -> (l>>4)*4+r ; f64 16x16x4 -> (l>>4)+4r
__device__ __forceinline__ int acc_row(float, int lane, int r) { return (lane >> 4) * 4 + r; }
__device__ __forceinline__ int acc_row(double, int lane, int r) { return (lane >> 4) + 4 * r; }

template <typename T>
__global__ __launch_bounds__(256) void gram_small_kernel(
    const T* __restrict__ X, int64_t ld, const T* __restrict__ w,
    const int2* __restrict__ tiles, int ntiles, const Chunk* __restrict__ chunks, int nchunks,
    T* __restrict__ slab, const int* __restrict__ done) {
  if (done && *done) return;
  typedef typename AccT<T>::type acc_t;
  __shared__ T lds[2][FT * (FK + 1)];   // [A/B][col*(FK+1)+row], +1 pad vs bank conflicts
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int c = L / ntiles, t = L % ntiles;
  const Chunk ch = chunks[c];
  const int2 tl = tiles[t];
  const int a0 = tl.x * FT, b0 = tl.y * FT;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  acc_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = acc_t{0, 0, 0, 0};

  for (int64_t i0 = ch.row0; i0 < ch.row1; i0 += FK) {
    // stage 64 cols x 16 rows for A (row-weighted) and B: 1024 values each, 4 per thread
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int idx = r * 256 + tid, col = idx >> 4, row = idx & 15;
      int64_t gi = i0 + row;
      T wv = w ? w[gi] : T(1);
      lds[0][col * (FK + 1) + row] = X[(int64_t)(a0 + col) * ld + gi] * wv;
      lds[1][col * (FK + 1) + row] = X[(int64_t)(b0 + col) * ld + gi];
    }
    __syncthreads();
#pragma unroll
    for (int k4 = 0; k4 < FK; k4 += 4) {
      T af[2], bfv[2];
#pragma unroll
      for (int m = 0; m < 2; ++m)
        af[m] = lds[0][(wr * 32 + m * 16 + (lane & 15)) * (FK + 1) + k4 + (lane >> 4)];
#pragma unroll
      for (int n = 0; n < 2; ++n)
        bfv[n] = lds[1][(wc * 32 + n * 16 + (lane & 15)) * (FK + 1) + k4 + (lane >> 4)];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[m][n] = mfma_16x16x4(af[m], bfv[n], acc[m][n]);
    }
    __syncthreads();
  }
  T* out = slab + ((int64_t)c * ntiles + t) * (FT * FT);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int row = wr * 32 + m * 16 + acc_row(T(0), lane, r);
        int col = wc * 32 + n * 16 + (lane & 15);
        out[row * FT + col] = acc[m][n][r];
      }
}

// ------------------------------------------------------------------ slab reduce (fp64, fixed order)
template <typename S>
__global__ void gram_reduce_kernel(const S* __restrict__ slab, int T, const int2* __restrict__ tiles,
                                   int ntiles, const int* __restrict__ seg_chunk0, int nseg, int P,
                                   double* __restrict__ G, const int* __restrict__ done) {
  if (done && *done) return;
  const int tt = T * T;
  const int64_t total = (int64_t)nseg * ntiles * tt;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    int s = (int)(e / ((int64_t)ntiles * tt));
    int rem = (int)(e % ((int64_t)ntiles * tt));
    int t = rem / tt, ij = rem % tt;
    double acc = 0.0;
    for (int c = seg_chunk0[s]; c < seg_chunk0[s + 1]; ++c)
      acc += (double)slab[((int64_t)c * ntiles + t) * tt + ij];
    int a = tiles[t].x * T + ij / T, b = tiles[t].y * T + ij % T;
    double* Gs = G + (int64_t)s * P * P;
    Gs[(int64_t)a * P + b] = acc;
    Gs[(int64_t)b * P + a] = acc;
  }
}

// ------------------------------------------------------------------ host API
// chunks/tiles/seg_chunk0 are device arrays prepared by the caller (ops/gram.py).
// tile = 128 (4 waves, register-staged) or 256 (8 waves, LDS-DMA staged); the caller's
// tile table and chunk plan must use the same tile size.
// variant (tile 256 only): 0 = 4-stage BK=32 pipelined kernel, 1 = 2-stage BK=64 kernel.
ATE_API int ate_gram_bf16(const void* X, int64_t ld, int P, int tile, int variant,
                          const void* tiles, int ntiles, const void* chunks, int nchunks,
                          const void* seg_chunk0, int nseg, void* slab, void* G, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int nwg = nchunks * ntiles;
  if (tile == GT) {
    if (P % GT) return -1;
    if (variant == 0)
      hipLaunchKernelGGL(gram_bf16_256p_kernel, dim3(nwg), dim3(512), 0, s, (const bf16_t*)X, ld,
                         (const int2*)tiles, ntiles, (const Chunk*)chunks, nchunks, (float*)slab);
    else
      hipLaunchKernelGGL(gram_bf16_256_kernel, dim3(nwg), dim3(512), 0, s, (const bf16_t*)X, ld,
                         (const int2*)tiles, ntiles, (const Chunk*)chunks, nchunks, (float*)slab);
  } else if (tile == BT) {
    if (P % BT) return -1;
    hipLaunchKernelGGL(gram_bf16_kernel, dim3(nwg), dim3(256), 0, s, (const bf16_t*)X, ld,
                       (const int2*)tiles, ntiles, (const Chunk*)chunks, nchunks, (float*)slab);
  } else {
    return -1;
  }
  ATE_CHECK_LAUNCH();
  int64_t total = (int64_t)nseg * ntiles * tile * tile;
  hipLaunchKernelGGL(gram_reduce_kernel<float>, dim3(grid_for(total, 256, 4096)), dim3(256), 0, s,
                     (const float*)slab, tile, (const int2*)tiles, ntiles, (const int*)seg_chunk0,
                     nseg, P, (double*)G, (const int*)nullptr);
  ATE_CHECK_LAUNCH();
  return 0;
}

template <typename T>
static int gram_small(const void* X, int64_t ld, int P, const void* w, const void* tiles,
                      int ntiles, const void* chunks, int nchunks, const void* seg_chunk0,
                      int nseg, void* slab, void* G, const void* done, void* stream) {
  if (P % FT) return -1;
  hipStream_t s = (hipStream_t)stream;
  int nwg = nchunks * ntiles;
  hipLaunchKernelGGL(gram_small_kernel<T>, dim3(nwg), dim3(256), 0, s, (const T*)X, ld,
                     (const T*)w, (const int2*)tiles, ntiles, (const Chunk*)chunks, nchunks,
                     (T*)slab, (const int*)done);
  ATE_CHECK_LAUNCH();
  int64_t total = (int64_t)nseg * ntiles * FT * FT;
  hipLaunchKernelGGL(gram_reduce_kernel<T>, dim3(grid_for(total, 256, 4096)), dim3(256), 0, s,
                     (const T*)slab, FT, (const int2*)tiles, ntiles, (const int*)seg_chunk0,
                     nseg, P, (double*)G, (const int*)done);
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_gram_f32(const void* X, int64_t ld, int P, const void* w, const void* tiles,
                         int ntiles, const void* chunks, int nchunks, const void* seg_chunk0,
                         int nseg, void* slab, void* G, const void* done, void* stream) {
  return gram_small<float>(X, ld, P, w, tiles, ntiles, chunks, nchunks, seg_chunk0, nseg, slab, G,
                           done, stream);
}

ATE_API int ate_gram_f64(const void* X, int64_t ld, int P, const void* w, const void* tiles,
                         int ntiles, const void* chunks, int nchunks, const void* seg_chunk0,
                         int nseg, void* slab, void* G, const void* done, void* stream) {
  return gram_small<double>(X, ld, P, w, tiles, ntiles, chunks, nchunks, seg_chunk0, nseg, slab, G,
                            done, stream);
}

ATE_API int ate_gram_tile_sizes(int* bf16_tile, int* bf16_kstep, int* f32_tile, int* f32_kstep) {
  *bf16_tile = BT; *bf16_kstep = BK; *f32_tile = FT; *f32_kstep = FK;
  return 0;
}
