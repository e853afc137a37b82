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
#ifndef GRAM_CPOL
#define GRAM_CPOL 0   // cache policy of the panel stream (2 = nt), A/B builds only
#endif

__device__ __forceinline__ void glds16(const void* src, bf16_t* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(lds_base), 16, 0,
                                   GRAM_CPOL);
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

// ------------------------------------------------------------------ bf16 paired-tile kernel
// Symmetry-aware decomposition for P % 512 == 0. For a pair of 256-column tiles (a, b)
// two workgroups stream the SAME 512 columns of a row chunk:
//   type 0: the off-diagonal tile (a, b), 8 waves x (128 x 64) = 256 16x16 MFMA blocks;
//   type 1: the upper TRIANGLES of both diagonal tiles (a, a) and (b, b) = 2 x 136 blocks.
//           Per diagonal tile: two waves own the 8 x 8-block rectangle (rows 0-127 x cols
//           128-255, 32 blocks each) and two waves the triangles I <= J inside rows/cols
//           0-127 and 128-255 (36 blocks each, 8 fragments serve as both A and B);
//   type 2: type 1 for a single diagonal tile (odd tile count; b's waves idle).
// So MFMA work is 528 blocks per 512 columns instead of 768 (three full 256 tiles), and
// the two workgroups of a chunk read identical byte streams in lockstep (one of them
// hits L2 on what the other fetched). Every wave writes its 16x16 blocks contiguously
// into a 272-block slab slot; a host-built table maps slab blocks to Gram blocks.
constexpr int PAIR_SLOTS = 272;
#ifndef GRAM_NSTAGE
// > 2 (or GRAM_RING=1): the paired-tile K-loop runs a ring of GRAM_NSTAGE stages of 32 rows
// (NSTAGE - 1 of them in flight while one is multiplied) instead of two 64-row stages (one
// in flight). Measured slower (profiles/r05_gram_ring): A/B builds only.
#define GRAM_NSTAGE 2
#endif
#ifndef GRAM_RING
#define GRAM_RING (GRAM_NSTAGE > 2)
#endif
constexpr int PKS = GRAM_RING ? 32 : GK;                     // rows per stage
constexpr int PNS = GRAM_NSTAGE;                             // stages in the ring
constexpr int PAIR_LDS = PNS * 2 * GT * PKS;                 // bf16 elements
static_assert(PAIR_LDS * 2 <= 160 * 1024, "paired-tile LDS ring exceeds 160 KB");

// s_waitcnt vmcnt(n) for a runtime n <= 15 (expcnt / lgkmcnt not waited on)
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
#define WV(k) case k: __builtin_amdgcn_s_waitcnt(0x0F70 | k); break;
    WV(0) WV(1) WV(2) WV(3) WV(4) WV(5) WV(6) WV(7)
    WV(8) WV(9) WV(10) WV(11) WV(12) WV(13) WV(14) WV(15)
#undef WV
    default: __builtin_amdgcn_s_waitcnt(0x0F70); break;
  }
}
#ifndef GRAM_CROSS
// 1: the two workgroups of a chunk issue a stage's 64 LDS-DMA pieces in crossed orders
// (type-1 wave w issues what type-0 wave (w+4)%8 issues), so the pair never requests the same
// line at the same moment; tools/hbm_stream.hip: a paired stream 4.5 -> 5.3 TB/s of unique
// bytes. 2: type 1 issues its B pieces before its A pieces instead. 0: same order.
// In the Gram itself neither changed anything (tile kernel 2.63 / 2.62 / 2.69 ms for 1 / 0 /
// 2, bench step 3.81 / 3.83, profiles/r02c_gram/ab_cross.log): kept as an option, default 0.
#define GRAM_CROSS 0
#endif
#ifndef GRAM_PRELOAD
// 1: both 32-row halves' fragments of a stage are read before its MFMAs, the second half's
// reads interleaved one per MFMA of the first (sched_group_barrier): one LDS wait per half
// instead of one per 8 MFMAs. Tile kernel 2.59-2.62 -> 2.55-2.59 ms, same bits
// (profiles/r05_gram_sync)
#define GRAM_PRELOAD 1
#endif
#ifndef GRAM_PRIO
// s_setprio 1 for waves 4-7 of the paired-tile kernel (see gram_bf16_pair_kernel):
// 1 = in every workgroup, 2 = in diagonal-pair workgroups only (their waves 4-7 are the
// heavier triangle waves; the off-diagonal tile's waves are symmetric). Tile kernel, one
// box: none 2.66-2.67, 1: 2.60, 2: 2.57 ms, same bits (profiles/r05_gram_sync)
#define GRAM_PRIO 2
#endif
#ifndef GRAM_DIAG
#define GRAM_DIAG 0   // timing-only builds (tools/gram_diag.py): 1 = no MFMA work, 2 = no DMA,
                      // 3 = 1 with only the off-diagonal tile's workgroups (each K-step
                      // loaded once), 4 = normal work on the off-diagonal tiles only,
                      // 5 = no per-stage barrier (wrong results; the cost of the stage
                      // hand-off between the 8 waves: 2.66 -> 1.90 ms, profiles/r05_gram_sync)
#endif

__device__ __forceinline__ int tri_index(int m, int n) {   // m <= n < 8, row-major triangle
  return m * 8 - (m * (m - 1)) / 2 + (n - m);
}

#ifndef GRAM_BAL
// 1: the diagonal-pair workgroup's eight waves hold 34 blocks each instead of 32 (rectangle)
// and 36 (triangle): each triangle wave's last two blocks, (6, 7) and (7, 7) of its 8-block
// triangle, move to the rectangle wave of the same region and half, which already holds
// both fragments (half 0: A fragments 6, 7; half 1: B fragments 2, 3 = blocks 14, 15). Every
// block still sums the same K sequence: the Gram bits do not change.
#define GRAM_BAL 0
#endif
constexpr int PAIR_RECT = 0, PAIR_RECT_D0 = 1, PAIR_TRI = 2, PAIR_RECT_D1 = 3;
template <int MODE> struct PairRole {
  static constexpr bool TRI = MODE == PAIR_TRI;
  static constexpr int NB = MODE == PAIR_RECT ? 32 : GRAM_BAL ? 34 : TRI ? 36 : 32;
};

// The MFMAs of one 32-deep k-step of a wave role: a rectangle (8 A x 4 B fragments, plus the
// two balanced-away triangle blocks in a diagonal-pair workgroup) or a triangle (8 fragments
// as A and B, blocks m <= n in tri_index order, the last two dropped under GRAM_BAL).
template <int MODE>
__device__ __forceinline__ void pair_mfma(f32x4* acc, const bf16x8* af, const bf16x8* bfr) {
  if constexpr (MODE != PAIR_TRI) {
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
        acc[m * 4 + n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m * 4 + n],
                                                                 0, 0, 0);
    if constexpr (GRAM_BAL && MODE == PAIR_RECT_D0) {
      acc[32] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[6], af[7], acc[32], 0, 0, 0);
      acc[33] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[7], af[7], acc[33], 0, 0, 0);
    }
    if constexpr (GRAM_BAL && MODE == PAIR_RECT_D1) {
      acc[32] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[2], bfr[3], acc[32], 0, 0, 0);
      acc[33] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[3], bfr[3], acc[33], 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = m; n < 8; ++n)
        if (tri_index(m, n) < PairRole<MODE>::NB)
          acc[tri_index(m, n)] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              af[m], af[n], acc[tri_index(m, n)], 0, 0, 0);
  }
}

// One wave role for the whole K-loop (MODE: PAIR_TRI = triangle wave, else a rectangle wave;
// PAIR_RECT_D0 / D1 = the rectangle waves of a diagonal-pair workgroup, halves 0 / 1). Each
// instantiation keeps only its own accumulators live; every wave runs the same number of
// barriers.
// One-byte columns (X8 != null; P == 512): physical columns 384..511 -- tile b's second half,
// the panel's {0, 1}-valued columns (data/device_dgp.synthetic_panel puts them there) -- are
// also kept as bytes, [row block][128 columns][64 rows], byte 0x3F for 1. The B image of a
// stage then holds tile b's columns 0..127 as bf16 and 128..255 as bytes (24 KB instead of
// 32: a chunk streams 896 instead of 1,024 bytes per row). A byte column's 16-byte piece q
// (rows 8q..8q+7 and 32+8q..32+8q+7, csrc/dgp.hip x8_pos) sits at slot q ^ ((column >> 1) & 2):
// lane l reads both MFMA halves' rows of its column with one ds_read_b128, conflict-free over
// that instruction's 16-lane groups. v_perm puts each byte into the high byte of a bf16
// (0x3F00 = 0.5), so the MFMA products are exact halves and the slab reduce scales them back
// by 2 per byte column: the same Gram bits.
__device__ __forceinline__ bf16x8 bytes_to_bf16x8(uint2 d) {
  uint4 w;
  w.x = __builtin_amdgcn_perm(0u, d.x, 0x010C000Cu);
  w.y = __builtin_amdgcn_perm(0u, d.x, 0x030C020Cu);
  w.z = __builtin_amdgcn_perm(0u, d.y, 0x010C000Cu);
  w.w = __builtin_amdgcn_perm(0u, d.y, 0x030C020Cu);
  return __builtin_bit_cast(bf16x8, w);
}
constexpr int PAIR_BYTE0 = 384;   // first one-byte column (P == 512)

// BYTES: the launch streams one-byte columns (X8 != null); BY: this wave's B fragments
// (rectangle) or all its fragments (triangle) are byte columns.
template <int MODE, bool BYTES, bool BY>
__device__ __forceinline__ void pair_wave(const bf16_t* __restrict__ X, int64_t cs, int64_t bs, int a0,
                                          int b0, bool haveB, bool idle, int abuf, int bbuf,
                                          int arow0, int bcol0, const Chunk& ch,
                                          bf16_t* lds_raw, float* __restrict__ out,
                                          bool second, const uint8_t* __restrict__ X8) {
  constexpr bool TRI = PairRole<MODE>::TRI;
  constexpr int NB = PairRole<MODE>::NB;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  f32x4 acc[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#if GRAM_RING
  // ---- ring of PNS stages of PKS = 32 rows: LDS image [stage][A|B][column][32 rows], four
  // 16-byte pieces per column, piece p stored at slot p ^ ((col >> 1) & 3) (8 consecutive
  // lanes of a fragment read hit 8 distinct 16-byte bank groups)
  (void)second;
  (void)X8;   // one-byte columns: the double-buffered path only
  auto buf = [&](int st, int side) { return lds_raw + (st * 2 + side) * (GT * PKS); };
  auto stage = [&](int st, int64_t i0) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int q = wid * 2 + r;                       // 16-column group
      const int col = q * 16 + (lane >> 2);
      const int pc = (lane & 3) ^ ((col >> 1) & 3);    // piece this lane fetches
      const bf16_t* Xk = X + (i0 >> 6) * bs + (i0 & 63) + pc * 8;
      glds16(Xk + (int64_t)(a0 + col) * cs, buf(st, 0) + q * 16 * PKS);
      if (haveB) glds16(Xk + (int64_t)(b0 + col) * cs, buf(st, 1) + q * 16 * PKS);
    }
  };
  auto frag = [&](const bf16_t* P_, int col, int cc) {
    return *reinterpret_cast<const bf16x8*>(&P_[col * PKS + ((cc ^ ((col >> 1) & 3)) << 3)]);
  };
  const int per = haveB ? 4 : 2;                        // LDS-DMA loads per thread per stage
  const int64_t nsteps = (ch.row1 - ch.row0) / PKS;
  for (int j = 0; j < PNS - 1; ++j)
    if (j < nsteps) stage(j, ch.row0 + j * PKS);
  for (int64_t s = 0; s < nsteps; ++s) {
    // stage s landed: at most the later stages' loads are outstanding
    const int64_t later = nsteps - 1 - s < PNS - 2 ? nsteps - 1 - s : PNS - 2;
    wait_vmcnt((int)later * per);
    // ... in every wave; stage s-1 consumed. A raw s_barrier: __syncthreads()'s fence would
    // drain every LDS-DMA in flight (the later stages' too) and undo the ring (round 6: the
    // rings measured in round 5 had that drain)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (s + PNS - 1 < nsteps) stage((int)((s + PNS - 1) % PNS), ch.row0 + (s + PNS - 1) * PKS);
    const int cur = (int)(s % PNS);
    const bf16_t* As = buf(cur, abuf);
    const bf16_t* Bs = buf(cur, bbuf);
    if (!idle) {
      const int cc = lane >> 4;
      if constexpr (!TRI) {
        bf16x8 af[8], bfr[4];
#pragma unroll
        for (int m = 0; m < 8; ++m) af[m] = frag(As, arow0 + m * 16 + (lane & 15), cc);
#pragma unroll
        for (int n = 0; n < 4; ++n) bfr[n] = frag(Bs, bcol0 + n * 16 + (lane & 15), cc);
        pair_mfma<MODE>(acc, af, bfr);
      } else {
        bf16x8 fr[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) fr[m] = frag(As, arow0 + m * 16 + (lane & 15), cc);
        pair_mfma<MODE>(acc, fr, fr);
      }
    }
  }
#else
  bf16_t (*lds)[2][GT * GK] = reinterpret_cast<bf16_t (*)[2][GT * GK]>(lds_raw);
  // which 8-column pieces this wave copies (any wave may copy any piece: the LDS image only
  // depends on q); `second` = the chunk's type-1 workgroup
  const int qw = (GRAM_CROSS == 1 && second) ? ((wid + 4) & 7) : wid;
  const bool bfirst = GRAM_CROSS == 2 && second && haveB;
  auto stage = [&](int st, int64_t i0) {
    if constexpr (BYTES) {
      // A: 32 pieces of 8 bf16 columns (4 per wave); B: 16 pieces of its bf16 half (2 per
      // wave) and 8 pieces of 16 byte columns (1 per wave)
      const bf16_t* Xk0 = X + (i0 >> 6) * bs;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = wid * 4 + r;
        const int col = q * 8 + (lane >> 3);
        const int cc = (lane & 7) ^ (col & 7);
        glds16(Xk0 + cc * 8 + (int64_t)(a0 + col) * cs, &lds[st][0][q * 8 * GK]);
      }
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int q = wid * 2 + r;
        const int col = q * 8 + (lane >> 3);
        const int cc = (lane & 7) ^ (col & 7);
        glds16(Xk0 + cc * 8 + (int64_t)(b0 + col) * cs, &lds[st][1][q * 8 * GK]);
      }
      const int cb = wid * 16 + (lane >> 2);                  // byte column 0..127
      const int pc = (lane & 3) ^ ((cb >> 1) & 2);             // its 16-byte piece this lane moves
      glds16(X8 + (i0 >> 6) * (128 * GK) + cb * GK + pc * 16,
             reinterpret_cast<bf16_t*>(reinterpret_cast<uint8_t*>(&lds[st][1][128 * GK]) +
                                       wid * 1024));
      return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = qw * 4 + r;
      const int col = q * 8 + (lane >> 3);
      const int cc = (lane & 7) ^ (col & 7);
      const bf16_t* Xk = X + (i0 >> 6) * bs + cc * 8;      // i0: multiple of GK = 64
      if (bfirst) glds16(Xk + (int64_t)(b0 + col) * cs, &lds[st][1][q * 8 * GK]);
      glds16(Xk + (int64_t)(a0 + col) * cs, &lds[st][0][q * 8 * GK]);
      if (haveB && !bfirst) glds16(Xk + (int64_t)(b0 + col) * cs, &lds[st][1][q * 8 * GK]);
    }
  };
  auto frag = [&](const bf16_t* P_, int col, int cc) {
    return *reinterpret_cast<const bf16x8*>(&P_[col * GK + ((cc ^ (col & 7)) << 3)]);
  };
  // a byte column's raw fragments (image column col >= 128: byte column col - 128): both
  // halves of the stage for lane l, rows 8r..8r+7 (.xy) and 32+8r..32+8r+7 (.zw), r = l >> 4.
  // (Round 6 first read each half with its own ds_read_b64 from a 16-row-chunk layout; the
  // compiler paired those into ds_read2st64_b64, which banks mod 32 over 16 lanes: 4e7
  // conflict cycles per launch, profiles/r06_pmc.)
  auto raw16 = [&](const bf16_t* P_, int col) {
    const int cb = col - 128;
    const uint8_t* b8 = reinterpret_cast<const uint8_t*>(P_ + 128 * GK);
    const int slot = (lane >> 4) ^ ((cb >> 1) & 2);
    return *reinterpret_cast<const uint4*>(b8 + cb * GK + slot * 16);
  };
  auto frag8 = [&](const bf16_t* P_, int col, int cc) {
    const uint4 w = raw16(P_, col);
    return bytes_to_bf16x8(cc >= 4 ? make_uint2(w.z, w.w) : make_uint2(w.x, w.y));
  };
  const int64_t nsteps = (ch.row1 - ch.row0) / GK;
  if (nsteps > 0) stage(0, ch.row0);
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
  __syncthreads();
  for (int64_t s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
#if GRAM_DIAG != 2
    if (s + 1 < nsteps) stage(cur ^ 1, ch.row0 + (s + 1) * GK);
#endif
    const bf16_t* As = lds[cur][abuf];
    const bf16_t* Bs = lds[cur][bbuf];
#if GRAM_PRELOAD
    // every fragment of the stage (both 32-row halves) read from LDS up front, then the
    // MFMAs: the waits on LDS leave the MFMA chains of the stage
    if (!idle && GRAM_DIAG != 1 && GRAM_DIAG != 3) {
      if constexpr (BY && !TRI) {
        // byte B fragments: one 16-byte read per column holds both halves' rows, converted
        // per half just ahead of its MFMAs; the second half's conversion interleaved with the
        // first half's MFMAs (mask 0x002 VALU)
        bf16x8 af[2][8];
        uint4 braw[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) braw[n] = raw16(Bs, bcol0 + n * 16 + (lane & 15));
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int cc = kk * 4 + (lane >> 4);
#pragma unroll
          for (int m = 0; m < 8; ++m) af[kk][m] = frag(As, arow0 + m * 16 + (lane & 15), cc);
        }
        bf16x8 b0v[4], b1v[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) b0v[n] = bytes_to_bf16x8(make_uint2(braw[n].x, braw[n].y));
#pragma unroll
        for (int n = 0; n < 4; ++n) b1v[n] = bytes_to_bf16x8(make_uint2(braw[n].z, braw[n].w));
        pair_mfma<MODE>(acc, af[0], b0v);
        pair_mfma<MODE>(acc, af[1], b1v);
        __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);     // B (both halves) + A half 0
        __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);     // half 0 conversion
#pragma unroll
        for (int i = 0; i < 8; ++i) {                           // A half 1 reads beside
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);    // half 0's MFMAs
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {                          // half 1 conversion beside
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);    // the next MFMAs
          __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * NB - 24, 0);
      } else if constexpr (BY) {
        uint4 fraw[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) fraw[m] = raw16(As, arow0 + m * 16 + (lane & 15));
        bf16x8 f0[8], f1[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) f0[m] = bytes_to_bf16x8(make_uint2(fraw[m].x, fraw[m].y));
#pragma unroll
        for (int m = 0; m < 8; ++m) f1[m] = bytes_to_bf16x8(make_uint2(fraw[m].z, fraw[m].w));
        pair_mfma<MODE>(acc, f0, f0);
        pair_mfma<MODE>(acc, f1, f1);
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);      // both halves' reads
        __builtin_amdgcn_sched_group_barrier(0x002, 32, 0);     // half 0 conversion
#pragma unroll
        for (int i = 0; i < 16; ++i) {                          // half 1 conversion beside
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);    // half 0's MFMAs
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * NB - 16, 0);
      } else if constexpr (!TRI) {
        bf16x8 af[2][8], bfr[2][4];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int cc = kk * 4 + (lane >> 4);
#pragma unroll
          for (int m = 0; m < 8; ++m) af[kk][m] = frag(As, arow0 + m * 16 + (lane & 15), cc);
#pragma unroll
          for (int n = 0; n < 4; ++n) bfr[kk][n] = frag(Bs, bcol0 + n * 16 + (lane & 15), cc);
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) pair_mfma<MODE>(acc, af[kk], bfr[kk]);
        // schedule: the first half's 12 reads, then the second half's 12 reads one per
        // MFMA of the first half, then the remaining MFMAs (mask 0x100 DS read, 0x008 MFMA)
        __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
#pragma unroll
        for (int i = 0; i < 12; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * NB - 12, 0);
      } else {
        bf16x8 fr[2][8];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int cc = kk * 4 + (lane >> 4);
#pragma unroll
          for (int m = 0; m < 8; ++m) fr[kk][m] = frag(As, arow0 + m * 16 + (lane & 15), cc);
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) pair_mfma<MODE>(acc, fr[kk], fr[kk]);
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * NB - 8, 0);
      }
    }
#else
    if (!idle && GRAM_DIAG != 1 && GRAM_DIAG != 3) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int cc = kk * 4 + (lane >> 4);
        if constexpr (!TRI) {
          bf16x8 af[8], bfr[4];
#pragma unroll
          for (int m = 0; m < 8; ++m) af[m] = frag(As, arow0 + m * 16 + (lane & 15), cc);
#pragma unroll
          for (int n = 0; n < 4; ++n)
            bfr[n] = BY ? frag8(Bs, bcol0 + n * 16 + (lane & 15), cc)
                        : frag(Bs, bcol0 + n * 16 + (lane & 15), cc);
          pair_mfma<MODE>(acc, af, bfr);
        } else {
          bf16x8 fr[8];
#pragma unroll
          for (int m = 0; m < 8; ++m)
            fr[m] = BY ? frag8(As, arow0 + m * 16 + (lane & 15), cc)
                       : frag(As, arow0 + m * 16 + (lane & 15), cc);
          pair_mfma<MODE>(acc, fr, fr);
        }
      }
    }
#endif
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): next stage landed
#if GRAM_DIAG != 5
    __syncthreads();
#endif
  }
#endif
  if (idle) return;
  // Slab block image is lane-major: float4 `lane` holds acc regs r = 0..3 = (row (l>>4)*4+r,
  // col l&15) of the 16x16 block, so each block is ONE 1-KB dwordx4 store per wave (4x fewer
  // store instructions than a row-major image; the epilogue is store-issue bound).
#pragma unroll
  for (int i = 0; i < NB; ++i)
    *reinterpret_cast<f32x4*>(out + i * 256 + lane * 4) = acc[i];
}

#ifdef GRAM_CLOCK
// profiling build (tools/enet_profile.py --build): per-workgroup shader clock cycles [0] and
// 100 MHz wall ticks [1] of the tile kernel, workgroups [2] (tools/enet_clock.py: the Gram's
// clock alone and beside the CV path kernel)
__device__ unsigned long long gram_clock[3];
extern "C" __attribute__((visibility("default"))) int ate_gram_clock_read(void* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(gram_clock), sizeof(gram_clock));
}
extern "C" __attribute__((visibility("default"))) int ate_gram_clock_reset() {
  static unsigned long long z[3];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(gram_clock), z, sizeof(z));
}
#endif

template <bool BYTES>
__global__ __launch_bounds__(512) void gram_bf16_pair_kernel(
    const bf16_t* __restrict__ X, int64_t cs, int64_t bs, const int4* __restrict__ tiles, int ntiles,
    const Chunk* __restrict__ chunks, int nchunks, float* __restrict__ slab,
    const uint8_t* __restrict__ X8) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[PAIR_LDS];   // 128 KB (ring: up to 160)
#ifdef GRAM_CLOCK
  const unsigned long long gc0 = clock64(), gw0 = wall_clock64();
#endif
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int c = L / ntiles, t = L % ntiles;
  ATE_DASSERT(c < nchunks && t < ntiles);
  const Chunk ch = chunks[c];
  const int4 tl = tiles[t];
  const int type = tl.z;
  // row chunks are whole K-steps of one segment; tiles name 256-column blocks a <= b
  ATE_DASSERT(ch.row0 >= 0 && ch.row0 <= ch.row1 && ch.row0 % GK == 0 && ch.row1 % GK == 0);
  ATE_DASSERT(tl.x >= 0 && tl.y >= tl.x && type >= 0 && type <= 2);
#if GRAM_DIAG >= 3
  if (type != 0) return;
#endif
  const bool haveB = type != 2;
  const int a0 = tl.x * GT, b0 = tl.y * GT;
  const int wid = threadIdx.x >> 6;
  const bool tri = type != 0 && wid >= 4;
  const int region = type == 0 ? 0 : (tri ? (wid - 4) >> 1 : wid >> 1);   // 0: tile a, 1: tile b
  const int half = type == 0 ? 0 : (wid & 1);
  const bool idle = type == 2 && region == 1;
  int arow0, bcol0;
  if (type == 0) { arow0 = (wid >> 2) * 128; bcol0 = (wid & 3) * 64; }
  else if (!tri) { arow0 = 0; bcol0 = 128 + half * 64; }
  else { arow0 = half * 128; bcol0 = half * 128; }
  const int abuf = type == 0 ? 0 : region;
  const int bbuf = type == 0 ? 1 : region;
  constexpr int RS = PairRole<PAIR_RECT_D0>::NB, TS = PairRole<PAIR_TRI>::NB;  // 34 / 34 (32 / 36)
  const int base = type == 0 ? wid * 32 : tri ? 4 * RS + (wid - 4) * TS : wid * RS;
  float* out = slab + ((int64_t)c * ntiles + t) * (PAIR_SLOTS * 256) + (int64_t)base * 256;
#if GRAM_PRIO
  // the second-dispatched half (waves 4-7: the triangle waves of a diagonal pair, the
  // heavier role) loses VALU / LDS issue arbitration to the older half on every stage;
  // one static priority raise for it (uniform branches: readfirstlane, type)
#if GRAM_PRIO == 2
  if (type != 0 && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
#else
  if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
#endif
#endif
  // byte fragments: tile b's columns 128..255 (type 0: the waves of B columns 128..255;
  // type 1, tile b: the rectangle waves' B and the second triangle)
  const bool by = BYTES && (type == 0 ? (wid & 3) >= 2 : region == 1 && (!tri || half == 1));
  ATE_DASSERT(!BYTES || (X8 != nullptr && ntiles == 2 && b0 == 256));
#define PAIR_WAVE(M, B) pair_wave<M, BYTES, B>(X, cs, bs, a0, b0, haveB, idle, abuf, bbuf, arow0, \
                                               bcol0, ch, lds, out, type != 0, X8)
  if (tri) { if (by) PAIR_WAVE(PAIR_TRI, BYTES); else PAIR_WAVE(PAIR_TRI, false); }
  else if (type == 0) { if (by) PAIR_WAVE(PAIR_RECT, BYTES); else PAIR_WAVE(PAIR_RECT, false); }
  else if (half == 0) { if (by) PAIR_WAVE(PAIR_RECT_D0, BYTES); else PAIR_WAVE(PAIR_RECT_D0, false); }
  else { if (by) PAIR_WAVE(PAIR_RECT_D1, BYTES); else PAIR_WAVE(PAIR_RECT_D1, false); }
#undef PAIR_WAVE
#ifdef GRAM_CLOCK
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&gram_clock[0], (unsigned long long)(clock64() - gc0));
    atomicAdd(&gram_clock[1], (unsigned long long)(wall_clock64() - gw0));
    atomicAdd(&gram_clock[2], 1ull);
  }
#endif
}

// ------------------------------------------------------------------ bf16 split-triangle kernel
// P == 512 (32 column blocks of 16). Two workgroups per row chunk, both on one XCD:
//   type 0 ("T"): stages columns 0..351 (22 blocks) and computes the upper triangle of blocks
//                 I <= J < 22 (253 blocks);
//   type 1 ("R"): stages all 512 columns and computes every block with J >= 22 (rows 0..21 x
//                 cols 22..31 and the triangle 22..31: 275 blocks).
// The paired-tile kernel's two workgroups each stage all 512 columns (the second reader of
// every byte hits L2 on the first one's fetch); here only 352 of them are read twice, so a
// chunk moves 864 column-reads into LDS instead of 1024 (-16 %) for the same 528 blocks.
// Each wave owns a fixed role (a rectangle of A x B blocks, a triangle, or the one mixed role),
// described at compile time by its fragment columns and block list; roles hold <= 36 blocks.
constexpr int TRI_SLOTS = 288;            // slab blocks per (chunk, workgroup): 8 waves x 36
constexpr int TRI_SPLIT = 22;             // column blocks staged by the type-0 workgroup

template <int NF> struct FragCols { int c[NF]; };
template <int NB> struct BlockPairs { int a[NB], b[NB]; };

// rect<A0, NA, B0, NB>: fragments A0.., then B0..; block m*NB + n = (A0 + m, B0 + n)
template <int A0, int NA, int B0, int NB>
struct RoleRect {
  static constexpr int NF = NA + NB, NBK = NA * NB;
  static constexpr FragCols<NF> fc() {
    FragCols<NF> r{};
    for (int f = 0; f < NF; ++f) r.c[f] = f < NA ? A0 + f : B0 + (f - NA);
    return r;
  }
  static constexpr BlockPairs<NBK> bp() {
    BlockPairs<NBK> r{};
    for (int m = 0; m < NA; ++m)
      for (int n = 0; n < NB; ++n) { r.a[m * NB + n] = m; r.b[m * NB + n] = NA + n; }
    return r;
  }
};
// tri<S0, S>: fragments S0..S0+S-1 serve as A and B; blocks (m, n), m <= n, row-major
template <int S0, int S>
struct RoleTri {
  static constexpr int NF = S, NBK = S * (S + 1) / 2;
  static constexpr FragCols<NF> fc() {
    FragCols<NF> r{};
    for (int f = 0; f < NF; ++f) r.c[f] = S0 + f;
    return r;
  }
  static constexpr BlockPairs<NBK> bp() {
    BlockPairs<NBK> r{};
    int i = 0;
    for (int m = 0; m < S; ++m)
      for (int n = m; n < S; ++n) { r.a[i] = m; r.b[i] = n; ++i; }
    return r;
  }
};
// the mixed role of type 1: fragments 21..31; (21, 22..26), triangle 22..26, triangle 27..31
struct RoleMix {
  static constexpr int NF = 11, NBK = 35;
  static constexpr FragCols<NF> fc() {
    FragCols<NF> r{};
    for (int f = 0; f < NF; ++f) r.c[f] = 21 + f;
    return r;
  }
  static constexpr BlockPairs<NBK> bp() {
    BlockPairs<NBK> r{};
    int i = 0;
    for (int n = 1; n <= 5; ++n) { r.a[i] = 0; r.b[i] = n; ++i; }
    for (int g = 0; g < 2; ++g)
      for (int m = 0; m < 5; ++m)
        for (int n = m; n < 5; ++n) { r.a[i] = 1 + 5 * g + m; r.b[i] = 1 + 5 * g + n; ++i; }
    return r;
  }
};

// One wave's whole K-loop in its role. The workgroup stages NPC 8-column pieces (columns
// 0 .. 8 NPC - 1) per 64-row stage by LDS-DMA, double buffered; every wave issues its share
// of the pieces, computes the current stage, waits for its own pieces of the next one and
// meets the others at the barrier. PRE: both 32-row halves' fragments read before the MFMAs
// (only where registers allow: 4 NBK + 8 NF <= 224).
template <class R, int NSTG>
__device__ __forceinline__ void tri_role(const bf16_t* __restrict__ X, int64_t cs, int64_t bs,
                                         const Chunk& ch, int npc, bf16_t* lds_raw,
                                         float* __restrict__ out) {
  constexpr int NF = R::NF, NBK = R::NBK;
  constexpr FragCols<NF> FC = R::fc();
  constexpr BlockPairs<NBK> BP = R::bp();
  constexpr bool PRE = 4 * NBK + 8 * NF <= 224;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int stage_elems = npc * 8 * GK;
  const int mine = (npc - wid + 7) >> 3;          // LDS-DMA pieces this wave issues per stage
  f32x4 acc[NBK];
#pragma unroll
  for (int i = 0; i < NBK; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto stage = [&](int st, int64_t i0) {
    bf16_t* dst = lds_raw + st * stage_elems;
    const bf16_t* Xk = X + (i0 >> 6) * bs;
    for (int q = wid; q < npc; q += 8) {
      const int col = q * 8 + (lane >> 3);
      const int cc = (lane & 7) ^ (col & 7);
      glds16(Xk + (int64_t)col * cs + cc * 8, dst + q * 8 * GK);
    }
  };
  auto frag = [&](const bf16_t* P_, int col, int cc) {
    return *reinterpret_cast<const bf16x8*>(&P_[col * GK + ((cc ^ (col & 7)) << 3)]);
  };
  const int64_t nsteps = (ch.row1 - ch.row0) / GK;
#pragma unroll
  for (int j = 0; j < NSTG - 1; ++j)
    if (j < nsteps) stage(j, ch.row0 + j * GK);
  for (int64_t s = 0; s < nsteps; ++s) {
    // stage s landed (this wave's pieces; at most the later stages' are outstanding), then
    // the barrier: every wave's pieces of stage s landed, stage s - 1 consumed by every wave
    // (raw s_barrier, not __syncthreads(): its fence would drain every LDS-DMA in flight,
    // including the later stages'; lgkmcnt(0) retires this wave's reads of stage s - 1, whose
    // buffer the DMA issued after the barrier overwrites)
    if constexpr (NSTG > 2) {
      const int64_t left = nsteps - 1 - s;
      if (left > 0) wait_vmcnt((NSTG - 2) * mine);
      else __builtin_amdgcn_s_waitcnt(0x0F70);
    } else {
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (s + NSTG - 1 < nsteps) stage((int)((s + NSTG - 1) % NSTG), ch.row0 + (s + NSTG - 1) * GK);
    const bf16_t* S_ = lds_raw + (int)(s % NSTG) * stage_elems;
    if constexpr (PRE) {
      bf16x8 fr[2][NF];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int cc = kk * 4 + (lane >> 4);
#pragma unroll
        for (int f = 0; f < NF; ++f) fr[kk][f] = frag(S_, FC.c[f] * 16 + (lane & 15), cc);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int b = 0; b < NBK; ++b)
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[kk][BP.a[b]], fr[kk][BP.b[b]],
                                                           acc[b], 0, 0, 0);
      // the first half's reads, then the second half's reads one per MFMA of the first half
      __builtin_amdgcn_sched_group_barrier(0x100, NF, 0);
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * NBK - NF, 0);
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int cc = kk * 4 + (lane >> 4);
        bf16x8 fr[NF];
#pragma unroll
        for (int f = 0; f < NF; ++f) fr[f] = frag(S_, FC.c[f] * 16 + (lane & 15), cc);
#pragma unroll
        for (int b = 0; b < NBK; ++b)
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[BP.a[b]], fr[BP.b[b]], acc[b],
                                                           0, 0, 0);
      }
    }
  }
  // lane-major 16x16 block images, one dwordx4 store per block (as the paired-tile kernel)
#pragma unroll
  for (int i = 0; i < NBK; ++i)
    *reinterpret_cast<f32x4*>(out + i * 256 + lane * 4) = acc[i];
}

#ifndef GRAM_TRI_NSTG0
// LDS stages of the type-0 workgroup (352 columns x 64 rows = 44 KB each): 3 = two stages in
// flight while one is multiplied (132 KB); the type-1 workgroup's 64 KB stages fit only 2
#define GRAM_TRI_NSTG0 3
#endif
constexpr int TRI_LDS = (GRAM_TRI_NSTG0 * TRI_SPLIT * 16 > 2 * 512 ? GRAM_TRI_NSTG0 * TRI_SPLIT * 16
                                                                   : 2 * 512) * GK;

__global__ __launch_bounds__(512) void gram_bf16_tri_kernel(
    const bf16_t* __restrict__ X, int64_t cs, int64_t bs, const Chunk* __restrict__ chunks,
    int nchunks, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[TRI_LDS];   // 128 / 132 KB
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int c = L >> 1, type = L & 1;
  ATE_DASSERT(c < nchunks);
  const Chunk ch = chunks[c];
  ATE_DASSERT(ch.row0 >= 0 && ch.row0 <= ch.row1 && ch.row0 % GK == 0 && ch.row1 % GK == 0);
  const int wid = threadIdx.x >> 6;
  float* out = slab + ((int64_t)c * 2 + type) * (TRI_SLOTS * 256) + (int64_t)wid * 36 * 256;
  if (type == 0) {
    constexpr int npc = TRI_SPLIT * 2;          // 352 columns = 44 pieces of 8
    switch (wid) {
      case 0: tri_role<RoleTri<0, 8>, GRAM_TRI_NSTG0>(X, cs, bs, ch, npc, lds, out); break;
      case 1: tri_role<RoleTri<8, 8>, GRAM_TRI_NSTG0>(X, cs, bs, ch, npc, lds, out); break;
      case 2: tri_role<RoleRect<0, 4, 8, 8>, GRAM_TRI_NSTG0>(X, cs, bs, ch, npc, lds, out); break;
      case 3: tri_role<RoleRect<4, 4, 8, 8>, GRAM_TRI_NSTG0>(X, cs, bs, ch, npc, lds, out); break;
      case 4: tri_role<RoleRect<0, 6, 16, 6>, GRAM_TRI_NSTG0>(X, cs, bs, ch, npc, lds, out); break;
      case 5: tri_role<RoleRect<6, 5, 16, 6>, GRAM_TRI_NSTG0>(X, cs, bs, ch, npc, lds, out); break;
      case 6: tri_role<RoleRect<11, 5, 16, 6>, GRAM_TRI_NSTG0>(X, cs, bs, ch, npc, lds, out); break;
      default: tri_role<RoleTri<16, 6>, GRAM_TRI_NSTG0>(X, cs, bs, ch, npc, lds, out); break;
    }
  } else {
    constexpr int npc = 64;                     // all 512 columns
    switch (wid) {
      case 0: tri_role<RoleRect<0, 7, 22, 5>, 2>(X, cs, bs, ch, npc, lds, out); break;
      case 1: tri_role<RoleRect<7, 7, 22, 5>, 2>(X, cs, bs, ch, npc, lds, out); break;
      case 2: tri_role<RoleRect<14, 7, 22, 5>, 2>(X, cs, bs, ch, npc, lds, out); break;
      case 3: tri_role<RoleRect<0, 7, 27, 5>, 2>(X, cs, bs, ch, npc, lds, out); break;
      case 4: tri_role<RoleRect<7, 7, 27, 5>, 2>(X, cs, bs, ch, npc, lds, out); break;
      case 5: tri_role<RoleRect<14, 7, 27, 5>, 2>(X, cs, bs, ch, npc, lds, out); break;
      case 6: tri_role<RoleRect<21, 6, 27, 5>, 2>(X, cs, bs, ch, npc, lds, out); break;
      default: tri_role<RoleMix, 2>(X, cs, bs, ch, npc, lds, out); break;
    }
  }
}

// Exact (world-size-invariant) reduction: a chunk partial v is split into two int64 limbs
// of fixed scale, hi = floor(v 2^24), lo = rint((v 2^24 - hi) 2^32) (both exact in fp64),
// and the limbs of all chunks are summed as integers -- associative, so the rank that
// reduces a chunk and the all-reduce order cannot change a bit (ops/exact.py from_limbs).
__device__ __forceinline__ void gram_limbs(double v, long long& hi, long long& lo) {
  const double x = v * 16777216.0;                      // 2^24
  const double h = floor(x);
  hi = (long long)h;
  lo = (long long)rint((x - h) * 4294967296.0);         // 2^32
}

// blocks: [ntiles][PAIR_SLOTS] int2 (I, J) = 16-column block coordinates of the Gram (I: A
// side = row), (-1, -1) = unused slot. Blocks with I == J are full 16x16 diagonal blocks: only
// their r <= c entries are written (plus mirror), so every Gram entry has ONE writer.
// byte0: first one-byte column (their slab partials are halves: scaled back by 2 per byte
// column, exactly), P when there are none.
__global__ void gram_pair_reduce_kernel(const float* __restrict__ slab, const int2* __restrict__ blocks,
                                        int ntiles, int slots, const int* __restrict__ seg_chunk0,
                                        int nseg, int P, double* __restrict__ G,
                                        long long* __restrict__ Gx, int byte0) {
  const int64_t per = (int64_t)ntiles * slots * 256;
  const int64_t total = (int64_t)nseg * per;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int s = (int)(e / per);
    const int64_t rem = e % per;
    const int tb = (int)(rem >> 8);                 // tile * slots + slot
    const int ln = (int)(rem & 255) >> 2;           // lane-major image (pair_wave epilogue)
    const int r = ((ln >> 4) << 2) | (int)(rem & 3), cl = ln & 15;
    const int2 bl = blocks[tb];
    if (bl.x < 0) continue;
    if (bl.x == bl.y && r > cl) continue;
    // fixed chunk order; 8 independent loads in flight per batch
    const int c0 = seg_chunk0[s], c1 = seg_chunk0[s + 1];
    const float* src = slab + rem;
    const int a = bl.x * 16 + r, b = bl.y * 16 + cl;
    ATE_DASSERT(s < nseg && c0 >= 0 && c0 <= c1 && a >= 0 && a < P && b >= 0 && b < P);
    const double sc = (a >= byte0 ? 2.0 : 1.0) * (b >= byte0 ? 2.0 : 1.0);
    if (Gx) {                                       // exact mode: int64 limbs
      long long hs = 0, ls = 0;
      int ci = c0;
      for (; ci + 8 <= c1; ci += 8) {               // 8 independent loads in flight
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(ci + u) * per];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          long long h, l;
          gram_limbs((double)v[u] * sc, h, l);
          hs += h;
          ls += l;
        }
      }
      for (; ci < c1; ++ci) {
        long long h, l;
        gram_limbs((double)src[(int64_t)ci * per] * sc, h, l);
        hs += h;
        ls += l;
      }
      const int64_t PP = (int64_t)nseg * P * P;
      long long* Xs = Gx + (int64_t)s * P * P;
      Xs[(int64_t)a * P + b] = hs;
      Xs[(int64_t)b * P + a] = hs;
      Xs[PP + (int64_t)a * P + b] = ls;
      Xs[PP + (int64_t)b * P + a] = ls;
      continue;
    }
    double acc = 0.0;
    int ci = c0;
    for (; ci + 8 <= c1; ci += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(ci + u) * per];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += (double)v[u];
    }
    for (; ci < c1; ++ci) acc += (double)src[(int64_t)ci * per];
    acc *= sc;
    double* Gs = G + (int64_t)s * P * P;
    Gs[(int64_t)a * P + b] = acc;
    Gs[(int64_t)b * P + a] = acc;
  }
}

ATE_KERNEL_SHAPE("gram_bf16_pair_kernel", 512, 0, gram_bf16_pair_kernel<false>)
ATE_KERNEL_SHAPE("gram_bf16_pair_kernel<bytes>", 512, 0, gram_bf16_pair_kernel<true>)
ATE_KERNEL_SHAPE("gram_bf16_tri_kernel", 512, 0, gram_bf16_tri_kernel)
ATE_KERNEL_SHAPE("gram_bf16_256_kernel", 512, 0, gram_bf16_256_kernel)
ATE_KERNEL_SHAPE("gram_bf16_kernel", 256, 0, gram_bf16_kernel)

// what: 1 = tile kernel (slab partials), 2 = fixed-order slab reduce into G, 3 = both.
// Split so a caller can run the reduce on another stream than the next tile kernel.
// X8: the one-byte copies of columns 384..511 (P == 512 only), or null.
ATE_API int ate_gram_bf16_pair(const void* X, int64_t cs, int64_t bs, int P, const void* tiles, int ntiles,
                               const void* blocks, const void* chunks, int nchunks,
                               const void* seg_chunk0, int nseg, void* slab, void* G, int what,
                               void* Gx, const void* X8, void* stream) {
  if (P % (2 * GT) || what < 1 || what > 3) return -1;
  if (X8 != nullptr && (P != 512 || ntiles != 2 || GRAM_RING)) return -1;
  hipStream_t s = (hipStream_t)stream;
  if (what & 1) {
  if (X8 != nullptr)
    ATE_LAUNCH(gram_bf16_pair_kernel<true>, dim3(nchunks * ntiles), dim3(512), 0, s,
               (const bf16_t*)X, cs, bs, (const int4*)tiles, ntiles, (const Chunk*)chunks,
               nchunks, (float*)slab, (const uint8_t*)X8);
  else
    ATE_LAUNCH(gram_bf16_pair_kernel<false>, dim3(nchunks * ntiles), dim3(512), 0, s,
               (const bf16_t*)X, cs, bs, (const int4*)tiles, ntiles, (const Chunk*)chunks,
               nchunks, (float*)slab, (const uint8_t*)nullptr);
  ATE_CHECK_LAUNCH();
  }
  if (what & 2) {
    const int64_t total = (int64_t)nseg * ntiles * PAIR_SLOTS * 256;
    ATE_LAUNCH(gram_pair_reduce_kernel, dim3(grid_for(total, 256, 4096)), dim3(256), 0, s,
                       (const float*)slab, (const int2*)blocks, ntiles, PAIR_SLOTS,
                       (const int*)seg_chunk0, nseg, P, (double*)G, (long long*)Gx,
                       X8 != nullptr ? PAIR_BYTE0 : P);
    ATE_CHECK_LAUNCH();
  }
  return 0;
}

// The slab layout of the paired-tile kernel's diagonal-pair workgroups (ops/gram.py
// _pair_tiles reads it): 1 = 34 blocks per wave (GRAM_BAL), 0 = 32 / 36.
ATE_API int ate_gram_pair_bal() { return GRAM_BAL; }

// Split-triangle Gram (P == 512): what as ate_gram_bf16_pair; blocks = [2][TRI_SLOTS] int2.
ATE_API int ate_gram_bf16_tri(const void* X, int64_t cs, int64_t bs, int P, const void* blocks,
                              const void* chunks, int nchunks, const void* seg_chunk0, int nseg,
                              void* slab, void* G, int what, void* Gx, void* stream) {
  if (P != 512 || what < 1 || what > 3) return -1;
  hipStream_t s = (hipStream_t)stream;
  if (what & 1) {
    ATE_LAUNCH(gram_bf16_tri_kernel, dim3(nchunks * 2), dim3(512), 0, s,
                       (const bf16_t*)X, cs, bs, (const Chunk*)chunks, nchunks, (float*)slab);
    ATE_CHECK_LAUNCH();
  }
  if (what & 2) {
    const int64_t total = (int64_t)nseg * 2 * TRI_SLOTS * 256;
    ATE_LAUNCH(gram_pair_reduce_kernel, dim3(grid_for(total, 256, 4096)), dim3(256), 0, s,
                       (const float*)slab, (const int2*)blocks, 2, TRI_SLOTS,
                       (const int*)seg_chunk0, nseg, P, (double*)G, (long long*)Gx, P);
    ATE_CHECK_LAUNCH();
  }
  return 0;
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
                                   double* __restrict__ G, const int* __restrict__ done,
                                   long long* __restrict__ Gx) {
  if (done && *done) return;
  const int tt = T * T;
  const int64_t total = (int64_t)nseg * ntiles * tt;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    int s = (int)(e / ((int64_t)ntiles * tt));
    int rem = (int)(e % ((int64_t)ntiles * tt));
    int t = rem / tt, ij = rem % tt;
    // diagonal tiles: only the upper entry of each (i, j) / (j, i) pair is reduced and it
    // writes both G[a][b] and G[b][a] -- ONE writer per Gram entry. (With row weights the
    // tile's (i, j) and (j, i) partials round differently, (x_i w) x_j vs (x_j w) x_i, and
    // two writers made the weighted Gram differ run to run at rounding level.)
    if (tiles[t].x == tiles[t].y && ij / T > ij % T) continue;
    if (Gx) {                                       // exact mode: int64 limbs
      long long hs = 0, ls = 0;
      for (int c = seg_chunk0[s]; c < seg_chunk0[s + 1]; ++c) {
        long long h, l;
        gram_limbs((double)slab[((int64_t)c * ntiles + t) * tt + ij], h, l);
        hs += h;
        ls += l;
      }
      const int a = tiles[t].x * T + ij / T, b = tiles[t].y * T + ij % T;
      const int64_t PP = (int64_t)nseg * P * P;
      long long* Xs = Gx + (int64_t)s * P * P;
      Xs[(int64_t)a * P + b] = hs;
      Xs[(int64_t)b * P + a] = hs;
      Xs[PP + (int64_t)a * P + b] = ls;
      Xs[PP + (int64_t)b * P + a] = ls;
      continue;
    }
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
ATE_API int ate_gram_bf16(const void* X, int64_t ld, int P, int tile,
                          const void* tiles, int ntiles, const void* chunks, int nchunks,
                          const void* seg_chunk0, int nseg, void* slab, void* G, void* Gx,
                          void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int nwg = nchunks * ntiles;
  if (tile == GT) {
    if (P % GT) return -1;
    ATE_LAUNCH(gram_bf16_256_kernel, dim3(nwg), dim3(512), 0, s, (const bf16_t*)X, ld,
                       (const int2*)tiles, ntiles, (const Chunk*)chunks, nchunks, (float*)slab);
  } else if (tile == BT) {
    if (P % BT) return -1;
    ATE_LAUNCH(gram_bf16_kernel, dim3(nwg), dim3(256), 0, s, (const bf16_t*)X, ld,
                       (const int2*)tiles, ntiles, (const Chunk*)chunks, nchunks, (float*)slab);
  } else {
    return -1;
  }
  ATE_CHECK_LAUNCH();
  int64_t total = (int64_t)nseg * ntiles * tile * tile;
  ATE_LAUNCH(gram_reduce_kernel<float>, dim3(grid_for(total, 256, 4096)), dim3(256), 0, s,
                     (const float*)slab, tile, (const int2*)tiles, ntiles, (const int*)seg_chunk0,
                     nseg, P, (double*)G, (const int*)nullptr, (long long*)Gx);
  ATE_CHECK_LAUNCH();
  return 0;
}

template <typename T>
static int gram_small(const void* X, int64_t ld, int P, const void* w, const void* tiles,
                      int ntiles, const void* chunks, int nchunks, const void* seg_chunk0,
                      int nseg, void* slab, void* G, const void* done, void* Gx, void* stream) {
  if (P % FT) return -1;
  hipStream_t s = (hipStream_t)stream;
  int nwg = nchunks * ntiles;
  ATE_LAUNCH(gram_small_kernel<T>, dim3(nwg), dim3(256), 0, s, (const T*)X, ld,
                     (const T*)w, (const int2*)tiles, ntiles, (const Chunk*)chunks, nchunks,
                     (T*)slab, (const int*)done);
  ATE_CHECK_LAUNCH();
  int64_t total = (int64_t)nseg * ntiles * FT * FT;
  ATE_LAUNCH(gram_reduce_kernel<T>, dim3(grid_for(total, 256, 4096)), dim3(256), 0, s,
                     (const T*)slab, FT, (const int2*)tiles, ntiles, (const int*)seg_chunk0,
                     nseg, P, (double*)G, (const int*)done, (long long*)Gx);
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_gram_f32(const void* X, int64_t ld, int P, const void* w, const void* tiles,
                         int ntiles, const void* chunks, int nchunks, const void* seg_chunk0,
                         int nseg, void* slab, void* G, const void* done, void* Gx, void* stream) {
  return gram_small<float>(X, ld, P, w, tiles, ntiles, chunks, nchunks, seg_chunk0, nseg, slab, G,
                        done, Gx, stream);
}

ATE_API int ate_gram_f64(const void* X, int64_t ld, int P, const void* w, const void* tiles,
                         int ntiles, const void* chunks, int nchunks, const void* seg_chunk0,
                         int nseg, void* slab, void* G, const void* done, void* Gx, void* stream) {
  return gram_small<double>(X, ld, P, w, tiles, ntiles, chunks, nchunks, seg_chunk0, nseg, slab, G,
                        done, Gx, stream);
}

ATE_API int ate_gram_tile_sizes(int* bf16_tile, int* bf16_kstep, int* f32_tile, int* f32_kstep) {
  *bf16_tile = BT; *bf16_kstep = BK; *f32_tile = FT; *f32_kstep = FK;
  return 0;
}
