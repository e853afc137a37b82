// Tutorial-shape synthetic DGP generated directly in HBM, and the
// selection-bias transform (K04, ate_replication.Rmd:97-121) applied to GENERATED rows
// before any panel row is written.
//
// Same generative model as ate_replication_causalml_amd/data/dgp.py::raw_columns
// (Philox keyed by (seed, P_DGP, column stream, GLOBAL generated-row id)), so any shard of
// any world size produces identical rows. The model constants arrive as a DgpParams block
// (dgp.py PANEL = the RCT panel, TUTORIAL = the calibrated tutorial model). Writes the
// panel layout of ops/panel.py:
//   [one, 15 cts, sex, 5 vote-history, extras..., W, Y, W_hi, W_lo, Y_hi, Y_lo]
// rows of a segment are written at [row0, row0 + count) of the panel; generated row ids
// come either as gid0 + r or from a gid list (the rows a selection kept).
//
// Selection at scale (data/panel_selection.py): a generated row's selection flag needs only
// yob, city, the latent score, the five vote-history bits and W -- nine Philox draws, no
// panel. Pass 1 (sel_gen_count) counts per-arm candidates per block of SEL_BR generated
// rows (each rank its share of the blocks; the counts are all-reduced); the host then
// finds the generated-row count n_gen whose transform keeps exactly N rows and the two
// thresholds round(0.85 k). Pass 2 (sel_gen_mark) re-derives the flags of the blocks a
// rank needs, ranks the candidates and kept rows in global row order from the blocks'
// prefix counts, and writes the generated ids of the rank's kept-row slices.
#include "common.hpp"

using namespace ate;

namespace {

struct DgpP {
  float intercept, b_hist[5], b_latent, tau_logit, p_treat, thr[5], hist_latent, yob_latent,
      factor_load, factor_rest;
  int uniform_b;      // all b_hist equal: eta uses b * (sum of history bits)
  // the selection rule's parameters at full precision (core_draws works in fp64)
  double p_treat_d, thr_d[5], hist_latent_d, yob_latent_d;
};

DgpP load_params(const double* a) {
  DgpP P;
  P.p_treat_d = a[8];
  for (int k = 0; k < 5; ++k) P.thr_d[k] = a[9 + k];
  P.hist_latent_d = a[14];
  P.yob_latent_d = a[15];
  P.intercept = a[0];
  for (int k = 0; k < 5; ++k) P.b_hist[k] = a[1 + k];
  P.b_latent = a[6];
  P.tau_logit = a[7];
  P.p_treat = a[8];
  for (int k = 0; k < 5; ++k) P.thr[k] = a[9 + k];
  P.hist_latent = a[14];
  P.yob_latent = a[15];
  P.factor_load = a[16];
  P.factor_rest = a[17];
  P.uniform_b = 1;
  for (int k = 1; k < 5; ++k) P.uniform_b &= (P.b_hist[k] == P.b_hist[0]);
  return P;
}

__device__ __forceinline__ float dgp_normal(uint64_t seed, uint32_t stream, uint64_t idx) {
  u32x4 w = rand4(seed, P_DGP, stream, idx);
  float u1 = ((float)(w.x >> 8) + 1.0f) * (1.0f / 16777217.0f);
  float u2 = (float)(w.y >> 8) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}
__device__ __forceinline__ float dgp_uniform(uint64_t seed, uint32_t stream, uint64_t idx) {
  u32x4 w = rand4(seed, P_DGP, stream, idx);
  return (float)(w.x >> 8) * (1.0f / 16777216.0f);
}
// fp64 twins with the host's exact formulas (parallel/rng.py normal_pair / uniform): the
// draws the selection rule reads are computed in fp64 on both sides, so the CPU and the GPU
// panel keep the same rows (a flag can differ only where a draw lies within an ulp of a
// threshold)
__device__ __forceinline__ double dgp_normal_d(uint64_t seed, uint32_t stream, uint64_t idx) {
#pragma clang fp contract(off)
  u32x4 w = rand4(seed, P_DGP, stream, idx);
  const double u1 = ((double)(w.x >> 8) + 1.0) * (1.0 / 16777217.0);
  const double u2 = (double)(w.y >> 8) * (1.0 / 16777216.0);
  return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}
__device__ __forceinline__ double dgp_uniform_d(uint64_t seed, uint32_t stream, uint64_t idx) {
  u32x4 w = rand4(seed, P_DGP, stream, idx);
  return (double)(w.x >> 8) * (1.0 / 16777216.0);
}

// The draws the selection rule reads (one definition for the fill and both selection
// passes, so a kept row's stored values are exactly the ones its flag was computed from)
struct Core {
  double yob, city, latent;
  float w;
  int hist;          // bit k = vote-history column k (g2000, g2002, p2000, p2002, p2004)
};

// fp64, no FMA contraction: the operations of data/dgp.py selection_flags / raw_columns in
// their order (x + a * b as a product, then a sum)
__device__ __forceinline__ Core core_draws(uint64_t seed, uint64_t g, const DgpP& P) {
#pragma clang fp contract(off)
  Core c;
  c.yob = dgp_normal_d(seed, 0, g);    // individual covariates (j < 3): the raw N(0,1) draw
  c.city = dgp_normal_d(seed, 1, g);
  c.latent = dgp_normal_d(seed, 41, g) + P.yob_latent_d * c.yob;
  c.hist = 0;
#pragma unroll
  for (int k = 0; k < 5; ++k)
    c.hist |= (dgp_normal_d(seed, 50 + k, g) + P.hist_latent_d * c.latent > P.thr_d[k])
                  ? (1 << k) : 0;
  c.w = dgp_uniform_d(seed, 61, g) < P.p_treat_d ? 1.f : 0.f;
  return c;
}

// Selection flag of ate_replication.Rmd:103-110 on the population-standardised continuous
// covariates (yob, city are N(0,1) draws: the thresholds are +-2 on the raw values):
// 1 = treated candidate (drop_from_treat; ``last`` = 3 repeats p2002 under quirk Q17, 4 =
// p2004), 2 = control candidate (drop_from_control), 0 = neither.
__device__ __forceinline__ int sel_flag(const Core& c, int last) {
  const int h = c.hist;
  if (c.w == 1.f) {
    const bool d = (h & 0xF) != 0 || ((h >> last) & 1) || c.city > 2.0 || c.yob > 2.0;
    return d ? 1 : 0;
  }
  const bool d = (h & 0x1F) != 0x1F || c.city < -2.0 || c.yob < -2.0;
  return d ? 2 : 0;
}

// element (c, i) at c*cs + (i/64)*bs + i%64: column-major panels (cs = ld, bs = 64) or
// 64-row blocked panels (cs = 64, bs = 64*P; ops/panel.py DevicePanel.blocked)
__device__ __forceinline__ int64_t pidx(int c, int64_t i, int64_t cs, int64_t bs) {
  return (int64_t)c * cs + (i >> 6) * bs + (i & 63);
}
template <typename T>
__device__ __forceinline__ void put(T* X, int64_t cs, int64_t bs, int c, int64_t i, float v) {
  X[pidx(c, i, cs, bs)] = (T)v;
}
template <>
__device__ __forceinline__ void put<bf16_t>(bf16_t* X, int64_t cs, int64_t bs, int c, int64_t i,
                                            float v) {
  X[pidx(c, i, cs, bs)] = f32_to_bf16_rne(v);
}
// an fp64 core draw: stored at the panel's precision (fp64 panels keep every bit)
template <typename T>
__device__ __forceinline__ void put_d(T* X, int64_t cs, int64_t bs, int c, int64_t i, double v) {
  if constexpr (sizeof(T) == 8) X[pidx(c, i, cs, bs)] = (T)v;
  else put(X, cs, bs, c, i, (float)v);
}

// Column c of the generator's order (one, x0..x{p-1}, W, Y[, W_hi, W_lo, Y_hi, Y_lo]) is
// stored at physical column pcol[c] (null: c). X8 (bf16 panels, data/device_dgp.py): the
// one-byte copy of physical columns X8_COL0.. (all {0, 1}-valued), [row block][128][64],
// byte 0x3F for 1 (csrc/gram.hip reads it as bf16 0.5 and scales back). Inside a column's
// 64 bytes, 16-byte piece q holds rows 8q..8q+7 then 32+8q..32+8q+7: the two 8-row groups
// one MFMA lane needs from a 64-row stage, so the Gram reads both with one ds_read_b128.
constexpr int X8_COL0 = 384;
__device__ __forceinline__ int x8_pos(int64_t i) {
  const int r = (int)(i & 63);
  return ((r >> 3) & 3) * 16 + (r >> 5) * 8 + (r & 7);
}

template <typename T>
__global__ void dgp_fill_kernel(T* __restrict__ X, int64_t cs, int64_t bs, int64_t row0, int64_t count,
                                int64_t gid0, const int64_t* __restrict__ gids, uint64_t seed,
                                int p_extra, int hi_lo, DgpP P, const int16_t* __restrict__ pcol,
                                uint8_t* __restrict__ X8) {
  const float FL = P.factor_load, FS = P.factor_rest;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < count;
       r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t g = gids != nullptr ? (uint64_t)gids[r] : (uint64_t)(gid0 + r);
    const int64_t i = row0 + r;
    const Core cr = core_draws(seed, g, P);
    const float f = dgp_normal(seed, 40, g);
    int c = 0;
    auto phys = [&](int cl) { return pcol != nullptr ? (int)pcol[cl] : cl; };
    auto emit = [&](float v) {
      const int pc = phys(c++);
      put(X, cs, bs, pc, i, v);
      if (X8 != nullptr && pc >= X8_COL0) {
        ATE_DASSERT(v == 0.f || v == 1.f);
        X8[(i >> 6) * (128 * 64) + (pc - X8_COL0) * 64 + x8_pos(i)] = v != 0.f ? 0x3F : 0;
      }
    };
    emit(1.0f);
    ATE_DASSERT(phys(1) < X8_COL0 || X8 == nullptr);
    put_d(X, cs, bs, phys(c++), i, cr.yob);
    put_d(X, cs, bs, phys(c++), i, cr.city);
    for (int j = 2; j < 15; ++j) {
      float z = dgp_normal(seed, j, g);
      emit(j < 3 ? z : FL * f + FS * z);
    }
    const float sex = dgp_uniform(seed, 60, g) < 0.5f ? 1.f : 0.f;
    emit(sex);
    float hsum = 0.f, hb = 0.f;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const float h = ((cr.hist >> k) & 1) ? 1.f : 0.f;
      hsum += h;
      hb += P.b_hist[k] * h;
      emit(h);
    }
    for (int j = 0; j < p_extra; ++j) {
      float z = dgp_normal(seed, 100 + j, g);
      float v = (j % 4 == 3) ? (z > 0.f ? 1.f : 0.f) : FL * f + FS * z;
      emit(v);
    }
    const float w = cr.w;
    const float hterm = P.uniform_b ? P.b_hist[0] * hsum : hb;
    const float eta = P.intercept + hterm + P.b_latent * (float)cr.latent + P.tau_logit * w;
    const float y = dgp_uniform(seed, 62, g) < 1.0f / (1.0f + expf(-eta)) ? 1.f : 0.f;
    emit(w);
    emit(y);
    if (hi_lo) {  // binary -> hi exact, lo 0
      emit(w);
      emit(0.f);
      emit(y);
      emit(0.f);
    }
  }
}

constexpr int NT = 256;
constexpr int SEL_BR = 16384;          // generated rows per selection block (64 per thread)

// pass 1: per-arm candidate counts of blocks [b0, b0 + nblk) (rows < n_lim); cnt[2 b + arm]
__global__ __launch_bounds__(NT) void sel_gen_count_kernel(uint64_t seed, DgpP P, int last,
                                                           int64_t b0, int64_t n_lim,
                                                           int64_t* __restrict__ cnt) {
  __shared__ int ws[2][NT / 64];
  const int64_t b = b0 + blockIdx.x;
  const int64_t g0 = b * SEL_BR;
  int ct = 0, cc = 0;
  for (int k = threadIdx.x; k < SEL_BR; k += NT) {
    const int64_t g = g0 + k;
    if (g >= n_lim) break;
    const int f = sel_flag(core_draws(seed, (uint64_t)g, P), last);
    ct += f == 1;
    cc += f == 2;
  }
  ct = wave_sum(ct);
  cc = wave_sum(cc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { ws[0][wid] = ct; ws[1][wid] = cc; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0, c = 0;
    for (int w = 0; w < NT / 64; ++w) { t += ws[0][w]; c += ws[1][w]; }
    cnt[2 * blockIdx.x] = t;
    cnt[2 * blockIdx.x + 1] = c;
  }
}

// flags of generated rows [g0, g0 + count) (the block where the kept count reaches N)
__global__ __launch_bounds__(NT) void sel_gen_flags_kernel(uint64_t seed, DgpP P, int last,
                                                           int64_t g0, int64_t count,
                                                           uint8_t* __restrict__ flags) {
  for (int64_t r = blockIdx.x * (int64_t)NT + threadIdx.x; r < count; r += (int64_t)gridDim.x * NT)
    flags[r] = (uint8_t)sel_flag(core_draws(seed, (uint64_t)(g0 + r), P), last);
}

// block-exclusive scan of NT ints; ws[NT/64] receives the block total
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
  if (threadIdx.x == 0) ws[NT / 64] = tot;
  __syncthreads();
  return off + incl - x;
}

// pass 2: one workgroup per listed block. blk[6 j ..]: generated start, end (clipped at
// n_gen), treated / control candidates before the block, kept rows before the block.
// A kept row with global kept rank q inside slice s ([sl[3s], sl[3s+1]) in kept-rank
// order, output offset sl[3s+2]) writes its generated id to out[sl[3s+2] + q - sl[3s]].
__global__ __launch_bounds__(NT) void sel_gen_mark_kernel(uint64_t seed, DgpP P, int last,
                                                          const int64_t* __restrict__ blk,
                                                          int64_t thr_t, int64_t thr_c,
                                                          const int64_t* __restrict__ sl, int ns,
                                                          int64_t* __restrict__ out, int64_t cap) {
  __shared__ int ws[3][NT / 64 + 1];
  const int64_t* B = blk + 6 * (int64_t)blockIdx.x;
  const int64_t g0 = B[0], g1 = B[1];
  int64_t ct = B[2], cc = B[3], kp = B[4];
  ATE_DASSERT(g1 - g0 <= SEL_BR && g0 <= g1);
  for (int64_t base = g0; base < g1; base += NT) {
    const int64_t g = base + threadIdx.x;
    const int f = g < g1 ? sel_flag(core_draws(seed, (uint64_t)g, P), last) : 0;
    const int et = block_scan(f == 1, ws[0]);
    const int ec = block_scan(f == 2, ws[1]);
    const bool drop = (f == 1 && ct + et < thr_t) || (f == 2 && cc + ec < thr_c);
    const int k = g < g1 && !drop;
    const int ek = block_scan(k, ws[2]);
    if (k) {
      const int64_t q = kp + ek;
      for (int s = 0; s < ns; ++s) {
        if (q >= sl[3 * s] && q < sl[3 * s + 1]) {
          const int64_t o = sl[3 * s + 2] + (q - sl[3 * s]);
          ATE_DASSERT(o >= 0 && o < cap);
          out[o] = g;
          break;
        }
      }
    }
    ct += ws[0][NT / 64];
    cc += ws[1][NT / 64];
    kp += ws[2][NT / 64];
  }
}

}  // namespace

// params: double[18] (data/dgp.py DgpParams.device_block). dtype 1 f32, 2 f64, 3 bf16.
// gids: optional int64 generated-row ids of the count rows (else gid0 + r).
// pcol: int16 physical column of each generator column (null: identity); X8: the one-byte
// copy of physical columns 384..511 (null: none; bf16 panels only).
ATE_API int ate_dgp_fill(int dtype, void* X, int64_t cs, int64_t bs, int64_t row0, int64_t count,
                         int64_t gid0, const void* gids, uint64_t seed, int p_extra, int hi_lo,
                         const void* params, const void* pcol, void* X8, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const DgpP P = load_params((const double*)params);
  const int64_t* gl = (const int64_t*)gids;
  const int16_t* pc = (const int16_t*)pcol;
  dim3 grid(grid_for(count, 256, 8192)), block(256);
  if (X8 != nullptr && dtype != 3) return -1;
  if (dtype == 1)
    ATE_LAUNCH(dgp_fill_kernel<float>, grid, block, 0, s, (float*)X, cs, bs, row0, count, gid0,
                       gl, seed, p_extra, hi_lo, P, pc, (uint8_t*)nullptr);
  else if (dtype == 2)
    ATE_LAUNCH(dgp_fill_kernel<double>, grid, block, 0, s, (double*)X, cs, bs, row0, count,
                       gid0, gl, seed, p_extra, hi_lo, P, pc, (uint8_t*)nullptr);
  else if (dtype == 3)
    ATE_LAUNCH(dgp_fill_kernel<bf16_t>, grid, block, 0, s, (bf16_t*)X, cs, bs, row0, count,
                       gid0, gl, seed, p_extra, hi_lo, P, pc, (uint8_t*)X8);
  else
    return -1;
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_sel_block_rows() { return SEL_BR; }

// per-arm candidate counts of selection blocks [b0, b0 + nblk): cnt int64[2 nblk]
ATE_API int ate_sel_gen_count(uint64_t seed, const void* params, int last, int64_t b0, int64_t nblk,
                              int64_t n_lim, void* cnt, void* stream) {
  if (nblk <= 0) return 0;
  const DgpP P = load_params((const double*)params);
  ATE_LAUNCH(sel_gen_count_kernel, dim3((unsigned)nblk), dim3(NT), 0, (hipStream_t)stream,
                     seed, P, last, b0, n_lim, (int64_t*)cnt);
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_sel_gen_flags(uint64_t seed, const void* params, int last, int64_t g0, int64_t count,
                              void* flags, void* stream) {
  if (count <= 0) return 0;
  const DgpP P = load_params((const double*)params);
  ATE_LAUNCH(sel_gen_flags_kernel, dim3(grid_for(count, NT, 4096)), dim3(NT), 0,
                     (hipStream_t)stream, seed, P, last, g0, count, (uint8_t*)flags);
  ATE_CHECK_LAUNCH();
  return 0;
}

// blk: int64[6 nl] (device); sl: int64[3 ns] (device); out: int64[cap] (device)
ATE_API int ate_sel_gen_mark(uint64_t seed, const void* params, int last, const void* blk, int64_t nl,
                             int64_t thr_t, int64_t thr_c, const void* sl, int ns, void* out,
                             int64_t cap, void* stream) {
  if (nl <= 0) return 0;
  const DgpP P = load_params((const double*)params);
  ATE_LAUNCH(sel_gen_mark_kernel, dim3((unsigned)nl), dim3(NT), 0, (hipStream_t)stream,
                     seed, P, last, (const int64_t*)blk, thr_t, thr_c, (const int64_t*)sl, ns,
                     (int64_t*)out, cap);
  ATE_CHECK_LAUNCH();
  return 0;
}
