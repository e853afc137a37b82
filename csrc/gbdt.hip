// Histogram gradient-boosted trees (extension nuisance learner, BASELINE config 5).
// Spec and numpy reference: ate_replication_causalml_amd/reference/gbdt.py.
//
// * gradients/hessians are int64 fixed point (2^-28): every histogram sum is an exact
//   integer, so LDS/global atomics in any order, row shards + RCCL all-reduce (C04),
//   and the host reference all produce the same bits;
// * level-wise growth, heap-indexed trees; per level: hist (LDS int64 atomics, F
//   features per workgroup so the row's node id and gradient pair are loaded once per
//   F features; F = 32 / nodes so the LDS histogram stays <= 128 KB), split search
//   (one workgroup per node, wave-parallel prefix over 256 bins, deterministic
//   (gain, feature, bin) tie-break), partition (row -> child id);
// * compiled with -ffp-contract=off: the split gains round exactly like numpy's.
#include "common.hpp"

namespace {

constexpr int NT = 256;
constexpr double GFIX = 268435456.0;   // 2^28

typedef unsigned long long u64;

// g, h of the loss at the current raw score; rows outside the training set get node -1
__global__ __launch_bounds__(NT) void gbdt_grad_kernel(int loss, const double* __restrict__ f,
                                                       const double* __restrict__ y,
                                                       const uint8_t* __restrict__ train,
                                                       int64_t n, int64_t* __restrict__ gh,
                                                       int32_t* __restrict__ node,
                                                       int64_t* __restrict__ root) {
  __shared__ int64_t red[2][NT / 64];
  int64_t sg = 0, sh = 0;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    if (!train[i]) {
      node[i] = -1;
      continue;
    }
    double g, h;
    if (loss == 0) {
      g = f[i] - y[i];
      h = 1.0;
    } else {
      const double s = 1.0 / (1.0 + exp(-f[i]));
      g = s - y[i];
      h = fmax(s * (1.0 - s), 1e-16);
    }
    const int64_t G = llrint(g * GFIX), H = llrint(h * GFIX);
    gh[2 * i] = G;
    gh[2 * i + 1] = H;
    node[i] = 0;
    sg += G;
    sh += H;
  }
  sg = ate::wave_sum(sg);
  sh = ate::wave_sum(sh);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { red[0][wid] = sg; red[1][wid] = sh; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t a = 0, b = 0;
    for (int w = 0; w < NT / 64; ++w) { a += red[0][w]; b += red[1][w]; }
    atomicAdd((u64*)&root[0], (u64)a);
    atomicAdd((u64*)&root[1], (u64)b);
  }
}

// H[((k*p + j)*256 + b)*2 + c] += sum over rows of node k with bin b in feature j
__global__ __launch_bounds__(NT) void gbdt_hist_kernel(const uint8_t* __restrict__ Xb, int64_t ld,
                                                       const int32_t* __restrict__ node,
                                                       const int64_t* __restrict__ gh, int64_t n,
                                                       int nn, int p, int F, int64_t chunk,
                                                       int64_t* __restrict__ H) {
  extern __shared__ u64 sh[];                 // [F][nn][256][2]
  const int j0 = blockIdx.y * F;
  const int nf = min(F, p - j0);
  const int tot = nf * nn * 512;
  for (int k = threadIdx.x; k < tot; k += NT) sh[k] = 0;
  __syncthreads();
  const int64_t r0 = blockIdx.x * chunk, r1 = min(n, r0 + chunk);
  for (int64_t i = r0 + threadIdx.x; i < r1; i += NT) {
    const int nd = node[i];
    if (nd < 0) continue;
    const u64 g = (u64)gh[2 * i], h = (u64)gh[2 * i + 1];
    for (int f = 0; f < nf; ++f) {
      const int b = Xb[(int64_t)(j0 + f) * ld + i];
      u64* e = sh + (((int64_t)f * nn + nd) * 256 + b) * 2;
      atomicAdd(e, g);
      atomicAdd(e + 1, h);
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < tot; k += NT) {
    const u64 v = sh[k];
    if (!v) continue;
    const int c = k & 1, b = (k >> 1) & 255, rest = k >> 9;
    const int nd = rest % nn, f = rest / nn;
    atomicAdd((u64*)&H[(((int64_t)nd * p + j0 + f) * 256 + b) * 2 + c], v);
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

// one workgroup per node of level d; writes the split or the leaf value
__global__ __launch_bounds__(NT) void gbdt_split_kernel(const int64_t* __restrict__ H, int nn, int p,
                                                        int d, int depth, double lam,
                                                        int64_t min_child, double min_gain,
                                                        double lr, int64_t* __restrict__ tot,
                                                        int32_t* __restrict__ feat,
                                                        int32_t* __restrict__ thr,
                                                        double* __restrict__ value) {
  __shared__ Best wb[NT / 64];
  __shared__ int64_t wgl[NT / 64], whl[NT / 64];
  const int k = blockIdx.x;
  const int hk = (1 << d) - 1 + k;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (d > 0 && feat[(hk - 1) / 2] < 0) {       // parent is a leaf or absent
    if (threadIdx.x == 0) feat[hk] = -2;
    return;
  }
  const int64_t G = tot[2 * hk], Hh = tot[2 * hk + 1];
  const double gf = (double)G / GFIX, hf = (double)Hh / GFIX;
  Best best{-INFINITY, 0x7fffffff, 0x7fffffff};
  int64_t bgl = 0, bhl = 0;
  if (d < depth) {
    const double parent = gf * gf / (hf + lam);
    for (int j = wid; j < p; j += NT / 64) {
      const int64_t* hj = H + (((int64_t)k * p + j) * 256) * 2;
      int64_t cg[4], ch[4];
      int64_t sg = 0, sh2 = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        sg += hj[(4 * lane + q) * 2];
        sh2 += hj[(4 * lane + q) * 2 + 1];
        cg[q] = sg;
        ch[q] = sh2;
      }
      // exclusive scan of the lane totals across the wave
      int64_t eg = sg, eh = sh2;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int64_t tg = __shfl_up(eg, o, 64), th = __shfl_up(eh, o, 64);
        if (lane >= o) { eg += tg; eh += th; }
      }
      eg -= sg;
      eh -= sh2;
      Best lb{-INFINITY, j, 0x7fffffff};
      int64_t lgl = 0, lhl = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t GL = eg + cg[q], HL = eh + ch[q];
        if (HL >= min_child && Hh - HL >= min_child) {
          const double glf = (double)GL / GFIX, hlf = (double)HL / GFIX;
          const double grf = gf - glf, hrf = hf - hlf;
          const double gain = glf * glf / (hlf + lam) + grf * grf / (hrf + lam) - parent;
          if (better(gain, j, 4 * lane + q, lb)) {
            lb = {gain, j, 4 * lane + q};
            lgl = GL;
            lhl = HL;
          }
        }
      }
      // wave argmax (gain desc, bin asc)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        Best ob;
        ob.gain = __shfl_xor(lb.gain, o, 64);
        ob.j = __shfl_xor(lb.j, o, 64);
        ob.b = __shfl_xor(lb.b, o, 64);
        const int64_t ogl = __shfl_xor(lgl, o, 64), ohl = __shfl_xor(lhl, o, 64);
        if (better(ob.gain, ob.j, ob.b, lb)) { lb = ob; lgl = ogl; lhl = ohl; }
      }
      if (better(lb.gain, lb.j, lb.b, best)) { best = lb; bgl = lgl; bhl = lhl; }
    }
  }
  if (lane == 0) { wb[wid] = best; wgl[wid] = bgl; whl[wid] = bhl; }
  __syncthreads();
  if (threadIdx.x == 0) {
    Best b = wb[0];
    int64_t gl = wgl[0], hl = whl[0];
    for (int w = 1; w < NT / 64; ++w)
      if (better(wb[w].gain, wb[w].j, wb[w].b, b)) { b = wb[w]; gl = wgl[w]; hl = whl[w]; }
    if (d < depth && b.gain > -INFINITY && b.gain > min_gain) {
      feat[hk] = b.j;
      thr[hk] = b.b;
      tot[2 * (2 * hk + 1)] = gl;
      tot[2 * (2 * hk + 1) + 1] = hl;
      tot[2 * (2 * hk + 2)] = G - gl;
      tot[2 * (2 * hk + 2) + 1] = Hh - hl;
    } else {
      feat[hk] = -1;
      value[hk] = -lr * gf / (hf + lam);
    }
  }
}

__global__ __launch_bounds__(NT) void gbdt_partition_kernel(const uint8_t* __restrict__ Xb,
                                                            int64_t ld, int32_t* __restrict__ node,
                                                            int64_t n, int d,
                                                            const int32_t* __restrict__ feat,
                                                            const int32_t* __restrict__ thr) {
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int nd = node[i];
    if (nd < 0) continue;
    const int hk = (1 << d) - 1 + nd;
    const int fj = feat[hk];
    node[i] = fj < 0 ? -1 : 2 * nd + (Xb[(int64_t)fj * ld + i] > thr[hk] ? 1 : 0);
  }
}

// f[i] += value of the leaf row i reaches in the tree (all rows, training or not)
__global__ __launch_bounds__(NT) void gbdt_apply_kernel(const uint8_t* __restrict__ Xb, int64_t ld,
                                                        int64_t n, int ntree, int M,
                                                        const int32_t* __restrict__ feat,
                                                        const int32_t* __restrict__ thr,
                                                        const double* __restrict__ value,
                                                        double* __restrict__ f) {
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    double acc = f[i];
    for (int t = 0; t < ntree; ++t) {
      const int32_t* ft = feat + (int64_t)t * M;
      const int32_t* th = thr + (int64_t)t * M;
      int k = 0;
      while (ft[k] >= 0) k = 2 * k + 1 + (Xb[(int64_t)ft[k] * ld + i] > th[k] ? 1 : 0);
      acc += value[(int64_t)t * M + k];
    }
    f[i] = acc;
  }
}

}  // namespace

ATE_API int ate_gbdt_grad(int loss, const void* f, const void* y, const void* train, int64_t n,
                          void* gh, void* node, void* root, void* stream) {
  hipLaunchKernelGGL(gbdt_grad_kernel, dim3(ate::grid_for(n, NT, 1024)), dim3(NT), 0,
                     (hipStream_t)stream, loss, (const double*)f, (const double*)y,
                     (const uint8_t*)train, n, (int64_t*)gh, (int32_t*)node, (int64_t*)root);
  ATE_CHECK_LAUNCH();
  return 0;
}

// H must be zeroed by the caller ([nn][p][256][2] int64); nn <= 32
ATE_API int ate_gbdt_hist(const void* Xb, int64_t ld, const void* node, const void* gh, int64_t n,
                          int nn, int p, void* H, void* stream) {
  if (nn < 1 || nn > 32) return -1;
  const int F = max(1, min(p, 32 / nn));
  const int64_t chunk = 16384;
  dim3 grid((unsigned)((n + chunk - 1) / chunk), (unsigned)((p + F - 1) / F));
  const size_t shb = (size_t)F * nn * 512 * sizeof(u64);
  hipLaunchKernelGGL(gbdt_hist_kernel, grid, dim3(NT), shb, (hipStream_t)stream,
                     (const uint8_t*)Xb, ld, (const int32_t*)node, (const int64_t*)gh, n, nn, p, F,
                     chunk, (int64_t*)H);
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_gbdt_split(const void* H, int nn, int p, int d, int depth, double lam,
                           int64_t min_child, double min_gain, double lr, void* tot, void* feat,
                           void* thr, void* value, void* stream) {
  hipLaunchKernelGGL(gbdt_split_kernel, dim3(nn), dim3(NT), 0, (hipStream_t)stream,
                     (const int64_t*)H, nn, p, d, depth, lam, min_child, min_gain, lr,
                     (int64_t*)tot, (int32_t*)feat, (int32_t*)thr, (double*)value);
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_gbdt_partition(const void* Xb, int64_t ld, void* node, int64_t n, int d,
                               const void* feat, const void* thr, void* stream) {
  hipLaunchKernelGGL(gbdt_partition_kernel, dim3(ate::grid_for(n, NT, 2048)), dim3(NT), 0,
                     (hipStream_t)stream, (const uint8_t*)Xb, ld, (int32_t*)node, n, d,
                     (const int32_t*)feat, (const int32_t*)thr);
  ATE_CHECK_LAUNCH();
  return 0;
}

ATE_API int ate_gbdt_apply(const void* Xb, int64_t ld, int64_t n, int ntree, int M,
                           const void* feat, const void* thr, const void* value, void* f,
                           void* stream) {
  hipLaunchKernelGGL(gbdt_apply_kernel, dim3(ate::grid_for(n, NT, 2048)), dim3(NT), 0,
                     (hipStream_t)stream, (const uint8_t*)Xb, ld, n, ntree, M,
                     (const int32_t*)feat, (const int32_t*)thr, (const double*)value,
                     (double*)f);
  ATE_CHECK_LAUNCH();
  return 0;
}
