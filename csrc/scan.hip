// Exclusive prefix sum without inter-workgroup waiting (reduce -> scan of the tile sums
// -> rescan), for the host loops that run beside other streams' kernels.
//
// Why not torch.cumsum / torch.nonzero there: both run rocprim's single-pass
// decoupled-lookback kernels, whose workgroups spin until their predecessors publish.
// With several forests grown side by side on their own streams (estimators/crossfit.py),
// the config-3 per-GPU shard stalled for 33 s with two such kernels and three others
// resident at once, all ending at the same instant (profiles/r03_cfg3b). Three plain
// launches never wait on another workgroup, so they cannot take part in such a stall.
//
// T = int32 or int64 input, the same type out; out[i] = sum(in[0..i-1]); out[n] = total
// when total != nullptr-style request (tot pointer, may be null).
#include "common.hpp"

using namespace ate;

namespace {

constexpr int SNT = 256;                 // threads per workgroup
constexpr int SPT = 16;                  // elements per thread
constexpr int STILE = SNT * SPT;         // 4096 elements per tile

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

// exclusive scan of one value per thread over the workgroup; returns the workgroup total
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* red, T& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const T inc = wave_incl_scan(v);
  if (lane == 63) red[wid] = inc;
  __syncthreads();
  T off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < SNT / 64; ++w) {
    const T r = red[w];
    off += w < wid ? r : (T)0;
    tot += r;
  }
  __syncthreads();
  total = tot;
  return off + inc - v;
}

template <typename T>
__global__ __launch_bounds__(SNT) void scan_tile_sum_kernel(const T* __restrict__ in, int64_t n,
                                                            T* __restrict__ part) {
  __shared__ T red[SNT / 64];
  const int64_t b0 = (int64_t)blockIdx.x * STILE;
  ATE_DASSERT(b0 < n || n == 0);
  T s = 0;
#pragma unroll
  for (int k = 0; k < SPT; ++k) {
    const int64_t i = b0 + (int64_t)k * SNT + threadIdx.x;
    if (i < n) s += in[i];
  }
  T tot;
  block_excl_scan(s, red, tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// one workgroup: exclusive scan of the nt tile sums in place; *tot = grand total
template <typename T>
__global__ __launch_bounds__(SNT) void scan_parts_kernel(T* __restrict__ part, int64_t nt,
                                                        T* __restrict__ tot) {
  __shared__ T red[SNT / 64];
  T carry = 0;
  for (int64_t c = 0; c < nt; c += SNT) {
    const int64_t i = c + threadIdx.x;
    const T v = i < nt ? part[i] : (T)0;
    T chunk;
    const T ex = block_excl_scan(v, red, chunk);
    if (i < nt) part[i] = carry + ex;
    carry += chunk;
  }
  if (threadIdx.x == 0 && tot) *tot = carry;
}

// each thread owns SPT CONSECUTIVE elements of the tile (sequential sum, then a block scan
// of the thread totals), so reads are per-thread strided; the tile stays L2-resident from
// the first pass's read at this size
template <typename T>
__global__ __launch_bounds__(SNT) void scan_apply_kernel(const T* __restrict__ in, int64_t n,
                                                         const T* __restrict__ part,
                                                         T* __restrict__ out) {
  __shared__ T red[SNT / 64];
  const int64_t b0 = (int64_t)blockIdx.x * STILE + (int64_t)threadIdx.x * SPT;
  T v[SPT];
  T s = 0;
#pragma unroll
  for (int k = 0; k < SPT; ++k) {
    const int64_t i = b0 + k;
    v[k] = i < n ? in[i] : (T)0;
    s += v[k];
  }
  T tot;
  ATE_DASSERT((int64_t)blockIdx.x * STILE < n || n == 0);
  T run = part[blockIdx.x] + block_excl_scan(s, red, tot);
#pragma unroll
  for (int k = 0; k < SPT; ++k) {
    const int64_t i = b0 + k;
    if (i < n) out[i] = run;
    run += v[k];
  }
}

template <typename T>
int launch_scan(const T* in, int64_t n, T* out, T* part, T* tot, hipStream_t st) {
  if (n <= 0) return 0;
  const int64_t nt = (n + STILE - 1) / STILE;
  ATE_LAUNCH(scan_tile_sum_kernel<T>, dim3((unsigned)nt), dim3(SNT), 0, st, in, n, part);
  ATE_LAUNCH(scan_parts_kernel<T>, dim3(1), dim3(SNT), 0, st, part, nt, tot);
  ATE_LAUNCH(scan_apply_kernel<T>, dim3((unsigned)nt), dim3(SNT), 0, st, in, n,
                     (const T*)part, out);
  ATE_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// scratch: ate_scan_parts(n) entries of the element type; tot: optional [1] grand total
ATE_API int64_t ate_scan_parts(int64_t n) { return (n + STILE - 1) / STILE; }

ATE_API int ate_excl_scan_i32(const void* in, int64_t n, void* out, void* part, void* tot,
                              void* stream) {
  return launch_scan((const int32_t*)in, n, (int32_t*)out, (int32_t*)part, (int32_t*)tot,
                     (hipStream_t)stream);
}

ATE_API int ate_excl_scan_i64(const void* in, int64_t n, void* out, void* part, void* tot,
                              void* stream) {
  return launch_scan((const int64_t*)in, n, (int64_t*)out, (int64_t*)part, (int64_t*)tot,
                     (hipStream_t)stream);
}
