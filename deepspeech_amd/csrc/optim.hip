// Fused Adam + weight EMA over ONE flat fp32 parameter arena (gfx950).
//
// Reference: tf.train.AdamOptimizer (src/deepSpeech_train.py:430,457) followed by
// ExponentialMovingAverage(moving_avg_decay, global_step).apply(trainables)
// (:461-462). TF semantics:
//   lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t)
//   m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2 ; p -= lr_t * m / (sqrt(v) + eps)
//   d = min(decay, (1 + step) / (10 + step)) ; ema -= (1 - d) (ema - p)
// Every trainable parameter is a view into the arena, so the whole optimizer step is a
// single streaming kernel (one read of p,g,m,v,ema; one write of p,m,v,ema and of the
// bf16 compute copy of the weights). The gradient is pre-scaled by `gscale` (1/world for
// the data-parallel mean, or a loss-scale inverse). A separate reduction kernel computes
// the squared gradient norm and a non-finite flag for the NaN guard.
// `hyper` (optional, device [2] fp32 = {lr_t, ema_keep}) replaces the two per-step scalars
// of the argument list: a captured training step (Trainer step graphs) bakes its kernel
// arguments into the graph, so the step-dependent values are read from device memory that
// the host rewrites before each replay.
#include <algorithm>

#include "common.h"

using namespace ds2;

namespace {

constexpr int OPT_THREADS = 256;

// One float4 group: loads issued for U groups before any math (U x 5 loads in flight per
// lane), non-temporal: every byte is touched exactly once per step, so nothing is worth
// keeping in L2 / MALL for the next kernel.
template <typename T>
__device__ __forceinline__ T ld_s(const T* p) { return __builtin_nontemporal_load(p); }
template <typename T>
__device__ __forceinline__ void st_s(T v, T* p) { __builtin_nontemporal_store(v, p); }
// adam1 / ema1 (common.h): one element's update with every rounding spelled out, so the
// vector-group paths, the scalar tail and the fused GEMM epilogue round identically: the
// result of an element does not depend on how the arena is split into launches (Trainer's
// per-layer optimizer ranges are bitwise the single launch).

template <int U>
__device__ __forceinline__ void adam_groups(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                            float* __restrict__ v, float* __restrict__ ema, bf16_t* __restrict__ p16,
                                            long long i0, long long step, float lr_t, float b1, float b2, float eps,
                                            float gscale, float ema_keep) {
  f32x4 pp[U], gg[U], mm[U], vv[U], ee[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = i0 + u * step;
    pp[u] = ld_s(reinterpret_cast<const f32x4*>(p) + i);
    gg[u] = ld_s(reinterpret_cast<const f32x4*>(g) + i);
    mm[u] = ld_s(reinterpret_cast<const f32x4*>(m) + i);
    vv[u] = ld_s(reinterpret_cast<const f32x4*>(v) + i);
    if (ema != nullptr) ee[u] = ld_s(reinterpret_cast<const f32x4*>(ema) + i);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = i0 + u * step;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float pj = pp[u][j], mj = mm[u][j], vj = vv[u][j];
      adam1(pj, gg[u][j], mj, vj, lr_t, b1, b2, eps, gscale);
      pp[u][j] = pj; mm[u][j] = mj; vv[u][j] = vj;
    }
    st_s(pp[u], reinterpret_cast<f32x4*>(p) + i);
    st_s(mm[u], reinterpret_cast<f32x4*>(m) + i);
    st_s(vv[u], reinterpret_cast<f32x4*>(v) + i);
    if (ema != nullptr) {
#pragma unroll
      for (int j = 0; j < 4; ++j) ee[u][j] = ema1(ee[u][j], pp[u][j], ema_keep);
      st_s(ee[u], reinterpret_cast<f32x4*>(ema) + i);
    }
    if (p16 != nullptr) {
      const unsigned lo = (unsigned)f2bf(pp[u][0]) | ((unsigned)f2bf(pp[u][1]) << 16);
      const unsigned hi = (unsigned)f2bf(pp[u][2]) | ((unsigned)f2bf(pp[u][3]) << 16);
      reinterpret_cast<uint2*>(p16)[i] = make_uint2(lo, hi);
    }
  }
}

__global__ __launch_bounds__(OPT_THREADS) void adam_ema_kernel(
    float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    float* __restrict__ ema, bf16_t* __restrict__ p16, long long n, float lr_t, float b1, float b2, float eps,
    float gscale, float ema_keep, const int* __restrict__ skip, const float* __restrict__ hyper) {
  if (skip != nullptr && *skip) return;
  if (hyper != nullptr) { lr_t = hyper[0]; ema_keep = hyper[1]; }
  const long long n4 = n / 4;
  const long long stride = (long long)gridDim.x * OPT_THREADS;
  long long i = (long long)blockIdx.x * OPT_THREADS + threadIdx.x;
  // two float4 groups in flight per lane (four measured no faster)
  for (; i + stride < n4; i += 2 * stride)
    adam_groups<2>(p, g, m, v, ema, p16, i, stride, lr_t, b1, b2, eps, gscale, ema_keep);
  for (; i < n4; i += stride) adam_groups<1>(p, g, m, v, ema, p16, i, stride, lr_t, b1, b2, eps, gscale, ema_keep);
  // tail
  for (long long k = n4 * 4 + (long long)blockIdx.x * OPT_THREADS + threadIdx.x; k < n; k += stride) {
    float pk = p[k], mk = m[k], vk = v[k];
    adam1(pk, g[k], mk, vk, lr_t, b1, b2, eps, gscale);
    p[k] = pk; m[k] = mk; v[k] = vk;
    if (ema != nullptr) ema[k] = ema1(ema[k], pk, ema_keep);
    if (p16 != nullptr) p16[k] = f2bf(pk);
  }
}

// Same update, block-contiguous: block b streams float4 groups [b*chunk, (b+1)*chunk) of every
// array (U groups in flight per lane, lanes 16 B apart), so each CU walks its own contiguous
// pages instead of the whole grid sweeping one stride-spaced front across the arena.
template <int U>
__global__ __launch_bounds__(OPT_THREADS) void adam_ema_chunk_kernel(
    float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    float* __restrict__ ema, bf16_t* __restrict__ p16, long long n, long long chunk4, float lr_t, float b1,
    float b2, float eps, float gscale, float ema_keep, const int* __restrict__ skip,
    const float* __restrict__ hyper) {
  if (skip != nullptr && *skip) return;
  if (hyper != nullptr) { lr_t = hyper[0]; ema_keep = hyper[1]; }
  const long long n4 = n / 4;
  const long long lo = (long long)blockIdx.x * chunk4, hi = min(n4, lo + chunk4);
  long long i = lo + threadIdx.x;
  for (; i + (U - 1) * OPT_THREADS < hi; i += U * OPT_THREADS)
    adam_groups<U>(p, g, m, v, ema, p16, i, OPT_THREADS, lr_t, b1, b2, eps, gscale, ema_keep);
  for (; i < hi; i += OPT_THREADS) adam_groups<1>(p, g, m, v, ema, p16, i, OPT_THREADS, lr_t, b1, b2, eps, gscale, ema_keep);
  if (blockIdx.x == gridDim.x - 1) {                 // tail elements past the last float4
    for (long long k = n4 * 4 + threadIdx.x; k < n; k += OPT_THREADS) {
      float pk = p[k], mk = m[k], vk = v[k];
      adam1(pk, g[k], mk, vk, lr_t, b1, b2, eps, gscale);
      p[k] = pk; m[k] = mk; v[k] = vk;
      if (ema != nullptr) ema[k] = ema1(ema[k], pk, ema_keep);
      if (p16 != nullptr) p16[k] = f2bf(pk);
    }
  }
}

// The same update over a list of arena ranges in ONE launch (the elements of a step that the
// grouped weight-gradient GEMM's fused epilogue did not update: FC head, biases, padding):
// thread i takes float4 group i of the ranges' concatenation. Ranges start and end on
// float4 boundaries (host-checked).
constexpr int ADAM_MAXR = 64;
struct AdamRanges {
  long long lo4[ADAM_MAXR];     // first float4 group of range r
  long long pre4[ADAM_MAXR + 1];  // float4 groups before range r (pre4[nr] = total)
  int nr;
};

__global__ __launch_bounds__(OPT_THREADS) void adam_ema_ranges_kernel(
    float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    float* __restrict__ ema, bf16_t* __restrict__ p16, AdamRanges rg, float lr_t, float b1, float b2, float eps,
    float gscale, float ema_keep, const float* __restrict__ hyper) {
  if (hyper != nullptr) { lr_t = hyper[0]; ema_keep = hyper[1]; }
  const long long total = rg.pre4[rg.nr];
  const long long stride = (long long)gridDim.x * OPT_THREADS;
  int r = 0;
  for (long long i = (long long)blockIdx.x * OPT_THREADS + threadIdx.x; i < total; i += stride) {
    while (i >= rg.pre4[r + 1]) ++r;          // i only grows: the range index only advances
    adam_groups<1>(p, g, m, v, ema, p16, rg.lo4[r] + (i - rg.pre4[r]), 0, lr_t, b1, b2, eps, gscale, ema_keep);
  }
}

// partial sums of g^2 (fp32 per block), plus a non-finite flag
__global__ __launch_bounds__(OPT_THREADS) void grad_norm_kernel(const float* __restrict__ g, long long n, float gscale,
                                                                float* __restrict__ part, int* __restrict__ bad) {
  __shared__ float sh[OPT_THREADS / 64];
  float s = 0.f;
  int nf = 0;
  const long long stride = (long long)gridDim.x * OPT_THREADS;
  for (long long i = (long long)blockIdx.x * OPT_THREADS + threadIdx.x; i < n; i += stride) {
    const float x = g[i] * gscale;
    if (!isfinite(x)) nf = 1;
    s += x * x;
  }
  s = wave_sum(s);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sh[w] = s;
  if (__any(nf) && lane == 0) atomicOr(bad, 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < OPT_THREADS / 64; ++i) t += sh[i];
    part[blockIdx.x] = t;
  }
}

__global__ void cast_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = f2bf(x[i]);
}

int grid_for(long long n) {
  long long g = (n / 4 + OPT_THREADS - 1) / OPT_THREADS;
  if (g > 16384) g = 16384;     // measured (tools/bench_adam.py): 46 M params 270 us at 16384 blocks vs 311 at 2048
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" {

// max_grid > 0 caps the grid (an update issued beside a persistent kernel that holds most
// of the CUs: a few workgroups stream the range instead of queueing behind it)
// lds_reserve > 0: every block also reserves that many bytes of (unused) dynamic LDS, so no
// block fits on a CU whose LDS a persistent recurrence workgroup holds: a range streaming beside
// a forward recurrence (132 KB of LDS per workgroup; 32 KB keeps the blocks off its CUs) then
// runs only on the CUs it leaves idle, several blocks per idle CU.
int ds2_adam_ema(float* p, const float* g, float* m, float* v, float* ema, void* p16, long long n, float lr_t,
                 float b1, float b2, float eps, float gscale, float ema_keep, const int* skip, int max_grid,
                 const float* hyper, int lds_reserve, hipStream_t st) {
  if (lds_reserve > 0) {
    static int configured = 0;
    if (lds_reserve > configured) {
      DS2_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(adam_ema_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, lds_reserve));
      configured = lds_reserve;
    }
    int grid = grid_for(n);
    if (max_grid > 0 && grid > max_grid) grid = max_grid;
    hipLaunchKernelGGL(adam_ema_kernel, dim3(grid), dim3(OPT_THREADS), (unsigned)lds_reserve, st, p, g, m, v, ema,
                       (bf16_t*)p16, n, lr_t, b1, b2, eps, gscale, ema_keep, skip, hyper);
    return (int)hipGetLastError();
  }
  // arenas past ~120 M parameters (config 5: 146 M) stream faster block-contiguous (1098 vs
  // 1200 us, interleaved A/B in tools/bench_adam.py); smaller ones (46 M: 278 vs 328 us, 89 M:
  // 634 vs 748) faster grid-strided
  if (max_grid == 0 && n >= 120000000LL) max_grid = -2048;
  if (max_grid < 0) {                                // block-contiguous variant, grid = -max_grid
    const long long n4 = n / 4;
    const int grid = (int)std::max<long long>(1, std::min<long long>(-max_grid, (n4 + OPT_THREADS - 1) / OPT_THREADS));
    const long long chunk4 = (n4 + grid - 1) / grid;
    hipLaunchKernelGGL(adam_ema_chunk_kernel<2>, dim3(grid), dim3(OPT_THREADS), 0, st, p, g, m, v, ema, (bf16_t*)p16,
                       n, chunk4, lr_t, b1, b2, eps, gscale, ema_keep, skip, hyper);
    return (int)hipGetLastError();
  }
  int grid = grid_for(n);
  if (max_grid > 0 && grid > max_grid) grid = max_grid;
  hipLaunchKernelGGL(adam_ema_kernel, dim3(grid), dim3(OPT_THREADS), 0, st, p, g, m, v, ema, (bf16_t*)p16, n,
                     lr_t, b1, b2, eps, gscale, ema_keep, skip, hyper);
  return (int)hipGetLastError();
}

// lohi: nr (lo, hi) element ranges of the arena, each a multiple of 4 at both ends
int ds2_adam_ema_ranges(float* p, const float* g, float* m, float* v, float* ema, void* p16, const long long* lohi,
                        int nr, float lr_t, float b1, float b2, float eps, float gscale, float ema_keep,
                        const float* hyper, hipStream_t st) {
  if (nr < 0 || nr > ADAM_MAXR) return (int)hipErrorInvalidValue;
  AdamRanges rg;
  rg.nr = nr;
  rg.pre4[0] = 0;
  for (int r = 0; r < nr; ++r) {
    const long long lo = lohi[2 * r], hi = lohi[2 * r + 1];
    if (lo < 0 || hi < lo || lo % 4 || hi % 4) return (int)hipErrorInvalidValue;
    rg.lo4[r] = lo / 4;
    rg.pre4[r + 1] = rg.pre4[r] + (hi - lo) / 4;
  }
  if (rg.pre4[nr] == 0) return 0;
  hipLaunchKernelGGL(adam_ema_ranges_kernel, dim3(grid_for(rg.pre4[nr] * 4)), dim3(OPT_THREADS), 0, st, p, g, m, v,
                     ema, (bf16_t*)p16, rg, lr_t, b1, b2, eps, gscale, ema_keep, hyper);
  return (int)hipGetLastError();
}

int ds2_grad_norm_blocks(long long n) { return grid_for(n * 4 / 4); }

int ds2_grad_norm(const float* g, long long n, float gscale, float* part, int nblocks, int* bad, hipStream_t st) {
  hipLaunchKernelGGL(grad_norm_kernel, dim3(nblocks), dim3(OPT_THREADS), 0, st, g, n, gscale, part, bad);
  return (int)hipGetLastError();
}

int ds2_cast_bf16(const float* x, void* y, long long n, hipStream_t st) {
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid_for(n)), dim3(OPT_THREADS), 0, st, x, (bf16_t*)y, n);
  return (int)hipGetLastError();
}

}  // extern "C"
