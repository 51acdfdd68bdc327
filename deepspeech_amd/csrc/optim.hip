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
#include "common.h"

using namespace ds2;

namespace {

constexpr int OPT_THREADS = 256;

__global__ __launch_bounds__(OPT_THREADS) void adam_ema_kernel(
    float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    float* __restrict__ ema, bf16_t* __restrict__ p16, long long n, float lr_t, float b1, float b2, float eps,
    float gscale, float ema_keep, const int* __restrict__ skip) {
  if (skip != nullptr && *skip) return;
  const long long n4 = n / 4;
  const long long stride = (long long)gridDim.x * OPT_THREADS;
  for (long long i = (long long)blockIdx.x * OPT_THREADS + threadIdx.x; i < n4; i += stride) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    const float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float* pa = &pp.x; const float* ga = &gg.x; float* ma = &mm.x; float* va = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = ga[j] * gscale;
      ma[j] = b1 * ma[j] + (1.f - b1) * gj;
      va[j] = b2 * va[j] + (1.f - b2) * gj * gj;
      pa[j] -= lr_t * ma[j] / (sqrtf(va[j]) + eps);
    }
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (ema != nullptr) {
      float4 ee = reinterpret_cast<float4*>(ema)[i];
      ee.x = pp.x + ema_keep * (ee.x - pp.x);
      ee.y = pp.y + ema_keep * (ee.y - pp.y);
      ee.z = pp.z + ema_keep * (ee.z - pp.z);
      ee.w = pp.w + ema_keep * (ee.w - pp.w);
      reinterpret_cast<float4*>(ema)[i] = ee;
    }
    if (p16 != nullptr) {
      ushort4 h;
      h.x = f2bf(pp.x); h.y = f2bf(pp.y); h.z = f2bf(pp.z); h.w = f2bf(pp.w);
      reinterpret_cast<ushort4*>(p16)[i] = h;
    }
  }
  // tail
  for (long long i = n4 * 4 + (long long)blockIdx.x * OPT_THREADS + threadIdx.x; i < n; i += stride) {
    const float gj = g[i] * gscale;
    m[i] = b1 * m[i] + (1.f - b1) * gj;
    v[i] = b2 * v[i] + (1.f - b2) * gj * gj;
    p[i] -= lr_t * m[i] / (sqrtf(v[i]) + eps);
    if (ema != nullptr) ema[i] = p[i] + ema_keep * (ema[i] - p[i]);
    if (p16 != nullptr) p16[i] = f2bf(p[i]);
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
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" {

int ds2_adam_ema(float* p, const float* g, float* m, float* v, float* ema, void* p16, long long n, float lr_t,
                 float b1, float b2, float eps, float gscale, float ema_keep, const int* skip, hipStream_t st) {
  hipLaunchKernelGGL(adam_ema_kernel, dim3(grid_for(n)), dim3(OPT_THREADS), 0, st, p, g, m, v, ema, (bf16_t*)p16, n,
                     lr_t, b1, b2, eps, gscale, ema_keep, skip);
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
