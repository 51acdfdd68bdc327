// Conv front-end epilogue kernels for gfx950: training-mode BatchNorm (eps 1e-3) +
// clipped ReLU(20), forward and backward, with an optional time-major output store.
//
// Reference: src/custom_ops.py:107-160 (batch_norm2 -> fused_batch_norm, is_training)
// and :99-104 (relux); the NCHW -> [T, N, C*F] transpose+reshape of
// src/deepSpeech_NCHW.py:166-168 is fused into the apply kernel's store (layout 1), so
// the RNN input is written once, already time-major and in bf16.
//
// Statistics: per-(channel, chunk) partial sums in fp32 (sum, sum of squares about a
// per-channel shift = first element, which keeps the one-pass variance well conditioned),
// combined in fp64 by a finalize kernel that also updates the running statistics.
#include "common.h"

using namespace ds2;

namespace {

constexpr int BN_THREADS = 256;
constexpr float CLIP = 20.0f;

template <typename T> __device__ __forceinline__ float ldf(const T* p);
template <> __device__ __forceinline__ float ldf<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ldf<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <typename T> __device__ __forceinline__ void stf(T* p, float v);
template <> __device__ __forceinline__ void stf<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void stf<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float r = 0.f;
  if (threadIdx.x < 64) {
    r = (lane < (int)(blockDim.x >> 6)) ? sh[lane] : 0.f;
    r = wave_sum(r);
  }
  return r;   // valid in thread 0
}

// index of element i (flat over [N][TF]) of channel c in NCHW
__device__ __forceinline__ size_t nchw_idx(size_t i, int c, int C, int TF) {
  const size_t n = i / TF, r = i % TF;
  return (n * C + c) * TF + r;
}
// same element in the time-major layout out[T][N][C][F]
__device__ __forceinline__ size_t tmaj_idx(size_t i, int c, int N, int C, int T, int F) {
  const int TF = T * F;
  const size_t n = i / TF, r = i % TF;
  const size_t t = r / F, f = r % F;
  return ((t * N + n) * C + c) * F + f;
}

template <typename TI>
__global__ __launch_bounds__(BN_THREADS) void bn_stats_kernel(const TI* __restrict__ y, int N, int C, int TF,
                                                              float* __restrict__ part) {
  __shared__ float sh[BN_THREADS / 64];
  const int c = blockIdx.y, nb = gridDim.x, j = blockIdx.x;
  const size_t M = (size_t)N * TF;
  const float shift = ldf<TI>(y + (size_t)c * TF);
  float s = 0.f, q = 0.f;
  for (size_t i = (size_t)j * BN_THREADS + threadIdx.x; i < M; i += (size_t)nb * BN_THREADS) {
    const float v = ldf<TI>(y + nchw_idx(i, c, C, TF)) - shift;
    s += v;
    q += v * v;
  }
  s = block_sum(s, sh);
  q = block_sum(q, sh);
  if (threadIdx.x == 0) {
    part[((size_t)c * nb + j) * 2 + 0] = s;
    part[((size_t)c * nb + j) * 2 + 1] = q;
  }
}

template <typename TI>
__global__ void bn_finalize_kernel2(const float* __restrict__ part, int nb, const TI* __restrict__ y, int TF,
                                    int C, double M, float eps, float* mean, float* invstd,
                                    float* run_mean, float* run_var, float momentum) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, q = 0.0;
  for (int j = 0; j < nb; ++j) {
    s += part[((size_t)c * nb + j) * 2 + 0];
    q += part[((size_t)c * nb + j) * 2 + 1];
  }
  const double shift = ldf<TI>(y + (size_t)c * TF);
  const double ms = s / M;
  double var = q / M - ms * ms;
  if (var < 0) var = 0;
  const double mu = ms + shift;
  mean[c] = (float)mu;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (run_mean != nullptr) {
    const double unbiased = M > 1 ? var * M / (M - 1) : var;
    run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * mu);
    run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * unbiased);
  }
}

template <typename TI, typename TO>
__global__ __launch_bounds__(BN_THREADS) void bn_apply_kernel(const TI* __restrict__ y, const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, TO* __restrict__ out,
                                                              int N, int C, int T, int F, int layout) {
  const int c = blockIdx.y;
  const int TF = T * F;
  const size_t M = (size_t)N * TF;
  const float sc = invstd[c] * gamma[c];
  const float sh = beta[c] - mean[c] * sc;
  for (size_t i = (size_t)blockIdx.x * BN_THREADS + threadIdx.x; i < M; i += (size_t)gridDim.x * BN_THREADS) {
    const float v = ldf<TI>(y + nchw_idx(i, c, C, TF));
    const float z = fminf(fmaxf(v * sc + sh, 0.f), CLIP);
    const size_t o = layout == 0 ? nchw_idx(i, c, C, TF) : tmaj_idx(i, c, N, C, T, F);
    stf<TO>(out + o, z);
  }
}

// backward reduce: dbeta = sum(dz), dgamma = sum(dz * xhat), dz = dout * clip-mask
template <typename TI, typename TG>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_reduce_kernel(
    const TG* __restrict__ dout, const TI* __restrict__ y, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma, const float* __restrict__ beta,
    int N, int C, int T, int F, int layout, float* __restrict__ part) {
  __shared__ float sh[BN_THREADS / 64];
  const int c = blockIdx.y, nb = gridDim.x, j = blockIdx.x;
  const int TF = T * F;
  const size_t M = (size_t)N * TF;
  const float mu = mean[c], is = invstd[c], g = gamma[c], bt = beta[c];
  float s = 0.f, q = 0.f;
  for (size_t i = (size_t)j * BN_THREADS + threadIdx.x; i < M; i += (size_t)nb * BN_THREADS) {
    const float xh = (ldf<TI>(y + nchw_idx(i, c, C, TF)) - mu) * is;
    const float z = xh * g + bt;
    const size_t o = layout == 0 ? nchw_idx(i, c, C, TF) : tmaj_idx(i, c, N, C, T, F);
    const float dz = (z > 0.f && z < CLIP) ? ldf<TG>(dout + o) : 0.f;
    s += dz;
    q += dz * xh;
  }
  s = block_sum(s, sh);
  q = block_sum(q, sh);
  if (threadIdx.x == 0) {
    part[((size_t)c * nb + j) * 2 + 0] = s;
    part[((size_t)c * nb + j) * 2 + 1] = q;
  }
}

__global__ void bn_bwd_finalize_kernel(const float* __restrict__ part, int nb, int C, float* dbeta, float* dgamma) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, q = 0.0;
  for (int j = 0; j < nb; ++j) {
    s += part[((size_t)c * nb + j) * 2 + 0];
    q += part[((size_t)c * nb + j) * 2 + 1];
  }
  dbeta[c] = (float)s;
  dgamma[c] = (float)q;
}

template <typename TI, typename TG, typename TD>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_apply_kernel(
    const TG* __restrict__ dout, const TI* __restrict__ y, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ dbeta, const float* __restrict__ dgamma, TD* __restrict__ dy,
    int N, int C, int T, int F, int layout) {
  const int c = blockIdx.y;
  const int TF = T * F;
  const size_t M = (size_t)N * TF;
  const float mu = mean[c], is = invstd[c], g = gamma[c], bt = beta[c];
  const float mdb = dbeta[c] / (float)M, mdg = dgamma[c] / (float)M;
  const float k = g * is;
  for (size_t i = (size_t)blockIdx.x * BN_THREADS + threadIdx.x; i < M; i += (size_t)gridDim.x * BN_THREADS) {
    const size_t src = nchw_idx(i, c, C, TF);
    const float xh = (ldf<TI>(y + src) - mu) * is;
    const float z = xh * g + bt;
    const size_t o = layout == 0 ? src : tmaj_idx(i, c, N, C, T, F);
    const float dz = (z > 0.f && z < CLIP) ? ldf<TG>(dout + o) : 0.f;
    stf<TD>(dy + src, k * (dz - mdb - xh * mdg));
  }
}

int grid_chunks(size_t M) {
  size_t nb = (M + BN_THREADS * 8 - 1) / (BN_THREADS * 8);
  if (nb < 1) nb = 1;
  if (nb > 64) nb = 64;
  return (int)nb;
}

}  // namespace

extern "C" {

// dtype codes: 0 = fp32, 1 = bf16
int ds2_bn_stats(const void* y, int y_bf16, int N, int C, int T, int F, float* part, int nb, float eps,
                 float* mean, float* invstd, float* run_mean, float* run_var, float momentum, hipStream_t st) {
  const int TF = T * F;
  const double M = (double)N * TF;
  if (y_bf16) {
    hipLaunchKernelGGL(bn_stats_kernel<bf16_t>, dim3(nb, C), dim3(BN_THREADS), 0, st, (const bf16_t*)y, N, C, TF, part);
    hipLaunchKernelGGL(bn_finalize_kernel2<bf16_t>, dim3((C + 63) / 64), dim3(64), 0, st, part, nb, (const bf16_t*)y,
                       TF, C, M, eps, mean, invstd, run_mean, run_var, momentum);
  } else {
    hipLaunchKernelGGL(bn_stats_kernel<float>, dim3(nb, C), dim3(BN_THREADS), 0, st, (const float*)y, N, C, TF, part);
    hipLaunchKernelGGL(bn_finalize_kernel2<float>, dim3((C + 63) / 64), dim3(64), 0, st, part, nb, (const float*)y,
                       TF, C, M, eps, mean, invstd, run_mean, run_var, momentum);
  }
  return (int)hipGetLastError();
}

int ds2_bn_chunks(int N, int T, int F) { return grid_chunks((size_t)N * T * F); }

int ds2_bn_apply(const void* y, int y_bf16, const float* mean, const float* invstd, const float* gamma,
                 const float* beta, void* out, int out_bf16, int N, int C, int T, int F, int layout, hipStream_t st) {
  const size_t M = (size_t)N * T * F;
  int nb = (int)((M + BN_THREADS * 4 - 1) / (BN_THREADS * 4));
  if (nb > 1024) nb = 1024;
  const dim3 g(nb, C), b(BN_THREADS);
#define DS2_APPLY(TI, TO) hipLaunchKernelGGL((bn_apply_kernel<TI, TO>), g, b, 0, st, (const TI*)y, mean, invstd, gamma, beta, (TO*)out, N, C, T, F, layout)
  if (y_bf16 && out_bf16) DS2_APPLY(bf16_t, bf16_t);
  else if (y_bf16) DS2_APPLY(bf16_t, float);
  else if (out_bf16) DS2_APPLY(float, bf16_t);
  else DS2_APPLY(float, float);
#undef DS2_APPLY
  return (int)hipGetLastError();
}

int ds2_bn_bwd(const void* dout, int dout_bf16, const void* y, int y_bf16, const float* mean, const float* invstd,
               const float* gamma, const float* beta, float* part, int nb, float* dgamma, float* dbeta, void* dy,
               int dy_bf16, int N, int C, int T, int F, int layout, hipStream_t st) {
  const dim3 gr(nb, C), b(BN_THREADS);
  const size_t M = (size_t)N * T * F;
  int na = (int)((M + BN_THREADS * 4 - 1) / (BN_THREADS * 4));
  if (na > 1024) na = 1024;
  const dim3 ga(na, C);
  if (dy_bf16 != y_bf16) return -30;
#define DS2_BWD(TI, TG)                                                                                      \
  do {                                                                                                       \
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<TI, TG>), gr, b, 0, st, (const TG*)dout, (const TI*)y, mean, invstd, \
                       gamma, beta, N, C, T, F, layout, part);                                               \
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(64), 0, st, part, nb, C, dbeta, dgamma); \
    hipLaunchKernelGGL((bn_bwd_apply_kernel<TI, TG, TI>), ga, b, 0, st, (const TG*)dout, (const TI*)y, mean, invstd, \
                       gamma, beta, dbeta, dgamma, (TI*)dy, N, C, T, F, layout);                             \
  } while (0)
  if (y_bf16 && dout_bf16) DS2_BWD(bf16_t, bf16_t);
  else if (y_bf16) DS2_BWD(bf16_t, float);
  else if (dout_bf16) DS2_BWD(float, bf16_t);
  else DS2_BWD(float, float);
#undef DS2_BWD
  return (int)hipGetLastError();
}

}  // extern "C"
