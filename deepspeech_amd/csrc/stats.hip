// Device-side summaries and failure detection (no host synchronisation on the step path).
//
//   nonfinite_watch   per-step divergence check of the loss (reference: the NaN assert after
//                     every sess.run, src/deepSpeech_train.py:325): a device step counter and a
//                     sticky "first non-finite step" word, one 1-thread launch per step. The
//                     host reads the word wherever it synchronises anyway, so the check is never
//                     skipped (it reports the exact step) but never stalls the pipeline.
//   hist_stats        tf.summary.histogram + tf.nn.zero_fraction of an activation, weight or
//                     gradient (reference: _activation_summary, src/helper_routines.py:15-28;
//                     grad / var histograms, src/deepSpeech_train.py:401-416) in ONE pass over
//                     the tensor: counts in TensorFlow's default exponential buckets (limits
//                     +-1e-12 * 1.1^i, so no min/max pre-pass is needed) accumulated in LDS per
//                     workgroup, plus per-workgroup min / max / sum / sum of squares / zero /
//                     non-finite partials that the host reduces.
#include "common.h"

using namespace ds2;

namespace {

constexpr int NPOS = 775;                 // positive limits 1e-12 * 1.1^i, i < 774, then DBL_MAX
constexpr int NBUCKET = 2 * NPOS + 1;     // negative mirror + the bucket ending at 0
constexpr int HIST_THREADS = 256;
__constant__ float kLog11Inv = 10.492098f;   // 1 / ln(1.1)

__device__ __forceinline__ int bucket_of(float v) {
  const float a = fabsf(v);
  if (!(a >= 1e-12f)) return NPOS;                                   // (-1e-12, 0] and zero
  int i = (int)floorf(__logf(a * 1e12f) * kLog11Inv);                // largest i: 1e-12*1.1^i <= a
  i = min(max(i, 0), NPOS - 1);
  // positive: first limit >= v is 1e-12*1.1^(i+1) (rounding at exact limits is immaterial)
  return v > 0.f ? min(NPOS + 1 + i + 1, NBUCKET - 1) : max(NPOS - 1 - i, 0);
}

__global__ void nonfinite_watch_kernel(const float* loss, int* counter, int* first_bad) {
  const int s = counter[0];
  const float v = *loss;
  if (!(fabsf(v) <= 3.402823466e38f) && first_bad[0] < 0) first_bad[0] = s;   // NaN or +-inf
  counter[0] = s + 1;
}

template <typename T>
__device__ __forceinline__ float ld(const T* p, long long i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, long long i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, long long i) { return bf2f(p[i]); }

template <typename T>
__global__ __launch_bounds__(HIST_THREADS) void hist_stats_kernel(const T* __restrict__ x, long long n,
                                                                  unsigned* __restrict__ counts,
                                                                  float* __restrict__ part) {
  __shared__ unsigned h[NBUCKET];
  __shared__ float red[HIST_THREADS / 64][6];
  for (int i = threadIdx.x; i < NBUCKET; i += HIST_THREADS) h[i] = 0u;
  __syncthreads();
  float mn = INFINITY, mx = -INFINITY, s = 0.f, q = 0.f, zeros = 0.f, bad = 0.f;
  const long long stride = (long long)gridDim.x * HIST_THREADS;
  for (long long i = (long long)blockIdx.x * HIST_THREADS + threadIdx.x; i < n; i += stride) {
    const float v = ld<T>(x, i);
    if (!(fabsf(v) <= 3.402823466e38f)) {
      bad += 1.f;
      continue;
    }
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
    s += v;
    q += v * v;
    zeros += (v == 0.f) ? 1.f : 0.f;
    atomicAdd(&h[bucket_of(v)], 1u);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, o, 64));
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    s += __shfl_xor(s, o, 64);
    q += __shfl_xor(q, o, 64);
    zeros += __shfl_xor(zeros, o, 64);
    bad += __shfl_xor(bad, o, 64);
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    red[w][0] = mn; red[w][1] = mx; red[w][2] = s; red[w][3] = q; red[w][4] = zeros; red[w][5] = bad;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float r[6] = {red[0][0], red[0][1], red[0][2], red[0][3], red[0][4], red[0][5]};
    for (int k = 1; k < HIST_THREADS / 64; ++k) {
      r[0] = fminf(r[0], red[k][0]); r[1] = fmaxf(r[1], red[k][1]);
      r[2] += red[k][2]; r[3] += red[k][3]; r[4] += red[k][4]; r[5] += red[k][5];
    }
    for (int k = 0; k < 6; ++k) part[(size_t)blockIdx.x * 6 + k] = r[k];
  }
  for (int i = threadIdx.x; i < NBUCKET; i += HIST_THREADS)
    if (h[i]) atomicAdd(&counts[i], h[i]);
}

// CU occupier for co-residency tests: every workgroup spins on s_memrealtime for `ticks`
// (100 MHz) holding its CU slot, like an RCCL channel block for the length of a collective.
__global__ void spin_kernel(long long ticks, int* done) {
  extern __shared__ int spin_lds[];
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 0) {
    spin_lds[0] = 1;
    atomicAdd(done, spin_lds[0]);
  }
}

}  // namespace

extern "C" {

int ds2_spin(long long ticks, int blocks, int threads, int lds_bytes, int* done, hipStream_t st) {
  if (blocks <= 0 || threads <= 0 || threads > 1024 || lds_bytes < 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(threads), lds_bytes, st, ticks, done);
  return (int)hipGetLastError();
}

int ds2_hist_nbucket() { return NBUCKET; }
int ds2_hist_npos() { return NPOS; }

int ds2_hist_blocks(long long n) {
  long long b = (n + HIST_THREADS * 16 - 1) / (HIST_THREADS * 16);
  if (b < 1) b = 1;
  if (b > 1024) b = 1024;
  return (int)b;
}

// counts: [NBUCKET] uint32, ZEROED by the caller; part: [blocks][6] fp32
int ds2_hist_stats(const void* x, int bf16, long long n, unsigned* counts, float* part, int blocks, hipStream_t st) {
  if (bf16)
    hipLaunchKernelGGL(hist_stats_kernel<bf16_t>, dim3(blocks), dim3(HIST_THREADS), 0, st, (const bf16_t*)x, n, counts,
                       part);
  else
    hipLaunchKernelGGL(hist_stats_kernel<float>, dim3(blocks), dim3(HIST_THREADS), 0, st, (const float*)x, n, counts,
                       part);
  return (int)hipGetLastError();
}

int ds2_nonfinite_watch(const float* loss, int* counter, int* first_bad, hipStream_t st) {
  hipLaunchKernelGGL(nonfinite_watch_kernel, dim3(1), dim3(1), 0, st, loss, counter, first_bad);
  return (int)hipGetLastError();
}

}  // extern "C"
