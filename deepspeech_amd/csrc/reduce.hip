// Small gradient reductions that used to run as PyTorch reduce / elementwise / copy kernels in
// the training step (11 at::native::reduce_kernel launches, a 30 us bf16
// reduce, the scale multiply and the copy into the arena per headline step):
//
//   col_sum_kernel   recurrent-layer bias gradients: the BPTT kernels accumulate per-batch-group
//                    partials parts[k][dir][bg][j] in-kernel (csrc/rnn_xcd.hip); this sums the bg
//                    axis of up to 4 such slabs (input bias b and GRU recurrent bias b_h, both
//                    directions) straight into the packed arena rows, written or accumulated.
//                    Reference: src/custom_ops.py:68-71 (B added per step).
//   fc_bias_kernel   FC-head bias gradient db = scale * alpha * sum_rows G[:, :K] of the fused
//                    CTC's bf16 logit gradient G [M, ldg] (scale a device scalar: the upstream
//                    gradient, no host sync; alpha = 1/N), in one 1024-thread workgroup, fixed-order
//                    (bitwise reproducible), into the arena. Reference: src/deepSpeech_NCHW.py:
//                    188-198 (softmax_linear/biases).
// Both are bandwidth-trivial (<= 0.5 MB read); the point is one launch instead of three to five,
// each of which is a ~5 us hole on its stream.
#include "common.h"

using namespace ds2;

namespace {

constexpr int CS_MAX = 4;

struct ColSum {
  const float* in[CS_MAX];    // [R][B][C] contiguous
  float* out[CS_MAX];         // [R][C] contiguous
  int R[CS_MAX], B[CS_MAX], C[CS_MAX];
  int acc[CS_MAX];            // 1: out += sum, 0: out = sum
  long long start[CS_MAX + 1];   // prefix sums of R*C (job boundaries in the flat index space)
  int n;
};

__global__ __launch_bounds__(256) void col_sum_kernel(ColSum a) {
  const long long total = a.start[a.n];
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    int j = 0;
    while (j + 1 < a.n && i >= a.start[j + 1]) ++j;
    const long long e = i - a.start[j];
    const int C = a.C[j], B = a.B[j];
    const long long r = e / C, c = e - r * C;
    const float* p = a.in[j] + r * (long long)B * C + c;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += p[(long long)b * C];      // fixed order over batch groups
    if (a.acc[j]) a.out[j][e] += s;
    else a.out[j][e] = s;
  }
}

// one workgroup: thread (rg, q) = (tid / 4, tid % 4) sums rows rg, rg + 256, ... of the 16-B
// chunk q (8 columns) with one 16-B load per row; the 256 row groups are then reduced through
// LDS in a fixed order (bitwise reproducible). ldg % 8 == 0 and a 16-B aligned G (checked on
// the host) keep every chunk load aligned; columns >= K are loaded and never stored.
__global__ __launch_bounds__(1024) void fc_bias_kernel(const bf16_t* __restrict__ G, int M, int ldg, int K,
                                                       const float* __restrict__ scale, float alpha,
                                                       float* __restrict__ out, int acc) {
  __shared__ float part[256][33];
  const int q = threadIdx.x & 3, rg = threadIdx.x >> 2;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (8 * q < K) {
    for (int m = rg; m < M; m += 256) {
      const i32x4 v = *reinterpret_cast<const i32x4*>(G + (long long)m * ldg + 8 * q);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[2 * i] += bf2f((bf16_t)((unsigned)v[i] & 0xffffu));
        s[2 * i + 1] += bf2f((bf16_t)((unsigned)v[i] >> 16));
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) part[rg][8 * q + i] = s[i];
  __syncthreads();
  const int k = threadIdx.x;
  if (k < K) {
    float t = 0.f;
    for (int r = 0; r < 256; ++r) t += part[r][k];
    t = t * scale[0] * alpha;
    if (acc) out[k] += t;
    else out[k] = t;
  }
}

}  // namespace

extern "C" int ds2_col_sum(int n, const float* const* in, float* const* out, const int* R, const int* B,
                           const int* C, const int* acc, hipStream_t st) {
  if (n < 1 || n > CS_MAX) return -50;
  ColSum a{};
  a.n = n;
  a.start[0] = 0;
  for (int j = 0; j < n; ++j) {
    if (R[j] < 1 || B[j] < 1 || C[j] < 1) return -51;
    a.in[j] = in[j];
    a.out[j] = out[j];
    a.R[j] = R[j];
    a.B[j] = B[j];
    a.C[j] = C[j];
    a.acc[j] = acc[j];
    a.start[j + 1] = a.start[j] + (long long)R[j] * C[j];
  }
  long long blocks = (a.start[n] + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  ds2_launch(col_sum_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

extern "C" int ds2_fc_bias_grad(const void* G, int M, int ldg, int K, const float* scale, float alpha, float* out,
                                int acc, hipStream_t st) {
  if (K < 1 || K > 32 || ldg < 32 || ldg % 8 != 0 || (reinterpret_cast<uintptr_t>(G) & 15) != 0 || M < 0) return -50;
  ds2_launch(fc_bias_kernel, dim3(1), dim3(1024), 0, st, static_cast<const bf16_t*>(G), M, ldg, K, scale, alpha, out,
             acc);
  return (int)hipGetLastError();
}
