// Fused CTC loss + gradient for gfx950 (reference: tf.nn.ctc_loss at
// src/deepSpeech_NCHW.py:225, blank = last class, time-major logits).
//
// One workgroup per utterance:
//   phase 0  log-softmax of every frame t < len into a small global scratch lp[T][32]
//            (one wave per frame, 64-lane reductions);
//   phase 1  alpha recursion over the extended label lattice (2L+1 states), two LDS
//            rows, one barrier per frame; alpha rows spill to global for phase 2;
//   phase 2  beta recursion fused with the gradient: at frame t each state adds its
//            occupancy exp(alpha+beta-lp-logP) into a per-class LDS accumulator with an
//            LDS float atomic, then grad[t][k] = softmax_t(k) - occ_k(t). Frames past
//            the utterance length get a zero gradient.
// Infeasible utterances (logP = -inf) get loss 0 and zero gradient when zero_inf != 0.
#include "common.h"

using namespace ds2;

namespace {

constexpr int CTC_THREADS = 256;
constexpr int KPAD = 32;
constexpr float NEG_INF = -INFINITY;

__device__ __forceinline__ float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == NEG_INF) return NEG_INF;
  return m + __logf(__expf(a - m) + __expf(b - m));
}
__device__ __forceinline__ float lse3(float a, float b, float c) {
  const float m = fmaxf(fmaxf(a, b), c);
  if (m == NEG_INF) return NEG_INF;
  return m + __logf(__expf(a - m) + __expf(b - m) + __expf(c - m));
}

template <typename LT>
__device__ __forceinline__ float ld_logit(const LT* p);
template <>
__device__ __forceinline__ float ld_logit<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ld_logit<bf16_t>(const bf16_t* p) { return bf2f(*p); }

template <typename LT>
__device__ __forceinline__ void st_grad(LT* p, float v);
template <>
__device__ __forceinline__ void st_grad<float>(float* p, float v) { *p = v; }
template <>
__device__ __forceinline__ void st_grad<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

template <typename LT>
__global__ __launch_bounds__(CTC_THREADS) void ctc_fused_kernel(
    const LT* __restrict__ logits,      // [T, N, K]
    const int* __restrict__ lens,       // [N]
    const int* __restrict__ labels,     // [N, Lmax]
    const int* __restrict__ label_lens, // [N]
    float* __restrict__ loss,           // [N]
    LT* __restrict__ grad,              // [T, N, K]
    float* __restrict__ lp_ws,          // [N, T, KPAD]
    float* __restrict__ alpha_ws,       // [N, T, SPmax]
    int T, int N, int K, int Lmax, int SPmax, int blank, int zero_inf) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* arow = reinterpret_cast<float*>(smem);                 // [2][SPmax]
  int* lab = reinterpret_cast<int*>(arow + 2 * SPmax);          // [SPmax] class of state
  float* occ = reinterpret_cast<float*>(lab + SPmax);           // [2][KPAD]
  __shared__ float s_logp;

  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NWAVE = CTC_THREADS / 64;
  const int len = min(lens[b], T);
  const int L = label_lens[b];
  const int SP = 2 * L + 1;
  float* lp = lp_ws + (size_t)b * T * KPAD;
  float* al = alpha_ws + (size_t)b * T * SPmax;

  for (int s = tid; s < SP; s += CTC_THREADS) lab[s] = (s & 1) ? labels[(size_t)b * Lmax + (s >> 1)] : blank;
  if (tid < 2 * KPAD) occ[tid] = 0.f;

  // phase 0: log-softmax of each valid frame
  for (int t = wave; t < len; t += NWAVE) {
    const float x = (lane < K) ? ld_logit<LT>(logits + ((size_t)t * N + b) * K + lane) : NEG_INF;
    const float m = wave_max(x);
    const float e = (lane < K) ? __expf(x - m) : 0.f;
    const float sum = wave_sum(e);
    if (lane < KPAD) lp[(size_t)t * KPAD + lane] = (lane < K) ? (x - m - __logf(sum)) : NEG_INF;
  }
  // zero gradient past the utterance
  for (size_t i = (size_t)len * K + tid; i < (size_t)T * K; i += CTC_THREADS) {
    const size_t t = i / K, k = i % K;
    st_grad<LT>(grad + (t * N + b) * K + k, 0.f);
  }
  __syncthreads();

  if (len <= 0 || L > len) {   // nothing feasible (also covers empty frames)
    if (tid == 0) loss[b] = zero_inf ? 0.f : INFINITY;
    for (size_t i = tid; i < (size_t)len * K; i += CTC_THREADS) {
      const size_t t = i / K, k = i % K;
      st_grad<LT>(grad + (t * N + b) * K + k, 0.f);
    }
    return;
  }

  // phase 1: alpha
  for (int s = tid; s < SP; s += CTC_THREADS) {
    float v = NEG_INF;
    if (s == 0) v = lp[blank];
    else if (s == 1) v = lp[lab[1]];
    arow[s] = v;
    al[s] = v;
  }
  __syncthreads();
  for (int t = 1; t < len; ++t) {
    const float* prev = arow + ((t - 1) & 1) * SPmax;
    float* cur = arow + (t & 1) * SPmax;
    const float* lpt = lp + (size_t)t * KPAD;
    for (int s = tid; s < SP; s += CTC_THREADS) {
      const int c = lab[s];
      float a = prev[s];
      float b1 = (s >= 1) ? prev[s - 1] : NEG_INF;
      float b2 = (s >= 2 && c != blank && c != lab[s - 2]) ? prev[s - 2] : NEG_INF;
      const float v = lse3(a, b1, b2) + lpt[c];
      cur[s] = v;
      al[(size_t)t * SPmax + s] = v;
    }
    __syncthreads();
  }
  if (tid == 0) {
    const float* last = arow + ((len - 1) & 1) * SPmax;
    s_logp = lse2(last[SP - 1], SP >= 2 ? last[SP - 2] : NEG_INF);
  }
  __syncthreads();
  const float logp = s_logp;
  const bool infeasible = !(logp > NEG_INF);
  if (tid == 0) loss[b] = infeasible ? (zero_inf ? 0.f : INFINITY) : -logp;
  if (infeasible) {
    for (size_t i = tid; i < (size_t)len * K; i += CTC_THREADS) {
      const size_t t = i / K, k = i % K;
      st_grad<LT>(grad + (t * N + b) * K + k, 0.f);
    }
    return;
  }

  // phase 2: beta + gradient
  for (int t = len - 1; t >= 0; --t) {
    const float* nxt = arow + ((t + 1) & 1) * SPmax;
    float* cur = arow + (t & 1) * SPmax;
    const float* lpt = lp + (size_t)t * KPAD;
    float* oc = occ + (t & 1) * KPAD;
    for (int s = tid; s < SP; s += CTC_THREADS) {
      const int c = lab[s];
      float v;
      if (t == len - 1) {
        v = (s == SP - 1 || s == SP - 2) ? lpt[c] : NEG_INF;
      } else {
        const float a = nxt[s];
        const float b1 = (s + 1 < SP) ? nxt[s + 1] : NEG_INF;
        const float b2 = (s + 2 < SP && c != blank && c != lab[s + 2]) ? nxt[s + 2] : NEG_INF;
        v = lse3(a, b1, b2) + lpt[c];
      }
      cur[s] = v;
      const float ab = al[(size_t)t * SPmax + s] + v - lpt[c] - logp;
      if (ab > -80.f) atomicAdd(&oc[c], __expf(ab));
    }
    __syncthreads();
    if (tid < K) {
      const float g = __expf(lpt[tid]) - oc[tid];
      st_grad<LT>(grad + ((size_t)t * N + b) * K + tid, g);
      oc[tid] = 0.f;
    }
    // the next frame accumulates into the other occ buffer; its reset above is ordered
    // before that buffer's reuse by the barrier at the end of the next iteration
  }
}

}  // namespace

extern "C" {

size_t ds2_ctc_smem_bytes(int SPmax) { return (size_t)(2 * SPmax) * 4 + (size_t)SPmax * 4 + 2 * KPAD * 4; }

int ds2_ctc_fused(const void* logits, int logits_bf16, const int* lens, const int* labels,
                  const int* label_lens, float* loss, void* grad, float* lp_ws, float* alpha_ws,
                  int T, int N, int K, int Lmax, int blank, int zero_inf, hipStream_t st) {
  if (K > 64 || K > KPAD) return -20;
  const int SPmax = 2 * Lmax + 1;
  const size_t smem = ds2_ctc_smem_bytes(SPmax);
  if (smem > 160 * 1024) return -21;
  if (logits_bf16) {
    hipLaunchKernelGGL(ctc_fused_kernel<bf16_t>, dim3(N), dim3(CTC_THREADS), smem, st,
                       (const bf16_t*)logits, lens, labels, label_lens, loss, (bf16_t*)grad, lp_ws,
                       alpha_ws, T, N, K, Lmax, SPmax, blank, zero_inf);
  } else {
    hipLaunchKernelGGL(ctc_fused_kernel<float>, dim3(N), dim3(CTC_THREADS), smem, st,
                       (const float*)logits, lens, labels, label_lens, loss, (float*)grad, lp_ws,
                       alpha_ws, T, N, K, Lmax, SPmax, blank, zero_inf);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
