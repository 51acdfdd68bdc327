// Fused CTC loss + gradient for gfx950 (reference: tf.nn.ctc_loss at
// src/deepSpeech_NCHW.py:225, blank = last class, time-major logits).
//
// Three launches, each shaped for what it does:
//   1. ctc_lsm_kernel     log-softmax of every valid frame -> lp[N][T][32]. Fully parallel
//                         (one wave per (t, b) frame, 64-lane shuffle reductions).
//   2. ctc_recur_kernel   the two serial recursions, alpha (blockIdx.y = 0) and beta
//                         (blockIdx.y = 1) of every utterance CONCURRENTLY, ONE WAVE each:
//                         lane l owns lattice states [l*SPL, l*SPL+SPL) in registers, the
//                         s-1/s-2 (s+1/s+2) neighbours crossing a lane boundary come from a
//                         cross-lane shuffle, so a frame costs no barrier and no LDS round
//                         trip; the next frame's lp row is prefetched one frame ahead.
//                         alpha/beta rows are streamed (float4 stores, 64*SPL row stride)
//                         to ab_ws[2][N][T][64*SPL].
//   3. ctc_grad_kernel    fully parallel over frames (one wave per (t, b)): occupancy
//                         gamma_t(s) = alpha+beta-lp-logP, blank states summed with a wave
//                         reduction, label states with per-wave LDS atomics, then
//                         grad[t][k] = softmax_t(k) - occ_t(k). Frames past the length get 0.
// Infeasible utterances (logP = -inf) get loss 0 and zero gradient when zero_inf != 0.
#include "common.h"

using namespace ds2;

namespace {

constexpr int KPAD = 32;
constexpr float NEG_INF = -INFINITY;

__device__ __forceinline__ float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == NEG_INF) return NEG_INF;
  return m + __logf(__expf(a - m) + __expf(b - m));
}

// log2-domain lse of three values with ONE of the three exponentials known to be 2^0:
// m = max, the other two are the median and the minimum (v_max3 / v_med3 / v_min3), so a
// state costs 2 v_exp_f32 + 1 v_log_f32 (no ln<->log2 scaling, no branch).
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
__device__ __forceinline__ float lse3_2(float a, float b, float c) {
  const float m = fmaxf(fmaxf(a, b), c);
  const float lo = fminf(fminf(a, b), c);
  const float mid = __builtin_amdgcn_fmed3f(a, b, c);
  const float mc = fmaxf(m, -1e30f);                   // all -inf: keep the differences finite
  const float r = mc + __builtin_amdgcn_logf(1.f + __builtin_amdgcn_exp2f(mid - mc) +
                                             __builtin_amdgcn_exp2f(lo - mc));
  return (m == NEG_INF) ? NEG_INF : r;
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

__device__ __forceinline__ int state_class(const int* labels, int b, int Lmax, int s, int blank) {
  return (s & 1) ? labels[(size_t)b * Lmax + (s >> 1)] : blank;
}

// ---------------------------------------------------------------- 1. log-softmax
template <typename LT>
__global__ __launch_bounds__(256) void ctc_lsm_kernel(const LT* __restrict__ logits, const int* __restrict__ lens,
                                                      float* __restrict__ lp_ws, int T, int N, int K) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (w >= T * N) return;
  const int t = w / N, b = w % N;
  if (t >= lens[b]) return;
  const float x = (lane < K) ? ld_logit<LT>(logits + (size_t)w * K + lane) : NEG_INF;
  const float m = wave_max(x);
  const float sum = wave_sum((lane < K) ? __expf(x - m) : 0.f);
  if (lane < KPAD) lp_ws[((size_t)b * T + t) * KPAD + lane] = (lane < K) ? (x - m - __logf(sum)) : NEG_INF;
}

// ---------------------------------------------------------------- 2. alpha / beta
template <int SPL>
__global__ __launch_bounds__(64) void ctc_recur_kernel(const int* __restrict__ lens, const int* __restrict__ labels,
                                                       const int* __restrict__ label_lens,
                                                       const float* __restrict__ lp_ws, float* __restrict__ ab_ws,
                                                       float* __restrict__ logp_out, int T, int N, int Lmax,
                                                       int SPmax, int blank) {
  const int b = blockIdx.x, beta = blockIdx.y, lane = threadIdx.x;
  const int len = min(lens[b], T);
  const int L = label_lens[b];
  const int SP = 2 * L + 1;
  if (len <= 0 || L > len) {
    if (!beta && lane == 0) logp_out[b] = NEG_INF;
    return;
  }
  const int s0 = lane * SPL;
  int cls[SPL];
  unsigned skip = 0;   // bit j: the s-2 (alpha) / s+2 (beta) transition into/out of state s0+j exists
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    const int s = s0 + j;
    cls[j] = (s < SP) ? state_class(labels, b, Lmax, s, blank) : blank;
    DS2_DCHECK(cls[j] >= 0 && cls[j] < KPAD);      // label ids index the 32-wide lp rows
    bool ok = false;
    if (s < SP && cls[j] != blank) {
      if (!beta) ok = s >= 2 && cls[j] != state_class(labels, b, Lmax, s - 2, blank);
      else ok = s + 2 < SP && cls[j] != state_class(labels, b, Lmax, s + 2, blank);
    }
    skip |= (ok ? 1u : 0u) << j;
  }
  const float* lp = lp_ws + (size_t)b * T * KPAD;
  constexpr int SPS = 64 * SPL;                    // row stride: whole register tile, 16-B aligned
  float* out = ab_ws + ((size_t)beta * N + b) * (size_t)T * SPS;
  auto put_row = [&](int t, const float* v) {
    float4* o = reinterpret_cast<float4*>(out + (size_t)t * SPS + s0);
#pragma unroll
    for (int j = 0; j < SPL / 4; ++j)   // rows in natural-log units for the gradient kernel
      o[j] = make_float4(v[4 * j] * LN2, v[4 * j + 1] * LN2, v[4 * j + 2] * LN2, v[4 * j + 3] * LN2);
  };
  // lp rows are staged through LDS in chunks of 64 frames (one 128-B row per lane), so
  // the per-frame gathers are LDS reads: a global load in the frame loop would make the
  // wave wait (vmcnt) behind its own streaming alpha/beta stores every frame.
  __shared__ float lps[64][KPAD + 1];
  const int dt = beta ? -1 : 1;
  const int t0 = beta ? len - 1 : 0;
  auto stage = [&](int c0) {   // frames c0 .. c0+63 (forward) or c0 .. c0-63 (backward)
    const int t = c0 + dt * lane;
    __builtin_amdgcn_wave_barrier();
    if (t >= 0 && t < len) {
      const float4* src = reinterpret_cast<const float4*>(lp + (size_t)t * KPAD);
#pragma unroll
      for (int q = 0; q < KPAD / 4; ++q) {
        const float4 v4 = src[q];
        lps[lane][4 * q + 0] = v4.x * LOG2E; lps[lane][4 * q + 1] = v4.y * LOG2E;   // log2 units
        lps[lane][4 * q + 2] = v4.z * LOG2E; lps[lane][4 * q + 3] = v4.w * LOG2E;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
  };

  float v[SPL];
  stage(t0);
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    const int s = s0 + j;
    const float l = lps[0][cls[j]];
    if (!beta) v[j] = (s == 0 || s == 1) && s < SP ? l : NEG_INF;
    else v[j] = (s == SP - 1 || s == SP - 2) ? l : NEG_INF;
  }
  put_row(t0, v);

  for (int step = 1; step < len; ++step) {
    const int t = t0 + dt * step;
    if ((step & 63) == 0) stage(t);
    float lcur[SPL];
#pragma unroll
    for (int j = 0; j < SPL; ++j) lcur[j] = lps[step & 63][cls[j]];
    float nv[SPL];
    if (!beta) {
      // neighbours s-1, s-2 of this lane's first two states live in the previous lane
      float p1 = __shfl_up(v[SPL - 1], 1, 64);
      float p2 = __shfl_up(v[SPL - 2], 1, 64);
      if (lane == 0) { p1 = NEG_INF; p2 = NEG_INF; }
#pragma unroll
      for (int j = 0; j < SPL; ++j) {
        const float a1 = (j >= 1) ? v[j - 1] : p1;
        const float a2 = (j >= 2) ? v[j - 2] : (j == 1 ? p1 : p2);
        const float r = lse3_2(v[j], a1, ((skip >> j) & 1u) ? a2 : NEG_INF);
        nv[j] = (s0 + j < SP) ? r + lcur[j] : NEG_INF;
      }
    } else {
      float n1 = __shfl_down(v[0], 1, 64);
      float n2 = __shfl_down(v[1], 1, 64);
      if (lane == 63) { n1 = NEG_INF; n2 = NEG_INF; }
#pragma unroll
      for (int j = 0; j < SPL; ++j) {
        const float b1 = (j + 1 < SPL) ? v[j + 1] : n1;
        const float b2 = (j + 2 < SPL) ? v[j + 2] : (j + 1 < SPL ? n1 : n2);
        const float r = lse3_2(v[j], b1, ((skip >> j) & 1u) ? b2 : NEG_INF);
        nv[j] = (s0 + j < SP) ? r + lcur[j] : NEG_INF;
      }
    }
#pragma unroll
    for (int j = 0; j < SPL; ++j) v[j] = nv[j];
    put_row(t, v);
  }
  if (!beta) {
    // logP = lse(alpha_{len-1}(SP-1), alpha_{len-1}(SP-2))
    float mine = NEG_INF;
#pragma unroll
    for (int j = 0; j < SPL; ++j)
      if (s0 + j == SP - 1 || s0 + j == SP - 2) mine = lse2(mine, v[j] * LN2);
    // at most two lanes hold a term: combine with a max-shifted wave reduction
    const float m = wave_max(mine);
    float e = (m == NEG_INF) ? 0.f : __expf(mine - m);
    e = wave_sum(e);
    if (lane == 0) logp_out[b] = (m == NEG_INF) ? NEG_INF : m + __logf(e);
  }
}

// ---------------------------------------------------------------- 3. gradient
template <typename LT>
__global__ __launch_bounds__(256) void ctc_grad_kernel(const LT* __restrict__ logits, const int* __restrict__ lens,
                                                       const int* __restrict__ labels,
                                                       const int* __restrict__ label_lens,
                                                       const float* __restrict__ ab_ws,
                                                       const float* __restrict__ logp_in, float* __restrict__ loss,
                                                       LT* __restrict__ grad, int T, int N, int K, int Lmax, int SPS,
                                                       int blank, int zero_inf) {
  __shared__ float occ_s[4][KPAD];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + wv;
  if (w >= T * N) return;
  const int t = w / N, b = w % N;
  const int len = min(lens[b], T);
  const int L = label_lens[b];
  const float logp = (len > 0 && L <= len) ? logp_in[b] : NEG_INF;
  const bool feasible = logp > NEG_INF;
  if (t == 0 && lane == 0) loss[b] = feasible ? -logp : (zero_inf ? 0.f : INFINITY);
  LT* g = grad + (size_t)w * K;
  if (t >= len || !feasible) {
    if (lane < K) st_grad<LT>(g + lane, 0.f);
    return;
  }
  float* occ = occ_s[wv];
  if (lane < KPAD) occ[lane] = 0.f;
  const float x = (lane < K) ? ld_logit<LT>(logits + (size_t)w * K + lane) : NEG_INF;
  const float m = wave_max(x);
  const float sum = wave_sum((lane < K) ? __expf(x - m) : 0.f);
  const float lpk = (lane < K) ? (x - m - __logf(sum)) : NEG_INF;    // lane k holds lp_t(k)
  const int SP = 2 * L + 1;
  const float* A = ab_ws + ((size_t)b * T + t) * SPS;
  const float* B = ab_ws + ((size_t)(N + b) * T + t) * SPS;
  float blank_acc = 0.f;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  for (int base = 0; base < SP; base += 64) {       // wave-uniform trip count (shuffles below)
    const int s = base + lane;
    const bool in = s < SP;
    const int c = in ? state_class(labels, b, Lmax, s, blank) : blank;
    const float lc = __shfl(lpk, c, 64);
    float e = 0.f;
    if (in) {
      const float ga = A[s] + B[s] - lc - logp;
      e = (ga > -80.f) ? __expf(ga) : 0.f;
    }
    if (in && c != blank) atomicAdd(&occ[c], e);
    else blank_acc += e;
  }
  blank_acc = wave_sum(blank_acc);
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   // this wave's LDS atomics have landed
  if (lane < K) {
    const float p = __expf(lpk);
    const float o = (lane == blank) ? blank_acc : occ[lane];
    st_grad<LT>(g + lane, p - o);
  }
}

template <int SPL>
static void launch_recur(const int* lens, const int* labels, const int* label_lens, const float* lp_ws, float* ab_ws,
                         float* logp, int T, int N, int Lmax, int SPmax, int blank, hipStream_t st) {
  hipLaunchKernelGGL(ctc_recur_kernel<SPL>, dim3(N, 2), dim3(64), 0, st, lens, labels, label_lens, lp_ws, ab_ws, logp,
                     T, N, Lmax, SPmax, blank);
}

}  // namespace

extern "C" {

static int ctc_spl(int SPmax) {
  const int need = (SPmax + 63) / 64;
  for (int k : {4, 8, 16, 32}) if (k >= need) return k;
  return -1;
}

// workspace floats: lp [N][T][32] + alpha/beta [2][N][T][64*SPL] + logP [N]
long long ds2_ctc_ws_floats(int T, int N, int Lmax) {
  const int spl = ctc_spl(2 * Lmax + 1);
  const long long SPS = 64LL * (spl > 0 ? spl : 32);
  return (long long)N * T * KPAD + 2LL * N * T * SPS + N;
}

int ds2_ctc_fused(const void* logits, int logits_bf16, const int* lens, const int* labels,
                  const int* label_lens, float* loss, void* grad, float* ws, int T, int N, int K, int Lmax, int blank,
                  int zero_inf, hipStream_t st) {
  if (K > 64 || K > KPAD) return -20;
  const int SPmax = 2 * Lmax + 1;
  if (SPmax > 64 * 32) return -21;    // > 1023 labels per utterance
  const int spl = ctc_spl(SPmax);
  const int SPS = 64 * spl;
  float* lp_ws = ws;
  float* ab_ws = lp_ws + (size_t)N * T * KPAD;
  float* logp = ab_ws + 2 * (size_t)N * T * SPS;
  const int nw = T * N;
  const dim3 g4((nw + 3) / 4);
  if (logits_bf16)
    hipLaunchKernelGGL(ctc_lsm_kernel<bf16_t>, g4, dim3(256), 0, st, (const bf16_t*)logits, lens, lp_ws, T, N, K);
  else
    hipLaunchKernelGGL(ctc_lsm_kernel<float>, g4, dim3(256), 0, st, (const float*)logits, lens, lp_ws, T, N, K);
  if (spl == 4) launch_recur<4>(lens, labels, label_lens, lp_ws, ab_ws, logp, T, N, Lmax, SPmax, blank, st);
  else if (spl == 8) launch_recur<8>(lens, labels, label_lens, lp_ws, ab_ws, logp, T, N, Lmax, SPmax, blank, st);
  else if (spl == 16) launch_recur<16>(lens, labels, label_lens, lp_ws, ab_ws, logp, T, N, Lmax, SPmax, blank, st);
  else launch_recur<32>(lens, labels, label_lens, lp_ws, ab_ws, logp, T, N, Lmax, SPmax, blank, st);
  if (logits_bf16)
    hipLaunchKernelGGL(ctc_grad_kernel<bf16_t>, g4, dim3(256), 0, st, (const bf16_t*)logits, lens, labels, label_lens,
                       ab_ws, logp, loss, (bf16_t*)grad, T, N, K, Lmax, SPS, blank, zero_inf);
  else
    hipLaunchKernelGGL(ctc_grad_kernel<float>, g4, dim3(256), 0, st, (const float*)logits, lens, labels, label_lens,
                       ab_ws, logp, loss, (float*)grad, T, N, K, Lmax, SPS, blank, zero_inf);
  return (int)hipGetLastError();
}

}  // extern "C"
