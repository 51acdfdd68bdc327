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
//                         alpha/beta rows are streamed (float4/2 stores, 64*SPL row stride)
//                         to ab_ws[2][N][T][64*SPL].
//   3. ctc_grad_kernel    fully parallel over frames (one wave per (t, b)): occupancy
//                         gamma_t(s) = alpha+beta-lp-logP, blank states summed with a wave
//                         reduction, label states with per-wave LDS atomics, then
//                         grad[t][k] = softmax_t(k) - occ_t(k). Frames past the length get 0.
// Infeasible utterances (logP = -inf) get loss 0 and zero gradient when zero_inf != 0.
//
// Training path with the FC head fused in (ds2_head_ctc; reference FC + CTC at
// src/deepSpeech_NCHW.py:188-198,225): the logits never reach memory.
//   0. fc_lsm_kernel      logits = h W_fc^T + b on MFMA (16 frames per wave, W_fc in LDS),
//                         log-softmax in registers, lp rows straight into the workspace
//   2. ctc_recur_kernel   as above
//   3. ctc_grad_lp_kernel gradient from lp (no logits re-read), written as a zero-padded
//                         [T*N][32] bf16 matrix: the operand of the FC backward GEMMs
//                         (dh = G W_fc, dW_fc = G^T h in csrc/gemm.hip)
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
// state costs 2 v_exp_f32 + 1 v_log_f32 (no ln<->log2 scaling, no branch). No all--inf
// select either: the max is clamped to -1e30, so three -inf inputs give exactly -1e30 (fp32
// ulp there ~7.6e22: adding log-probs keeps it at -1e30). The recursion carries -1e30 as its
// "log 0", the gradient kernels' ga > -80 test maps it to 0 like -inf, and a logP below
// -1e29 is returned as -inf (infeasible utterance).
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
__device__ __forceinline__ float lse3_rec(float a, float b, float c) {
  const float m = fmaxf(fmaxf(fmaxf(a, b), c), -1e30f);
  const float lo = fminf(fminf(a, b), c);
  const float mid = __builtin_amdgcn_fmed3f(a, b, c);
  return m + __builtin_amdgcn_logf(1.f + __builtin_amdgcn_exp2f(mid - m) + __builtin_amdgcn_exp2f(lo - m));
}
constexpr float LOG_ZERO_LIMIT = -1e29f;

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
  const int L = min(label_lens[b], Lmax);   // a label length past the padded width reads no other row
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
    // states past the lattice read the staged rows' padding column KPAD, which holds -inf:
    // their values stay -inf without a per-state select in the frame loop
    cls[j] = (s < SP) ? state_class(labels, b, Lmax, s, blank) : KPAD;
    DS2_DCHECK(cls[j] >= 0 && cls[j] <= KPAD);     // label ids index the 32-wide lp rows
    bool ok = false;
    if (s < SP && cls[j] != blank) {   // (s >= SP: cls = KPAD, no skip transition)
      if (!beta) ok = s >= 2 && cls[j] != state_class(labels, b, Lmax, s - 2, blank);
      else ok = s + 2 < SP && cls[j] != state_class(labels, b, Lmax, s + 2, blank);
    }
    skip |= (ok ? 1u : 0u) << j;
  }
  const float* lp = lp_ws + (size_t)b * T * KPAD;
  constexpr int SPS = 64 * SPL;                    // row stride: whole register tile, 16-B aligned
  float* out = ab_ws + ((size_t)beta * N + b) * (size_t)T * SPS;
  auto put_row = [&](int t, const float* v) {   // rows in natural-log units for the gradient kernel
    float* o = out + (size_t)t * SPS + s0;       // 4*SPL-B aligned: widest store that divides it
    if constexpr (SPL % 4 == 0) {
#pragma unroll
      for (int j = 0; j < SPL / 4; ++j)
        reinterpret_cast<float4*>(o)[j] = make_float4(v[4 * j] * LN2, v[4 * j + 1] * LN2, v[4 * j + 2] * LN2,
                                                      v[4 * j + 3] * LN2);
    } else if constexpr (SPL % 2 == 0) {
#pragma unroll
      for (int j = 0; j < SPL / 2; ++j)
        reinterpret_cast<float2*>(o)[j] = make_float2(v[2 * j] * LN2, v[2 * j + 1] * LN2);
    } else {
#pragma unroll
      for (int j = 0; j < SPL; ++j) o[j] = v[j] * LN2;
    }
  };
  // lp rows are staged through LDS in chunks of 64 frames (one 128-B row per lane), so
  // the per-frame gathers are LDS reads: a global load in the frame loop would make the
  // wave wait (vmcnt) behind its own streaming alpha/beta stores every frame.
  __shared__ float lps[64][KPAD + 1];
  lps[lane][KPAD] = NEG_INF;                       // never overwritten by stage()
  const int dt = beta ? -1 : 1;
  const int t0 = beta ? len - 1 : 0;
  // A NaN log-prob (a diverged model: the log-softmax turns a NaN logit into a whole NaN
  // frame) must reach the loss as NaN, not as an "infeasible" -inf that zero_infinity hides.
  // The recursion cannot carry it (lse3_rec's fmaxf / fminf drop NaN operands, so a NaN
  // frame decays to "log 0"), so the staged rows are tested instead: off the frame chain.
  bool nan = false;
  auto stage = [&](int c0) {   // frames c0 .. c0+63 (forward) or c0 .. c0-63 (backward)
    const int t = c0 + dt * lane;
    __builtin_amdgcn_wave_barrier();
    if (t >= 0 && t < len) {
      const float4* src = reinterpret_cast<const float4*>(lp + (size_t)t * KPAD);
#pragma unroll
      for (int q = 0; q < KPAD / 4; ++q) {
        const float4 v4 = src[q];
        nan = nan || (v4.x != v4.x) || (v4.y != v4.y) || (v4.z != v4.z) || (v4.w != v4.w);
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
      // previous lane's last two states: DPP wave_shr:1 (a VALU move, lane 0 keeps the
      // NEG_INF 'old' operand) instead of ds_bpermute shuffles, whose LDS round trip sat on
      // the frame recursion's dependency chain
      const float p1 = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(NEG_INF), __float_as_int(v[SPL - 1]),
                                                                  0x138, 0xf, 0xf, false));
      const float p2 = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(NEG_INF), __float_as_int(v[SPL - 2]),
                                                                  0x138, 0xf, 0xf, false));
#pragma unroll
      for (int j = 0; j < SPL; ++j) {
        const float a1 = (j >= 1) ? v[j - 1] : p1;
        const float a2 = (j >= 2) ? v[j - 2] : (j == 1 ? p1 : p2);
        nv[j] = lse3_rec(v[j], a1, ((skip >> j) & 1u) ? a2 : NEG_INF) + lcur[j];
      }
    } else {
      const float n1 = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(NEG_INF), __float_as_int(v[0]),
                                                                  0x130, 0xf, 0xf, false));   // wave_shl:1
      const float n2 = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(NEG_INF), __float_as_int(v[1]),
                                                                  0x130, 0xf, 0xf, false));
#pragma unroll
      for (int j = 0; j < SPL; ++j) {
        const float b1 = (j + 1 < SPL) ? v[j + 1] : n1;
        const float b2 = (j + 2 < SPL) ? v[j + 2] : (j + 1 < SPL ? n1 : n2);
        nv[j] = lse3_rec(v[j], b1, ((skip >> j) & 1u) ? b2 : NEG_INF) + lcur[j];
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
    const bool any_nan = __any(nan);          // a NaN frame anywhere in the utterance
    if (lane == 0) logp_out[b] = any_nan ? __builtin_nanf("") : (m < LOG_ZERO_LIMIT) ? NEG_INF : m + __logf(e);
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
  const int L = min(label_lens[b], Lmax);   // a label length past the padded width reads no other row
  const float logp = (len > 0 && L <= len) ? logp_in[b] : NEG_INF;
  const bool feasible = !(logp == NEG_INF);        // NaN stays "feasible": it must reach the loss
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

// ---------------------------------------------------------------- 0. FC + log-softmax
// One wave per 16 frames (rows m = t*N + b of the time-major h). MFMA operands swapped
// (D = W.h^T) so lane l ends with row m = l&15 and classes 4(l>>4)+j (+16): a row's 32
// values sit in 4 lanes (l, l^16, l^32, l^48) and the row max / sum are two shuffles.
constexpr int FC_WAVES = 4;
template <typename OT>
__global__ __launch_bounds__(FC_WAVES * 64) void fc_lsm_kernel(const bf16_t* __restrict__ h, const bf16_t* __restrict__ W,
                                                             const bf16_t* __restrict__ bias,
                                                             const int* __restrict__ lens, float* __restrict__ lp_ws,
                                                             OT* __restrict__ logits, int T, int N, int H, int K) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int pitch = H * 2 + 16;                     // padded rows: 16 consecutive rows -> 16 distinct slots
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // stage W_fc (K <= 32 rows, zero rows past K) as [32][H] bf16
  const int cpr = H / 8;
  for (int q = tid; q < 32 * cpr; q += FC_WAVES * 64) {
    const int r = q / cpr, c = q - r * cpr;
    i32x4 v = {0, 0, 0, 0};
    if (r < K) v = *reinterpret_cast<const i32x4*>(W + (size_t)r * H + 8 * c);
    *reinterpret_cast<i32x4*>(smem + r * pitch + 16 * c) = v;
  }
  __syncthreads();
  const int M = T * N;
  const int blk = blockIdx.x * FC_WAVES + wave;
  if (blk * 16 >= M) return;
  const int mrow = blk * 16 + (lane & 15);
  const bf16_t* hr = h + (size_t)min(mrow, M - 1) * H + 8 * (lane >> 4);
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const unsigned char* w0 = smem + (lane & 15) * pitch + 16 * (lane >> 4);
  const unsigned char* w1 = w0 + 16 * pitch;
  const int KS = H / 32;
  constexpr int CH = 5;                              // A fragments in flight per lane
  for (int k0 = 0; k0 < KS; k0 += CH) {
    bf16x8 af[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) af[i] = *reinterpret_cast<const bf16x8*>(hr + 32 * min(k0 + i, KS - 1));
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (k0 + i < KS) {
        const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(w0 + 64 * (k0 + i));
        const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(w1 + 64 * (k0 + i));
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0, af[i], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1, af[i], acc1, 0, 0, 0);
      }
    }
  }
  const int g = lane >> 4;
  float x[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n0 = 4 * g + j, n1 = 16 + 4 * g + j;
    x[j] = n0 < K ? acc0[j] + bf2f(bias[n0]) : NEG_INF;
    x[4 + j] = n1 < K ? acc1[j] + bf2f(bias[n1]) : NEG_INF;
  }
  float m = x[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) m = fmaxf(m, x[j]);
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float e = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) e += __expf(x[j] - m);
  e += __shfl_xor(e, 16, 64);
  e += __shfl_xor(e, 32, 64);
  const float lz = m + __logf(e);
  if (mrow < M) {
    const int t = mrow / N, b = mrow - (mrow / N) * N;
    if (lp_ws && t < lens[b]) {
      float4* o = reinterpret_cast<float4*>(lp_ws + ((size_t)b * T + t) * KPAD);
      o[g] = make_float4(x[0] - lz, x[1] - lz, x[2] - lz, x[3] - lz);
      o[4 + g] = make_float4(x[4] - lz, x[5] - lz, x[6] - lz, x[7] - lz);
    }
    if (logits) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (4 * g + j < K) st_grad<OT>(logits + (size_t)mrow * K + 4 * g + j, x[j]);
        if (16 + 4 * g + j < K) st_grad<OT>(logits + (size_t)mrow * K + 16 + 4 * g + j, x[4 + j]);
      }
    }
  }
}

// ---------------------------------------------------------------- 3'. gradient from lp
// As ctc_grad_kernel, reading lp_t(k) from the workspace; G[t*N+b][0..31] = p - occ (bf16),
// zero past the length / for infeasible utterances / in the padding classes.
__global__ __launch_bounds__(256) void ctc_grad_lp_kernel(const int* __restrict__ lens, const int* __restrict__ labels,
                                                        const int* __restrict__ label_lens,
                                                        const float* __restrict__ lp_ws,
                                                        const float* __restrict__ ab_ws,
                                                        const float* __restrict__ logp_in, float* __restrict__ loss,
                                                        bf16_t* __restrict__ G, int T, int N, int K, int Lmax, int SPS,
                                                        int blank, int zero_inf, float* __restrict__ mean_out,
                                                        int* __restrict__ counter, int* __restrict__ first_bad) {
  __shared__ float occ_s[4][KPAD];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (mean_out != nullptr && blockIdx.x == 0 && wv == 0) {
    // the batch-mean loss (every per-utterance loss is final: ctc_recur wrote logp) and the
    // per-step divergence watch (stats.hip nonfinite_watch_kernel) in this launch instead of a
    // reduction kernel and a 1-thread kernel behind it on the step's critical path
    float s = 0.f;
    for (int b0 = 0; b0 < N; b0 += 64) {
      const int bb = b0 + lane;
      float l = 0.f;
      if (bb < N) {
        const int lb = min(lens[bb], T), Lb = min(label_lens[bb], Lmax);
        const float lp = (lb > 0 && Lb <= lb) ? logp_in[bb] : NEG_INF;
        l = !(lp == NEG_INF) ? -lp : (zero_inf ? 0.f : INFINITY);
      }
      s += wave_sum(l);
    }
    if (lane == 0) {
      const float m = s / (float)N;
      *mean_out = m;
      if (counter != nullptr) {
        const int st = counter[0];
        if (!(fabsf(m) <= 3.402823466e38f) && first_bad[0] < 0) first_bad[0] = st;   // NaN or +-inf
        counter[0] = st + 1;
      }
    }
  }
  const int w = blockIdx.x * 4 + wv;
  if (w >= T * N) return;
  const int t = w / N, b = w % N;
  const int len = min(lens[b], T);
  const int L = min(label_lens[b], Lmax);   // a label length past the padded width reads no other row
  const float logp = (len > 0 && L <= len) ? logp_in[b] : NEG_INF;
  const bool feasible = !(logp == NEG_INF);        // NaN stays "feasible": it must reach the loss
  if (t == 0 && lane == 0) loss[b] = feasible ? -logp : (zero_inf ? 0.f : INFINITY);
  bf16_t* g = G + (size_t)w * KPAD;
  if (t >= len || !feasible) {
    if (lane < KPAD) g[lane] = 0;
    return;
  }
  float* occ = occ_s[wv];
  if (lane < KPAD) occ[lane] = 0.f;
  const float lpk = (lane < K) ? lp_ws[((size_t)b * T + t) * KPAD + lane] : NEG_INF;
  const int SP = 2 * L + 1;
  const float* A = ab_ws + ((size_t)b * T + t) * SPS;
  const float* B = ab_ws + ((size_t)(N + b) * T + t) * SPS;
  float blank_acc = 0.f;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  for (int base = 0; base < SP; base += 64) {
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
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  if (lane < KPAD) {
    float v = 0.f;
    if (lane < K) {
      const float p = __expf(lpk);
      const float o = (lane == blank) ? blank_acc : occ[lane];
      v = p - o;
    }
    g[lane] = f2bf(v);
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

// States per lane: the smallest instantiation that holds the longest label. The frame
// recursion is latency/issue bound on ONE wave (2 v_exp + 1 v_log per state), so every
// unused state slot costs time: 10-s utterances (~150 labels, 301 states) run SPL 5, not 8.
static int ctc_spl(int SPmax) {
  const int need = (SPmax + 63) / 64;
  // (the round-1 power-of-two set {4, 8, 16, 32} measured slower: profiles/r2_s4_ctc_spl.md)
  for (int k : {4, 5, 6, 8, 12, 16, 32}) if (k >= need) return k;
  return -1;
}

static void launch_recur_spl(int spl, const int* lens, const int* labels, const int* label_lens, const float* lp_ws,
                             float* ab_ws, float* logp, int T, int N, int Lmax, int SPmax, int blank, hipStream_t st) {
  switch (spl) {
    case 4: launch_recur<4>(lens, labels, label_lens, lp_ws, ab_ws, logp, T, N, Lmax, SPmax, blank, st); break;
    case 5: launch_recur<5>(lens, labels, label_lens, lp_ws, ab_ws, logp, T, N, Lmax, SPmax, blank, st); break;
    case 6: launch_recur<6>(lens, labels, label_lens, lp_ws, ab_ws, logp, T, N, Lmax, SPmax, blank, st); break;
    case 8: launch_recur<8>(lens, labels, label_lens, lp_ws, ab_ws, logp, T, N, Lmax, SPmax, blank, st); break;
    case 12: launch_recur<12>(lens, labels, label_lens, lp_ws, ab_ws, logp, T, N, Lmax, SPmax, blank, st); break;
    case 16: launch_recur<16>(lens, labels, label_lens, lp_ws, ab_ws, logp, T, N, Lmax, SPmax, blank, st); break;
    default: launch_recur<32>(lens, labels, label_lens, lp_ws, ab_ws, logp, T, N, Lmax, SPmax, blank, st); break;
  }
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
  launch_recur_spl(spl, lens, labels, label_lens, lp_ws, ab_ws, logp, T, N, Lmax, SPmax, blank, st);
  if (logits_bf16)
    hipLaunchKernelGGL(ctc_grad_kernel<bf16_t>, g4, dim3(256), 0, st, (const bf16_t*)logits, lens, labels, label_lens,
                       ab_ws, logp, loss, (bf16_t*)grad, T, N, K, Lmax, SPS, blank, zero_inf);
  else
    hipLaunchKernelGGL(ctc_grad_kernel<float>, g4, dim3(256), 0, st, (const float*)logits, lens, labels, label_lens,
                       ab_ws, logp, loss, (float*)grad, T, N, K, Lmax, SPS, blank, zero_inf);
  return (int)hipGetLastError();
}

// W_fc staged in LDS: > 64 KB for H > 1000 needs the opt-in (160 KB per CU on gfx950)
static int fc_attr(int lds) {
  static int done = 0;
  if (lds > 64 * 1024 && !done) {
    hipError_t e = hipFuncSetAttribute((const void*)fc_lsm_kernel<float>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)fc_lsm_kernel<bf16_t>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    if (e != hipSuccess) return (int)e;
    done = 1;
  }
  return lds > 160 * 1024 ? (int)hipErrorInvalidValue : 0;
}

// FC head + CTC for training: h [T*N][H] bf16 (time-major rows), W [K][H] bf16, bias [K] bf16.
// Outputs loss [N] and G [T*N][32] bf16 (dloss_b/dlogits, zero-padded). ws as ds2_ctc_ws_floats.
int ds2_head_ctc(const void* h, const void* W, const void* bias, const int* lens, const int* labels,
                 const int* label_lens, float* loss, void* G, float* ws, int T, int N, int H, int K, int Lmax,
                 int blank, int zero_inf, float* mean, int* counter, int* first_bad, hipStream_t st) {
  if (K > KPAD || H % 32 != 0) return -20;
  const int SPmax = 2 * Lmax + 1;
  if (SPmax > 64 * 32) return -21;
  const int spl = ctc_spl(SPmax);
  const int SPS = 64 * spl;
  float* lp_ws = ws;
  float* ab_ws = lp_ws + (size_t)N * T * KPAD;
  float* logp = ab_ws + 2 * (size_t)N * T * SPS;
  const int M = T * N;
  const int lds = 32 * (H * 2 + 16);
  if (const int e = fc_attr(lds)) return e;
  hipLaunchKernelGGL(fc_lsm_kernel<float>, dim3((M + 16 * FC_WAVES - 1) / (16 * FC_WAVES)), dim3(FC_WAVES * 64), lds,
                     st, (const bf16_t*)h, (const bf16_t*)W, (const bf16_t*)bias, lens, lp_ws, (float*)nullptr, T, N,
                     H, K);
  launch_recur_spl(spl, lens, labels, label_lens, lp_ws, ab_ws, logp, T, N, Lmax, SPmax, blank, st);
  hipLaunchKernelGGL(ctc_grad_lp_kernel, dim3((M + 3) / 4), dim3(256), 0, st, lens, labels, label_lens, lp_ws, ab_ws,
                     logp, loss, (bf16_t*)G, T, N, K, Lmax, SPS, blank, zero_inf, mean, counter, first_bad);
  return (int)hipGetLastError();
}

// FC head alone (inference): logits [T*N][K] (fp32 or bf16) = h W^T + b.
int ds2_fc_logits(const void* h, const void* W, const void* bias, void* logits, int out_bf16, int M, int H, int K,
                  hipStream_t st) {
  if (K > KPAD || H % 32 != 0) return -20;
  const int lds = 32 * (H * 2 + 16);
  if (const int e = fc_attr(lds)) return e;
  const dim3 grid((M + 16 * FC_WAVES - 1) / (16 * FC_WAVES));
  if (out_bf16)
    hipLaunchKernelGGL(fc_lsm_kernel<bf16_t>, grid, dim3(FC_WAVES * 64), lds, st, (const bf16_t*)h, (const bf16_t*)W,
                       (const bf16_t*)bias, (const int*)nullptr, (float*)nullptr, (bf16_t*)logits, M, 1, H, K);
  else
    hipLaunchKernelGGL(fc_lsm_kernel<float>, grid, dim3(FC_WAVES * 64), lds, st, (const bf16_t*)h, (const bf16_t*)W,
                       (const bf16_t*)bias, (const int*)nullptr, (float*)nullptr, (float*)logits, M, 1, H, K);
  return (int)hipGetLastError();
}

}  // extern "C"
