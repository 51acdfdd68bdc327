// Greedy CTC decoding on the GPU (gfx950).
//
// Reference: tf.nn.log_softmax + tf.nn.ctc_greedy_decoder(merge_repeated=True) of
// src/deepSpeech_test.py:212-215: per frame take the most likely class, merge runs of the
// same class, drop the blank. Log-softmax does not change the argmax, so the kernel reads
// the logits directly. One workgroup per utterance; the frames are processed in blocks of
// 256 (one per thread): argmax per frame, "emit" flag = (class != blank && class !=
// previous frame's class), block prefix sum of the flags (wave ballots + LDS) gives each
// emitted label its output slot, and the block carries its last class and count into the
// next block. The per-frame score (max log-prob) is summed too, so the caller gets the
// greedy path log-probability (TF's neg_sum_logits, negated) without a second pass.
#include "common.h"

using namespace ds2;

namespace {

constexpr int DT = 256;

template <typename T>
__device__ __forceinline__ float ld(const T* p);
template <>
__device__ __forceinline__ float ld<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p) { return bf2f(*p); }

template <typename T>
__global__ __launch_bounds__(DT) void ctc_greedy_kernel(const T* __restrict__ logits, const int* __restrict__ lens,
                                                        int Tn, int N, int K, int blank, int* __restrict__ labels,
                                                        int* __restrict__ counts, float* __restrict__ score) {
  __shared__ int wsum[DT / 64];
  __shared__ int cls_sh[DT];
  __shared__ float sc_sh[DT / 64];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int L = min(lens[n], Tn);
  int prev_last = -1;     // class of the frame before this block
  int base = 0;           // labels emitted so far
  float total = 0.f;
  for (int t0 = 0; t0 < L; t0 += DT) {
    const int t = t0 + tid;
    int c = -1;
    float lp = 0.f;
    if (t < L) {
      const T* row = logits + ((size_t)t * N + n) * K;
      float mx = ld<T>(row);
      c = 0;
      for (int k = 1; k < K; ++k) {
        const float v = ld<T>(row + k);
        if (v > mx) { mx = v; c = k; }
      }
      float s = 0.f;
      for (int k = 0; k < K; ++k) s += __expf(ld<T>(row + k) - mx);
      lp = -__logf(s);                         // log-softmax of the argmax class
    }
    cls_sh[tid] = c;
    __syncthreads();
    const int pc = tid == 0 ? prev_last : cls_sh[tid - 1];
    const bool emit = t < L && c != blank && c != pc;
    const unsigned long long m = __ballot(emit);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    float ws = wave_sum(lp);
    if (lane == 0) { wsum[w] = __popcll(m); sc_sh[w] = ws; }
    __syncthreads();
    int off = base;
    for (int i = 0; i < w; ++i) off += wsum[i];
    if (emit) labels[(size_t)n * Tn + off + before] = c;
    int blk = 0;
    float bs = 0.f;
    for (int i = 0; i < DT / 64; ++i) { blk += wsum[i]; bs += sc_sh[i]; }
    base += blk;
    total += bs;
    prev_last = cls_sh[min(DT - 1, L - 1 - t0)];
    __syncthreads();
  }
  if (tid == 0) {
    counts[n] = base;
    if (score) score[n] = total;
  }
}

}  // namespace

extern "C" int ds2_ctc_greedy(const void* logits, int bf16, const int* lens, int T, int N, int K, int blank,
                              int* labels, int* counts, float* score, hipStream_t st) {
  if (bf16)
    hipLaunchKernelGGL(ctc_greedy_kernel<bf16_t>, dim3(N), dim3(DT), 0, st, (const bf16_t*)logits, lens, T, N, K,
                       blank, labels, counts, score);
  else
    hipLaunchKernelGGL(ctc_greedy_kernel<float>, dim3(N), dim3(DT), 0, st, (const float*)logits, lens, T, N, K,
                       blank, labels, counts, score);
  return (int)hipGetLastError();
}
