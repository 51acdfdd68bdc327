// One launch for the small per-launch buffer initialisations of the persistent recurrence
// kernels (exchange sentinels, census words, error word, initial state slot, bias-gradient
// partials): up to 8 (pointer, bytes, 32-bit pattern) regions filled by one grid instead of
// one torch fill kernel (~5 us of launch + tail each on the critical path) per region.
#include "common.h"

using namespace ds2;

namespace {

constexpr int MF_MAX = 8;

struct MultiFill {
  unsigned* ptr[MF_MAX];
  unsigned long long words[MF_MAX];   // region sizes in 32-bit words
  unsigned pattern[MF_MAX];
  int n;
};

__global__ __launch_bounds__(256) void multi_fill_kernel(MultiFill f) {
  const unsigned long long stride = (unsigned long long)gridDim.x * 256;
  for (int r = 0; r < f.n; ++r) {
    unsigned* p = f.ptr[r];
    const unsigned v = f.pattern[r];
    const unsigned long long nw = f.words[r];
    const unsigned long long n4 = ((reinterpret_cast<uintptr_t>(p) & 15) == 0) ? nw / 4 : 0;
    const i32x4 v4 = {(int)v, (int)v, (int)v, (int)v};
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride)
      reinterpret_cast<i32x4*>(p)[i] = v4;
    for (unsigned long long i = n4 * 4 + (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < nw; i += stride)
      p[i] = v;
  }
}

thread_local hipEvent_t g_stop_event = nullptr;

}  // namespace

extern "C" void ds2_arm_stop_event(hipEvent_t e) { g_stop_event = e; }
extern "C" hipEvent_t ds2_take_stop_event() {
  hipEvent_t e = g_stop_event;
  g_stop_event = nullptr;
  return e;
}

// ---------------------------------------------------------------------------------------
// Residency gate: one wave spins (bounded) until a persistent recurrence launch's LAST
// workgroup has published its census word (csrc/rnn_xcd.hip group_census; pre-filled
// 0xFFFFFFFF). Workgroups are dispatched in order, so the whole grid then holds its CUs, and
// the work queued behind this gate on another stream (the weight-gradient GEMMs beside a
// BPTT, the carried optimizer chunks beside a forward recurrence) lands only on the CUs the
// recurrence left idle instead of racing it for them at dispatch. A pure scheduling hint: on a
// timeout (a launch that never came, e.g. a different plan than expected) the wave just exits.
namespace {
__global__ __launch_bounds__(64) void wait_resident_kernel(const unsigned* word, long long timeout) {
  if (threadIdx.x != 0) return;
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0xFFFFFFFFu) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) return;
    __builtin_amdgcn_s_sleep(4);
  }
}
}  // namespace

extern "C" int ds2_wait_resident(const unsigned* word, long long timeout, hipStream_t st) {
  ds2_launch(wait_resident_kernel, dim3(1), dim3(64), 0, st, word, timeout);
  return (int)hipGetLastError();
}

extern "C" int ds2_multi_fill(int n, void* const* ptrs, const unsigned long long* bytes, const unsigned* patterns,
                              hipStream_t st) {
  if (n < 0 || n > MF_MAX) return -50;
  MultiFill f{};
  unsigned long long total = 0;
  for (int i = 0; i < n; ++i) {
    if (bytes[i] % 4 != 0 || (reinterpret_cast<uintptr_t>(ptrs[i]) & 3) != 0) return -51;
    f.ptr[i] = static_cast<unsigned*>(ptrs[i]);
    f.words[i] = bytes[i] / 4;
    f.pattern[i] = patterns[i];
    total += f.words[i];
  }
  f.n = n;
  if (total == 0) return 0;
  unsigned long long blocks = (total / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  ds2_launch(multi_fill_kernel, dim3((unsigned)blocks), dim3(256), 0, st, f);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// One launch for the inputs of a replayed training-step graph (trainer.py _replay): up to 8
// row copies (rows x src_row bytes from a src of pitch src_pitch into a dst of pitch dst_pitch,
// the rest of each dst row up to dst_row bytes zeroed: a label matrix narrower than the
// captured width) plus up to 4 fp32 scalars written to one device slot (the optimizer's step
// constants), instead of one copy or fill launch each (~5 us apiece between two replays).
namespace {

constexpr int MC_MAX = 8;

struct MultiCopy {
  unsigned char* dst[MC_MAX];
  const unsigned char* src[MC_MAX];
  unsigned long long rows[MC_MAX];
  unsigned src_row[MC_MAX], dst_row[MC_MAX], src_pitch[MC_MAX], dst_pitch[MC_MAX];
  int n;
  float* sdst;
  float sval[4];
  int ns;
};

__global__ __launch_bounds__(256) void multi_copy_kernel(MultiCopy c) {
  const unsigned long long stride = (unsigned long long)gridDim.x * 256;
  const unsigned long long tid = (unsigned long long)blockIdx.x * 256 + threadIdx.x;
  if (tid < (unsigned long long)c.ns) c.sdst[tid] = c.sval[tid];
  for (int r = 0; r < c.n; ++r) {
    // 4-byte words (every row length, pitch and base is a multiple of 4: checked on the host)
    const unsigned dw = c.dst_row[r] / 4, sw = c.src_row[r] / 4;
    const unsigned long long total = c.rows[r] * dw;
    const unsigned* s = reinterpret_cast<const unsigned*>(c.src[r]);
    unsigned* d = reinterpret_cast<unsigned*>(c.dst[r]);
    const unsigned sp = c.src_pitch[r] / 4, dp = c.dst_pitch[r] / 4;
    for (unsigned long long i = tid; i < total; i += stride) {
      const unsigned long long row = i / dw;
      const unsigned col = (unsigned)(i - row * dw);
      d[row * dp + col] = col < sw ? s[row * sp + col] : 0u;
    }
  }
}

}  // namespace

extern "C" int ds2_multi_copy(int n, void* const* dst, const void* const* src, const unsigned long long* rows,
                              const unsigned* src_row, const unsigned* dst_row, const unsigned* src_pitch,
                              const unsigned* dst_pitch, float* sdst, const float* svals, int ns, hipStream_t st) {
  if (n < 0 || n > MC_MAX || ns < 0 || ns > 4 || (ns > 0 && sdst == nullptr)) return -50;
  MultiCopy c{};
  unsigned long long total = (unsigned long long)ns;
  for (int i = 0; i < n; ++i) {
    if ((src_row[i] | dst_row[i] | src_pitch[i] | dst_pitch[i]) % 4 != 0 || src_row[i] > dst_row[i] ||
        dst_row[i] > dst_pitch[i] || src_row[i] > src_pitch[i] ||
        ((reinterpret_cast<uintptr_t>(dst[i]) | reinterpret_cast<uintptr_t>(src[i])) & 3) != 0)
      return -51;
    c.dst[i] = static_cast<unsigned char*>(dst[i]);
    c.src[i] = static_cast<const unsigned char*>(src[i]);
    c.rows[i] = rows[i];
    c.src_row[i] = src_row[i]; c.dst_row[i] = dst_row[i];
    c.src_pitch[i] = src_pitch[i]; c.dst_pitch[i] = dst_pitch[i];
    total += rows[i] * (dst_row[i] / 4);
  }
  c.n = n;
  c.sdst = sdst;
  for (int i = 0; i < ns; ++i) c.sval[i] = svals[i];
  c.ns = ns;
  if (total == 0) return 0;
  unsigned long long blocks = (total + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(multi_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, st, c);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Step inputs in one launch: the features cast to the compute dtype (fp32 -> bf16, 4 per
// thread) and the recurrence lengths T2 = floor((T - 34) / 4) of the conv front-end
// (ops/reference.py get_rnn_seqlen; src/deepSpeech.py:38-48) from the utterance lengths,
// instead of a cast kernel and two integer kernels in front of every step.
namespace {

__global__ __launch_bounds__(256) void prep_inputs_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                          long long n, const int* __restrict__ lens_in,
                                                          int* __restrict__ lens_out, int nl) {
  const long long tid = (long long)blockIdx.x * 256 + threadIdx.x;
  if (tid < nl) {
    const int t = lens_in[tid] - 34;
    lens_out[tid] = t >= 0 ? t / 4 : -((-t + 3) / 4);          // floor division
  }
  const long long stride = (long long)gridDim.x * 256;
  const long long n4 = n / 4;
  for (long long i = tid; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    uint2 o;
    o.x = (unsigned)f2bf(v.x) | ((unsigned)f2bf(v.y) << 16);
    o.y = (unsigned)f2bf(v.z) | ((unsigned)f2bf(v.w) << 16);
    reinterpret_cast<uint2*>(y)[i] = o;
  }
  for (long long i = n4 * 4 + tid; i < n; i += stride) y[i] = f2bf(x[i]);
}

}  // namespace

extern "C" int ds2_prep_inputs(const float* x, void* y, long long n, const int* lens_in, int* lens_out, int nl,
                               hipStream_t st) {
  if ((reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(y) & 7)) return -52;
  long long blocks = (n / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(prep_inputs_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, (bf16_t*)y, n, lens_in,
                     lens_out, nl);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// bf16 transpose out[c][r] = in[r][c] ([R][C] -> [C][R], both row-major, unit-stride rows):
// the K-contiguous W^T shadow of a recurrent layer's [W_fw; W_bw] that the input-gradient
// GEMM dx = dgx W reads as a row-major operand (csrc/gemm.hip measured faster on it than on
// W's column-major reading). 64 x 64 tiles through LDS: 16-B row reads of the input
// (8 bf16 per lane) and 16-B row writes of the output; the LDS tile is padded by one
// 4-byte word per row so the column gathers of the write pass spread over the banks.
namespace {

constexpr int TT = 64;

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ in, bf16_t* __restrict__ out,
                                                             int R, int C, int ldi, int ldo) {
  __shared__ bf16_t tile[TT][TT + 2];
  const int tc = blockIdx.x * TT, tr = blockIdx.y * TT;
  const int t = threadIdx.x;
  // read: 64 rows x 8 chunks of 8 bf16 = 512 chunks, 2 per thread
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = t + 256 * k, r = q >> 3, c8 = (q & 7) * 8;
    const int gr = tr + r, gc = tc + c8;
    bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (gr < R && gc + 8 <= C) v = *reinterpret_cast<const bf16x8*>(in + (size_t)gr * ldi + gc);
    else if (gr < R)
      for (int j = 0; j < 8; ++j) v[j] = gc + j < C ? (short)in[(size_t)gr * ldi + gc + j] : (short)0;
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[r][c8 + j] = (bf16_t)v[j];
  }
  __syncthreads();
  // write: output rows = input columns
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = t + 256 * k, c = q >> 3, r8 = (q & 7) * 8;
    const int oc = tc + c, orr = tr + r8;
    if (oc >= C) continue;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (short)tile[r8 + j][c];
    if (orr + 8 <= R) *reinterpret_cast<bf16x8*>(out + (size_t)oc * ldo + orr) = v;
    else
      for (int j = 0; j < 8; ++j)
        if (orr + j < R) out[(size_t)oc * ldo + orr + j] = (bf16_t)v[j];
  }
}

}  // namespace

extern "C" int ds2_transpose_bf16(const void* in, void* out, int R, int C, int ldi, int ldo, hipStream_t st) {
  if (R <= 0 || C <= 0 || ldi < C || ldo < R || ldi % 8 || ldo % 8 || (reinterpret_cast<uintptr_t>(in) & 15) ||
      (reinterpret_cast<uintptr_t>(out) & 15))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((C + TT - 1) / TT, (R + TT - 1) / TT), dim3(256), 0, st,
                     (const bf16_t*)in, (bf16_t*)out, R, C, ldi, ldo);
  return (int)hipGetLastError();
}
