// Shared device helpers for the deepspeech_amd gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

namespace ds2 {

typedef __attribute__((ext_vector_type(8))) short bf16x8;   // MFMA 16x16x32 A/B fragment
typedef __attribute__((ext_vector_type(4))) float f32x4;    // MFMA 16x16 accumulator
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef unsigned short bf16_t;                               // raw bf16 bits

__device__ __forceinline__ float bf2f(bf16_t u) { return __uint_as_float(((unsigned)u) << 16); }

// round-to-nearest-even f32 -> bf16 in hardware (gfx950 v_cvt_pk_bf16_f32; NaN stays a quiet
// NaN). The integer emulation it replaces cost ~6 VALU ops + a NaN branch per value.
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

// v_exp_f32 + v_rcp_f32 (1 ulp): the IEEE-correct division would add a 10-instruction
// div_scale/div_fmas/div_fixup sequence per call on the recurrence's critical path
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float tanhf_(float x) { return 1.0f - 2.0f * __builtin_amdgcn_rcpf(__expf(2.0f * x) + 1.0f); }

// Buffer resource over [base, base+bytes) — wave-uniform inputs only (T8/T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

constexpr int AUX_SC1 = 16;   // gfx950 cache-policy bit: sc1 (bypass L1, write-through)

__device__ __forceinline__ i32x4 load_sc1_b128(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX_SC1));
}
__device__ __forceinline__ void store_sc1_b128(__amdgpu_buffer_rsrc_t r, unsigned off, i32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                         r, off, 0, AUX_SC1);
}

// Device-side checks of the debug build (DS2_DEBUG=1 python build.py): print the failing
// condition with its block/thread and carry on. Deliberately no trap: on the shared MI355X
// pool a faulting kernel can reset every GPU of the node, so a debug build reports instead.
#ifdef DS2_DEBUG
#define DS2_DCHECK(cond)                                                                      \
  do {                                                                                        \
    if (!(cond))                                                                              \
      printf("DS2_DCHECK failed %s:%d block %d thread %d: %s\n", __FILE__, __LINE__,          \
             (int)blockIdx.x, (int)threadIdx.x, #cond);                                       \
  } while (0)
#else
#define DS2_DCHECK(cond) \
  do {                   \
  } while (0)
#endif

// plain (L2 write-back) store through the same resource: the base stays in the resource's
// SGPRs (a pointer store made the compiler re-load the base from the kernel arguments, an
// s_load + lgkmcnt(0) wait per store inside the latency-critical publish loops)
__device__ __forceinline__ void store_b128(__amdgpu_buffer_rsrc_t r, unsigned off, i32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                         r, off, 0, 0);
}

__device__ __forceinline__ unsigned ld_flag(const unsigned* p) {
  return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Two bf16 partials in one dword, each carrying the use tag of a reduce-scatter ring slot in
// its mantissa LSB (the BPTT kernels of rnn_xcd.hip and rnn_fp8.hip); this conversion sits on
// the critical path of every BPTT step.
// Hardware RNE pair conversion (one v_cvt_pk_bf16_f32), then the LSB set to the tag: |error|
// <= 1.5 bf16 ulp, 3 VALU ops per pair on the publish critical path (a truncate-and-step
// variant is < 1 ulp but 5-6 ops, measured slower). No carry, so no 0xFFFF special case.
__device__ __forceinline__ unsigned bf16x2_tagged(float lo, float hi, unsigned tagmask) {
  typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
  const bf2_t p = {(__bf16)lo, (__bf16)hi};
  const unsigned d = __builtin_bit_cast(unsigned, p);
  // one bitfield insert instead of and + or (gfx9 VOP3 takes no literal, so the compiler
  // cannot fuse them into v_and_or_b32): r = (mask & tagmask) | (~mask & d)
  unsigned r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(0x00010001u), "s"(tagmask), "v"(d));
  return r;
}

__device__ __forceinline__ bool granule_tagged16(i32x4 v, unsigned tag) {
  const unsigned want = tag ? 0x00010001u : 0u;
  return (((unsigned)v[0] & 0x00010001u) == want) && (((unsigned)v[1] & 0x00010001u) == want) &&
         (((unsigned)v[2] & 0x00010001u) == want) && (((unsigned)v[3] & 0x00010001u) == want);
}

// Workgroup barrier that orders LDS only. __syncthreads() also emits s_waitcnt vmcnt(0),
// which makes every wave wait for ALL its outstanding global loads and stores at the
// barrier — fatal for a wave that keeps prefetches in flight across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One element of TF's Adam (epsilon-hat form) and of the weight EMA, every rounding spelled out
// (explicit fma / _rn products, nothing left to the compiler's contraction choice), so every
// kernel that applies the update — the streaming optimizer (optim.hip) and the fused epilogue
// of the grouped weight-gradient GEMM (gemm8.hip) — rounds identically: the result of an
// element does not depend on which kernel or which launch split updated it.
__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, float lr_t, float b1, float b2,
                                      float eps, float gscale) {
  const float gj = __fmul_rn(g, gscale);
  m = __fmaf_rn(b1, m, __fmul_rn(1.f - b1, gj));
  v = __fmaf_rn(b2, v, __fmul_rn(__fmul_rn(1.f - b2, gj), gj));
  p = __fmaf_rn(-lr_t, __fdiv_rn(m, __fadd_rn(__fsqrt_rn(v), eps)), p);
}
__device__ __forceinline__ float ema1(float e, float p, float keep) { return __fmaf_rn(keep, __fsub_rn(e, p), p); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace ds2

// Buffers the NEXT kernel of a stream needs initialised (a recurrence's h0 slots, sentinel-
// filled exchange slots, census words, bias partials): written by a persistent GEMM launch's
// lighter workgroups (one work unit fewer than the busiest) after their last unit, while the
// others finish theirs, instead of by a separate multi_fill launch on the critical path
// (csrc/fill.hip semantics: region r = words[r] 32-bit words of pattern[r]).
struct DS2Fill {
  int n;
  unsigned* ptr[8];
  unsigned long long words[8];
  unsigned pattern[8];
};

// This workgroup's share of a DS2Fill in a persistent grid over `total` work units where XCD x
// walks [x * tx, (x + 1) * tx) and its workgroup l (blockIdx = 8 l + x, per = gridDim / 8 of
// them) owns units l, l + per, ...: a workgroup is light when it owns fewer than
// ceil(tx / per), and the light ones (all of them when none is) split the regions' 16-B chunks
// in (XCD, l) order. nthr: threads per workgroup.
__device__ inline void fill_idle(const DS2Fill& f, int total, int tx, int nthr) {
  const int per = gridDim.x >> 3, x = blockIdx.x & 7, l = blockIdx.x >> 3;
  const int cmax = (tx + per - 1) / per;
  int nl = 0, me = -1;
  for (int xx = 0; xx < 8; ++xx) {             // uniform: scalar arithmetic
    const int cnt = max(0, min(total, (xx + 1) * tx) - xx * tx);
    // light workgroups of XCD xx: ceil((cnt - l) / per) < cmax, i.e. l >= cnt - (cmax - 1) * per
    const int first = max(0, min(per, cnt - (cmax - 1) * per));
    if (xx == x && l >= first) me = nl + (l - first);
    nl += per - first;
  }
  if (nl == 0) {                               // every workgroup equally busy: all of them fill
    nl = gridDim.x;
    me = x * per + l;
  }
  if (me < 0) return;
  const unsigned long long stride = (unsigned long long)nl * nthr;
  const unsigned long long t0 = (unsigned long long)me * nthr + threadIdx.x;
  for (int r = 0; r < f.n; ++r) {
    unsigned* p = f.ptr[r];
    const unsigned v = f.pattern[r];
    const unsigned long long nw = f.words[r];
    const unsigned long long n4 = ((reinterpret_cast<uintptr_t>(p) & 15) == 0) ? nw / 4 : 0;
    const ds2::i32x4 v4 = {(int)v, (int)v, (int)v, (int)v};
    for (unsigned long long i = t0; i < n4; i += stride) reinterpret_cast<ds2::i32x4*>(p)[i] = v4;
    for (unsigned long long i = n4 * 4 + t0; i < nw; i += stride) p[i] = v;
  }
}

// Completion event armed for the next launch made through ds2_launch (hipExtLaunchKernel's stop
// event; fill.hip ds2_arm_stop_event / ds2_take_stop_event): another stream can wait for that
// kernel without a marker packet in this kernel's queue, each of which holds the queue ~6 us
// between two kernels (tools/probe_event_gap.py). The host launchers whose kernel is the last
// of an op take the event themselves and hand it to that launch.
extern "C" hipEvent_t ds2_take_stop_event();
extern "C" void ds2_arm_stop_event(hipEvent_t e);

template <typename F, typename... Args>
inline void ds2_launch(F kern, dim3 grid, dim3 block, unsigned lds, hipStream_t st, Args... args) {
  hipEvent_t e = ds2_take_stop_event();
  if (e != nullptr) hipExtLaunchKernelGGL(kern, grid, block, lds, st, nullptr, e, 0, args...);
  else hipLaunchKernelGGL(kern, grid, block, lds, st, args...);
}

#define DS2_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) return (int)_e;                                          \
  } while (0)
