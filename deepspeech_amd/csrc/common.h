// Shared device helpers for the deepspeech_amd gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
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

// Workgroup barrier that orders LDS only. __syncthreads() also emits s_waitcnt vmcnt(0),
// which makes every wave wait for ALL its outstanding global loads and stores at the
// barrier — fatal for a wave that keeps prefetches in flight across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

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

#define DS2_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) return (int)_e;                                          \
  } while (0)
