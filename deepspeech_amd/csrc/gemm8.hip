// 256x256-tile, 8-phase MFMA GEMM for the recurrent layers' big GEMMs (gfx950), bf16 or
// fp8 e4m3 operands, fp32 accumulation.
//
//   C[m][n] = epi( alpha * alpha_dev[0] * alpha_dev2[0] * sum_k A[m][k] B[n][k] )
//   A row-major [M][K] (lda), B row-major [N][K] (ldb) — both K-contiguous ("NT").
//   epi 0: bf16 C = . + bias[n] (bf16, optional);  1: fp32 C = .;  2: fp32 C += .
//
// Reference call sites: the hoisted input projection x W^T of CustomRNNCell2
// (src/custom_ops.py:59-61) for every direction at once, and the input gradient
// dx = dgx W (autograd of the same op, src/deepSpeech_train.py:287) on a K-contiguous W^T.
//
// Structure (cdna_hip_programming.md §5 "The 256^2 8-phase template"): one workgroup of 8
// waves per CU computes a 256x256 C tile; K advances in 128-byte k-tiles (64 bf16 or 128
// fp8 elements) staged global -> LDS by global_load_lds_dwordx4 into two LDS buffers (2 x
// 64 KB: A rows 0-127 | A rows 128-255 | B rows 0-127 | B rows 128-255, "half-tiles" of
// 16 KB). A k-tile is consumed in 4 phases, one 128x128 C quadrant each, in the order
// Q(0,0) Q(0,1) Q(1,1) Q(1,0): a phase reads only the A half qm and the B half qn, so a
// half-tile of the buffer is free again one phase after its last reader (A0 after Q(0,1),
// B1 after Q(1,1), A1 / B0 after Q(1,0)) and the next-but-one k-tile streams into it while
// the current k-tile is still being multiplied. Each phase:
//     ds_read the wave's register subtile (8 A and/or 4 B ds_read_b128)
//     issue one half-tile of a later k-tile (2 glds per wave)
//     [phases 3 and 7: s_waitcnt vmcnt(4) — every half-tile but the two just issued landed]
//     s_waitcnt lgkmcnt(0) ; s_barrier ; 16 MFMAs of the wave's 64x32 share ; s_barrier
// Staggered wave groups (MI355X_MICROARCH.md item 9): waves 4-7 execute one extra barrier
// before the k-loop (waves 0-3 one after it), so every barrier pairs group 0's "after MFMA"
// with group 1's "before MFMA" of the same phase: the SIMD partners w / w + 4 alternate, one
// issuing its LDS reads and glds while the other runs its MFMA cluster (measured +11-27 %
// over both groups bursting together). The lgkmcnt(0) before the first barrier of a phase
// keeps the 1-phase restage WAR-safe under the half-phase offset.
// Iteration = 2 k-tiles (even k-tile in buffer 0, odd in buffer 1) = 8 phases; stage plan:
//     phase 0, 1: odd k-tile t+1's A1, B0 (buffer 1; its A0, B1 were issued a phase 6, 7 earlier)
//     phase 2..5: k-tile t+2's A0, B1, A1, B0 (buffer 0, each one phase after its last read)
//     phase 6, 7: k-tile t+3's A0, B1 (buffer 1)
// so a staged half-tile is retired by the vmcnt of phase 3 / 7 and first read in the phase
// after it (RAW: LDS-DMA data is ordered for ds_read only by the issuing waves' vmcnt and a
// barrier every reader has passed), and is rewritten only after the barrier that follows
// every wave's last read of it (WAR). No __syncthreads in the loop: its vmcnt(0) would
// drain the in-flight half-tiles; every other global access sits outside the loop.
//
// LDS images: 128-B rows, 16-B chunk c of row r at position c ^ ((r >> 1) & 7) (the swizzle
// goes on the per-lane glds SOURCE address: glds writes lane-linear), conflict-free for the
// 16-row x one-chunk ds_read_b128 of a 16x16x32 operand. Operands are swapped in the MFMA
// (D' = B A^T), so a lane ends with 4 consecutive C columns of one row: one 8-B (bf16) /
// 16-B (fp32) store per fragment.
// fp8: one v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, unit E8M0 block scales: the
// per-tensor scales are folded into alpha_dev / alpha_dev2) per fragment per k-tile in
// place of the bf16 pair: same LDS bytes, same cycles, twice the K per k-tile. A lane's 32
// fp8 of a row are the two 16-B chunks the bf16 k-substeps 0 and 1 read; A and B use the
// same k assignment, so the product is the full sum over the k-tile.
// Persistent grid: one workgroup per CU (a multiple of 8); XCD x = blockIdx % 8 walks the
// contiguous work-unit range [x*Tx, (x+1)*Tx) of a grouped order (8 m-tiles x all n-tiles,
// m fastest), so the tiles an XCD holds at once share A rows and B columns in its L2.
// Problem table: a launch carries up to 24 independent GEMMs of the same operand modes
// (batch members, or every recurrent layer's deferred weight gradients); work units are
// numbered problem by problem and a workgroup looks its problem up from the kernel
// arguments (scalar loads), so one grid covers all their tiles.
// Tails: K % 32 == 0 (bf16; a last k-tile of 32 skips its second k-substep) or K % 128 == 0
// (fp8: the quantiser pads K with zeros); rows past M / N are clamped on load and masked on
// store.
//
// Column-mode operands (bf16): an operand stored [K][M] (A) or [K][N] (B), M / N contiguous —
// the input gradient dx = dgx W reads W [6H][D] as its B, the weight gradients dW = dgx^T x
// and dU = dgh^T h read both operands that way. Its half-tile is a [64 k][128 cols] image
// (256-B k-rows, 16-B chunk c of k-row k at c ^ 2((k & 3) | ((k >> 1) & 4)), 4 k-rows per
// glds wave-instruction), read as MFMA fragments with ds_read_b64_tr_b16 (8 k of one column
// per lane from two 4-row transposed reads; inline asm, see rdtr). k-rows past K come back
// as zeros from the bounds-checked buffer load, so any K works.
// Fused optimizer epilogue (G8Opt.on, group launches of fp32 first-write members): the launch
// is the tail of a single-device backward that produces every recurrent weight gradient, so
// instead of storing a gradient tile for a separate Adam pass to read back, the epilogue
// applies Adam + weight EMA to the same arena elements at once (adam1 / ema1 of common.h,
// bitwise the streaming optimizer's update): per element it reads p, m, v, ema and writes p, m,
// v, ema and the bf16 compute shadow (the gradient itself only with store_g). The members' C
// are views of the gradient arena; p / m / v / ema / p16 are indexed at the same element.
// Split-K (S > 1): work unit = (tile, k-slice); each unit stores its raw fp32 partial tile to
// a workspace [S][M][N] per problem, and the tile's last-arriving slice sums the S partials in
// slice order (deterministic) and applies the epilogue, in the same launch. For the
// tall-skinny shapes (dx with D = 800: 124 256^2 tiles; dW / dU: 76-80) that would
// otherwise leave most CUs idle.
#include <algorithm>
#include <type_traits>

#include "common.h"

using namespace ds2;

// Adam + EMA applied in the epilogue (see the header): arena bases and this step's constants
// (the same layout is declared in bindings.cpp)
struct DS2G8Opt {
  float* p;
  float* m;
  float* v;
  float* ema;             // may be null (no EMA)
  unsigned short* p16;    // bf16 shadow, may be null
  const float* gbase;     // gradient arena base: element index of C(m, n) = C - gbase + m*ldc + n
  float lr_t, b1, b2, eps, gscale, keep;
  int on, store_g;
};

namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((ext_vector_type(8))) int i32x8;

// one GEMM of a launch. A launch holds one problem, the members of a batched GEMM, or a
// group of unrelated GEMMs of the same operand modes (the deferred weight gradients of every
// recurrent layer: one grid over all their tiles instead of one launch each)
struct G8Prob {
  const unsigned char* A;
  const unsigned char* B;
  void* C;
  float* ws;              // S > 1: fp32 partials [S][M][N]
  unsigned* cnt;          // S > 1: per-tile arrival counters [tiles], zero between launches
  int M, N, Kb;           // Kb: reduction length in BYTES (2K for bf16, K for fp8)
  int lda, ldb, ldc;      // lda / ldb in bytes, ldc in elements
  int epi;
  int S, kps;             // split-K: S k-slices of kps k-tiles each (S = 1: no split)
  int ustart;             // first work unit of this problem in the launch
};

constexpr int G8_MAXP = 24;
constexpr int G8_MAXFILL = 8;


using G8Opt = DS2G8Opt;

// Epilogue arithmetic with every rounding spelled out (no compiler-chosen contraction), shared
// by the GEMM's own epilogue and g8_reduce_kernel so both give bitwise the same C
__device__ __forceinline__ uint2 epi_bf16(float alpha, f32x4 v, const float (&bv)[4]) {
  const unsigned lo = (unsigned)f2bf(__fmaf_rn(alpha, v[0], bv[0])) | ((unsigned)f2bf(__fmaf_rn(alpha, v[1], bv[1])) << 16);
  const unsigned hi = (unsigned)f2bf(__fmaf_rn(alpha, v[2], bv[2])) | ((unsigned)f2bf(__fmaf_rn(alpha, v[3], bv[3])) << 16);
  return make_uint2(lo, hi);
}
__device__ __forceinline__ float4 epi_f32(float alpha, f32x4 v) {
  return make_float4(__fmul_rn(alpha, v[0]), __fmul_rn(alpha, v[1]), __fmul_rn(alpha, v[2]), __fmul_rn(alpha, v[3]));
}
__device__ __forceinline__ float4 epi_acc(float alpha, f32x4 v, float4 c) {
  return make_float4(__fmaf_rn(alpha, v[0], c.x), __fmaf_rn(alpha, v[1], c.y), __fmaf_rn(alpha, v[2], c.z),
                     __fmaf_rn(alpha, v[3], c.w));
}

struct G8Args {
  G8Prob p[G8_MAXP];
  G8Opt opt;
  DS2Fill fill;
  const bf16_t* bias;
  const float* alpha_dev;
  const float* alpha_dev2;
  float alpha;
  int np, total;          // problems, work units of all problems
  int ext_red;            // split units only store their fp32 partial; g8_reduce_kernel sums them
};

constexpr int NWV = 8;
constexpr int NTHR = NWV * 64;
constexpr int ROWB = 128;               // bytes of a staged row (one k-tile)
constexpr int HALF = 128 * ROWB;        // 16 KB
constexpr int BUFB = 4 * HALF;          // A0 A1 B0 B1
constexpr int LDS_BYTES = 2 * BUFB;     // 128 KB
constexpr int GROUP_M = 8;

__device__ __forceinline__ int rsw(int r) { return (r >> 1) & 7; }

// Per-lane byte offsets of a half-tile's two glds (k-tile 0): rows [row0, row0 + 128) of an
// operand (clamped to lim - 1), the lane's swizzled 16-B chunk. A k-tile adds kb0.
__device__ __forceinline__ void half_offsets(unsigned (&o)[2], int ld, int row0, int lim, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = wave + NWV * j;                 // 1-KB wave-instruction: rows 8i .. 8i+7
    const int r = 8 * i + (lane >> 3);
    const int c = (lane & 7) ^ rsw(r);
    o[j] = (unsigned)(min(row0 + r, lim - 1) * ld + 16 * c);
  }
}

// one half-tile through the operand's buffer resource (32-bit offsets: 2 VGPRs per half
// instead of 64-bit pointers). Chunks past the row's end (a ragged last bf16 k-tile) read
// the next row, or zeros past the operand (bounds-checked), and are never multiplied.
// AUX: the loads' cache-policy bits (0 default; 2 = nt, a streaming hint).
template <int AUX = 0>
__device__ __forceinline__ void stage_half(unsigned char* dst, __amdgpu_buffer_rsrc_t rs, const unsigned (&o)[2],
                                           unsigned kb0, int wave) {
#pragma unroll
  for (int j = 0; j < 2; ++j)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(dst + (wave + NWV * j) * 1024), 16, o[j] + kb0, 0, 0,
                                             AUX);
}

// cache policy of the weight-gradient (column-column) kernels' operand loads: these launches
// run beside the latency-bound persistent BPTT, whose per-step loads and partial-sum exchange
// live in the same XCD L2. nt (aux 2, a streaming hint) measured, not kept:
// with dW + dU beside each BPTT, 7.549 / 7.583 / 7.560 ms/step vs 7.584 / 7.683 / 7.594 default
// (scripts/r6_defer2.sh); once the dU GEMMs moved to the next forward (trainer.py _CARRY_DU),
// 7.450 / 7.439 vs 7.422 / 7.430, and on the ReLU-1760 stack, whose weight gradients all run
// as ONE grouped tail launch with nothing beside it, 14.54 / 14.54 vs 13.83 / 13.79; config 5
// fp8 neutral (scripts/r6_nt.sh). Compile-time A/B: build.py --variant NAME -D G8_COL_AUX=2.
#ifndef G8_COL_AUX
#define G8_COL_AUX 0
#endif

__device__ __forceinline__ i32x4 rd16(const unsigned char* half, int r, int chunk) {
  return *(const i32x4*)(half + r * ROWB + ((chunk ^ rsw(r)) << 4));
}

// s_barrier that is also a compiler memory barrier (the builtin is IntrNoMem: LLVM may move
// LDS reads and the glds issue across it); lgkmcnt is not waited here — the compiler puts
// its own counted lgkmcnt in front of each MFMA that consumes a ds_read result
__device__ __forceinline__ void bar() { asm volatile("s_barrier" ::: "memory"); }

// ---- column-mode operands ([K][cols] storage) ----
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4_t;
__device__ __forceinline__ int csw(int k) { return 2 * ((k & 3) | ((k >> 1) & 4)); }

// per-lane byte offsets of a col half-tile's two glds (k-tile 0): k-rows 4i + lane / 16,
// columns [col0, col0 + 128) clamped to the last full 16-B chunk below lim (lim % 8 == 0)
__device__ __forceinline__ void half_offsets_col(unsigned (&o)[2], int ld, int col0, int lim, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = wave + NWV * j;
    const int kr = 4 * i + (lane >> 4);
    const int c = (lane & 15) ^ csw(kr);
    o[j] = (unsigned)(kr * ld + 2 * min(col0 + 8 * c, lim - 8));
  }
}

// LDS byte offsets (within a col half-tile) of the two transposed 4-row reads that give a
// lane its 8 k of fragment column block rb, k-substep 0 (substep 1: + 32 k-rows = 8 KB)
__device__ __forceinline__ void col_frag_offsets(unsigned& o0, unsigned& o1, int rb, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int c = (rb * 16 + 4 * p) >> 3;
  const int k0 = 8 * g + q;
  o0 = (unsigned)(k0 * 256 + ((c ^ csw(k0)) << 4) + 8 * (p & 1));
  o1 = (unsigned)((k0 + 4) * 256 + ((c ^ csw(k0 + 4)) << 4) + 8 * (p & 1));
}

// The transposed read as inline asm: hipcc puts an s_waitcnt vmcnt(0) in front of every
// __builtin_amdgcn_ds_read_tr16_b64 (it cannot tell the read from the in-flight LDS-DMA
// writes of later k-tiles), which drained the glds pipeline in every phase of a column-mode
// GEMM (measured: col-col at ~60 % of the row-row kernel's rate). The compiler then also does
// not wait for these results: the k-loop retires them with an explicit lgkmcnt(0) before the
// phase's MFMA barrier. addr: LDS byte address (lds_addr), OFF: immediate byte offset.
template <int OFF>
__device__ __forceinline__ s16x4 rdtr(unsigned addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// fragment of the col half-tile at LDS byte offset HOFF (< 48 KB + 8 KB: immediates) from the
// lane's two transposed-read addresses a0 / a1 (buffer base included)
template <int HOFF>
__device__ __forceinline__ i32x8 col_frag(unsigned a0, unsigned a1) {
  const s16x4 a = rdtr<HOFF>(a0), b = rdtr<HOFF>(a1);
  const s16x4 c = rdtr<HOFF + 8192>(a0), d = rdtr<HOFF + 8192>(a1);
  const i32x4 lo = __builtin_bit_cast(i32x4, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
  const i32x4 hi = __builtin_bit_cast(i32x4, __builtin_shufflevector(c, d, 0, 1, 2, 3, 4, 5, 6, 7));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}

// wave's register subtile: 4 A fragments (rows wr*64 + 16i) or 2 B fragments (rows wc*32 +
// 16j) of one half, both k-substeps (chunks g and 4 + g of the row, g = lane / 16)
struct Frag {
  i32x8 v;       // k-substep 0 in elements 0..3, k-substep 1 in 4..7 (one register tuple)
};
__device__ __forceinline__ i32x8 cat(i32x4 lo, i32x4 hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x8 lo8(i32x8 v) {
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(v, v, 0, 1, 2, 3));
}
__device__ __forceinline__ bf16x8 hi8(i32x8 v) {
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(v, v, 4, 5, 6, 7));
}

template <bool FP8, int UNUSED>
__device__ __forceinline__ void mfma_tile(f32x4 (&acc)[2][4], const Frag (&a)[4], const Frag (&b)[2], bool full) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (FP8) {
        acc[j][i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b[j].v, a[i].v, acc[j][i], 0, 0, 0, 0x7f7f7f7f,
                                                                     0, 0x7f7f7f7f);
      } else {
        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lo8(b[j].v), lo8(a[i].v), acc[j][i], 0, 0, 0);
      }
    }
  if constexpr (!FP8) {
    if (full) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hi8(b[j].v), hi8(a[i].v), acc[j][i], 0, 0, 0);
    }
  }
  __builtin_amdgcn_s_setprio(0);
  // pin the cluster here: the MFMAs are pure, and without a use at this point IR-level code
  // motion sinks them past the barriers to the end of the k-loop (all fragments of all 8
  // phases then stay live: spills)
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(acc[j][i]));
}

// Adam + EMA of the 4 consecutive arena elements [e, e + 4) with gradient gv and their loaded
// state p, m, v, em (e % 4 == 0: the host checks the members' offsets and row strides).
// Non-temporal: the optimizer state is touched once per step and must not evict the GEMM's
// operands from L2.
__device__ __forceinline__ void opt_update4(const G8Opt& o, long long e, f32x4 gv, f32x4 p, f32x4 m, f32x4 v,
                                            f32x4 em) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float pj = p[j], mj = m[j], vj = v[j];
    adam1(pj, gv[j], mj, vj, o.lr_t, o.b1, o.b2, o.eps, o.gscale);
    p[j] = pj; m[j] = mj; v[j] = vj;
    em[j] = ema1(em[j], pj, o.keep);
  }
  __builtin_nontemporal_store(p, (f32x4*)(o.p + e));
  __builtin_nontemporal_store(m, (f32x4*)(o.m + e));
  __builtin_nontemporal_store(v, (f32x4*)(o.v + e));
  if (o.ema) __builtin_nontemporal_store(em, (f32x4*)(o.ema + e));
  if (o.p16) {
    bf16_t* p16 = o.p16;
    const unsigned lo = (unsigned)f2bf(p[0]) | ((unsigned)f2bf(p[1]) << 16);
    const unsigned hi = (unsigned)f2bf(p[2]) | ((unsigned)f2bf(p[3]) << 16);
    *(uint2*)(p16 + e) = make_uint2(lo, hi);
  }
  if (o.store_g) __builtin_nontemporal_store(gv, (f32x4*)(const_cast<float*>(o.gbase) + e));
}

template <bool FP8, int AC, int BC>
__global__ __launch_bounds__(NTHR) void gemm8_kernel(G8Args g) {
  static_assert(!FP8 || (!AC && !BC), "fp8 operands are K-contiguous");
  // the fused optimizer epilogue exists only in the weight-gradient (column-column) variant
  constexpr bool OPTEPI = !FP8 && AC && BC;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;         // wave's 64-row x 32-col share of a quadrant
  // work units of all problems, numbered problem by problem; XCD x = blockIdx % 8 walks the
  // contiguous range [x*Tx, (x+1)*Tx)
  const int total = g.total, tx = (total + 7) >> 3, xg = blockIdx.x & 7;
  int id = xg * tx + (blockIdx.x >> 3);
  const int id_end = min(total, (xg + 1) * tx), id_step = gridDim.x >> 3;
  float alpha = g.alpha;
  if (g.alpha_dev) alpha *= *g.alpha_dev;
  if (g.alpha_dev2) alpha *= *g.alpha_dev2;
  const int g16 = lane >> 4, r16 = lane & 15;

  // fragment addresses. Row mode: row r = base + 16i + lane % 16 has swizzle (r >> 1) & 7 =
  // (lane % 16 >> 1) & 7 for every fragment of the wave (bases are multiples of 16), so each
  // lane needs one byte offset per k-substep and every read is base + immediate. Col mode:
  // two offsets per fragment (the swizzle depends on the column block).
  const int sw = rsw(r16);
  const int c_lo = (g16 ^ sw) << 4, c_hi = ((4 + g16) ^ sw) << 4;
  // col mode: LDS byte addresses of the lane's transposed reads in buffer 0
  unsigned ca0[4], ca1[4], cb0[2], cb1[2];
  const unsigned lds0 = lds_addr(smem);
  if constexpr (AC) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      col_frag_offsets(ca0[i], ca1[i], wr * 4 + i, lane);
      ca0[i] += lds0;
      ca1[i] += lds0;
    }
  }
  if constexpr (BC) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      col_frag_offsets(cb0[j], cb1[j], wc * 2 + j, lane);
      cb0[j] += lds0 + 2 * HALF;
      cb1[j] += lds0 + 2 * HALF;
    }
  }

  int q = 0;                                         // problem of unit id (ids only grow)
  for (; id < id_end; id += id_step) {
    while (q + 1 < g.np && id >= g.p[q + 1].ustart) ++q;
    q = __builtin_amdgcn_readfirstlane(q);
    const G8Prob& P = g.p[q];
    const int M = P.M, N = P.N, S = P.S;
    const int ntm = (M + 255) / 256, ntn = (N + 255) / 256;
    const int nkt_all = (P.Kb + ROWB - 1) / ROWB;
    // a last k-tile of 32 bf16 with a row-mode operand: its second k-substep holds the next
    // row's data there (a col-mode operand's k-rows past K load as zeros), so it is skipped
    const bool ragged = !FP8 && !(AC && BC) && (P.Kb % ROWB) != 0;
    const int K = P.Kb / (FP8 ? 1 : 2);
    // bounds of the buffer resources: a row-mode operand holds its rows, a col-mode one K
    // k-rows (k-rows past K then load as zeros)
    const __amdgpu_buffer_rsrc_t rsA = make_rsrc(P.A, (unsigned)((size_t)(AC ? K : M) * P.lda));
    const __amdgpu_buffer_rsrc_t rsB = make_rsrc(P.B, (unsigned)((size_t)(BC ? K : N) * P.ldb));
    const int uid = id - P.ustart;
    const int tile = uid / S, ks = uid - tile * S;
    const int gsz = GROUP_M * ntn, grp = tile / gsz, first_m = grp * GROUP_M;
    const int gm = min(ntm - first_m, GROUP_M), within = tile - grp * gsz;
    const int m0 = (first_m + within % gm) * 256, n0 = (within / gm) * 256;
    const int kt0 = ks * P.kps;                      // this unit's k-tiles [kt0, kt0 + nkt)
    const int nkt = max(0, min(nkt_all - kt0, P.kps));
    // a ragged last tile whose second 128-row / 128-column quadrant lies wholly past M / N (the
    // weight gradients' N = 800 tile column holds 32 valid columns): those quadrants' MFMAs are
    // skipped (their accumulators are never stored); loads and barriers stay, so the staging
    // pipeline's vmcnt accounting is unchanged
#ifdef G8_NO_SKIP
    const bool live_m1 = true, live_n1 = true;       // A/B build: every quadrant multiplied
#else
    const bool live_m1 = m0 + 128 < M, live_n1 = n0 + 128 < N;
#endif

    unsigned oA0[2], oA1[2], oB0[2], oB1[2];
    if constexpr (AC) {
      half_offsets_col(oA0, P.lda, m0, M, wave, lane);
      half_offsets_col(oA1, P.lda, m0 + 128, M, wave, lane);
    } else {
      half_offsets(oA0, P.lda, m0, M, wave, lane);
      half_offsets(oA1, P.lda, m0 + 128, M, wave, lane);
    }
    if constexpr (BC) {
      half_offsets_col(oB0, P.ldb, n0, N, wave, lane);
      half_offsets_col(oB1, P.ldb, n0 + 128, N, wave, lane);
    } else {
      half_offsets(oB0, P.ldb, n0, N, wave, lane);
      half_offsets(oB1, P.ldb, n0 + 128, N, wave, lane);
    }
    // half-tile h of local k-tile t into buffer t & 1: h 0/1 = A rows 0-127 / 128-255, 2/3 = B.
    // A k-tile advances 128 bytes along a row-mode operand's rows, 64 k-rows of a col one.
    auto stage = [&](int t, int h) {
      if (t >= nkt) return;
      unsigned char* dst = smem + (t & 1) * BUFB + h * HALF;
      const int kt = kt0 + t;
      const unsigned ka = AC ? (unsigned)(kt * 64) * (unsigned)P.lda : (unsigned)(kt * ROWB);
      const unsigned kb = BC ? (unsigned)(kt * 64) * (unsigned)P.ldb : (unsigned)(kt * ROWB);
      constexpr int aux = (AC && BC) ? G8_COL_AUX : 0;
      if (h == 0) stage_half<aux>(dst, rsA, oA0, ka, wave);
      else if (h == 1) stage_half<aux>(dst, rsA, oA1, ka, wave);
      else if (h == 2) stage_half<aux>(dst, rsB, oB0, kb, wave);
      else stage_half<aux>(dst, rsB, oB1, kb, wave);
    };
    auto read_a = [&](Frag (&a)[4], auto BUF, auto QM) {
      constexpr int buf = decltype(BUF)::value, qm = decltype(QM)::value;
      if constexpr (AC) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i].v = col_frag<qm * HALF>(ca0[i] + buf * BUFB, ca1[i] + buf * BUFB);
      } else {
        const unsigned char* h = smem + (wr * 64 + r16) * ROWB + buf * BUFB + qm * HALF;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          a[i].v = cat(*(const i32x4*)(h + i * 16 * ROWB + c_lo), *(const i32x4*)(h + i * 16 * ROWB + c_hi));
      }
    };
    auto read_b = [&](Frag (&b)[2], auto BUF, auto QN) {
      constexpr int buf = decltype(BUF)::value, qn = decltype(QN)::value;
      if constexpr (BC) {
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j].v = col_frag<qn * HALF>(cb0[j] + buf * BUFB, cb1[j] + buf * BUFB);
      } else {
        const unsigned char* h = smem + 2 * HALF + (wc * 32 + r16) * ROWB + buf * BUFB + qn * HALF;
#pragma unroll
        for (int j = 0; j < 2; ++j)
          b[j].v = cat(*(const i32x4*)(h + j * 16 * ROWB + c_lo), *(const i32x4*)(h + j * 16 * ROWB + c_hi));
      }
    };

    f32x4 acc[2][2][2][4];
#pragma unroll
    for (int a0 = 0; a0 < 2; ++a0)
#pragma unroll
      for (int a1 = 0; a1 < 2; ++a1)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[a0][a1][j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    // prologue: k-tile 0 whole, k-tile 1's A0 and B1 (the halves its phases 6, 7 would stage)
    stage(0, 0); stage(0, 2); stage(0, 3); stage(0, 1);
    stage(1, 0); stage(1, 3);
    // a vmcnt count names the glds issued AFTER the retire point, so a skipped stage (past
    // the last k-tile) needs the smaller count, never the steady-state one
    if (nkt > 1) wait_vm<4>();
    else wait_vm<0>();
    bar();

    Frag fa[4], fb[2];
    // One phase: quadrant Q(qm, qn) of the k-tile in buffer buf, staging half-tile sh of
    // k-tile st (skipped past the last k-tile), optionally retiring all but the last two
    // half-tiles (wait: 0 none, 1 = vmcnt(4) if half-tile st exists, else vmcnt(0)).
    auto phase = [&](auto BUF, auto QM, auto QN, auto RA, auto RB, int st, int sh, int wait, bool full) {
      constexpr int bf = decltype(BUF)::value, qm = decltype(QM)::value, qn = decltype(QN)::value;
      if constexpr (decltype(RB)::value) read_b(fb, BUF, QN);
      if constexpr (decltype(RA)::value && decltype(RB)::value) __builtin_amdgcn_sched_barrier(0);
      if constexpr (decltype(RA)::value) read_a(fa, BUF, QM);
      stage(st, sh);
      if (wait) {
        if (st < nkt) wait_vm<4>();
        else wait_vm<0>();
      }
      // staggered: the other wave group still reads this phase's half-tiles after this
      // barrier, so a wave's reads are retired before it (WAR of the 1-phase restage; the
      // asm transposed reads of column mode are waited for only here)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bar();
      __builtin_amdgcn_sched_barrier(0);
      if ((qm == 0 || live_m1) && (qn == 0 || live_n1)) mfma_tile<FP8, 0>(acc[qm][qn], fa, fb, full);
      __builtin_amdgcn_sched_barrier(0);   // the cluster stays between its barriers
      bar();
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using T_ = std::true_type;
    using F_ = std::false_type;
    // stagger: one extra barrier for waves 4-7 before the k-loop and for waves 0-3 after it,
    // so every barrier of the loop pairs group 0's phase p "after MFMA" with group 1's phase p
    // "before MFMA": one group's LDS reads and glds issue run under the other's MFMAs (the SIMD
    // partners w and w + 4 alternate roles) instead of both bursting together
    if (wr == 1) bar();
    int t0 = 0;
    for (; t0 + 1 < nkt; t0 += 2) {
      const bool full1 = !(ragged && kt0 + t0 + 1 == nkt_all - 1);
      // even k-tile t0 (buffer 0): Q(0,0) Q(0,1) Q(1,1) Q(1,0)
      phase(I0{}, I0{}, I0{}, T_{}, T_{}, t0 + 1, 1, 0, true);
      phase(I0{}, I0{}, I1{}, F_{}, T_{}, t0 + 1, 2, 0, true);
      phase(I0{}, I1{}, I1{}, T_{}, F_{}, t0 + 2, 0, 0, true);
      phase(I0{}, I1{}, I0{}, F_{}, T_{}, t0 + 2, 3, 1, true);   // retires k-tile t0 + 1
      // odd k-tile t0 + 1 (buffer 1)
      phase(I1{}, I0{}, I0{}, T_{}, T_{}, t0 + 2, 1, 0, full1);
      phase(I1{}, I0{}, I1{}, F_{}, T_{}, t0 + 2, 2, 0, full1);
      phase(I1{}, I1{}, I1{}, T_{}, F_{}, t0 + 3, 0, 0, full1);
      phase(I1{}, I1{}, I0{}, F_{}, T_{}, t0 + 3, 3, 1, full1);   // retires k-tile t0 + 2
    }
    if (t0 < nkt) {                     // an odd k-tile count: the last (even) k-tile alone
      const bool full0 = !(ragged && kt0 + t0 == nkt_all - 1);
      phase(I0{}, I0{}, I0{}, T_{}, T_{}, nkt, 0, 0, full0);
      phase(I0{}, I0{}, I1{}, F_{}, T_{}, nkt, 0, 0, full0);
      phase(I0{}, I1{}, I1{}, T_{}, F_{}, nkt, 0, 0, full0);
      phase(I0{}, I1{}, I0{}, F_{}, T_{}, nkt, 0, 0, full0);
    }
    if (wr == 0) bar();

    // epilogue: lane holds C[m][n .. n+3], m = .. + lane % 16, n = .. + 4 (lane / 16). A
    // split unit stores its raw fp32 partial into workspace slice ks (fp32, ld = N).
    const bool part = S > 1;
    // the final epilogue: lane's fragment (qm, qn, j, i) holds C[m][n .. n+3]
    auto finish = [&](auto&& value) {
      const int epi = P.epi;
      if constexpr (OPTEPI) {
        if (epi == 1 && g.opt.on) {
          // fused optimizer: OB row fragments of one (qm, qn, j) column block at a time, all
          // their state loads issued before any update (OB x the loads in flight of a
          // fragment-by-fragment chain, which left the epilogue latency-bound)
          constexpr int OB = 2;
          const long long cb = (long long)((const float*)P.C - g.opt.gbase);
#pragma unroll
          for (int qn = 0; qn < 2; ++qn)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const int n = n0 + qn * 128 + wc * 32 + 16 * j + 4 * g16;
#pragma unroll
              for (int qm = 0; qm < 2; ++qm)
#pragma unroll
                for (int i0 = 0; i0 < 4; i0 += OB) {
                  long long e[OB];
                  bool ok[OB];
                  f32x4 sp[OB], sm[OB], sv[OB], se[OB];
#pragma unroll
                  for (int b = 0; b < OB; ++b) {
                    const int m = m0 + qm * 128 + wr * 64 + 16 * (i0 + b) + r16;
                    ok[b] = m < M && n < N;
                    e[b] = cb + (long long)(ok[b] ? m : 0) * P.ldc + (ok[b] ? n : 0);
                    sp[b] = __builtin_nontemporal_load((const f32x4*)(g.opt.p + e[b]));
                    sm[b] = __builtin_nontemporal_load((const f32x4*)(g.opt.m + e[b]));
                    sv[b] = __builtin_nontemporal_load((const f32x4*)(g.opt.v + e[b]));
                    se[b] = g.opt.ema ? __builtin_nontemporal_load((const f32x4*)(g.opt.ema + e[b]))
                                      : f32x4{0.f, 0.f, 0.f, 0.f};
                  }
#pragma unroll
                  for (int b = 0; b < OB; ++b) {
                    if (!ok[b]) continue;
                    const int m = m0 + qm * 128 + wr * 64 + 16 * (i0 + b) + r16;
                    const f32x4 v = value(qm, qn, j, i0 + b, m, n);
                    opt_update4(g.opt, e[b], f32x4{alpha * v[0], alpha * v[1], alpha * v[2], alpha * v[3]}, sp[b],
                                sm[b], sv[b], se[b]);
                  }
                  // one batch's loads in flight at a time (hoisting the next batch's loads above
                  // these updates needs more VGPRs than the kernel has: spills)
                  __builtin_amdgcn_sched_barrier(0);
                }
            }
          return;
        }
      }
      char* Cz = (char*)P.C;
      const bool has_bias = epi == 0 && g.bias != nullptr;
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int n = n0 + qn * 128 + wc * 32 + 16 * j + 4 * g16;
          if (n >= N) continue;
          float bv[4] = {0.f, 0.f, 0.f, 0.f};
          if (has_bias) {
            const uint2 b2 = *(const uint2*)(g.bias + n);
            bv[0] = bf2f((bf16_t)(b2.x & 0xffff)); bv[1] = bf2f((bf16_t)(b2.x >> 16));
            bv[2] = bf2f((bf16_t)(b2.y & 0xffff)); bv[3] = bf2f((bf16_t)(b2.y >> 16));
          }
#pragma unroll
          for (int qm = 0; qm < 2; ++qm)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int m = m0 + qm * 128 + wr * 64 + 16 * i + r16;
              if (m >= M) continue;
              const f32x4 v = value(qm, qn, j, i, m, n);
              const size_t off = (size_t)m * P.ldc + n;
              if (epi == 0) {
                *(uint2*)(Cz + off * 2) = epi_bf16(alpha, v, bv);
              } else {
                float4* cp = (float4*)(Cz + off * 4);
                *cp = epi == 2 ? epi_acc(alpha, v, *cp) : epi_f32(alpha, v);
              }
            }
        }
    };
    if (!part) {
      finish([&](int qm, int qn, int j, int i, int, int) { return acc[qm][qn][j][i]; });
    } else {
      // Split-K, reduced in this launch by the tile's last-arriving slice (the guide's
      // counter hand-off, cdna_hip_programming.md §5 "Projection GEMM at M = 256" item 2, in
      // its write-through form): every slice stores its raw fp32 partial to workspace slab
      // ks with sc1 (write-through) stores, each wave drains them, the workgroup syncs and
      // one lane takes a ticket (relaxed, agent scope); the slice drawing S - 1 reads the S
      // slabs with sc1 loads (every load of them) and sums them in slice order 0 .. S-1
      // (deterministic whatever the arrival order), then resets the counter for the next
      // launch. No agent-scope release / acquire fence: on gfx950 those write back / flush
      // this XCD's whole L2, which beside the persistent BPTT cost ~20 % of the GEMM.
      const unsigned slab = (unsigned)((size_t)M * N * 4);
      const __amdgpu_buffer_rsrc_t rsw_ = make_rsrc(P.ws, (unsigned)(slab * (size_t)S));
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int n = n0 + qn * 128 + wc * 32 + 16 * j + 4 * g16;
          if (n >= N) continue;
#pragma unroll
          for (int qm = 0; qm < 2; ++qm)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int m = m0 + qm * 128 + wr * 64 + 16 * i + r16;
              if (m >= M) continue;
              store_sc1_b128(rsw_, (unsigned)ks * slab + (unsigned)((m * N + n) * 4),
                             __builtin_bit_cast(i32x4, acc[qm][qn][j][i]));
            }
        }
      if (g.ext_red) {
        // g8_reduce_kernel (the next launch on the stream) sums the slabs: nothing to wait for
        // here, and the next unit's prologue only rewrites LDS (every wave's last reads were
        // retired by the final phase's barrier)
        continue;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* flag = (int*)smem;                       // LDS is free: the k-loop has finished
      unsigned* cnt = P.cnt + tile;
      if (tid == 0) {
        const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == (unsigned)(S - 1);
        if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
      }
      __syncthreads();
      const bool last = *flag != 0;
      __syncthreads();                              // flag read before the next prologue's glds
      if (last)
        finish([&](int, int, int, int, int m, int n) {
          const unsigned off = (unsigned)((m * N + n) * 4);
          f32x4 v = __builtin_bit_cast(f32x4, load_sc1_b128(rsw_, off));
          for (int s2 = 1; s2 < S; ++s2) v += __builtin_bit_cast(f32x4, load_sc1_b128(rsw_, off + s2 * slab));
          return v;
        });
    }
    // the next tile's prologue restages buffer 0: every wave's last reads were retired by
    // the final phase's barrier, and the stores above only read registers
  }
  // only the row-row (projection) variant carries the fill: in the column-mode ones its live
  // values pushed the k-loop over 256 VGPRs
  if constexpr (!FP8 && AC == 0 && BC == 0) {
    if (g.fill.n > 0) fill_idle(g.fill, total, tx, NTHR);
  }
}

template <bool FP8, int AC, int BC>
int launch8(const G8Args& a, int cus, hipStream_t st) {
  auto kern = gemm8_kernel<FP8, AC, BC>;
  static bool attr = false;
  if (!attr) {
    DS2_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
    attr = true;
  }
  int grid = min(cus, (a.total + 7) & ~7);          // cus: the CU budget (device CUs or a cap)
  grid = max(8, grid & ~7);
  ds2_launch(kern, dim3(grid), dim3(NTHR), (unsigned)LDS_BYTES, st, a);
  return (int)hipGetLastError();
}

// validate one problem and fill its table entry (units from ustart); 0 or a hipError_t
int fill_prob(G8Prob& p, const void* A, const void* B, void* C, float* ws, unsigned* cnt, int M, int N, int K,
              int lda, int ldb, int ldc, int fp8, int a_col, int b_col, int epi, int S, int ustart) {
  const int es = fp8 ? 1 : 2;
  if (M <= 0 || N <= 0 || K <= 0 || N % 4 != 0 || S < 1) return (int)hipErrorInvalidValue;
  if (fp8 && (a_col || b_col || K % 128 != 0)) return (int)hipErrorInvalidValue;
  if (!fp8 && (!a_col || !b_col) && K % 32 != 0) return (int)hipErrorInvalidValue;
  if ((a_col && M % 8) || (b_col && N % 8)) return (int)hipErrorInvalidValue;
  if (((lda * es) % 16) || ((ldb * es) % 16) || ((uintptr_t)A % 16) || ((uintptr_t)B % 16))
    return (int)hipErrorInvalidValue;
  // 32-bit buffer offsets: each operand under 2 GB, a split's workspace too
  if ((long long)(a_col ? K : M) * lda * es >= (1LL << 31) || (long long)(b_col ? K : N) * ldb * es >= (1LL << 31))
    return (int)hipErrorInvalidValue;
  if (epi < 0 || epi > 2) return (int)hipErrorInvalidValue;
  const int nkt = (K * es + ROWB - 1) / ROWB;
  p.kps = (nkt + S - 1) / S;
  p.S = (nkt + p.kps - 1) / p.kps;                // no empty slice
  if (p.S > 1 && (!ws || !cnt || (long long)M * N * 4 * p.S >= (1LL << 32))) return (int)hipErrorInvalidValue;
  p.A = (const unsigned char*)A;
  p.B = (const unsigned char*)B;
  p.C = C;
  p.ws = ws;
  p.cnt = cnt;
  p.M = M; p.N = N; p.Kb = K * es;
  p.lda = lda * es; p.ldb = ldb * es; p.ldc = ldc;
  p.epi = epi;
  p.ustart = ustart;
  return 0;
}

int dispatch8(const G8Args& a, int fp8, int a_col, int b_col, int cus, hipStream_t st) {
  if (fp8) return launch8<true, 0, 0>(a, cus, st);
  if (!a_col && !b_col) return launch8<false, 0, 0>(a, cus, st);
  if (!a_col && b_col) return launch8<false, 0, 1>(a, cus, st);
  if (a_col && b_col) return launch8<false, 1, 1>(a, cus, st);
  return launch8<false, 1, 0>(a, cus, st);
}

int units_of(const G8Prob& p) { return ((p.M + 255) / 256) * ((p.N + 255) / 256) * p.S; }

// Split-K partials of one problem summed in slice order 0 .. S-1 (the same order and the
// same epilogue arithmetic as the in-launch last-arriver reduction, so the result is bitwise
// identical): every thread owns 4 consecutive columns of one row. Launched right behind the
// GEMM on the same stream when its k-slices only stored their slabs (G8Args.ext_red): all
// CUs reduce in parallel instead of each tile's last-arriving slice reading S slabs alone,
// which dominated small-M launches (dx of a 100-frame batch: 12 tiles x 4 slices).
__global__ __launch_bounds__(256) void g8_reduce_kernel(const float* __restrict__ ws, int S, int M, int N,
                                                        void* __restrict__ C, int ldc, int epi,
                                                        const bf16_t* __restrict__ bias, float alpha,
                                                        const float* __restrict__ alpha_dev,
                                                        const float* __restrict__ alpha_dev2) {
  if (alpha_dev) alpha *= *alpha_dev;
  if (alpha_dev2) alpha *= *alpha_dev2;
  const int n4 = N >> 2;
  const long long total = (long long)M * n4;
  const size_t slab = (size_t)M * N;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(i / n4), n = (int)(i - (long long)m * n4) * 4;
    const size_t off = (size_t)m * N + n;
    f32x4 v = __builtin_nontemporal_load((const f32x4*)(ws + off));
    for (int s2 = 1; s2 < S; ++s2) v += __builtin_nontemporal_load((const f32x4*)(ws + off + s2 * slab));
    const size_t co = (size_t)m * ldc + n;
    if (epi == 0) {
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (bias != nullptr) {
        const uint2 b2 = *(const uint2*)(bias + n);
        bv[0] = bf2f((bf16_t)(b2.x & 0xffff)); bv[1] = bf2f((bf16_t)(b2.x >> 16));
        bv[2] = bf2f((bf16_t)(b2.y & 0xffff)); bv[3] = bf2f((bf16_t)(b2.y >> 16));
      }
      *(uint2*)((bf16_t*)C + co) = epi_bf16(alpha, v, bv);
    } else {
      float4* cp = (float4*)((float*)C + co);
      *cp = epi == 2 ? epi_acc(alpha, v, *cp) : epi_f32(alpha, v);
    }
  }
}

}  // namespace

extern "C" {

// fp8: A / B hold e4m3 bytes (K elements per row, K % 128 == 0, row mode only); bf16: row-mode
// operands need K % 32 == 0, col-mode ones (a_col: A stored [K][M]; b_col: B stored [K][N])
// M % 8 / N % 8 == 0 and any K. lda / ldb / ldc in elements, batch strides likewise; the batch
// members are the launch's problems (batch <= 24).
// S > 1: split-K over S k-slices through ws (fp32, >= S * batch * M * N floats) and cnt
// (>= batch * tiles unsigned, all zero; every launch leaves them zero again). Launches that
// may run concurrently (different streams) need separate cnt buffers.
// ext_red (batch 1, S > 1): the k-slices only store their partials and g8_reduce_kernel,
// launched right after on the same stream, sums them on the whole chip.
int ds2_gemm8(const void* A, const void* B, void* C, const void* bias, const float* alpha_dev,
              const float* alpha_dev2, int M, int N, int K, int lda, int ldb, int ldc, int fp8, int a_col, int b_col,
              int epi, float alpha, int batch, long long sA, long long sB, long long sC, int S, float* ws,
              unsigned* cnt, int cus, const DS2Fill* fill, int ext_red, hipStream_t st) {
  const int es = fp8 ? 1 : 2;
  if (batch <= 0 || batch > G8_MAXP || (epi != 0 && bias)) return (int)hipErrorInvalidValue;
  if (ext_red && batch != 1) return (int)hipErrorInvalidValue;
  G8Args a;
  a.opt = G8Opt{};
  a.fill = DS2Fill{};
  if (fill != nullptr && fill->n > 0) {
    if (fill->n > G8_MAXFILL || fp8 || a_col || b_col) return (int)hipErrorInvalidValue;
    for (int i = 0; i < fill->n; ++i)
      if ((reinterpret_cast<uintptr_t>(fill->ptr[i]) & 3) != 0) return (int)hipErrorInvalidValue;
    a.fill = *fill;
  }
  a.bias = (const bf16_t*)bias;
  a.alpha_dev = alpha_dev;
  a.alpha_dev2 = alpha_dev2;
  a.alpha = alpha;
  a.np = batch;
  a.ext_red = 0;
  int u = 0;
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  for (int b = 0; b < batch; ++b) {
    G8Prob& p = a.p[b];
    const int rc = fill_prob(p, (const char*)A + b * sA * es, (const char*)B + b * sB * es,
                             (char*)C + b * sC * (epi == 0 ? 2 : 4), ws, cnt ? cnt + (size_t)b * tiles : nullptr, M,
                             N, K, lda, ldb, ldc, fp8, a_col, b_col, epi, S, u);
    if (rc) return rc;
    if (ws) p.ws = ws + (size_t)b * p.S * M * N;
    u += units_of(p);
  }
  a.total = u;
  const G8Prob& red = a.p[a.np - 1];
  a.ext_red = (ext_red && red.S > 1) ? 1 : 0;
  // an armed stop event belongs to the op's last launch: the reduction when one follows
  hipEvent_t stop = a.ext_red ? ds2_take_stop_event() : nullptr;
  int rc = dispatch8(a, fp8, a_col, b_col, cus, st);
  if (rc || !a.ext_red) {
    if (stop != nullptr) ds2_arm_stop_event(stop);
    return rc;
  }
  const long long work = (long long)red.M * (N / 4);
  const int grid = (int)std::max<long long>(1, std::min<long long>(4 * (long long)cus, (work + 255) / 256));
  ds2_arm_stop_event(stop);
  ds2_launch(g8_reduce_kernel, dim3(grid), dim3(256), 0u, st, (const float*)red.ws, red.S, red.M, N, red.C, ldc, epi,
             (const bf16_t*)bias, alpha, alpha_dev, alpha_dev2);
  return (int)hipGetLastError();
}

// A group of independent bf16 GEMMs in one launch (one grid over all their work units): the
// same operand modes for every member, fp32 C (epi 1 / 2), no bias, alpha = 1. Member i:
// A[i], B[i], C[i], dims[i] = {M, N, K, lda, ldb, ldc, epi, S}; ws[i] / cnt[i] for S > 1 as in
// ds2_gemm8 (separate ranges per member).
// opt (may be null): Adam + EMA applied in the epilogue instead of storing the gradient (every
// member epi 1, C a view of the gradient arena opt->gbase with element offset and ldc % 4 == 0)
int ds2_gemm8_group(int np, const void* const* A, const void* const* B, void* const* C, float* const* ws,
                    unsigned* const* cnt, const int* dims, int a_col, int b_col, int cus, const DS2G8Opt* opt,
                    hipStream_t st) {
  if (np <= 0 || np > G8_MAXP) return (int)hipErrorInvalidValue;
  G8Args a;
  a.opt = G8Opt{};
  a.fill = DS2Fill{};
  if (opt != nullptr && opt->on) {
    if (!a_col || !b_col) return (int)hipErrorInvalidValue;   // only that variant has the epilogue
    if (!opt->p || !opt->m || !opt->v || !opt->gbase) return (int)hipErrorInvalidValue;
    for (int i = 0; i < np; ++i) {
      const int* d = dims + 8 * i;
      const long long e0 = (const float*)C[i] - opt->gbase;
      if (d[6] != 1 || d[5] % 4 != 0 || e0 < 0 || e0 % 4 != 0) return (int)hipErrorInvalidValue;
    }
    a.opt = *opt;
  }
  a.bias = nullptr;
  a.alpha_dev = a.alpha_dev2 = nullptr;
  a.alpha = 1.f;
  a.np = np;
  a.ext_red = 0;
  int u = 0;
  for (int i = 0; i < np; ++i) {
    const int* d = dims + 8 * i;
    if (d[6] == 0) return (int)hipErrorInvalidValue;
    const int rc = fill_prob(a.p[i], A[i], B[i], C[i], ws[i], cnt[i], d[0], d[1], d[2], d[3], d[4], d[5], 0, a_col,
                             b_col, d[6], d[7], u);
    if (rc) return rc;
    u += units_of(a.p[i]);
  }
  a.total = u;
  return dispatch8(a, 0, a_col, b_col, cus, st);
}

// k-slices ds2_gemm8 actually uses for a requested S (no empty slice)
int ds2_gemm8_splits(int K, int fp8, int S) {
  const int nkt = (K * (fp8 ? 1 : 2) + ROWB - 1) / ROWB;
  const int kps = (nkt + S - 1) / S;
  return (nkt + kps - 1) / kps;
}

}  // extern "C"
