// Hand-written MFMA GEMM family for the recurrent layers' projection / gradient GEMMs and
// their fused epilogues (gfx950, v_mfma_f32_16x16x32_bf16, bf16 in, fp32 accumulate).
//
// Reference call sites (src/custom_ops.py:59-67, src/deepSpeech_NCHW.py:188-198): the
// per-step W.x_t of CustomRNNCell2 hoisted over all T2 steps of both directions, and its
// autograd counterparts. One kernel template, two operand layouts per side:
//
//   C[m][n] = epi( sum_k A(m,k) B(n,k) )
//     A row ("R"): A(m,k) = A[m*lda + k]   (K contiguous)       B row: B(n,k) = B[n*ldb + k]
//     A col ("C"): A(m,k) = A[k*lda + m]   (M contiguous)       B col: B(n,k) = B[k*ldb + n]
//
//   forward projection  gx = alpha * x W^T + b      A row (x [T*N][D]),   B row (W [6H][D])
//   input gradient      dx = dgx W                  A row (dgx [T*N][6H]), B col (W as [K=6H][N=D])
//   weight gradients    dW = dgx^T x, dU = dgh^T h  A col, B col          (fp32 into the arena)
//
// Structure (cdna_hip_programming.md §5): BK = 64 k-tiles staged global -> LDS with
// global_load_lds_dwordx4 into two LDS buffers (the load of tile t+1 is in flight while
// tile t is read and multiplied), one vmcnt(0) + barrier per k-tile.
//   * row images: [rows][64 k] with 128-B rows, 16-B chunk c stored at c ^ ((r>>1)&7) —
//     conflict-free ds_read_b128 for the 16x16x32 operand (16 rows x one chunk per lane group);
//   * col images: [64 k][W] (W >= 128 columns), 16-B chunk c of k-row k stored at
//     c ^ 2*((k&3) | ((k>>1)&4)) — the 32-lane halves of ds_read_b64_tr_b16 (rows 8 apart,
//     two chunks each) hit 16 distinct slots. The swizzle goes on the per-lane SOURCE
//     address; glds writes lane-linear (rule 21).
//   * operands swapped in the MFMA (D' = B.A^T = C^T), so each lane ends with 4 CONSECUTIVE
//     columns of one C row: one 8-B (bf16) or 16-B (fp32) store per fragment, with the bias
//     as one vector load.
//   * blockIdx -> tile through the bijective XCD remap (T1): a run of tiles sharing an A row
//     block stays on one XCD's L2.
// Tails: K % 8 == 0; a last 64-tile with K % 32 != 0 gets its k >= K part zeroed in LDS
// (a 32-deep half past K is skipped); rows/columns past M/N are clamped on load and masked
// on store; col-mode operands need their M/N % 8 == 0.
#include "common.h"

using namespace ds2;

namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4_t;

constexpr int BK = 64;

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  const bf16_t* bias;     // [N] bf16 (epi 0) or null
  const float* alpha_dev;  // optional device scalar multiplied into alpha (no host sync)
  long long sA, sB, sC;   // batch strides (elements)
  int M, N, K, lda, ldb, ldc;
  int Ml, Nl, Kl;         // load limits (>= M/N/K for col-mode operands padded in memory; Kl <= K
                          // for a col-mode operand whose k-rows past Kl multiply zeros)
  int epi;                // 0: bf16 = alpha*acc + bias; 1: fp32 = alpha*acc; 2: fp32 += alpha*acc
  float alpha;
  DS2Fill fill;           // persistent configurations: regions the lighter workgroups initialise
};

__device__ __forceinline__ void glds16(const void* g, unsigned char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ unsigned rsw(int r) { return (unsigned)((r >> 1) & 7); }
__device__ __forceinline__ unsigned csw(int k) { return (unsigned)(2 * ((k & 3) | ((k >> 1) & 4))); }

// Stage a [ROWS x 64k] row image (ROWMODE) or a [64k x ROWS] col image of one operand.
//   row image: G(r, k) = P[(r0+r)*ld + k0+k]      (r < ROWS, rows clamped to < lim)
//   col image: G(r, k) = P[(k0+k)*ld + r0+r]      (k clamped to < K, columns to < lim)
template <bool COLMODE, int ROWS, int NW>
__device__ __forceinline__ void stage(unsigned char* img, const bf16_t* P, int ld, int r0, int lim, int k0, int K,
                                      int wave, int lane) {
  constexpr int NINS = ROWS / 8;                   // 1-KB wave-instructions per image
  if constexpr (!COLMODE) {
#pragma unroll
    for (int i0 = 0; i0 < NINS; i0 += NW) {
      const int i = i0 + wave;
      if (NINS % NW == 0 || i < NINS) {
        const int r = 8 * i + (lane >> 3), p = lane & 7;
        const int c = p ^ (int)rsw(r);
        const int gr = min(r0 + r, lim - 1);
        const int gk = min(k0 + 8 * c, K - 8);
        glds16(P + (size_t)gr * ld + gk, img + i * 1024);
      }
    }
  } else {
    constexpr int CPR = ROWS / 8;                  // 16-B chunks per k-row
    constexpr int RPI = 64 / CPR;                  // k-rows per wave-instruction
#pragma unroll
    for (int i0 = 0; i0 < NINS; i0 += NW) {
      const int i = i0 + wave;
      if (NINS % NW == 0 || i < NINS) {
        const int kr = RPI * i + lane / CPR, p = lane % CPR;
        const int c = p ^ (int)csw(kr);
        const int gk = min(k0 + kr, K - 1);
        const int gc = min(r0 + 8 * c, lim - 8);
        glds16(P + (size_t)gk * ld + gc, img + i * 1024);
      }
    }
  }
}

// Zero the k >= kval part of a staged image (last k-tile of a K that is not a multiple of 64):
// the clamped tail loads hold real (finite or not) data that must not enter the products.
template <bool COLMODE, int ROWS, int NTH>
__device__ __forceinline__ void zero_ktail(unsigned char* img, int kval, int tid) {
  const i32x4 z = {0, 0, 0, 0};
  if constexpr (!COLMODE) {
    // [ROWS][8 chunks]: logical chunk c (k = 8c..8c+7) of row r sits at position c ^ rsw(r)
    for (int q = tid; q < ROWS * 8; q += NTH) {
      const int r = q >> 3, pos = q & 7;
      const int c = pos ^ (int)rsw(r);
      if (8 * c >= kval) *(i32x4*)(img + r * 128 + pos * 16) = z;
    }
  } else {
    // [64 k-rows][ROWS columns]: whole k-rows
    constexpr int CPR = ROWS / 8;
    for (int q = kval * CPR + tid; q < 64 * CPR; q += NTH) *(i32x4*)(img + q * 16) = z;
  }
}

// one 16x32 operand fragment (rows rb*16.., k-substep ks) from a staged image
template <bool COLMODE, int ROWS>
__device__ __forceinline__ bf16x8 frag(const unsigned char* img, int rb, int ks, int lane) {
  if constexpr (!COLMODE) {
    const int r = rb * 16 + (lane & 15);
    const int c = ks * 4 + (lane >> 4);
    return *(const bf16x8*)(img + r * 128 + ((c ^ (int)rsw(r)) << 4));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int m = rb * 16 + 4 * p;
    const int c = m >> 3;
    const int k0 = ks * 32 + 8 * g + q;
    const unsigned char* b0 = img + k0 * (ROWS * 2) + ((c ^ (int)csw(k0)) << 4) + 8 * (p & 1);
    const unsigned char* b1 = img + (k0 + 4) * (ROWS * 2) + ((c ^ (int)csw(k0 + 4)) << 4) + 8 * (p & 1);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)b0);
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)b1);
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = orig & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (orig >> 3);
}

// vmcnt-only wait with a compile-time count (expcnt / lgkmcnt left at "no wait")
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}

// One tile's C-store: lane (row mb + 16i, columns nb + 16j .. +3). Buffer stores with an
// exact per-lane count (rows / columns past M / N get an out-of-range offset and are dropped
// by the resource's bounds check), so a persistent workgroup can count vmcnt across it.
template <int FM, int FN>
__device__ __forceinline__ void store_tile(const GemmArgs& g, const f32x4 (&acc)[FN][FM], const float (&bv)[FN][4],
                                           float alpha, int mb, int nb) {
  const size_t esz = g.epi == 0 ? 2 : 4;
  const size_t cbytes = (size_t)g.M * g.ldc * esz;
  char* Cz = (char*)g.C + (size_t)blockIdx.z * g.sC * esz;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(Cz, (unsigned)min(cbytes, (size_t)0xFFFFFFF0u));
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = nb + j * 16;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = mb + i * 16;
      const unsigned off = (m < g.M && n < g.N) ? (unsigned)(((size_t)m * g.ldc + n) * esz) : 0xFFFFFFF0u;
      const f32x4 v = acc[j][i];
      if (g.epi == 0) {
        const unsigned lo = (unsigned)f2bf(alpha * v[0] + bv[j][0]) | ((unsigned)f2bf(alpha * v[1] + bv[j][1]) << 16);
        const unsigned hi = (unsigned)f2bf(alpha * v[2] + bv[j][2]) | ((unsigned)f2bf(alpha * v[3] + bv[j][3]) << 16);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned,
                                                                 make_uint2(lo, hi)), rs, off, 0, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned,
                               make_float4(alpha * v[0], alpha * v[1], alpha * v[2], alpha * v[3])), rs, off, 0, 0);
      }
    }
  }
}

// PERS: persistent grid (one workgroup per CU, a multiple of 8): XCD x = blockIdx % 8 owns the
// contiguous tile-id range [x*Tx, (x+1)*Tx) of the grouped order and its workgroups stride
// through it. At a tile seam the next tile's first NS-1 LDS stages go out BEFORE this tile's
// C stores, so the next prologue's load latency hides under the epilogue (the per-tile fixed
// cost was ~1/3 of the K = 800 projection). epi 2 (read-modify-write) is not persistent.
template <int AC, int BC, int FM, int FN, int WM, int WN, int NS, bool PERS>
__global__ __launch_bounds__(WM * WN * 64) void gemm_kernel(GemmArgs g) {
  constexpr int NW = WM * WN, BM = WM * FM * 16, BN = WN * FN * 16;
  constexpr int A_BYTES = BM * BK * 2, STAGE_BYTES = (BM + BN) * BK * 2;
  static_assert(!AC || BM >= 128, "col-mode A image needs >= 128 columns");
  static_assert(!BC || BN >= 128, "col-mode B image needs >= 128 columns");
  static_assert((BM / 8) % NW == 0 && (BN / 8) % NW == 0, "every wave issues the same glds count");
  static_assert(NS == 2 || NS == 3, "2 or 3 LDS stages");
  constexpr int LPW = (BM / 8) / NW + (BN / 8) / NW;   // glds per wave per stage (vmcnt unit)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int ntm = (g.M + BM - 1) / BM, ntn = (g.N + BN - 1) / BN;
  // Tile order: the XCD remap gives every XCD a contiguous run of ids, and ids run through
  // groups of GROUP_M m-tiles x all n-tiles with m fastest, so the ~32 tiles an XCD holds at
  // once form a GROUP_M x (32/GROUP_M) block whose A rows and B columns share that XCD's L2
  // (row-major tile order streamed all of B through every XCD: MALL-bound, 25 % MFMA busy).
  constexpr int GROUP_M = 8;
  int id, id_end, id_step;
  if constexpr (PERS) {
    const int total = ntm * ntn, tx = (total + 7) >> 3, x = blockIdx.x & 7;
    id = x * tx + (blockIdx.x >> 3);
    id_end = min(total, (x + 1) * tx);
    id_step = gridDim.x >> 3;
  } else {
    id = xcd_remap(blockIdx.x, gridDim.x);
    id_end = id + 1;
    id_step = 1;
  }
  auto coords = [&](int t, int& m0_, int& n0_) -> bool {
    const int gsz = GROUP_M * ntn;
    const int grp = t / gsz, first_m = grp * GROUP_M;
    const int gm = min(ntm - first_m, GROUP_M);
    if (gm <= 0) return false;
    const int within = t - grp * gsz;
    m0_ = (first_m + within % gm) * BM;
    n0_ = (within / gm) * BN;
    return true;
  };
  int m0, n0;
  if (id >= id_end || !coords(id, m0, n0)) {
    if constexpr (PERS) {
      if (g.fill.n > 0) fill_idle(g.fill, ntm * ntn, (ntm * ntn + 7) >> 3, NW * 64);
    }
    return;
  }
  const bf16_t* A = g.A + (size_t)blockIdx.z * g.sA;
  const bf16_t* B = g.B + (size_t)blockIdx.z * g.sB;
  const int tid = threadIdx.x, lane = tid & 63, wave = uni(tid >> 6);
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int K = g.K;
  const int nkt = (K + BK - 1) / BK;
  const float alpha = g.alpha_dev ? g.alpha * *g.alpha_dev : g.alpha;

  f32x4 acc[FN][FM];
  auto stage_all = [&](int buf, int kt, int mm0, int nn0) {
    unsigned char* base = smem + buf * STAGE_BYTES;
    stage<AC != 0, BM, NW>(base, A, g.lda, mm0, g.Ml, kt * BK, AC ? g.Kl : K, wave, lane);
    stage<BC != 0, BN, NW>(base + A_BYTES, B, g.ldb, nn0, g.Nl, kt * BK, BC ? g.Kl : K, wave, lane);
  };

  // Pipeline (cdna_hip_programming.md §5 'Pipelining across barriers'), NS LDS stages:
  //   iteration kt:  glds tile kt+NS-1 | read half 1 of tile kt | MFMA half 0 of kt
  //                  counted vmcnt (tile kt+1 landed) + raw barrier
  //                  read half 0 of tile kt+1 | MFMA half 1 of kt
  // so every fragment read is in flight under the other half's MFMAs and tile kt+2's loads
  // stay in flight across the barrier (no __syncthreads: its fence would drain them).
  // WAR: the buffer refilled at iteration kt held tile kt-1, whose last reads were retired
  // by the lgkmcnt(0) of iteration kt-1's barrier.
  auto kvalid = [&](int t) { return min(BK, K - t * BK); };
  auto prep = [&](int t, unsigned char* base) {   // ragged last tile: zero k >= kval, re-sync
    const int kv = kvalid(t);
    if (kv < BK && (kv & 31)) {
      zero_ktail<AC != 0, BM, NW * 64>(base, kv, tid);
      zero_ktail<BC != 0, BN, NW * 64>(base + A_BYTES, kv, tid);
      lds_barrier();
    }
  };
  bf16x8 af0[FM], bf0[FN], af1[FM], bf1[FN];
  auto read_half = [&](const unsigned char* base, int ks, bf16x8 (&af)[FM], bf16x8 (&bfr)[FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = frag<AC != 0, BM>(base, wm * FM + i, ks, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[j] = frag<BC != 0, BN>(base + A_BYTES, wn * FN + j, ks, lane);
  };
  auto mfma_half = [&](const bf16x8 (&af)[FM], const bf16x8 (&bfr)[FN]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i)
        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[j][i], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto prologue_issue = [&](int mm0, int nn0) {
    stage_all(0, 0, mm0, nn0);
    if (NS == 3 && nkt > 1) stage_all(1, 1, mm0, nn0);
  };

  prologue_issue(m0, n0);
  bool first = true;
  while (true) {
    // stage 0 landed: behind it are stage 1 (NS = 3) and, after a seam, the previous tile's
    // FM*FN C stores (vmcnt counts stores too and retires in order)
    if (first) {
      if (NS == 3 && nkt > 1) wait_vm<LPW>();
      else wait_vm<0>();
    } else {
      if (NS == 3 && nkt > 1) wait_vm<LPW + FM * FN>();
      else wait_vm<FM * FN>();
    }
    first = false;
    lds_barrier();
    // this tile's bias columns, loaded now so their latency hides under the k-loop
    // (unconditional, clamped loads: a conditional load gets a vmcnt(0) right behind it)
    const int nb = n0 + wn * FN * 16 + 4 * (lane >> 4);
    const bool has_bias = g.epi == 0 && g.bias != nullptr;
    const bf16_t* bsrc = has_bias ? g.bias : B;
    uint2 braw[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) braw[j] = *(const uint2*)(bsrc + min(nb + j * 16, g.N - 4));
    prep(0, smem);
    read_half(smem, 0, af0, bf0);
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    int buf = 0;
    for (int kt = 0; kt < nkt; ++kt) {
      const bool more = kt + NS - 1 < nkt;
      if (more) {
        const int nb = buf + NS - 1;
        stage_all(nb >= NS ? nb - NS : nb, kt + NS - 1, m0, n0);
      }
      unsigned char* cur = smem + buf * STAGE_BYTES;
      const bool half2 = kvalid(kt) > 32;
      if (half2) read_half(cur, 1, af1, bf1);
      mfma_half(af0, bf0);
      const int nxt = (buf + 1 == NS) ? 0 : buf + 1;
      if (kt + 1 < nkt) {
        if (NS == 3 && more) wait_vm<LPW>();
        else wait_vm<0>();
        lds_barrier();
        prep(kt + 1, smem + nxt * STAGE_BYTES);
        read_half(smem + nxt * STAGE_BYTES, 0, af0, bf0);
      }
      if (half2) mfma_half(af1, bf1);
      buf = nxt;
    }

    // epilogue: acc[j][i][e] = C[m][n + e], m = row of A fragment lane&15, n = 4 consecutive
    const int mb = m0 + wm * FM * 16 + (lane & 15);
    float bv[FN][4];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const uint2 b2 = braw[j];
      const float on = has_bias ? 1.f : 0.f;
      bv[j][0] = on * bf2f((bf16_t)(b2.x & 0xffff)); bv[j][1] = on * bf2f((bf16_t)(b2.x >> 16));
      bv[j][2] = on * bf2f((bf16_t)(b2.y & 0xffff)); bv[j][3] = on * bf2f((bf16_t)(b2.y >> 16));
    }
    if constexpr (PERS) {
      const int nid = id + id_step;
      int nm0 = 0, nn0 = 0;
      const bool next = nid < id_end && coords(nid, nm0, nn0);
      if (next) {
        lds_barrier();                 // every wave's last fragment reads of this tile retired
        prologue_issue(nm0, nn0);      // next tile's loads fly under this tile's stores
      }
      store_tile<FM, FN>(g, acc, bv, alpha, mb, nb);
      if (!next) break;
      id = nid;
      m0 = nm0;
      n0 = nn0;
      continue;
    } else {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = nb + j * 16;
        if (n >= g.N) continue;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int m = mb + i * 16;
          if (m >= g.M) continue;
          const f32x4 v = acc[j][i];
          if (g.epi == 0) {
            bf16_t* C = (bf16_t*)g.C + (size_t)blockIdx.z * g.sC + (size_t)m * g.ldc + n;
            const unsigned lo = (unsigned)f2bf(alpha * v[0] + bv[j][0]) | ((unsigned)f2bf(alpha * v[1] + bv[j][1]) << 16);
            const unsigned hi = (unsigned)f2bf(alpha * v[2] + bv[j][2]) | ((unsigned)f2bf(alpha * v[3] + bv[j][3]) << 16);
            *(uint2*)C = make_uint2(lo, hi);
          } else {
            float* C = (float*)g.C + (size_t)blockIdx.z * g.sC + (size_t)m * g.ldc + n;
            float4 o = make_float4(alpha * v[0], alpha * v[1], alpha * v[2], alpha * v[3]);
            if (g.epi == 2) {
              const float4 c = *(const float4*)C;
              o.x += c.x; o.y += c.y; o.z += c.z; o.w += c.w;
            }
            *(float4*)C = o;
          }
        }
      }
      break;
    }
  }
  if constexpr (PERS) {
    if (g.fill.n > 0) fill_idle(g.fill, ntm * ntn, (ntm * ntn + 7) >> 3, NW * 64);
  }
}

template <int AC, int BC, int FM, int FN, int WM, int WN, int NS, bool PERS = false>
int launch(const GemmArgs& a, int batch, hipStream_t st) {
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  const int lds = (BM + BN) * BK * 2 * NS;
  auto kern = gemm_kernel<AC, BC, FM, FN, WM, WN, NS, PERS>;
  static bool attr = false;
  if (!attr) {
    DS2_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr = true;
  }
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  int grid = tiles;
  if (PERS) {
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      DS2_HIP_CHECK(hipGetDevice(&dev));
      DS2_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    grid = min(cus, (tiles + 7) & ~7);          // one workgroup per CU (>= 96 KB of LDS), x8 for the XCD map
    grid = max(8, grid & ~7);
  }
  ds2_launch(kern, dim3(grid, 1, batch), dim3(WM * WN * 64), (unsigned)lds, st, a);
  return (int)hipGetLastError();
}

// tile configurations (BM x BN, waves, LDS stages):
//   0 = 256x256 8w 2st (128 KB)   1 = 128x256 8w 3st (144 KB)   2 = 256x128 8w 3st (144 KB)
//   3 = 128x128 4w 2st (64 KB, 2 per CU)   4 = 128x128 4w 3st (96 KB)   5 = 128x128 8w 3st (96 KB)
//   6/7/8 = persistent 0/1/2 (epilogue overlapped with the next tile's loads; epi 0/1 only)
constexpr int NCFG = 9;
template <int AC, int BC>
int dispatch(const GemmArgs& a, int batch, int cfg, hipStream_t st) {
  if (cfg >= 6 && a.epi == 2) return (int)hipErrorInvalidValue;
  switch (cfg) {
    case 0: return launch<AC, BC, 8, 4, 2, 4, 2>(a, batch, st);
    case 1: return launch<AC, BC, 4, 4, 2, 4, 3>(a, batch, st);
    case 2: return launch<AC, BC, 4, 4, 4, 2, 3>(a, batch, st);
    case 3: return launch<AC, BC, 4, 4, 2, 2, 2>(a, batch, st);
    case 4: return launch<AC, BC, 4, 4, 2, 2, 3>(a, batch, st);
    case 5: return launch<AC, BC, 2, 4, 4, 2, 3>(a, batch, st);
    case 6: return launch<AC, BC, 8, 4, 2, 4, 2, true>(a, batch, st);
    case 7: return launch<AC, BC, 4, 4, 2, 4, 3, true>(a, batch, st);
    case 8: return launch<AC, BC, 4, 4, 4, 2, 3, true>(a, batch, st);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace

extern "C" {

int ds2_multi_fill(int n, void* const* ptrs, const unsigned long long* bytes, const unsigned* patterns,
                   hipStream_t st);

// Returns the tile (BM, BN) of configuration cfg, or -1.
int ds2_gemm_tile(int cfg, int* bm, int* bn) {
  static const int T[NCFG][2] = {{256, 256}, {128, 256}, {256, 128}, {128, 128}, {128, 128}, {128, 128},
                                 {256, 256}, {128, 256}, {256, 128}};
  if (cfg < 0 || cfg >= NCFG) return -1;
  *bm = T[cfg][0];
  *bn = T[cfg][1];
  return 0;
}

// Ml/Nl/Kl: load limits (0 = M/N/K). A col-mode operand may be padded in memory to Ml >= M
// columns (Ml % 8 == 0 required instead of M % 8); k-rows of a col-mode operand at or past Kl
// re-read row Kl-1 (their products must meet zeros in the other operand).
int ds2_gemm(const void* A, const void* B, void* C, const void* bias, const float* alpha_dev, int M, int N, int K,
             int lda, int ldb, int ldc, int Ml, int Nl, int Kl, int a_col, int b_col, int epi, float alpha, int batch,
             long long sA, long long sB, long long sC, int cfg, const DS2Fill* fill, hipStream_t st) {
  Ml = Ml ? Ml : M;
  Nl = Nl ? Nl : N;
  Kl = Kl ? Kl : K;
  // K: any length for col-mode operands; a row-mode operand's rows are read in 16-B chunks
  if (((!a_col || !b_col) && K % 8 != 0) || N % 4 != 0 || M <= 0 || N <= 0 || K <= 0 || batch <= 0)
    return (int)hipErrorInvalidValue;
  if (Ml < M || Nl < N || Kl > K || Kl <= 0) return (int)hipErrorInvalidValue;
  if ((a_col && Ml % 8) || (b_col && Nl % 8)) return (int)hipErrorInvalidValue;
  if (Kl != K && !a_col && !b_col) return (int)hipErrorInvalidValue;   // Kl clamps col-mode operands only
  GemmArgs a;
  a.alpha_dev = alpha_dev;
  a.Ml = Ml; a.Nl = Nl; a.Kl = Kl;
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = C;
  a.bias = (const bf16_t*)bias;
  a.sA = sA; a.sB = sB; a.sC = sC;
  a.M = M; a.N = N; a.K = K;
  a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.epi = epi;
  a.alpha = alpha;
  a.fill = DS2Fill{};
  // the persistent single-GEMM configurations fill from their lighter workgroups; any other
  // launch is followed by the plain fill kernel
  const bool fused_fill = fill != nullptr && fill->n > 0 && cfg >= 6 && batch == 1;
  if (fused_fill) a.fill = *fill;
  // an armed stop event belongs to the op's last launch: the plain fill kernel when one follows
  const bool tail_fill = fill != nullptr && fill->n > 0 && !fused_fill;
  hipEvent_t stop = tail_fill ? ds2_take_stop_event() : nullptr;
  int rc;
  if (!a_col && !b_col) rc = dispatch<0, 0>(a, batch, cfg, st);
  else if (!a_col && b_col) rc = dispatch<0, 1>(a, batch, cfg, st);
  else if (a_col && b_col) rc = dispatch<1, 1>(a, batch, cfg, st);
  else rc = dispatch<1, 0>(a, batch, cfg, st);
  if (rc == 0 && fill != nullptr && fill->n > 0 && !fused_fill) {
    unsigned long long bytes[8];
    for (int i = 0; i < fill->n; ++i) bytes[i] = fill->words[i] * 4;
    ds2_arm_stop_event(stop);
    rc = ds2_multi_fill(fill->n, (void* const*)fill->ptr, bytes, fill->pattern, st);
  } else if (stop != nullptr) {
    ds2_arm_stop_event(stop);          // not launched: left armed for the caller to see
  }
  return rc;
}

}  // extern "C"
