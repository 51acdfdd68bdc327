// DeepSpeech2 conv front-end for gfx950: implicit-GEMM convolutions on MFMA
// (v_mfma_f32_32x32x16_bf16) with channels-last activations, BatchNorm statistics fused
// into the forward epilogues, and channels-last BatchNorm + clipped-ReLU kernels.
//
// Reference graph (src/deepSpeech_NCHW.py:110-168, src/custom_ops.py:99-160):
//   conv1  [20x5] stride (2,2) VALID, 1 -> C   + bias + BN(train, eps 1e-3) + clip(0, 20)
//   conv2  [10x5] stride (2,1) VALID, C -> C   + bias + BN + clip
//   transpose/reshape to time-major [T2, N, C*F2]   (feature index c*F2 + f)
//
// Layouts (C = 32 channels, fixed: the reference's num_filters):
//   feats x0   [N][T][F0]            bf16 (F0 = 161)
//   conv1 y1   [N][T1][F1][C]        bf16, channels-last (F1 = 79)
//   conv2 in   z1 = clip(BN(y1))     same layout
//   conv2 y2   [N][T2][F2][C]        bf16, channels-last (F2 = 75)
//   rnn input  [T2][N][C*F2]         bf16, written by the BN apply through an LDS transpose
//   weights    OIHW bf16 shadows of the fp32 arena (w1 [C][1][20][5], w2 [C][C][10][5])
//
// MFMA mapping (32x32x16 bf16: lane l holds A[row l&31][k 8(l>>5)+j], B[k 8(l>>5)+j][col l&31],
// accumulator reg r -> row (r&3) + 8(r>>2) + 4(l>>5), col l&31):
//   conv2 fwd   rows = 32 output positions f2, cols = 32 co, k = (kt, kf, ci) in 100 k-steps of 16.
//               Persistent: each wave keeps ITS quarter of the weight fragments (25 k-steps) in
//               VGPRs for the whole launch; the 10 input rows of an output row (one contiguous
//               50.5 KB block) are double-buffered in LDS by global_load_lds (XOR-swizzled
//               16-B chunks -> conflict-free ds_read_b128); the 4 K-quarters are summed
//               through LDS in the epilogue, which also adds the bias, stores bf16 and
//               accumulates the BN batch statistics of the stored values.
//   conv2 dgrad rows = 32 input positions f1, cols = 32 ci, k = (kt, kf, co); a tile is the
//               output row pair (2u, 2u+1), whose kt parities read the same 5 rows of dy.
//   conv2 wgrad rows = co, cols = ci, k = positions; both operands are read with
//               ds_read_b64_tr_b16 (hardware transpose) from channels-last LDS images;
//               per-workgroup fp32 partials are summed by a reduce kernel into the arena.
//   conv1 fwd   rows = f1, cols = co, k = (kt, kf' in 0..7) (kf' >= 5 carry zero weights),
//               so a lane's 8 k-values are 8 consecutive input samples.
//   conv1 wgrad rows = co, cols = (kt, kf'), k = positions, input staged de-interleaved
//               (x[t][2p + kf'] as [t][kf'][p]) so the B fragment is one ds_read_b128.
//
// BatchNorm backward in training mode: dbeta = sum(dz*m), dgamma = sum(dz*m*xhat),
// dy = gamma*invstd*(dz*m - dbeta/M - xhat*dgamma/M), m = clip mask. The conv bias gradient
// is identically zero under train-mode BN (the mean subtraction cancels any shift).
#include "common.h"

using namespace ds2;

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4_t;

constexpr int CC = 32;          // channels
constexpr float CLIP = 20.0f;
constexpr int MT = 3;           // m-tiles of 32 positions (F1, F2 <= 96)

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// async 16-B global -> LDS copy; lds_wave_base must be wave-uniform (lane L lands at +16L)
__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

// byte offset of 16-B chunk c (0..3) of 64-B LDS position row R in the XOR-swizzled image
__device__ __forceinline__ unsigned swz(unsigned R, unsigned c) { return R * 64u + ((c ^ ((R >> 2) & 3u)) << 4); }

// transposed read: 4 rows x 16 columns of 16-bit elements per 16-lane group (T10)
__device__ __forceinline__ s16x4 tr_read(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p));
}

__device__ __forceinline__ bf16x8 cat8(s16x4 a, s16x4 b) {
  bf16x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// per-workgroup channel statistics: lanes l and l^32 hold the same channel (l & 31)
__device__ __forceinline__ void write_stats(float s, float q, float* sh /* [waves][32][2] */, int nwaves,
                                            float* part) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  s += __shfl_xor(s, 32, 64);
  q += __shfl_xor(q, 32, 64);
  __syncthreads();
  if (lane < 32) {
    sh[(w * 32 + lane) * 2 + 0] = s;
    sh[(w * 32 + lane) * 2 + 1] = q;
  }
  __syncthreads();
  if (tid < 64) {
    const int c = tid >> 1, k = tid & 1;
    float v = 0.f;
    for (int i = 0; i < nwaves; ++i) v += sh[(i * 32 + c) * 2 + k];
    part[(size_t)blockIdx.x * 64 + tid] = v;
  }
}

// =====================================================================================
// conv2 forward
// =====================================================================================
struct Conv2Fwd {
  const bf16_t* x;    // z1 [N][T1][F1][32]
  const bf16_t* w;    // [32][32][10][5]
  const float* bias;  // [32] or null
  bf16_t* y;          // [N][T2][F2][32]
  float* part;        // [grid][32][2]
  int N, T1, F1, T2, F2;
};
constexpr int C2_KT = 10, C2_KF = 5;
constexpr int C2_WAVES = 8;                     // 2 waves per SIMD: one's LDS reads hide under the other's MFMAs
constexpr int C2_KPW = 13;                      // k-steps per wave (100 = 4 x 13 + 4 x 12 for fwd)
constexpr int PR = 80;                          // LDS bytes per position row: 64 data + 16 pad
// With 80-B rows the 16 lanes of every ds_read_b128 lane group (consecutive positions, one
// 16-B chunk) hit 16 distinct 16-B bank slots: conflict-free with affine addresses, so each
// A-fragment read is one lane-base VGPR + a wave-uniform offset.
constexpr int C2_STG = 7;                       // 16-B staging loads per thread (512 threads)

// copy `nch` 16-B chunks of a contiguous run of 64-B position rows into 80-B LDS rows
struct Stager {
  i32x4 v[C2_STG];
  __device__ __forceinline__ void load(const unsigned char* src, int nch) {
#pragma unroll
    for (int k = 0; k < C2_STG; ++k) {
      const int p = min((int)threadIdx.x + 512 * k, nch - 1);     // clamp, never predicate a load
      v[k] = *(const i32x4*)(src + (size_t)p * 16);
    }
  }
  __device__ __forceinline__ void store(unsigned char* dst, int nch) const {
#pragma unroll
    for (int k = 0; k < C2_STG; ++k) {
      const int p = (int)threadIdx.x + 512 * k;
      if (p < nch) *(i32x4*)(dst + (p >> 2) * PR + (p & 3) * 16) = v[k];
    }
  }
};

// wave w's k-step range within a K of `total` steps split over `nw` waves (first waves +1)
__device__ __forceinline__ void kspan(int w, int nw, int total, int& s0, int& n) {
  const int q = total / nw, r = total % nw;
  n = q + (w < r ? 1 : 0);
  s0 = w * q + min(w, r);
}

__global__ __launch_bounds__(512) void conv2_fwd_kernel(Conv2Fwd a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  DS2_DCHECK(a.T2 == (a.T1 - C2_KT) / 2 + 1 && a.F2 == a.F1 - 4 && a.F1 <= 80);
  const int tid = threadIdx.x, lane = tid & 63, w = uni(tid >> 6);
  const int hi = lane >> 5, col = lane & 31;
  unsigned char* const buf = smem;                                   // [10*F1][80 B]
  f32x4* red = (f32x4*)(smem + C2_KT * a.F1 * PR);                   // [8 waves][12][64] f32x4
  int s0, nks;
  kspan(w, C2_WAVES, C2_KT * C2_KF * 2, s0, nks);

  bf16x8 bfr[C2_KPW];
#pragma unroll
  for (int i = 0; i < C2_KPW; ++i) {
    const int s = s0 + min(i, nks - 1);
    const int kt = s / 10, kf = (s % 10) >> 1, hh = s & 1;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ci = 16 * hh + 8 * hi + j;
      v[j] = (short)a.w[((col * CC + ci) * C2_KT + kt) * C2_KF + kf];
    }
    bfr[i] = v;
  }
  unsigned lb[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) lb[m] = (unsigned)(min(32 * m + col, a.F2 - 1) * PR + hi * 16);
  const float bco = a.bias ? a.bias[col] : 0.f;

  const int ntiles = a.N * a.T2;
  const int nch = C2_KT * a.F1 * 4;
  auto src_of = [&](int t) {
    const int n = t / a.T2, t2 = t - n * a.T2;
    return (const unsigned char*)(a.x + ((size_t)n * a.T1 + 2 * t2) * a.F1 * CC);
  };
  Stager stg;
  float ssum = 0.f, ssq = 0.f;
  if ((int)blockIdx.x < ntiles) {
    stg.load(src_of(blockIdx.x), nch);
    stg.store(buf, nch);
    if ((int)(blockIdx.x + gridDim.x) < ntiles) stg.load(src_of(blockIdx.x + gridDim.x), nch);
  }
  lds_barrier();
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    f32x16 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = (f32x16){};
    bf16x8 af[2][MT];
    auto ldA = [&](int i, bf16x8 (&dst)[MT]) {
      const int s = s0 + i;
      const unsigned off = (unsigned)(((s / 10) * a.F1 + ((s % 10) >> 1)) * PR + (s & 1) * 32);
#pragma unroll
      for (int m = 0; m < MT; ++m) dst[m] = *(const bf16x8*)(buf + lb[m] + off);
    };
    ldA(0, af[0]);
#pragma unroll
    for (int i = 0; i < C2_KPW; ++i) {
      if (i < nks) {                               // wave-uniform (only the last step varies)
        if (i + 1 < nks) ldA(i + 1, af[(i + 1) & 1]);
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = mfma32(af[i & 1][m], bfr[i], acc[m]);
      }
    }
    lds_barrier();                                   // every wave is done reading buf
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4)
        red[(w * 12 + m * 4 + r4) * 64 + lane] =
            (f32x4){acc[m][4 * r4], acc[m][4 * r4 + 1], acc[m][4 * r4 + 2], acc[m][4 * r4 + 3]};
    const int next = tile + gridDim.x;
    if (next < ntiles) stg.store(buf, nch);
    lds_barrier();
    if (next + (int)gridDim.x < ntiles) stg.load(src_of(next + gridDim.x), nch);
    const int n = tile / a.T2, t2 = tile - n * a.T2;
    bf16_t* yrow = a.y + ((size_t)n * a.T2 + t2) * a.F2 * CC;
    for (int item = tid; item < 12 * 64; item += 512) {   // (e = m*4 + r4, lane) items; channel = tid & 31
      const int e = item >> 6, l2 = item & 63, m = e >> 2, r4 = e & 3;
      f32x4 v = red[e * 64 + l2];
#pragma unroll
      for (int wv = 1; wv < C2_WAVES; ++wv) v += red[(wv * 12 + e) * 64 + l2];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int f2 = 32 * m + j + 8 * r4 + 4 * (l2 >> 5);
        if (f2 < a.F2) {
          const bf16_t b = f2bf(v[j] + bco);
          yrow[f2 * CC + col] = b;
          const float vb = bf2f(b);
          ssum += vb;
          ssq += vb * vb;
        }
      }
    }
    // red is rewritten only after the next tile's MFMA loop and its barrier
  }
  lds_barrier();
  write_stats(ssum, ssq, (float*)red, C2_WAVES, a.part);
}

// =====================================================================================
// conv2 data gradient: dx[n][t1][f1][ci] = sum dy[n][(t1-kt)/2][f1-kf][co] w[co][ci][kt][kf]
// =====================================================================================
struct Conv2Dgrad {
  const bf16_t* dy;   // [N][T2][F2][32]
  const bf16_t* w;    // [32][32][10][5]
  bf16_t* dx;         // [N][T1][F1][32]
  int N, T1, F1, T2, F2;
};
constexpr int C2D_STG = 3;                       // 16-B staging loads per thread (5 rows x F2 <= 76)

__global__ __launch_bounds__(512) void conv2_dgrad_kernel(Conv2Dgrad a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = uni(tid >> 6);
  const int hi = lane >> 5, col = lane & 31;
  const int par = w >> 2, wq = w & 3;            // waves 0-3: even output row, 4-7: odd
  unsigned char* const buf = smem;                                   // [5*F2][80 B]
  f32x4* red = (f32x4*)(smem + 5 * a.F2 * PR);                       // [8 waves][12][64]
  int s0, nks;
  kspan(wq, 4, C2_KT * C2_KF, s0, nks);          // 50 k-steps per parity

  bf16x8 bfr[C2_KPW];
#pragma unroll
  for (int i = 0; i < C2_KPW; ++i) {
    const int s = s0 + min(i, nks - 1);
    const int ai = s / 10, kf = (s % 10) >> 1, hh = s & 1;
    const int kt = 2 * ai + par;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int co = 16 * hh + 8 * hi + j;
      v[j] = (short)a.w[((co * CC + col) * C2_KT + kt) * C2_KF + kf];
    }
    bfr[i] = v;
  }
  const int U = (a.T1 + 1) >> 1;
  const int ntiles = a.N * U;
  const int nch = 5 * a.F2 * 4;
  const size_t rowEl = (size_t)a.F2 * CC;
  // rows u-4 .. u of dy (row slot j = row - (u-4)); rows outside [0, T2) are never read
  i32x4 stg[C2D_STG];
  auto load = [&](int t) {
    const int n = t / U, u = t - n * U;
    const bf16_t* base = a.dy + (size_t)n * a.T2 * rowEl;
#pragma unroll
    for (int k = 0; k < C2D_STG; ++k) {
      const int p = min(tid + 512 * k, nch - 1);
      const int row = min(max(u - 4 + (p >> 2) / a.F2, 0), a.T2 - 1);
      const int pos = (p >> 2) % a.F2;
      stg[k] = *(const i32x4*)(base + row * rowEl + pos * CC + (p & 3) * 8);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int k = 0; k < C2D_STG; ++k) {
      const int p = tid + 512 * k;
      if (p < nch) *(i32x4*)(buf + (p >> 2) * PR + (p & 3) * 16) = stg[k];
    }
  };
  if ((int)blockIdx.x < ntiles) {
    load(blockIdx.x);
    store();
    if ((int)(blockIdx.x + gridDim.x) < ntiles) load(blockIdx.x + gridDim.x);
  }
  lds_barrier();
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = tile / U, u = tile - n * U;
    f32x16 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = (f32x16){};
#pragma unroll
    for (int i = 0; i < C2_KPW; ++i) {
      const int s = s0 + i;
      const int ai = s / 10, kf = (s % 10) >> 1;
      const int t2 = u - ai;
      if (i < nks && t2 >= 0 && t2 < a.T2) {     // wave-uniform
        const int slotb = (4 - ai) * a.F2;
        bf16x8 av[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const int f2 = 32 * m + col - kf;
          const unsigned R = (unsigned)(slotb + min(max(f2, 0), a.F2 - 1));
          av[m] = *(const bf16x8*)(buf + R * PR + (s & 1) * 32 + hi * 16);
          if (!(f2 >= 0 && f2 < a.F2)) av[m] = (bf16x8){};
        }
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = mfma32(av[m], bfr[i], acc[m]);
      }
    }
    lds_barrier();
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4)
        red[(w * 12 + m * 4 + r4) * 64 + lane] =
            (f32x4){acc[m][4 * r4], acc[m][4 * r4 + 1], acc[m][4 * r4 + 2], acc[m][4 * r4 + 3]};
    const int next = tile + gridDim.x;
    if (next < ntiles) store();
    lds_barrier();
    if (next + (int)gridDim.x < ntiles) load(next + gridDim.x);
    for (int item = tid; item < 2 * 12 * 64; item += 512) {
      const int opar = item / 768, e = (item >> 6) % 12, l2 = item & 63, m = e >> 2, r4 = e & 3;
      const int t1 = 2 * u + opar;
      f32x4 v = red[((4 * opar) * 12 + e) * 64 + l2];
#pragma unroll
      for (int wv = 1; wv < 4; ++wv) v += red[((4 * opar + wv) * 12 + e) * 64 + l2];
      if (t1 < a.T1) {
        bf16_t* xrow = a.dx + ((size_t)n * a.T1 + t1) * a.F1 * CC;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int f1 = 32 * m + j + 8 * r4 + 4 * (l2 >> 5);
          if (f1 < a.F1) xrow[f1 * CC + (l2 & 31)] = f2bf(v[j]);
        }
      }
    }
  }
}

// =====================================================================================
// conv2 weight gradient (per-workgroup fp32 partials in fragment order)
// =====================================================================================
struct Conv2Wgrad {
  const bf16_t* dy;   // [N][T2][F2][32]
  const bf16_t* x;    // z1 [N][T1][F1][32]
  float* part;        // [grid][50][4][64][4]
  int N, T1, F1, T2, F2;
};
constexpr int C2W_PAIRS = C2_KT * C2_KF;   // 50 (kt, kf) output tiles of 32x32
constexpr int C2W_WAVES = 8;
constexpr int C2W_PPW = 7;                 // ceil(50 / 8)

__global__ __launch_bounds__(512) void conv2_wgrad_kernel(Conv2Wgrad a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = uni(tid >> 6);
  const int dyBytes = 80 * 64;
  const int xBytes = (9 * a.F1 + 84) * 64;         // covers row (kt*F1 + pos + kf) for pos < 80
  const int bufBytes = dyBytes + xBytes;
  unsigned char* const buf0 = smem;
  unsigned char* const buf1 = smem + bufBytes;
  // zero the pads that no copy writes: dy positions F2..79, x positions 10*F1 .. 9*F1+83
  for (int b = 0; b < 2; ++b) {
    unsigned char* bb = b ? buf1 : buf0;
    for (int o = a.F2 * 64 + tid * 4; o < dyBytes; o += 512 * 4) *(unsigned*)(bb + o) = 0u;
    for (int o = 10 * a.F1 * 64 + tid * 4; o < xBytes; o += 512 * 4) *(unsigned*)(bb + dyBytes + o) = 0u;
  }
  const int ntiles = a.N * a.T2;
  const int dyChunks = a.F2 * 4, xChunks = 10 * a.F1 * 4;
  auto issue = [&](int t, unsigned char* dst) {
    const int n = t / a.T2, t2 = t - n * a.T2;
    const unsigned char* sdy = (const unsigned char*)(a.dy + ((size_t)n * a.T2 + t2) * a.F2 * CC);
    const unsigned char* sx = (const unsigned char*)(a.x + ((size_t)n * a.T1 + 2 * t2) * a.F1 * CC);
    for (int p0 = w * 64; p0 < dyChunks; p0 += 512) {
      const int p = p0 + lane;
      if (p < dyChunks) glds16(sdy + (size_t)p * 16, dst + (size_t)p0 * 16);
    }
    for (int p0 = w * 64; p0 < xChunks; p0 += 512) {
      const int p = p0 + lane;
      if (p < xChunks) glds16(sx + (size_t)p * 16, dst + dyBytes + (size_t)p0 * 16);
    }
  };
  // transposed-read lane geometry
  const int g = lane >> 4, h = g >> 1, cb = (g & 1) * 16, q = (lane & 15) >> 2, pp = lane & 3;
  const unsigned lofs = (unsigned)((8 * h + q) * 64 + (cb + 4 * pp) * 2);
  const int npairs = (w < C2W_PAIRS - 6 * C2W_WAVES) ? 7 : 6;   // waves 0,1 take pairs 48,49

  f32x16 acc[C2W_PPW];
#pragma unroll
  for (int i = 0; i < C2W_PPW; ++i) acc[i] = (f32x16){};
  __syncthreads();
  int it = 0;
  if ((int)blockIdx.x < ntiles) issue(blockIdx.x, buf0);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
    const unsigned char* cur = (it & 1) ? buf1 : buf0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tile + (int)gridDim.x < ntiles) issue(tile + gridDim.x, (it & 1) ? buf0 : buf1);
    const unsigned char* xs = cur + dyBytes;
#pragma unroll
    for (int kk = 0; kk < 5; ++kk) {
      const unsigned k0 = (unsigned)(16 * kk) * 64u;
      const bf16x8 av = cat8(tr_read(cur + k0 + lofs), tr_read(cur + k0 + lofs + 4 * 64));
#pragma unroll
      for (int i = 0; i < C2W_PPW; ++i) {
        if (i < npairs) {
          const int P = w + C2W_WAVES * i;
          const int kt = P / 5, kf = P - 5 * (P / 5);
          const unsigned rb = (unsigned)(kt * a.F1 + kf) * 64u + k0 + lofs;
          const bf16x8 bv = cat8(tr_read(xs + rb), tr_read(xs + rb + 4 * 64));
          acc[i] = mfma32(av, bv, acc[i]);
        }
      }
    }
  }
  f32x4* out = (f32x4*)(a.part + (size_t)blockIdx.x * C2W_PAIRS * 1024);
#pragma unroll
  for (int i = 0; i < C2W_PPW; ++i) {
    if (i < npairs) {
      const int P = w + C2W_WAVES * i;
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4)
        out[(P * 4 + r4) * 64 + lane] = (f32x4){acc[i][4 * r4], acc[i][4 * r4 + 1], acc[i][4 * r4 + 2], acc[i][4 * r4 + 3]};
    }
  }
}

// sum of per-workgroup partials (fragment order) -> dw in OIHW, KIND 0: conv2 [32][32][10][5],
// KIND 1: conv1 [32][1][20][5]. A block owns 256 consecutive elements (64 f32x4 columns)
// and 4 interleaved groups of partials, so every thread keeps several 16-B loads in flight.
template <int KIND>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int nb, int E,
                                                           float* __restrict__ dw) {
  __shared__ f32x4 sh[4][64];
  const int tid = threadIdx.x, g = tid >> 6, l = tid & 63;
  const int e4 = blockIdx.x * 64 + l, E4 = E >> 2;
  const f32x4* p4 = (const f32x4*)part;
  f32x4 s0 = {}, s1 = {};
  int b = g;
  for (; b + 4 < nb; b += 8) {
    s0 += p4[(size_t)b * E4 + e4];
    s1 += p4[(size_t)(b + 4) * E4 + e4];
  }
  if (b < nb) s0 += p4[(size_t)b * E4 + e4];
  sh[g][l] = s0 + s1;
  __syncthreads();
  if (g != 0) return;
  const f32x4 v = sh[0][l] + sh[1][l] + sh[2][l] + sh[3][l];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = e4 * 4 + j;
    const int P = e >> 10, rem = e & 1023, r4 = rem >> 8, ln = (rem >> 2) & 63;
    const int row = (rem & 3) + 8 * r4 + 4 * (ln >> 5), c = ln & 31;
    if (KIND == 0) {
      const int kt = P / 5, kf = P % 5;
      dw[((row * CC + c) * C2_KT + kt) * C2_KF + kf] = v[j];
    } else {
      const int kt = 4 * P + (c >> 3), kf = c & 7;
      if (kf < 5) dw[(row * 20 + kt) * 5 + kf] = v[j];
    }
  }
}

// =====================================================================================
// conv1 forward (C_in = 1)
// =====================================================================================
struct Conv1Fwd {
  const bf16_t* x;    // [N][T][F0]
  const bf16_t* w;    // [32][1][20][5]
  const float* bias;  // [32] or null
  bf16_t* y;          // [N][T1][F1][32]
  float* part;        // [grid][32][2]
  int N, T, F0, T1, F1;
};
constexpr int C1_KT = 20, C1_KF = 5;
constexpr int C1_XS = 200;     // staged row stride (elements): covers 2*95 + 7
constexpr int C1_ROWS = 4;     // output rows per workgroup (one per wave)
constexpr int C1_IN = 2 * (C1_ROWS - 1) + C1_KT;   // 26 input rows

// stage input rows t0 .. t0+C1_IN-1 of one utterance ([T][F0] bf16, rows 2-B aligned only) into
// LDS rows of C1_XS elements, zero outside the utterance / beyond F0. Loads are unconditional
// (clamped addresses) so all of them are in flight together; the select happens afterwards.
__device__ __forceinline__ void stage_rows(bf16_t* xs, const bf16_t* xu, int t0, int T, int F0) {
  constexpr int NE = C1_IN * C1_XS, K = (NE + 255) / 256;
  bf16_t v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int idx = min((int)threadIdx.x + 256 * k, NE - 1);
    const int r = idx / C1_XS, c = idx - r * C1_XS;
    v[k] = xu[(size_t)min(t0 + r, T - 1) * F0 + min(c, F0 - 1)];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int idx = (int)threadIdx.x + 256 * k;
    const int r = idx / C1_XS, c = idx - r * C1_XS;
    if (idx < NE) xs[idx] = (t0 + r < T && c < F0) ? v[k] : (bf16_t)0;
  }
}

__global__ __launch_bounds__(256) void conv1_fwd_kernel(Conv1Fwd a) {
  __shared__ __attribute__((aligned(16))) bf16_t xs[C1_IN * C1_XS];
  __shared__ float statsh[4 * 32 * 2];
  const int tid = threadIdx.x, lane = tid & 63, w = uni(tid >> 6);
  const int hi = lane >> 5, col = lane & 31;
  const int tb = (a.T1 + C1_ROWS - 1) / C1_ROWS;
  const int n = blockIdx.x / tb, t1_0 = (blockIdx.x - n * tb) * C1_ROWS;
  stage_rows(xs, a.x + (size_t)n * a.T * a.F0, 2 * t1_0, a.T, a.F0);
  bf16x8 bfr[10];
#pragma unroll
  for (int s = 0; s < 10; ++s) {
    const int kt = 2 * s + hi;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = j < C1_KF ? (short)a.w[(col * C1_KT + kt) * C1_KF + j] : (short)0;
    bfr[s] = v;
  }
  const float bco = a.bias ? a.bias[col] : 0.f;
  __syncthreads();
  float ssum = 0.f, ssq = 0.f;
  const int t1 = t1_0 + w;
  if (t1 < a.T1) {
    f32x16 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = (f32x16){};
#pragma unroll
    for (int s = 0; s < 10; ++s) {
      const int r = 2 * w + 2 * s + hi;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const unsigned* p = (const unsigned*)(xs + r * C1_XS + 2 * (32 * m + col));
        const unsigned u0 = p[0], u1 = p[1], u2 = p[2], u3 = p[3];
        const bf16x8 av = __builtin_bit_cast(bf16x8, (i32x4){(int)u0, (int)u1, (int)u2, (int)u3});
        acc[m] = mfma32(av, bfr[s], acc[m]);
      }
    }
    bf16_t* yrow = a.y + ((size_t)n * a.T1 + t1) * a.F1 * CC;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int f1 = 32 * m + (r & 3) + 8 * (r >> 2) + 4 * hi;
        if (f1 < a.F1) {
          const bf16_t b = f2bf(acc[m][r] + bco);
          yrow[f1 * CC + col] = b;
          const float vb = bf2f(b);
          ssum += vb;
          ssq += vb * vb;
        }
      }
  }
  write_stats(ssum, ssq, statsh, 4, a.part);
}

// =====================================================================================
// conv1 weight gradient
// =====================================================================================
struct Conv1Wgrad {
  const bf16_t* dy;   // [N][T1][F1][32]
  const bf16_t* x;    // [N][T][F0]
  float* part;        // [grid][5][4][64][4]
  int N, T, F0, T1, F1;
};
constexpr int C1W_XP = 88;                       // de-interleaved row stride (positions)
constexpr int C1W_DY = C1_ROWS * 80 * 64;        // dy image bytes (4 rows x 80 positions)
constexpr int C1W_XD = C1_IN * 8 * C1W_XP * 2;   // x image bytes
constexpr int C1W_RED = 4 * 5 * 4 * 64 * 16;     // wave partials
constexpr int C1W_RAW = C1_IN * C1_XS * 2;             // raw input rows
constexpr int C1W_SMEM = (C1W_DY + C1W_XD + C1W_RAW) > C1W_RED ? (C1W_DY + C1W_XD + C1W_RAW) : C1W_RED;

__global__ __launch_bounds__(256) void conv1_wgrad_kernel(Conv1Wgrad a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = uni(tid >> 6);
  const int hi = lane >> 5, col = lane & 31;
  unsigned char* dys = smem;
  bf16_t* xd = (bf16_t*)(smem + C1W_DY);
  bf16_t* raw = (bf16_t*)(smem + C1W_DY + C1W_XD);
  const int tb = (a.T1 + C1_ROWS - 1) / C1_ROWS;
  const int ntiles = a.N * tb;
  const int g = lane >> 4, h = g >> 1, cb = (g & 1) * 16, q = (lane & 15) >> 2, pp = lane & 3;
  const unsigned lofs = (unsigned)((8 * h + q) * 64 + (cb + 4 * pp) * 2);
  const int bkt = col >> 3, bkf = col & 7;

  f32x16 acc[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) acc[i] = (f32x16){};
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int n = tile / tb, t1_0 = (tile - n * tb) * C1_ROWS;
    __syncthreads();   // previous tile's reads done
    // dy rows t1_0 .. t1_0+3 -> [row][80][32] (positions >= F1 zero)
    for (int ch = tid; ch < C1_ROWS * 80 * 4; ch += 256) {
      const int r = ch / 320, rem = ch - r * 320, pos = rem >> 2, c4 = rem & 3;
      const int t1 = t1_0 + r;
      i32x4 v = (i32x4){0, 0, 0, 0};
      if (pos < a.F1 && t1 < a.T1)
        v = *(const i32x4*)(a.dy + (((size_t)n * a.T1 + t1) * a.F1 + pos) * CC + c4 * 8);
      *(i32x4*)(dys + ch * 16) = v;
    }
    // x rows 2*t1_0 + r: raw rows into LDS, then de-interleaved xd[r][kf'][p] = x[t][2p + kf']
    stage_rows(raw, a.x + (size_t)n * a.T * a.F0, 2 * t1_0, a.T, a.F0);
    __syncthreads();
    for (int ch = tid; ch < C1_IN * 8 * 10; ch += 256) {
      const int r = ch / 80, rem = ch - r * 80, kf = rem / 10, p0 = (rem - kf * 10) * 8;
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (short)raw[r * C1_XS + min(2 * (p0 + j) + kf, C1_XS - 1)];
      *(bf16x8*)(xd + (r * 8 + kf) * C1W_XP + p0) = v;
    }
    __syncthreads();
    const int t1 = t1_0 + w;
    if (t1 < a.T1) {
#pragma unroll
      for (int kk = 0; kk < 5; ++kk) {
        const unsigned k0 = (unsigned)(16 * kk);
        const unsigned char* ab = dys + (w * 80 + k0) * 64 + lofs;
        const bf16x8 av = cat8(tr_read(ab), tr_read(ab + 4 * 64));
#pragma unroll
        for (int nt = 0; nt < 5; ++nt) {
          const int r = 2 * w + 4 * nt + bkt;
          const bf16x8 bv = *(const bf16x8*)(xd + (r * 8 + bkf) * C1W_XP + k0 + 8 * hi);
          acc[nt] = mfma32(av, bv, acc[nt]);
        }
      }
    }
  }
  __syncthreads();
  f32x4* red = (f32x4*)smem;
#pragma unroll
  for (int nt = 0; nt < 5; ++nt)
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4)
      red[((w * 5 + nt) * 4 + r4) * 64 + lane] =
          (f32x4){acc[nt][4 * r4], acc[nt][4 * r4 + 1], acc[nt][4 * r4 + 2], acc[nt][4 * r4 + 3]};
  __syncthreads();
  f32x4* out = (f32x4*)(a.part + (size_t)blockIdx.x * 5 * 1024);
  for (int e = tid; e < 5 * 4 * 64; e += 256) {
    f32x4 v = red[e];
    for (int wv = 1; wv < 4; ++wv) v += red[wv * 5 * 4 * 64 + e];
    out[e] = v;
  }
}

// =====================================================================================
// channels-last BatchNorm (+ clipped ReLU)
// =====================================================================================
// part [nb][32][2] -> mean / invstd (+ running stats, unbiased variance, momentum)
__global__ __launch_bounds__(256) void bn_cl_finalize_kernel(const float* __restrict__ part, int nb, double M,
                                                             float eps, float* mean, float* invstd, float* run_mean,
                                                             float* run_var, float momentum) {
  __shared__ double sh[2][4];
  const int c = blockIdx.x, tid = threadIdx.x;
  double s = 0.0, q = 0.0;
  for (int b = tid; b < nb; b += 256) {
    s += part[((size_t)b * 32 + c) * 2 + 0];
    q += part[((size_t)b * 32 + c) * 2 + 1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    q += __shfl_xor(q, o, 64);
  }
  if ((tid & 63) == 0) { sh[0][tid >> 6] = s; sh[1][tid >> 6] = q; }
  __syncthreads();
  if (tid == 0) {
    s = sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3];
    q = sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3];
    const double mu = s / M;
    double var = q / M - mu * mu;
    if (var < 0) var = 0;
    if (mean) mean[c] = (float)mu;
    if (invstd) invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
    if (run_mean) {
      const double unb = M > 1 ? var * M / (M - 1) : var;
      run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * mu);
      run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * unb);
    }
  }
}

// z = clip(y * sc + sh) elementwise, channels-last in and out (8 channels per thread)
__global__ __launch_bounds__(256) void bn_cl_apply_kernel(const bf16_t* __restrict__ y, const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, bf16_t* __restrict__ z,
                                                          long long nchunks) {
  const int c0 = (threadIdx.x & 3) * 8;     // 256 % 4 == 0: a thread keeps its channel octet
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = invstd[c0 + j] * gamma[c0 + j];
    sh[j] = beta[c0 + j] - mean[c0 + j] * sc[j];
  }
  for (long long ch = (long long)blockIdx.x * 256 + threadIdx.x; ch < nchunks; ch += (long long)gridDim.x * 256) {
    const bf16x8 v = *(const bf16x8*)(y + ch * 8);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (short)f2bf(fminf(fmaxf(bf2f((bf16_t)v[j]) * sc[j] + sh[j], 0.f), CLIP));
    *(bf16x8*)(z + ch * 8) = o;
  }
}

// rows (n, t) of F positions x 32 channels; time-major output out[t][n][c*F + f]
__global__ __launch_bounds__(256) void bn_cl_apply_tmaj_kernel(const bf16_t* __restrict__ y,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta,
                                                               bf16_t* __restrict__ out, int N, int T, int F) {
  __shared__ bf16_t tr[32 * 97];            // [c][f], stride F+? (F <= 96)
  const int tid = threadIdx.x, c0 = (tid & 3) * 8;
  const int stride = F + 1;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = invstd[c0 + j] * gamma[c0 + j];
    sh[j] = beta[c0 + j] - mean[c0 + j] * sc[j];
  }
  for (int row = blockIdx.x; row < N * T; row += gridDim.x) {
    const int n = row / T, t = row - n * T;
    const bf16_t* yr = y + (size_t)row * F * CC;
    __syncthreads();
    for (int ch = tid; ch < F * 4; ch += 256) {
      const int f = ch >> 2;
      const bf16x8 v = *(const bf16x8*)(yr + ch * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        tr[(c0 + j) * stride + f] = f2bf(fminf(fmaxf(bf2f((bf16_t)v[j]) * sc[j] + sh[j], 0.f), CLIP));
    }
    __syncthreads();
    bf16_t* orow = out + ((size_t)t * N + n) * CC * F;
    for (int e = tid; e < CC * F; e += 256) {
      const int c = e / F, f = e - c * F;
      orow[e] = tr[c * stride + f];
    }
  }
}

// backward reduce over rows: sums of dz*m and dz*m*xhat per channel; dz either channels-
// last (tmaj == 0) or time-major [T][N][c*F + f] (tmaj == 1)
__global__ __launch_bounds__(256) void bn_cl_bwd_reduce_kernel(const bf16_t* __restrict__ dz,
                                                               const bf16_t* __restrict__ y,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, float* part,
                                                               int N, int T, int F, int tmaj,
                                                               bf16_t* __restrict__ dz_cl) {
  __shared__ bf16_t tr[32 * 97];
  const int tid = threadIdx.x, c0 = (tid & 3) * 8;
  float mu[8], is[8], g[8], bt[8], s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = mean[c0 + j]; is[j] = invstd[c0 + j]; g[j] = gamma[c0 + j]; bt[j] = beta[c0 + j];
    s[j] = 0.f; q[j] = 0.f;
  }
  const int stride = F + 1;
  for (int row = blockIdx.x; row < N * T; row += gridDim.x) {
    const int n = row / T, t = row - n * T;
    const bf16_t* yr = y + (size_t)row * F * CC;
    if (tmaj) {
      __syncthreads();
      const bf16_t* dr = dz + ((size_t)t * N + n) * CC * F;
      for (int e = tid; e < CC * F; e += 256) {
        const int c = e / F, f = e - c * F;
        tr[c * stride + f] = dr[e];
      }
      __syncthreads();
    }
    for (int ch = tid; ch < F * 4; ch += 256) {
      const int f = ch >> 2;
      const bf16x8 v = *(const bf16x8*)(yr + ch * 8);
      bf16x8 d;
      if (tmaj) {
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = (short)tr[(c0 + j) * stride + f];
        // the transposed (channels-last) copy, so the apply pass reads it coalesced
        if (dz_cl != nullptr) *(bf16x8*)(dz_cl + (size_t)row * F * CC + ch * 8) = d;
      } else {
        d = *(const bf16x8*)(dz + (size_t)row * F * CC + ch * 8);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (bf2f((bf16_t)v[j]) - mu[j]) * is[j];
        const float zz = xh * g[j] + bt[j];
        const float dd = (zz > 0.f && zz < CLIP) ? bf2f((bf16_t)d[j]) : 0.f;
        s[j] += dd;
        q[j] += dd * xh;
      }
    }
  }
  // reduce over the 64 threads sharing a channel octet (tid & 3)
  __syncthreads();
  float* red = (float*)tr;   // [4 waves][4 octets][8] floats, reused per pass
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    float* v = pass == 0 ? s : q;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      // threads with equal (tid & 3): lanes differ in bits 2..5 within a wave
      float x = v[j];
      x += __shfl_xor(x, 4, 64);
      x += __shfl_xor(x, 8, 64);
      x += __shfl_xor(x, 16, 64);
      x += __shfl_xor(x, 32, 64);
      v[j] = x;
    }
    __syncthreads();
    if ((tid & 63) < 4) {
#pragma unroll
      for (int j = 0; j < 8; ++j) red[((tid >> 6) * 4 + (tid & 3)) * 8 + j] = v[j];
    }
    __syncthreads();
    if (tid < 32) {
      const int oc = tid >> 3, j = tid & 7;    // channel = oc*8 + j
      float x = 0.f;
      for (int wv = 0; wv < 4; ++wv) x += red[(wv * 4 + oc) * 8 + j];
      part[((size_t)blockIdx.x * 32 + tid) * 2 + pass] = x;
    }
  }
}

// part [nb][32][2] -> dbeta, dgamma (fp32)
__global__ __launch_bounds__(256) void bn_cl_bwd_finalize_kernel(const float* __restrict__ part, int nb,
                                                                 float* dbeta, float* dgamma) {
  __shared__ double sh[2][4];
  const int c = blockIdx.x, tid = threadIdx.x;
  double s = 0.0, q = 0.0;
  for (int b = tid; b < nb; b += 256) {
    s += part[((size_t)b * 32 + c) * 2 + 0];
    q += part[((size_t)b * 32 + c) * 2 + 1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    q += __shfl_xor(q, o, 64);
  }
  if ((tid & 63) == 0) { sh[0][tid >> 6] = s; sh[1][tid >> 6] = q; }
  __syncthreads();
  if (tid == 0) {
    dbeta[c] = (float)(sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3]);
    dgamma[c] = (float)(sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3]);
  }
}

// dy = gamma*invstd*(dz*m - dbeta/M - xhat*dgamma/M), channels-last out. dz may alias dy
// (each thread reads and writes the same 16 B), so neither is __restrict__.
__global__ __launch_bounds__(256) void bn_cl_bwd_apply_kernel(const bf16_t* dz,
                                                              const bf16_t* __restrict__ y,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta,
                                                              const float* __restrict__ dbeta,
                                                              const float* __restrict__ dgamma,
                                                              bf16_t* dy, int N, int T, int F, int tmaj) {
  __shared__ bf16_t tr[32 * 97];
  const int tid = threadIdx.x, c0 = (tid & 3) * 8;
  const float M = (float)N * T * F;
  float mu[8], is[8], g[8], bt[8], mdb[8], mdg[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = mean[c0 + j]; is[j] = invstd[c0 + j]; g[j] = gamma[c0 + j]; bt[j] = beta[c0 + j];
    mdb[j] = dbeta[c0 + j] / M; mdg[j] = dgamma[c0 + j] / M;
  }
  const int stride = F + 1;
  for (int row = blockIdx.x; row < N * T; row += gridDim.x) {
    const int n = row / T, t = row - n * T;
    const bf16_t* yr = y + (size_t)row * F * CC;
    if (tmaj) {
      __syncthreads();
      const bf16_t* dr = dz + ((size_t)t * N + n) * CC * F;
      for (int e = tid; e < CC * F; e += 256) {
        const int c = e / F, f = e - c * F;
        tr[c * stride + f] = dr[e];
      }
      __syncthreads();
    }
    for (int ch = tid; ch < F * 4; ch += 256) {
      const int f = ch >> 2;
      const bf16x8 v = *(const bf16x8*)(yr + ch * 8);
      bf16x8 d;
      if (tmaj) {
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = (short)tr[(c0 + j) * stride + f];
      } else {
        d = *(const bf16x8*)(dz + (size_t)row * F * CC + ch * 8);
      }
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (bf2f((bf16_t)v[j]) - mu[j]) * is[j];
        const float zz = xh * g[j] + bt[j];
        const float dd = (zz > 0.f && zz < CLIP) ? bf2f((bf16_t)d[j]) : 0.f;
        o[j] = (short)f2bf(g[j] * is[j] * (dd - mdb[j] - xh * mdg[j]));
      }
      *(bf16x8*)(dy + (size_t)row * F * CC + ch * 8) = o;
    }
  }
}

template <typename K>
int set_smem(K kernel, size_t bytes) {
  return (int)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)bytes);
}

int shape_ok(int T1, int F1, int T2, int F2) {
  if (F1 < 5 || F1 > 80 || F2 != F1 - 4) return -40;   // LDS (10*F1*80 + 96 KiB) and staging capacity
  if (T1 < 10 || T2 != (T1 - 10) / 2 + 1) return -41;
  return 0;
}

}  // namespace

extern "C" {

size_t ds2_conv2_fwd_smem(int F1) { return (size_t)C2_KT * F1 * PR + C2_WAVES * 12 * 64 * 16; }
size_t ds2_conv2_dgrad_smem(int F2) { return (size_t)5 * F2 * PR + C2_WAVES * 12 * 64 * 16; }
size_t ds2_conv2_wgrad_smem(int F1) { return (size_t)2 * (80 * 64 + (9 * F1 + 84) * 64); }
long long ds2_conv2_wgrad_part_floats(int grid) { return (long long)grid * C2W_PAIRS * 1024; }
long long ds2_conv1_wgrad_part_floats(int grid) { return (long long)grid * 5 * 1024; }
int ds2_conv1_fwd_grid(int N, int T1) { return N * ((T1 + C1_ROWS - 1) / C1_ROWS); }

int ds2_conv2_fwd(const void* x, const void* w, const float* bias, void* y, float* part, int grid, int N, int T1,
                  int F1, int T2, int F2, hipStream_t st) {
  if (int e = shape_ok(T1, F1, T2, F2)) return e;
  const size_t smem = ds2_conv2_fwd_smem(F1);
  DS2_HIP_CHECK((hipError_t)set_smem(conv2_fwd_kernel, smem));
  Conv2Fwd a{(const bf16_t*)x, (const bf16_t*)w, bias, (bf16_t*)y, part, N, T1, F1, T2, F2};
  hipLaunchKernelGGL(conv2_fwd_kernel, dim3(grid), dim3(512), smem, st, a);
  return (int)hipGetLastError();
}

int ds2_conv2_dgrad(const void* dy, const void* w, void* dx, int grid, int N, int T1, int F1, int T2, int F2,
                    hipStream_t st) {
  if (int e = shape_ok(T1, F1, T2, F2)) return e;
  const size_t smem = ds2_conv2_dgrad_smem(F2);
  DS2_HIP_CHECK((hipError_t)set_smem(conv2_dgrad_kernel, smem));
  Conv2Dgrad a{(const bf16_t*)dy, (const bf16_t*)w, (bf16_t*)dx, N, T1, F1, T2, F2};
  hipLaunchKernelGGL(conv2_dgrad_kernel, dim3(grid), dim3(512), smem, st, a);
  return (int)hipGetLastError();
}

int ds2_conv2_wgrad(const void* dy, const void* x, float* part, int grid, float* dw, int N, int T1, int F1, int T2,
                    int F2, hipStream_t st) {
  if (int e = shape_ok(T1, F1, T2, F2)) return e;
  const size_t smem = ds2_conv2_wgrad_smem(F1);
  DS2_HIP_CHECK((hipError_t)set_smem(conv2_wgrad_kernel, smem));
  Conv2Wgrad a{(const bf16_t*)dy, (const bf16_t*)x, part, N, T1, F1, T2, F2};
  hipLaunchKernelGGL(conv2_wgrad_kernel, dim3(grid), dim3(512), smem, st, a);
  hipLaunchKernelGGL(wgrad_reduce_kernel<0>, dim3(C2W_PAIRS * 1024 / 256), dim3(256), 0, st, part, grid,
                     C2W_PAIRS * 1024, dw);
  return (int)hipGetLastError();
}

int ds2_conv1_fwd(const void* x, const void* w, const float* bias, void* y, float* part, int N, int T, int F0,
                  int T1, int F1, hipStream_t st) {
  if (F1 > 96 || F1 != (F0 - 5) / 2 + 1 || T1 != (T - 20) / 2 + 1 || T1 < 1) return -42;
  Conv1Fwd a{(const bf16_t*)x, (const bf16_t*)w, bias, (bf16_t*)y, part, N, T, F0, T1, F1};
  hipLaunchKernelGGL(conv1_fwd_kernel, dim3(ds2_conv1_fwd_grid(N, T1)), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

int ds2_conv1_wgrad(const void* dy, const void* x, float* part, int grid, float* dw, int N, int T, int F0, int T1,
                    int F1, hipStream_t st) {
  if (F1 > 80 || F1 != (F0 - 5) / 2 + 1 || T1 != (T - 20) / 2 + 1 || T1 < 1) return -43;
  DS2_HIP_CHECK((hipError_t)set_smem(conv1_wgrad_kernel, C1W_SMEM));
  Conv1Wgrad a{(const bf16_t*)dy, (const bf16_t*)x, part, N, T, F0, T1, F1};
  hipLaunchKernelGGL(conv1_wgrad_kernel, dim3(grid), dim3(256), C1W_SMEM, st, a);
  hipLaunchKernelGGL(wgrad_reduce_kernel<1>, dim3(5 * 1024 / 256), dim3(256), 0, st, part, grid, 5 * 1024, dw);
  return (int)hipGetLastError();
}

int ds2_bn_cl_finalize(const float* part, int nb, double M, float eps, float* mean, float* invstd, float* run_mean,
                       float* run_var, float momentum, hipStream_t st) {
  hipLaunchKernelGGL(bn_cl_finalize_kernel, dim3(CC), dim3(256), 0, st, part, nb, M, eps, mean, invstd, run_mean,
                     run_var, momentum);
  return (int)hipGetLastError();
}

int ds2_bn_cl_apply(const void* y, const float* mean, const float* invstd, const float* gamma, const float* beta,
                    void* out, int N, int T, int F, int tmaj, hipStream_t st) {
  if (F > 96) return -44;
  if (tmaj) {
    const int rows = N * T;
    hipLaunchKernelGGL(bn_cl_apply_tmaj_kernel, dim3(rows < 4096 ? rows : 4096), dim3(256), 0, st, (const bf16_t*)y,
                       mean, invstd, gamma, beta, (bf16_t*)out, N, T, F);
  } else {
    const long long nch = (long long)N * T * F * 4;
    long long nb = (nch + 255) / 256;
    if (nb > 8192) nb = 8192;
    hipLaunchKernelGGL(bn_cl_apply_kernel, dim3((unsigned)nb), dim3(256), 0, st, (const bf16_t*)y, mean, invstd,
                       gamma, beta, (bf16_t*)out, nch);
  }
  return (int)hipGetLastError();
}

int ds2_bn_cl_bwd(const void* dz, const void* y, const float* mean, const float* invstd, const float* gamma,
                  const float* beta, float* part, int nb, float* dgamma, float* dbeta, void* dy, int N, int T, int F,
                  int tmaj, hipStream_t st) {
  if (F > 96) return -45;
  // time-major dz: the reduce pass (which transposes it through LDS anyway) leaves a
  // channels-last copy in dy, and the apply pass then works in place on dy, coalesced
  // (the apply's own per-row LDS transpose ran at ~1/9 of the bandwidth roofline)
  hipLaunchKernelGGL(bn_cl_bwd_reduce_kernel, dim3(nb), dim3(256), 0, st, (const bf16_t*)dz, (const bf16_t*)y, mean,
                     invstd, gamma, beta, part, N, T, F, tmaj, tmaj ? (bf16_t*)dy : (bf16_t*)nullptr);
  hipLaunchKernelGGL(bn_cl_bwd_finalize_kernel, dim3(CC), dim3(256), 0, st, part, nb, dbeta, dgamma);
  const int rows = N * T;
  hipLaunchKernelGGL(bn_cl_bwd_apply_kernel, dim3(rows < 4096 ? rows : 4096), dim3(256), 0, st,
                     tmaj ? (const bf16_t*)dy : (const bf16_t*)dz, (const bf16_t*)y, mean, invstd, gamma, beta,
                     dbeta, dgamma, (bf16_t*)dy, N, T, F, 0);
  return (int)hipGetLastError();
}

}  // extern "C"
