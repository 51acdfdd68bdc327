// Persistent bidirectional recurrence (ReLU-RNN and reset-after GRU) for gfx950.
//
// Reference behaviour: src/custom_ops.py:36-96 (CustomRNNCell2 + stacked_brnn via
// tf.nn.bidirectional_dynamic_rnn: zero outputs past each length, backward direction
// reversed within each utterance, directions summed by the caller).
//
// Design (MI355X-first):
//  * The input projection W.x for all T steps is a separate library GEMM; this kernel
//    runs only the serial part: gh = U.h_{t-1} + gates, for BOTH directions at once.
//  * Grid = ndir x BG x S workgroups. A workgroup owns 16 hidden units ("slice") of one
//    direction for 16*MT batch rows; its slice of U (all G gates, 16 rows x H) lives in
//    VGPRs for the whole sequence as MFMA B fragments. K (=H) is split across the NW
//    waves and reduced through LDS.
//  * The fp32 recurrent state of the workgroup's (rows x units) tile is register
//    resident (each thread owns its elements across all steps); only the bf16 copy used
//    as the next step's MFMA operand is exchanged.
//  * Exchange between workgroups of a (direction, batch-group) uses write-through (sc1)
//    16-B stores of h_t, an s_waitcnt vmcnt(0) drain, and one per-workgroup flag stored
//    with an agent-scope atomic; consumers poll the flags with sc1 loads and read h_t
//    with sc1 buffer loads (MI355X_MICROARCH.md, inter-workgroup visibility, valid form
//    row 1: no release/acquire fences on the critical path).
//  * Every spin is bounded (s_memrealtime timeout) and sets an error word, so a grid
//    that is not fully resident cannot hang the GPU.
//  * Step mode: the same kernel launched once per step (s_end = s_begin + 1) needs no
//    co-residency; it is the fallback and the numerics cross-check of the persistent path.
//
// Buffers (step-indexed = processing order, time-indexed = utterance time):
//   gx   [T, N, gstride] bf16  time-indexed input projection, direction d at column d*G*H
//   hx   [steps+1, NP, H] bf16 step-indexed exchange; slot 0 = h0, slot s+1 = h after step s
//   hsave[steps+1, NP, H] fp32 step-indexed state (backward + step-mode carry)
//   gates[steps, NP, H, 4] fp32 (GRU: r, z, n, U_n h + b_hn)
//   y    [T, N, H] bf16 time-indexed output per direction
//   dgh  [steps, NP, G*H] bf16 step-indexed gradient of the recurrent pre-activation
//   dgx  [T, N, gstride] bf16 time-indexed gradient of the input projection
#include "common.h"

using namespace ds2;

namespace {

constexpr int CELL_RELU = 0;
constexpr int CELL_GRU = 1;
constexpr float RELU_CAP = 20.0f;

struct FwdArgs {
  int T, N, NP, H, S, BG, steps, s_begin, s_end, gstride;
  const int* lens;
  const bf16_t* gx;
  const bf16_t* U[2];
  const float* bh[2];
  bf16_t* y[2];
  bf16_t* hx[2];
  float* hsave[2];
  float* gates[2];
  unsigned* flags;
  unsigned* err;
  long long timeout;
  unsigned long long* stamps;
};

struct BwdArgs {
  int T, N, NP, H, S, BG, steps, s_begin, s_end, gstride;
  const int* lens;
  const bf16_t* dy;
  const bf16_t* U[2];
  const float* hsave[2];
  const float* gates[2];
  bf16_t* dgh[2];
  bf16_t* dgx;
  float* carry[2];
  float* dbx_part[2];   // [BG, G*H] per direction: sum of dgx over steps and rows (input bias grad)
  float* dbh_part[2];   // [BG, G*H] per direction: sum of dgh (GRU recurrent bias grad)
  float dgx_scale;      // dgx is stored pre-multiplied (frozen sequence-BN scale folded in)
  unsigned* flags;
  unsigned* err;
  long long timeout;
  unsigned long long* stamps;
};

// Diagnostic build (rnn_persistent_stamps.hip): per-phase s_memtime cycle sums per
// workgroup, recorded by wave 0 (cdna_hip_programming.md §7 "In-kernel stamps"). The
// production build compiles every STAMP away.
#ifdef DS2_RNN_STAMPS
#define DS2_STAMP_DECL unsigned long long st_prev = 0, st_acc[6] = {0, 0, 0, 0, 0, 0};
#define DS2_STAMP(i)                                                                      \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    unsigned long long _t;                                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    if (st_prev) st_acc[i] += _t - st_prev;                                               \
    st_prev = _t;                                                                         \
  } while (0)
#define DS2_STAMP_STORE(a)                                                                \
  do {                                                                                    \
    if (threadIdx.x == 0 && (a).stamps)                                                   \
      for (int _k = 0; _k < 6; ++_k) (a).stamps[blockIdx.x * 8 + _k] = st_acc[_k];        \
  } while (0)
#define DS2_EXPORT(name) name##_stamps
#else
#define DS2_STAMP_DECL
#define DS2_STAMP(i)
#define DS2_STAMP_STORE(a)
#define DS2_EXPORT(name) name
#endif

// Wait until every workgroup of the group published iteration `need`-1.
// Returns false on timeout (error word set).  Executed by wave 0 only.
__device__ __forceinline__ bool wait_group(const unsigned* f, int S, unsigned need, int lane,
                                           long long timeout, unsigned* err) {
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  while (true) {
    bool ok = true;
    for (int q = lane; q < S; q += 64) ok = ok && (ld_flag(f + q) >= need);
    if (__all(ok)) return true;
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
      if (lane == 0) atomicOr(err, 1u);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

template <int CELL, int NW, int MT, int KPW>
__global__ __launch_bounds__(NW * 64) void rnn_fwd_kernel(FwdArgs a) {
  constexpr int G = (CELL == CELL_GRU) ? 3 : 1;
  constexpr int NT = NW * 64;
  constexpr int ROWS = 16 * MT;
  constexpr int NE = ROWS * 16;                 // tile elements
  constexpr int EPT = (NE + NT - 1) / NT;       // elements per thread

  __shared__ float red[NW][ROWS][G * 16];
  __shared__ __attribute__((aligned(16))) bf16_t stage[ROWS][16];
  __shared__ int abort_flag;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int S = a.S;
  const int slice = blockIdx.x % S;
  const int grp = blockIdx.x / S;
  const int bg = grp % a.BG, dir = grp / a.BG;
  const int r0 = bg * ROWS, u0 = slice * 16;
  const int H = a.H, KS = H / 32;
  const int N = a.N, NP = a.NP;

  if (tid == 0) abort_flag = 0;

  // ---- resident U fragments: B[k][c] = U[g*H + u0 + c][k] --------------------------
  bf16x8 uf[KPW][G];
  const bf16_t* Ud = a.U[dir];
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    const int ks = wave + kk * NW;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (ks < KS) {
        const bf16_t* p = Ud + (size_t)(g * H + u0 + (lane & 15)) * H + ks * 32 + 8 * (lane >> 4);
        uf[kk][g] = *reinterpret_cast<const bf16x8*>(p);
      } else {
        uf[kk][g] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
  }

  // ---- per-thread elements -----------------------------------------------------------
  float hreg[EPT];
  int lenr[EPT];
  float bhv[EPT][G];
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int e = tid + i * NT;
    const int row = e >> 4, c = e & 15;
    const int b = r0 + row, u = u0 + c;
    hreg[i] = 0.f;
    lenr[i] = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) bhv[i][g] = 0.f;
    if (e < NE) {
      hreg[i] = a.hsave[dir][((size_t)a.s_begin * NP + b) * H + u];
      lenr[i] = (b < N) ? a.lens[b] : 0;
      if (CELL == CELL_GRU && a.bh[dir] != nullptr) {
#pragma unroll
        for (int g = 0; g < G; ++g) bhv[i][g] = a.bh[dir][g * H + u];
      }
    }
  }

  const unsigned hx_bytes = (unsigned)((size_t)(a.steps + 1) * NP * H * 2);
  const __amdgpu_buffer_rsrc_t rs_hx = make_rsrc(a.hx[dir], hx_bytes);
  const unsigned* gflags = a.flags + grp * S;
  __syncthreads();
  DS2_STAMP_DECL

  for (int s = a.s_begin; s < a.s_end; ++s) {
    DS2_STAMP(5);
    // (1) prefetch this step's input projection (independent of the recurrence)
    float gxv[EPT][G];
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tid + i * NT;
      const int row = e >> 4, c = e & 15;
      const int b = r0 + row, u = u0 + c;
      const bool act = (e < NE) && (s < lenr[i]);
      const int t = (dir == 0) ? s : (lenr[i] - 1 - s);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        gxv[i][g] = act ? bf2f(a.gx[((size_t)t * N + b) * a.gstride + dir * G * H + g * H + u]) : 0.f;
      }
    }

    // (2) wait for every slice of h_{s-1}
    if (s > a.s_begin) {
      if (wave == 0) {
        if (!wait_group(gflags, S, (unsigned)(s - a.s_begin), lane, a.timeout, a.err)) {
          if (lane == 0) abort_flag = 1;
        }
      }
      __syncthreads();
      if (abort_flag) break;
    }
    DS2_STAMP(0);

    // (3) gh = h_{s-1} . U^T over this wave's k-steps
    f32x4 acc[MT][G];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int g = 0; g < G; ++g) acc[m][g] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
      bf16x8 af[MT][KPW];
#pragma unroll
      for (int kk = 0; kk < KPW; ++kk) {
        const int ks = wave + kk * NW;
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          if (ks < KS) {
            const unsigned off = (unsigned)((((size_t)s * NP + r0 + m * 16 + (lane & 15)) * H +
                                             ks * 32 + 8 * (lane >> 4)) * 2);
            af[m][kk] = __builtin_bit_cast(bf16x8, load_sc1_b128(rs_hx, off));
          }
        }
      }
#pragma unroll
      for (int kk = 0; kk < KPW; ++kk) {
        const int ks = wave + kk * NW;
        if (ks < KS) {
#pragma unroll
          for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int g = 0; g < G; ++g)
              acc[m][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m][kk], uf[kk][g], acc[m][g], 0, 0, 0);
        }
      }
    }

    DS2_STAMP(1);
    // (4) cross-wave reduction through LDS
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          red[wave][m * 16 + (lane >> 4) * 4 + j][g * 16 + (lane & 15)] = acc[m][g][j];
    __syncthreads();

    DS2_STAMP(2);
    // (5) cell epilogue: only the bf16 exchange copy is written before the publish
    float hout[EPT];
    float4 gsv[EPT];
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tid + i * NT;
      hout[i] = 0.f;
      gsv[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < NE) {
        const int row = e >> 4, c = e & 15;
        float pre[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
          float v = 0.f;
#pragma unroll
          for (int w = 0; w < NW; ++w) v += red[w][row][g * 16 + c];
          pre[g] = v;
        }
        const bool act = s < lenr[i];
        float hn;
        if (CELL == CELL_GRU) {
          const float ghr = pre[0] + bhv[i][0];
          const float ghz = pre[1] + bhv[i][1];
          const float ghn = pre[2] + bhv[i][2];
          const float r = sigmoidf_(gxv[i][0] + ghr);
          const float z = sigmoidf_(gxv[i][1] + ghz);
          const float n = tanhf_(gxv[i][2] + r * ghn);
          hn = (1.f - z) * n + z * hreg[i];
          if (act) gsv[i] = make_float4(r, z, n, ghn);
        } else {
          hn = fminf(fmaxf(gxv[i][0] + pre[0], 0.f), RELU_CAP);
        }
        const float hnew = act ? hn : hreg[i];
        hreg[i] = hnew;
        hout[i] = act ? hn : 0.f;
        stage[row][c] = f2bf(hnew);
      }
    }
    __syncthreads();
    DS2_STAMP(3);

    // (6) publish h_s: write-through 16-B stores, drain, one flag per workgroup
    if (wave == 0) {
      for (int q = lane; q < ROWS * 2; q += 64) {
        const int row = q >> 1, half = q & 1;
        const i32x4 v = *reinterpret_cast<const i32x4*>(&stage[row][half * 8]);
        const unsigned off = (unsigned)((((size_t)(s + 1) * NP + r0 + row) * H + u0 + half * 8) * 2);
        store_sc1_b128(rs_hx, off, v);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) st_flag(a.flags + grp * S + slice, (unsigned)(s - a.s_begin + 1));
    }

    DS2_STAMP(4);
    // (7) off-critical-path stores: fp32 state, gates, time-indexed output
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tid + i * NT;
      if (e < NE) {
        const int row = e >> 4, c = e & 15;
        const int b = r0 + row, u = u0 + c;
        const bool act = s < lenr[i];
        a.hsave[dir][((size_t)(s + 1) * NP + b) * H + u] = hreg[i];
        if (CELL == CELL_GRU) reinterpret_cast<float4*>(a.gates[dir])[((size_t)s * NP + b) * H + u] = gsv[i];
        if (b < N) {
          const int t = act ? ((dir == 0) ? s : (lenr[i] - 1 - s)) : s;
          a.y[dir][((size_t)t * N + b) * H + u] = f2bf(hout[i]);
        }
      }
    }
  }
  DS2_STAMP_STORE(a);
}

template <int CELL, int NW, int MT, int KPW>
__global__ __launch_bounds__(NW * 64) void rnn_bwd_kernel(BwdArgs a) {
  constexpr int G = (CELL == CELL_GRU) ? 3 : 1;
  constexpr int NT = NW * 64;
  constexpr int ROWS = 16 * MT;
  constexpr int NE = ROWS * 16;
  constexpr int EPT = (NE + NT - 1) / NT;

  __shared__ float red[NW][ROWS][16];
  __shared__ __attribute__((aligned(16))) bf16_t stage[ROWS][G * 16];
  __shared__ int abort_flag;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int S = a.S;
  const int slice = blockIdx.x % S;
  const int grp = blockIdx.x / S;
  const int bg = grp % a.BG, dir = grp / a.BG;
  const int r0 = bg * ROWS, u0 = slice * 16;
  const int H = a.H, GH = G * H, KS = GH / 32;
  const int N = a.N, NP = a.NP;

  if (tid == 0) abort_flag = 0;

  // ---- resident U column fragments: B[k][c] = U[k][u0 + c], k over all G*H ----------
  bf16x8 uf[KPW];
  const bf16_t* Ud = a.U[dir];
#pragma unroll
  for (int kk = 0; kk < KPW; ++kk) {
    const int ks = wave + kk * NW;
    bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (ks < KS) {
      const int k0 = ks * 32 + 8 * (lane >> 4);
      const bf16_t* p = Ud + (size_t)k0 * H + u0 + (lane & 15);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (short)p[(size_t)j * H];
    }
    uf[kk] = v;
  }

  float carry[EPT];
  int lenr[EPT];
  float sbx[EPT][G];      // per-element bias-gradient sums over this launch's steps
  float sbh[EPT];         // GRU: sum of d(U_n h + b_hn) (the only gate where dgh != dgx)
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int e = tid + i * NT;
    const int row = e >> 4, c = e & 15;
    const int b = r0 + row, u = u0 + c;
    carry[i] = 0.f;
    sbh[i] = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g) sbx[i][g] = 0.f;
    lenr[i] = 0;
    if (e < NE) {
      lenr[i] = (b < N) ? a.lens[b] : 0;
      if (a.s_end < a.steps && a.carry[dir] != nullptr) carry[i] = a.carry[dir][(size_t)b * H + u];
    }
  }

  const unsigned dgh_bytes = (unsigned)((size_t)a.steps * NP * GH * 2);
  const __amdgpu_buffer_rsrc_t rs_dgh = make_rsrc(a.dgh[dir], dgh_bytes);
  const unsigned* gflags = a.flags + grp * S;
  __syncthreads();
  DS2_STAMP_DECL

  for (int s = a.s_end - 1; s >= a.s_begin; --s) {
    const int it = a.s_end - 1 - s;
    DS2_STAMP(5);
    // (1) prefetch everything that does not depend on the recurrence
    float dyv[EPT];
    float4 gsv[EPT];
    float hp[EPT];
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tid + i * NT;
      const int row = e >> 4, c = e & 15;
      const int b = r0 + row, u = u0 + c;
      const bool act = (e < NE) && (s < lenr[i]);
      const int t = (dir == 0) ? s : (lenr[i] - 1 - s);
      dyv[i] = (act && b < N) ? bf2f(a.dy[((size_t)t * N + b) * H + u]) : 0.f;
      if (CELL == CELL_GRU) {
        gsv[i] = act ? reinterpret_cast<const float4*>(a.gates[dir])[((size_t)s * NP + b) * H + u]
                     : make_float4(0.f, 0.f, 0.f, 0.f);
        hp[i] = act ? a.hsave[dir][((size_t)s * NP + b) * H + u] : 0.f;
      } else {
        hp[i] = act ? a.hsave[dir][((size_t)(s + 1) * NP + b) * H + u] : 0.f;   // h_s itself
      }
    }

    // (2) wait for dgh of step s+1 from every slice of the group
    if (it > 0) {
      if (wave == 0) {
        if (!wait_group(gflags, S, (unsigned)it, lane, a.timeout, a.err)) {
          if (lane == 0) abort_flag = 1;
        }
      }
      __syncthreads();
      if (abort_flag) break;
    }
    DS2_STAMP(0);

    // (3) dh_rec = dgh_{s+1} . U[:, slice]
    f32x4 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (s + 1 < a.steps) {
      bf16x8 af[MT][KPW];
#pragma unroll
      for (int kk = 0; kk < KPW; ++kk) {
        const int ks = wave + kk * NW;
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          if (ks < KS) {
            const unsigned off = (unsigned)((((size_t)(s + 1) * NP + r0 + m * 16 + (lane & 15)) * GH +
                                             ks * 32 + 8 * (lane >> 4)) * 2);
            af[m][kk] = __builtin_bit_cast(bf16x8, load_sc1_b128(rs_dgh, off));
          }
        }
      }
#pragma unroll
      for (int kk = 0; kk < KPW; ++kk) {
        const int ks = wave + kk * NW;
        if (ks < KS) {
#pragma unroll
          for (int m = 0; m < MT; ++m)
            acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m][kk], uf[kk], acc[m], 0, 0, 0);
        }
      }
    }
    DS2_STAMP(1);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[wave][m * 16 + (lane >> 4) * 4 + j][lane & 15] = acc[m][j];
    __syncthreads();

    DS2_STAMP(2);
    // (4) cell backward epilogue (exchange copy first; dgx stores after the publish)
    float gxs[EPT][G];
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tid + i * NT;
#pragma unroll
      for (int g = 0; g < G; ++g) gxs[i][g] = 0.f;
      if (e < NE) {
        const int row = e >> 4, c = e & 15;
        float dhrec = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) dhrec += red[w][row][c];
        const bool act = s < lenr[i];
        const float dh = dyv[i] + carry[i] + dhrec;
        float ghv[G];
        float cnew = 0.f;
        if (CELL == CELL_GRU) {
          const float r = gsv[i].x, z = gsv[i].y, n = gsv[i].z, ghn = gsv[i].w;
          const float dn = dh * (1.f - z);
          const float dz = dh * (hp[i] - n);
          cnew = dh * z;
          const float dan = dn * (1.f - n * n);
          const float dr = dan * ghn;
          const float dghn = dan * r;
          const float daz = dz * z * (1.f - z);
          const float dar = dr * r * (1.f - r);
          ghv[0] = dar; ghv[1] = daz; ghv[2] = dghn;
          gxs[i][0] = dar; gxs[i][1] = daz; gxs[i][2] = dan;
        } else {
          const float h = hp[i];
          const float da = (h > 0.f && h < RELU_CAP) ? dh : 0.f;
          ghv[0] = da;
          gxs[i][0] = da;
        }
        if (!act) {
          cnew = 0.f;
#pragma unroll
          for (int g = 0; g < G; ++g) { ghv[g] = 0.f; gxs[i][g] = 0.f; }
        }
        carry[i] = cnew;
#pragma unroll
        for (int g = 0; g < G; ++g) {
          stage[row][g * 16 + c] = f2bf(ghv[g]);
          sbx[i][g] += gxs[i][g];
        }
        if (CELL == CELL_GRU) sbh[i] += ghv[G - 1];
      }
    }
    __syncthreads();
    DS2_STAMP(3);

    // (5) publish dgh_s
    if (wave == 0) {
      for (int q = lane; q < ROWS * G * 2; q += 64) {
        const int row = q / (2 * G), rem = q % (2 * G);
        const int g = rem >> 1, half = rem & 1;
        const i32x4 v = *reinterpret_cast<const i32x4*>(&stage[row][g * 16 + half * 8]);
        const unsigned off = (unsigned)((((size_t)s * NP + r0 + row) * GH + g * H + u0 + half * 8) * 2);
        store_sc1_b128(rs_dgh, off, v);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) st_flag(a.flags + grp * S + slice, (unsigned)(it + 1));
    }

    DS2_STAMP(4);
    // (6) time-indexed input-projection gradient (off the critical path)
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tid + i * NT;
      if (e < NE) {
        const int row = e >> 4, c = e & 15;
        const int b = r0 + row, u = u0 + c;
        if (b < N) {
          const bool act = s < lenr[i];
          const int t = act ? ((dir == 0) ? s : (lenr[i] - 1 - s)) : s;
          bf16_t* dst = a.dgx + ((size_t)t * N + b) * a.gstride + dir * GH + u;
#pragma unroll
          for (int g = 0; g < G; ++g) dst[g * H] = f2bf(gxs[i][g] * a.dgx_scale);
        }
      }
    }
  }

  DS2_STAMP_STORE(a);
  // bias gradients: reduce this workgroup's rows through LDS, then one read-modify-write
  // per (gate, unit) of the workgroup's own [bg] partial row (no atomics: every element
  // has exactly one writer per launch; step-mode launches are stream-ordered)
  if (a.dbx_part[dir] != nullptr) {
    constexpr int BW = (G + 1) * 16;
    static_assert(NW * ROWS * 16 >= ROWS * BW, "bias reduction does not fit the LDS scratch");
    float* bred = &red[0][0][0];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tid + i * NT;
      if (e < NE) {
        const int row = e >> 4, c = e & 15;
#pragma unroll
        for (int g = 0; g < G; ++g) bred[row * BW + g * 16 + c] = sbx[i][g];
        bred[row * BW + G * 16 + c] = sbh[i];
      }
    }
    __syncthreads();
    for (int q = tid; q < BW; q += NT) {
      float sum = 0.f;
#pragma unroll
      for (int r = 0; r < ROWS; ++r) sum += bred[r * BW + q];
      const int g = q >> 4, c = q & 15;
      const size_t base = (size_t)bg * GH + u0 + c;
      if (g < G) {
        a.dbx_part[dir][base + (size_t)g * H] += sum;
        if (CELL == CELL_GRU && a.dbh_part[dir] != nullptr && g < G - 1) a.dbh_part[dir][base + (size_t)g * H] += sum;
      } else if (CELL == CELL_GRU && a.dbh_part[dir] != nullptr) {
        a.dbh_part[dir][base + (size_t)(G - 1) * H] += sum;
      }
    }
  }
  // step-mode carry hand-over
  if (a.carry[dir] != nullptr && a.s_begin > 0) {
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tid + i * NT;
      if (e < NE) {
        const int row = e >> 4, c = e & 15;
        a.carry[dir][(size_t)(r0 + row) * H + u0 + c] = carry[i];
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// dispatch
// ------------------------------------------------------------------------------------
static const int KPW_SET[] = {4, 8, 12, 16, 24, 32};

static int pick_kpw(int need) {
  for (int k : KPW_SET)
    if (k >= need) return k;
  return -1;
}

template <int CELL, int NW, int MT>
static int launch_fwd_kpw(int kpw, const FwdArgs& a, int grid, hipStream_t st) {
  switch (kpw) {
#define DS2_CASE(K) case K: hipLaunchKernelGGL((rnn_fwd_kernel<CELL, NW, MT, K>), dim3(grid), dim3(NW * 64), 0, st, a); break;
    DS2_CASE(4) DS2_CASE(8) DS2_CASE(12) DS2_CASE(16) DS2_CASE(24) DS2_CASE(32)
#undef DS2_CASE
    default: return -2;
  }
  return (int)hipGetLastError();
}

template <int CELL, int NW, int MT>
static int launch_bwd_kpw(int kpw, const BwdArgs& a, int grid, hipStream_t st) {
  switch (kpw) {
#define DS2_CASE(K) case K: hipLaunchKernelGGL((rnn_bwd_kernel<CELL, NW, MT, K>), dim3(grid), dim3(NW * 64), 0, st, a); break;
    DS2_CASE(4) DS2_CASE(8) DS2_CASE(12) DS2_CASE(16) DS2_CASE(24) DS2_CASE(32)
#undef DS2_CASE
    default: return -2;
  }
  return (int)hipGetLastError();
}

template <typename Args, typename F4, typename F8>
static int dispatch_nw_mt(int nw, int mt, F4 f4, F8 f8) {
  (void)sizeof(Args);
  if (nw == 4) return f4(mt);
  if (nw == 8) return f8(mt);
  return -3;
}

}  // namespace

extern "C" {

// Python-visible descriptors (flat, fixed-layout structs filled by the bindings).
struct DS2RnnFwd {
  int T, N, NP, H, S, BG, steps, gstride, ndir, cell, nw, mt, persistent;
  const int* lens;
  const void* gx;
  const void* U[2];
  const float* bh[2];
  void* y[2];
  void* hx[2];
  float* hsave[2];
  float* gates[2];
  unsigned* flags;
  unsigned* err;
  long long timeout;
  unsigned long long* stamps;
};

struct DS2RnnBwd {
  int T, N, NP, H, S, BG, steps, gstride, ndir, cell, nw, mt, persistent;
  const int* lens;
  const void* dy;
  const void* U[2];
  const float* hsave[2];
  const float* gates[2];
  void* dgh[2];
  void* dgx;
  float* carry[2];
  float* dbx_part[2];
  float* dbh_part[2];
  float dgx_scale;
  unsigned* flags;
  unsigned* err;
  long long timeout;
  unsigned long long* stamps;
};

int DS2_EXPORT(ds2_rnn_kpw)(int H, int G, int nw, int fwd) {
  const int ks = fwd ? H / 32 : G * H / 32;
  return pick_kpw((ks + nw - 1) / nw);
}

int DS2_EXPORT(ds2_rnn_fwd)(const DS2RnnFwd* d, hipStream_t st) {
  if (d->H % 32 != 0 || d->NP % (16 * d->mt) != 0) return -10;
  const int G = d->cell == CELL_GRU ? 3 : 1;
  const int kpw = DS2_EXPORT(ds2_rnn_kpw)(d->H, G, d->nw, 1);
  if (kpw < 0) return -11;
  FwdArgs a;
  a.T = d->T; a.N = d->N; a.NP = d->NP; a.H = d->H; a.S = d->S; a.BG = d->BG;
  a.steps = d->steps; a.gstride = d->gstride; a.lens = d->lens;
  a.gx = (const bf16_t*)d->gx;
  for (int i = 0; i < 2; ++i) {
    a.U[i] = (const bf16_t*)d->U[i]; a.bh[i] = d->bh[i]; a.y[i] = (bf16_t*)d->y[i];
    a.hx[i] = (bf16_t*)d->hx[i]; a.hsave[i] = d->hsave[i]; a.gates[i] = d->gates[i];
  }
  a.flags = d->flags; a.err = d->err; a.timeout = d->timeout; a.stamps = d->stamps;
  const int grid = d->ndir * d->BG * d->S;
  auto run = [&](int s0, int s1) -> int {
    a.s_begin = s0; a.s_end = s1;
    auto f4 = [&](int mt) -> int {
      if (d->cell == CELL_GRU) return mt == 1 ? launch_fwd_kpw<CELL_GRU, 4, 1>(kpw, a, grid, st)
                                              : launch_fwd_kpw<CELL_GRU, 4, 2>(kpw, a, grid, st);
      return mt == 1 ? launch_fwd_kpw<CELL_RELU, 4, 1>(kpw, a, grid, st)
                     : launch_fwd_kpw<CELL_RELU, 4, 2>(kpw, a, grid, st);
    };
    auto f8 = [&](int mt) -> int {
      if (d->cell == CELL_GRU) return mt == 1 ? launch_fwd_kpw<CELL_GRU, 8, 1>(kpw, a, grid, st)
                                              : launch_fwd_kpw<CELL_GRU, 8, 2>(kpw, a, grid, st);
      return mt == 1 ? launch_fwd_kpw<CELL_RELU, 8, 1>(kpw, a, grid, st)
                     : launch_fwd_kpw<CELL_RELU, 8, 2>(kpw, a, grid, st);
    };
    if (d->mt != 1 && d->mt != 2) return -12;
    return dispatch_nw_mt<FwdArgs>(d->nw, d->mt, f4, f8);
  };
  if (d->steps <= 0) return 0;
  if (d->persistent) return run(0, d->steps);
  for (int s = 0; s < d->steps; ++s) {
    const int r = run(s, s + 1);
    if (r) return r;
  }
  return 0;
}

int DS2_EXPORT(ds2_rnn_bwd)(const DS2RnnBwd* d, hipStream_t st) {
  if (d->H % 32 != 0 || d->NP % (16 * d->mt) != 0) return -10;
  const int G = d->cell == CELL_GRU ? 3 : 1;
  const int kpw = DS2_EXPORT(ds2_rnn_kpw)(d->H, G, d->nw, 0);
  if (kpw < 0) return -11;
  BwdArgs a;
  a.T = d->T; a.N = d->N; a.NP = d->NP; a.H = d->H; a.S = d->S; a.BG = d->BG;
  a.steps = d->steps; a.gstride = d->gstride; a.lens = d->lens;
  a.dy = (const bf16_t*)d->dy; a.dgx = (bf16_t*)d->dgx;
  for (int i = 0; i < 2; ++i) {
    a.U[i] = (const bf16_t*)d->U[i]; a.hsave[i] = d->hsave[i]; a.gates[i] = d->gates[i];
    a.dgh[i] = (bf16_t*)d->dgh[i]; a.carry[i] = d->carry[i];
    a.dbx_part[i] = d->dbx_part[i]; a.dbh_part[i] = d->dbh_part[i];
  }
  a.dgx_scale = d->dgx_scale;
  a.flags = d->flags; a.err = d->err; a.timeout = d->timeout; a.stamps = d->stamps;
  const int grid = d->ndir * d->BG * d->S;
  auto run = [&](int s0, int s1) -> int {
    a.s_begin = s0; a.s_end = s1;
    auto f4 = [&](int mt) -> int {
      if (d->cell == CELL_GRU) return mt == 1 ? launch_bwd_kpw<CELL_GRU, 4, 1>(kpw, a, grid, st)
                                              : launch_bwd_kpw<CELL_GRU, 4, 2>(kpw, a, grid, st);
      return mt == 1 ? launch_bwd_kpw<CELL_RELU, 4, 1>(kpw, a, grid, st)
                     : launch_bwd_kpw<CELL_RELU, 4, 2>(kpw, a, grid, st);
    };
    auto f8 = [&](int mt) -> int {
      if (d->cell == CELL_GRU) return mt == 1 ? launch_bwd_kpw<CELL_GRU, 8, 1>(kpw, a, grid, st)
                                              : launch_bwd_kpw<CELL_GRU, 8, 2>(kpw, a, grid, st);
      return mt == 1 ? launch_bwd_kpw<CELL_RELU, 8, 1>(kpw, a, grid, st)
                     : launch_bwd_kpw<CELL_RELU, 8, 2>(kpw, a, grid, st);
    };
    if (d->mt != 1 && d->mt != 2) return -12;
    return dispatch_nw_mt<BwdArgs>(d->nw, d->mt, f4, f8);
  };
  if (d->steps <= 0) return 0;
  if (d->persistent) return run(0, d->steps);
  for (int s = d->steps - 1; s >= 0; --s) {
    const int r = run(s, s + 1);
    if (r) return r;
  }
  return 0;
}

}  // extern "C"
