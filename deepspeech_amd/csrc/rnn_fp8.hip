// Persistent bidirectional GRU forward with fp8 recurrent weights and an fp8 hidden-state
// exchange (gfx950 MX-scaled fp8 MFMA) — the config-5 "fp8 mixed precision" recurrence.
//
// Reference behaviour: src/custom_ops.py:36-72 (CustomRNNCell2 GRU, tf.nn.bidirectional_dynamic_rnn:
// outputs zero past each length, the backward direction reversed within each utterance). Same
// saved-state buffers as csrc/rnn_xcd.hip (h fp32, gates fp32, h_{t-1} bf16 for the dU GEMM),
// so the bf16 reduce-scatter BPTT of rnn_xcd.hip runs unchanged on them.
//
// Why fp8: a bf16 U slice of 32 units x 3 gates x H = 1280 is 245 KB per workgroup, so a group
// needs P = H/32 = 40 workgroups — more than the 32 CUs of an XCD — and exchanges write-through
// across XCDs (5.4 us/step at config 5). In fp8 the slice of 64 units is the same 245 KB, a
// group is P = H/64 = 20 workgroups on ONE XCD, and its per-step exchange stays in that XCD's
// L2 (plain stores), like the headline H = 800 layers.
//
//  * U: e4m3 with ONE power-of-two scale per tensor (ds2_fp8_quant_pow2: amax, scale 2^e with
//    amax / 2^e <= 448), applied exactly as the MFMA's E8M0 B-scale. h: e4m3 with unit scale
//    (|h| < 1 for the GRU), requantised every step when it is published.
//  * Workgroup = 64 units of one group (direction x batch group of R <= 8 rows), 9 waves:
//    8 MFMA waves = 4 unit quarters (uq = wave & 3, 16 units, all 3 gates) x 2 K halves
//    (kh = wave >> 2); wave 8 is the memory wave (gx one step ahead into LDS, outputs two
//    steps behind out of LDS staging: no MFMA wave ever waits behind a bulk store).
//  * k-step = 128 of K (one v_mfma_scale_f32_16x16x128_f8f6f4 per gate): a lane's A fragment
//    (row lane % 16; k in [16g, 16g+16) u [64+16g, 64+16g+16), g = lane / 16) is two 16-B
//    exchange granules of 16 units each; every granule of the lane's K half is loaded at once
//    and re-polled in one round (no serial round trips). The last KL of a wave's KB k-steps of
//    U live in (dynamic) LDS, the rest in VGPRs.
//  * Exchange: hq[step+1][NP][H] bytes, pre-filled with 0xFF (e4m3 NaN, never published: a NaN
//    h is canonicalised to 0x7F). A producer packs 16 lanes' bytes into one 16-B granule with
//    DPP row shifts and stores it (plain when the census finds the group on one XCD, else sc1
//    write-through); consumers load with sc1 and spin until no byte is the sentinel.
//  * Transpose-reduce: of a 16x16 accumulator tile, the kh = 0 wave finalises elements j = 0, 1
//    (rows 4 (lane >> 4) + j) and the kh = 1 wave j = 2, 3: each stores the two it does not own
//    (lane-contiguous, conflict-free), ONE LDS barrier, then adds the partner's. A lane then
//    runs the GRU cell for two (row, unit) elements in registers.
//  * Every spin is bounded (s_memrealtime timeout -> error word, the launch aborts).
#include <type_traits>

#include "common.h"

using namespace ds2;

namespace {

constexpr int UPW8 = 64;                 // hidden units per workgroup
constexpr int G8W = 8;                   // MFMA waves
constexpr int F8TH = (G8W + 1) * 64;     // + the memory wave
constexpr int MEMW8 = G8W;
constexpr int ROWS8 = 8;                 // staged rows (R <= 8; the MFMA tile has 16)
constexpr int G3 = 3;                    // GRU gates
typedef __attribute__((ext_vector_type(8))) int i32x8;

struct XF8 {
  int T, N, NP, H, P, BG, R, steps, gstride, ngroups, xcd_map;
  const int* lens;
  const bf16_t* gx;                 // [T][N][gstride] bf16, direction d at columns d*3H
  const unsigned char* U8[2];       // [3H][H] e4m3 (row = gate*H + unit)
  const int* uexp;                  // [2] E8M0 exponent of each direction's U scale (127 + e)
  const float* bh[2];               // [3H] recurrent bias (fp32) or null
  bf16_t* y[2];                     // [T][N][H] per-direction outputs
  unsigned char* hq[2];             // [steps+1][NP][H] e4m3 exchange, slots 1.. sentinel 0xFF
  bf16_t* hx[2];                    // [steps+1][NP][H] bf16 h (slot 0 = h0): the dU GEMM operand
  float* hsave[2];                  // [steps+1][NP][H] fp32 h
  float* gates[2];                  // [steps][NP][H][4] fp32 (r, z, n, U_n h + b_hn)
  unsigned* census;                 // [ngroups * P] pre-filled 0xFFFFFFFF
  unsigned* err;
  long long timeout;
};

// Pre-poll sleep (s_sleep 1 units) after a step's publish, before the next step's first
// exchange poll: these kernels issue that poll right behind their own store, where the bf16
// forward measured stale reads competing with the producers' stores in the XCD's L2
// (profiles/r6_recurrence_poll.md). Compile-time (A/B: build.py --variant ... -D).
#ifndef DS2_F8_FWD_SLEEP
#define DS2_F8_FWD_SLEEP 0
#endif
#ifndef DS2_F8_BWD_SLEEP
#define DS2_F8_BWD_SLEEP 3          // config-5 fp8: 17.30-17.39 vs 17.55-17.65 ms/step (scripts/r6_f8sleep2.sh)
#endif
template <int N>
__device__ __forceinline__ void f8_presleep() {
#pragma unroll
  for (int i = 0; i < N; ++i) __builtin_amdgcn_s_sleep(1);
}

__device__ __forceinline__ unsigned xcc_id8() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

// group = blockIdx % 8 (<= 8 groups: one XCD each under round-robin dispatch), member =
// blockIdx / 8; otherwise contiguous ranges
__device__ __forceinline__ bool take_role8(int xcd_map, int ngroups, int P, int& grp, int& mem) {
  if (xcd_map) {
    const int slot = blockIdx.x & 7;
    if (slot >= ngroups) return false;
    grp = slot;
    mem = blockIdx.x >> 3;
  } else {
    grp = blockIdx.x / P;
    mem = blockIdx.x % P;
  }
  return mem < P;
}

// 1: every member on one XCD, 0: spread, -1: timeout (wave 0)
__device__ int census8(unsigned* census, int grp, int mem, int P, long long timeout, unsigned* err) {
  const int lane = threadIdx.x & 63;
  unsigned* c = census + (size_t)grp * P;
  if (lane == 0) __hip_atomic_store(c + mem, xcc_id8(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  while (true) {
    bool ready = true, same = true;
    unsigned first = 0xffffffffu;
    for (int q = lane; q < P; q += 64) {
      const unsigned v = __hip_atomic_load(c + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ready = ready && (v != 0xffffffffu);
      if (q == lane) first = v;
      same = same && (v == first);
    }
    if (__all(ready)) {
      const unsigned x0 = __shfl(first, 0, 64);
      return __all(same && (lane >= P || first == x0)) ? 1 : 0;
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
      if (lane == 0) atomicOr(err, 2u);
      return -1;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// no byte of the granule is the sentinel 0xFF: SWAR "has a zero byte" on the complement
__device__ __forceinline__ bool granule8_ready(i32x4 v) {
  unsigned any = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const unsigned w = ~(unsigned)v[i];
    any |= (w - 0x01010101u) & ~w & 0x80808080u;
  }
  return any == 0;
}

// f32 -> e4m3 byte (OCP, round to nearest even, saturating); a NaN becomes 0x7F, never the
// sentinel 0xFF
__device__ __forceinline__ unsigned f2e4m3(float x) {
  const unsigned b = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(x, x, 0, false) & 0xffu;
  return b == 0xffu ? 0x7fu : b;
}

template <int KB, int KL>
__global__ __launch_bounds__(F8TH) void rnnf8_fwd_kernel(XF8 a) {
  constexpr int KR = KB - KL;               // register-resident U k-steps
  static_assert(KL >= 0 && KR >= 1, "k-steps");
  constexpr int GP = G3 * UPW8 + 8;         // gx ring row pitch (bf16)
  constexpr int OP = UPW8 + 4;              // output staging row pitch
  __shared__ float red_s[2][4][2][2][G3][64];     // [parity][uq][owner kh][element][gate][lane]
  __shared__ bf16_t gxr_s[2][ROWS8][GP];          // bf16: with KL = 2 the LDS is full
  __shared__ __attribute__((aligned(16))) float oh_s[2][ROWS8][OP];
  __shared__ __attribute__((aligned(16))) float oy_s[2][ROWS8][OP];
  __shared__ float4 og_s[2][ROWS8][OP];
  __shared__ int len_s[ROWS8];
  __shared__ int s_mode, s_abort;
  extern __shared__ __attribute__((aligned(16))) i32x8 ul_dyn[];   // [KL][G8W][G3][64]

  int grp, mem;
  if (!take_role8(a.xcd_map, a.ngroups, a.P, grp, mem)) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, N = a.N, NP = a.NP, R = a.R;
  const int bg = grp % a.BG, dir = grp / a.BG;
  const int r0 = bg * R, u0 = mem * UPW8;
  const int uq = wave & 3, kh = wave >> 2;
  const int g16 = lane >> 4;                     // lane group: rows 4 g16 .. 4 g16 + 3 of the tile
  const int ec = 16 * uq + (lane & 15);          // this lane's unit within the workgroup
  const int erow0 = 4 * g16 + 2 * kh;            // its two cell elements: rows erow0, erow0 + 1
  if (tid < ROWS8) len_s[tid] = (tid < R && r0 + tid < N) ? a.lens[r0 + tid] : 0;
  if (wave == 0) {
    const int m = census8(a.census, grp, mem, a.P, a.timeout, a.err);
    if (lane == 0) { s_mode = m; s_abort = (m < 0); }
  }
  __syncthreads();
  if (s_abort) return;

  // memory wave: gx granule q -> (row, gate, 8-unit chunk); R x 3 x 8 = 192 granules max
  constexpr int RGL = (ROWS8 * G3 * (UPW8 / 8) + 63) / 64;     // 3
  i32x4 gpre[RGL];
  const int NRG = R * G3 * (UPW8 / 8);
  auto mw_load = [&](int s) {
#pragma unroll
    for (int j = 0; j < RGL; ++j) {
      const int q = lane + 64 * j;
      const int qq = q < NRG ? q : 0;
      const int row = qq / (G3 * 8), rem = qq - row * (G3 * 8), g = rem >> 3, c8 = rem & 7;
      const int b = min(r0 + row, N - 1);
      const int t = max(0, min((dir == 0) ? s : (len_s[row] - 1 - s), a.T - 1));
      gpre[j] = *reinterpret_cast<const i32x4*>(a.gx + ((size_t)t * N + b) * a.gstride + dir * G3 * H + g * H + u0 +
                                                c8 * 8);
    }
  };
  auto mw_put = [&](int s) {
#pragma unroll
    for (int j = 0; j < RGL; ++j) {
      const int q = lane + 64 * j;
      if (q < NRG) {
        const int row = q / (G3 * 8), rem = q - row * (G3 * 8), g = rem >> 3, c8 = rem & 7;
        const bool act = s < len_s[row];
        const bf16x8 v = __builtin_bit_cast(bf16x8, gpre[j]);
#pragma unroll
        for (int k = 0; k < 8; ++k) gxr_s[s & 1][row][g * UPW8 + c8 * 8 + k] = act ? (bf16_t)v[k] : (bf16_t)0;
      }
    }
  };
  // outputs of step s: lane -> (row = lane / 8, 8 units (lane % 8) * 8)
  auto mw_store = [&](int s) {
    const int row = lane >> 3, c8 = (lane & 7) * 8;
    if (row >= R) return;
    const int b = r0 + row, u = u0 + c8;
    const int sl = s & 1;
    f32x4 h0 = *reinterpret_cast<const f32x4*>(&oh_s[sl][row][c8]);
    f32x4 h1 = *reinterpret_cast<const f32x4*>(&oh_s[sl][row][c8 + 4]);
    f32x4 y0 = *reinterpret_cast<const f32x4*>(&oy_s[sl][row][c8]);
    f32x4 y1 = *reinterpret_cast<const f32x4*>(&oy_s[sl][row][c8 + 4]);
    float4 gv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) gv[i] = og_s[sl][row][c8 + i];
    float* hsp = a.hsave[dir] + ((size_t)(s + 1) * NP + b) * H + u;
    *reinterpret_cast<f32x4*>(hsp) = h0;
    *reinterpret_cast<f32x4*>(hsp + 4) = h1;
    bf16x8 hb;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      hb[i] = (short)f2bf(h0[i]);
      hb[4 + i] = (short)f2bf(h1[i]);
    }
    *reinterpret_cast<bf16x8*>(a.hx[dir] + ((size_t)(s + 1) * NP + b) * H + u) = hb;
    float4* gp = reinterpret_cast<float4*>(a.gates[dir]) + ((size_t)s * NP + b) * H + u;
#pragma unroll
    for (int i = 0; i < 8; ++i) gp[i] = gv[i];
    if (b < N) {
      const int L = len_s[row];
      const int t = (s < L) ? ((dir == 0) ? s : (L - 1 - s)) : s;
      bf16x8 yb;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        yb[i] = (short)f2bf(y0[i]);
        yb[4 + i] = (short)f2bf(y1[i]);
      }
      *reinterpret_cast<bf16x8*>(a.y[dir] + ((size_t)t * N + b) * H + u) = yb;
    }
  };
  if (wave == MEMW8) {
    mw_load(0);
    mw_put(0);
    if (a.steps > 1) mw_load(1);
  }
  __syncthreads();                                   // gx ring slot 0
  const bool plain = s_mode == 1;
  const unsigned hq_bytes = (unsigned)((size_t)(a.steps + 1) * NP * H);
  const __amdgpu_buffer_rsrc_t rs_hq = make_rsrc(a.hq[dir], hq_bytes);

  if (wave < G8W) {
    const int KS = H / 128;                          // k-steps of 128 (host: even, 2 KB)
    // resident U fragments: B[k][n] = U8[g H + u0 + 16 uq + n][128 ks + k] for this lane's n =
    // lane % 16 and k in [16 g16, +16) u [64 + 16 g16, +16); ks = kh KB + kk
    i32x8 uf[KR][G3];
    const unsigned char* Ud = a.U8[dir];
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
      const int ks = kh * KB + kk;
#pragma unroll
      for (int g = 0; g < G3; ++g) {
        const unsigned char* p = Ud + (size_t)(g * H + u0 + ec) * H + ks * 128 + 16 * g16;
        const i32x4 lo = *reinterpret_cast<const i32x4*>(p);
        const i32x4 hi = *reinterpret_cast<const i32x4*>(p + 64);
        const i32x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        if (kk < KR) uf[kk < KR ? kk : 0][g] = v;
        else ul_dyn[(((kk >= KR ? kk - KR : 0) * G8W + wave) * G3 + g) * 64 + lane] = v;   // own slot
      }
    }
    (void)KS;
    const int sb = __builtin_amdgcn_readfirstlane(a.uexp[dir]);          // E8M0 B scale
    const int sbw = sb | (sb << 8) | (sb << 16) | (sb << 24);
    float bhr[G3];
#pragma unroll
    for (int g = 0; g < G3; ++g) bhr[g] = a.bh[dir] ? a.bh[dir][g * H + u0 + ec] : 0.f;
    float hreg[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int row = erow0 + e;
      hreg[e] = (row < R) ? a.hsave[dir][(size_t)(r0 + row) * H + u0 + ec] : 0.f;   // slot 0 = h0
    }
    // padding rows of the 16-row tile re-read row R - 1 (a real, polled row)
    const int arow = r0 + min(lane & 15, R - 1);
    for (int s = 0; s < a.steps; ++s) {
      if (s > 0) f8_presleep<DS2_F8_FWD_SLEEP>();
      float gxv[2][G3];
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int g = 0; g < G3; ++g) gxv[e][g] = bf2f(gxr_s[s & 1][min(erow0 + e, ROWS8 - 1)][g * UPW8 + ec]);
      // every granule of this lane's K half at once; k-step kk's two granules are 64 B apart,
      // consecutive k-steps 128 B apart (immediate offsets off one base)
      const unsigned o0 = (unsigned)(((size_t)s * NP + arow) * H + kh * KB * 128 + 16 * g16);
      i32x4 v[KB][2];
#pragma unroll
      for (int kk = 0; kk < KB; ++kk) {
        v[kk][0] = load_sc1_b128(rs_hq, o0 + 128u * kk);
        v[kk][1] = load_sc1_b128(rs_hq, o0 + 128u * kk + 64u);
      }
      f32x4 acc[G3];
#pragma unroll
      for (int g = 0; g < G3; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
      const long long t0 = __builtin_amdgcn_s_memrealtime();
      unsigned done = 0;                             // wave-uniform prefix of consumed k-steps
      constexpr unsigned FULL = (1u << KB) - 1u;
      bool ok = true;
      while (true) {
#pragma unroll
        for (int kk = 0; kk < KB; ++kk) {
          if (done == (1u << kk) - 1u && __all(granule8_ready(v[kk][0]) && granule8_ready(v[kk][1]))) {
            const i32x8 af = __builtin_shufflevector(v[kk][0], v[kk][1], 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
            for (int g = 0; g < G3; ++g) {
              const i32x8 b = kk < KR ? uf[kk < KR ? kk : 0][g]
                                      : ul_dyn[(((kk >= KR ? kk - KR : 0) * G8W + wave) * G3 + g) * 64 + lane];
              acc[g] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, b, acc[g], 0, 0, 0, 0x7f7f7f7f, 0, sbw);
            }
            done |= 1u << kk;
          }
        }
        if (done == FULL) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) { ok = false; break; }
#pragma unroll
        for (int kk = 0; kk < KB; ++kk)
          if (!(done & (1u << kk))) {
            v[kk][0] = load_sc1_b128(rs_hq, o0 + 128u * kk);
            v[kk][1] = load_sc1_b128(rs_hq, o0 + 128u * kk + 64u);
          }
      }
      if (!ok) { s_abort = 1; atomicOr(a.err, 1u); }
      // transpose-reduce: hand the two elements the partner finalises to it
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int g = 0; g < G3; ++g) red_s[s & 1][uq][kh ^ 1][e][g][lane] = acc[g][2 * (kh ^ 1) + e];
      lds_barrier();
      if (s_abort) break;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int row = erow0 + e;
        float pre[G3];
#pragma unroll
        for (int g = 0; g < G3; ++g) pre[g] = acc[g][2 * kh + e] + red_s[s & 1][uq][kh][e][g][lane];
        const bool real = row < R;
        const int L = real ? len_s[row] : 0;
        const bool act = s < L;
        const float ghn = pre[2] + bhr[2];
        const float r = sigmoidf_(gxv[e][0] + pre[0] + bhr[0]);
        const float z = sigmoidf_(gxv[e][1] + pre[1] + bhr[1]);
        const float n = tanhf_(gxv[e][2] + r * ghn);
        const float hn = (1.f - z) * n + z * hreg[e];
        const float hnew = act ? hn : hreg[e];
        hreg[e] = hnew;
        // publish: 16 lanes (the tile's 16 units of this row) -> one 16-B e4m3 granule
        const unsigned b = f2e4m3(hnew);
        const unsigned w1 = b | ((unsigned)__builtin_amdgcn_update_dpp(0, (int)b, 0x101, 0xf, 0xf, false) << 8);
        const unsigned w2 = w1 | ((unsigned)__builtin_amdgcn_update_dpp(0, (int)w1, 0x102, 0xf, 0xf, false) << 16);
        const int d1 = __builtin_amdgcn_update_dpp(0, (int)w2, 0x104, 0xf, 0xf, false);
        const int d2 = __builtin_amdgcn_update_dpp(0, (int)w2, 0x108, 0xf, 0xf, false);
        const int d3 = __builtin_amdgcn_update_dpp(0, (int)w2, 0x10c, 0xf, 0xf, false);
        if ((lane & 15) == 0 && real) {
          const i32x4 gv = {(int)w2, d1, d2, d3};
          const unsigned off = (unsigned)(((size_t)(s + 1) * NP + r0 + row) * H + u0 + 16 * uq);
          if (plain) store_b128(rs_hq, off, gv);
          else store_sc1_b128(rs_hq, off, gv);
        }
        if (real) {
          oh_s[s & 1][row][ec] = hnew;
          oy_s[s & 1][row][ec] = act ? hn : 0.f;
          og_s[s & 1][row][ec] = act ? make_float4(r, z, n, ghn) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
  } else {
    for (int s = 0; s < a.steps; ++s) {
      if (s + 1 < a.steps) mw_put(s + 1);
      if (s >= 2) mw_store(s - 2);
      if (s + 2 < a.steps) mw_load(s + 2);
      lds_barrier();
      if (s_abort) break;
    }
  }
  __syncthreads();
  if (wave == MEMW8 && !s_abort) {
    if (a.steps >= 2) mw_store(a.steps - 2);
    if (a.steps >= 1) mw_store(a.steps - 1);
  }
}

// Generation 2 of the fp8 forward (rnnf8h_fwd_kernel): 8 MFMA waves = 2 unit halves (uh =
// wave & 1: 32 units = 2 quarters x 3 gates = 6 tiles) x 4 K-quarters (kq = wave >> 1: k-steps
// kq + 4 kk). Generation 1 (rnnf8_fwd_kernel: 4 unit quarters x 2 K halves) had each exchange
// granule polled by 4 waves of the workgroup; here by 2 (the wide bf16 kernels showed the CU's
// vector-memory pipe, not the MFMAs, setting such a step). K-quarters kq < KS % 4 have one
// more k-step than the rest: that k-step's U lives in LDS (4 wave slots), the others in VGPRs.
// Transpose-reduce as in generation 4 of the bf16 forward: a lane finalises element j = kq of
// its 6 tiles (two GRU cells: units 32 uh + 16 q + lane % 16, q = 0, 1).
template <int KS>
__global__ __launch_bounds__(F8TH) void rnnf8h_fwd_kernel(XF8 a) {
  constexpr int NT = 2 * G3;                 // tiles t = 3 q + g
  constexpr int KR = KS / 4;                 // k-steps every K-quarter has (VGPR-resident U)
  constexpr int NLW = KS % 4;                // K-quarters with one more k-step (LDS-resident U)
  constexpr int KB = KR + (NLW ? 1 : 0);
  constexpr int GP = G3 * UPW8 + 8;          // gx ring row pitch (bf16)
  constexpr int OP = UPW8 + 4;               // output staging row pitch
  __shared__ float red_s[2][2][4][3][NT][64];     // [parity][uh][element j][source][tile][lane]
  // three gx slots: the MFMA waves read step s's slot after the step's barrier, while the
  // memory wave (already past it) fills step s + 2's
  __shared__ bf16_t gxr_s[3][ROWS8][GP];
  __shared__ __attribute__((aligned(16))) float oh_s[2][ROWS8][OP];
  __shared__ __attribute__((aligned(16))) float oy_s[2][ROWS8][OP];
  __shared__ float4 og_s[2][ROWS8][OP];
  __shared__ int len_s[ROWS8];
  __shared__ int s_mode, s_abort;
  __shared__ float bh_s[G3][UPW8];                // recurrent bias (read after the barrier: VGPR budget)
  __shared__ i32x8 ul_s[NLW > 0 ? 2 * NLW : 1][NT][64];   // [uh + 2 kq][tile][lane], kq < NLW

  int grp, mem;
  if (!take_role8(a.xcd_map, a.ngroups, a.P, grp, mem)) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, N = a.N, NP = a.NP, R = a.R;
  const int bg = grp % a.BG, dir = grp / a.BG;
  const int r0 = bg * R, u0 = mem * UPW8;
  const int uh = wave & 1, kq = (wave >> 1) & 3;
  const int g16 = lane >> 4;
  const int erow = 4 * g16 + kq;                 // this lane's cell row (element j = kq)
  const int er = min(erow, ROWS8 - 1);           // for LDS reads (rows >= R are not real)
  if (tid < ROWS8) len_s[tid] = (tid < R && r0 + tid < N) ? a.lens[r0 + tid] : 0;
  if (tid < G3 * UPW8) bh_s[tid / UPW8][tid % UPW8] = a.bh[dir] ? a.bh[dir][(tid / UPW8) * H + u0 + tid % UPW8] : 0.f;
  if (wave == 0) {
    const int m = census8(a.census, grp, mem, a.P, a.timeout, a.err);
    if (lane == 0) { s_mode = m; s_abort = (m < 0); }
  }
  __syncthreads();
  if (s_abort) return;

  // memory wave: gx granule q -> (row, gate, 8-unit chunk); R x 3 x 8 = 192 granules max
  constexpr int RGL = (ROWS8 * G3 * (UPW8 / 8) + 63) / 64;     // 3
  i32x4 gpre[RGL];
  const int NRG = R * G3 * (UPW8 / 8);
  auto mw_load = [&](int s) {
#pragma unroll
    for (int j = 0; j < RGL; ++j) {
      const int q = lane + 64 * j;
      const int qq = q < NRG ? q : 0;
      const int row = qq / (G3 * 8), rem = qq - row * (G3 * 8), g = rem >> 3, c8 = rem & 7;
      const int b = min(r0 + row, N - 1);
      const int t = max(0, min((dir == 0) ? s : (len_s[row] - 1 - s), a.T - 1));
      gpre[j] = *reinterpret_cast<const i32x4*>(a.gx + ((size_t)t * N + b) * a.gstride + dir * G3 * H + g * H + u0 +
                                                c8 * 8);
    }
  };
  auto mw_put = [&](int s) {
#pragma unroll
    for (int j = 0; j < RGL; ++j) {
      const int q = lane + 64 * j;
      if (q < NRG) {
        const int row = q / (G3 * 8), rem = q - row * (G3 * 8), g = rem >> 3, c8 = rem & 7;
        const bool act = s < len_s[row];
        const bf16x8 v = __builtin_bit_cast(bf16x8, gpre[j]);
#pragma unroll
        for (int k = 0; k < 8; ++k) gxr_s[s % 3][row][g * UPW8 + c8 * 8 + k] = act ? (bf16_t)v[k] : (bf16_t)0;
      }
    }
  };
  // outputs of step s: lane -> (row = lane / 8, 8 units (lane % 8) * 8)
  auto mw_store = [&](int s) {
    const int row = lane >> 3, c8 = (lane & 7) * 8;
    if (row >= R) return;
    const int b = r0 + row, u = u0 + c8;
    const int sl = s & 1;
    f32x4 h0 = *reinterpret_cast<const f32x4*>(&oh_s[sl][row][c8]);
    f32x4 h1 = *reinterpret_cast<const f32x4*>(&oh_s[sl][row][c8 + 4]);
    f32x4 y0 = *reinterpret_cast<const f32x4*>(&oy_s[sl][row][c8]);
    f32x4 y1 = *reinterpret_cast<const f32x4*>(&oy_s[sl][row][c8 + 4]);
    float4 gv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) gv[i] = og_s[sl][row][c8 + i];
    float* hsp = a.hsave[dir] + ((size_t)(s + 1) * NP + b) * H + u;
    *reinterpret_cast<f32x4*>(hsp) = h0;
    *reinterpret_cast<f32x4*>(hsp + 4) = h1;
    bf16x8 hb;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      hb[i] = (short)f2bf(h0[i]);
      hb[4 + i] = (short)f2bf(h1[i]);
    }
    *reinterpret_cast<bf16x8*>(a.hx[dir] + ((size_t)(s + 1) * NP + b) * H + u) = hb;
    float4* gp = reinterpret_cast<float4*>(a.gates[dir]) + ((size_t)s * NP + b) * H + u;
#pragma unroll
    for (int i = 0; i < 8; ++i) gp[i] = gv[i];
    if (b < N) {
      const int L = len_s[row];
      const int t = (s < L) ? ((dir == 0) ? s : (L - 1 - s)) : s;
      bf16x8 yb;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        yb[i] = (short)f2bf(y0[i]);
        yb[4 + i] = (short)f2bf(y1[i]);
      }
      *reinterpret_cast<bf16x8*>(a.y[dir] + ((size_t)t * N + b) * H + u) = yb;
    }
  };
  if (wave == MEMW8) {
    mw_load(0);
    mw_put(0);
    if (a.steps > 1) mw_load(1);
  }
  __syncthreads();                                   // gx ring slot 0
  const bool plain = s_mode == 1;
  const unsigned hq_bytes = (unsigned)((size_t)(a.steps + 1) * NP * H);
  const __amdgpu_buffer_rsrc_t rs_hq = make_rsrc(a.hq[dir], hq_bytes);

  if (wave < G8W) {
    const int nk = KR + (kq < NLW ? 1 : 0);          // this wave's k-steps (wave-uniform)
    // resident U fragments: B[k][n] = U8[g H + u0 + 32 uh + 16 q + n][128 ks + k], n = lane % 16,
    // k in [16 g16, +16) u [64 + 16 g16, +16); ks = kq + 4 kk
    i32x8 uf[KR > 0 ? KR : 1][NT];
    const unsigned char* Ud = a.U8[dir];
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
      if (kk >= nk) continue;
      const int ks = kq + 4 * kk;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int q = t / G3, g = t % G3;
        const unsigned char* p = Ud + (size_t)(g * H + u0 + 32 * uh + 16 * q + (lane & 15)) * H + ks * 128 + 16 * g16;
        const i32x4 lo = *reinterpret_cast<const i32x4*>(p);
        const i32x4 hi = *reinterpret_cast<const i32x4*>(p + 64);
        const i32x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        if (kk < KR) uf[kk < KR ? kk : 0][t] = v;
        else ul_s[uh + 2 * kq][t][lane] = v;         // kq < NLW: own slot, no barrier needed
      }
    }
    const int sb = __builtin_amdgcn_readfirstlane(a.uexp[dir]);          // E8M0 B scale
    const int sbw = sb | (sb << 8) | (sb << 16) | (sb << 24);
    float hreg[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int u = u0 + 32 * uh + 16 * q + (lane & 15);
      hreg[q] = (erow < R) ? a.hsave[dir][(size_t)(r0 + erow) * H + u] : 0.f;   // slot 0 = h0
    }
    const int arow = r0 + min(lane & 15, R - 1);
    for (int s = 0; s < a.steps; ++s) {
      if (s > 0) f8_presleep<DS2_F8_FWD_SLEEP>();
      // every granule of this lane's K-quarter at once: k-step kk's two granules are 64 B
      // apart, consecutive k-steps of the quarter 512 B
      const unsigned o0 = (unsigned)(((size_t)s * NP + arow) * H + kq * 128 + 16 * g16);
      i32x4 v[KB][2];
#pragma unroll
      for (int kk = 0; kk < KB; ++kk) {
        v[kk][0] = load_sc1_b128(rs_hq, o0 + 512u * kk);
        v[kk][1] = load_sc1_b128(rs_hq, o0 + 512u * kk + 64u);
      }
      f32x4 acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const long long t0 = __builtin_amdgcn_s_memrealtime();
      unsigned done = 0;                             // wave-uniform prefix of consumed k-steps
      constexpr unsigned FULL = (1u << KB) - 1u;
      bool ok = true;
      while (true) {
#pragma unroll
        for (int kk = 0; kk < KB; ++kk) {
          if (done != (1u << kk) - 1u) continue;
          if (kk >= nk) {                            // past this quarter's K: nothing to wait on
            done |= 1u << kk;
          } else if (__all(granule8_ready(v[kk][0]) && granule8_ready(v[kk][1]))) {
            const i32x8 af = __builtin_shufflevector(v[kk][0], v[kk][1], 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
            for (int t = 0; t < NT; ++t) {
              const i32x8 b = kk < KR ? uf[kk < KR ? kk : 0][t] : ul_s[uh + 2 * kq][t][lane];
              acc[t] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, b, acc[t], 0, 0, 0, 0x7f7f7f7f, 0, sbw);
            }
            done |= 1u << kk;
          }
        }
        if (done == FULL) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) { ok = false; break; }
#pragma unroll
        for (int kk = 0; kk < KB; ++kk)
          if (!(done & (1u << kk))) {
            v[kk][0] = load_sc1_b128(rs_hq, o0 + 512u * kk);
            v[kk][1] = load_sc1_b128(rs_hq, o0 + 512u * kk + 64u);
          }
      }
      if (!ok) { s_abort = 1; atomicOr(a.err, 1u); }
      // transpose-reduce: hand the three elements this wave does not finalise to their owners
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j == kq) continue;
        const int src = kq < j ? kq : kq - 1;
#pragma unroll
        for (int t = 0; t < NT; ++t) red_s[s & 1][uh][j][src][t][lane] = acc[t][j];
      }
      lds_barrier();
      if (s_abort) break;
      // lane-derived LDS / store addresses recomputed from an opaque copy of the lane id each
      // step: hoisted out of the loop they were held across the poll and spilled (11 scratch
      // reloads per step)
      int ln = lane;
      asm volatile("" : "+v"(ln));
      const int er_l = min(4 * (ln >> 4) + kq, ROWS8 - 1);
      const bool real = 4 * (ln >> 4) + kq < R;
      const bool act = s < len_s[er_l];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        float pre[G3];
#pragma unroll
        for (int g = 0; g < G3; ++g) {
          const int t = G3 * q + g;
          const float own = kq == 0 ? acc[t][0] : kq == 1 ? acc[t][1] : kq == 2 ? acc[t][2] : acc[t][3];
          pre[g] = own + red_s[s & 1][uh][kq][0][t][ln] + red_s[s & 1][uh][kq][1][t][ln] +
                   red_s[s & 1][uh][kq][2][t][ln];
        }
        // gx (filled before the previous barrier) and the bias from LDS after the exchange:
        // held across the poll they pushed the kernel into spilling
        const int c = 32 * uh + 16 * q + (ln & 15);
        float gxv[G3];
#pragma unroll
        for (int g = 0; g < G3; ++g) gxv[g] = bf2f(gxr_s[s % 3][er_l][g * UPW8 + c]) + bh_s[g][c];
        const float ghn = pre[2] + bh_s[2][c];
        const float r = sigmoidf_(gxv[0] + pre[0]);
        const float z = sigmoidf_(gxv[1] + pre[1]);
        const float n = tanhf_(gxv[2] - bh_s[2][c] + r * ghn);
        const float hn = (1.f - z) * n + z * hreg[q];
        const float hnew = act ? hn : hreg[q];
        hreg[q] = hnew;
        // publish: 16 lanes (the tile's 16 units of this row) -> one 16-B e4m3 granule
        const unsigned b = f2e4m3(hnew);
        const unsigned w1 = b | ((unsigned)__builtin_amdgcn_update_dpp(0, (int)b, 0x101, 0xf, 0xf, false) << 8);
        const unsigned w2 = w1 | ((unsigned)__builtin_amdgcn_update_dpp(0, (int)w1, 0x102, 0xf, 0xf, false) << 16);
        const int d1 = __builtin_amdgcn_update_dpp(0, (int)w2, 0x104, 0xf, 0xf, false);
        const int d2 = __builtin_amdgcn_update_dpp(0, (int)w2, 0x108, 0xf, 0xf, false);
        const int d3 = __builtin_amdgcn_update_dpp(0, (int)w2, 0x10c, 0xf, 0xf, false);
        const int ec = c;
        if ((ln & 15) == 0 && real) {
          const i32x4 gv = {(int)w2, d1, d2, d3};
          const unsigned off = (unsigned)(((size_t)(s + 1) * NP + r0 + er_l) * H + u0 + ec);
          if (plain) store_b128(rs_hq, off, gv);
          else store_sc1_b128(rs_hq, off, gv);
        }
        if (real) {
          oh_s[s & 1][er_l][ec] = hnew;
          oy_s[s & 1][er_l][ec] = act ? hn : 0.f;
          og_s[s & 1][er_l][ec] = act ? make_float4(r, z, n, ghn) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
  } else {
    for (int s = 0; s < a.steps; ++s) {
      if (s + 1 < a.steps) mw_put(s + 1);
      if (s >= 2) mw_store(s - 2);
      if (s + 2 < a.steps) mw_load(s + 2);
      lds_barrier();
      if (s_abort) break;
    }
  }
  __syncthreads();
  if (wave == MEMW8 && !s_abort) {
    if (a.steps >= 2) mw_store(a.steps - 2);
    if (a.steps >= 1) mw_store(a.steps - 1);
  }
}

// ------------------------------------------------------------------------------------
// fp8 BPTT (rnnf8_bwd_kernel): config 5's backward on the forward's geometry — groups of
// P = H/64 workgroups of 64 units, one XCD per group (8 groups: 2 directions x 4 batch groups
// of R <= 8 rows), so the per-step exchange stays in the XCD's L2 (plain stores). The bf16
// reduce-scatter BPTT of rnn_xcd.hip needs 32-unit workgroups at H = 1280 (a 64-unit bf16
// U^T slice, 491 KB, does not fit a CU), i.e. P = 40 > 32 CUs: groups straddle XCDs and
// exchange write-through (5.2 us/step).
//  * Same protocol as rnnw_bwd_kernel: P_j(s) = dg_s[:, own cols] . U[own cols, :] for all H
//    units, published as tagged bf16 unit pairs into a 3-slot ring; a consumer gathers its
//    two pairs from every producer (two producers per 16-B load).
//  * Own columns: 3 gates x 64 units = 192 = k-step 0 (gates 0 and 1, 128 deep) + k-step 1
//    (gate 2, the second 64 of its 128 zero), one v_mfma_scale_f32_16x16x128_f8f6f4 each. U^T
//    is e4m3 with the forward's per-tensor power-of-two scale (E8M0 A scale); k-step 0's
//    fragments live in VGPRs, k-step 1's real half (16 B per lane) in LDS.
//  * dg (the gate-gradient operand) is requantised to e4m3 every step with one power-of-two
//    scale per (batch row, 32-unit group) over the three gates: the scale byte of B lane (n, b)
//    covers the contiguous K block [32b, 32b + 32) (not the 32 bytes lane group b holds), which
//    in the k-step layout is one gate's 32 units, so block b of both k-steps takes group b & 1's
//    scale; the dU GEMM and dgx outputs stay bf16.
// ------------------------------------------------------------------------------------
constexpr int BMW8 = 7;                  // worker waves (gather + MFMA); 0..3 also run the cell
constexpr int BEW8 = 4;
constexpr int BMEM8 = 7;                 // memory wave
constexpr int BTH8 = 8 * 64;

struct XF8B {
  int T, N, NP, H, P, BG, R, steps, gstride, ngroups, xcd_map;
  const int* lens;
  const bf16_t* dy;                 // [T][N][H]
  const unsigned char* U8T[2];      // [H][3H] e4m3 U^T: U8T[m][g H + u] = U[g H + u][m] / 2^e
  const int* uexp;                  // [2] E8M0 exponent of each direction's U scale
  const float* hsave[2];            // [steps+1][NP][H] fp32 h (slot s = h before step s)
  const float* gates[2];            // [steps][NP][H][4] (r, z, n, U_n h + b_hn)
  bf16_t* dgh[2];                   // [steps][NP][3H] bf16 output (dU GEMM operand)
  bf16_t* dgx;                      // [T][N][gstride] bf16 (x dgx_scale)
  unsigned* ring[2];                // [3][BG][P][H/32][R][4] 16-B granules, filled 0xFFFFFFFF
  float* dbx_part[2];               // [BG][3H] (+=)
  float* dbh_part[2];
  float dgx_scale;
  unsigned* census;
  unsigned* err;
  long long timeout;
};

// max over the 16 lanes of a DPP row (row_ror 8, 4, 2, 1): every lane ends with the row's max
__device__ __forceinline__ float row16_max(float v) {
#define DS2_ROR(N) v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + (N), 0xf, 0xf, false)))
  DS2_ROR(8); DS2_ROR(4); DS2_ROR(2); DS2_ROR(1);
#undef DS2_ROR
  return v;
}

// E8M0 exponent byte of the smallest power of two 2^e with amax / 2^e <= 448 (e4m3 max), from the
// bits of a non-negative finite amax: 448 = 1.75 * 2^8, so amax = (1 + f) 2^(E-127)
// needs e = E - 135, or E - 134 when its mantissa exceeds 0.75 (integer ops only: scalar when
// amax is wave-uniform)
__device__ __forceinline__ int e8m0_bits(unsigned amax_bits) {
  if (amax_bits == 0u) return 127;
  const int eb = (int)(amax_bits >> 23) - 8 + ((amax_bits & 0x7fffffu) > 0x600000u ? 1 : 0);
  return min(254, max(1, eb));
}

template <int MTU, int GPT>
__global__ __launch_bounds__(BTH8) void rnnf8_bwd_kernel(XF8B a) {
  constexpr int ROWS = 16;                        // MFMA tile rows (R <= 8 real)
  constexpr int EPT = 2;                          // epilogue elements per thread (rows wave + 4 i, i < 2)
  constexpr int LT = ROWS8 * (UPW8 / 4) / 64;     // memory-wave load tasks per lane (2)
  constexpr int ST = ROWS8 * G3 * (UPW8 / 8) / 64;  // store tasks per lane (3)
  static_assert(GPT % 2 == 0, "two producers per gather load");
  __shared__ float red_s[BMW8][ROWS][UPW8 + 1];
  __shared__ __attribute__((aligned(16))) unsigned char dq_s[2][ROWS][128];   // e4m3 dg by k-step
  __shared__ int dsc_s[ROWS][4];                 // E8M0 (4 copies) per (row, K block of either k-step)
  __shared__ float dyr_s[2][ROWS8][UPW8];
  __shared__ float hpr_s[2][ROWS8][UPW8];
  __shared__ float4 gr_s[2][ROWS8][UPW8];
  __shared__ __attribute__((aligned(16))) bf16_t ox_s[2][ROWS8][G3][UPW8];  // dgx (scaled)
  __shared__ __attribute__((aligned(16))) bf16_t oh_s[2][ROWS8][G3][UPW8];  // dgh
  __shared__ i32x4 ul_s[MTU][BMW8][64];                                     // k-step 1 A halves
  __shared__ int len_s[ROWS8];
  __shared__ int s_mode, s_abort;

  int grp, mem;
  if (!take_role8(a.xcd_map, a.ngroups, a.P, grp, mem)) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, GH = G3 * H, N = a.N, NP = a.NP, R = a.R, P = a.P, MTS = H / 16, NPR = MTS / 2;
  const int bg = grp % a.BG, dir = grp / a.BG;
  const int r0 = bg * R, u0 = mem * UPW8;
  if (tid < ROWS8) len_s[tid] = (tid < R && r0 + tid < N) ? a.lens[r0 + tid] : 0;
  if (tid < ROWS * 4) (&dsc_s[0][0])[tid] = 0x7f7f7f7f;
  for (int i = tid; i < 2 * ROWS * 128 / 4; i += BTH8) reinterpret_cast<int*>(&dq_s[0][0][0])[i] = 0;
  if (wave == 0) {
    const int m = census8(a.census, grp, mem, P, a.timeout, a.err);
    if (lane == 0) { s_mode = m; s_abort = (m < 0); }
  }
  // resident A fragments of m-tile mt = 2 (wave + 7 (i >> 1)) + (i & 1): A[m][k] = U^T, unit m =
  // 16 mt + lane % 16, k-step 0: k in [16 g, +16) = gate 0 units u0 + 16 g.., [64 + 16 g, +16) =
  // gate 1; k-step 1: [16 g, +16) = gate 2 (the rest zero), g = lane / 16
  i32x8 ua[MTU];
  {
    const unsigned char* Ut = a.U8T[dir];
#pragma unroll
    for (int i = 0; i < MTU; ++i) {
      const int mt = 2 * (wave + BMW8 * (i >> 1)) + (i & 1);
      i32x4 lo = {0, 0, 0, 0}, hi = lo, l2 = lo;
      if (wave < BMW8 && mt < MTS) {
        const unsigned char* p = Ut + (size_t)(16 * mt + (lane & 15)) * GH + u0 + 16 * (lane >> 4);
        lo = *reinterpret_cast<const i32x4*>(p);
        hi = *reinterpret_cast<const i32x4*>(p + H);
        l2 = *reinterpret_cast<const i32x4*>(p + 2 * H);
      }
      ua[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      if (wave < BMW8) ul_s[i][wave][lane] = l2;
    }
  }
  float carry[EPT], sbx[EPT][G3], sbh[EPT];
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    carry[i] = 0.f;
    sbh[i] = 0.f;
#pragma unroll
    for (int g = 0; g < G3; ++g) sbx[i][g] = 0.f;
  }
  __syncthreads();   // len_s, dq_s zeros, ul_s, census

  // memory wave: load task = (row, 4 units), store task = (row, gate, 8 units)
  uint2 pdy[LT];
  float4 php[LT];
  float4 pgt[LT][4];
  auto mw_load = [&](int s) {
#pragma unroll
    for (int k = 0; k < LT; ++k) {
      const int q = lane + 64 * k;
      const int row = q / (UPW8 / 4), c4 = (q % (UPW8 / 4)) * 4;
      if (row < R) {
        const int bp = min(r0 + row, NP - 1), bn = min(r0 + row, N - 1), u = u0 + c4;
        const int t = max(0, min((dir == 0) ? s : (len_s[row] - 1 - s), a.T - 1));
        pdy[k] = *reinterpret_cast<const uint2*>(a.dy + ((size_t)t * N + bn) * H + u);
        const float4* gp = reinterpret_cast<const float4*>(a.gates[dir]) + ((size_t)s * NP + bp) * H + u;
#pragma unroll
        for (int i = 0; i < 4; ++i) pgt[k][i] = gp[i];
        php[k] = *reinterpret_cast<const float4*>(a.hsave[dir] + ((size_t)s * NP + bp) * H + u);
      }
    }
  };
  auto mw_put = [&](int s) {
    const int slot = s & 1;
#pragma unroll
    for (int k = 0; k < LT; ++k) {
      const int q = lane + 64 * k;
      const int row = q / (UPW8 / 4), c4 = (q % (UPW8 / 4)) * 4;
      if (row < R) {
        const bool act = s < len_s[row];
        const float dv[4] = {bf2f((bf16_t)(pdy[k].x & 0xffffu)), bf2f((bf16_t)(pdy[k].x >> 16)),
                             bf2f((bf16_t)(pdy[k].y & 0xffffu)), bf2f((bf16_t)(pdy[k].y >> 16))};
        const float hv[4] = {php[k].x, php[k].y, php[k].z, php[k].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          dyr_s[slot][row][c4 + i] = act ? dv[i] : 0.f;
          hpr_s[slot][row][c4 + i] = act ? hv[i] : 0.f;
          gr_s[slot][row][c4 + i] = act ? pgt[k][i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
  };
  auto mw_store = [&](int s) {          // dgx and dgh of step s from the staging area
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      const int q = lane + 64 * k;
      const int row = q / (G3 * 8), rem = q - row * (G3 * 8), g = rem >> 3, c8 = (rem & 7) * 8;
      if (row < R) {
        const int b = r0 + row, u = u0 + c8;
        *reinterpret_cast<i32x4*>(a.dgh[dir] + ((size_t)s * NP + b) * GH + g * H + u) =
            *reinterpret_cast<const i32x4*>(&oh_s[s & 1][row][g][c8]);
        if (b < N) {
          const int L = len_s[row];
          const int t = (s < L) ? ((dir == 0) ? s : (L - 1 - s)) : s;
          *reinterpret_cast<i32x4*>(a.dgx + ((size_t)t * N + b) * a.gstride + dir * GH + g * H + u) =
              *reinterpret_cast<const i32x4*>(&ox_s[s & 1][row][g][c8]);
        }
      }
    }
  };
  if (s_abort) return;
  if (wave == BMEM8 && a.steps > 0) mw_load(a.steps - 1);
  const bool plain = s_mode == 1;
  const unsigned ring_bytes = (unsigned)((size_t)3 * a.BG * P * NPR * R * 64);
  const __amdgpu_buffer_rsrc_t rs_ring = make_rsrc(a.ring[dir], ring_bytes);
  auto tag_of = [&](int s) -> unsigned { return (unsigned)(((a.steps - 1 - s) / 3) & 1); };
  // [slot][bg][producer][unit pair][row][granule g][8 bf16]: granule (row, g) of pair p holds
  // units 32 p + {4 g .. 4 g + 3, 16 + 4 g .. 16 + 4 g + 3}
  auto ring_off16 = [&](int slot, int j, int pr, int row, int g) -> unsigned {
    return (unsigned)((((((size_t)slot * a.BG + bg) * P + j) * NPR + pr) * R + row) * 4 + g) * 16u;
  };

  if (wave < BMW8) {
    const int sa = __builtin_amdgcn_readfirstlane(a.uexp[dir]);
    const int saw = sa | (sa << 8) | (sa << 16) | (sa << 24);       // U^T: one E8M0 for all blocks
    for (int s = a.steps - 1; s >= 0; --s) {
      const bool has_next = s + 1 < a.steps;
      if (has_next) f8_presleep<DS2_F8_BWD_SLEEP>();
      // (G) lane -> (producer half h, row, granule g); the two unit pairs of this workgroup
      {
        const int h = lane >> 5, grow = (lane >> 2) & 7, gg = lane & 3;
        constexpr int NI = GPT / 2;
        float acc8[2][8];
#pragma unroll
        for (int pp = 0; pp < 2; ++pp)
#pragma unroll
          for (int q = 0; q < 8; ++q) acc8[pp][q] = 0.f;
        if (has_next && grow < R) {
          const int cs = (s + 1) % 3;
          const unsigned want = tag_of(s + 1);
          unsigned off[2][NI];
          i32x4 v[2][NI];
#pragma unroll
          for (int pp = 0; pp < 2; ++pp)
#pragma unroll
            for (int i = 0; i < NI; ++i) {
              const int j = min(wave + BMW8 * (2 * i + h), P - 1);
              off[pp][i] = ring_off16(cs, j, 2 * mem + pp, grow, gg);
              v[pp][i] = load_sc1_b128(rs_ring, off[pp][i]);
            }
          const long long t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
          for (int pp = 0; pp < 2; ++pp) {
#pragma unroll
            for (int i = 0; i < NI; ++i) {
              if (wave + BMW8 * (2 * i + h) < P) {
                while (!granule_tagged16(v[pp][i], want)) {
                  if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) { s_abort = 1; atomicOr(a.err, 1u); break; }
                  __builtin_amdgcn_s_sleep(1);
                  v[pp][i] = load_sc1_b128(rs_ring, off[pp][i]);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  acc8[pp][2 * q] += __uint_as_float((unsigned)v[pp][i][q] << 16);
                  acc8[pp][2 * q + 1] += __uint_as_float((unsigned)v[pp][i][q] & 0xffff0000u);
                }
              }
            }
          }
        }
        if (grow < R) {
#pragma unroll
          for (int pp = 0; pp < 2; ++pp)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              red_s[wave][grow + 8 * h][32 * pp + 4 * gg + q] = acc8[pp][q];
              red_s[wave][grow + 8 * h][32 * pp + 16 + 4 * gg + q] = acc8[pp][4 + q];
            }
        }
      }
      lds_barrier();                                                        // #1
      if (s_abort) break;
      // (E) cell backward (waves 0..3, row wave + 4 i, unit = lane): dgh / dgx staging and the
      // e4m3 dg operand with one power-of-two scale per (row, gate, 32-unit K block)
      if (wave < BEW8) {
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
          const int row = wave + BEW8 * i, c = lane;
          if (row < R) {                                  // wave-uniform
            float dhrec = 0.f;
            if (has_next) {
#pragma unroll
              for (int w = 0; w < BMW8; ++w) dhrec += red_s[w][row][c] + red_s[w][row + 8][c];
            }
            const bool act = s < len_s[row];
            const float dh = dyr_s[s & 1][row][c] + carry[i] + dhrec;
            const float hp = hpr_s[s & 1][row][c];
            const float4 gv = gr_s[s & 1][row][c];
            const float r = gv.x, z = gv.y, n = gv.z, ghn = gv.w;
            const float dn = dh * (1.f - z);
            const float dz = dh * (hp - n);
            const float dan = dn * (1.f - n * n);
            const float dr = dan * ghn;
            float ghv[G3] = {dr * r * (1.f - r), dz * z * (1.f - z), dan * r};
            float gxs[G3] = {ghv[0], ghv[1], dan};
            carry[i] = act ? dh * z : 0.f;
            if (!act) {
#pragma unroll
              for (int g = 0; g < G3; ++g) { ghv[g] = 0.f; gxs[g] = 0.f; }
            }
            // K block b of k-step 0 is gate b >> 1's units 32 (b & 1) + [0, 32), of k-step 1 gate
            // 2's (b < 2; blocks 2, 3 are zero): one scale per (row, 32-unit group) over the three
            // gates serves block b of both k-steps as the group b & 1's. Its amax: DPP max inside
            // each 16-lane row, then the 4 row maxima through SGPRs (non-negative floats order
            // as unsigned ints).
            const unsigned m = __float_as_uint(row16_max(fmaxf(fmaxf(fabsf(ghv[0]), fabsf(ghv[1])), fabsf(ghv[2]))));
            const int e01 = e8m0_bits(max(__builtin_amdgcn_readlane(m, 0), __builtin_amdgcn_readlane(m, 16)));
            const int e23 = e8m0_bits(max(__builtin_amdgcn_readlane(m, 32), __builtin_amdgcn_readlane(m, 48)));
            const int ebl = c < 32 ? e01 : e23;
            const float invl = __uint_as_float((unsigned)(254 - ebl) << 23);    // 2^-(eb - 127)
            dq_s[0][row][c] = (unsigned char)f2e4m3(ghv[0] * invl);
            dq_s[0][row][64 + c] = (unsigned char)f2e4m3(ghv[1] * invl);
            dq_s[1][row][c] = (unsigned char)f2e4m3(ghv[2] * invl);
            if (c == 0) {
              const int w01 = e01 * 0x01010101, w23 = e23 * 0x01010101;
              dsc_s[row][0] = w01; dsc_s[row][1] = w23; dsc_s[row][2] = w01; dsc_s[row][3] = w23;
            }
#pragma unroll
            for (int g = 0; g < G3; ++g) {
              oh_s[s & 1][row][g][c] = f2bf(ghv[g]);
              ox_s[s & 1][row][g][c] = f2bf(gxs[g] * a.dgx_scale);
              sbx[i][g] += gxs[g];
            }
            sbh[i] += ghv[G3 - 1];
          }
        }
      }
      lds_barrier();                                                        // #2
      // (M) publish P(s) = dg_s[:, own cols] . U[own cols, :] into ring slot s % 3
      if (s > 0) {
        const int ws = s % 3;
        const unsigned tagmask = tag_of(s) ? 0x00010001u : 0u;
        const bool prow = (lane & 15) < R;
        const unsigned char* dr = &dq_s[0][lane & 15][16 * (lane >> 4)];
        const i32x8 b0 = __builtin_shufflevector(*reinterpret_cast<const i32x4*>(dr),
                                                 *reinterpret_cast<const i32x4*>(dr + 64), 0, 1, 2, 3, 4, 5, 6, 7);
        const i32x4 z4 = {0, 0, 0, 0};
        const i32x8 b1 = __builtin_shufflevector(*reinterpret_cast<const i32x4*>(dr + ROWS * 128), z4, 0, 1, 2, 3, 4,
                                                 5, 6, 7);
        const int sbw0 = dsc_s[lane & 15][lane >> 4], sbw1 = sbw0;
        constexpr int NPW = MTU / 2;
        unsigned offp[NPW];
#pragma unroll
        for (int k = 0; k < NPW; ++k) offp[k] = ring_off16(ws, mem, min(wave + BMW8 * k, NPR - 1), lane & 15, lane >> 4);
        auto publish = [&](auto PLAIN) {
#pragma unroll
          for (int k = 0; k < NPW; ++k) {
            const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
            f32x4 a0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(ua[2 * k], b0, zero, 0, 0, 0, saw, 0, sbw0);
            f32x4 a1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(ua[2 * k + 1], b0, zero, 0, 0, 0, saw, 0, sbw0);
            const i32x8 u2a = __builtin_shufflevector(ul_s[2 * k][wave][lane], z4, 0, 1, 2, 3, 4, 5, 6, 7);
            const i32x8 u2b = __builtin_shufflevector(ul_s[2 * k + 1][wave][lane], z4, 0, 1, 2, 3, 4, 5, 6, 7);
            a0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(u2a, b1, a0, 0, 0, 0, saw, 0, sbw1);
            a1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(u2b, b1, a1, 0, 0, 0, saw, 0, sbw1);
            // the VALU conversion below reads the scaled MFMA's accumulators: hipcc (ROCm 7.2)
            // pads only 12 wait states after v_mfma_scale_f32_16x16x128_f8f6f4, too few here (the
            // publish then stored partly-updated sums: tools/probe_mfma_layout.hip and the
            // emulation test). The operand-tied s_nop keeps 8 more between them.
            asm volatile("s_nop 7" : "+v"(a0), "+v"(a1));
            if (prow && wave + BMW8 * k < NPR) {
              const i32x4 v = {(int)bf16x2_tagged(a0[0], a0[1], tagmask), (int)bf16x2_tagged(a0[2], a0[3], tagmask),
                               (int)bf16x2_tagged(a1[0], a1[1], tagmask), (int)bf16x2_tagged(a1[2], a1[3], tagmask)};
              if constexpr (decltype(PLAIN)::value) store_b128(rs_ring, offp[k], v);
              else store_sc1_b128(rs_ring, offp[k], v);
            }
          }
        };
        if (plain) publish(std::true_type{});
        else publish(std::false_type{});
      }
    }
  } else {
    for (int s = a.steps - 1; s >= 0; --s) {
      mw_put(s);
      if (s + 2 < a.steps) mw_store(s + 2);
      if (s >= 1) mw_load(s - 1);
      lds_barrier();                                                        // #1
      if (s_abort) break;
      lds_barrier();                                                        // #2
    }
  }
  __syncthreads();
  if (wave == BMEM8 && !s_abort) {
    if (a.steps >= 2) mw_store(1);
    if (a.steps >= 1) mw_store(0);
  }
  // bias gradients: the epilogue waves' rows reduced through LDS, one read-modify-write per
  // (gate, unit) of the workgroup's own [bg] partial row (layout of rnnrs_bwd_kernel)
  if (a.dbx_part[dir] != nullptr && !s_abort) {
    constexpr int BW = (G3 + 1) * UPW8;
    static_assert(BMW8 * ROWS * (UPW8 + 1) >= ROWS8 * BW, "bias reduction does not fit the LDS scratch");
    float* bred = &red_s[0][0][0];
    if (wave < BEW8) {
#pragma unroll
      for (int i = 0; i < EPT; ++i) {
        const int row = wave + BEW8 * i;
#pragma unroll
        for (int g = 0; g < G3; ++g) bred[row * BW + g * UPW8 + lane] = sbx[i][g];
        bred[row * BW + G3 * UPW8 + lane] = sbh[i];
      }
    }
    __syncthreads();
    for (int q = tid; q < BW; q += BTH8) {
      float sum = 0.f;
      for (int r = 0; r < ROWS8; ++r) sum += bred[r * BW + q];
      const int g = q / UPW8, c = q % UPW8;
      const size_t base = (size_t)bg * GH + u0 + c;
      if (g < G3) {
        a.dbx_part[dir][base + (size_t)g * H] += sum;
        if (a.dbh_part[dir] != nullptr && g < G3 - 1) a.dbh_part[dir][base + (size_t)g * H] += sum;
      } else if (a.dbh_part[dir] != nullptr) {
        a.dbh_part[dir][base + (size_t)(G3 - 1) * H] += sum;
      }
    }
  }
}

// e4m3 TRANSPOSED copy q[c][r] = x[r][c] / 2^e of a bf16 [rows][cols] tensor (the BPTT's U^T),
// with e from *amax as quant_pow2_kernel (uexp written as 127 + e). 64 x 64 tiles through LDS.
__global__ __launch_bounds__(256) void quant_pow2_t_kernel(const bf16_t* __restrict__ x, int rows, int cols,
                                                           const unsigned* __restrict__ amax,
                                                           unsigned char* __restrict__ q, int* __restrict__ uexp) {
  __shared__ float t_s[64][65];
  const float am = __uint_as_float(*amax);
  int e = 0;
  if (am > 0.f) {
    e = (int)ceilf(log2f(am / 448.f));
    if (ldexpf(448.f, e) < am) ++e;
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *uexp = 127 + e;
  const float inv = ldexpf(1.f, -e);
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i >> 6, c = i & 63;
    t_s[r][c] = (r0 + r < rows && c0 + c < cols) ? bf2f(x[(size_t)(r0 + r) * cols + c0 + c]) : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int c = i >> 6, r = i & 63;
    if (c0 + c < cols && r0 + r < rows) q[(size_t)(c0 + c) * rows + r0 + r] = (unsigned char)f2e4m3(t_s[r][c] * inv);
  }
}

// amax of |x| over a bf16 tensor into *amax (as float bits; zeroed by the caller)
__global__ __launch_bounds__(256) void amax_bf16_kernel(const bf16_t* __restrict__ x, long long n,
                                                        unsigned* __restrict__ amax) {
  float m = 0.f;
  const long long stride = (long long)gridDim.x * 256 * 8;
  for (long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 8; i < n; i += stride) {
    if (i + 8 <= n) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + i);
#pragma unroll
      for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf(bf2f((bf16_t)v[k])));
    } else {
      for (long long k = i; k < n; ++k) m = fmaxf(m, fabsf(bf2f(x[k])));
    }
  }
  // one atomic per workgroup (one per wave serialised ~4k atomics on one L2 line: 50 us for a
  // 10 MB U at config 5)
  __shared__ float wm[4];
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(amax, __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));   // non-negative floats order as uints
}

// e4m3 copy x / 2^e with the smallest e such that amax / 2^e <= 448; uexp = 127 + e (E8M0)
__global__ __launch_bounds__(256) void quant_pow2_kernel(const bf16_t* __restrict__ x, long long n,
                                                         const unsigned* __restrict__ amax,
                                                         unsigned char* __restrict__ q, int* __restrict__ uexp) {
  const float am = __uint_as_float(*amax);
  int e = 0;
  if (am > 0.f) {
    e = (int)ceilf(log2f(am / 448.f));
    if (ldexpf(448.f, e) < am) ++e;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *uexp = 127 + e;
  const float inv = ldexpf(1.f, -e);
  const long long stride = (long long)gridDim.x * 256 * 8;
  for (long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 8; i < n; i += stride) {
    if (i + 8 <= n) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + i);
      unsigned w[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        int lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f((bf16_t)v[4 * h]) * inv, bf2f((bf16_t)v[4 * h + 1]) * inv, 0,
                                                 false);
        lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f((bf16_t)v[4 * h + 2]) * inv, bf2f((bf16_t)v[4 * h + 3]) * inv, lo,
                                             true);
        w[h] = (unsigned)lo;
      }
      *reinterpret_cast<uint2*>(q + i) = make_uint2(w[0], w[1]);
    } else {
      for (long long k = i; k < n; ++k) q[k] = (unsigned char)f2e4m3(bf2f(x[k]) * inv);
    }
  }
}

// ---- U of both directions in one pass each (config 5's fp8 layers): per-block |U| maxima, then
// e4m3 copies in both layouts the recurrences read (row-major for the forward, transposed for
// the BPTT, which keeps the forward's) from one read of U. No atomics and no zeroed scratch:
// the quantiser reduces the QU_NB partials of its direction itself.
constexpr int QU_NB = 256;

__global__ __launch_bounds__(256) void amax_parts_kernel(const bf16_t* __restrict__ x0, const bf16_t* __restrict__ x1,
                                                         long long n, float* __restrict__ part) {
  const bf16_t* x = blockIdx.y ? x1 : x0;
  float m = 0.f;
  for (long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 8; i < n; i += (long long)QU_NB * 256 * 8) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + i);
#pragma unroll
    for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf(bf2f((bf16_t)v[k])));
  }
  __shared__ float wm[4];
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.y * QU_NB + blockIdx.x] = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
}

// 64 x 64 tiles of direction blockIdx.z's [rows][cols] U: q row-major, qt [cols][rows] (either
// may be null), both / 2^e with e from the direction's amax (uexp[d] = 127 + e, E8M0)
__global__ __launch_bounds__(256) void quant_u_kernel(const bf16_t* __restrict__ x0, const bf16_t* __restrict__ x1,
                                                      int rows, int cols, const float* __restrict__ part,
                                                      unsigned char* q0, unsigned char* q1, unsigned char* qt0,
                                                      unsigned char* qt1, int* __restrict__ uexp) {
  const int d = blockIdx.z;
  const bf16_t* x = d ? x1 : x0;
  unsigned char* q = d ? q1 : q0;
  unsigned char* qt = d ? qt1 : qt0;
  __shared__ float wm[4];
  __shared__ unsigned char t_s[64][64 + 16];
  float m = part[d * QU_NB + threadIdx.x];               // QU_NB == blockDim.x
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  const int eb = e8m0_bits(__float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) uexp[d] = eb;
  const float inv = __uint_as_float((unsigned)(254 - eb) << 23);          // 2^-(eb - 127)
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int k = threadIdx.x; k < 512; k += 256) {         // chunk k: row k >> 3, columns 8 (k & 7) ..
    const int r = k >> 3, c = (k & 7) * 8;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + (size_t)(r0 + r) * cols + c0 + c);
    unsigned w[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f((bf16_t)v[4 * h]) * inv, bf2f((bf16_t)v[4 * h + 1]) * inv, 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f((bf16_t)v[4 * h + 2]) * inv, bf2f((bf16_t)v[4 * h + 3]) * inv, lo, true);
      w[h] = (unsigned)lo;
    }
    if (q) *reinterpret_cast<uint2*>(q + (size_t)(r0 + r) * cols + c0 + c) = make_uint2(w[0], w[1]);
    *reinterpret_cast<uint2*>(&t_s[r][c]) = make_uint2(w[0], w[1]);
  }
  if (qt) {
    __syncthreads();
    const int c = threadIdx.x >> 2, rr = (threadIdx.x & 3) * 16;    // qt row c0 + c, 16 rows from rr
    unsigned w4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w4[j] = (unsigned)t_s[rr + 4 * j][c] | ((unsigned)t_s[rr + 4 * j + 1][c] << 8) |
              ((unsigned)t_s[rr + 4 * j + 2][c] << 16) | ((unsigned)t_s[rr + 4 * j + 3][c] << 24);
    *reinterpret_cast<uint4*>(qt + (size_t)(c0 + c) * rows + r0 + rr) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
  }
}

}  // namespace

extern "C" {

struct DS2RnnF8 {
  int T, N, NP, H, BG, R, steps, gstride, ndir, xcd_map;
  const int* lens;
  const void* gx;
  const void* U8[2];
  const int* uexp;
  const float* bh[2];
  void* y[2];
  void* hq[2];
  void* hx[2];
  float* hsave[2];
  float* gates[2];
  unsigned* census;
  unsigned* err;
  long long timeout;
};

// k-steps of 128 per wave (K half) and how many of them live in LDS, for H
static int f8_kb(int H) { return H / 256; }
static int f8_kl(int kb) { return kb > 3 ? kb - 3 : 0; }

int ds2_rnnf8_supported(int H, int N, int ndir) {
  if (H % 256 != 0 || H / 64 > 32 || H / 256 > 6 || H / 256 < 1) return 0;
  const int BG = 8 / ndir;
  const int R = (N + BG - 1) / BG;
  return R <= ROWS8 ? 1 : 0;
}

size_t ds2_rnnf8_smem(int H) { return (size_t)f8_kl(f8_kb(H)) * G8W * G3 * 64 * sizeof(i32x8); }

int ds2_rnnf8_fwd(const DS2RnnF8* d, hipStream_t st) {
  if (d->H % 256 != 0 || d->R < 1 || d->R > ROWS8 || d->NP != d->BG * d->R || d->H / UPW8 > 32) return -40;
  XF8 a;
  a.T = d->T; a.N = d->N; a.NP = d->NP; a.H = d->H; a.P = d->H / UPW8; a.BG = d->BG; a.R = d->R;
  a.steps = d->steps; a.gstride = d->gstride; a.ngroups = d->ndir * d->BG;
  a.xcd_map = (d->xcd_map & 1) && a.ngroups <= 8;
  a.lens = d->lens; a.gx = (const bf16_t*)d->gx; a.uexp = d->uexp;
  for (int i = 0; i < 2; ++i) {
    a.U8[i] = (const unsigned char*)d->U8[i]; a.bh[i] = d->bh[i]; a.y[i] = (bf16_t*)d->y[i];
    a.hq[i] = (unsigned char*)d->hq[i]; a.hx[i] = (bf16_t*)d->hx[i]; a.hsave[i] = d->hsave[i];
    a.gates[i] = d->gates[i];
  }
  a.census = d->census; a.err = d->err; a.timeout = d->timeout;
  if (d->steps <= 0) return 0;
  const int grid = a.xcd_map ? 8 * a.P : a.ngroups * a.P;
  // generation 2 where it is instantiated (H = 1024, 1280); generation 1 for the other widths
  switch (d->H / 128) {
    case 8: hipLaunchKernelGGL((rnnf8h_fwd_kernel<8>), dim3(grid), dim3(F8TH), 0, st, a); return (int)hipGetLastError();
    case 10: hipLaunchKernelGGL((rnnf8h_fwd_kernel<10>), dim3(grid), dim3(F8TH), 0, st, a); return (int)hipGetLastError();
    default: break;
  }
  const int kb = f8_kb(d->H);
  const size_t smem = ds2_rnnf8_smem(d->H);
  switch (kb) {
#define DS2_F8(K)                                                                                     \
  case K: {                                                                                           \
    auto kern = rnnf8_fwd_kernel<K, (K > 3 ? K - 3 : 0)>;                                             \
    if (smem > 0)                                                                                     \
      DS2_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem)); \
    hipLaunchKernelGGL(kern, dim3(grid), dim3(F8TH), smem, st, a);                                    \
    break;                                                                                            \
  }
    DS2_F8(1) DS2_F8(2) DS2_F8(3) DS2_F8(4) DS2_F8(5) DS2_F8(6)
#undef DS2_F8
    default: return -41;
  }
  return (int)hipGetLastError();
}

struct DS2RnnF8B {
  int T, N, NP, H, BG, R, steps, gstride, ndir, xcd_map;
  const int* lens;
  const void* dy;
  const void* U8T[2];
  const int* uexp;
  const float* hsave[2];
  const float* gates[2];
  void* dgh[2];
  void* dgx;
  void* ring[2];
  float* dbx_part[2];
  float* dbh_part[2];
  float dgx_scale;
  unsigned* census;
  unsigned* err;
  long long timeout;
};

// fp8 BPTT geometry: H = 256 k, k = 1..5 (P = H/64 <= 20 workgroups per group), R <= 8
int ds2_rnnf8_bwd_supported(int H, int N, int ndir) {
  if (H % 256 != 0 || H / 256 < 1 || H / 256 > 5) return 0;
  const int BG = 8 / ndir;
  return (N + BG - 1) / BG <= ROWS8 ? 1 : 0;
}

// ring words (uint32) of one direction: [3][BG][P][H/32][R][4] granules of 4 words
long long ds2_rnnf8_ring_words(int H, int BG, int R) { return 3LL * BG * (H / 64) * (H / 32) * R * 16; }

int ds2_rnnf8_bwd(const DS2RnnF8B* d, hipStream_t st) {
  if (!ds2_rnnf8_bwd_supported(d->H, d->N, d->ndir) || d->R < 1 || d->R > ROWS8 || d->NP != d->BG * d->R ||
      d->BG * d->ndir > 8)
    return -40;
  XF8B a;
  a.T = d->T; a.N = d->N; a.NP = d->NP; a.H = d->H; a.P = d->H / UPW8; a.BG = d->BG; a.R = d->R;
  a.steps = d->steps; a.gstride = d->gstride; a.ngroups = d->ndir * d->BG;
  a.xcd_map = (d->xcd_map & 1) && a.ngroups <= 8;
  a.lens = d->lens; a.dy = (const bf16_t*)d->dy; a.uexp = d->uexp;
  for (int i = 0; i < 2; ++i) {
    a.U8T[i] = (const unsigned char*)d->U8T[i]; a.hsave[i] = d->hsave[i]; a.gates[i] = d->gates[i];
    a.dgh[i] = (bf16_t*)d->dgh[i]; a.ring[i] = (unsigned*)d->ring[i];
    a.dbx_part[i] = d->dbx_part[i]; a.dbh_part[i] = d->dbh_part[i];
  }
  a.dgx = (bf16_t*)d->dgx; a.dgx_scale = d->dgx_scale;
  a.census = d->census; a.err = d->err; a.timeout = d->timeout;
  if (d->steps <= 0) return 0;
  const int grid = a.xcd_map ? 8 * a.P : a.ngroups * a.P;
  switch (d->H / 256) {
    case 1: hipLaunchKernelGGL((rnnf8_bwd_kernel<4, 2>), dim3(grid), dim3(BTH8), 0, st, a); break;
    case 2: hipLaunchKernelGGL((rnnf8_bwd_kernel<6, 2>), dim3(grid), dim3(BTH8), 0, st, a); break;
    case 3: hipLaunchKernelGGL((rnnf8_bwd_kernel<8, 2>), dim3(grid), dim3(BTH8), 0, st, a); break;
    case 4: hipLaunchKernelGGL((rnnf8_bwd_kernel<10, 4>), dim3(grid), dim3(BTH8), 0, st, a); break;
    case 5: hipLaunchKernelGGL((rnnf8_bwd_kernel<12, 4>), dim3(grid), dim3(BTH8), 0, st, a); break;
    default: return -41;
  }
  return (int)hipGetLastError();
}

// U of ndir directions ([rows][cols] bf16 each, rows and cols multiples of 64): row-major q[d]
// and / or transposed qt[d] e4m3 copies with one power-of-two scale per direction, uexp[d] =
// 127 + e; part: ndir * 256 floats of scratch. Two launches for all directions and layouts.
int ds2_fp8_quant_u(int ndir, const void* const* x, int rows, int cols, void* const* q, void* const* qt, int* uexp,
                    float* part, hipStream_t st) {
  if (ndir < 1 || ndir > 2 || rows <= 0 || cols <= 0 || rows % 64 || cols % 64) return (int)hipErrorInvalidValue;
  const bf16_t* x1 = (const bf16_t*)x[ndir - 1];
  hipLaunchKernelGGL(amax_parts_kernel, dim3(QU_NB, ndir), dim3(256), 0, st, (const bf16_t*)x[0], x1,
                     (long long)rows * cols, part);
  hipLaunchKernelGGL(quant_u_kernel, dim3(cols / 64, rows / 64, ndir), dim3(256), 0, st, (const bf16_t*)x[0], x1,
                     rows, cols, part, (unsigned char*)q[0], (unsigned char*)q[ndir - 1], (unsigned char*)qt[0],
                     (unsigned char*)qt[ndir - 1], uexp);
  return (int)hipGetLastError();
}

// transposed per-tensor power-of-two e4m3 quantisation (the BPTT's U^T): q [cols][rows]
int ds2_fp8_quant_pow2_t(const void* x, int rows, int cols, void* q, int* uexp, unsigned* amax, hipStream_t st) {
  const long long n = (long long)rows * cols;
  if (n <= 0) return 0;
  long long blocks = (n + 256 * 8 - 1) / (256 * 8);
  if (blocks > 512) blocks = 512;
  DS2_HIP_CHECK(hipMemsetAsync(amax, 0, sizeof(unsigned), st));
  hipLaunchKernelGGL(amax_bf16_kernel, dim3((int)blocks), dim3(256), 0, st, (const bf16_t*)x, n, amax);
  hipLaunchKernelGGL(quant_pow2_t_kernel, dim3((cols + 63) / 64, (rows + 63) / 64), dim3(256), 0, st,
                     (const bf16_t*)x, rows, cols, amax, (unsigned char*)q, uexp);
  return (int)hipGetLastError();
}

// per-tensor power-of-two e4m3 quantisation of a bf16 tensor (amax scratch: one zeroed uint)
int ds2_fp8_quant_pow2(const void* x, long long n, void* q, int* uexp, unsigned* amax, hipStream_t st) {
  if (n <= 0) return 0;
  long long blocks = (n + 256 * 8 - 1) / (256 * 8);
  if (blocks > 1024) blocks = 1024;
  const long long ablocks = blocks > 512 ? 512 : blocks;      // 2 per CU: enough to stream 10 MB
  DS2_HIP_CHECK(hipMemsetAsync(amax, 0, sizeof(unsigned), st));
  hipLaunchKernelGGL(amax_bf16_kernel, dim3((int)ablocks), dim3(256), 0, st, (const bf16_t*)x, n, amax);
  hipLaunchKernelGGL(quant_pow2_kernel, dim3((int)blocks), dim3(256), 0, st, (const bf16_t*)x, n, amax,
                     (unsigned char*)q, uexp);
  return (int)hipGetLastError();
}

}  // extern "C"
