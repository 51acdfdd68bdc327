// Persistent bidirectional recurrence on XCD-local workgroup groups with a sentinel hand-off.
// Kernels in this file (host dispatch at the end):
//   rnnx_fwd_kernel   generation 2 forward (fallback geometries)
//   rnnq_fwd_kernel   generation 4 forward: 2 unit halves x 4 K-quarters (GRU H = 1280, ReLU)
//   rnne_fwd_kernel   generation 5 GRU forward (H <= 1024): 8 K-eighths, one poller per granule
//   rnnrs_bwd_kernel  generation 3 BPTT: reduce-scatter of tagged-bf16 partials
//   rnnw_fwd_kernel / rnnw_bwd_kernel   64-unit one-gate layers wider than an XCD (ReLU-1760)
// The notes below describe the shared exchange protocol (introduced with generation 2).
//
// Reference behaviour: src/custom_ops.py:36-96 (CustomRNNCell2 + stacked_brnn through
// tf.nn.bidirectional_dynamic_rnn: outputs zero past each length, the backward direction
// reversed within each utterance, directions summed by the caller). Same buffers and
// numerics as rnn_persistent.hip (generation 1, kept as the step-mode fallback); what
// changed is how the per-step state crosses workgroups, measured with
// tools/exchange_bench.hip on MI355X (all-gather of one step, no math):
//
//   gen-1: 4 groups x 50 WGs, flag per producer, sc1 payload      4.4 us/step
//   gen-2: 8 groups x 25 WGs, sentinel payload, XCD-local, plain   1.1 us/step
//
//  * Group = (direction, batch group of R <= 16*MT rows); a workgroup owns UPW = 32 hidden
//    units of its group (all gates), so a group is P = H/32 workgroups. With <= 8 groups,
//    group = blockIdx % 8: under the observed round-robin dispatch a group then shares
//    ONE XCD, its exchange stays in that XCD's L2, and its producers can store plain
//    (L2-resident) instead of write-through. Placement is never assumed: a start-up census
//    (every member publishes its HW_REG_XCC_ID) decides per group; a group that straddles
//    XCDs stores write-through (sc1), which is correct for any placement.
//  * Sentinel hand-off: the exchange buffer (one slot per step, never reused within a
//    launch) is pre-filled with 0xFFFF (a bf16 NaN that the producers never store: NaN
//    results are canonicalised to 0x7FC0). Producers store 16-B granules and move on: no
//    drain, no flag. Consumers load each granule with sc1 (L1-bypassing) loads and spin on
//    it until none of its 8 halves is the sentinel, staging it in LDS. 16-B stores were
//    observed untorn on gfx950; checking all 8 halves keeps the protocol correct even if
//    a granule landed in pieces (a half is only ever sentinel or final).
//  * Forward: gh = h_{t-1} . U^T (M = rows, N = 3*32, K = H) with U's slice resident in
//    VGPRs as MFMA B fragments; one wave per 16-column N-tile runs the whole K from the
//    LDS A tile, so there is no cross-wave reduction.
//  * Backward (BPTT): dh = dgh_{t+1} . U[:, slice] (N = 32, K = 3H) with U's columns
//    resident, K split over the 8 waves, reduced through LDS.
//  * Every spin is bounded by an s_memrealtime timeout that sets an error word and
//    aborts the launch, so a grid that is not co-resident cannot hang the GPU.
#include <type_traits>

#include "common.h"

using namespace ds2;

namespace {

constexpr int CELL_RELU = 0;
constexpr int CELL_GRU = 1;
constexpr float RELU_CAP = 20.0f;
constexpr int UPW = 32;          // hidden units per workgroup
constexpr int NWV = 8;           // waves per workgroup
constexpr int NTH = NWV * 64;

struct XFwd {
  int T, N, NP, H, P, BG, R, steps, gstride, ngroups, xcd_map, knobs;
  const int* lens;
  const bf16_t* gx;
  const bf16_t* U[2];
  const float* bh[2];
  bf16_t* y[2];
  bf16_t* ysum;           // gen 4, two directions: fused direction sum [T][N][H], sentinel-filled
  bf16_t* hx[2];          // [steps+1][NP][H]: slot 0 = h0, slots 1.. pre-filled with sentinel
  float* hsave[2];
  float* gates[2];
  unsigned* census;       // [ngroups * P] pre-filled 0xFFFFFFFF
  unsigned* err;
  long long timeout;
  unsigned long long* stamps;   // optional [grid][8] phase cycle sums (diagnostics)
};

// Phase stamps (diagnostics; a null stamps pointer costs one uniform branch per phase).
struct Stamps {
  unsigned long long acc[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long prev = 0;
  bool on;
  __device__ explicit Stamps(bool o) : on(o) {}
  __device__ __forceinline__ void mark(int i) {
    if (!on) return;
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    if (prev && i >= 0) acc[i] += t - prev;
    prev = t;
  }
  __device__ __forceinline__ void store(unsigned long long* dst, int base) {
    if (!on) return;
    for (int k = 0; k < 6; ++k) dst[(size_t)blockIdx.x * 8 + base + k] = acc[k];
  }
};

// compile-time-off variant: the stamp accumulators would otherwise hold ~14 VGPRs of every
// wave for the whole launch (enough to push a 3-waves-per-SIMD kernel into spilling)
struct NoStamps {
  unsigned long long acc[6];
  bool on = false;
  __device__ explicit NoStamps(bool) {}
  __device__ __forceinline__ void mark(int) {}
  __device__ __forceinline__ void store(unsigned long long*, int) {}
};

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

// bf16 rounding that never produces the sentinel 0xFFFF (any NaN -> canonical 0x7FC0)
__device__ __forceinline__ bf16_t f2bf_x(float f) {
  const bf16_t b = f2bf(f);
  return ((b & 0x7f80u) == 0x7f80u && (b & 0x7fu)) ? (bf16_t)0x7fc0 : b;
}

// no 16-bit half of the granule is the sentinel 0xFFFF: SWAR "has a zero half" test on the
// complement, (~w - 0x00010001) & w & 0x80008000 (a few VALU ops per dword; this check runs
// on every poll of the latency-critical exchange)
__device__ __forceinline__ bool granule_ready(i32x4 v) {
  unsigned any = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const unsigned w = (unsigned)v[i];
    any |= (~w - 0x00010001u) & w & 0x80008000u;
  }
  return any == 0;
}

__device__ __forceinline__ void store_granule(bool plain, __amdgpu_buffer_rsrc_t rs, bf16_t* base, unsigned off,
                                              i32x4 v) {
  (void)base;
  if (plain) {
    store_b128(rs, off, v);
  } else {
    store_sc1_b128(rs, off, v);
  }
}

// Group role. xcd_map (host-chosen: <= 8 groups of <= CUs/8 members): group =
// blockIdx % 8, so under round-robin dispatch a group shares one XCD; otherwise groups
// are contiguous block ranges. Returns false for surplus blocks (no role).
__device__ __forceinline__ bool take_role(int xcd_map, int ngroups, int P, int& grp, int& mem) {
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

// Every member of the group publishes its XCC id; the group is "local" iff all agree.
// Runs on wave 0; returns 1 (local), 0 (spread) or -1 (timeout).
__device__ int group_census(unsigned* census, int grp, int mem, int P, long long timeout, unsigned* err) {
  const int lane = threadIdx.x & 63;
  unsigned* c = census + (size_t)grp * P;
  if (lane == 0) __hip_atomic_store(c + mem, xcc_id(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  while (true) {
    bool ready = true;
    unsigned first = 0xffffffffu;
    bool same = true;
    for (int q = lane; q < P; q += 64) {
      const unsigned v = __hip_atomic_load(c + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ready = ready && (v != 0xffffffffu);
      if (q == lane) first = v;
      same = same && (v == first);
    }
    if (__all(ready)) {
      const unsigned x0 = __shfl(first, 0, 64);
      const bool all_same = __all(same && (lane >= P || first == x0));
      return all_same ? 1 : 0;
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
      if (lane == 0) atomicOr(err, 2u);
      return -1;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// ------------------------------------------------------------------------------------
// Workgroup roles (8 waves):
//   waves 0..6  MFMA waves, K split 7 ways (k-step ks = wave + 7*kk). A k-step's 32 columns
//               are ONE producer's 32-unit chunk (forward) or one gate-chunk (backward), so
//               each lane's MFMA A fragment (row = lane % 16, 8 columns) is exactly one 16-B
//               exchange granule: the wave polls its fragments straight into registers
//               (sentinel spin per lane) and issues each k-step's MFMAs as soon as it is
//               ready. No LDS staging of the exchanged state, no gather barrier.
//   waves 0..3  cell epilogue (EPT elements each) + the critical 16-B exchange stores;
//   wave  7     memory wave: per-step inputs two steps ahead into an LDS ring, per-step
//               outputs out of a double-buffered LDS staging area. Its loads and stores
//               never sit in another wave's vmcnt queue (vmcnt retires in order per wave).
// One LDS-only barrier per step (partials ready -> epilogue); partials are double-buffered
// by step parity because waves 4..6 run into the next step while 0..3 are in the epilogue.
// ------------------------------------------------------------------------------------
constexpr int EW = 4;             // epilogue waves
constexpr int ETH = EW * 64;
constexpr int MW = 7;             // MFMA waves
constexpr int MEMW = 7;           // memory wave

// Poll this lane's A-fragment granules (one per k-step) until none carries the sentinel,
// issuing the k-step's MFMAs as each becomes ready. need = this lane's row is a real row.
// Returns false on timeout.
template <int KB, int NT, int CH, typename MfmaFn>
__device__ __forceinline__ bool poll_mfma(__amdgpu_buffer_rsrc_t rs, const unsigned (&off)[KB], const bool (&kval)[KB],
                                          bool need, long long timeout, MfmaFn&& mfma) {
  // at most CH granules in flight per lane (a register budget: the U slice already holds
  // most of the VGPRs); the load for k-step kk+CH is issued before k-step kk is waited on
  i32x4 v[KB];
#pragma unroll
  for (int kk = 0; kk < (KB < CH ? KB : CH); ++kk) v[kk] = load_sc1_b128(rs, off[kk]);
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  bool ok_all = true;
#pragma unroll
  for (int kk = 0; kk < KB; ++kk) {
    if (kk + CH < KB) v[kk + CH] = load_sc1_b128(rs, off[kk + CH]);
    if (!kval[kk]) continue;                       // wave-uniform: k-step beyond K
    while (true) {
      const bool ok = !need || granule_ready(v[kk]);
      if (__all(ok)) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) { ok_all = false; break; }
      __builtin_amdgcn_s_sleep(1);
      if (!ok) v[kk] = load_sc1_b128(rs, off[kk]);
    }
    const i32x4 z = {0, 0, 0, 0};
    mfma(kk, __builtin_bit_cast(bf16x8, need ? v[kk] : z));
  }
  return ok_all;
}

// Same contract as poll_mfma, but every granule is loaded up front and each retry round
// re-issues ALL granules not yet consumed, back to back (no divergent branch around a load,
// so no vmcnt(0) between them): a round costs ONE L2 round trip however many producers are
// late. (poll_mfma reloads only the granule it is waiting on, so k-steps whose first load
// came back early-stale cost one serial round trip each.) The MFMAs still run in k order,
// so the accumulation order — and the result — is deterministic.
// Explicit vmcnt(0) at the poll's exits. Every load of the poll has been waited for there
// already (the last check consumed it), but the CFG also has an edge from a re-issue to the
// exit, so the waitcnt pass assumed loads in flight and put a vmcnt(0) at the head of the
// NEXT step — behind the step's own h store, whose write acknowledgement then delayed the
// next step's first poll by an L2 round trip. A counted wait here costs nothing (nothing is
// in flight) and tells the pass so.
__device__ __forceinline__ void drain_vm() {
#ifndef DS2_NO_DRAIN          // A/B: build.py --variant nodrain -D DS2_NO_DRAIN
  __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
}

template <int KB, typename MfmaFn>
__device__ __forceinline__ bool poll_mfma_par(__amdgpu_buffer_rsrc_t rs, const unsigned (&off)[KB],
                                              const bool (&kval)[KB], long long timeout, int nap, MfmaFn&& mfma) {
  i32x4 v[KB];
#pragma unroll
  for (int kk = 0; kk < KB; ++kk) v[kk] = load_sc1_b128(rs, off[kk]);
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned done = 0;                     // wave-uniform: k-steps consumed (an in-order prefix)
  constexpr unsigned FULL = (1u << KB) - 1u;
  while (true) {
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
      if (done == (1u << kk) - 1u) {
        if (!kval[kk]) {
          done |= 1u << kk;
        } else if (__all(granule_ready(v[kk]))) {
          mfma(kk, __builtin_bit_cast(bf16x8, v[kk]));
          done |= 1u << kk;
        }
      }
    }
    if (done == FULL) { drain_vm(); return true; }
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) { drain_vm(); return false; }
    if (nap == 1) __builtin_amdgcn_s_sleep(1);           // retry back-off (0: busy re-poll)
    else if (nap == 2) __builtin_amdgcn_s_sleep(3);
#pragma unroll
    for (int kk = 0; kk < KB; ++kk)
      if (!(done & (1u << kk))) v[kk] = load_sc1_b128(rs, off[kk]);
  }
}

// ------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------
template <int CELL, int MT, int KB>
__global__ __launch_bounds__(NTH) void rnnx_fwd_kernel(XFwd a) {
  static_assert(MT == 1, "16-row tiles");
  constexpr int G = (CELL == CELL_GRU) ? 3 : 1;
  constexpr int ROWS = 16;
  constexpr int EPT = ROWS * UPW / ETH;           // 2
  constexpr int GC = G * UPW;                     // gate columns of the workgroup
  constexpr int NTL = 2 * G;                      // 16-column N-tiles
  constexpr int RG = ROWS * G * (UPW / 8);        // gx granules per step (upper bound)
  constexpr int RGL = (RG + 63) / 64;             // ... per memory-wave lane
  constexpr int OPL = ROWS * UPW / 64;            // output elements per memory-wave lane
  __shared__ float red_s[2][MW][ROWS][GC + 1];    // K-split partials, by step parity
  __shared__ float gxr_s[2][ROWS][GC];            // input-projection ring (memory wave -> epilogue)
  __shared__ float oh_s[2][ROWS][UPW];            // output staging, by step parity
  __shared__ float oy_s[2][ROWS][UPW];
  __shared__ float4 og_s[(CELL == CELL_GRU) ? 2 : 1][(CELL == CELL_GRU) ? ROWS : 1][UPW];
  __shared__ int len_s[ROWS];                     // utterance length per row (0 = padding row)
  __shared__ float bh_s[G][UPW];                  // recurrent bias slice (GRU)
  __shared__ int s_mode, s_abort;

  int grp, mem;
  if (!take_role(a.xcd_map, a.ngroups, a.P, grp, mem)) return;
  DS2_DCHECK(grp < a.ngroups && mem < a.P && a.NP >= a.BG * a.R && a.R <= 16);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, KS = H / 32, N = a.N, NP = a.NP, R = a.R;
  const int bg = grp % a.BG, dir = grp / a.BG;
  const int r0 = bg * R, u0 = mem * UPW;
  if (tid < ROWS) len_s[tid] = (tid < R && r0 + tid < N) ? a.lens[r0 + tid] : 0;
  if (tid < G * UPW)
    bh_s[tid / UPW][tid % UPW] = (CELL == CELL_GRU && a.bh[dir]) ? a.bh[dir][(tid / UPW) * H + u0 + tid % UPW] : 0.f;
  if (wave == 0) {
    int m = group_census(a.census, grp, mem, a.P, a.timeout, a.err);
    if ((a.knobs & 32768) && m > 0) m = 0;      // knob 32768: force write-through (timing)
    if (lane == 0) { s_mode = m; s_abort = (m < 0); }
  }

  // resident U fragments of the MFMA waves: B[k][c] = U[g*H + u0 + 16*half + c][k]
  bf16x8 uf[KB][NTL];
  bool kval[KB];
  {
    const bf16_t* Ud = a.U[dir];
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
      const int ks = wave + kk * MW;
      kval[kk] = wave < MW && ks < KS;
#pragma unroll
      for (int t = 0; t < NTL; ++t) {
        const int g = t >> 1, half = t & 1;
        bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        if (kval[kk])
          v = *reinterpret_cast<const bf16x8*>(Ud + (size_t)(g * H + u0 + 16 * half + (lane & 15)) * H + ks * 32 +
                                               8 * (lane >> 4));
        uf[kk][t] = v;
      }
    }
  }
  const bool frag_row = (lane & 15) < R;          // this lane's A row is a real batch row

  // epilogue elements (waves 0..3): e = tid + i*ETH -> row = e / 32, unit = e % 32
  float hreg[EPT];
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int e = tid + i * ETH;
    const int row = e >> 5, c = e & 31;
    const bool live = tid < ETH && row < R;
    hreg[i] = live ? a.hsave[dir][(size_t)(r0 + row) * H + u0 + c] : 0.f;        // slot 0 = h0
  }
  __syncthreads();   // len_s / bh_s / census

  // memory wave: gx granule q -> (row, gate, 8-unit chunk)
  i32x4 gpre[RGL];
  const int NRG = R * G * (UPW / 8);
  auto mw_load = [&](int s) {          // issue this lane's gx loads for step s
#pragma unroll
    for (int j = 0; j < RGL; ++j) {
      const int q = lane + 64 * j;
      const int qq = q < NRG ? q : 0;
      const int row = qq / (G * 4), rem = qq - row * (G * 4), g = rem >> 2, c8 = rem & 3;
      const int b = min(r0 + row, N - 1);
      const int t = max(0, min((dir == 0) ? s : (len_s[row] - 1 - s), a.T - 1));
      gpre[j] = *reinterpret_cast<const i32x4*>(a.gx + ((size_t)t * N + b) * a.gstride + dir * G * H + g * H + u0 +
                                                c8 * 8);
    }
  };
  auto mw_put = [&](int s) {           // ring slot s&1 <- registers (masked past each length)
#pragma unroll
    for (int j = 0; j < RGL; ++j) {
      const int q = lane + 64 * j;
      if (q < NRG) {
        const int row = q / (G * 4), rem = q - row * (G * 4), g = rem >> 2, c8 = rem & 3;
        const bool act = s < len_s[row];
        const bf16x8 v = __builtin_bit_cast(bf16x8, gpre[j]);
#pragma unroll
        for (int k = 0; k < 8; ++k) gxr_s[s & 1][row][g * UPW + c8 * 8 + k] = act ? bf2f((bf16_t)v[k]) : 0.f;
      }
    }
  };
  auto mw_store = [&](int s) {          // outputs of step s from staging slot s&1
    float vh[OPL], vy[OPL];
    float4 vg[OPL];
#pragma unroll
    for (int j = 0; j < OPL; ++j) {       // all LDS reads first, then the stores
      const int e = lane + 64 * j;
      const int row = e >> 5, c = e & 31;
      vh[j] = oh_s[s & 1][row][c];
      vy[j] = oy_s[s & 1][row][c];
      if (CELL == CELL_GRU) vg[j] = og_s[(CELL == CELL_GRU) ? (s & 1) : 0][row][c];
    }
#pragma unroll
    for (int j = 0; j < OPL; ++j) {
      const int e = lane + 64 * j;
      const int row = e >> 5, c = e & 31;
      if (row < R) {
        const int b = r0 + row, u = u0 + c;
        a.hsave[dir][((size_t)(s + 1) * NP + b) * H + u] = vh[j];
        if (CELL == CELL_GRU) reinterpret_cast<float4*>(a.gates[dir])[((size_t)s * NP + b) * H + u] = vg[j];
        if (b < N) {
          const int L = len_s[row];
          const int t = (s < L) ? ((dir == 0) ? s : (L - 1 - s)) : s;
          a.y[dir][((size_t)t * N + b) * H + u] = f2bf(vy[j]);
        }
      }
    }
  };
  if (s_abort) return;
  if (wave == MEMW) mw_load(0);
  const bool plain = s_mode == 1;
  const unsigned hx_bytes = (unsigned)((size_t)(a.steps + 1) * NP * H * 2);
  bf16_t* hxd = a.hx[dir];
  const __amdgpu_buffer_rsrc_t rs_hx = make_rsrc(hxd, hx_bytes);
  Stamps st(a.stamps != nullptr && (wave == 0 || wave == MEMW) && lane == 0);
  // padding lanes of the 16-row fragment (row >= R) re-read row R-1: same cache line as a
  // real lane, so the wave's poll moves only R rows (knob 512: old per-lane rows, A/B)
  const int arow = (a.knobs & 512) ? min(r0 + (lane & 15), NP - 1) : r0 + min(lane & 15, R - 1);

  // The two roles run separate copies of the step loop (one LDS barrier per iteration in
  // both), so the memory wave's prefetch registers and the MFMA waves' resident U slice are
  // never live at the same time: the register budget is their max, not their sum.
  if (wave < MW) {
    for (int s = 0; s < a.steps; ++s) {
      st.mark(-1);
        // (M) poll this wave's A fragments of h_{s-1} (slot s) and accumulate its k-steps
        unsigned off[KB];
#pragma unroll
        for (int kk = 0; kk < KB; ++kk)
          off[kk] = (unsigned)((((size_t)s * NP + arow) * H + min(wave + kk * MW, KS - 1) * 32 + 8 * (lane >> 4)) * 2);
        f32x4 acc[NTL];
#pragma unroll
        for (int t = 0; t < NTL; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        const bool ok = poll_mfma<KB, NTL, KB>(rs_hx, off, kval, frag_row, a.timeout, [&](int kk, bf16x8 af) {
#pragma unroll
          for (int t = 0; t < NTL; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, uf[kk][t], acc[t], 0, 0, 0);
        });
        if (!ok) { s_abort = 1; atomicOr(a.err, 1u); }
        st.mark(0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = (lane >> 4) * 4 + j;
          if (row < R) {
#pragma unroll
            for (int t = 0; t < NTL; ++t) red_s[s & 1][wave][row][t * 16 + (lane & 15)] = acc[t][j];
          }
        }
      st.mark(1);
      lds_barrier();                                                        // partials ready
      st.mark(2);
      if (s_abort) break;
      // (E) cell epilogue; the exchange copy goes out first
      if (wave < EW) {
        unsigned hq[EPT];                  // this lane's new h (bf16 bits) per epilogue element
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
          const int e = tid + i * ETH;
          const int row = e >> 5, c = e & 31;
          hq[i] = 0u;
          if (row < R) {
            float pre[G], gxv[G];
#pragma unroll
            for (int g = 0; g < G; ++g) {
              float v = 0.f;
#pragma unroll
              for (int w = 0; w < MW; ++w) v += red_s[s & 1][w][row][g * UPW + c];
              pre[g] = v;
              gxv[g] = gxr_s[s & 1][row][g * UPW + c];
            }
            const bool act = s < len_s[row];
            float hn;
            float4 gsv = make_float4(0.f, 0.f, 0.f, 0.f);
            if (CELL == CELL_GRU) {
              const float ghn = pre[2] + bh_s[2][c];
              const float r = sigmoidf_(gxv[0] + pre[0] + bh_s[0][c]);
              const float z = sigmoidf_(gxv[1] + pre[1] + bh_s[1][c]);
              const float n = tanhf_(gxv[2] + r * ghn);
              hn = (1.f - z) * n + z * hreg[i];
              if (act) gsv = make_float4(r, z, n, ghn);
            } else {
              hn = fminf(fmaxf(gxv[0] + pre[0], 0.f), RELU_CAP);
            }
            const float hnew = act ? hn : hreg[i];
            hreg[i] = hnew;
            hq[i] = (unsigned)(unsigned short)f2bf_x(hnew);
            oh_s[s & 1][row][c] = hnew;
            oy_s[s & 1][row][c] = act ? hn : 0.f;
            if (CELL == CELL_GRU) og_s[(CELL == CELL_GRU) ? (s & 1) : 0][row][c] = gsv;
          }
        }
        // assemble each 16-B granule (8 consecutive units = 8 consecutive lanes of one row)
        // in its first lane with DPP row shifts instead of an LDS round trip + fence
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
          if ((i * ETH) / UPW >= R) break;                 // wave-uniform: no row of this pass
          const int e = tid + i * ETH;
          const int row = e >> 5, c = e & 31;
          const unsigned pr = hq[i] | ((unsigned)__builtin_amdgcn_update_dpp(0, (int)hq[i], 0x101, 0xf, 0xf, false) << 16);
          const int q1 = __builtin_amdgcn_update_dpp(0, (int)pr, 0x102, 0xf, 0xf, false);
          const int q2 = __builtin_amdgcn_update_dpp(0, (int)pr, 0x104, 0xf, 0xf, false);
          const int q3 = __builtin_amdgcn_update_dpp(0, (int)pr, 0x106, 0xf, 0xf, false);
          if ((c & 7) == 0 && row < R) {
            const i32x4 v = {(int)pr, q1, q2, q3};
            const unsigned off = (unsigned)((((size_t)(s + 1) * NP + r0 + row) * H + u0 + c) * 2);
            store_granule(plain, rs_hx, hxd, off, v);
          }
        }
      }
      st.mark(4);
    }
  } else {
    for (int s = 0; s < a.steps; ++s) {
      // memory wave: this step's inputs (loaded one step ago) into the ring, outputs of
      // step s-2 out of staging, next loads
      st.mark(-1);
      mw_put(s);
      if (s >= 2) mw_store(s - 2);
      if (s + 1 < a.steps) mw_load(s + 1);
      st.mark(0);
      lds_barrier();
      st.mark(1);
      if (s_abort) break;
    }
  }
  __syncthreads();
  if (wave == MEMW && !s_abort) {
    if (a.steps >= 2) mw_store(a.steps - 2);
    if (a.steps >= 1) mw_store(a.steps - 1);
  }
  if (wave == 0) { st.acc[5] = (unsigned long long)(s_mode + 10); st.store(a.stamps, 0); }
  if (wave == MEMW && st.on) { a.stamps[(size_t)blockIdx.x * 8 + 6] = st.acc[0]; a.stamps[(size_t)blockIdx.x * 8 + 7] = st.acc[1]; }
}

// ------------------------------------------------------------------------------------
// forward, generation 4: K-quarter split with a register-resident cell epilogue.
//
// Stamps of generation 2 at the headline (cycles/step): poll+MFMA 3.1k, partial store 0.4k,
// barrier 1.0k, epilogue 1.3k. Everything after the poll sits on the step's critical path,
// and most of it is the 7-way K reduction (24 partial floats written per lane, 21 read
// back per element) feeding 4 epilogue waves that run 2 elements each.
//  * 8 MFMA waves: wave w owns unit half uh = w & 1 (16 of the workgroup's 32 units, all G
//    gates, so G accumulator tiles) over K quarter kq = w >> 1 (k-steps kq, kq+4, ...).
//  * Transpose-reduce: element j of a 16x16 tile (row 4*(lane>>4)+j, unit lane&15) is
//    finalised by the wave with kq == j. Each wave stores the 3 elements it does not own
//    (3*G floats per lane, lane-contiguous: conflict-free), ONE barrier, then reads the
//    3 other quarters of its own element. Every lane then holds the full pre-activations
//    of exactly one (row, unit) and runs the cell in registers: h_{t-1} stays in the
//    lane across steps, gx and the recurrent bias are read before the exchange wait.
//  * Wave 8 is the memory wave: gx one step ahead into an LDS ring, outputs two steps
//    behind out of an LDS staging area (vmcnt retires in order per wave, so no MFMA wave
//    ever waits behind a bulk store).
// Same exchange protocol and buffers as generation 2 (sentinel hx slots, census-decided
// plain/write-through stores), so the host-side plan is shared.
// ------------------------------------------------------------------------------------
constexpr int QW = 8;             // MFMA waves of the generation-4 forward
constexpr int DS2_NARROW_CH = 0;  // KL == 0: 0 = all granules in flight with wave-wide re-poll (poll_mfma_par)
constexpr int DS2_WIDE_CH = 2;    // wide layers (KL > 0): granules in flight per lane, 0 = all (CH 2/3/4/6/8 measured 5.67/5.75/5.77/6.16/7.49 us/step at H = 1280)
constexpr int QTH = (QW + 1) * 64;

// KL > 0 (wide layers, H = 1280 GRU: 10 k-steps per wave): the LAST KL k-steps of each
// wave's U slice live in LDS instead of VGPRs (KB - KL register k-steps fit the 3-waves-per-
// SIMD budget that KB = 8..10 would spill), read back as one conflict-free ds_read_b128 per
// gate when the poll reaches that k-step.
template <int CELL, int KB, bool STAMPS, int KL = 0>
__global__ __launch_bounds__(QTH) void rnnq_fwd_kernel(XFwd a) {
  using StampT = typename std::conditional<STAMPS, Stamps, NoStamps>::type;
  constexpr int G = (CELL == CELL_GRU) ? 3 : 1;
  constexpr int KR = KB - KL;                     // k-steps with register-resident U
  static_assert(KL >= 0 && KR >= 1, "register k-steps");
  constexpr int ROWS = 16;
  constexpr int GP = G * UPW + 4;                 // gx ring row pitch: 4*GP = 16 (mod 64) banks
  constexpr int OP = UPW + 4;                     // output staging row pitch
  constexpr int RG = ROWS * G * (UPW / 8);        // gx granules per step (upper bound)
  constexpr int RGL = (RG + 63) / 64;
  __shared__ float red_s[2][2][4][3][G][64];      // [parity][uh][element j][source][gate][lane]
  __shared__ float gxr_s[2][ROWS][GP];
  __shared__ __attribute__((aligned(16))) float oh_s[2][ROWS][OP];
  __shared__ __attribute__((aligned(16))) float oy_s[2][ROWS][OP];
  __shared__ float4 og_s[(CELL == CELL_GRU) ? 2 : 1][(CELL == CELL_GRU) ? ROWS : 1][OP];
  __shared__ int len_s[ROWS];
  __shared__ int s_mode, s_abort;
  __shared__ bf16x8 ul_s[KL > 0 ? KL : 1][QW][G][64];   // LDS-resident U k-steps (KL > 0)

  int grp, mem;
  if (!take_role(a.xcd_map, a.ngroups, a.P, grp, mem)) return;
  DS2_DCHECK(grp < a.ngroups && mem < a.P && a.NP >= a.BG * a.R && a.R <= 16);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, KS = H / 32, N = a.N, NP = a.NP, R = a.R;
  const int bg = grp % a.BG, dir = grp / a.BG;
  const int r0 = bg * R, u0 = mem * UPW;
  const int uh = wave & 1, kq = wave >> 1;
  // Every wave finalises element j = kq of its tiles. (Measured: handing the R <= 8 rows'
  // elements to 4 waves only, one per SIMD, so the other 4 go straight back to polling, was
  // 10 % slower: the early pollers' retry loads compete with the epilogue.)
  const int erow = 4 * (lane >> 4) + (kq & 3);    // this lane's cell element (MFMA waves)
  const int ec = 16 * uh + (lane & 15);
  if (tid < ROWS) len_s[tid] = (tid < R && r0 + tid < N) ? a.lens[r0 + tid] : 0;
  if (wave == 0) {
    int m = group_census(a.census, grp, mem, a.P, a.timeout, a.err);
    if ((a.knobs & 32768) && m > 0) m = 0;      // knob 32768: force write-through (timing)
    if (lane == 0) { s_mode = m; s_abort = (m < 0); }
  }

  __syncthreads();   // len_s / census
  if (s_abort) return;

  // memory wave: gx granule q -> (row, gate, 8-unit chunk)
  i32x4 gpre[RGL];
  const int NRG = R * G * (UPW / 8);
  auto mw_load = [&](int s) {
#pragma unroll
    for (int j = 0; j < RGL; ++j) {
      const int q = lane + 64 * j;
      const int qq = q < NRG ? q : 0;
      const int row = qq / (G * 4), rem = qq - row * (G * 4), g = rem >> 2, c8 = rem & 3;
      const int b = min(r0 + row, N - 1);
      const int t = max(0, min((dir == 0) ? s : (len_s[row] - 1 - s), a.T - 1));
      gpre[j] = *reinterpret_cast<const i32x4*>(a.gx + ((size_t)t * N + b) * a.gstride + dir * G * H + g * H + u0 +
                                                c8 * 8);
    }
  };
  auto mw_put = [&](int s) {
#pragma unroll
    for (int j = 0; j < RGL; ++j) {
      const int q = lane + 64 * j;
      if (q < NRG) {
        const int row = q / (G * 4), rem = q - row * (G * 4), g = rem >> 2, c8 = rem & 3;
        const bool act = s < len_s[row];
        const bf16x8 v = __builtin_bit_cast(bf16x8, gpre[j]);
#pragma unroll
        for (int k = 0; k < 8; ++k) gxr_s[s & 1][row][g * UPW + c8 * 8 + k] = act ? bf2f((bf16_t)v[k]) : 0.f;
      }
    }
  };
  // fused direction sum: the other direction's value for this lane's 2 output granules of
  // step s, loaded ahead (before the gx put) so the round trip hides under the put
  unsigned long long yq[2] = {0ull, 0ull};
  auto ysum_ptr = [&](int s, int j) -> unsigned long long* {
    const int row = min((lane >> 3) + 8 * j, R - 1), c4 = (lane & 7) * 4;
    const int b = min(r0 + row, N - 1), L = len_s[row];
    const int t = (s < L) ? ((dir == 0) ? s : (L - 1 - s)) : s;
    return reinterpret_cast<unsigned long long*>(a.ysum + ((size_t)t * N + b) * H + u0 + c4);
  };
  auto mw_ysum_load = [&](int s) {
#pragma unroll
    for (int j = 0; j < 2; ++j) yq[j] = __hip_atomic_load(ysum_ptr(s, j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // outputs of step s out of staging slot s&1: lane -> (row, 4 consecutive units) x 2
  auto mw_store = [&](int s) {
    f32x4 vh[2], vy[2];
    float4 vg[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j) {         // all LDS reads first, then the stores
      const int row = (lane >> 3) + 8 * j, c4 = (lane & 7) * 4;
      vh[j] = *reinterpret_cast<const f32x4*>(&oh_s[s & 1][row][c4]);
      vy[j] = *reinterpret_cast<const f32x4*>(&oy_s[s & 1][row][c4]);
      if (CELL == CELL_GRU)
#pragma unroll
        for (int i = 0; i < 4; ++i) vg[j][i] = og_s[(CELL == CELL_GRU) ? (s & 1) : 0][row][c4 + i];
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = (lane >> 3) + 8 * j, c4 = (lane & 7) * 4;
      if (row < R) {
        const int b = r0 + row, u = u0 + c4;
        *reinterpret_cast<f32x4*>(a.hsave[dir] + ((size_t)(s + 1) * NP + b) * H + u) = vh[j];
        if (CELL == CELL_GRU) {
          float4* gp = reinterpret_cast<float4*>(a.gates[dir]) + ((size_t)s * NP + b) * H + u;
#pragma unroll
          for (int i = 0; i < 4; ++i) gp[i] = vg[j][i];
        }
      }
    }
    // y (or the fused direction sum) after the state stores: the gate registers are dead
    // before any wait on the other direction
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = (lane >> 3) + 8 * j, c4 = (lane & 7) * 4;
      if (row < R) {
        const int b = r0 + row, u = u0 + c4;
        if (b < N) {
          const int L = len_s[row];
          const int t = (s < L) ? ((dir == 0) ? s : (L - 1 - s)) : s;
          uint2 o;
          o.x = (unsigned)f2bf(vy[j][0]) | ((unsigned)f2bf(vy[j][1]) << 16);
          o.y = (unsigned)f2bf(vy[j][2]) | ((unsigned)f2bf(vy[j][3]) << 16);
          if (a.ysum == nullptr) {
            *reinterpret_cast<uint2*>(a.y[dir] + ((size_t)t * N + b) * H + u) = o;
          } else {
            // Fused direction sum (reference: the fw + bw outputs summed by the caller,
            // src/custom_ops.py:36-96). Position t is produced by the forward direction at
            // step t and by the backward one at step L-1-t (padding positions: both at step
            // t). The direction that produces it LATER (ties: the backward one) waits for the
            // other's bf16 value in the sentinel-filled sum buffer and writes the bf16 sum,
            // rounding exactly like bf16 + bf16 in torch; the earlier one writes its value
            // through (sc1: the other direction's groups live on other XCDs). No cycle: the
            // later side of a pair only waits for a step the earlier side reached first.
            unsigned long long* p = ysum_ptr(s, j);
            const int other = (s < L) ? (L - 1 - s) : s;
            const bool later = s > other || (s == other && dir == 1);
            auto canon = [](unsigned h) { return (h & 0xffffu) == 0xffffu ? 0x7fc0u : (h & 0xffffu); };
            if (!later) {
              o.x = canon(o.x) | (canon(o.x >> 16) << 16);
              o.y = canon(o.y) | (canon(o.y >> 16) << 16);
              __hip_atomic_store(p, ((unsigned long long)o.y << 32) | o.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
              const long long t0 = __builtin_amdgcn_s_memrealtime();
              unsigned long long q = yq[j];           // usually already there (loaded ahead)
              while (true) {
                const unsigned w0 = (unsigned)q, w1 = (unsigned)(q >> 32);
                const bool ready = ((~w0 - 0x00010001u) & w0 & 0x80008000u) == 0 &&
                                   ((~w1 - 0x00010001u) & w1 & 0x80008000u) == 0;
                if (ready) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) { atomicOr(a.err, 4u); break; }
                __builtin_amdgcn_s_sleep(2);
                q = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              }
              const unsigned q0 = (unsigned)q, q1 = (unsigned)(q >> 32);
              auto add2 = [](unsigned x, unsigned y) {      // two bf16 pairs -> rounded bf16 sums
                const unsigned lo = f2bf(__uint_as_float(x << 16) + __uint_as_float(y << 16));
                const unsigned hi = f2bf(__uint_as_float(x & 0xffff0000u) + __uint_as_float(y & 0xffff0000u));
                return lo | (hi << 16);
              };
              *reinterpret_cast<uint2*>(p) = make_uint2(add2(o.x, q0), add2(o.y, q1));
            }
          }
        }
      }
    }
  };
  if (wave == QW) {
    mw_load(0);
    mw_put(0);
    if (a.steps > 1) mw_load(1);
  }
  __syncthreads();   // gx ring slot 0
  const bool plain = s_mode == 1;
  const unsigned hx_bytes = (unsigned)((size_t)(a.steps + 1) * NP * H * 2);
  bf16_t* hxd = a.hx[dir];
  const __amdgpu_buffer_rsrc_t rs_hx = make_rsrc(hxd, hx_bytes);
  StampT st(a.stamps != nullptr && (wave == 0 || wave == QW) && lane == 0);

  if (wave < QW) {
    // resident U fragments: B[k][c] = U[g*H + u0 + 16*uh + c][ks*32 + k], ks = kq + 4*kk
    bf16x8 uf[KR][G];
    bool kval[KB];
    float hreg = 0.f, bhr[G];
    {
      const bf16_t* Ud = a.U[dir];
#pragma unroll
      for (int kk = 0; kk < KB; ++kk) {
        const int ks = kq + 4 * kk;
        kval[kk] = ks < KS;
#pragma unroll
        for (int g = 0; g < G; ++g) {
          bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
          if (kval[kk])
            v = *reinterpret_cast<const bf16x8*>(Ud + (size_t)(g * H + u0 + ec) * H + ks * 32 + 8 * (lane >> 4));
          if (kk < KR) uf[kk < KR ? kk : 0][g] = v;
          else ul_s[kk >= KR ? kk - KR : 0][wave][g][lane] = v;   // own slot: no barrier needed
        }
      }
#pragma unroll
      for (int g = 0; g < G; ++g)
        bhr[g] = (CELL == CELL_GRU && a.bh[dir]) ? a.bh[dir][g * H + u0 + ec] : 0.f;
      if (erow < R) hreg = a.hsave[dir][(size_t)(r0 + erow) * H + u0 + ec];   // slot 0 = h0
    }
    // padding lanes of the 16-row fragment re-read row R-1 (a real, polled row: same cache
    // line as its own lane), so every lane can wait on its granule and use it unmasked
    const int arow = r0 + min(lane & 15, R - 1);
    // retry back-off: none by default (same-box A/B: 9.03 / 8.99 / 9.02 vs 9.08 / 9.04 / 9.05
    // ms/step with s_sleep 1); knob bits 12-13 = 1: s_sleep 1, 2: s_sleep 3
    const int nap = (a.knobs >> 12) & 3;
    const bool erow_ok = erow < R;
    const int L = len_s[erow];
    drain_vm();        // the U / bias / h0 loads: nothing from before the loop is pending inside it
    // pre-poll sleep (ops/rnn.py _kernel_knobs), in units of s_sleep 4 here: the cross-XCD
    // write-through exchange of this kernel's wide groups lands later than the XCD-local one
    const int presleep = (a.knobs >> 17) & 7;
    for (int s = 0; s < a.steps; ++s) {
      st.mark(-1);
      if (s > 0)
        for (int i = 0; i < presleep; ++i) __builtin_amdgcn_s_sleep(4);
      float gxv[G];                    // slot s&1 was filled before the previous barrier
#pragma unroll
      for (int g = 0; g < G; ++g) gxv[g] = gxr_s[s & 1][erow][g * UPW + ec];
      unsigned off[KB];
      if constexpr (KL > 0) {
        // wide layers have KS == 4 * KB (host-checked): no clamp, and every k-step's granule
        // is a constant 256 B past the first, so the loads take it as an immediate offset
        // (one live VGPR instead of KB)
        const unsigned o0 = (unsigned)((((size_t)s * NP + arow) * H + kq * 32 + 8 * (lane >> 4)) * 2);
#pragma unroll
        for (int kk = 0; kk < KB; ++kk) off[kk] = o0 + 256u * kk;
      } else {
#pragma unroll
        for (int kk = 0; kk < KB; ++kk)
          off[kk] = (unsigned)((((size_t)s * NP + arow) * H + min(kq + 4 * kk, KS - 1) * 32 + 8 * (lane >> 4)) * 2);
      }
      f32x4 acc[G];
#pragma unroll
      for (int g = 0; g < G; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
      auto mfma_k = [&](int kk, bf16x8 af) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const bf16x8 b = kk < KR ? uf[kk < KR ? kk : 0][g] : ul_s[kk >= KR ? kk - KR : 0][wave][g][lane];
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, b, acc[g], 0, 0, 0);
        }
      };
      bool ok;
      if constexpr ((KL > 0 && DS2_WIDE_CH > 0) || (KL == 0 && DS2_NARROW_CH > 0))
        // wide layers: at most DS2_WIDE_CH granules in flight per lane (register budget)
        ok = poll_mfma<KB, 1, (KL > 0 ? DS2_WIDE_CH : DS2_NARROW_CH)>(rs_hx, off, kval, true, a.timeout, mfma_k);
      else
        ok = poll_mfma_par<KB>(rs_hx, off, kval, a.timeout, nap, mfma_k);
      if (!ok) { s_abort = 1; atomicOr(a.err, 1u); }
      st.mark(0);
      // transpose-reduce: hand the three elements this wave does not finalise to their owners
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j == kq) continue;
        const int src = kq < j ? kq : kq - 1;
#pragma unroll
        for (int g = 0; g < G; ++g) red_s[s & 1][uh][j][src][g][lane] = acc[g][j];
      }
      st.mark(1);
      lds_barrier();
      st.mark(2);
      if (s_abort) break;
      float pre[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float own = kq == 0 ? acc[g][0] : kq == 1 ? acc[g][1] : kq == 2 ? acc[g][2] : acc[g][3];
        pre[g] = own + red_s[s & 1][uh][kq][0][g][lane] + red_s[s & 1][uh][kq][1][g][lane] +
                 red_s[s & 1][uh][kq][2][g][lane];
      }
      const bool act = s < L;
      float hn;
      float4 gsv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (CELL == CELL_GRU) {
        const float ghn = pre[2] + bhr[2];
        const float r = sigmoidf_(gxv[0] + pre[0] + bhr[0]);
        const float z = sigmoidf_(gxv[1] + pre[1] + bhr[1]);
        const float n = tanhf_(gxv[2] + r * ghn);
        hn = (1.f - z) * n + z * hreg;
        if (act) gsv = make_float4(r, z, n, ghn);
      } else {
        hn = fminf(fmaxf(gxv[0] + pre[0], 0.f), RELU_CAP);
      }
      const float hnew = act ? hn : hreg;
      hreg = hnew;
      // hardware RNE conversion; 0xFFFF (the sentinel, a negative NaN) -> canonical NaN
      unsigned hq = (unsigned)__builtin_bit_cast(unsigned short, (__bf16)hnew);
      hq = hq == 0xffffu ? 0x7fc0u : hq;
      // 16-B exchange granule = 8 consecutive units of one row = 8 consecutive lanes
      const unsigned pr = hq | ((unsigned)__builtin_amdgcn_update_dpp(0, (int)hq, 0x101, 0xf, 0xf, false) << 16);
      const int q1 = __builtin_amdgcn_update_dpp(0, (int)pr, 0x102, 0xf, 0xf, false);
      const int q2 = __builtin_amdgcn_update_dpp(0, (int)pr, 0x104, 0xf, 0xf, false);
      const int q3 = __builtin_amdgcn_update_dpp(0, (int)pr, 0x106, 0xf, 0xf, false);
      if ((lane & 7) == 0 && erow_ok) {
        const i32x4 v = {(int)pr, q1, q2, q3};
        const unsigned off = (unsigned)((((size_t)(s + 1) * NP + r0 + erow) * H + u0 + ec) * 2);
        store_granule(plain, rs_hx, hxd, off, v);
      }
      oh_s[s & 1][erow][ec] = hnew;
      oy_s[s & 1][erow][ec] = act ? hn : 0.f;
      if (CELL == CELL_GRU) og_s[(CELL == CELL_GRU) ? (s & 1) : 0][erow][ec] = gsv;
      st.mark(4);
    }
  } else {
    for (int s = 0; s < a.steps; ++s) {
      st.mark(-1);
      if (a.ysum != nullptr && s >= 2) mw_ysum_load(s - 2);
      if (s + 1 < a.steps) mw_put(s + 1);
      if (s >= 2) mw_store(s - 2);
      if (s + 2 < a.steps) mw_load(s + 2);
      st.mark(0);
      lds_barrier();
      st.mark(1);
      if (s_abort) break;
    }
  }
  __syncthreads();
  if (wave == QW && !s_abort) {
    if (a.steps >= 2) {
      if (a.ysum != nullptr) mw_ysum_load(a.steps - 2);
      mw_store(a.steps - 2);
    }
    if (a.steps >= 1) {
      if (a.ysum != nullptr) mw_ysum_load(a.steps - 1);
      mw_store(a.steps - 1);
    }
  }
  if (STAMPS && wave == 0) { st.acc[5] = (unsigned long long)(s_mode + 10); st.store(a.stamps, 0); }
  if (STAMPS && wave == QW && st.on) { a.stamps[(size_t)blockIdx.x * 8 + 6] = st.acc[0]; a.stamps[(size_t)blockIdx.x * 8 + 7] = st.acc[1]; }
}

// ------------------------------------------------------------------------------------
// GRU forward, generation 5 (rnne_fwd_kernel, H <= 1024): the K-eighth structure of the wide
// forward for 32-unit GRU workgroups. Generation 4 split its 8 MFMA waves into 2 unit halves x
// 4 K-quarters, so each exchange granule was polled by both halves; here wave w polls K-eighth
// w (k-steps w + 8 kk) once and multiplies it into all six 16-unit tiles (2 unit halves x 3
// gates). Every wave stores its 24 partial slots (tile, element j) to LDS, ONE barrier, and the
// owner of cell slot (unit half w & 1, element j = w >> 1) sums the 8 K-eighths of its three
// gates in wave order and runs the GRU cell in registers, as generation 4 does.
// ------------------------------------------------------------------------------------
// KL: the last KL of each wave's U k-steps live in LDS; SB: one partial buffer and a second
// barrier per step instead of two buffers by step parity (the LDS of H = 1280: 48 KB of U)
template <int KB, int KL, bool SB, bool STAMPS>
__global__ __launch_bounds__(QTH) void rnne_fwd_kernel(XFwd a) {
  using StampT = typename std::conditional<STAMPS, Stamps, NoStamps>::type;
  constexpr int CELL = CELL_GRU;
  constexpr int G = 3;
  constexpr int NT = 2 * G;                       // tiles t = 3 uh + g
  constexpr int ROWS = 16;
  constexpr int GP = G * UPW + 8;                 // gx ring row pitch (bf16: one 16-B LDS store per granule)
  constexpr int OP = UPW + 4;                     // output staging row pitch
  constexpr int RG = ROWS * G * (UPW / 8);        // gx granules per step (upper bound)
  constexpr int RGL = (RG + 63) / 64;
  constexpr int KR = KB - KL;
  static_assert(KL >= 0 && KR >= 1, "register k-steps");
  __shared__ float red_s[SB ? 1 : 2][QW][NT][4][64];   // [parity][source wave][tile][element j][lane]
  __shared__ bf16x8 ul_s[KL > 0 ? KL : 1][QW][NT][64];  // LDS-resident U k-steps
  __shared__ __attribute__((aligned(16))) bf16_t gxr_s[2][ROWS][GP];
  __shared__ __attribute__((aligned(16))) float oh_s[2][ROWS][OP];
  __shared__ __attribute__((aligned(16))) float oy_s[2][ROWS][OP];
  __shared__ float4 og_s[2][ROWS][OP];
  __shared__ int len_s[ROWS];
  __shared__ int s_mode, s_abort;

  int grp, mem;
  if (!take_role(a.xcd_map, a.ngroups, a.P, grp, mem)) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, KS = H / 32, N = a.N, NP = a.NP, R = a.R;
  const int bg = grp % a.BG, dir = grp / a.BG;
  const int r0 = bg * R, u0 = mem * UPW;
  const int uh = wave & 1, jo = (wave >> 1) & 3;  // owned cell slot
  // K-eighth of this MFMA wave: K-eighth 0 (the one with an extra k-step when H/32 % 8 != 0)
  // goes to wave 7, away from SIMD 0, which waves 0 and 4 share with the memory wave 8
  // (same-box A/B 8.030-8.037 vs 8.024-8.055 ms/step: neutral)
  const int ke = (wave + 1) & 7;
  const int erow = 4 * (lane >> 4) + jo;
  const int ec = 16 * uh + (lane & 15);
  if (tid < ROWS) len_s[tid] = (tid < R && r0 + tid < N) ? a.lens[r0 + tid] : 0;
  if (wave == 0) {
    int m = group_census(a.census, grp, mem, a.P, a.timeout, a.err);
    if ((a.knobs & 32768) && m > 0) m = 0;      // knob 32768: force write-through (timing)
    if (lane == 0) { s_mode = m; s_abort = (m < 0); }
  }
  __syncthreads();
  if (s_abort) return;

  // memory wave: gx granule q -> (row, gate, 8-unit chunk)
  i32x4 gpre[RGL];
  const int NRG = R * G * (UPW / 8);
  auto mw_load = [&](int s) {
#pragma unroll
    for (int j = 0; j < RGL; ++j) {
      const int q = lane + 64 * j;
      const int qq = q < NRG ? q : 0;
      const int row = qq / (G * 4), rem = qq - row * (G * 4), g = rem >> 2, c8 = rem & 3;
      const int b = min(r0 + row, N - 1);
      const int t = max(0, min((dir == 0) ? s : (len_s[row] - 1 - s), a.T - 1));
      gpre[j] = *reinterpret_cast<const i32x4*>(a.gx + ((size_t)t * N + b) * a.gstride + dir * G * H + g * H + u0 +
                                                c8 * 8);
    }
  };
  auto mw_put = [&](int s) {
#pragma unroll
    for (int j = 0; j < RGL; ++j) {
      const int q = lane + 64 * j;
      if (q < NRG) {
        const int row = q / (G * 4), rem = q - row * (G * 4), g = rem >> 2, c8 = rem & 3;
        const bool act = s < len_s[row];
        const i32x4 z = {0, 0, 0, 0};
        *reinterpret_cast<i32x4*>(&gxr_s[s & 1][row][g * UPW + c8 * 8]) = act ? gpre[j] : z;
      }
    }
  };
  // fused direction sum: the other direction's value for this lane's 2 output granules of
  // step s, loaded ahead (before the gx put) so the round trip hides under the put
  unsigned long long yq[2] = {0ull, 0ull};
  auto ysum_ptr = [&](int s, int j) -> unsigned long long* {
    const int row = min((lane >> 3) + 8 * j, R - 1), c4 = (lane & 7) * 4;
    const int b = min(r0 + row, N - 1), L = len_s[row];
    const int t = (s < L) ? ((dir == 0) ? s : (L - 1 - s)) : s;
    return reinterpret_cast<unsigned long long*>(a.ysum + ((size_t)t * N + b) * H + u0 + c4);
  };
  auto mw_ysum_load = [&](int s) {
#pragma unroll
    for (int j = 0; j < 2; ++j) yq[j] = __hip_atomic_load(ysum_ptr(s, j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // outputs of step s out of staging slot s&1: lane -> (row, 4 consecutive units) x 2
  auto mw_store = [&](int s) {
    f32x4 vh[2], vy[2];
    float4 vg[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j) {         // all LDS reads first, then the stores
      const int row = (lane >> 3) + 8 * j, c4 = (lane & 7) * 4;
      vh[j] = *reinterpret_cast<const f32x4*>(&oh_s[s & 1][row][c4]);
      vy[j] = *reinterpret_cast<const f32x4*>(&oy_s[s & 1][row][c4]);
      if (CELL == CELL_GRU)
#pragma unroll
        for (int i = 0; i < 4; ++i) vg[j][i] = og_s[(CELL == CELL_GRU) ? (s & 1) : 0][row][c4 + i];
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = (lane >> 3) + 8 * j, c4 = (lane & 7) * 4;
      if (row < R) {
        const int b = r0 + row, u = u0 + c4;
        *reinterpret_cast<f32x4*>(a.hsave[dir] + ((size_t)(s + 1) * NP + b) * H + u) = vh[j];
        if (CELL == CELL_GRU) {
          float4* gp = reinterpret_cast<float4*>(a.gates[dir]) + ((size_t)s * NP + b) * H + u;
#pragma unroll
          for (int i = 0; i < 4; ++i) gp[i] = vg[j][i];
        }
      }
    }
    // y (or the fused direction sum) after the state stores: the gate registers are dead
    // before any wait on the other direction
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = (lane >> 3) + 8 * j, c4 = (lane & 7) * 4;
      if (row < R) {
        const int b = r0 + row, u = u0 + c4;
        if (b < N) {
          const int L = len_s[row];
          const int t = (s < L) ? ((dir == 0) ? s : (L - 1 - s)) : s;
          uint2 o;
          o.x = (unsigned)f2bf(vy[j][0]) | ((unsigned)f2bf(vy[j][1]) << 16);
          o.y = (unsigned)f2bf(vy[j][2]) | ((unsigned)f2bf(vy[j][3]) << 16);
          if (a.ysum == nullptr) {
            *reinterpret_cast<uint2*>(a.y[dir] + ((size_t)t * N + b) * H + u) = o;
          } else {
            // Fused direction sum (reference: the fw + bw outputs summed by the caller,
            // src/custom_ops.py:36-96). Position t is produced by the forward direction at
            // step t and by the backward one at step L-1-t (padding positions: both at step
            // t). The direction that produces it LATER (ties: the backward one) waits for the
            // other's bf16 value in the sentinel-filled sum buffer and writes the bf16 sum,
            // rounding exactly like bf16 + bf16 in torch; the earlier one writes its value
            // through (sc1: the other direction's groups live on other XCDs). No cycle: the
            // later side of a pair only waits for a step the earlier side reached first.
            unsigned long long* p = ysum_ptr(s, j);
            const int other = (s < L) ? (L - 1 - s) : s;
            const bool later = s > other || (s == other && dir == 1);
            auto canon = [](unsigned h) { return (h & 0xffffu) == 0xffffu ? 0x7fc0u : (h & 0xffffu); };
            if (!later) {
              o.x = canon(o.x) | (canon(o.x >> 16) << 16);
              o.y = canon(o.y) | (canon(o.y >> 16) << 16);
              __hip_atomic_store(p, ((unsigned long long)o.y << 32) | o.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
              const long long t0 = __builtin_amdgcn_s_memrealtime();
              unsigned long long q = yq[j];           // usually already there (loaded ahead)
              while (true) {
                const unsigned w0 = (unsigned)q, w1 = (unsigned)(q >> 32);
                const bool ready = ((~w0 - 0x00010001u) & w0 & 0x80008000u) == 0 &&
                                   ((~w1 - 0x00010001u) & w1 & 0x80008000u) == 0;
                if (ready) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) { atomicOr(a.err, 4u); break; }
                __builtin_amdgcn_s_sleep(2);
                q = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              }
              const unsigned q0 = (unsigned)q, q1 = (unsigned)(q >> 32);
              auto add2 = [](unsigned x, unsigned y) {      // two bf16 pairs -> rounded bf16 sums
                const unsigned lo = f2bf(__uint_as_float(x << 16) + __uint_as_float(y << 16));
                const unsigned hi = f2bf(__uint_as_float(x & 0xffff0000u) + __uint_as_float(y & 0xffff0000u));
                return lo | (hi << 16);
              };
              *reinterpret_cast<uint2*>(p) = make_uint2(add2(o.x, q0), add2(o.y, q1));
            }
          }
        }
      }
    }
  };
  if (wave == QW) {
    mw_load(0);
    mw_put(0);
    if (a.steps > 1) mw_load(1);
  }
  __syncthreads();   // gx ring slot 0
  const bool plain = s_mode == 1;
  const unsigned hx_bytes = (unsigned)((size_t)(a.steps + 1) * NP * H * 2);
  bf16_t* hxd = a.hx[dir];
  const __amdgpu_buffer_rsrc_t rs_hx = make_rsrc(hxd, hx_bytes);
  const int stw = (a.knobs >> 24) & 7;   // stamps: the MFMA wave recorded (diagnostics; 0 = wave 0)
  StampT st(a.stamps != nullptr && (wave == stw || wave == QW) && lane == 0);

  if (wave < QW) {
    // resident U fragments: B[k][c] = U[g H + u0 + 16 h + c][ks*32 + k], tile 3 h + g, ks = wave + 8 kk
    bf16x8 uf[KR][NT];
    bool kval[KB];
    float hreg = 0.f, bhr[G];
    {
      const bf16_t* Ud = a.U[dir];
#pragma unroll
      for (int kk = 0; kk < KB; ++kk) {
        const int ks = ke + 8 * kk;
        kval[kk] = ks < KS;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int g = t % G, h = t / G;
          bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
          if (kval[kk])
            v = *reinterpret_cast<const bf16x8*>(Ud + (size_t)(g * H + u0 + 16 * h + (lane & 15)) * H + ks * 32 +
                                                 8 * (lane >> 4));
          if (kk < KR) uf[kk < KR ? kk : 0][t] = v;
          else ul_s[kk >= KR ? kk - KR : 0][wave][t][lane] = v;   // own slot: no barrier needed
        }
      }
#pragma unroll
      for (int g = 0; g < G; ++g) bhr[g] = a.bh[dir] ? a.bh[dir][g * H + u0 + ec] : 0.f;
      if (erow < R) hreg = a.hsave[dir][(size_t)(r0 + erow) * H + u0 + ec];   // slot 0 = h0
    }
    const int arow = r0 + min(lane & 15, R - 1);
    const int nap = (a.knobs >> 12) & 3;
    const bool erow_ok = erow < R;
    const int L = len_s[erow];
    drain_vm();        // the U / bias / h0 loads: nothing from before the loop is pending inside it
    const int presleep = (a.knobs >> 17) & 7;
    for (int s = 0; s < a.steps; ++s) {
      st.mark(-1);
      if (s > 0)
        for (int i = 0; i < presleep; ++i) __builtin_amdgcn_s_sleep(1);
      float gxv[G];
#pragma unroll
      for (int g = 0; g < G; ++g) gxv[g] = bf2f(gxr_s[s & 1][erow][g * UPW + ec]);
      unsigned off[KB];
      const unsigned o0 = (unsigned)((((size_t)s * NP + arow) * H + ke * 32 + 8 * (lane >> 4)) * 2);
#pragma unroll
      for (int kk = 0; kk < KB; ++kk) off[kk] = o0 + 512u * kk;
      f32x4 acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      auto mfma_k = [&](int kk, bf16x8 af) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const bf16x8 b = kk < KR ? uf[kk < KR ? kk : 0][t] : ul_s[kk >= KR ? kk - KR : 0][wave][t][lane];
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, b, acc[t], 0, 0, 0);
        }
      };
      const bool ok = poll_mfma_par<KB>(rs_hx, off, kval, a.timeout, nap, mfma_k);
      if (!ok) { s_abort = 1; atomicOr(a.err, 1u); }
      st.mark(0);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) red_s[SB ? 0 : (s & 1)][wave][t][j][lane] = acc[t][j];
      st.mark(1);
      lds_barrier();
      st.mark(2);
      // the abort word is read together with the partials and tested only before the first
      // store: testing it first put one more LDS round trip (~100 cycles) on every step's path
      const int ab = s_abort;
      float pre[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        // pairwise tree over the 8 K-eighths (fixed order: deterministic), 3 dependent adds
        // instead of a chain of 8 on the step's critical path
        float p[QW];
#pragma unroll
        for (int w = 0; w < QW; ++w) p[w] = red_s[SB ? 0 : (s & 1)][w][3 * uh + g][jo][lane];
#pragma unroll
        for (int d = 1; d < QW; d *= 2)
#pragma unroll
          for (int w = 0; w + d < QW; w += 2 * d) p[w] += p[w + d];
        pre[g] = p[0];
      }
      if constexpr (SB) lds_barrier();               // every partial read before the next step's writes
      const bool act = s < L;
      float4 gsv = make_float4(0.f, 0.f, 0.f, 0.f);
      const float ghn = pre[2] + bhr[2];
      const float r = sigmoidf_(gxv[0] + pre[0] + bhr[0]);
      const float z = sigmoidf_(gxv[1] + pre[1] + bhr[1]);
      const float n = tanhf_(gxv[2] + r * ghn);
      const float hn = (1.f - z) * n + z * hreg;
      if (act) gsv = make_float4(r, z, n, ghn);
      const float hnew = act ? hn : hreg;
      hreg = hnew;
      unsigned hq = (unsigned)__builtin_bit_cast(unsigned short, (__bf16)hnew);
      hq = hq == 0xffffu ? 0x7fc0u : hq;
      const unsigned pr = hq | ((unsigned)__builtin_amdgcn_update_dpp(0, (int)hq, 0x101, 0xf, 0xf, false) << 16);
      const int q1 = __builtin_amdgcn_update_dpp(0, (int)pr, 0x102, 0xf, 0xf, false);
      const int q2 = __builtin_amdgcn_update_dpp(0, (int)pr, 0x104, 0xf, 0xf, false);
      const int q3 = __builtin_amdgcn_update_dpp(0, (int)pr, 0x106, 0xf, 0xf, false);
      if (ab) break;
      if ((lane & 7) == 0 && erow_ok) {
        const i32x4 v = {(int)pr, q1, q2, q3};
        const unsigned off2 = (unsigned)((((size_t)(s + 1) * NP + r0 + erow) * H + u0 + ec) * 2);
        store_granule(plain, rs_hx, hxd, off2, v);
      }
      oh_s[s & 1][erow][ec] = hnew;
      oy_s[s & 1][erow][ec] = act ? hn : 0.f;
      og_s[s & 1][erow][ec] = gsv;
      st.mark(4);
    }
  } else {
    for (int s = 0; s < a.steps; ++s) {
      st.mark(-1);
      if (a.ysum != nullptr && s >= 2) mw_ysum_load(s - 2);
      if (s + 1 < a.steps) mw_put(s + 1);
      if (s >= 2) mw_store(s - 2);
      if (s + 2 < a.steps) mw_load(s + 2);
      st.mark(0);
      lds_barrier();
      st.mark(1);
      const int ab = s_abort;     // same value the MFMA waves test (written before the barrier)
      if constexpr (SB) lds_barrier();
      if (ab) break;
    }
  }
  __syncthreads();
  if (wave == QW && !s_abort) {
    if (a.steps >= 2) {
      if (a.ysum != nullptr) mw_ysum_load(a.steps - 2);
      mw_store(a.steps - 2);
    }
    if (a.steps >= 1) {
      if (a.ysum != nullptr) mw_ysum_load(a.steps - 1);
      mw_store(a.steps - 1);
    }
  }
  if (STAMPS && wave == stw) { st.acc[5] = (unsigned long long)(s_mode + 10); st.store(a.stamps, 0); }
  if (STAMPS && wave == QW && st.on) { a.stamps[(size_t)blockIdx.x * 8 + 6] = st.acc[0]; a.stamps[(size_t)blockIdx.x * 8 + 7] = st.acc[1]; }
}

constexpr int DS2_BWD_CH = 3;     // R > 8 reduce-scatter gather: producers' granules in flight per lane (0 = all; H = 1280 BPTT 6.78 -> 6.63 us/step at 3, 6.65 at 2 and 4)


// ------------------------------------------------------------------------------------
// backward (BPTT), generation 3: reduce-scatter exchange.
//
// (Generation 2, removed in round 3, gathered dgh_{s+1} (R rows x 3H gate columns, bf16) to EVERY
// workgroup of the group each step, because a workgroup's dh slice needs all 3H columns
// of dgh times its U columns.) Here each workgroup instead multiplies ITS OWN gate columns
// by the U rows they index, producing a partial dh for ALL H units,
//     P_j(s) = dgh_s[:, cols_j] . U[cols_j, :]          (R x H, fp32)
// and a consumer sums the 25 producers' partials of its own 32 units:
//     dh_rec(s-1)[:, units_k] = sum_j P_j(s)[:, units_k].
// Per step a consumer then reads P x R x 32 fp32 (25.6 KB at H = 800, R = 8) instead of
// R x 3H bf16 (38.4 KB), and the exchange lives in a 3-slot ring (a few MB per group, L2
// resident) instead of a T-step buffer:
//  * ring[dir][slot][bg][producer][H/16 m-tiles][row][16] fp32, P(s) goes to slot s % 3. Readiness is a
//    use TAG in every word's mantissa LSB: slot s % 3 is written at processing index
//    k = steps-1-s, i.e. at k, k+3, k+6, ..., with tag (k/3) & 1, which alternates between
//    consecutive uses of a slot. The host fills the ring with 0xFFFFFFFF (tag 1) before each
//    launch and every slot's first use has tag 0. A consumer spins until all four words of
//    a 16-B granule carry the tag it expects, so a stale value (previous use) or a granule
//    landing in pieces is never taken. Nothing is reset: a producer rewrites slot s % 3 only
//    after it has gathered every producer's P(s+1), each published after that producer's
//    gather of P(s+2) and P(s+3) had returned, so no one still reads the old contents.
//    (Generation 3a reset every granule read to a sentinel: 25.6 KB of extra stores per
//    workgroup-step plus a vmcnt(0) drain before the first barrier.)
//  * R <= 8 (PBF): the partials travel as bf16 whose rounding is steered to carry the tag
//    (of the two bf16 neighbours of the fp32 value's truncation, the one with the right
//    LSB: error < 1 bf16 ulp), m-tiles published in unit pairs so a 16-B granule holds 8
//    units of one row: half the exchanged bytes (12.8 KB out + 12.8 KB in per workgroup-
//    step), BPTT 0.958 -> 0.911 ms per layer; gradient error vs an fp32 reference
//    (H=800, T=120): dgx 0.21 % (fp32 partials 0.18 %), dU 0.29 % (0.27 %).
//  * dgh (bf16) is now a plain output for the dU GEMM, stored by the memory wave off the
//    critical path; no T-step sentinel fill is needed.
// Worker waves 0..6: gather+sum (producer j = wave + 7i), then the MFMA
//   D[unit][row] = sum_k U[col_k][unit] . dgh[row][col_k]  (A = U resident, 16-unit tiles
//   w + 7i; B = the dgh tile from LDS), one 16-B fp32 granule per lane published straight
//   from the accumulator. Waves 0..3 run the cell epilogue; wave 7 is the memory wave.
// ------------------------------------------------------------------------------------
struct XBwdRS {
  int T, N, NP, H, P, BG, R, steps, gstride, ngroups, xcd_map, knobs;
  const int* lens;
  const bf16_t* dy;
  const bf16_t* U[2];
  const float* hsave[2];
  const float* gates[2];
  bf16_t* dgh[2];         // [steps][NP][G*H] output (dU GEMM operand)
  bf16_t* dgx;
  float* ring[2];         // [3][BG][P][H/16][R][16] fp32, filled with 0xFFFFFFFF (tag 1) per launch
  float* dbx_part[2];
  float* dbh_part[2];
  float dgx_scale;
  unsigned* census;
  unsigned* err;
  long long timeout;
  unsigned long long* stamps;
};

// bf16x2_tagged / granule_tagged16 (tagged bf16 partials of the reduce-scatter ring): common.h

// A ring word carries its use tag in the mantissa LSB (see rnnrs_bwd_kernel): the granule is
// ready when all four words carry the expected tag.
__device__ __forceinline__ bool granule_tagged(i32x4 v, unsigned tag) {
  return (((unsigned)v[0] & 1u) == tag) && (((unsigned)v[1] & 1u) == tag) && (((unsigned)v[2] & 1u) == tag) &&
         (((unsigned)v[3] & 1u) == tag);
}
__device__ __forceinline__ float canon32(float f) { return (f != f) ? __uint_as_float(0x7fc00000u) : f; }

template <int CELL, int MTU, int GPT, int PBF>
__global__ __launch_bounds__(NTH) void rnnrs_bwd_kernel(XBwdRS a) {
  // PBF (R <= 8): partials exchanged as tagged bf16, m-tiles published in unit pairs
  // (2p, 2p+1) so one 16-B granule = 8 units of one row (half the exchanged bytes)
  constexpr int G = (CELL == CELL_GRU) ? 3 : 1;
  constexpr int ROWS = 16;
  constexpr int EPT = ROWS * UPW / ETH;
  constexpr int OPL = ROWS * UPW / 64;            // elements per memory-wave lane
  // GPT: producers per gather thread (7 x GPT >= P)
  constexpr int DGP = G * UPW + 8;                // dgh tile pitch (bf16)
  __shared__ float red_s[MW][ROWS][UPW + 1];
  __shared__ __attribute__((aligned(16))) bf16_t dg_s[ROWS][DGP];
  __shared__ float dyr_s[2][ROWS][UPW];           // prefetch ring (memory wave -> epilogue)
  __shared__ float hpr_s[2][ROWS][UPW];
  __shared__ float4 gr_s[2][(CELL == CELL_GRU) ? ROWS : 1][UPW];
  __shared__ __attribute__((aligned(16))) float ox_s[2][ROWS][G][UPW];     // dgx staging by step parity
  __shared__ __attribute__((aligned(16))) bf16_t oh_s[2][ROWS][G][UPW];    // dgh staging (already rounded)
  __shared__ int len_s[ROWS];
  __shared__ int s_mode, s_abort;

  int grp, mem;
  if (!take_role(a.xcd_map, a.ngroups, a.P, grp, mem)) return;
  DS2_DCHECK(grp < a.ngroups && mem < a.P && a.NP >= a.BG * a.R && a.R <= 16);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, GH = G * H, N = a.N, NP = a.NP, R = a.R, P = a.P, MTS = H / 16;
  const int bg = grp % a.BG, dir = grp / a.BG;
  const int r0 = bg * R, u0 = mem * UPW;
  if (tid < ROWS) len_s[tid] = (tid < R && r0 + tid < N) ? a.lens[r0 + tid] : 0;
  for (int i = tid; i < ROWS * DGP; i += NTH) (&dg_s[0][0])[i] = 0;
  if (wave == 0) {
    int m = group_census(a.census, grp, mem, P, a.timeout, a.err);
    if ((a.knobs & 32768) && m > 0) m = 0;      // knob 32768: force write-through (timing)
    if (lane == 0) { s_mode = m; s_abort = (m < 0); }
  }

  // resident A fragments of the worker waves: A[m][k] = U[g*H + u0 + k][16*mt + m],
  // m-tile mt = wave + 7*i, k-step g (this workgroup's 32 columns of gate g)
  bf16x8 ua[MTU][G];
  {
    const bf16_t* Ud = a.U[dir];
#pragma unroll
    for (int i = 0; i < MTU; ++i) {
      const int mt = PBF ? 2 * (wave + MW * (i >> 1)) + (i & 1) : wave + MW * i;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        if (wave < MW && mt < MTS) {
          const bf16_t* p = Ud + (size_t)(g * H + u0 + 8 * (lane >> 4)) * H + 16 * mt + (lane & 15);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (short)p[(size_t)j * H];
        }
        ua[i][g] = v;
      }
    }
  }

  float carry[EPT];
  float sbx[EPT][G];
  float sbh[EPT];
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    carry[i] = 0.f;
    sbh[i] = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g) sbx[i][g] = 0.f;
  }
  __syncthreads();   // len_s, dg_s zero rows, census

  // memory wave: per-step inputs (dy, gates, h_prev) one step ahead, dgx / dgh stores,
  // all in 8- / 16-B pieces: load task = (row, 4 units), store task = (row, gate, 8 units)
  constexpr int LT = ROWS * 8 / 64, ST = (ROWS * G * 4 + 63) / 64;
  uint2 pdy[LT];
  float4 php[LT];
  float4 pg[LT][4];
  auto mw_load = [&](int s) {
#pragma unroll
    for (int k = 0; k < LT; ++k) {
      const int q = lane + 64 * k;
      const int row = q >> 3, c4 = (q & 7) * 4;
      if (row < R) {
        const int bp = min(r0 + row, NP - 1), bn = min(r0 + row, N - 1), u = u0 + c4;
        const int t = max(0, min((dir == 0) ? s : (len_s[row] - 1 - s), a.T - 1));
        pdy[k] = *reinterpret_cast<const uint2*>(a.dy + ((size_t)t * N + bn) * H + u);
        if (CELL == CELL_GRU) {
          const float4* gp = reinterpret_cast<const float4*>(a.gates[dir]) + ((size_t)s * NP + bp) * H + u;
#pragma unroll
          for (int i = 0; i < 4; ++i) pg[k][i] = gp[i];
          php[k] = *reinterpret_cast<const float4*>(a.hsave[dir] + ((size_t)s * NP + bp) * H + u);
        } else {
          php[k] = *reinterpret_cast<const float4*>(a.hsave[dir] + ((size_t)(s + 1) * NP + bp) * H + u);  // h_s
        }
      }
    }
  };
  auto mw_put = [&](int s) {
    const int slot = s & 1;
#pragma unroll
    for (int k = 0; k < LT; ++k) {
      const int q = lane + 64 * k;
      const int row = q >> 3, c4 = (q & 7) * 4;
      if (row < R) {
        const bool act = s < len_s[row];
        const float dv[4] = {bf2f((bf16_t)(pdy[k].x & 0xffffu)), bf2f((bf16_t)(pdy[k].x >> 16)),
                             bf2f((bf16_t)(pdy[k].y & 0xffffu)), bf2f((bf16_t)(pdy[k].y >> 16))};
        const float hv[4] = {php[k].x, php[k].y, php[k].z, php[k].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          dyr_s[slot][row][c4 + i] = act ? dv[i] : 0.f;
          hpr_s[slot][row][c4 + i] = act ? hv[i] : 0.f;
          if (CELL == CELL_GRU)
            gr_s[slot][(CELL == CELL_GRU) ? row : 0][c4 + i] = act ? pg[k][i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
  };
  auto mw_store = [&](int s) {          // dgx and dgh of step s from the staging area
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      const int q = lane + 64 * k;
      const int row = q / (G * 4), rem = q - row * (G * 4), g = rem >> 2, c8 = (rem & 3) * 8;
      if (row < R) {
        const int b = r0 + row, u = u0 + c8;
        *reinterpret_cast<i32x4*>(a.dgh[dir] + ((size_t)s * NP + b) * GH + g * H + u) =
            *reinterpret_cast<const i32x4*>(&oh_s[s & 1][row][g][c8]);
        if (b < N) {
          const int L = len_s[row];
          const bool act = s < L;
          const int t = act ? ((dir == 0) ? s : (L - 1 - s)) : s;
          const f32x4 x0 = *reinterpret_cast<const f32x4*>(&ox_s[s & 1][row][g][c8]);
          const f32x4 x1 = *reinterpret_cast<const f32x4*>(&ox_s[s & 1][row][g][c8 + 4]);
          bf16x8 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            o[i] = (short)f2bf(x0[i] * a.dgx_scale);
            o[4 + i] = (short)f2bf(x1[i] * a.dgx_scale);
          }
          *reinterpret_cast<bf16x8*>(a.dgx + ((size_t)t * N + b) * a.gstride + dir * GH + g * H + u) = o;
        }
      }
    }
  };
  if (s_abort) return;
  if (wave == MEMW && a.steps > 0) mw_load(a.steps - 1);
  const bool plain = s_mode == 1;
  float* ringd = a.ring[dir];
  const size_t slot_floats = (size_t)a.BG * P * R * H;
  const unsigned ring_bytes = (unsigned)(3 * slot_floats * 4);
  const __amdgpu_buffer_rsrc_t rs_ring = make_rsrc(ringd, ring_bytes);
  Stamps st(a.stamps != nullptr && (wave == 0 || wave == MEMW) && lane == 0);

  // ring layout [slot][bg][producer][m-tile of 16 units][row][16] fp32: a producer's MFMA
  // tile (R rows x 16 units) is R*64 contiguous bytes (whole cache lines per store
  // instruction), and a consumer's 32 units from one producer (m-tiles 2*mem, 2*mem+1) are
  // 2*R*64 contiguous bytes, read by one wave as one coalesced sweep.
  // gather geometry (workers): combo c = lane + 64*cb -> (half = c / 4R, row, 4-unit
  // granule); this wave sums producers j = wave + 7*i
  const int pg7 = wave;
  const int ncb = (R * 8 + 63) / 64;          // combos per thread: 1 (R <= 8) or 2
  auto combo = [&](int cb, int& row, int& ucol) -> bool {
    const int c = lane + 64 * cb;
    const int half = c / (4 * R), rem = c - half * 4 * R;
    row = rem >> 2;
    ucol = 16 * half + 4 * (rem & 3);         // unit within this workgroup's 32
    return half < 2;
  };
  auto ring_off = [&](int slot, int j, int mt, int row, int u16) -> unsigned {
    return (unsigned)(((((((size_t)slot * a.BG + bg) * P + j) * MTS + mt) * R + row) * 16) + u16) * 4u;
  };
  // use tag of P(s): slot s % 3 is written at processing index k = steps-1-s, so its uses
  // are k, k+3, k+6, ... and (k / 3) & 1 alternates between consecutive uses; the ring is
  // filled with 0xFFFFFFFF (tag 1) and every slot's first use has tag 0
  auto tag_of = [&](int s) -> unsigned { return (unsigned)(((a.steps - 1 - s) / 3) & 1); };
  // bf16 layout [slot][bg][producer][unit pair p][row][g 0..3][8 bf16]: granule (row, g) of
  // pair p holds units 32p + {4g..4g+3, 16+4g..16+4g+3}
  const int NPR = MTS / 2;
  auto ring_off16 = [&](int slot, int j, int pr, int row, int g) -> unsigned {
    return (unsigned)((((((size_t)slot * a.BG + bg) * P + j) * NPR + pr) * R + row) * 4 + g) * 16u;
  };

  if (wave < MW) {
    // pre-gather sleep (ops/rnn.py poll_default), s_sleep 1 units; bit 29: units of 4 (the wide
    // plans, whose groups exchange across XCDs)
    const int presleep = ((a.knobs >> 20) & 7) << (((a.knobs >> 29) & 1) ? 2 : 0);
    for (int s = a.steps - 1; s >= 0; --s) {
      st.mark(-1);
      const bool has_next = s + 1 < a.steps;
      if (has_next)
        for (int i = 0; i < presleep; ++i) __builtin_amdgcn_s_sleep(1);
      // (G) sum this thread's producers' partials of dh_rec
      if constexpr (PBF == 2) {
        // 8 < R <= 16: lane -> (row, granule g), one producer per load instruction
        const int grow = lane >> 2, gg = lane & 3;
        float acc8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (has_next && grow < R) {
          const int cs = (s + 1) % 3;
          const unsigned want = tag_of(s + 1);
          unsigned off[GPT];
          i32x4 v[GPT];
          // at most CHB producers' granules in flight per lane (DS2_BWD_CH; 0 = all)
          constexpr int CHB = (DS2_BWD_CH > 0 && DS2_BWD_CH < GPT) ? DS2_BWD_CH : GPT;
#pragma unroll
          for (int i = 0; i < GPT; ++i) {
            const int j = min(pg7 + MW * i, P - 1);
            off[i] = ring_off16(cs, j, mem, grow, gg);
            if (i < CHB) v[i] = load_sc1_b128(rs_ring, off[i]);
          }
          const long long t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
          for (int i = 0; i < GPT; ++i) {
            if (i + CHB < GPT) v[i + CHB < GPT ? i + CHB : 0] = load_sc1_b128(rs_ring, off[i + CHB < GPT ? i + CHB : 0]);
            if (pg7 + MW * i < P) {
              while (!(a.knobs & 4) && !granule_tagged16(v[i], want)) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) { s_abort = 1; atomicOr(a.err, 1u); break; }
                if (!(a.knobs & 16384)) __builtin_amdgcn_s_sleep(1);   // back-off (knob 16384: none; measured neutral)
                v[i] = load_sc1_b128(rs_ring, off[i]);
              }
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                acc8[2 * q] += __uint_as_float((unsigned)v[i][q] << 16);
                acc8[2 * q + 1] += __uint_as_float((unsigned)v[i][q] & 0xffff0000u);
              }
            }
          }
        }
        if (grow < R) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            red_s[wave][grow][4 * gg + q] = acc8[q];
            red_s[wave][grow][16 + 4 * gg + q] = acc8[4 + q];
          }
        }
      } else if constexpr (PBF == 1) {
        // lane -> (producer half h, row, granule g); two producers per load instruction,
        // h = 1 partial sums go to red_s rows R..2R-1 (R <= 8), added in the epilogue
        const int h = lane >> 5, grow = (lane >> 2) & 7, gg = lane & 3;
        float acc8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (has_next && grow < R) {
          const int cs = (s + 1) % 3;
          const unsigned want = tag_of(s + 1);
          constexpr int NI = GPT / 2;
          unsigned off[NI];
          i32x4 v[NI];
#pragma unroll
          for (int i = 0; i < NI; ++i) {
            const int j = min(pg7 + MW * (2 * i + h), P - 1);
            off[i] = ring_off16(cs, j, mem, grow, gg);
            v[i] = load_sc1_b128(rs_ring, off[i]);
          }
          const long long t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
          for (int i = 0; i < NI; ++i) {
            if (pg7 + MW * (2 * i + h) < P) {
              while (!(a.knobs & 4) && !granule_tagged16(v[i], want)) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) { s_abort = 1; atomicOr(a.err, 1u); break; }
                if (!(a.knobs & 16384)) __builtin_amdgcn_s_sleep(1);   // back-off (knob 16384: none; measured neutral)
                v[i] = load_sc1_b128(rs_ring, off[i]);
              }
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                acc8[2 * q] += __uint_as_float((unsigned)v[i][q] << 16);
                acc8[2 * q + 1] += __uint_as_float((unsigned)v[i][q] & 0xffff0000u);
              }
            }
          }
        }
        if (grow < R) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            red_s[wave][grow + 8 * h][4 * gg + q] = acc8[q];
            red_s[wave][grow + 8 * h][16 + 4 * gg + q] = acc8[4 + q];
          }
        }
      } else
      for (int cb = 0; cb < ncb; ++cb) {
        int grow, gcol;
        if (!combo(cb, grow, gcol)) continue;
        f32x4 acc4 = f32x4{0.f, 0.f, 0.f, 0.f};
        if (has_next) {
          const int cs = (s + 1) % 3;
          const unsigned want = has_next ? tag_of(s + 1) : 0u;
          unsigned off[GPT];
          i32x4 v[GPT];
#pragma unroll
          for (int i = 0; i < GPT; ++i) {
            const int j = min(pg7 + MW * i, P - 1);
            off[i] = ring_off(cs, j, 2 * mem + (gcol >> 4), grow, gcol & 15);
            v[i] = load_sc1_b128(rs_ring, off[i]);
          }
          const long long t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
          for (int i = 0; i < GPT; ++i) {
            if (pg7 + MW * i < P) {
              while (!(a.knobs & 4) && !granule_tagged(v[i], want)) {   // knob 4: no wait (timing only)
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) { s_abort = 1; atomicOr(a.err, 1u); break; }
                if (!(a.knobs & 16384)) __builtin_amdgcn_s_sleep(1);   // back-off (knob 16384: none; measured neutral)
                v[i] = load_sc1_b128(rs_ring, off[i]);
              }
              acc4 += __builtin_bit_cast(f32x4, v[i]);
            }
          }
        }
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) red_s[wave][grow][gcol + jj] = acc4[jj];
      }
      st.mark(0);
      lds_barrier();                                                        // #1
      st.mark(1);
      // abort word read beside the partials, tested before barrier #2 (the memory wave tests
      // it there too): one LDS round trip less in front of the cell on every step
      const int ab = s_abort;
      // (E) cell backward (waves 0..3): dgh tile for the MFMA, dgx / dgh staging
      if (wave < EW) {
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
          const int e = tid + i * ETH;
          const int row = e >> 5, c = e & 31;
          if (row < R) {
            float dhrec = 0.f;
            if (has_next) {
              // pairwise tree over the worker waves' partials (fixed order: deterministic):
              // 3-4 dependent adds on the step's critical path instead of a chain of 7 / 14
              constexpr int NPART = (PBF == 1) ? 2 * MW : MW;
              float p[NPART];
#pragma unroll
              for (int w = 0; w < MW; ++w) {
                p[w] = red_s[w][row][c];
                if constexpr (PBF == 1) p[MW + w] = red_s[w][row + 8][c];
              }
#pragma unroll
              for (int d = 1; d < NPART; d *= 2)
#pragma unroll
                for (int w = 0; w + d < NPART; w += 2 * d) p[w] += p[w + d];
              dhrec = p[0];
            }
            const bool act = s < len_s[row];
            const float dh = dyr_s[s & 1][row][c] + carry[i] + dhrec;
            const float hp = hpr_s[s & 1][row][c];
            float ghv[G], gxs[G];
            float cnew = 0.f;
            if (CELL == CELL_GRU) {
              const float4 gv = gr_s[s & 1][(CELL == CELL_GRU) ? row : 0][c];
              const float r = gv.x, z = gv.y, n = gv.z, ghn = gv.w;
              const float dn = dh * (1.f - z);
              const float dz = dh * (hp - n);
              cnew = dh * z;
              const float dan = dn * (1.f - n * n);
              const float dr = dan * ghn;
              const float dghn = dan * r;
              const float daz = dz * z * (1.f - z);
              const float dar = dr * r * (1.f - r);
              ghv[0] = dar; ghv[1] = daz; ghv[2] = dghn;
              gxs[0] = dar; gxs[1] = daz; gxs[2] = dan;
            } else {
              const float da = (hp > 0.f && hp < RELU_CAP) ? dh : 0.f;
              ghv[0] = da;
              gxs[0] = da;
            }
            if (!act) {
              cnew = 0.f;
#pragma unroll
              for (int g = 0; g < G; ++g) { ghv[g] = 0.f; gxs[g] = 0.f; }
            }
            carry[i] = cnew;
#pragma unroll
            for (int g = 0; g < G; ++g) {
              const bf16_t hb = f2bf(ghv[g]);
              dg_s[row][g * UPW + c] = hb;
              oh_s[s & 1][row][g][c] = hb;
              ox_s[s & 1][row][g][c] = gxs[g];
              sbx[i][g] += gxs[g];
            }
            if (CELL == CELL_GRU) sbh[i] += ghv[G - 1];
          }
        }
      }
      st.mark(2);
      if (ab) break;
      lds_barrier();                                                        // #2
      st.mark(3);
      // (M) publish P(s) = dgh_s[:, own cols] . U[own cols, :] into ring slot s % 3
      if (s > 0) {
        const int ws = s % 3;
        const unsigned tg = tag_of(s);
        const unsigned tagmask = tg ? 0x00010001u : 0u;
        const bool prow = (lane & 15) < R;
        bf16x8 bfr[G];
#pragma unroll
        for (int g = 0; g < G; ++g)
          bfr[g] = *reinterpret_cast<const bf16x8*>(&dg_s[lane & 15][g * UPW + 8 * (lane >> 4)]);
        auto put = [&](int mt, f32x4 acc) {
          if (prow) {
            // the tag replaces the mantissa LSB (a 2^-23 relative perturbation of a partial)
            const i32x4 v = {(int)((__float_as_uint(canon32(acc[0])) & ~1u) | tg),
                             (int)((__float_as_uint(canon32(acc[1])) & ~1u) | tg),
                             (int)((__float_as_uint(canon32(acc[2])) & ~1u) | tg),
                             (int)((__float_as_uint(canon32(acc[3])) & ~1u) | tg)};
            const unsigned off = ring_off(ws, mem, mt, lane & 15, 4 * (lane >> 4));
            if (a.knobs & 32) {                          // knob 32 (timing only, with 4): no publish stores
            } else if (plain) store_b128(rs_ring, off, v);
            else store_sc1_b128(rs_ring, off, v);
          }
        };
        if constexpr (PBF) {
          // unit pair p = wave + 7k: m-tiles 2p, 2p+1 -> one tagged-bf16 granule per lane
          if (!(a.knobs & 40)) {
            // pair by pair: MFMA chains 2k, 2k+1, then the pair's convert/tag/store, so the
            // first granule leaves after 2G MFMAs. Measured against interleaving all MTU
            // chains (k-step outer, every store after the last MFMA; DS2_PUB_PIPE): 3.14 vs
            // 3.20 us/step, same box. No knob branch in here: a runtime `if` around the MFMAs
            // made the compiler zero 8 accumulator VGPRs per pair ahead of the first MFMA.
            constexpr int NP = MTU / 2;
            unsigned offp[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k) offp[k] = ring_off16(ws, mem, wave + MW * k, lane & 15, lane >> 4);
            // the store flavour is a compile-time branch of the whole loop (a runtime one per
            // store cost a select + compare + 3 scalar branches per pair)
            auto publish = [&](auto PLAIN) {
            auto store_pair = [&](int k, const f32x4& a0, const f32x4& a1) {
              if (prow && 2 * (wave + MW * k) + 1 < MTS) {
                const i32x4 v = {(int)bf16x2_tagged(a0[0], a0[1], tagmask), (int)bf16x2_tagged(a0[2], a0[3], tagmask),
                                 (int)bf16x2_tagged(a1[0], a1[1], tagmask), (int)bf16x2_tagged(a1[2], a1[3], tagmask)};
                if constexpr (decltype(PLAIN)::value) store_b128(rs_ring, offp[k], v);
                else store_sc1_b128(rs_ring, offp[k], v);
              }
            };
            // a pair past MTS multiplies the zero fragments loaded for it and is not stored
#pragma unroll
            for (int k = 0; k < NP; ++k) {
              f32x4 a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua[2 * k][0], bfr[0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
              f32x4 a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua[2 * k + 1][0], bfr[0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
              for (int g = 1; g < G; ++g) {
                a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua[2 * k][g], bfr[g], a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua[2 * k + 1][g], bfr[g], a1, 0, 0, 0);
              }
              store_pair(k, a0, a1);
            }
            };
            if (plain) publish(std::true_type{});
            else publish(std::false_type{});
          } else
#pragma unroll
          for (int i = 0; i < MTU; i += 2) {
            const int pr = wave + MW * (i >> 1);
            if (2 * pr + 1 < MTS) {
              f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
              if (!(a.knobs & 8)) {
#pragma unroll
                for (int g = 0; g < G; ++g) {
                  a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua[i][g], bfr[g], a0, 0, 0, 0);
                  a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua[i + 1][g], bfr[g], a1, 0, 0, 0);
                }
              }
              if (prow && !(a.knobs & 32)) {
                i32x4 v;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                  v[q] = (int)bf16x2_tagged(q < 2 ? a0[2 * q] : a1[2 * q - 4], q < 2 ? a0[2 * q + 1] : a1[2 * q - 3],
                                            tagmask);
                const unsigned off = ring_off16(ws, mem, pr, lane & 15, lane >> 4);
                if (plain) store_b128(rs_ring, off, v);
                else store_sc1_b128(rs_ring, off, v);
              }
            }
          }
        } else
        // two independent accumulator chains at a time hide the MFMA dependency latency
#pragma unroll
        for (int i = 0; i < MTU; i += 2) {
          const int mt0 = wave + MW * i, mt1 = wave + MW * (i + 1);
          if (mt1 < MTS) {
            f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
            if (!(a.knobs & 8)) {                        // knob 8: no MFMA (timing only)
#pragma unroll
              for (int g = 0; g < G; ++g) {
                a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua[i][g], bfr[g], a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua[i + 1][g], bfr[g], a1, 0, 0, 0);
              }
            }
            put(mt0, a0);
            put(mt1, a1);
          } else if (mt0 < MTS) {
            f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int g = 0; g < G; ++g) a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua[i][g], bfr[g], a0, 0, 0, 0);
            put(mt0, a0);
          }
        }
      }
      st.mark(4);
    }
  } else {
    for (int s = a.steps - 1; s >= 0; --s) {
      // memory wave, while the others wait on the exchange
      st.mark(-1);
      mw_put(s);
      st.mark(2);                 // memory wave: acc[2] = put (incl. its load wait), acc[0] = store + load issue
      if (s + 2 < a.steps) mw_store(s + 2);
      if (s >= 1) mw_load(s - 1);
      st.mark(0);
      lds_barrier();                                                        // #1
      st.mark(1);
      if (s_abort) break;
      lds_barrier();                                                        // #2
    }
  }
  __syncthreads();
  if (wave == MEMW && !s_abort) {
    if (a.steps >= 2) mw_store(1);
    if (a.steps >= 1) mw_store(0);
  }
  if (wave == 0) { st.acc[5] = (unsigned long long)(s_mode + 10); st.store(a.stamps, 0); }
  if (wave == MEMW && st.on) { a.stamps[(size_t)blockIdx.x * 8 + 6] = st.acc[0]; a.stamps[(size_t)blockIdx.x * 8 + 7] = st.acc[1]; }

  // bias gradients: reduce the epilogue waves' rows through LDS, one read-modify-write
  // per (gate, unit) of the workgroup's own [bg] partial row
  if (a.dbx_part[dir] != nullptr && !s_abort) {
    constexpr int BW = (G + 1) * UPW;
    static_assert(MW * ROWS * (UPW + 1) >= ROWS * BW, "bias reduction does not fit the LDS scratch");
    float* bred = &red_s[0][0][0];
    if (wave < EW) {
#pragma unroll
      for (int i = 0; i < EPT; ++i) {
        const int e = tid + i * ETH;
        const int row = e >> 5, c = e & 31;
#pragma unroll
        for (int g = 0; g < G; ++g) bred[row * BW + g * UPW + c] = sbx[i][g];
        bred[row * BW + G * UPW + c] = sbh[i];
      }
    }
    __syncthreads();
    for (int q = tid; q < BW; q += NTH) {
      float sum = 0.f;
      for (int r = 0; r < ROWS; ++r) sum += bred[r * BW + q];
      const int g = q / UPW, c = q % UPW;
      const size_t base = (size_t)bg * GH + u0 + c;
      if (g < G) {
        a.dbx_part[dir][base + (size_t)g * H] += sum;
        if (CELL == CELL_GRU && a.dbh_part[dir] != nullptr && g < G - 1) a.dbh_part[dir][base + (size_t)g * H] += sum;
      } else if (CELL == CELL_GRU && a.dbh_part[dir] != nullptr) {
        a.dbh_part[dir][base + (size_t)(G - 1) * H] += sum;
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// Wide one-gate layers (the reference's 7 x bi-RNN(ReLU)-1760, src/train.sh:42): 64 units
// per workgroup, so a group is P = ceil(H/64) <= 28 workgroups and fits ONE XCD (H/32 = 55
// did not: two per CU measured slower, profiles/r3_negative_results.md).
//
// Forward (rnnw_fwd_kernel): 8 MFMA waves = 8 K-eighths (k-steps ke + 8 kk), each over all
// four 16-unit n-tiles of the workgroup, so every exchange granule is polled by ONE wave of
// the workgroup. (The first version split the waves into 2 unit halves x 4 K-quarters like
// the generation-4 forward: both halves polled the same granules, and with 14 granules per
// lane the CU's vector-memory pipe, not the MFMAs, set the step: 5.4 us/step, 5.1 without any
// MFMA.) Transpose-reduce over the 8 K-eighths: of the 16 (tile, element j) slots of a lane,
// wave w finalises tile w >> 1, elements j = 2 (w & 1) + {0, 1}; every wave stores its 16
// slots, ONE barrier, then each owner adds the 8 partials of its two. Every exchange granule
// of the wave's K-eighth is in flight at once (poll_mfma_par); the last KL of its U k-steps
// live in LDS. The last workgroup of a group may be half empty (H % 64 == 32): its units >= H
// have zero U rows, load no gx and store nothing.
// ------------------------------------------------------------------------------------
constexpr int UWW = 64;           // hidden units per workgroup of the wide kernels
constexpr int wide_kl(int kb) { return kb >= 7 ? 2 : 0; }   // U k-steps per wave in LDS (register budget: 1 spilled at KB = 7)

template <int KB, int KL, bool STAMPS = false>
__global__ __launch_bounds__(QTH) void rnnw_fwd_kernel(XFwd a) {
  using StampT = typename std::conditional<STAMPS, Stamps, NoStamps>::type;
  constexpr int NT = 4;                           // 16-unit n-tiles per MFMA wave (all 64 units)
  constexpr int KR = KB - KL;
  static_assert(KL >= 0 && KR >= 1, "register k-steps");
  constexpr int ROWS = 16;
  constexpr int GP = UWW + 4;                     // gx ring row pitch (floats)
  constexpr int OP = UWW + 4;                     // output staging row pitch
  constexpr int RGL = ROWS * (UWW / 8) / 64;      // gx granules per memory-wave lane (2)
  constexpr int LPR = UWW / 4;                    // output lanes per row (4 units each)
  constexpr int RPP = 64 / LPR;                   // rows per output pass
  constexpr int NPS = ROWS / RPP;                 // output passes
  __shared__ float red_s[2][QW][16][64];          // [parity][source wave][slot 4 t + j][lane]
  __shared__ float gxr_s[2][ROWS][GP];
  // h only: the output y is h where the step is active and 0 past the length (the memory
  // wave knows which), so no y staging
  __shared__ __attribute__((aligned(16))) float oh_s[2][ROWS][OP];
  __shared__ int len_s[ROWS];
  __shared__ int s_mode, s_abort;
  __shared__ bf16x8 ul_s[KL > 0 ? KL : 1][QW][NT][64];   // LDS-resident U k-steps

  int grp, mem;
  if (!take_role(a.xcd_map, a.ngroups, a.P, grp, mem)) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, KS = H / 32, N = a.N, NP = a.NP, R = a.R;
  const int bg = grp % a.BG, dir = grp / a.BG;
  const int r0 = bg * R, u0 = mem * UWW;
  const int ke = wave;                            // K-eighth (MFMA waves)
  const int tw = wave >> 1, j0 = 2 * (wave & 1);  // owned tile and first owned element
  if (tid < ROWS) len_s[tid] = (tid < R && r0 + tid < N) ? a.lens[r0 + tid] : 0;
  if (wave == 0) {
    const int m = group_census(a.census, grp, mem, a.P, a.timeout, a.err);
    if (lane == 0) { s_mode = m; s_abort = (m < 0); }
  }
  __syncthreads();
  if (s_abort) return;

  // memory wave: gx granule q -> (row, 8-unit chunk)
  i32x4 gpre[RGL];
  auto mw_load = [&](int s) {
#pragma unroll
    for (int j = 0; j < RGL; ++j) {
      const int q = lane + 64 * j;
      const int row = q / (UWW / 8), c8 = q % (UWW / 8);
      const int b = min(r0 + min(row, R - 1), N - 1);
      const int t = max(0, min((dir == 0) ? s : (len_s[min(row, R - 1)] - 1 - s), a.T - 1));
      const int u = min(u0 + c8 * 8, H - 8);
      gpre[j] = *reinterpret_cast<const i32x4*>(a.gx + ((size_t)t * N + b) * a.gstride + dir * H + u);
    }
  };
  auto mw_put = [&](int s) {
#pragma unroll
    for (int j = 0; j < RGL; ++j) {
      const int q = lane + 64 * j;
      const int row = q / (UWW / 8), c8 = q % (UWW / 8);
      if (row < R) {
        const bool act = s < len_s[row] && u0 + c8 * 8 < H;
        const bf16x8 v = __builtin_bit_cast(bf16x8, gpre[j]);
#pragma unroll
        for (int k = 0; k < 8; ++k) gxr_s[s & 1][row][c8 * 8 + k] = act ? bf2f((bf16_t)v[k]) : 0.f;
      }
    }
  };
  unsigned long long yq[NPS];
#pragma unroll
  for (int j = 0; j < NPS; ++j) yq[j] = 0ull;
  auto ysum_ptr = [&](int s, int j) -> unsigned long long* {
    const int row = min((lane / LPR) + RPP * j, R - 1), c4 = (lane % LPR) * 4;
    const int b = min(r0 + row, N - 1), L = len_s[row];
    const int t = (s < L) ? ((dir == 0) ? s : (L - 1 - s)) : s;
    return reinterpret_cast<unsigned long long*>(a.ysum + ((size_t)t * N + b) * H + min(u0 + c4, H - 4));
  };
  auto mw_ysum_load = [&](int s) {
#pragma unroll
    for (int j = 0; j < NPS; ++j)
      if (RPP * j < R) yq[j] = __hip_atomic_load(ysum_ptr(s, j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // outputs of step s out of staging slot s & 1: lane -> (row, 4 consecutive units) per pass
  auto mw_store = [&](int s) {
#pragma unroll
    for (int j = 0; j < NPS; ++j) {
      const int row = (lane / LPR) + RPP * j, c4 = (lane % LPR) * 4;
      const int u = u0 + c4;
      if (row < R && u < H) {
        const int b = r0 + row;
        const f32x4 vh = *reinterpret_cast<const f32x4*>(&oh_s[s & 1][row][c4]);
        *reinterpret_cast<f32x4*>(a.hsave[dir] + ((size_t)(s + 1) * NP + b) * H + u) = vh;
        if (b < N) {
          const int L = len_s[row];
          const int t = (s < L) ? ((dir == 0) ? s : (L - 1 - s)) : s;
          const f32x4 vy = (s < L) ? vh : f32x4{0.f, 0.f, 0.f, 0.f};
          uint2 o;
          o.x = (unsigned)f2bf(vy[0]) | ((unsigned)f2bf(vy[1]) << 16);
          o.y = (unsigned)f2bf(vy[2]) | ((unsigned)f2bf(vy[3]) << 16);
          if (a.ysum == nullptr) {
            *reinterpret_cast<uint2*>(a.y[dir] + ((size_t)t * N + b) * H + u) = o;
          } else {
            // fused direction sum: same protocol as rnnq_fwd_kernel (the later producer of a
            // position waits for the other's bf16 value and stores the rounded bf16 sum)
            unsigned long long* p = ysum_ptr(s, j);
            const int other = (s < L) ? (L - 1 - s) : s;
            const bool later = s > other || (s == other && dir == 1);
            auto canon = [](unsigned h) { return (h & 0xffffu) == 0xffffu ? 0x7fc0u : (h & 0xffffu); };
            if (!later) {
              o.x = canon(o.x) | (canon(o.x >> 16) << 16);
              o.y = canon(o.y) | (canon(o.y >> 16) << 16);
              __hip_atomic_store(p, ((unsigned long long)o.y << 32) | o.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
              const long long t0 = __builtin_amdgcn_s_memrealtime();
              unsigned long long q = yq[j];
              while (true) {
                const unsigned w0 = (unsigned)q, w1 = (unsigned)(q >> 32);
                const bool ready = ((~w0 - 0x00010001u) & w0 & 0x80008000u) == 0 &&
                                   ((~w1 - 0x00010001u) & w1 & 0x80008000u) == 0;
                if (ready) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) { atomicOr(a.err, 4u); break; }
                __builtin_amdgcn_s_sleep(2);
                q = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              }
              const unsigned q0 = (unsigned)q, q1 = (unsigned)(q >> 32);
              auto add2 = [](unsigned x, unsigned y) {
                const unsigned lo = f2bf(__uint_as_float(x << 16) + __uint_as_float(y << 16));
                const unsigned hi = f2bf(__uint_as_float(x & 0xffff0000u) + __uint_as_float(y & 0xffff0000u));
                return lo | (hi << 16);
              };
              *reinterpret_cast<uint2*>(p) = make_uint2(add2(o.x, q0), add2(o.y, q1));
            }
          }
        }
      }
    }
  };
  if (wave == QW) {
    mw_load(0);
    mw_put(0);
    if (a.steps > 1) mw_load(1);
  }
  __syncthreads();   // gx ring slot 0
  const bool plain = s_mode == 1;
  const unsigned hx_bytes = (unsigned)((size_t)(a.steps + 1) * NP * H * 2);
  bf16_t* hxd = a.hx[dir];
  const __amdgpu_buffer_rsrc_t rs_hx = make_rsrc(hxd, hx_bytes);
  StampT st(a.stamps != nullptr && (wave == 0 || wave == QW) && lane == 0);

  if (wave < QW) {
    const int lu = 16 * tw + (lane & 15);          // this lane's local unit (owned tile)
    const bool uok = u0 + lu < H;
    // resident U fragments: B[k][c] = U[u0 + 16 t + c][ks*32 + k], ks = ke + 8*kk
    bf16x8 uf[KR][NT];
    bool kval[KB];
    float hreg[2];
    int erow[2];
    {
      const bf16_t* Ud = a.U[dir];
#pragma unroll
      for (int kk = 0; kk < KB; ++kk) {
        const int ks = ke + 8 * kk;
        kval[kk] = ks < KS;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
          const int ur = u0 + 16 * t + (lane & 15);
          if (kval[kk] && ur < H)
            v = *reinterpret_cast<const bf16x8*>(Ud + (size_t)ur * H + ks * 32 + 8 * (lane >> 4));
          if (kk < KR) uf[kk < KR ? kk : 0][t] = v;
          else ul_s[kk >= KR ? kk - KR : 0][wave][t][lane] = v;   // own slot: no barrier needed
        }
      }
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        erow[e] = 4 * (lane >> 4) + j0 + e;
        hreg[e] = (erow[e] < R && uok) ? a.hsave[dir][(size_t)(r0 + erow[e]) * H + u0 + lu] : 0.f;   // slot 0 = h0
      }
    }
    const int arow = r0 + min(lane & 15, R - 1);
    drain_vm();        // nothing from before the loop pending inside it (as rnne_fwd_kernel)
    const int presleep = (a.knobs >> 17) & 7;   // pre-poll sleep (ops/rnn.py POLL_DEFAULT)
    for (int s = 0; s < a.steps; ++s) {
      st.mark(-1);
      if (s > 0)
        for (int i = 0; i < presleep; ++i) __builtin_amdgcn_s_sleep(1);
      float gxv[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) gxv[e] = gxr_s[s & 1][erow[e]][lu];
      // every k-step's granule is a constant 512 B past the first (immediate offsets); a
      // k-step past K (kval false) is never waited on
      unsigned off[KB];
      const unsigned o0 = (unsigned)((((size_t)s * NP + arow) * H + ke * 32 + 8 * (lane >> 4)) * 2);
#pragma unroll
      for (int kk = 0; kk < KB; ++kk) off[kk] = o0 + 512u * kk;
      f32x4 acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const bool nomfma = (a.knobs & 4) != 0;           // knob 4: no MFMA (timing only, wrong results)
      auto mfma_k = [&](int kk, bf16x8 af) {
        if (nomfma) { acc[0][0] += __builtin_bit_cast(float, (int)af[0]); return; }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const bf16x8 b = kk < KR ? uf[kk < KR ? kk : 0][t] : ul_s[kk >= KR ? kk - KR : 0][wave][t][lane];
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, b, acc[t], 0, 0, 0);
        }
      };
      const bool ok = poll_mfma_par<KB>(rs_hx, off, kval, a.timeout, (a.knobs >> 12) & 3, mfma_k);
      if (!ok) { s_abort = 1; atomicOr(a.err, 1u); }
      st.mark(0);
      // transpose-reduce: every slot q = 4 t + j to LDS (the owned two as well: a register
      // array indexed by the wave-dependent tile would live in scratch), one barrier, then
      // the owner sums the 8 K-eighths of its slots 4 tw + j0 + {0, 1} in wave order
#pragma unroll
      for (int q = 0; q < 16; ++q) red_s[s & 1][wave][q][lane] = acc[q >> 2][q & 3];
      st.mark(1);
      lds_barrier();
      st.mark(2);
      if (s_abort) break;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int q = 4 * tw + j0 + e;
        float pre = 0.f;
#pragma unroll
        for (int w = 0; w < QW; ++w) pre += red_s[s & 1][w][q][lane];
        const int row = erow[e];
        const int L = len_s[row];
        const bool act = s < L;
        const float hn = fminf(fmaxf(gxv[e] + pre, 0.f), RELU_CAP);
        const float hnew = act ? hn : hreg[e];
        hreg[e] = hnew;
        unsigned hq = (unsigned)__builtin_bit_cast(unsigned short, (__bf16)hnew);
        hq = hq == 0xffffu ? 0x7fc0u : hq;
        // 16-B exchange granule = 8 consecutive units of one row = 8 consecutive lanes
        const unsigned pr = hq | ((unsigned)__builtin_amdgcn_update_dpp(0, (int)hq, 0x101, 0xf, 0xf, false) << 16);
        const int q1 = __builtin_amdgcn_update_dpp(0, (int)pr, 0x102, 0xf, 0xf, false);
        const int q2 = __builtin_amdgcn_update_dpp(0, (int)pr, 0x104, 0xf, 0xf, false);
        const int q3 = __builtin_amdgcn_update_dpp(0, (int)pr, 0x106, 0xf, 0xf, false);
        if ((lane & 7) == 0 && row < R && uok) {
          const i32x4 v = {(int)pr, q1, q2, q3};
          const unsigned off2 = (unsigned)((((size_t)(s + 1) * NP + r0 + row) * H + u0 + lu) * 2);
          store_granule(plain, rs_hx, hxd, off2, v);
        }
        oh_s[s & 1][row][lu] = hnew;
      }
      st.mark(4);
    }
  } else {
    for (int s = 0; s < a.steps; ++s) {
      st.mark(-1);
      if (a.ysum != nullptr && s >= 2) mw_ysum_load(s - 2);
      if (s + 1 < a.steps) mw_put(s + 1);
      if (s >= 2 && !(a.knobs & 2)) mw_store(s - 2);     // knob 2: no output stores (timing only)
      if (s + 2 < a.steps) mw_load(s + 2);
      st.mark(0);
      lds_barrier();
      st.mark(1);
      if (s_abort) break;
    }
  }
  __syncthreads();
  if (wave == QW && !s_abort) {
    if (a.steps >= 2) {
      if (a.ysum != nullptr) mw_ysum_load(a.steps - 2);
      mw_store(a.steps - 2);
    }
    if (a.steps >= 1) {
      if (a.ysum != nullptr) mw_ysum_load(a.steps - 1);
      mw_store(a.steps - 1);
    }
  }
  if (STAMPS && wave == 0) { st.acc[5] = (unsigned long long)(s_mode + 10); st.store(a.stamps, 0); }
  if (STAMPS && wave == QW && st.on) { a.stamps[(size_t)blockIdx.x * 8 + 6] = st.acc[0]; a.stamps[(size_t)blockIdx.x * 8 + 7] = st.acc[1]; }
}

// ------------------------------------------------------------------------------------
// Wide one-gate BPTT (rnnw_bwd_kernel): the reduce-scatter protocol of rnnrs_bwd_kernel
// (tagged-bf16 partials in a 3-slot ring, R <= 8 rows, two producers per gather load) with
// 64-unit workgroups. A producer's own columns are its 64 units (two 32-column k-steps), so
// its partial P_j(s) = da_s[:, own] . U[own, :] covers all H units in MTS = H/16 m-tiles,
// published in unit pairs (32 units per 16-B granule row); a consumer gathers the two pairs
// of its 64 units from every producer.
// ------------------------------------------------------------------------------------
template <int MTU, int GPT, bool STAMPS = false>
__global__ __launch_bounds__(NTH) void rnnw_bwd_kernel(XBwdRS a) {
  using StampT = typename std::conditional<STAMPS, Stamps, NoStamps>::type;
  constexpr int ROWS = 16;
  constexpr int KG = UWW / 32;                    // 32-column k-steps of the own columns (2)
  constexpr int EPT = ROWS * UWW / ETH;           // epilogue elements per thread (4)
  constexpr int DGP = UWW + 8;                    // da tile pitch (bf16)
  constexpr int LT = ROWS * (UWW / 4) / 64;       // memory-wave load tasks per lane (4)
  constexpr int ST = ROWS * (UWW / 8) / 64;       // memory-wave store tasks per lane (2)
  static_assert(GPT % 2 == 0, "two producers per gather load");
  __shared__ float red_s[MW][ROWS][UWW + 1];
  __shared__ __attribute__((aligned(16))) bf16_t dg_s[ROWS][DGP];
  __shared__ float dyr_s[2][ROWS][UWW];
  __shared__ float hpr_s[2][ROWS][UWW];
  __shared__ __attribute__((aligned(16))) float ox_s[2][ROWS][UWW];
  __shared__ __attribute__((aligned(16))) bf16_t oh_s[2][ROWS][UWW];
  __shared__ int len_s[ROWS];
  __shared__ int s_mode, s_abort;

  int grp, mem;
  if (!take_role(a.xcd_map, a.ngroups, a.P, grp, mem)) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, N = a.N, NP = a.NP, R = a.R, P = a.P, MTS = H / 16, NPR = MTS / 2;
  const int bg = grp % a.BG, dir = grp / a.BG;
  const int r0 = bg * R, u0 = mem * UWW;
  if (tid < ROWS) len_s[tid] = (tid < R && r0 + tid < N) ? a.lens[r0 + tid] : 0;
  for (int i = tid; i < ROWS * DGP; i += NTH) (&dg_s[0][0])[i] = 0;
  if (wave == 0) {
    const int m = group_census(a.census, grp, mem, P, a.timeout, a.err);
    if (lane == 0) { s_mode = m; s_abort = (m < 0); }
  }

  // resident A fragments: A[m][k] = U[u0 + 32 kg + k][16 mt + m], m-tile mt of unit pair
  // wave + 7 (i >> 1) (tiles 2p, 2p + 1); own columns >= H (half-empty last workgroup) are 0
  bf16x8 ua[MTU][KG];
  {
    const bf16_t* Ud = a.U[dir];
#pragma unroll
    for (int i = 0; i < MTU; ++i) {
      const int mt = 2 * (wave + MW * (i >> 1)) + (i & 1);
#pragma unroll
      for (int kg = 0; kg < KG; ++kg) {
        bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        const int col0 = u0 + 32 * kg + 8 * (lane >> 4);
        if (wave < MW && mt < MTS && col0 < H) {
          const bf16_t* p = Ud + (size_t)col0 * H + 16 * mt + (lane & 15);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (short)p[(size_t)j * H];
        }
        ua[i][kg] = v;
      }
    }
  }
  float sbx[EPT];
#pragma unroll
  for (int i = 0; i < EPT; ++i) sbx[i] = 0.f;
  __syncthreads();   // len_s, dg_s zero rows, census

  // memory wave: load task = (row, 4 units), store task = (row, 8 units)
  uint2 pdy[LT];
  float4 php[LT];
  auto mw_load = [&](int s) {
#pragma unroll
    for (int k = 0; k < LT; ++k) {
      const int q = lane + 64 * k;
      const int row = q / (UWW / 4), c4 = (q % (UWW / 4)) * 4;
      if (row < R && u0 + c4 < H) {
        const int bp = min(r0 + row, NP - 1), bn = min(r0 + row, N - 1), u = u0 + c4;
        const int t = max(0, min((dir == 0) ? s : (len_s[row] - 1 - s), a.T - 1));
        pdy[k] = *reinterpret_cast<const uint2*>(a.dy + ((size_t)t * N + bn) * H + u);
        php[k] = *reinterpret_cast<const float4*>(a.hsave[dir] + ((size_t)(s + 1) * NP + bp) * H + u);   // h_s
      }
    }
  };
  auto mw_put = [&](int s) {
    const int slot = s & 1;
#pragma unroll
    for (int k = 0; k < LT; ++k) {
      const int q = lane + 64 * k;
      const int row = q / (UWW / 4), c4 = (q % (UWW / 4)) * 4;
      if (row < R) {
        const bool act = s < len_s[row] && u0 + c4 < H;
        const float dv[4] = {bf2f((bf16_t)(pdy[k].x & 0xffffu)), bf2f((bf16_t)(pdy[k].x >> 16)),
                             bf2f((bf16_t)(pdy[k].y & 0xffffu)), bf2f((bf16_t)(pdy[k].y >> 16))};
        const float hv[4] = {php[k].x, php[k].y, php[k].z, php[k].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          dyr_s[slot][row][c4 + i] = act ? dv[i] : 0.f;
          hpr_s[slot][row][c4 + i] = act ? hv[i] : 0.f;
        }
      }
    }
  };
  auto mw_store = [&](int s) {          // da (= dgh = dgx of the one gate) of step s
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      const int q = lane + 64 * k;
      const int row = q / (UWW / 8), c8 = (q % (UWW / 8)) * 8;
      const int b = r0 + row, u = u0 + c8;
      if (row < R && u < H) {
        *reinterpret_cast<i32x4*>(a.dgh[dir] + ((size_t)s * NP + b) * H + u) =
            *reinterpret_cast<const i32x4*>(&oh_s[s & 1][row][c8]);
        if (b < N) {
          const int L = len_s[row];
          const int t = (s < L) ? ((dir == 0) ? s : (L - 1 - s)) : s;
          const f32x4 x0 = *reinterpret_cast<const f32x4*>(&ox_s[s & 1][row][c8]);
          const f32x4 x1 = *reinterpret_cast<const f32x4*>(&ox_s[s & 1][row][c8 + 4]);
          bf16x8 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            o[i] = (short)f2bf(x0[i] * a.dgx_scale);
            o[4 + i] = (short)f2bf(x1[i] * a.dgx_scale);
          }
          *reinterpret_cast<bf16x8*>(a.dgx + ((size_t)t * N + b) * a.gstride + dir * H + u) = o;
        }
      }
    }
  };
  if (s_abort) return;
  if (wave == MEMW && a.steps > 0) mw_load(a.steps - 1);
  const bool plain = s_mode == 1;
  const size_t slot_floats = (size_t)a.BG * P * R * H;
  const unsigned ring_bytes = (unsigned)(3 * slot_floats * 4);
  const __amdgpu_buffer_rsrc_t rs_ring = make_rsrc(a.ring[dir], ring_bytes);
  auto tag_of = [&](int s) -> unsigned { return (unsigned)(((a.steps - 1 - s) / 3) & 1); };
  StampT st(a.stamps != nullptr && (wave == 0 || wave == MEMW) && lane == 0);
  // [slot][bg][producer][unit pair][row][granule g][8 bf16]: granule (row, g) of pair p holds
  // units 32 p + {4 g .. 4 g + 3, 16 + 4 g .. 16 + 4 g + 3}
  auto ring_off16 = [&](int slot, int j, int pr, int row, int g) -> unsigned {
    return (unsigned)((((((size_t)slot * a.BG + bg) * P + j) * NPR + pr) * R + row) * 4 + g) * 16u;
  };

  if (wave < MW) {
    const int presleep = (a.knobs >> 20) & 7;     // A/B: s_sleep 1 units before the gather
    for (int s = a.steps - 1; s >= 0; --s) {
      st.mark(-1);
      const bool has_next = s + 1 < a.steps;
      if (has_next)
        for (int i = 0; i < presleep; ++i) __builtin_amdgcn_s_sleep(1);
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
              const int j = min(wave + MW * (2 * i + h), P - 1);
              off[pp][i] = ring_off16(cs, j, min(2 * mem + pp, NPR - 1), grow, gg);
              v[pp][i] = load_sc1_b128(rs_ring, off[pp][i]);
            }
          const long long t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
          for (int pp = 0; pp < 2; ++pp) {
            if (2 * mem + pp >= NPR) continue;            // half-empty last workgroup
#pragma unroll
            for (int i = 0; i < NI; ++i) {
              if (wave + MW * (2 * i + h) < P) {
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
      st.mark(0);
      lds_barrier();                                                        // #1
      st.mark(1);
      if (s_abort) break;
      // (E) cell backward (waves 0..3): da tile for the MFMA, dgh / dgx staging
      if (wave < EW) {
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
          const int e = tid + i * ETH;
          const int row = e / UWW, c = e % UWW;
          if (row < R) {
            float dhrec = 0.f;
            if (has_next) {
#pragma unroll
              for (int w = 0; w < MW; ++w) dhrec += red_s[w][row][c] + red_s[w][row + 8][c];
            }
            const bool act = s < len_s[row] && u0 + c < H;
            const float dh = dyr_s[s & 1][row][c] + dhrec;
            const float hp = hpr_s[s & 1][row][c];
            const float da = (act && hp > 0.f && hp < RELU_CAP) ? dh : 0.f;
            const bf16_t hb = f2bf(da);
            dg_s[row][c] = hb;
            oh_s[s & 1][row][c] = hb;
            ox_s[s & 1][row][c] = da;
            sbx[i] += da;
          }
        }
      }
      st.mark(2);
      lds_barrier();                                                        // #2
      st.mark(3);
      // (M) publish P(s) = da_s[:, own cols] . U[own cols, :] into ring slot s % 3
      if (s > 0) {
        const int ws = s % 3;
        const unsigned tagmask = tag_of(s) ? 0x00010001u : 0u;
        const bool prow = (lane & 15) < R;
        bf16x8 bfr[KG];
#pragma unroll
        for (int kg = 0; kg < KG; ++kg)
          bfr[kg] = *reinterpret_cast<const bf16x8*>(&dg_s[lane & 15][32 * kg + 8 * (lane >> 4)]);
        constexpr int NPW = MTU / 2;
        unsigned offp[NPW];
#pragma unroll
        for (int k = 0; k < NPW; ++k) offp[k] = ring_off16(ws, mem, min(wave + MW * k, NPR - 1), lane & 15, lane >> 4);
        auto publish = [&](auto PLAIN) {
#pragma unroll
          for (int k = 0; k < NPW; ++k) {
            f32x4 a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua[2 * k][0], bfr[0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            f32x4 a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua[2 * k + 1][0], bfr[0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
            for (int kg = 1; kg < KG; ++kg) {
              a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua[2 * k][kg], bfr[kg], a0, 0, 0, 0);
              a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua[2 * k + 1][kg], bfr[kg], a1, 0, 0, 0);
            }
            if (prow && wave + MW * k < NPR) {
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
      st.mark(4);
    }
  } else {
    for (int s = a.steps - 1; s >= 0; --s) {
      st.mark(-1);
      mw_put(s);
      if (s + 2 < a.steps) mw_store(s + 2);
      if (s >= 1) mw_load(s - 1);
      st.mark(0);
      lds_barrier();                                                        // #1
      st.mark(1);
      if (s_abort) break;
      lds_barrier();                                                        // #2
    }
  }
  __syncthreads();
  if (wave == MEMW && !s_abort) {
    if (a.steps >= 2) mw_store(1);
    if (a.steps >= 1) mw_store(0);
  }
  if (STAMPS && wave == 0) { st.acc[5] = (unsigned long long)(s_mode + 10); st.store(a.stamps, 0); }
  if (STAMPS && wave == MEMW && st.on) { a.stamps[(size_t)blockIdx.x * 8 + 6] = st.acc[0]; a.stamps[(size_t)blockIdx.x * 8 + 7] = st.acc[1]; }
  // input-bias gradient: reduce the epilogue waves' rows through LDS
  if (a.dbx_part[dir] != nullptr && !s_abort) {
    float* bred = &red_s[0][0][0];
    if (wave < EW) {
#pragma unroll
      for (int i = 0; i < EPT; ++i) {
        const int e = tid + i * ETH;
        bred[(e / UWW) * UWW + e % UWW] = sbx[i];
      }
    }
    __syncthreads();
    for (int q = tid; q < UWW; q += NTH) {
      float sum = 0.f;
      for (int r = 0; r < ROWS; ++r) sum += bred[r * UWW + q];
      if (u0 + q < H) a.dbx_part[dir][(size_t)bg * H + u0 + q] += sum;
    }
  }
}

template <int CELL, int MT>
static int launch_fwd(const XFwd& a, int kb, int grid, size_t smem, hipStream_t st) {
  switch (kb) {
#define DS2_CASE(K)                                                                           \
  case K:                                                                                     \
    hipLaunchKernelGGL((rnnx_fwd_kernel<CELL, MT, K>), dim3(grid), dim3(NTH), smem, st, a); \
    break;
    DS2_CASE(1) DS2_CASE(2) DS2_CASE(3) DS2_CASE(4) DS2_CASE(5) DS2_CASE(6)
#undef DS2_CASE
    default: return -31;
  }
  return (int)hipGetLastError();
}

template <typename F>
static int set_smem_attr(F kernel, size_t smem) {
  return (int)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
}

}  // namespace

extern "C" {

struct DS2RnnX {
  int T, N, NP, H, BG, R, steps, gstride, ndir, cell, mt, xcd_map, knobs;
  const int* lens;
  const void* gx;        // fwd: gx;  bwd: dy
  const void* U[2];
  const float* bh[2];
  void* y[2];            // fwd: y
  void* ex[2];           // fwd: hx exchange;  bwd: dgh exchange
  float* hsave[2];
  float* gates[2];
  void* dgx;
  float* dbx_part[2];
  float* dbh_part[2];
  float dgx_scale;
  unsigned* census;
  unsigned* err;
  long long timeout;
  unsigned long long* stamps;
  void* ring[2];         // bwd reduce-scatter exchange ring (fp32, sentinel-filled)
  void* ysum;            // fwd gen 4: fused direction sum (sentinel-filled) or null
};

// 1 if the forward launch for these parameters is generation 4 (which can fuse the
// direction sum into its output stores)
// generation 4 serves k-steps per wave kbq <= 8 (ReLU) / <= 10 (GRU: beyond 7, the last
// kbq - 7 of each wave's U k-steps are LDS-resident; knob 65536 keeps H = 1280 on gen 2)
// wide one-gate layers (rnnw_*): 64 units per workgroup, 32 < H/32 and H <= 1792
static bool wide_ok(int H, int cell) { return cell == CELL_RELU && H % 32 == 0 && H / 32 > 32 && H <= 1792; }
static int xcd_p(int H, int cell) { return wide_ok(H, cell) ? (H + UWW - 1) / UWW : H / UPW; }

static bool gen4_ok(int H, int cell, int mt, int knobs) {
  const int kbq = (H / 32 + 3) / 4;
  if ((knobs & 256) || mt != 1) return false;
  if (cell == CELL_GRU) return kbq <= 7 || (kbq <= 10 && (H / 32) % 4 == 0 && !(knobs & 65536));
  return kbq <= 8;
}

int ds2_rnnx_kb(int H, int G, int fwd);

// Which forward kernel family ds2_rnnx_fwd launches for a geometry (the dispatch below and
// the report binding rnnx_fwd_family share this one function): 6 rnnw (wide one-gate), 5 rnne
// (GRU, K-eighths), 4 rnnq (K-quarters), 2 rnnx (generation 2); 0 = not covered (-30/-31/-33)
int ds2_rnnx_fwd_family(int H, int cell, int mt, int knobs) {
  if (wide_ok(H, cell)) return 6;
  if (H % UPW != 0 || mt != 1 || ds2_rnnx_kb(H, cell == CELL_GRU ? 3 : 1, 1) < 0) return 0;
  if (gen4_ok(H, cell, mt, knobs)) return (cell == CELL_GRU && H / 32 <= 32) ? 5 : 4;
  return 2;
}

// BPTT family of ds2_rnnx_bwd_rs: 6 rnnw_bwd, 3 rnnrs (reduce-scatter), 0 = not covered
int ds2_rnnx_bwd_family(int H, int cell, int mt, int R) {
  if (wide_ok(H, cell)) return (R >= 1 && R <= 8 && mt == 1 && xcd_p(H, cell) <= 4 * MW) ? 6 : 0;
  if (H % UPW != 0 || R < 1 || R > 16 || mt != 1 || H / UPW > 6 * MW) return 0;
  return (H / 16 + MW - 1) / MW <= 12 ? 3 : 0;          // rnnrs_bwd_kernel's unit tiles (-36 past)
}

int ds2_rnnx_fwd_fuses_sum(int H, int cell, int mt, int ndir, int knobs) {
  return ndir == 2 && mt == 1 && (wide_ok(H, cell) || gen4_ok(H, cell, mt, knobs)) ? 1 : 0;
}

// grid size of a launch (blocks with no role exit at once)
int ds2_rnnx_grid(int H, int cell, int ngroups, int xcd_map) {
  const int P = xcd_p(H, cell);
  return (xcd_map && ngroups <= 8) ? 8 * P : ngroups * P;
}

// k-steps register tile of the generation-2 forward: whole K per wave
int ds2_rnnx_kb(int H, int G, int fwd) {
  (void)G;
  if (!fwd) return -1;                                    // the gather BPTT was removed
  const int need = (H / 32 + MW - 1) / MW;
  return need <= 6 ? need : -1;
}

// dynamic LDS: none (the exchanged state goes straight into MFMA registers)
size_t ds2_rnnx_smem(int H, int G, int mt, int fwd) {
  (void)H; (void)G; (void)mt; (void)fwd;
  return 0;
}

static int rnnw_fwd(const DS2RnnX* d, hipStream_t st) {
  if (d->R < 1 || d->R > 8 || d->mt != 1 || d->NP != d->BG * d->R) return -30;
  XFwd a;
  a.T = d->T; a.N = d->N; a.NP = d->NP; a.H = d->H; a.P = xcd_p(d->H, d->cell); a.BG = d->BG; a.R = d->R;
  a.steps = d->steps; a.gstride = d->gstride; a.ngroups = d->ndir * d->BG;
  a.xcd_map = d->xcd_map && a.ngroups <= 8; a.knobs = d->knobs;
  a.lens = d->lens; a.gx = (const bf16_t*)d->gx;
  for (int i = 0; i < 2; ++i) {
    a.U[i] = (const bf16_t*)d->U[i]; a.bh[i] = d->bh[i]; a.y[i] = (bf16_t*)d->y[i];
    a.hx[i] = (bf16_t*)d->ex[i]; a.hsave[i] = d->hsave[i]; a.gates[i] = d->gates[i];
  }
  a.ysum = (bf16_t*)d->ysum;
  a.census = d->census; a.err = d->err; a.timeout = d->timeout; a.stamps = d->stamps;
  if (d->ysum != nullptr && d->ndir != 2) return -37;
  if (d->steps <= 0) return 0;
  const int grid = ds2_rnnx_grid(d->H, d->cell, a.ngroups, a.xcd_map);
  const int kb8 = (d->H / 32 + 7) / 8;                 // k-steps per K-eighth: 5..7 for 1024 < H <= 1792
  switch (kb8) {
#define DS2_W(K)                                                                                      \
  case K:                                                                                             \
    if (a.stamps) hipLaunchKernelGGL((rnnw_fwd_kernel<K, wide_kl(K), true>), dim3(grid), dim3(QTH), 0, st, a); \
    else hipLaunchKernelGGL((rnnw_fwd_kernel<K, wide_kl(K), false>), dim3(grid), dim3(QTH), 0, st, a); \
    break;
    DS2_W(5) DS2_W(6) DS2_W(7)
#undef DS2_W
    default: return -31;
  }
  return (int)hipGetLastError();
}

int ds2_rnnx_fwd(const DS2RnnX* d, hipStream_t st) {
  if (wide_ok(d->H, d->cell)) return rnnw_fwd(d, st);
  if (d->H % UPW != 0 || d->R < 1 || d->R > 16 * d->mt || d->NP != d->BG * d->R) return -30;
  const int G = d->cell == CELL_GRU ? 3 : 1;
  const int kb = ds2_rnnx_kb(d->H, G, 1);
  if (kb < 0) return -31;
  XFwd a;
  a.T = d->T; a.N = d->N; a.NP = d->NP; a.H = d->H; a.P = d->H / UPW; a.BG = d->BG; a.R = d->R;
  a.steps = d->steps; a.gstride = d->gstride; a.ngroups = d->ndir * d->BG;
  a.xcd_map = d->xcd_map && a.ngroups <= 8; a.knobs = d->knobs;
  a.lens = d->lens; a.gx = (const bf16_t*)d->gx;
  for (int i = 0; i < 2; ++i) {
    a.U[i] = (const bf16_t*)d->U[i]; a.bh[i] = d->bh[i]; a.y[i] = (bf16_t*)d->y[i];
    a.hx[i] = (bf16_t*)d->ex[i]; a.hsave[i] = d->hsave[i]; a.gates[i] = d->gates[i];
  }
  a.ysum = (bf16_t*)d->ysum;
  a.census = d->census; a.err = d->err; a.timeout = d->timeout; a.stamps = d->stamps;
  if (d->steps <= 0) return 0;
  const int grid = ds2_rnnx_grid(d->H, d->cell, a.ngroups, a.xcd_map);
  // generation 4 (K-quarter split, register epilogue) unless knob 256 asks for generation 2
  const int kbq = (d->H / 32 + 3) / 4;
  // (GRU at kbq = 8 spills under the 3-waves-per-SIMD register budget: kbq 8..10 keep
  // kbq - 7 k-steps of U in LDS)
  const int fam = ds2_rnnx_fwd_family(d->H, d->cell, d->mt, d->knobs);
  const bool gen4 = fam == 4 || fam == 5;
  if (d->ysum != nullptr && (!gen4 || d->ndir != 2)) return -37;   // only gen 4 / 5 fuse the sum
  // generation 5 (K-eighths, each granule polled once) for GRU layers with H <= 1024
  // (H = 1280 measured slower on generation 5: 7.4 vs 5.75 us/step, its 40-workgroup groups
  // span XCDs and the U slice needs LDS k-steps and a single partial buffer)
  if (fam == 5) {
    switch ((d->H / 32 + 7) / 8) {
#define DS2_E(K, L, B)                                                                                    \
  case K:                                                                                                 \
    if (a.stamps) hipLaunchKernelGGL((rnne_fwd_kernel<K, L, B, true>), dim3(grid), dim3(QTH), 0, st, a); \
    else hipLaunchKernelGGL((rnne_fwd_kernel<K, L, B, false>), dim3(grid), dim3(QTH), 0, st, a);      \
    break;
      DS2_E(1, 0, false) DS2_E(2, 0, false) DS2_E(3, 0, false) DS2_E(4, 0, false)
#undef DS2_E
      default: return -31;
    }
    return (int)hipGetLastError();
  }
  if (gen4) {
#define DS2_QL(C, K)                                                                                  \
  if (a.stamps) hipLaunchKernelGGL((rnnq_fwd_kernel<C, K, true>), dim3(grid), dim3(QTH), 0, st, a);    \
  else hipLaunchKernelGGL((rnnq_fwd_kernel<C, K, false>), dim3(grid), dim3(QTH), 0, st, a);
#define DS2_QK(C, K) \
  case K: DS2_QL(C, K) break;
#define DS2_Q(C)                                                                                      \
  switch (kbq) {                                                                                      \
    DS2_QK(C, 1) DS2_QK(C, 2) DS2_QK(C, 3) DS2_QK(C, 4) DS2_QK(C, 5) DS2_QK(C, 6) DS2_QK(C, 7)        \
    default: DS2_QL(C, 8) break;                                                                      \
  }
#define DS2_QW(K, L)                                                                                  \
  case K:                                                                                             \
    if (a.stamps) hipLaunchKernelGGL((rnnq_fwd_kernel<CELL_GRU, K, true, L>), dim3(grid), dim3(QTH), 0, st, a); \
    else hipLaunchKernelGGL((rnnq_fwd_kernel<CELL_GRU, K, false, L>), dim3(grid), dim3(QTH), 0, st, a); \
    break;
    if (d->cell == CELL_GRU && kbq > 7) {
      switch (kbq) { DS2_QW(8, 1) DS2_QW(9, 2) default: DS2_QW(10, 3) }
    } else if (d->cell == CELL_GRU) { DS2_Q(CELL_GRU) } else { DS2_Q(CELL_RELU) }
#undef DS2_QW
#undef DS2_QL
#undef DS2_QK
#undef DS2_Q
    return (int)hipGetLastError();
  }
  const size_t smem = ds2_rnnx_smem(d->H, G, d->mt, 1);
  int rc;
#define DS2_FWD(C, M)                                                                        \
  {                                                                                          \
    switch (kb) {                                                                            \
      case 1: rc = set_smem_attr(rnnx_fwd_kernel<C, M, 1>, smem); break;                     \
      case 2: rc = set_smem_attr(rnnx_fwd_kernel<C, M, 2>, smem); break;                     \
      case 3: rc = set_smem_attr(rnnx_fwd_kernel<C, M, 3>, smem); break;                     \
      case 4: rc = set_smem_attr(rnnx_fwd_kernel<C, M, 4>, smem); break;                     \
      case 5: rc = set_smem_attr(rnnx_fwd_kernel<C, M, 5>, smem); break;                     \
      default: rc = set_smem_attr(rnnx_fwd_kernel<C, M, 6>, smem); break;                    \
    }                                                                                        \
    if (rc) return rc;                                                                       \
    return launch_fwd<C, M>(a, kb, grid, smem, st);                                          \
  }
  if (d->mt != 1) return -33;     // 16-row tiles only: the 32-row LDS footprint exceeds 160 KB
  if (d->cell == CELL_GRU) DS2_FWD(CELL_GRU, 1) else DS2_FWD(CELL_RELU, 1)
#undef DS2_FWD
}

// floats of the reduce-scatter ring of ONE direction: [3 slots][BG][P][R][H]
long long ds2_rnnx_ring_floats(int H, int BG, int R) { return 3LL * BG * (H / UPW) * R * H; }

static int rnnw_bwd(const DS2RnnX* d, hipStream_t st) {
  if (d->R < 1 || d->R > 8 || d->mt != 1 || d->NP != d->BG * d->R) return -30;
  if (d->ring[0] == nullptr || (d->ndir == 2 && d->ring[1] == nullptr)) return -34;
  const int P = xcd_p(d->H, d->cell);
  if (P > 4 * MW) return -35;                         // GPT = 4 producers per gather thread
  XBwdRS a;
  a.T = d->T; a.N = d->N; a.NP = d->NP; a.H = d->H; a.P = P; a.BG = d->BG; a.R = d->R;
  a.steps = d->steps; a.gstride = d->gstride; a.ngroups = d->ndir * d->BG;
  a.xcd_map = d->xcd_map && a.ngroups <= 8; a.knobs = d->knobs;
  a.lens = d->lens; a.dy = (const bf16_t*)d->gx;
  for (int i = 0; i < 2; ++i) {
    a.U[i] = (const bf16_t*)d->U[i]; a.hsave[i] = d->hsave[i]; a.gates[i] = d->gates[i];
    a.dgh[i] = (bf16_t*)d->ex[i]; a.ring[i] = (float*)d->ring[i];
    a.dbx_part[i] = d->dbx_part[i]; a.dbh_part[i] = d->dbh_part[i];
  }
  a.dgx = (bf16_t*)d->dgx; a.dgx_scale = d->dgx_scale;
  a.census = d->census; a.err = d->err; a.timeout = d->timeout; a.stamps = d->stamps;
  if (d->steps <= 0) return 0;
  const int grid = ds2_rnnx_grid(d->H, d->cell, a.ngroups, a.xcd_map);
  const int npw = (d->H / 32 + MW - 1) / MW;          // unit pairs per publishing wave
  if (a.stamps != nullptr && npw == 8) {
    ds2_launch((rnnw_bwd_kernel<16, 4, true>), dim3(grid), dim3(NTH), 0u, st, a);
    return (int)hipGetLastError();
  }
  switch (2 * npw) {
    case 10: ds2_launch((rnnw_bwd_kernel<10, 4>), dim3(grid), dim3(NTH), 0u, st, a); break;
    case 12: ds2_launch((rnnw_bwd_kernel<12, 4>), dim3(grid), dim3(NTH), 0u, st, a); break;
    case 14: ds2_launch((rnnw_bwd_kernel<14, 4>), dim3(grid), dim3(NTH), 0u, st, a); break;
    case 16: ds2_launch((rnnw_bwd_kernel<16, 4>), dim3(grid), dim3(NTH), 0u, st, a); break;
    default: return -36;
  }
  return (int)hipGetLastError();
}

int ds2_rnnx_bwd_rs(const DS2RnnX* d, hipStream_t st) {
  if (wide_ok(d->H, d->cell)) return rnnw_bwd(d, st);
  if (d->H % UPW != 0 || d->R < 1 || d->R > 16 || d->NP != d->BG * d->R || d->mt != 1) return -30;
  if (d->ring[0] == nullptr || (d->ndir == 2 && d->ring[1] == nullptr)) return -34;
  const int P = d->H / UPW;
  if (P > 6 * MW) return -35;                       // at most GPT = 6 producers per gather thread
  const int mtu_need = (d->H / 16 + MW - 1) / MW;
  XBwdRS a;
  a.T = d->T; a.N = d->N; a.NP = d->NP; a.H = d->H; a.P = P; a.BG = d->BG; a.R = d->R;
  a.steps = d->steps; a.gstride = d->gstride; a.ngroups = d->ndir * d->BG;
  a.xcd_map = d->xcd_map && a.ngroups <= 8; a.knobs = d->knobs;
  a.lens = d->lens; a.dy = (const bf16_t*)d->gx;
  for (int i = 0; i < 2; ++i) {
    a.U[i] = (const bf16_t*)d->U[i]; a.hsave[i] = d->hsave[i]; a.gates[i] = d->gates[i];
    a.dgh[i] = (bf16_t*)d->ex[i]; a.ring[i] = (float*)d->ring[i];
    a.dbx_part[i] = d->dbx_part[i]; a.dbh_part[i] = d->dbh_part[i];
  }
  a.dgx = (bf16_t*)d->dgx; a.dgx_scale = d->dgx_scale;
  a.census = d->census; a.err = d->err; a.timeout = d->timeout; a.stamps = d->stamps;
  if (d->steps <= 0) return 0;
  const int grid = ds2_rnnx_grid(d->H, d->cell, a.ngroups, a.xcd_map);
  // bf16 partials (knob 64: fp32): PBF 1 for R <= 8 (two producers per load), 2 for R <= 16
  const int pbf = ((d->H / 16) % 2 != 0 || (d->knobs & 64)) ? 0 : (d->R <= 8 ? 1 : 2);
#define DS2_RS(C, M, GP)                                                                    \
  do {                                                                                      \
    if (pbf == 1) ds2_launch((rnnrs_bwd_kernel<C, M, GP, 1>), dim3(grid), dim3(NTH), 0u, st, a); \
    else if (pbf == 2) ds2_launch((rnnrs_bwd_kernel<C, M, GP, 2>), dim3(grid), dim3(NTH), 0u, st, a); \
    else ds2_launch((rnnrs_bwd_kernel<C, M, GP, 0>), dim3(grid), dim3(NTH), 0u, st, a);     \
  } while (0)
#define DS2_RS_CELL(C)                                  \
  if (mtu_need <= 2) DS2_RS(C, 2, 4);                   \
  else if (mtu_need <= 4) DS2_RS(C, 4, 4);              \
  else if (mtu_need <= 6) DS2_RS(C, 6, 4);              \
  else if (mtu_need <= 8) DS2_RS(C, 8, 4);              \
  else if (mtu_need <= 10 && P <= 4 * MW) DS2_RS(C, 10, 4); \
  else if (mtu_need <= 12) DS2_RS(C, 12, 6);            \
  else return -36;
  if (d->cell == CELL_GRU) { DS2_RS_CELL(CELL_GRU) } else { DS2_RS_CELL(CELL_RELU) }
#undef DS2_RS_CELL
#undef DS2_RS
  return (int)hipGetLastError();
}

}  // extern "C"
