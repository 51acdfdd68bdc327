// Per-step all-gather floor of the persistent recurrence (no math): G groups of P
// workgroups; every step each workgroup waits for the P flags of its group, reads the
// whole group's previous-step slab (P x CB bytes) and publishes its own CB-byte chunk.
//   hipcc --offload-arch=gfx950 -O3 tools/exchange_bench.hip -o build/exchange_bench
//   build/exchange_bench
// Placement: "spread" = group = blockIdx / P (groups straddle XCDs; the current kernel);
//            "local"  = group = blockIdx % 8 (under round-robin dispatch a group's blocks
//                        share one XCD; the XCC id of every block is checked, not assumed).
// Stores:    sc1 = write-through (placement-independent); plain = stays in the XCD's L2
//            (valid only for XCD-local groups; every word read back is verified).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

struct Args {
  int G, P, CB, steps, local, plain, tag;
  unsigned* slab;     // [2][G][P*CB/4]
  unsigned* flags;    // [G][P]
  unsigned* xcc;      // [grid]
  long long* t;       // [grid][2]
  unsigned* err;      // [1]
};

template <int NT>
__global__ __launch_bounds__(NT) void xbench(Args a) {
  __shared__ int abort_flag;
  __shared__ unsigned sink;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = a.local ? (blockIdx.x % a.G) : (blockIdx.x / a.P);
  const int slot = a.local ? (blockIdx.x / a.G) : (blockIdx.x % a.P);
  if (tid == 0) { a.xcc[blockIdx.x] = xcc_id(); abort_flag = 0; sink = 0; }
  const int words = a.P * a.CB / 4;                  // group slab (dwords)
  const int cw = a.CB / 4;                           // own chunk (dwords)
  unsigned* f = a.flags + grp * a.P;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned acc = 0, bad = 0;
  for (int s = 1; s <= a.steps; ++s) {
    if (s > 1 && a.tag) {
      // sentinel protocol: poll the payload itself (fresh per-step slot pre-filled 0xFFFFFFFF)
      const unsigned* src = a.slab + ((size_t)(s - 1) * a.G + grp) * words;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(src), (short)0,
                                                                          words * 4, 0x00020000);
      const long long ts = __builtin_amdgcn_s_memrealtime();
      for (int q = tid * 4; q < words; q += NT * 4) {
        u32x4 v;
        while (true) {
          v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, q * 4, 0, 16));
          if (v.x != 0xffffffffu && v.y != 0xffffffffu && v.z != 0xffffffffu && v.w != 0xffffffffu) break;
          if (__builtin_amdgcn_s_memrealtime() - ts > 100000000) { abort_flag = 1; break; }
          __builtin_amdgcn_s_sleep(1);
        }
        const unsigned want = (unsigned)((s - 1) * 1024 + (q / cw));
        bad += (v.x != want) + (v.w != want);
        acc += v.y;
      }
      __syncthreads();
      if (abort_flag) break;
    } else if (s > 1) {
      if (wave == 0) {
        const long long ts = __builtin_amdgcn_s_memrealtime();
        while (true) {
          bool ok = true;
          for (int q = lane; q < a.P; q += 64)
            ok = ok && (__hip_atomic_load(f + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)(s - 1));
          if (__all(ok)) break;
          if (__builtin_amdgcn_s_memrealtime() - ts > 100000000) { if (lane == 0) abort_flag = 1; break; }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
      if (abort_flag) break;
      // read the group's step s-1 slab
      const unsigned* src = a.slab + ((size_t)((s - 1) & 1) * a.G + grp) * words;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(src), (short)0,
                                                                          words * 4, 0x00020000);
      for (int q = tid * 4; q < words; q += NT * 4) {
        const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, q * 4, 0, 16));
        const unsigned want = (unsigned)((s - 1) * 1024 + (q / cw));
        bad += (v.x != want) + (v.w != want);
        acc += v.y;
      }
    }
    __syncthreads();   // stands in for the reduce / epilogue barriers
    // publish own chunk for step s
    unsigned* dst = a.slab + ((size_t)(a.tag ? s : (s & 1)) * a.G + grp) * words + slot * cw;
    const unsigned val = (unsigned)(s * 1024 + slot);
    if (tid * 4 < cw) {
      const u32x4 v = {val, val, val, val};
      if (a.plain) *reinterpret_cast<u32x4*>(dst + tid * 4) = v;
      else {
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, cw * 4, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v, rd, tid * 16, 0, 16);
      }
      if (!a.tag) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (!a.tag) {
      __syncthreads();
      if (tid == 0) __hip_atomic_store(f + slot, (unsigned)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) { a.t[blockIdx.x * 2] = t0; a.t[blockIdx.x * 2 + 1] = t1; }
  if (bad) atomicAdd(a.err, bad);
  if (acc == 0xdeadbeef) sink = acc;
}

int main() {
  struct Cfg { int G, P, CB, local, plain, nt, tag; const char* what; };
  std::vector<Cfg> cfgs = {
      {4, 50, 512, 0, 0, 512, 0, "current: 4 groups x 50 WG, 16 rows x 16 units, spread, sc1"},
      {4, 50, 512, 0, 0, 512, 1, "  same, sentinel (no flags)"},
      {4, 25, 1024, 1, 1, 512, 0, "4 groups x 25 WG, 16 rows x 32 units, XCD-local, plain"},
      {4, 25, 1024, 1, 1, 512, 1, "  same, sentinel"},
      {4, 25, 1024, 1, 0, 512, 1, "  same, sentinel, sc1 stores"},
      {8, 25, 512, 0, 0, 512, 0, "8 groups x 25 WG, 8 rows x 32 units, spread, sc1"},
      {8, 25, 512, 0, 0, 512, 1, "  same, sentinel"},
      {8, 25, 512, 1, 1, 512, 0, "8 groups x 25 WG, 8 rows x 32 units, XCD-local, plain"},
      {8, 25, 512, 1, 1, 512, 1, "  same, sentinel"},
      {8, 25, 512, 1, 0, 512, 1, "  same, sentinel, sc1 stores"},
      {8, 25, 512, 1, 1, 256, 1, "  same, sentinel, plain, 256 threads"},
      {8, 25, 1536, 1, 1, 512, 1, "bwd-sized: 8 groups x 25 WG, 8 rows x 96 cols, XCD-local, sentinel, plain"},
      {8, 25, 1536, 1, 0, 512, 1, "  same, sc1 stores"},
      {8, 25, 1536, 1, 1, 448, 1, "  plain, 448 gather threads"},
  };
  const int steps = 1000;
  unsigned *slab, *flags, *xcc, *err;
  long long* t;
  const size_t slab_bytes = (size_t)(steps + 2) * 8 * 25 * 1536;   // per-step slots for sentinel mode
  hipMalloc(&slab, slab_bytes);
  hipMalloc(&flags, 8 * 64 * 4);
  hipMalloc(&xcc, 1024 * 4);
  hipMalloc(&t, 1024 * 16);
  hipMalloc(&err, 4);
  for (auto& c : cfgs) {
    const int grid = c.G * c.P;
    if (c.local && c.G != 8 && c.G != 4) continue;
    Args a{c.G, c.P, c.CB, steps, c.local, c.plain, c.tag, slab, flags, xcc, t, err};
    if (c.local && c.G == 4) {
      // local with 4 groups: groups are blockIdx % 8 in {0..3}; launch 8*P blocks, the
      // other 4 "XCD groups" run the same exchange on their own (harmless, symmetric)
      a.G = 8;
    }
    const int g2 = a.G * c.P;
    double best = 1e30;
    unsigned e = 0;
    std::vector<unsigned> xs(g2);
    bool placement_ok = true;
    for (int rep = 0; rep < 3; ++rep) {
      hipMemset(slab, c.tag ? 0xff : 0, slab_bytes);
      hipMemset(flags, 0, 8 * 64 * 4);
      hipMemset(err, 0, 4);
      if (c.nt == 512) hipLaunchKernelGGL(xbench<512>, dim3(g2), dim3(512), 0, 0, a);
      else if (c.nt == 448) hipLaunchKernelGGL(xbench<448>, dim3(g2), dim3(448), 0, 0, a);
      else hipLaunchKernelGGL(xbench<256>, dim3(g2), dim3(256), 0, 0, a);
      if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
      std::vector<long long> tt(2 * g2);
      hipMemcpy(tt.data(), t, 16 * g2, hipMemcpyDeviceToHost);
      hipMemcpy(xs.data(), xcc, 4 * g2, hipMemcpyDeviceToHost);
      unsigned ee;
      hipMemcpy(&ee, err, 4, hipMemcpyDeviceToHost);
      e += ee;
      long long lo = tt[0], hi = tt[1];
      for (int i = 0; i < g2; ++i) { lo = std::min(lo, tt[2 * i]); hi = std::max(hi, tt[2 * i + 1]); }
      best = std::min(best, (double)(hi - lo) * 10.0 / steps);   // 100 MHz ticks -> ns per step
    }
    if (c.local)
      for (int i = 0; i < g2; ++i)
        if (xs[i] != xs[i % a.G]) placement_ok = false;
    printf("%-70s grid %4d  %7.1f ns/step  errors %u  placement %s\n", c.what, g2, best, e,
           c.local ? (placement_ok ? "XCD-local verified" : "NOT local") : "n/a");
    (void)grid;
  }
  return 0;
}
