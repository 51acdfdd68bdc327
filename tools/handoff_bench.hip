// Inter-workgroup hand-off latency on MI355X: ping-pong between two workgroups.
//   hipcc --offload-arch=gfx950 -O3 tools/handoff_bench.hip -o build/handoff_bench && build/handoff_bench
// Modes (producer store flavour / consumer load flavour):
//   0: sc1 (write-through) store, sc1 load       — placement-independent (our global mode)
//   1: plain store, sc1 load                      — valid only when both WGs share an XCD (L2)
// Pairs: blocks (0, 8) share an XCD under round-robin dispatch; (0, 1) do not. Every WG
// reports its XCC id (s_getreg HW_REG_XCC_ID) so the placement is checked, not assumed.
// Each spin is bounded; a timed-out run reports -1.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

template <int MODE>
__global__ void pingpong(unsigned* buf, int a, int b, int iters, long long* out, unsigned* xcc) {
  const int me = blockIdx.x;
  if (threadIdx.x == 0) xcc[me] = xcc_id();
  if (me != a && me != b) return;
  if (threadIdx.x != 0) return;
  unsigned* mine = buf + (me == a ? 0 : 64);     // separate 256-B lines
  unsigned* peer = buf + (me == a ? 64 : 0);
  const bool starter = me == a;
  long long t0 = __builtin_amdgcn_s_memrealtime();
  const long long limit = 200000000;   // 2 s
  for (int i = 1; i <= iters; ++i) {
    if (!starter || i > 1) {
      const unsigned want = starter ? (unsigned)(i - 1) : (unsigned)i;
      long long ts = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(peer, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
        if (__builtin_amdgcn_s_memrealtime() - ts > limit) { out[me] = -1; return; }
      }
    }
    if (MODE == 0) {
      __hip_atomic_store(mine, (unsigned)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      *(volatile unsigned*)mine = (unsigned)i;
    }
    if (starter && i == 1) continue;
  }
  out[me] = __builtin_amdgcn_s_memrealtime() - t0;
}

int main() {
  unsigned* buf; long long* out; unsigned* xcc;
  hipMalloc(&buf, 4096); hipMalloc(&out, 64 * 8); hipMalloc(&xcc, 64 * 4);
  const int iters = 2000;
  struct P { int a, b; const char* name; };
  P pairs[] = {{0, 8, "blocks 0,8"}, {0, 1, "blocks 0,1"}, {3, 11, "blocks 3,11"}};
  for (int mode = 0; mode < 2; ++mode) {
    for (auto& p : pairs) {
      hipMemset(buf, 0, 4096);
      hipMemset(out, 0, 64 * 8);
      if (mode == 0) hipLaunchKernelGGL(pingpong<0>, dim3(16), dim3(64), 0, 0, buf, p.a, p.b, iters, out, xcc);
      else hipLaunchKernelGGL(pingpong<1>, dim3(16), dim3(64), 0, 0, buf, p.a, p.b, iters, out, xcc);
      hipDeviceSynchronize();
      long long o[64]; unsigned x[64];
      hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
      hipMemcpy(x, xcc, sizeof(x), hipMemcpyDeviceToHost);
      const double ticks = (double)o[p.a];
      // one iteration = one round trip = two hand-offs; s_memrealtime is 100 MHz
      printf("mode %d (%s) %s: xcc %u/%u  %s  one-way hand-off = %.3f us\n", mode,
             mode == 0 ? "sc1 store/sc1 load" : "plain store/sc1 load", p.name, x[p.a], x[p.b],
             (o[p.a] < 0 || o[p.b] < 0) ? "TIMEOUT" : "ok",
             (o[p.a] < 0) ? -1.0 : ticks * 10.0 / 1000.0 / (2.0 * iters));
    }
  }
  return 0;
}
