// CU-mask probe for MI355X (gfx950): which physical CU (XCC, SE, SH, CU) each bit of a
// hipExtStreamCreateWithCUMask mask selects, and whether a persistent-style grid (one
// 125 KB-LDS workgroup per CU, all required co-resident) fits under a given mask.
//   hipcc --offload-arch=gfx950 -O2 tools/cu_mask_probe.hip -o tools/cu_mask_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <tuple>
#include <vector>

__global__ void probe(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned x, h;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(h));
    long t0 = clock64();
    while (clock64() - t0 < 20000) {
    }
    out[2 * blockIdx.x] = x;
    out[2 * blockIdx.x + 1] = h;
  }
}

// every workgroup arrives, then waits (bounded) for all peers: co-residency test
__global__ void __launch_bounds__(512) coresident(unsigned* count, unsigned* ok, int n) {
  extern __shared__ unsigned char lds[];
  if (threadIdx.x == 0) {
    lds[0] = 1;
    __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long t0 = wall_clock64();
    unsigned c = 0;
    while ((c = __hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < (unsigned)n &&
           wall_clock64() - t0 < 20000000) {  // 0.2 s at 100 MHz
      __builtin_amdgcn_s_sleep(8);
    }
    if (c >= (unsigned)n) __hip_atomic_fetch_add(ok, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

static void ck(hipError_t e, const char* w) {
  if (e != hipSuccess) {
    printf("%s failed %d\n", w, (int)e);
    exit(1);
  }
}

int main(int argc, char** argv) {
  const bool map_bits = argc < 2;  // any argument: skip the (slow) per-bit map
  int ncu = 0;
  ck(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0), "attr");
  printf("CUs %d\n", ncu);
  const int NB = 2048, W = (ncu + 31) / 32;
  unsigned* d;
  ck(hipMalloc(&d, NB * 8), "malloc");
  std::vector<unsigned> h(NB * 2);
  auto mk = [&](std::vector<uint32_t>& m) {
    hipStream_t s;
    ck(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size() * 32, m.data()), "create");
    return s;
  };
  // 1. bit -> physical CU
  printf("bit: xcc se sh cu (HW_ID>>8)\n");
  for (int b = 0; map_bits && b < ncu; ++b) {
    std::vector<uint32_t> m(W, 0);
    m[b / 32] |= 1u << (b % 32);
    hipStream_t s = mk(m);
    hipLaunchKernelGGL(probe, dim3(NB), dim3(64), 0, s, d);
    ck(hipStreamSynchronize(s), "sync");
    ck(hipMemcpy(h.data(), d, NB * 8, hipMemcpyDeviceToHost), "memcpy");
    std::set<std::tuple<unsigned, unsigned, unsigned, unsigned, unsigned>> t;
    for (int i = 0; i < NB; ++i)
      if ((h[2 * i] & 15) == (unsigned)(b % 8)) {
        unsigned v = h[2 * i + 1];
        t.insert({h[2 * i] & 15, (v >> 13) & 7, (v >> 12) & 1, (v >> 8) & 15, v >> 8});
      }
    printf("%d:", b);
    for (auto& e : t)
      printf("  %u %u %u %u (%x)", std::get<0>(e), std::get<1>(e), std::get<2>(e), std::get<3>(e), std::get<4>(e));
    printf("\n");
    ck(hipStreamDestroy(s), "destroy");
  }
  // 2. co-residency of n persistent workgroups (125 KB LDS each) under "first k CUs per XCD"
  unsigned *cnt, *ok;
  ck(hipMalloc(&cnt, 4), "m");
  ck(hipMalloc(&ok, 4), "m");
  ck(hipFuncSetAttribute((const void*)coresident, hipFuncAttributeMaxDynamicSharedMemorySize, 128000), "attr");
  for (int k : {32, 28, 26, 25, 24}) {
    std::vector<uint32_t> m(W, 0);
    for (int i = 0; i < 8 * k; ++i) m[i / 32] |= 1u << (i % 32);
    hipStream_t s = mk(m);
    for (int n : {8 * k, 200}) {
      if (n > 8 * k) continue;
      ck(hipMemset(cnt, 0, 4), "ms");
      ck(hipMemset(ok, 0, 4), "ms");
      hipLaunchKernelGGL(coresident, dim3(n), dim3(512), 128000, s, cnt, ok, n);
      ck(hipStreamSynchronize(s), "sync");
      unsigned a = 0, b = 0;
      ck(hipMemcpy(&a, cnt, 4, hipMemcpyDeviceToHost), "c");
      ck(hipMemcpy(&b, ok, 4, hipMemcpyDeviceToHost), "c");
      printf("mask first %d CUs/XCD, %d WGs: all co-resident in %u of %u\n", k, n, b, a);
    }
    ck(hipStreamDestroy(s), "destroy");
  }
  return 0;
}
