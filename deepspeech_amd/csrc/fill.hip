// One launch for the small per-launch buffer initialisations of the persistent recurrence
// kernels (exchange sentinels, census words, error word, initial state slot, bias-gradient
// partials): up to 8 (pointer, bytes, 32-bit pattern) regions filled by one grid instead of
// one torch fill kernel (~5 us of launch + tail each on the critical path) per region.
#include "common.h"

using namespace ds2;

namespace {

constexpr int MF_MAX = 8;

struct MultiFill {
  unsigned* ptr[MF_MAX];
  unsigned long long words[MF_MAX];   // region sizes in 32-bit words
  unsigned pattern[MF_MAX];
  int n;
};

__global__ __launch_bounds__(256) void multi_fill_kernel(MultiFill f) {
  const unsigned long long stride = (unsigned long long)gridDim.x * 256;
  for (int r = 0; r < f.n; ++r) {
    unsigned* p = f.ptr[r];
    const unsigned v = f.pattern[r];
    const unsigned long long nw = f.words[r];
    const unsigned long long n4 = ((reinterpret_cast<uintptr_t>(p) & 15) == 0) ? nw / 4 : 0;
    const i32x4 v4 = {(int)v, (int)v, (int)v, (int)v};
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride)
      reinterpret_cast<i32x4*>(p)[i] = v4;
    for (unsigned long long i = n4 * 4 + (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < nw; i += stride)
      p[i] = v;
  }
}

}  // namespace

extern "C" int ds2_multi_fill(int n, void* const* ptrs, const unsigned long long* bytes, const unsigned* patterns,
                              hipStream_t st) {
  if (n < 0 || n > MF_MAX) return -50;
  MultiFill f{};
  unsigned long long total = 0;
  for (int i = 0; i < n; ++i) {
    if (bytes[i] % 4 != 0 || (reinterpret_cast<uintptr_t>(ptrs[i]) & 3) != 0) return -51;
    f.ptr[i] = static_cast<unsigned*>(ptrs[i]);
    f.words[i] = bytes[i] / 4;
    f.pattern[i] = patterns[i];
    total += f.words[i];
  }
  f.n = n;
  if (total == 0) return 0;
  unsigned long long blocks = (total / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(multi_fill_kernel, dim3((unsigned)blocks), dim3(256), 0, st, f);
  return (int)hipGetLastError();
}
