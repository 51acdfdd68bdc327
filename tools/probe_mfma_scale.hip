// Which lane's E8M0 scale byte scales which (row, K block) of v_mfma_scale_f32_16x16x128_f8f6f4?
// A and B are all e4m3 1.0 (0x38); every scale byte is 127 (2^0) except lane L of the probed
// operand, which gets 128 (2^1). D[i][j] = sum_k A[i][k] B[j][k] * 2^(eA + eB) = 128 + 32 per
// K block of 32 that lane L scales. Prints, per probed lane, the output elements that moved.
//   hipcc --offload-arch=gfx950 -O2 tools/probe_mfma_scale.hip -o /tmp/probe && /tmp/probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__global__ void probe(int which, int L, float* out) {
  const int lane = threadIdx.x;
  const int one4 = 0x38383838;
  const i32x8 a = {one4, one4, one4, one4, one4, one4, one4, one4};
  const int base = 0x7f7f7f7f, hot = 0x80808080;
  const int sa = (which == 0 && lane == L) ? hot : base;
  const int sb = (which == 1 && lane == L) ? hot : base;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, a, acc, 0, 0, 0, sa, 0, sb);
  // C/D layout: lane holds D[4 (lane >> 4) + j][lane & 15]
  for (int j = 0; j < 4; ++j) out[(4 * (lane >> 4) + j) * 16 + (lane & 15)] = acc[j];
}

int main() {
  float* d;
  hipMalloc(&d, 256 * sizeof(float));
  float h[256];
  for (int which = 0; which < 2; ++which) {
    printf("operand %s (first = rows i of D, second = columns j)\n", which == 0 ? "A" : "B");
    for (int L = 0; L < 64; ++L) {
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, which, L, d);
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      printf("  lane %2d:", L);
      int n = 0;
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j)
          if (h[i * 16 + j] != 128.f) {
            if (n < 20) printf(" D[%d][%d]=%g", i, j, h[i * 16 + j]);
            ++n;
          }
      printf("  (%d moved)\n", n);
    }
  }
  hipFree(d);
  return 0;
}
