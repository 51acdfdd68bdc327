// Operand K-layout of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3, unit scales), checked with exact
// small-integer data: lane l feeds row l % 16 and its 32 bytes are taken as k = PERM(g, byte)
// for g = l / 16 under several candidate layouts; the one whose host product matches D exactly
// is the hardware's. Also checks a zero upper half (k-step with 64 real K).
//   hipcc --offload-arch=gfx950 -O2 tools/probe_mfma_layout.hip -o tools/probe_mfma_layout.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

// candidate layouts: k of byte b (0..31) of lane group g (0..3)
__host__ __device__ int kmap(int layout, int g, int b) {
  switch (layout) {
    case 0: return b < 16 ? 16 * g + b : 64 + 16 * g + (b - 16);   // two 16-B chunks (rnn_fp8.hip)
    case 1: return 32 * g + b;                                      // one contiguous 32-B block
    case 2: return b < 8 ? 8 * g + b : b < 16 ? 32 + 8 * g + (b - 8) : b < 24 ? 64 + 8 * g + (b - 16) : 96 + 8 * g + (b - 24);
    default: return 0;
  }
}

__global__ void run(const unsigned char* A, const unsigned char* B, int layout, float* out) {
  const int lane = threadIdx.x, g = lane >> 4, r = lane & 15;
  unsigned char a[32], b[32];
  for (int i = 0; i < 32; ++i) {
    a[i] = A[r * 128 + kmap(layout, g, i)];
    b[i] = B[r * 128 + kmap(layout, g, i)];
  }
  i32x8 av, bv;
  for (int i = 0; i < 8; ++i) {
    av[i] = a[4 * i] | (a[4 * i + 1] << 8) | (a[4 * i + 2] << 16) | (a[4 * i + 3] << 24);
    bv[i] = b[4 * i] | (b[4 * i + 1] << 8) | (b[4 * i + 2] << 16) | (b[4 * i + 3] << 24);
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
  for (int j = 0; j < 4; ++j) out[(4 * g + j) * 16 + r] = acc[j];
}

// e4m3 encodings of small integers 0..4 and their values
static const unsigned char enc[5] = {0x00, 0x38, 0x40, 0x44, 0x48};

int main() {
  unsigned char hA[16 * 128], hB[16 * 128];
  float vA[16 * 128], vB[16 * 128];
  srand(3);
  for (int i = 0; i < 16 * 128; ++i) {
    int x = rand() % 5, y = rand() % 5;
    hA[i] = enc[x]; vA[i] = (float)x;
    hB[i] = enc[y]; vB[i] = (float)y;
  }
  unsigned char *dA, *dB;
  float* dD;
  hipMalloc(&dA, sizeof(hA)); hipMalloc(&dB, sizeof(hB)); hipMalloc(&dD, 256 * sizeof(float));
  hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
  float ref[256];
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      float s = 0.f;
      for (int k = 0; k < 128; ++k) s += vA[i * 128 + k] * vB[j * 128 + k];
      ref[i * 16 + j] = s;
    }
  for (int layout = 0; layout < 3; ++layout) {
    float d[256];
    hipLaunchKernelGGL(run, dim3(1), dim3(64), 0, 0, dA, dB, layout, dD);
    hipMemcpy(d, dD, sizeof(d), hipMemcpyDeviceToHost);
    int bad = 0;
    double maxerr = 0;
    for (int i = 0; i < 256; ++i) {
      if (d[i] != ref[i]) ++bad;
      maxerr = fmax(maxerr, fabs(d[i] - ref[i]));
    }
    printf("layout %d: %d of 256 outputs differ (max abs err %g); D[0][0] = %g ref %g\n", layout, bad, maxerr, d[0],
           ref[0]);
  }
  // the same product with the upper 64 K of A and B zero (real K = 64 in the lower bytes of
  // layout 0's chunks): does a half-empty operand work?
  for (int i = 0; i < 16; ++i)
    for (int k = 64; k < 128; ++k) { hA[i * 128 + k] = 0; hB[i * 128 + k] = 0; vA[i * 128 + k] = 0; vB[i * 128 + k] = 0; }
  hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      float s = 0.f;
      for (int k = 0; k < 128; ++k) s += vA[i * 128 + k] * vB[j * 128 + k];
      ref[i * 16 + j] = s;
    }
  for (int layout = 0; layout < 3; ++layout) {
    float d[256];
    hipLaunchKernelGGL(run, dim3(1), dim3(64), 0, 0, dA, dB, layout, dD);
    hipMemcpy(d, dD, sizeof(d), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += d[i] != ref[i];
    printf("upper K zero, layout %d: %d of 256 differ\n", layout, bad);
  }
  return 0;
}
