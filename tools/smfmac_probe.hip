// Probe the operand layout of v_smfmac_f32_16x16x64_f16 on gfx950 (diagnostic tool, run on the GPU
// box: hipcc -O2 --offload-arch=gfx950 tools/smfmac_probe.hip -o /tmp/probe && /tmp/probe).
// A (sparse 16x64, compressed to 8 halves per lane) holds unique ids lane*8+j+1; B selects one K column
// per output column: B_m[k][c] = (k == 16m + c).  D_m[row][c] is then the id placed at dense K = 16m+c of
// that row (0 if none).  Printed for two index patterns.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(float* out, int idxpat) {
  const int l = threadIdx.x;
  f16x8 a;
  for (int j = 0; j < 8; ++j) a[j] = (_Float16)(float)(l * 8 + j + 1);
  for (int m = 0; m < 4; ++m) {
    f16x16 b;
    for (int j = 0; j < 16; ++j) {
      // hypothesis for B: lane l holds B[k = 16*(l>>4) + j][col = l & 15]
      const int k = 16 * (l >> 4) + j, c = l & 15;
      b[j] = (_Float16)((k == 16 * m + c) ? 1.f : 0.f);
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_smfmac_f32_16x16x64_f16(a, b, acc, idxpat, 0, 0);
    for (int q = 0; q < 4; ++q) out[(m * 64 + l) * 4 + q] = acc[q];
  }
}

int main() {
  float* d;
  hipMalloc(&d, 4 * 64 * 4 * sizeof(float));
  float h[4 * 64 * 4];
  const int pats[2] = {0x8888, 0xDDDD};
  for (int p = 0; p < 2; ++p) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, pats[p]);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("pattern 0x%X\n", pats[p]);
    // D layout (16x16 MFMA): lane l holds col = l & 15, rows 4*(l>>4) + q
    for (int row = 0; row < 16; ++row) {
      printf("row %2d:", row);
      for (int m = 0; m < 4; ++m)
        for (int c = 0; c < 16; ++c) {
          const int lane = 16 * (row / 4) + c, q = row % 4;
          printf(" %g", h[(m * 64 + lane) * 4 + q]);
        }
      printf("\n");
    }
  }
  return 0;
}
