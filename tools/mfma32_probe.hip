// Probe the operand layouts of v_mfma_f32_32x32x16_f16 and v_smfmac_f32_32x32x32_f16 on gfx950
// (diagnostic tool: hipcc -O2 --offload-arch=gfx950 tools/mfma32_probe.hip -o /tmp/p32 && /tmp/p32).
// Random small-integer matrices (exact in f16/f32) are packed under a layout hypothesis, multiplied on
// the matrix cores and compared with a host product; the max |error| per hypothesis is printed (0 =
// the hypothesis is the hardware's layout).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x16 __attribute__((ext_vector_type(16)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// dense: A[32][16], B[16][32]; lane l: A[l%32][8(l/32)+j], B[8(l/32)+j][l%32];
// D: register r of lane l = D[8(r/4) + 4(l/32) + r%4][l%32]
__global__ void dense(const float* A, const float* B, float* D) {
  const int l = threadIdx.x, h = l >> 5, c = l & 31;
  f16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (_Float16)A[c * 16 + 8 * h + j];
    b[j] = (_Float16)B[(8 * h + j) * 32 + c];
  }
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[(8 * (r / 4) + 4 * h + (r % 4)) * 32 + c] = acc[r];
}

// sparse: dense A[32][32] with 2 nonzeros per group of 4 along K (positions p0 < p1 per group);
// lane l covers row l%32, dense K [16(l/32), 16(l/32)+16) = groups q = 0..3: a[2q], a[2q+1] = the two
// nonzeros, idx nibble q = p0 | p1 << 2.  B[32][32]: hypothesis bh (0: lane half h holds K = 8h..8h+7
// and 16+8h..16+8h+7; 1: K = 16h..16h+15).
__global__ void sparse(const float* A, const int* P, const float* B, float* D, int bh) {
  const int l = threadIdx.x, h = l >> 5, c = l & 31;
  f16x8 a;
  int idx = 0;
  for (int q = 0; q < 4; ++q) {
    const int g = 4 * h + q;  // group of 4 along K in row c
    const int p0 = P[(c * 8 + g) * 2], p1 = P[(c * 8 + g) * 2 + 1];
    a[2 * q] = (_Float16)A[c * 32 + 4 * g + p0];
    a[2 * q + 1] = (_Float16)A[c * 32 + 4 * g + p1];
    idx |= (p0 | (p1 << 2)) << (4 * q);
  }
  f16x16 b;
  for (int j = 0; j < 16; ++j) {
    const int k = bh == 0 ? (j < 8 ? 8 * h + j : 16 + 8 * h + (j - 8)) : 16 * h + j;
    b[j] = (_Float16)B[k * 32 + c];
  }
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  acc = __builtin_amdgcn_smfmac_f32_32x32x32_f16(a, b, acc, idx, 0, 0);
  for (int r = 0; r < 16; ++r) D[(8 * (r / 4) + 4 * h + (r % 4)) * 32 + c] = acc[r];
}

int main() {
  srand(7);
  float hA[32 * 32], hB[32 * 32], hD[32 * 32];
  int hP[32 * 8 * 2];
  float *A, *B, *D;
  int* P;
  hipMalloc(&A, sizeof(hA));
  hipMalloc(&B, sizeof(hB));
  hipMalloc(&D, sizeof(hD));
  hipMalloc(&P, sizeof(hP));
  // dense
  for (int i = 0; i < 32 * 16; ++i) hA[i] = (float)(rand() % 7 - 3);
  for (int i = 0; i < 16 * 32; ++i) hB[i] = (float)(rand() % 7 - 3);
  hipMemcpy(A, hA, sizeof(hA), hipMemcpyHostToDevice);
  hipMemcpy(B, hB, sizeof(hB), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(dense, dim3(1), dim3(64), 0, 0, A, B, D);
  hipMemcpy(hD, D, sizeof(hD), hipMemcpyDeviceToHost);
  double err = 0;
  for (int i = 0; i < 32; ++i)
    for (int n = 0; n < 32; ++n) {
      double s = 0;
      for (int k = 0; k < 16; ++k) s += hA[i * 16 + k] * hB[k * 32 + n];
      err = fmax(err, fabs(s - hD[i * 32 + n]));
    }
  printf("dense 32x32x16 f16: max err %g\n", err);
  // sparse
  for (int i = 0; i < 32 * 32; ++i) hA[i] = 0.f;
  for (int row = 0; row < 32; ++row)
    for (int g = 0; g < 8; ++g) {
      int p0 = rand() % 4, p1 = rand() % 4;
      while (p1 == p0) p1 = rand() % 4;
      if (p1 < p0) { int t = p0; p0 = p1; p1 = t; }
      hP[(row * 8 + g) * 2] = p0;
      hP[(row * 8 + g) * 2 + 1] = p1;
      hA[row * 32 + 4 * g + p0] = (float)(rand() % 5 + 1);
      hA[row * 32 + 4 * g + p1] = (float)(rand() % 5 + 1);
    }
  for (int i = 0; i < 32 * 32; ++i) hB[i] = (float)(rand() % 7 - 3);
  hipMemcpy(A, hA, sizeof(hA), hipMemcpyHostToDevice);
  hipMemcpy(B, hB, sizeof(hB), hipMemcpyHostToDevice);
  hipMemcpy(P, hP, sizeof(hP), hipMemcpyHostToDevice);
  for (int bh = 0; bh < 2; ++bh) {
    hipLaunchKernelGGL(sparse, dim3(1), dim3(64), 0, 0, A, P, B, D, bh);
    hipMemcpy(hD, D, sizeof(hD), hipMemcpyDeviceToHost);
    err = 0;
    for (int i = 0; i < 32; ++i)
      for (int n = 0; n < 32; ++n) {
        double s = 0;
        for (int k = 0; k < 32; ++k) s += hA[i * 32 + k] * hB[k * 32 + n];
        err = fmax(err, fabs(s - hD[i * 32 + n]));
      }
    printf("sparse 32x32x32 f16, B hypothesis %d: max err %g\n", bh, err);
  }
  return 0;
}
