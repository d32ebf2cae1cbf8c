// tools/mfma_overlap.hip -- does VALU work overlap f32 / f16 MFMA on gfx950? (dev microbenchmark)
// Each kernel: every wave runs ITER iterations of {M MFMAs} and/or {V independent v_fma chains}.
// Compare time(mfma only) + time(valu only) against time(both in the same wave).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int MF32, int MF16, int VF>
__global__ __launch_bounds__(256) void k(float* out, int iters, float seed) {
  f32x4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  float a = seed + threadIdx.x, b = seed * 2.f;
  f16x8 ha, hb;
  for (int i = 0; i < 8; ++i) { ha[i] = (_Float16)(a * 0.001f + i); hb[i] = (_Float16)(b * 0.001f - i); }
  float v[8];
  for (int i = 0; i < 8; ++i) v[i] = a + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < MF32; ++m) acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m & 3], 0, 0, 0);
#pragma unroll
    for (int m = 0; m < MF16; ++m) acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, hb, acc[m & 3], 0, 0, 0);
#pragma unroll
    for (int r = 0; r < VF; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = fmaf(v[i], 0.999f, 0.5f);
    }
  }
  float s = 0;
  for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  for (int i = 0; i < 8; ++i) s += v[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

typedef void (*kf)(float*, int, float);

int main() {
  float* out;
  const int blocks = 256 * 8;  // 8 waves... 4 waves/block -> 32 waves per CU
  CHK(hipMalloc(&out, blocks * 256 * 4));
  struct { const char* name; kf f; } ks[] = {
      {"f32mfma x8", k<8, 0, 0>},   {"valu 8x8 fma", k<0, 0, 8>},  {"f32mfma x8 + valu 8x8", k<8, 0, 8>},
      {"f16mfma x8", k<0, 8, 0>},   {"f16mfma x8 + valu 8x8", k<0, 8, 8>},
      {"f16mfma x4 + valu 8x8", k<0, 4, 8>}, {"f32mfma x4 + valu 8x8", k<4, 0, 8>},
  };
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int iters = 4000;
  for (int round = 0; round < 3; ++round)
    for (auto& x : ks) {
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(x.f, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (round == 2) printf("%-26s %8.3f ms\n", x.name, ms);
    }
  return 0;
}
