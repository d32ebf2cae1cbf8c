// Matrix-instruction throughput on gfx950 (diagnostic): back-to-back MFMAs, 4 independent accumulators
// per wave, one or two waves per SIMD on every CU.  Prints cycles per instruction per SIMD at an
// assumed clock (pass the clock in GHz; the chip holds ~2.07 GHz under this load, GRBM_GUI_ACTIVE).
// hipcc -O3 --offload-arch=gfx950 tools/mfma_rate.hip -o tools/mfma_rate && tools/mfma_rate 2.07
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define ITERS 2048

template <int KIND>
__global__ __launch_bounds__(256) void rate(float* out, int seed) {
  f16x8 a, b;
  f16x16 b16;
  for (int j = 0; j < 8; ++j) {
    a[j] = (_Float16)(float)((threadIdx.x + j + seed) & 3);
    b[j] = (_Float16)(float)((threadIdx.x * 3 + j) & 3);
  }
  for (int j = 0; j < 16; ++j) b16[j] = (_Float16)(float)((threadIdx.x + 5 * j) & 3);
  if (KIND < 2) {
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < ITERS; ++i) {
      if (KIND == 0) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c3, 0, 0, 0);
      } else {
        c0 = __builtin_amdgcn_smfmac_f32_32x32x32_f16(a, b16, c0, 0x4444, 0, 0);
        c1 = __builtin_amdgcn_smfmac_f32_32x32x32_f16(a, b16, c1, 0x4444, 0, 0);
        c2 = __builtin_amdgcn_smfmac_f32_32x32x32_f16(a, b16, c2, 0x4444, 0, 0);
        c3 = __builtin_amdgcn_smfmac_f32_32x32x32_f16(a, b16, c3, 0x4444, 0, 0);
      }
    }
    float s = 0.f;
    for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else {
    f32x4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < ITERS; ++i) {
      if (KIND == 2) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c3, 0, 0, 0);
      } else {
        c0 = __builtin_amdgcn_smfmac_f32_16x16x64_f16(a, b16, c0, 0x4444, 0, 0);
        c1 = __builtin_amdgcn_smfmac_f32_16x16x64_f16(a, b16, c1, 0x4444, 0, 0);
        c2 = __builtin_amdgcn_smfmac_f32_16x16x64_f16(a, b16, c2, 0x4444, 0, 0);
        c3 = __builtin_amdgcn_smfmac_f32_16x16x64_f16(a, b16, c3, 0x4444, 0, 0);
      }
    }
    float s = 0.f;
    for (int r = 0; r < 4; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  }
}

template <int KIND>
static void run(const char* name, float* d, double ghz) {
  for (int blocks_per_cu = 1; blocks_per_cu <= 2; ++blocks_per_cu) {
    const int grid = 256 * blocks_per_cu;
    hipLaunchKernelGGL(rate<KIND>, dim3(grid), dim3(256), 0, 0, d, 1);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    for (int k = 0; k < 5; ++k) hipLaunchKernelGGL(rate<KIND>, dim3(grid), dim3(256), 0, 0, d, k);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // every SIMD runs blocks_per_cu waves x ITERS x 4 instructions per launch
    const double instr_per_simd = 5.0 * blocks_per_cu * ITERS * 4;
    printf("%-28s waves/SIMD %d: %.1f cycles per instruction per SIMD\n", name, blocks_per_cu,
           ms * 1e-3 * ghz * 1e9 / instr_per_simd);
  }
}

int main(int argc, char** argv) {
  const double ghz = argc > 1 ? atof(argv[1]) : 2.07;
  float* d;
  hipMalloc(&d, 512 * 256 * sizeof(float));
  run<0>("mfma_f32_32x32x16_f16", d, ghz);
  run<1>("smfmac_f32_32x32x32_f16", d, ghz);
  run<2>("mfma_f32_16x16x32_f16", d, ghz);
  run<3>("smfmac_f32_16x16x64_f16", d, ghz);
  return 0;
}
