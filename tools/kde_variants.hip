// tools/kde_variants.hip -- design-space microbenchmark for the KDE scoring inner loop (dev tool,
// not part of the engine).  Times several ways of feeding the wave-uniform observation rows to the
// per-lane candidate FMAs, on the config-#3 "g" shape (8500 obs x 1e6 candidates, 24c + 8u):
//   sgpr<CPT>   rows through scalar loads (SGPR operands)          -- the engine's current scheme
//   lds<CPT>    rows staged in LDS per block, broadcast ds_read into VGPRs
//   ceil<CPT>   no observation loads at all (rows from a register ring) -- VALU ceiling
// Build/run on the GPU box:  hipcc -O3 --offload-arch=gfx950 -o /tmp/kv tools/kde_variants.hip && /tmp/kv
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>
#include <string.h>

#define DC 24
#define DU 8
#define STRIDE 36
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ float cat_match(float a, float b) {
  const float d = a - b;
  return __builtin_amdgcn_fmed3f(fmaf(-d, d, 1.f), 0.f, 1.f);
}

struct Cand { float xs[DC]; float xu[DU]; float ci; };

template <int CPT>
__device__ __forceinline__ void load_cands(const float* __restrict__ cand, int64_t Nc, int64_t base, Cand* c) {
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    int64_t i = base + k * 256;
    if (i >= Nc) i = Nc - 1;
    const float* x = cand + i * 32;
    float ci = 0.f;
#pragma unroll
    for (int d = 0; d < DC; ++d) { c[k].xs[d] = 2.f * x[d]; ci = fmaf(-x[d], x[d], ci); }
#pragma unroll
    for (int u = 0; u < DU; ++u) c[k].xu[u] = x[DC + u];
    c[k].ci = ci;
  }
}

template <int CPT>
__device__ __forceinline__ void pair_block(const float* r, const Cand* c, const float* dl, float* S) {
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    float t = c[k].ci + r[0];
#pragma unroll
    for (int d = 0; d < DC; ++d) t = fmaf(c[k].xs[d], r[1 + d], t);
#pragma unroll
    for (int u = 0; u < DU; ++u) t = fmaf(dl[u], cat_match(c[k].xu[u], r[1 + DC + u]), t);
    S[k] += __builtin_amdgcn_exp2f(t);
  }
}

template <int CPT, int UNR>
__global__ __launch_bounds__(256) void k_sgpr(const float* __restrict__ cand, int64_t Nc, const float* __restrict__ table,
                                              int n, const float* __restrict__ dlp, float* __restrict__ out) {
  Cand c[CPT];
  const int64_t base = (int64_t)blockIdx.x * 256 * CPT + threadIdx.x;
  load_cands<CPT>(cand, Nc, base, c);
  float dl[DU];
#pragma unroll
  for (int u = 0; u < DU; ++u) dl[u] = dlp[u];
  float S[CPT];
#pragma unroll
  for (int k = 0; k < CPT; ++k) S[k] = 0.f;
#pragma unroll UNR
  for (int j = 0; j < n; ++j) pair_block<CPT>(table + (int64_t)j * STRIDE, c, dl, S);
#pragma unroll
  for (int k = 0; k < CPT; ++k) if (base + k * 256 < Nc) out[base + k * 256] = S[k];
}

// rows staged in LDS, CH rows per chunk, whole block loads a chunk with 16-B vector loads
template <int CPT, int CH>
__global__ __launch_bounds__(256) void k_lds(const float* __restrict__ cand, int64_t Nc, const float* __restrict__ table,
                                             int n, const float* __restrict__ dlp, float* __restrict__ out) {
  __shared__ __align__(16) float sm[CH * STRIDE];
  Cand c[CPT];
  const int64_t base = (int64_t)blockIdx.x * 256 * CPT + threadIdx.x;
  load_cands<CPT>(cand, Nc, base, c);
  float dl[DU];
#pragma unroll
  for (int u = 0; u < DU; ++u) dl[u] = dlp[u];
  float S[CPT];
#pragma unroll
  for (int k = 0; k < CPT; ++k) S[k] = 0.f;
  for (int j0 = 0; j0 < n; j0 += CH) {
    const int rows = min(CH, n - j0);
    const float4* src = (const float4*)(table + (int64_t)j0 * STRIDE);
    float4* dst = (float4*)sm;
    for (int q = threadIdx.x; q < rows * STRIDE / 4; q += 256) dst[q] = src[q];
    __syncthreads();
#pragma unroll 2
    for (int j = 0; j < rows; ++j) {
      float r[STRIDE];
      const float4* rp = (const float4*)(sm + j * STRIDE);
#pragma unroll
      for (int q = 0; q < STRIDE / 4; ++q) { float4 v = rp[q]; r[4*q] = v.x; r[4*q+1] = v.y; r[4*q+2] = v.z; r[4*q+3] = v.w; }
      pair_block<CPT>(r, c, dl, S);
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < CPT; ++k) if (base + k * 256 < Nc) out[base + k * 256] = S[k];
}

// VALU ceiling: rows synthesized from registers (no memory traffic inside the loop)
template <int CPT>
__global__ __launch_bounds__(256) void k_ceil(const float* __restrict__ cand, int64_t Nc, const float* __restrict__ table,
                                              int n, const float* __restrict__ dlp, float* __restrict__ out) {
  Cand c[CPT];
  const int64_t base = (int64_t)blockIdx.x * 256 * CPT + threadIdx.x;
  load_cands<CPT>(cand, Nc, base, c);
  float dl[DU];
#pragma unroll
  for (int u = 0; u < DU; ++u) dl[u] = dlp[u];
  float r[STRIDE];
#pragma unroll
  for (int q = 0; q < STRIDE; ++q) r[q] = table[q];
  float S[CPT];
#pragma unroll
  for (int k = 0; k < CPT; ++k) S[k] = 0.f;
  for (int j = 0; j < n; ++j) {
    pair_block<CPT>(r, c, dl, S);
    r[0] = r[0] * 0.999f;  // keep the loop from being hoisted
    asm volatile("" : "+v"(r[0]));
  }
#pragma unroll
  for (int k = 0; k < CPT; ++k) if (base + k * 256 < Nc) out[base + k * 256] = S[k];
}

typedef void (*kfn)(const float*, int64_t, const float*, int, const float*, float*);

int main() {
  const int64_t Nc = 1000000;
  const int n = 8500;
  std::vector<float> hc(Nc * 32), ht((size_t)n * STRIDE), hd(DU);
  srand(1);
  for (auto& v : hc) v = (float)rand() / RAND_MAX;
  for (int64_t i = 0; i < Nc; ++i) for (int u = 0; u < DU; ++u) hc[i * 32 + DC + u] = (float)(rand() % 4);
  for (int j = 0; j < n; ++j) {
    float C = 0;
    for (int d = 0; d < DC; ++d) { float v = (float)rand() / RAND_MAX; ht[j * STRIDE + 1 + d] = v; C -= v * v; }
    for (int u = 0; u < DU; ++u) ht[j * STRIDE + 1 + DC + u] = (float)(rand() % 4);
    ht[j * STRIDE] = C - 3.f;
    for (int p = 1 + DC + DU; p < STRIDE; ++p) ht[j * STRIDE + p] = 0;
  }
  for (int u = 0; u < DU; ++u) hd[u] = 1.1f;
  float *dc, *dt, *dd, *dout;
  CHK(hipMalloc(&dc, hc.size() * 4)); CHK(hipMalloc(&dt, ht.size() * 4)); CHK(hipMalloc(&dd, 64)); CHK(hipMalloc(&dout, Nc * 4));
  CHK(hipMemcpy(dc, hc.data(), hc.size() * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dt, ht.data(), ht.size() * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dd, hd.data(), DU * 4, hipMemcpyHostToDevice));
  struct V { const char* name; kfn f; int cpt; } vs[] = {
    {"sgpr cpt1 unr2", k_sgpr<1, 2>, 1}, {"sgpr cpt2 unr2", k_sgpr<2, 2>, 2}, {"sgpr cpt4 unr1", k_sgpr<4, 1>, 4},
    {"sgpr cpt2 unr4", k_sgpr<2, 4>, 2},
    {"lds cpt1 ch128", k_lds<1, 128>, 1}, {"lds cpt2 ch128", k_lds<2, 128>, 2}, {"lds cpt4 ch128", k_lds<4, 128>, 4},
    {"lds cpt2 ch512", k_lds<2, 512>, 2},
    {"ceil cpt1", k_ceil<1>, 1}, {"ceil cpt2", k_ceil<2>, 2}, {"ceil cpt4", k_ceil<4>, 4},
  };
  const int NV = sizeof(vs) / sizeof(vs[0]);
  std::vector<float> best(NV, 1e30f), ref(Nc), got(Nc);
  hipEvent_t a, b;
  CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  for (int round = 0; round < 4; ++round) {
    for (int v = 0; v < NV; ++v) {
      const unsigned grid = (unsigned)((Nc + 256 * vs[v].cpt - 1) / (256 * vs[v].cpt));
      CHK(hipEventRecord(a));
      hipLaunchKernelGGL(vs[v].f, dim3(grid), dim3(256), 0, 0, dc, Nc, dt, n, dd, dout);
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms; CHK(hipEventElapsedTime(&ms, a, b));
      if (ms < best[v]) best[v] = ms;
      if (round == 0) {
        CHK(hipMemcpy(got.data(), dout, Nc * 4, hipMemcpyDeviceToHost));
        if (v == 0) ref = got;
        double md = 0;
        for (int64_t i = 0; i < Nc; i += 997) md = fmax(md, fabs(got[i] - ref[i]) / (fabs(ref[i]) + 1e-30));
        if (strncmp(vs[v].name, "ceil", 4)) printf("check %-16s max rel diff vs sgpr1 %.3g\n", vs[v].name, md);
      }
    }
  }
  for (int v = 0; v < NV; ++v)
    printf("%-16s %8.3f ms  %.3e pairs/s\n", vs[v].name, best[v], (double)Nc * n / (best[v] * 1e-3));
  return 0;
}
