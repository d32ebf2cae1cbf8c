// hbx_kde.hip -- KDE acquisition on MI355X (gfx950): l(x)/g(x) scoring of candidates against the
// good/bad product-kernel KDEs of BOHB, and the exact argmin.
//
// Reference path: bohb.py:124-152 calls statsmodels KDEMultivariate.pdf
// (SM:kernel_density.py:162-196 -> SM:_kernel_base.py:456-518 gpke -> SM:kernels.py:23-65,108-125)
// twice per candidate and keeps the first candidate with the smallest max(1e-8,g)/max(l,1e-8).
//
// Engine structure (one acquisition, all on one HIP stream, no host round trip until the result):
//   acq_init         U = +inf, counters = 0
//   kde_logpdf<..>   x2 (good, bad): fp32 log-domain sum over observations, one candidate per lane,
//                    observations broadcast through the scalar path; per candidate ln S+, ln S-, bound
//   kde_combine      per-candidate score interval [lo, hi] (ln units) + block min of hi -> U
//   kde_shortlist    every candidate with lo <= U (the only ones that can be the argmin)
//   kde_exact        fp64 re-score of the shortlist in the reference's arithmetic/operation order
//   kde_final        strict-'<', first-index argmin over the exact scores
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "hbx_common.h"

#define HBX_LN2f 0.69314718055994531f
#define HBX_LN_CLAMP (-18.420680743952367)   // ln(1e-8), bohb.py:129
#define HBX_INV_SQRT_2PI 0.3989422804014327  // 1. / np.sqrt(2 * np.pi), SM:kernels.py:125
#define EXACT_GRID 2048  // blocks of the exact re-score (grid-stride over its work items)
#define SUM_BLOCK 32
#define OBS_CHUNK 64   // observations per table chunk (= per LDS stage of the scoring kernel)
#define KROW 80        // floats per k-row of a chunk: 64 observations + 16 pad (LDS bank spread)
#define MFMA_WAVES 8   // waves per scoring block; each wave owns 16 candidates
#define H_ROW_TILES 2  // hmode: 16-candidate row tiles per wave (32 candidates)

// ------------------------------------------------------------------------------------------
// model preparation

static void bucket_dims(int dc, int du, int* dc_pad, int* du_pad) {
  static const int dcb[] = {0, 4, 8, 16, 24, 32, 64};
  static const int dub[] = {0, 4, 8, 16, 32};
  *dc_pad = -1;
  *du_pad = -1;
  for (int b : dcb)
    if (dc <= b) { *dc_pad = b; break; }
  for (int b : dub)
    if (du <= b) { *du_pad = b; break; }
}

// Observation table, chunked for the MFMA scoring kernel.  Chunk c holds observations 64c..64c+63:
//   [KP k-rows][KROW]   B operand, k-major: k=0 -> C_j, k=1 -> 1, k=2+c -> X'_jc, rest 0
//   [64][du_pad]        categorical codes (float), observation-major
// KP = dc_pad + 2 rounded up to a multiple of 4 (MFMA 16x16x4 K step).  Observations past n in the
// last chunk are padding with C_j = -1e30 (their terms are exactly 0).
//
// Categorical part when kc >= 1 (one-hot mode): 64 observations x kc*32 f16, observation-major,
// slot k = 2*t + p of one-hot position t = (dim u, level) holds delta_u's f16 hi (p=0) / lo (p=1)
// part when the observation has that level, else 0; for signed KDEs a second block of the same
// shape holds 1 in the hi slot of matches in dims with negative match weight (parity count).
#define OH_MAX_KC 4  // one-hot mode up to 4 f16 MFMA K-steps: sum over dims of levels <= 64
__host__ __device__ constexpr int kp_of(int dc_pad) { return (dc_pad + 2 + 3) & ~3; }
__host__ __device__ constexpr int cat_floats(int du_pad, int kc, int sgn) {
  return kc == 0 ? OBS_CHUNK * du_pad : OBS_CHUNK * kc * 16 * (sgn ? 2 : 1);
}
__host__ __device__ constexpr int chunk_floats(int dc_pad, int du_pad, int kc = 0, int sgn = 0) {
  return kp_of(dc_pad) * KROW + cat_floats(du_pad, kc, sgn);
}
// hmode (all-f16) chunk: [64 f32: C_j] [64 obs x KTP halves: hi/lo continuous + one-hot] [signed:
// 64 obs x KPP halves parity]; continuous slot k = 4c + pt of dim c holds (pt even ? Xh_c : Xl_c) so
// the four products xh.Xh + xh.Xl + xl.Xh + xl.Xl reassemble x''.X' (A side: pt < 2 ? xh : xl).
// Rows are padded by 16 halves (32 B) so the 16 observation rows a wave reads are spread over banks.
__host__ __device__ constexpr int nsc_of(int dc_pad) { return (4 * dc_pad + 31) / 32; }
// row strides are 8*odd dwords: the 16 rows a ds_read_b128 lane group touches then cover all 64
// banks exactly once (conflict-free)
__host__ __device__ constexpr int h_ktp(int dc_pad, int kc) { return 32 * (nsc_of(dc_pad) + kc) + 16; }
__host__ __device__ constexpr int h_kpp(int kc) { return 32 * kc + 16; }
// padded to a multiple of 8 KB: every wave of the scoring block moves the same number of 1-KB
// LDS-DMA pieces per chunk (the counted vmcnt of the pipeline depends on it)
__host__ __device__ constexpr int h_chunk_floats(int dc_pad, int kc, int sgn) {
  return (OBS_CHUNK + OBS_CHUNK * h_ktp(dc_pad, kc) / 2 + (sgn ? OBS_CHUNK * h_kpp(kc) / 2 : 0) + 2047) & ~2047;
}
static int table_stride(int dc_pad, int du_pad) { return chunk_floats(dc_pad, du_pad); }  // floats per chunk
static int64_t n_chunks(int64_t n) { return (n + OBS_CHUNK - 1) / OBS_CHUNK; }
// capacity of a table: the largest layout hbx_kde_prepare may choose for this bucket
static int64_t table_floats(int64_t n, int dc_pad, int du_pad) {
  int a = chunk_floats(dc_pad, du_pad, 0, 0), b = chunk_floats(dc_pad, du_pad, OH_MAX_KC, 1);
  const int c = h_chunk_floats(dc_pad, OH_MAX_KC, 1);
  a = a > b ? a : b;
  return n_chunks(n) * (int64_t)(a > c ? a : c);
}

// Per active categorical dim (one block each): max observed code, -1 if some code is not an
// integer in [0, 1024) (then the one-hot mode is not used).
__global__ __launch_bounds__(256) void kde_maxcode_kernel(const double* __restrict__ X, int32_t D,
                                                          const int64_t* __restrict__ rows,
                                                          KdeParams* __restrict__ P) {
  __shared__ int red[256];
  const int u = blockIdx.x;
  const int d = P->cat_dim[u];
  int m = -1, bad = 0;
  for (int j = threadIdx.x; j < P->n; j += blockDim.x) {
    const double v = X[rows[j] * (int64_t)D + d];
    if (!(v >= 0.0 && v < 1024.0) || v != floor(v)) bad = 1;
    else m = max(m, (int)v);
  }
  red[threadIdx.x] = bad ? 100000 : m;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) P->cat_maxcode[u] = red[0] >= 100000 ? -1 : red[0];
}

// Per continuous slot (one block each): mean of the KDE's data column, the centre of the scaled
// coordinates.  Any finite centre is correct (table and candidates use the same one); it only keeps
// the fp32 expansion well conditioned, so the summation order is free.
__global__ __launch_bounds__(256) void kde_center_kernel(const double* __restrict__ X, int32_t D,
                                                         const int64_t* __restrict__ rows,
                                                         KdeParams* __restrict__ P) {
  __shared__ double red[4];
  const int k = blockIdx.x;
  const int d = P->cont_dim[k];
  const int n = P->n;
  double acc = 0.0;
  for (int j = threadIdx.x; j < n; j += 256) acc += X[rows[j] * (int64_t)D + d];
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double m = ((red[0] + red[1]) + (red[2] + red[3])) / (double)n;
    P->center[k] = (m == m && m - m == 0.0) ? m : 0.0;
  }
}

// Fill the chunked observation table (layout above).  X'_jc = s_c * (X_jc - mu_c),
// C_j = -sum_c X'_jc^2 + lb_sum - M0 (log2 units).  One thread per table slot j < nchunks*64.
__global__ __launch_bounds__(256) void kde_table_kernel(const double* __restrict__ X, int32_t D,
                                                        const int64_t* __restrict__ rows,
                                                        KdeParams* __restrict__ P,
                                                        float* __restrict__ table) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = P->n;
  const int nslots = ((n + OBS_CHUNK - 1) / OBS_CHUNK) * OBS_CHUNK;
  const bool ok = j < n;
  const bool slot = j < nslots;
  const double* x = X + (ok ? rows[j] : rows[0]) * (int64_t)D;
  const int dc = P->dc, du = P->du, dcp = P->dc_pad, dup = P->du_pad;
  const int KP = kp_of(dcp);
  float* ch = table + (int64_t)(j / OBS_CHUNK) * P->chunk_floats;
  const int jj = j % OBS_CHUNK;
  const bool hm = P->hmode != 0;
  const int KTP = h_ktp(dcp, P->kc);
  _Float16* hrow = (_Float16*)(ch + OBS_CHUNK) + jj * KTP;
  double C = 0.0;
  for (int k = 0; k < (hm ? dcp : KP - 2); ++k) {
    float v = 0.f;
    if (ok && k < dc) v = (float)(P->cont_scale[k] * (x[P->cont_dim[k]] - P->center[k]));
    C -= (double)v * (double)v;
    if (slot) {
      if (hm) {
        const float vc = fminf(fmaxf(v, -60000.f), 60000.f);
        const _Float16 h = (_Float16)vc;
        const _Float16 l = (_Float16)(vc - (float)h);
        hrow[4 * k + 0] = h;
        hrow[4 * k + 1] = l;
        hrow[4 * k + 2] = h;
        hrow[4 * k + 3] = l;
      } else {
        ch[(2 + k) * KROW + jj] = v;
      }
    }
    float a = fabsf(v);
    for (int o = 32; o > 0; o >>= 1) a = fmaxf(a, __shfl_xor(a, o));
    if ((threadIdx.x & 63) == 0 && k < dc) atomicMax((unsigned int*)&P->xmax[k], __float_as_uint(a));
  }
  if (hm && slot) {
    for (int k = 4 * dcp; k < 32 * P->nsc; ++k) hrow[k] = (_Float16)0.f;
    for (int k = 32 * (P->nsc + P->kc); k < KTP; ++k) hrow[k] = (_Float16)0.f;
  }
  if (P->kc == 0) {
    for (int u = 0; u < dup; ++u) {
      const float v = (ok && u < du) ? (float)x[P->cat_dim[u]] : -2.0f;
      if (slot) ch[KP * KROW + jj * dup + u] = v;
    }
  } else if (slot) {
    const int W = P->kc * 32;  // one-hot halves per observation
    _Float16* oh;
    _Float16* par;
    if (hm) {
      oh = hrow + 32 * P->nsc;
      par = (_Float16*)(ch + OBS_CHUNK + OBS_CHUNK * KTP / 2) + jj * h_kpp(P->kc);
    } else {
      oh = (_Float16*)(ch + KP * KROW) + jj * W;
      par = (_Float16*)(ch + KP * KROW) + OBS_CHUNK * W + jj * W;
    }
    for (int k = 0; k < W; ++k) {
      const int t = k >> 1, p = k & 1;
      float v = 0.f, pv = 0.f;
      if (ok && t < P->oh_total) {
        const int u = P->oh_dim[t];
        if (x[P->cat_dim[u]] == (double)P->oh_level[t]) {
          const float dl = fminf(fmaxf(P->cat_delta[u], -60000.f), 60000.f);
          const float hi = (float)(_Float16)dl;
          v = (p == 0) ? hi : (fabsf(dl) < 60000.f ? dl - hi : 0.f);
          pv = (p == 0 && P->cat_negf[u] != 0.f) ? 1.f : 0.f;
        }
      }
      oh[k] = (_Float16)v;
      if (P->has_neg) par[k] = (_Float16)pv;
    }
    if (hm && P->has_neg)
      for (int k = W; k < h_kpp(P->kc); ++k) par[k] = (_Float16)0.f;
  }
  C += P->lb_sum - P->m0_log2;
  const float Cf = ok ? (float)C : -1e30f;
  if (slot) {
    if (hm) {
      ch[jj] = Cf;
    } else {
      ch[0 * KROW + jj] = Cf;
      ch[1 * KROW + jj] = 1.f;
      if (jj < KROW - OBS_CHUNK)  // zero the pad columns of every k-row once per chunk
        for (int k = 0; k < KP; ++k) ch[k * KROW + OBS_CHUNK + jj] = 0.f;
    }
  }
  float a = ok ? fabsf(Cf) : 0.f;
  for (int o = 32; o > 0; o >>= 1) a = fmaxf(a, __shfl_xor(a, o));
  if ((threadIdx.x & 63) == 0) atomicMax((unsigned int*)&P->cmax, __float_as_uint(a));
  if (j == 0)
    for (int q = 0; q < P->nconst; ++q) P->const_level[q] = x[P->const_dim[q]];
}

// ------------------------------------------------------------------------------------------
// fp32 log-domain scoring
//
// Per (candidate i, observation j), in log2 units and minus the static bound M0:
//   t_ij = C_j + c_i + sum_c x''_ic X'_jc + sum_u delta_u [x_iu == X_ju]
// with X' = s (X - mu), x'' = 2 s (x - mu), c_i = -|x'_i|^2, C_j = -|X'_j|^2 + lb_sum - M0
// (the expansion of -|x' - X'|^2).  The first three terms are one GEMM-shaped product
// [candidates x K] . [K x observations] with K = 2 + Dc: they run on the f32 matrix cores
// (v_mfma_f32_16x16x4_f32, an exact fp32 FMA chain in k order).  The categorical match,
// exp2 and the sums run on the VALU beside them.  The categorical match is m = clamp(1 - d*d) on
// the integer codes (d = x - X), which stays in the VALU (no VCC round trip).

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float cat_match(float a, float b) {
  const float d = a - b;
  return __builtin_amdgcn_fmed3f(fmaf(-d, d, 1.f), 0.f, 1.f);
}

__device__ __forceinline__ float cand_code(double xv) {
  // codes are integers; anything else (incl. NaN) never equals an observed code
  return (xv == rint(xv) && fabs(xv) < 1e6) ? (float)xv : -1e9f;
}

// Per-candidate epilogue: ln S+, ln S-, error bound (or the rescue marker err = -1)
__device__ __forceinline__ KdeEst finish_est(const KdeParams* __restrict__ P, float S, float Sn, float off,
                                             bool nan_c, float ci, float bnd, bool SIGNED, int chunk) {
  KdeEst o;
  o.pad = 0.f;
  if (nan_c || S != S) {
    o.lpos = NAN;
    o.lneg = -INFINITY;
    o.err = 0.f;
    return o;
  }
  const float lnorm = (float)P->log_norm;
  const float Sp = SIGNED ? (S - Sn) : S;
  o.lpos = (Sp > 0.f) ? (__log2f(Sp) + off) * HBX_LN2f + lnorm : -INFINITY;
  o.lneg = (SIGNED && Sn > 0.f) ? (__log2f(Sn) + off) * HBX_LN2f + lnorm : -INFINITY;
  const float u = 0x1p-24f;
  const float Mabs = fabsf(ci) + P->cmax + bnd + P->sum_abs_delta;
  const float dt = 3.f * (float)(P->dc + P->du + 4) * u * Mabs;  // |error of t|, log2 units
  const float es = ((float)chunk + (float)P->n / (float)chunk + 24.f) * u * (SIGNED ? 3.f : 1.f);
  o.err = 2.f * (dt * HBX_LN2f + es) + 16.f * u;
  return o;
}

template <int DCP, int DUP, bool SIGNED>
__global__ __launch_bounds__(64 * MFMA_WAVES) void kde_logpdf_kernel(const double* __restrict__ cand, int64_t Nc,
                                                                    int32_t D, const KdeParams* __restrict__ P,
                                                                    const float* __restrict__ table,
                                                                    KdeEst* __restrict__ out) {
  constexpr int KP = kp_of(DCP);
  constexpr int NS = KP / 4;
  constexpr int CHF = chunk_floats(DCP, DUP);
  constexpr int NU = DUP > 0 ? DUP : 1;
  __shared__ __align__(16) float lds[2 * CHF];  // double-buffered observation chunks

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t cbase = ((int64_t)blockIdx.x * MFMA_WAVES + wave) * 16;  // this wave's 16 candidates
  const int n = P->n, dc = P->dc, du = P->du;
  const int ia = lane & 15, kq = lane >> 4;

  // A fragments: lane holds A[i = ia][k = 4s + kq]; A[i][0] = 1 (x C_j), A[i][1] = c_i, A[i][2+c] = x''_ic
  float a[NS];
  float ci_a = 0.f, bnd_a = 0.f;
  {
    int64_t ii = cbase + ia;
    if (ii >= Nc) ii = Nc - 1;
    const double* x = cand + ii * (int64_t)D;
    for (int k = 0; k < dc; ++k) {
      const float v = (float)(P->cont_scale[k] * (x[P->cont_dim[k]] - P->center[k]));
      ci_a = fmaf(-v, v, ci_a);
      bnd_a = fmaf(2.f * fabsf(v), P->xmax[k], bnd_a);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int k = 4 * s + kq;
      float v = 0.f;
      if (k == 0) {
        v = 1.f;
      } else if (k == 1) {
        v = ci_a;
      } else if (k - 2 < dc) {
        const int c = k - 2;
        v = 2.f * (float)(P->cont_scale[c] * (x[P->cont_dim[c]] - P->center[c]));
      }
      a[s] = v;
    }
  }
  // epilogue rows: the accumulator of lane holds candidates 4*kq + q (q = 0..3), observation ia
  float xu[4][NU];
  bool nanc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    int64_t ii = cbase + 4 * kq + q;
    if (ii >= Nc) ii = Nc - 1;
    const double* x = cand + ii * (int64_t)D;
#pragma unroll
    for (int u = 0; u < DUP; ++u) xu[q][u] = (u < du) ? cand_code(x[P->cat_dim[u]]) : -1.f;
    bool nn = P->nan_all != 0;
    for (int c = 0; c < P->nconst; ++c)
      if (x[P->const_dim[c]] != P->const_level[c]) nn = true;
    nanc[q] = nn;
  }
  float dl[NU], ng[NU];
#pragma unroll
  for (int u = 0; u < DUP; ++u) {
    dl[u] = (u < du) ? P->cat_delta[u] : 0.f;
    ng[u] = (u < du) ? P->cat_negf[u] : 0.f;
  }

  float S[4] = {0.f, 0.f, 0.f, 0.f}, Sn[4] = {0.f, 0.f, 0.f, 0.f};
  const int nchunks = (n + OBS_CHUNK - 1) / OBS_CHUNK;
  constexpr int NT = 64 * MFMA_WAVES;                 // threads per block
  constexpr int NV4 = CHF / 4;                        // float4 per chunk
  constexpr int PER = (NV4 + NT - 1) / NT;            // float4 per thread per chunk
  float4 pre[PER];
  // stage chunk 0; later chunks are prefetched into registers during the previous chunk's math
  {
    const float4* __restrict__ src = (const float4*)table;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int v = threadIdx.x + q * NT;
      if (v < NV4) ((float4*)lds)[v] = src[v];
    }
  }
  __syncthreads();

  // one 16x16 tile: B fragments and categorical codes of observation column jt*16 + ia
  auto load_tile = [&](const float* buf, int jt, float* b, float* xo) {
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2) b[s2] = buf[(4 * s2 + kq) * KROW + jt * 16 + ia];
#pragma unroll
    for (int u = 0; u < DUP; ++u) xo[u] = buf[KP * KROW + (jt * 16 + ia) * DUP + u];
  };
  auto epilogue = [&](const f32x4& acc, const float* xo, float* Sb, float* Snb) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float t = acc[q];
      float par = 0.f;
#pragma unroll
      for (int u = 0; u < DUP; ++u) {
        const float m = cat_match(xu[q][u], xo[u]);
        t = fmaf(dl[u], m, t);
        if (SIGNED) par = fmaf(m, ng[u], -fabsf(par));
      }
      const float e = __builtin_amdgcn_exp2f(t);
      Sb[q] += e;
      if (SIGNED) Snb[q] = fmaf(fabsf(par), e, Snb[q]);
    }
  };

  for (int c = 0; c < nchunks; ++c) {
    float* buf = lds + (c & 1) * CHF;
    const bool more = c + 1 < nchunks;
    if (more) {  // prefetch the next chunk into registers (lands during this chunk's math)
      const float4* __restrict__ src = (const float4*)(table + (int64_t)(c + 1) * CHF);
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int v = threadIdx.x + q * NT;
        if (v < NV4) pre[q] = src[v];
      }
    }
    float Sb[4] = {0.f, 0.f, 0.f, 0.f}, Snb[4] = {0.f, 0.f, 0.f, 0.f};
    // software pipeline over tile pairs: MFMAs of pair p+1 are issued before the VALU epilogue of p
    float b0[NS], b1[NS], xo0[NU], xo1[NU];
    f32x4 acc0, acc1;
    load_tile(buf, 0, b0, xo0);
    load_tile(buf, 1, b1, xo1);
    acc0 = f32x4{0.f, 0.f, 0.f, 0.f};
    acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s2], b0[s2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s2], b1[s2], acc1, 0, 0, 0);
    }
#pragma unroll
    for (int p = 0; p < OBS_CHUNK / 32; ++p) {
      f32x4 n0 = acc0, n1 = acc1;
      float c0[NU], c1[NU];
#pragma unroll
      for (int u = 0; u < DUP; ++u) {
        c0[u] = xo0[u];
        c1[u] = xo1[u];
      }
      if (p + 1 < OBS_CHUNK / 32) {
        load_tile(buf, 2 * p + 2, b0, xo0);
        load_tile(buf, 2 * p + 3, b1, xo1);
        acc0 = f32x4{0.f, 0.f, 0.f, 0.f};
        acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s2], b0[s2], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s2], b1[s2], acc1, 0, 0, 0);
        }
      }
      epilogue(n0, c0, Sb, Snb);
      epilogue(n1, c1, Sb, Snb);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      S[q] += Sb[q];
      if (SIGNED) Sn[q] += Snb[q];
    }
    if (more) {  // publish the prefetched chunk into the other buffer
      float4* dst = (float4*)(lds + ((c + 1) & 1) * CHF);
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int v = threadIdx.x + q * NT;
        if (v < NV4) dst[v] = pre[q];
      }
    }
    __syncthreads();
  }
  // reduce over the 16 lanes (observation columns) that share kq
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      S[q] += __shfl_xor(S[q], o);
      if (SIGNED) Sn[q] += __shfl_xor(Sn[q], o);
    }
  }
  // lane ia = q of group kq writes candidate 4*kq + q; c_i / bound of that candidate live in lane
  // (4*kq + q) & 15 + 16*anything of the A layout -> fetch with a shuffle
  const int src_lane = (4 * kq + (ia & 3)) & 15;
  const float ci_q = __shfl(ci_a, src_lane);
  const float bnd_q = __shfl(bnd_a, src_lane);
  if (ia < 4) {
    const int q = ia;
    const int64_t ii = cbase + 4 * kq + q;
    float Sq = S[0], Snq = Sn[0];
    bool nq = nanc[0];
    if (q == 1) { Sq = S[1]; Snq = Sn[1]; nq = nanc[1]; }
    if (q == 2) { Sq = S[2]; Snq = Sn[2]; nq = nanc[2]; }
    if (q == 3) { Sq = S[3]; Snq = Sn[3]; nq = nanc[3]; }
    if (ii < Nc) {
      KdeEst o = finish_est(P, Sq, Snq, 0.f, nq, ci_q, bnd_q, SIGNED, OBS_CHUNK / 16);
      if (!nq && Sq == Sq && Sq < 0x1p-64f) o.err = -1.f;  // rescue marker (kde_rescue_kernel)
      out[ii] = o;
    }
  }
}

// One-hot mode: the categorical sum  sum_u delta_u [x_u == X_u]  is a second matrix product,
// (candidate one-hot) x (delta-weighted observation one-hot), on the f16 matrix cores: operands are
// 0/1 and the f16 hi+lo parts of delta_u, so every product is exact and only the fp32 accumulation
// rounds.  It continues the same accumulator as the f32 continuous product, leaving the VALU only
// exp2 and the running sums.  Signed KDEs add one more f16 product that counts matches in dims with
// a negative match weight (the sign of the term is (-1)^count).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int DCP, int KC, bool SIGNED>
__global__ __launch_bounds__(64 * MFMA_WAVES) void kde_logpdf_oh_kernel(const double* __restrict__ cand,
                                                                       int64_t Nc, int32_t D,
                                                                       const KdeParams* __restrict__ P,
                                                                       const float* __restrict__ table,
                                                                       KdeEst* __restrict__ out) {
  constexpr int KP = kp_of(DCP);
  constexpr int NS = KP / 4;
  constexpr int W = KC * 32;  // one-hot halves per observation
  constexpr int CHF = chunk_floats(DCP, 0, KC, SIGNED ? 1 : 0);
  __shared__ __align__(16) float lds[2 * CHF];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t cbase = ((int64_t)blockIdx.x * MFMA_WAVES + wave) * 16;
  const int n = P->n, dc = P->dc;
  const int ia = lane & 15, kq = lane >> 4;

  float a[NS];
  f16x8 ah[KC];
  float ci_a = 0.f, bnd_a = 0.f;
  {
    int64_t ii = cbase + ia;
    if (ii >= Nc) ii = Nc - 1;
    const double* x = cand + ii * (int64_t)D;
    for (int k = 0; k < dc; ++k) {
      const float v = (float)(P->cont_scale[k] * (x[P->cont_dim[k]] - P->center[k]));
      ci_a = fmaf(-v, v, ci_a);
      bnd_a = fmaf(2.f * fabsf(v), P->xmax[k], bnd_a);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int k = 4 * s + kq;
      float v = 0.f;
      if (k == 0) {
        v = 1.f;
      } else if (k == 1) {
        v = ci_a;
      } else if (k - 2 < dc) {
        const int c = k - 2;
        v = 2.f * (float)(P->cont_scale[c] * (x[P->cont_dim[c]] - P->center[c]));
      }
      a[s] = v;
    }
    // candidate one-hot: lane holds A[row ia][k = 32 s + 8 kq + j]
    const int tot = P->oh_total;
#pragma unroll
    for (int s = 0; s < KC; ++s) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int t = (32 * s + 8 * kq + j) >> 1;
        float v = 0.f;
        if (t < tot && x[P->cat_dim[P->oh_dim[t]]] == (double)P->oh_level[t]) v = 1.f;
        ah[s][j] = (_Float16)v;
      }
    }
  }
  bool nanc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    int64_t ii = cbase + 4 * kq + q;
    if (ii >= Nc) ii = Nc - 1;
    const double* x = cand + ii * (int64_t)D;
    bool nn = P->nan_all != 0;
    for (int c = 0; c < P->nconst; ++c)
      if (x[P->const_dim[c]] != P->const_level[c]) nn = true;
    nanc[q] = nn;
  }

  float S[4] = {0.f, 0.f, 0.f, 0.f}, Sn[4] = {0.f, 0.f, 0.f, 0.f};
  const int nchunks = (n + OBS_CHUNK - 1) / OBS_CHUNK;
  constexpr int NT = 64 * MFMA_WAVES;
  constexpr int NV4 = CHF / 4;
  constexpr int PER = (NV4 + NT - 1) / NT;
  float4 pre[PER];
  {
    const float4* __restrict__ src = (const float4*)table;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int v = threadIdx.x + q * NT;
      if (v < NV4) ((float4*)lds)[v] = src[v];
    }
  }
  __syncthreads();

  // accumulate one 16x16 tile: f32 continuous product, then the f16 one-hot product
  auto tile = [&](const float* buf, int jt, f32x4& acc, f32x4& accp) {
    const _Float16* ohb = (const _Float16*)(buf + KP * KROW);
    acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; ++s)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], buf[(4 * s + kq) * KROW + jt * 16 + ia], acc, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      const f16x8 b = *(const f16x8*)(ohb + (jt * 16 + ia) * W + 32 * s + 8 * kq);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[s], b, acc, 0, 0, 0);
    }
    if (SIGNED) {
      accp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KC; ++s) {
        const f16x8 b = *(const f16x8*)(ohb + OBS_CHUNK * W + (jt * 16 + ia) * W + 32 * s + 8 * kq);
        accp = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[s], b, accp, 0, 0, 0);
      }
    }
  };
  auto epilogue = [&](const f32x4& acc, const f32x4& accp, float* Sb, float* Snb) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float e = __builtin_amdgcn_exp2f(acc[q]);
      Sb[q] += e;
      if (SIGNED) {
        const float odd = 2.f * __builtin_amdgcn_fractf(0.5f * accp[q]);  // count mod 2
        Snb[q] = fmaf(odd, e, Snb[q]);
      }
    }
  };

  for (int c = 0; c < nchunks; ++c) {
    float* buf = lds + (c & 1) * CHF;
    const bool more = c + 1 < nchunks;
    if (more) {
      const float4* __restrict__ src = (const float4*)(table + (int64_t)(c + 1) * CHF);
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int v = threadIdx.x + q * NT;
        if (v < NV4) pre[q] = src[v];
      }
    }
    float Sb[4] = {0.f, 0.f, 0.f, 0.f}, Snb[4] = {0.f, 0.f, 0.f, 0.f};
    f32x4 acc0, acc1, ap0, ap1;
    tile(buf, 0, acc0, ap0);
    tile(buf, 1, acc1, ap1);
#pragma unroll
    for (int p = 0; p < OBS_CHUNK / 32; ++p) {
      const f32x4 n0 = acc0, n1 = acc1, m0 = ap0, m1 = ap1;
      if (p + 1 < OBS_CHUNK / 32) {
        tile(buf, 2 * p + 2, acc0, ap0);
        tile(buf, 2 * p + 3, acc1, ap1);
      }
      epilogue(n0, m0, Sb, Snb);
      epilogue(n1, m1, Sb, Snb);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      S[q] += Sb[q];
      if (SIGNED) Sn[q] += Snb[q];
    }
    if (more) {
      float4* dst = (float4*)(lds + ((c + 1) & 1) * CHF);
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int v = threadIdx.x + q * NT;
        if (v < NV4) dst[v] = pre[q];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      S[q] += __shfl_xor(S[q], o);
      if (SIGNED) Sn[q] += __shfl_xor(Sn[q], o);
    }
  }
  const int src_lane = (4 * kq + (ia & 3)) & 15;
  const float ci_q = __shfl(ci_a, src_lane);
  const float bnd_q = __shfl(bnd_a, src_lane);
  if (ia < 4) {
    const int q = ia;
    const int64_t ii = cbase + 4 * kq + q;
    float Sq = S[0], Snq = Sn[0];
    bool nq = nanc[0];
    if (q == 1) { Sq = S[1]; Snq = Sn[1]; nq = nanc[1]; }
    if (q == 2) { Sq = S[2]; Snq = Sn[2]; nq = nanc[2]; }
    if (q == 3) { Sq = S[3]; Snq = Sn[3]; nq = nanc[3]; }
    if (ii < Nc) {
      KdeEst o = finish_est(P, Sq, Snq, 0.f, nq, ci_q, bnd_q, SIGNED, OBS_CHUNK / 16);
      if (!nq && Sq == Sq && Sq < 0x1p-64f) o.err = -1.f;
      out[ii] = o;
    }
  }
}

// hmode: the whole exponent is one f16 matrix product.  Continuous coordinates are split into f16
// hi + lo parts and all four cross products are summed (every f16 x f16 product is exact in fp32, so
// the only extra error is the 2^-22 representation error of each coordinate -- accounted in the
// bound); the one-hot categorical product follows in the same K loop.  C_j + c_i seed the
// accumulator.  VALU work per pair: one add, exp2, one add.
template <int NSC, int KC, bool SIGNED>
__global__ __launch_bounds__(64 * MFMA_WAVES) void kde_logpdf_h_kernel(const double* __restrict__ cand,
                                                                      int64_t Nc, int32_t D,
                                                                      const KdeParams* __restrict__ P,
                                                                      const float* __restrict__ table,
                                                                      KdeEst* __restrict__ out) {
  constexpr int RT = H_ROW_TILES;           // 16-candidate row tiles per wave
  constexpr int NSH = NSC + KC;             // f16 K-steps of 32
  constexpr int KTP = h_ktp(NSC * 8, KC);   // halves per observation row (padded); nsc_of(8 NSC) = NSC
  constexpr int KPP = h_kpp(KC);
  constexpr int CHF = h_chunk_floats(NSC * 8, KC, SIGNED ? 1 : 0);
  // LDS ring: 3 buffers (chunk c+2 in flight while c is used) when they fit in the 160 KB, else 2
  constexpr int NBUF = (3 * CHF * 4 <= 160 * 1024) ? 3 : 2;
  static_assert(NBUF * CHF * 4 <= 160 * 1024, "observation chunk too large for LDS");
  constexpr int G = CHF * 4 / (1024 * MFMA_WAVES);         // 1-KB LDS-DMA pieces per wave per chunk
  static_assert(G * 1024 * MFMA_WAVES == CHF * 4, "chunk must be a multiple of 8 KB");
  __shared__ __align__(16) float lds[NBUF * CHF];          // the kernel's only LDS object

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t cbase = ((int64_t)blockIdx.x * MFMA_WAVES + wave) * 16 * RT;
  const int n = P->n, dc = P->dc;
  const int ia = lane & 15, kq = lane >> 4;

  // A operands (candidate side).  Every lane walks all dims with wave-uniform (scalar) parameter
  // indices -- independent loads of its candidate's row, no lane-varying parameter lookups -- and
  // keeps the f16 slots its lane group kq owns: continuous dim c -> step c/8, lanes kq = (c%8)/2,
  // halves 4(c%2)+{0,1} = hi, +{2,3} = lo; one-hot slot t -> step NSC + t/16, kq = (t%16)/4,
  // halves 2(t%4)+{0,1}.
  f16x8 ah[RT][NSH];
  float ci_a[RT], bnd_a[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    int64_t ii = cbase + 16 * r + ia;
    if (ii >= Nc) ii = Nc - 1;
    const double* x = cand + ii * (int64_t)D;
    float ci = 0.f, bnd = 0.f;
#pragma unroll
    for (int s = 0; s < NSH; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) ah[r][s][j] = (_Float16)0.f;
#pragma unroll
    for (int c = 0; c < 8 * NSC; ++c) {
      if (c < dc) {
        const float v = (float)(P->cont_scale[c] * (x[P->cont_dim[c]] - P->center[c]));
        ci = fmaf(-v, v, ci);
        bnd = fmaf(2.f * fabsf(v), P->xmax[c], bnd);
        const float xc = fminf(fmaxf(2.f * v, -60000.f), 60000.f);
        const _Float16 hi = (_Float16)xc;
        const _Float16 lo = (_Float16)(xc - (float)hi);
        const bool mine = kq == ((c & 7) >> 1);
        const int j0 = 4 * (c & 1);
        ah[r][c >> 3][j0 + 0] = mine ? hi : ah[r][c >> 3][j0 + 0];
        ah[r][c >> 3][j0 + 1] = mine ? hi : ah[r][c >> 3][j0 + 1];
        ah[r][c >> 3][j0 + 2] = mine ? lo : ah[r][c >> 3][j0 + 2];
        ah[r][c >> 3][j0 + 3] = mine ? lo : ah[r][c >> 3][j0 + 3];
      }
    }
    ci_a[r] = ci;
    bnd_a[r] = bnd;
    const int tot = P->oh_total;
#pragma unroll
    for (int t = 0; t < 16 * KC; ++t) {
      if (t < tot) {
        const bool hit = (kq == ((t & 15) >> 2)) && x[P->oh_col[t]] == P->oh_val[t];
        const int s = NSC + (t >> 4), j0 = 2 * (t & 3);
        ah[r][s][j0 + 0] = hit ? (_Float16)1.f : ah[r][s][j0 + 0];
        ah[r][s][j0 + 1] = hit ? (_Float16)1.f : ah[r][s][j0 + 1];
      }
    }
  }
  // accumulator rows of this lane: candidates cbase + 16 r + 4 kq + q
  float ciq[RT][4];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q) ciq[r][q] = __shfl(ci_a[r], 4 * kq + q);

  float S[RT][4], Sn[RT][4];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q) S[r][q] = Sn[r][q] = 0.f;
  const int nchunks = (n + OBS_CHUNK - 1) / OBS_CHUNK;
  // LDS-DMA (global_load_lds_dwordx4): each wave copies its G 1-KB pieces of a chunk straight into
  // the ring; completion is tracked by a counted vmcnt + one raw barrier per chunk
  auto issue = [&](int c) {
    const float* src = table + (int64_t)c * CHF;
    float* dst = lds + (c % NBUF) * CHF;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int piece = wave + g * MFMA_WAVES;
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) const void*)(src + piece * 256 + lane * 4),
                                       (__attribute__((address_space(3))) void*)(dst + piece * 256), 16, 0, 0);
    }
  };
  issue(0);
  if (NBUF == 3 && nchunks > 1) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  // MFMAs of one 16-observation column tile for every row tile
  auto tile = [&](const float* buf, int jt, f32x4* acc, f32x4* accp) {
    const int jo = jt * 16 + ia;
    const float Cj = buf[jo];
    const _Float16* hb = (const _Float16*)(buf + OBS_CHUNK) + jo * KTP + 8 * kq;
    f16x8 b[NSH];
#pragma unroll
    for (int s = 0; s < NSH; ++s) b[s] = *(const f16x8*)(hb + 32 * s);
#pragma unroll
    for (int r = 0; r < RT; ++r) acc[r] = f32x4{ciq[r][0] + Cj, ciq[r][1] + Cj, ciq[r][2] + Cj, ciq[r][3] + Cj};
#pragma unroll
    for (int s = 0; s < NSH; ++s)
#pragma unroll
      for (int r = 0; r < RT; ++r) acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[r][s], b[s], acc[r], 0, 0, 0);
    if (SIGNED) {
      const _Float16* pb = (const _Float16*)(buf + OBS_CHUNK + OBS_CHUNK * KTP / 2) + jo * KPP + 8 * kq;
#pragma unroll
      for (int r = 0; r < RT; ++r) accp[r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KC; ++s) {
        const f16x8 bp = *(const f16x8*)(pb + 32 * s);
#pragma unroll
        for (int r = 0; r < RT; ++r)
          accp[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[r][NSC + s], bp, accp[r], 0, 0, 0);
      }
    }
  };

  for (int c = 0; c < nchunks; ++c) {
    const float* buf = lds + (c % NBUF) * CHF;
    if (c + NBUF - 1 < nchunks) issue(c + NBUF - 1);  // its buffer was last read in iteration c-1
    float Sb[RT][4], Snb[RT][4];
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) Sb[r][q] = Snb[r][q] = 0.f;
    // software pipeline: MFMAs of tile jt+1 are issued before the exp2/sum epilogue of tile jt
    f32x4 acc[RT], accp[RT];
    tile(buf, 0, acc, accp);
#pragma unroll
    for (int jt = 0; jt < OBS_CHUNK / 16; ++jt) {
      f32x4 cur[RT], curp[RT];
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        cur[r] = acc[r];
        curp[r] = accp[r];
      }
      if (jt + 1 < OBS_CHUNK / 16) tile(buf, jt + 1, acc, accp);
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float e = __builtin_amdgcn_exp2f(cur[r][q]);
          Sb[r][q] += e;
          if (SIGNED) Snb[r][q] = fmaf(2.f * __builtin_amdgcn_fractf(0.5f * curp[r][q]), e, Snb[r][q]);
        }
    }
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        S[r][q] += Sb[r][q];
        if (SIGNED) Sn[r][q] += Snb[r][q];
      }
    // chunk c+1 complete for this wave (chunk c+2 may stay in flight), this wave's reads of buffer c
    // retired; then the barrier makes chunk c+1 visible to (and buffer c free from) every wave
    if (NBUF == 3 && c + 2 < nchunks)
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(G) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        S[r][q] += __shfl_xor(S[r][q], o);
        if (SIGNED) Sn[r][q] += __shfl_xor(Sn[r][q], o);
      }
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    const int src_lane = (4 * kq + (ia & 3)) & 15;
    const float ci_q = __shfl(ci_a[r], src_lane);
    const float bnd_q = __shfl(bnd_a[r], src_lane);
    if (ia < 4) {
      const int q = ia;
      const int64_t ii = cbase + 16 * r + 4 * kq + q;
      float Sq = S[r][0], Snq = Sn[r][0];
      if (q == 1) { Sq = S[r][1]; Snq = Sn[r][1]; }
      if (q == 2) { Sq = S[r][2]; Snq = Sn[r][2]; }
      if (q == 3) { Sq = S[r][3]; Snq = Sn[r][3]; }
      if (ii < Nc) {
        const double* x = cand + ii * (int64_t)D;
        bool nq = P->nan_all != 0;
        for (int cc = 0; cc < P->nconst; ++cc)
          if (x[P->const_dim[cc]] != P->const_level[cc]) nq = true;
        KdeEst o = finish_est(P, Sq, Snq, 0.f, nq, ci_q, bnd_q, SIGNED, OBS_CHUNK / 16);
        // f16 hi/lo representation error of the continuous coordinates: 2 * 2^-22 * sum|x''X'|
        if (o.err > 0.f) o.err += 4.f * 0x1p-22f * bnd_q * HBX_LN2f;
        if (!nq && Sq == Sq && Sq < 0x1p-64f) o.err = -1.f;
        out[ii] = o;
      }
    }
  }
}

// Rescue (rare): candidates whose every term sits far below the static bound M0 are recomputed
// with a true maximum (two passes over the observations), one candidate per thread on the VALU.
// Continuous coordinates come from the table's f32 part, categorical codes straight from the data.
template <int DCP, bool SIGNED>
__global__ __launch_bounds__(256) void kde_rescue_kernel(const double* __restrict__ cand, int64_t Nc, int32_t D,
                                                         const KdeParams* __restrict__ P,
                                                         const float* __restrict__ table,
                                                         KdeEst* __restrict__ out) {
  constexpr int NC = DCP > 0 ? DCP : 1;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool need = i < Nc && out[i].err == -1.f;
  if (!__any(need)) return;
  if (!need) return;
  const double* x = cand + i * (int64_t)D;
  const int n = P->n, dc = P->dc, du = P->du;
  const double* __restrict__ Xo = P->X;
  const int64_t* __restrict__ rows = P->rows;
  float xs[NC], ci = 0.f, bnd = 0.f;
#pragma unroll
  for (int k = 0; k < DCP; ++k) {
    float v = 0.f;
    if (k < dc) v = (float)(P->cont_scale[k] * (x[P->cont_dim[k]] - P->center[k]));
    ci = fmaf(-v, v, ci);
    xs[k] = 2.f * v;
    if (k < dc) bnd = fmaf(fabsf(xs[k]), P->xmax[k], bnd);
  }
  auto pair_t = [&](int j, float& par) -> float {
    // observation row rebuilt exactly as kde_table_kernel writes it (f32 X', f64 C_j rounded once)
    const double* xo = Xo + rows[j] * (int64_t)D;
    float Xp[NC];
    double Cd = 0.0;
#pragma unroll
    for (int k = 0; k < DCP; ++k) {
      float v = 0.f;
      if (k < dc) v = (float)(P->cont_scale[k] * (xo[P->cont_dim[k]] - P->center[k]));
      Cd -= (double)v * (double)v;
      Xp[k] = v;
    }
    const float Cj = (float)(Cd + P->lb_sum - P->m0_log2);
    float t = fmaf(1.f, Cj, 0.f);
    t = fmaf(ci, 1.f, t);
#pragma unroll
    for (int k = 0; k < DCP; ++k) t = fmaf(xs[k], Xp[k], t);
    par = 0.f;
    for (int u = 0; u < du; ++u) {
      const int d = P->cat_dim[u];
      const float m = (x[d] == xo[d]) ? 1.f : 0.f;
      t = fmaf(P->cat_delta[u], m, t);
      if (SIGNED) par = fmaf(m, P->cat_negf[u], -fabsf(par));
    }
    return t;
  };
  float mx = -INFINITY, par;
  for (int j = 0; j < n; ++j) mx = fmaxf(mx, pair_t(j, par));
  float S = 0.f, Sn = 0.f;
  if (mx > -INFINITY) {
    for (int j0 = 0; j0 < n; j0 += OBS_CHUNK) {
      float Sb = 0.f, Snb = 0.f;
      for (int j = j0; j < min(n, j0 + OBS_CHUNK); ++j) {
        const float e = __builtin_amdgcn_exp2f(pair_t(j, par) - mx);
        Sb += e;
        if (SIGNED) Snb = fmaf(fabsf(par), e, Snb);
      }
      S += Sb;
      Sn += Snb;
    }
  } else {
    mx = 0.f;
  }
  out[i] = finish_est(P, S, Sn, mx, false, ci, bnd, SIGNED, OBS_CHUNK);
}

// ------------------------------------------------------------------------------------------
// score intervals, shortlist, exact re-score, final argmin

__global__ void acq_init_kernel(uint32_t* U, int32_t* count, int32_t* flags, AcqResult* res) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    *U = hbx_f2ord(INFINITY);
    *count = 0;
    *flags = 0;
    res->index = -1;
    res->score = NAN;
    res->pdf_l = NAN;
    res->pdf_g = NAN;
    res->shortlist = 0;
    res->flags = 0;
    res->pad = 0;
  }
}

// ln-pdf interval [lo, hi] and point estimate from (ln S+, ln S-, relative bound); -inf means pdf <= 0
__device__ __forceinline__ void est_interval(const KdeEst e, float* lo, float* hi, float* pt) {
  const float m = fmaxf(e.lpos, e.lneg);
  if (m == -INFINITY) {
    *lo = *hi = *pt = -INFINITY;
    return;
  }
  const float a = __expf(e.lpos - m), b = __expf(e.lneg - m);
  const float S = a - b, E = e.err * (a + b) + 1e-6f * (a + b);
  *pt = S > 0.f ? m + __logf(S) : -INFINITY;
  *hi = (S + E) > 0.f ? m + __logf(S + E) + 1e-6f * fabsf(m) + 1e-5f : -INFINITY;
  *lo = (S - E) > 0.f ? m + __logf(S - E) - 1e-6f * fabsf(m) - 1e-5f : -INFINITY;
}

__global__ __launch_bounds__(256) void kde_combine_kernel(const KdeEst* __restrict__ el,
                                                          const KdeEst* __restrict__ eg, int64_t Nc,
                                                          float* __restrict__ logl, float* __restrict__ logg,
                                                          float* __restrict__ lo, float* __restrict__ hi,
                                                          uint32_t* __restrict__ U, int32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  float h = INFINITY;
  if (i < Nc) {
    const KdeEst a = el[i], b = eg[i];
    const float C = (float)HBX_LN_CLAMP;
    float slo, shi;
    bool of = false;
    float llo, lhi, lpt, glo, ghi, gpt;
    if (a.lpos != a.lpos) {  // l NaN -> max(l, 1e-8) is NaN -> score NaN (never selected)
      slo = shi = NAN;
      lpt = NAN;
      est_interval(b, &glo, &ghi, &gpt);
      if (b.lpos != b.lpos) gpt = NAN;
    } else {
      est_interval(a, &llo, &lhi, &lpt);
      float Glo, Ghi;
      if (b.lpos != b.lpos) {  // g NaN -> max(1e-8, g) == 1e-8
        Glo = Ghi = C;
        gpt = NAN;
      } else {
        est_interval(b, &glo, &ghi, &gpt);
        Glo = fmaxf(glo, C);
        Ghi = fmaxf(ghi, C);
        of = ghi > 700.f;
      }
      of = of || lhi > 700.f;
      slo = Glo - fmaxf(lhi, C);
      shi = Ghi - fmaxf(llo, C);
      h = shi;
    }
    if (logl) logl[i] = lpt;
    if (logg) logg[i] = gpt;
    lo[i] = slo;
    hi[i] = shi;
    if (of) atomicOr(flags, 1);
  }
  // block min of hi
  __shared__ float red[4];
  for (int o = 32; o > 0; o >>= 1) h = fminf(h, __shfl_xor(h, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = fminf(fminf(red[0], red[1]), fminf(red[2], red[3]));
    if (m < INFINITY) atomicMin(U, hbx_f2ord(m));
  }
}

__global__ __launch_bounds__(256) void kde_shortlist_kernel(const float* __restrict__ lo, int64_t Nc,
                                                            const uint32_t* __restrict__ U,
                                                            const int32_t* __restrict__ flags,
                                                            int32_t* __restrict__ list,
                                                            int32_t* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= Nc) return;
  const float u = hbx_ord2f(*U);
  const bool all = (*flags & 1) != 0;
  const float l = lo[i];
  if (l == l && (all || l <= u)) {
    const int pos = atomicAdd(count, 1);
    list[pos] = (int32_t)i;
  }
}

// numpy's pairwise summation (umath loops: n < 8 plain, <= 128 eight accumulators, else split at
// n/2 rounded down to a multiple of 8).  dens.sum(axis=0) (SM:_kernel_base.py:516) runs it over the
// ufunc buffer chunks of 8192 elements, accumulated left to right from 0.0 -- see exact_pdf.
__device__ double pw_leaf_sum(const double* p, int len) {
  if (len < 8) {
    double res = 0.0;
    for (int i = 0; i < len; ++i) res += p[i];
    return res;
  }
  double r0 = p[0], r1 = p[1], r2 = p[2], r3 = p[3], r4 = p[4], r5 = p[5], r6 = p[6], r7 = p[7];
  int i;
  for (i = 8; i < len - (len % 8); i += 8) {
    r0 += p[i + 0]; r1 += p[i + 1]; r2 += p[i + 2]; r3 += p[i + 3];
    r4 += p[i + 4]; r5 += p[i + 5]; r6 += p[i + 6]; r7 += p[i + 7];
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < len; ++i) res += p[i];
  return res;
}

#define PW_BUF 8192    // numpy ufunc buffer (elements)
#define PW_CUT 3       // a buffer's split tree is cut at depth 3 into <= 8 independent units
#define PW_UNITS 8
#define PW_UNIT_MAX 1040  // longest depth-3 node of any m <= 8192 is 1031 elements
#define PW_LEVELS 8    // a unit's own split tree has depth <= 7
#define EXACT_THREADS 256
#define EXACT_SPLIT_CAP 2048  // shortlists up to this size spread every (candidate, KDE) over units

// Node (lev, t) of the split tree of an m-element buffer: walk t's bits from the root.  Returns
// false when the node does not exist (an ancestor is already a leaf).
__device__ __forceinline__ bool pw_node(int m, int lev, int t, int* off, int* len) {
  int o = 0, l = m;
  for (int b = lev - 1; b >= 0; --b) {
    if (l <= 128) return false;
    int n2 = l / 2;
    n2 -= n2 % 8;
    if ((t >> b) & 1) {
      o += n2;
      l -= n2;
    } else {
      l = n2;
    }
  }
  *off = o;
  *len = l;
  return true;
}

// Unit u (0..7) of a buffer: the depth-3 node at position u, or the shallower leaf whose leftmost
// depth-3 position is u.  Returns false for positions covered by another unit.
__device__ __forceinline__ bool pw_unit(int m, int u, int* off, int* len) {
  for (int lev = 0; lev <= PW_CUT; ++lev) {
    const int sh = PW_CUT - lev;
    if (!pw_node(m, lev, u >> sh, off, len)) return false;
    if (lev == PW_CUT || *len <= 128) return (u & ((1 << sh) - 1)) == 0;
  }
  return false;
}

// Top of the tree (depth <= 3) from the unit sums, numpy's order; one thread.
__device__ double pw_combine_units(int m, const double* us) {
  double v[PW_CUT + 1][PW_UNITS];
  for (int lev = PW_CUT; lev >= 0; --lev)
    for (int t = 0; t < (1 << lev); ++t) {
      int off, len;
      if (!pw_node(m, lev, t, &off, &len)) continue;
      v[lev][t] = (lev == PW_CUT || len <= 128) ? us[t << (PW_CUT - lev)] : v[lev + 1][2 * t] + v[lev + 1][2 * t + 1];
    }
  return v[0][0];
}

struct ExactShared {
  double dens[PW_UNIT_MAX];
  double nsum[PW_LEVELS][128];
  double usum[PW_UNITS];
  // per-dim constants of the reference kernels (SM:kernels.py:62-64,125): continuous -> (h*h)*2 in
  // c0, categorical -> 1-h in c0 and h/(c-1) in c1; the point's coordinates in xd
  double c0[HBX_MAX_D], c1[HBX_MAX_D], xd[HBX_MAX_D];
  int32_t cont[HBX_MAX_D];
};

// Pairwise sum of a[0:m] (m <= 1040, in LDS) in numpy's order, whole block, level-synchronous:
// a leaf (len <= 128) is summed by one thread, an inner node adds its two children of the level
// below.  Same additions, same order, as the recursive reference loop.
__device__ double np_pairwise_block(const double* a, int m, double (*nsum)[128]) {
  for (int lev = PW_LEVELS - 1; lev >= 0; --lev) {
    for (int t = threadIdx.x; t < (1 << lev); t += blockDim.x) {
      int off, len;
      if (pw_node(m, lev, t, &off, &len))
        nsum[lev][t] = (len <= 128) ? pw_leaf_sum(a + off, len) : nsum[lev + 1][2 * t] + nsum[lev + 1][2 * t + 1];
    }
    __syncthreads();
  }
  return nsum[0][0];
}

// Per-dim constants + the point's coordinates into LDS (whole block).
__device__ void exact_setup(const KdeParams* __restrict__ P, int32_t D, const double* __restrict__ x,
                            ExactShared* sh) {
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    const double h = P->bw[d];
    const bool c = P->vartype[d] == 0;
    sh->cont[d] = c;
    sh->c0[d] = c ? (h * h) * 2. : 1. - h;
    sh->c1[d] = c ? 0. : h / (double)(P->nlev[d] - 1);
    sh->xd[d] = x[d];
  }
  __syncthreads();
}

// Sum of the per-observation terms Kval.prod(1) / prod(bw_c) (SM:_kernel_base.py:509-516) over
// the observations [first, first+len) -- one unit of one buffer, pairwise order; whole block.
__device__ double exact_unit(const double* __restrict__ X, int32_t D, const int64_t* __restrict__ rows,
                             const KdeParams* __restrict__ P, int first, int len, ExactShared* sh) {
  const double pbc = P->prod_bw_c;
  for (int j = threadIdx.x; j < len; j += blockDim.x) {
    const double* xr = X + rows[first + j] * (int64_t)D;
    double p = 1.0;
#pragma unroll 8
    for (int d = 0; d < D; ++d) {
      const double v = xr[d], xv = sh->xd[d];
      double k;
      if (sh->cont[d]) {
        const double diff = v - xv;
        k = HBX_INV_SQRT_2PI * exp(-(diff * diff) / sh->c0[d]);
      } else {
        k = (v == xv) ? sh->c0[d] : sh->c1[d];
      }
      p = (d == 0) ? k : p * k;
    }
    sh->dens[j] = p / pbc;
  }
  __syncthreads();
  return np_pairwise_block(sh->dens, len, sh->nsum);
}

// exact fp64 pdf of one KDE at the point staged by exact_setup, one block, all units in turn
__device__ double exact_pdf(const double* __restrict__ X, int32_t D, const int64_t* __restrict__ rows,
                            const KdeParams* __restrict__ P, ExactShared* sh) {
  const int n = P->n;
  double acc = 0.0;  // np.add.reduce: identity 0.0, then one pairwise sum per 8192-element buffer
  for (int c = 0; c < n; c += PW_BUF) {
    const int m = (n - c) < PW_BUF ? (n - c) : PW_BUF;
    for (int u = 0; u < PW_UNITS; ++u) {
      int off, len;
      if (!pw_unit(m, u, &off, &len)) continue;
      const double v = exact_unit(X, D, rows, P, c + off, len, sh);
      if (threadIdx.x == 0) sh->usum[u] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) acc = acc + pw_combine_units(m, sh->usum);
  }
  return acc / (double)n;  // valid in thread 0
}

// Exact re-score of the shortlist.  Small shortlists (<= EXACT_SPLIT_CAP): one work item per
// (candidate, KDE, 8192-buffer, unit) so one candidate spreads over many CUs; the unit sums go to
// `part` and kde_final combines them.  Larger: one item per (candidate, KDE), all units in turn.
__global__ __launch_bounds__(EXACT_THREADS) void kde_exact_kernel(
    const double* __restrict__ cand, int32_t D,
    const KdeParams* __restrict__ Pg, const double* __restrict__ Xg, const int64_t* __restrict__ rows_g,
    const KdeParams* __restrict__ Pb, const double* __restrict__ Xb, const int64_t* __restrict__ rows_b,
    const int32_t* __restrict__ list, const int32_t* __restrict__ count, int32_t nbuf, double* __restrict__ part,
    double* __restrict__ exact_l, double* __restrict__ exact_g) {
  __shared__ ExactShared sh;
  const int cnt = *count;
  const bool split = cnt <= EXACT_SPLIT_CAP;
  const int per = split ? nbuf * PW_UNITS : 1;  // items per (candidate, KDE)
  const int64_t items = (int64_t)cnt * 2 * per;
  for (int64_t item = blockIdx.x; item < items; item += gridDim.x) {
    const int64_t pk = item / per;  // (candidate, KDE)
    const int p = (int)(pk >> 1);
    const bool isl = pk & 1;
    const KdeParams* P = isl ? Pg : Pb;
    const double* X = isl ? Xg : Xb;
    const int64_t* rows = isl ? rows_g : rows_b;
    if (split) {
      const int r = (int)(item % per), b = r / PW_UNITS, u = r % PW_UNITS;
      const int n = P->n, c = b * PW_BUF;
      if (c >= n) continue;
      const int m = (n - c) < PW_BUF ? (n - c) : PW_BUF;
      int off, len;
      if (!pw_unit(m, u, &off, &len)) continue;
      exact_setup(P, D, cand + (int64_t)list[p] * D, &sh);
      const double v = exact_unit(X, D, rows, P, c + off, len, &sh);
      if (threadIdx.x == 0) part[pk * per + r] = v;
    } else {
      exact_setup(P, D, cand + (int64_t)list[p] * D, &sh);
      const double v = exact_pdf(X, D, rows, P, &sh);
      if (threadIdx.x == 0) (isl ? exact_l : exact_g)[p] = v;
    }
    __syncthreads();
  }
}

// split mode: pdf of every (shortlisted candidate, KDE) from its unit sums; one thread each
__global__ __launch_bounds__(256) void kde_exact_combine_kernel(const KdeParams* __restrict__ Pg,
                                                                const KdeParams* __restrict__ Pb,
                                                                const int32_t* __restrict__ count, int32_t nbuf,
                                                                const double* __restrict__ part,
                                                                double* __restrict__ exact_l,
                                                                double* __restrict__ exact_g) {
  const int cnt = *count;
  if (cnt > EXACT_SPLIT_CAP) return;
  const int64_t pk = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (pk >= 2 * (int64_t)cnt) return;
  const bool isl = pk & 1;
  const int n = (isl ? Pg : Pb)->n;
  const double* us = part + pk * nbuf * PW_UNITS;
  double acc = 0.0;
  for (int c = 0, b = 0; c < n; c += PW_BUF, ++b) {
    const int m = (n - c) < PW_BUF ? (n - c) : PW_BUF;
    acc = acc + pw_combine_units(m, us + b * PW_UNITS);
  }
  (isl ? exact_l : exact_g)[pk >> 1] = acc / (double)n;
}

// exact fp64 pdf of one KDE at every row of pts (grid-stride over points, one block per point)
__global__ __launch_bounds__(EXACT_THREADS) void kde_pdf_exact_kernel(const double* __restrict__ pts, int64_t Np,
                                                                      int32_t D, const KdeParams* __restrict__ P,
                                                                      const double* __restrict__ X,
                                                                      const int64_t* __restrict__ rows,
                                                                      double* __restrict__ out) {
  __shared__ ExactShared sh;
  for (int64_t p = blockIdx.x; p < Np; p += gridDim.x) {
    exact_setup(P, D, pts + p * D, &sh);
    const double v = exact_pdf(X, D, rows, P, &sh);
    if (threadIdx.x == 0) out[p] = v;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void kde_final_kernel(const int32_t* __restrict__ list,
                                                        const int32_t* __restrict__ count,
                                                        const double* __restrict__ exact_l,
                                                        const double* __restrict__ exact_g,
                                                        const int32_t* __restrict__ flags, int64_t index_base,
                                                        AcqResult* __restrict__ res) {
  __shared__ double bs[256];
  __shared__ int64_t bi[256];
  __shared__ int32_t bp[256];
  const int cnt = *count;
  double best = INFINITY;
  int64_t bidx = INT64_MAX;
  int32_t bpos = -1;
  for (int p = threadIdx.x; p < cnt; p += 256) {
    // bohb.py:129 with Python max(): max(1e-8, g) keeps 1e-8 unless g > 1e-8 (NaN -> 1e-8);
    // max(l, 1e-8) keeps l unless 1e-8 > l (NaN -> NaN)
    const double g = exact_g[p], l = exact_l[p];
    const double s = ((g > 1e-8) ? g : 1e-8) / ((1e-8 > l) ? 1e-8 : l);
    const int64_t idx = list[p];
    // valid iff s < +inf (bohb.py:150 'val < best' with best = inf); strict '<', first index wins
    if (s < INFINITY && (s < best || (s == best && idx < bidx))) {
      best = s;
      bidx = idx;
      bpos = p;
    }
  }
  bs[threadIdx.x] = best;
  bi[threadIdx.x] = bidx;
  bp[threadIdx.x] = bpos;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      const double s2 = bs[threadIdx.x + w];
      const int64_t i2 = bi[threadIdx.x + w];
      if (s2 < bs[threadIdx.x] || (s2 == bs[threadIdx.x] && i2 < bi[threadIdx.x])) {
        bs[threadIdx.x] = s2;
        bi[threadIdx.x] = i2;
        bp[threadIdx.x] = bp[threadIdx.x + w];
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    res->shortlist = cnt;
    res->flags = *flags;
    if (bp[0] >= 0) {
      res->index = bi[0] + index_base;
      res->score = bs[0];
      res->pdf_l = exact_l[bp[0]];
      res->pdf_g = exact_g[bp[0]];
    }
  }
}

// ------------------------------------------------------------------------------------------
// launch-side dispatch over the (dc_pad, du_pad, signed) template buckets

typedef void (*logpdf_fn)(const double*, int64_t, int32_t, const KdeParams*, const float*, KdeEst*);
struct ScoreFns {
  logpdf_fn main, rescue;
  int cands_per_block;
};

// variant code of a prepared KDE (hbx_kde_prepare info[0]): bit 0 = signed sums, bits 1-3 = kc,
// bit 4 = hmode (whole exponent on the f16 matrix cores)
template <int NSC, bool SG>
static logpdf_fn pick_h(int kc) {
  switch (kc) {
    case 0: return kde_logpdf_h_kernel<NSC, 0, SG>;
    case 1: return kde_logpdf_h_kernel<NSC, 1, SG>;
    case 2: return kde_logpdf_h_kernel<NSC, 2, SG>;
    case 3: return kde_logpdf_h_kernel<NSC, 3, SG>;
    case 4: return kde_logpdf_h_kernel<NSC, 4, SG>;
  }
  return nullptr;
}

template <int DCP, int DUP, bool SG>
static ScoreFns pick_kc(int kc, bool hm) {
  const logpdf_fn r = kde_rescue_kernel<DCP, SG>;
  if (hm) {
    if constexpr (DCP >= 16) return {pick_h<nsc_of(DCP), SG>(kc), r, 16 * MFMA_WAVES * H_ROW_TILES};
    return {nullptr, nullptr, 0};
  }
  switch (kc) {
    case 0: return {kde_logpdf_kernel<DCP, DUP, SG>, r, 16 * MFMA_WAVES};
    case 1: return {kde_logpdf_oh_kernel<DCP, 1, SG>, r, 16 * MFMA_WAVES};
    case 2: return {kde_logpdf_oh_kernel<DCP, 2, SG>, r, 16 * MFMA_WAVES};
    case 3: return {kde_logpdf_oh_kernel<DCP, 3, SG>, r, 16 * MFMA_WAVES};
    case 4: return {kde_logpdf_oh_kernel<DCP, 4, SG>, r, 16 * MFMA_WAVES};
  }
  return {nullptr, nullptr, 0};
}

template <int DCP, int DUP>
static ScoreFns pick_signed(int variant) {
  const int kc = (variant >> 1) & 7;
  const bool hm = (variant >> 4) & 1;
  return (variant & 1) ? pick_kc<DCP, DUP, true>(kc, hm) : pick_kc<DCP, DUP, false>(kc, hm);
}

template <int DCP>
static ScoreFns pick_du(int du_pad, int variant) {
  switch (du_pad) {
    case 0: return pick_signed<DCP, 0>(variant & 0x11);  // no categorical dims: kc irrelevant
    case 4: return pick_signed<DCP, 4>(variant);
    case 8: return pick_signed<DCP, 8>(variant);
    case 16: return pick_signed<DCP, 16>(variant);
    case 32: return pick_signed<DCP, 32>(variant);
  }
  return {nullptr, nullptr};
}

static ScoreFns pick_logpdf(int dc_pad, int du_pad, int variant) {
  switch (dc_pad) {
    case 0: return pick_du<0>(du_pad, variant);
    case 4: return pick_du<4>(du_pad, variant);
    case 8: return pick_du<8>(du_pad, variant);
    case 16: return pick_du<16>(du_pad, variant);
    case 24: return pick_du<24>(du_pad, variant);
    case 32: return pick_du<32>(du_pad, variant);
    case 64: return pick_du<64>(du_pad, variant);
  }
  return {nullptr, nullptr, 0};
}

// launch main + rescue scoring for one KDE
static int launch_score(ScoreFns f, const double* cand, int64_t Nc, int32_t D, const void* params, const float* table,
                        KdeEst* est, hipStream_t s) {
  const unsigned gm = (unsigned)((Nc + f.cands_per_block - 1) / f.cands_per_block);
  hipLaunchKernelGGL(f.main, dim3(gm), dim3(64 * MFMA_WAVES), 0, s, cand, Nc, D, (const KdeParams*)params, table,
                     est);
  HBX_LAUNCH_CHECK();
  hipLaunchKernelGGL(f.rescue, dim3((unsigned)((Nc + 255) / 256)), dim3(256), 0, s, cand, Nc, D,
                     (const KdeParams*)params, table, est);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

// workspace layout (bytes), shared by hbx_kde_workspace_bytes and hbx_kde_acquire
struct WsLayout {
  size_t U, count, flags, res, est_l, est_g, lo, hi, list, exact_l, exact_g, part, total;
};

static WsLayout ws_layout(int64_t Nc, int64_t nmax) {
  WsLayout w;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    size_t r = o;
    o += (bytes + 255) & ~(size_t)255;
    return r;
  };
  w.U = take(4);
  w.count = take(4);
  w.flags = take(4);
  w.res = take(sizeof(AcqResult));
  w.est_l = take(sizeof(KdeEst) * Nc);
  w.est_g = take(sizeof(KdeEst) * Nc);
  w.lo = take(4 * Nc);
  w.hi = take(4 * Nc);
  w.list = take(4 * Nc);
  w.exact_l = take(8 * Nc);
  w.exact_g = take(8 * Nc);
  w.part = take(8 * (size_t)2 * EXACT_SPLIT_CAP * PW_UNITS * ((nmax + PW_BUF - 1) / PW_BUF));
  w.total = o;
  return w;
}

extern "C" {

int64_t hbx_kde_table_floats(int32_t n, int32_t dc_pad, int32_t du_pad) { return table_floats(n, dc_pad, du_pad); }

int hbx_kde_bucket(int32_t dc, int32_t du, int32_t* dc_pad, int32_t* du_pad, int32_t* stride) {
  int a, b;
  bucket_dims(dc, du, &a, &b);
  if (a < 0 || b < 0)
    return hbx_fail(HBX_ERR_UNSUPPORTED, "no scoring kernel for %d continuous / %d categorical dims "
                    "(max 64 / 32)", dc, du);
  *dc_pad = a;
  *du_pad = b;
  *stride = table_stride(a, b);
  return HBX_OK;
}

int64_t hbx_kde_workspace_bytes(int64_t Nc, int64_t nmax) { return (int64_t)ws_layout(Nc, nmax).total; }

// Build one KDE (good or bad) for scoring.  Host arrays: vartype[D] (0='c', 1='u'), bw[D], nlev[D].
// Device arrays: X[N][D] fp64 (rows of the whole budget), rows[n] int64 (this KDE's rows, in the
// reference's order).  Outputs: params (device, hbx_kde_param_bytes()), table (device fp32,
// hbx_kde_table_floats(n, dc_pad, du_pad) floats), info[8] (host): {has_neg, nan_all, unsupported, dc, du, nconst, dc_pad, du_pad}.
int hbx_kde_prepare(const double* X, int32_t D, const int64_t* rows, int32_t n, const int32_t* vartype,
                    const double* bw, const int32_t* nlev, void* params, float* table, int64_t table_floats_,
                    int32_t* info, void* stream) {
  if (!X || !rows || !vartype || !bw || !nlev || !params || !table || !info)
    return hbx_fail(HBX_ERR_ARG, "hbx_kde_prepare: null pointer");
  if (D < 1 || D > HBX_MAX_D) return hbx_fail(HBX_ERR_UNSUPPORTED, "D=%d outside [1, %d]", D, HBX_MAX_D);
  if (n < 1) return hbx_fail(HBX_ERR_ARG, "hbx_kde_prepare: n=%d", n);
  KdeParams* P = (KdeParams*)calloc(1, sizeof(KdeParams));
  if (!P) return hbx_fail(HBX_ERR_ARG, "out of host memory");
  P->n = n;
  P->D = D;
  int dc_tot = 0, du_tot = 0;
  for (int d = 0; d < D; ++d) (vartype[d] == 0 ? dc_tot : du_tot)++;
  int dcp, dup;
  bucket_dims(dc_tot, du_tot, &dcp, &dup);
  if (dcp < 0 || dup < 0) {
    free(P);
    return hbx_fail(HBX_ERR_UNSUPPORTED, "no scoring kernel for %d continuous / %d categorical dims", dc_tot,
                    du_tot);
  }
  P->dc_pad = dcp;
  P->du_pad = dup;
  P->stride = table_stride(dcp, dup);
  if (table_floats_ < table_floats(n, dcp, dup)) {
    free(P);
    return hbx_fail(HBX_ERR_ARG, "table too small: %lld < %lld floats", (long long)table_floats_,
                    (long long)table_floats(n, dcp, dup));
  }
  const double LOG2E = 1.4426950408889634;
  double sum_ln_h = 0.0, m0 = 0.0, lb_sum = 0.0, prod_bw_c = 1.0;
  float sad = 0.f;
  for (int d = 0; d < D; ++d) {
    const double h = bw[d];
    P->vartype[d] = vartype[d];
    P->nlev[d] = nlev[d];
    P->bw[d] = h;
    if (vartype[d] == 0) {
      const int k = P->dc++;
      P->cont_dim[k] = d;
      prod_bw_c *= h;  // np.prod(bw[iscontinuous]), sequential in dim order
      if (!(h > 0.0)) {
        P->nan_all = 1;  // exp(-0/0) * ... / 0 -> NaN for every candidate
        P->cont_scale[k] = 0.0;
      } else {
        P->cont_scale[k] = sqrt(LOG2E / 2.0) / h;
        sum_ln_h += log(h);
      }
    } else {
      const int c = nlev[d];
      if (c == 1 && h == 0.0) {  // single observed level: match -> 1, mismatch -> 0/0 = NaN
        P->const_dim[P->nconst++] = d;
        continue;
      }
      if (c < 2 || !(h > 0.0) || h != h) {
        P->unsupported = 1;
        continue;
      }
      const double a = 1.0 - h, b = h / (double)(c - 1);
      const double lb = log2(b);
      const double la = (a == 0.0) ? -INFINITY : log2(fabs(a));
      const int u = P->du++;
      P->cat_dim[u] = d;
      m0 += (la > lb) ? la : lb;
      lb_sum += lb;
      if (a == 0.0) {
        P->cat_delta[u] = -1e30f;
      } else {
        P->cat_delta[u] = (float)(la - lb);
        sad += fabsf(P->cat_delta[u]);
      }
      P->cat_negf[u] = (a < 0.0) ? 1.f : 0.f;
      if (a < 0.0) P->has_neg = 1;
    }
  }
  P->m0_log2 = m0;
  P->lb_sum = lb_sum;
  P->prod_bw_c = prod_bw_c;
  P->sum_abs_delta = sad;
  P->log_norm = -log((double)n) - sum_ln_h - 0.5 * (double)P->dc * log(2.0 * M_PI) + m0 * M_LN2;
  P->X = X;
  P->rows = rows;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemcpyAsync(params, P, sizeof(KdeParams), hipMemcpyHostToDevice, s);
  // categorical mode: one-hot on the f16 matrix cores when every active dim has integer codes in
  // [0, 1024) and the one-hot width sum(max code + 1) fits OH_MAX_KC K-steps; else VALU matching
  if (e == hipSuccess && P->du > 0) {
    hipLaunchKernelGGL(kde_maxcode_kernel, dim3(P->du), dim3(256), 0, s, X, D, rows, (KdeParams*)params);
    e = hipGetLastError();
    if (e == hipSuccess)
      e = hipMemcpyAsync(P->cat_maxcode, ((KdeParams*)params)->cat_maxcode, sizeof(int32_t) * HBX_MAX_D,
                         hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
  }
  if (e != hipSuccess) {
    free(P);
    return hbx_fail(HBX_ERR_HIP, "params upload: %s", hipGetErrorString(e));
  }
  P->kc = 0;
  P->oh_total = 0;
  if (P->du > 0) {
    int tot = 0;
    bool ok = true;
    for (int u = 0; u < P->du; ++u) {
      if (P->cat_maxcode[u] < 0) ok = false;
      else tot += P->cat_maxcode[u] + 1;
    }
    if (ok && 2 * tot <= 32 * OH_MAX_KC && tot <= 64) {
      P->kc = (2 * tot + 31) / 32;
      P->oh_total = tot;
      int t = 0;
      for (int u = 0; u < P->du; ++u)
        for (int l = 0; l <= P->cat_maxcode[u]; ++l) {
          P->oh_dim[t] = u;
          P->oh_level[t] = l;
          P->oh_col[t] = P->cat_dim[u];
          P->oh_val[t] = (double)l;
          ++t;
        }
    }
  }
  // continuous product on the f16 matrix cores (hi/lo split) when it has >= 16 dims and the
  // categorical part is one-hot (or absent); otherwise the exact f32 MFMA product
  const char* hm_env = getenv("HBX_HMODE");
  const bool hm_ok = (P->du == 0 || P->kc > 0) && dcp >= 16;
  P->hmode = (hm_ok && !(hm_env && hm_env[0] == '0')) ? 1 : 0;
  P->nsc = nsc_of(dcp);
  if (P->hmode)
    P->chunk_floats = h_chunk_floats(dcp, P->kc, P->has_neg);
  else
    P->chunk_floats = chunk_floats(dcp, dup, P->kc, P->kc ? P->has_neg : 0);
  info[0] = P->has_neg | (P->kc << 1) | (P->hmode << 4);  // scoring variant (hbx_kde_logpdf / _acquire)
  info[1] = P->nan_all;
  info[2] = P->unsupported;
  info[3] = P->dc;
  info[4] = P->du;
  info[5] = P->nconst;
  info[6] = P->dc_pad;
  info[7] = P->du_pad;
  e = hipMemcpyAsync(params, P, sizeof(KdeParams), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  const int dc_n = P->dc;
  free(P);
  if (e != hipSuccess) return hbx_fail(HBX_ERR_HIP, "params upload: %s", hipGetErrorString(e));
  if (dc_n > 0) {
    hipLaunchKernelGGL(kde_center_kernel, dim3(dc_n), dim3(256), 0, s, X, D, rows, (KdeParams*)params);
    HBX_LAUNCH_CHECK();
  }
  const int nslots = ((n + OBS_CHUNK - 1) / OBS_CHUNK) * OBS_CHUNK;
  hipLaunchKernelGGL(kde_table_kernel, dim3((nslots + 255) / 256), dim3(256), 0, s, X, D, rows,
                     (KdeParams*)params, table);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

// fp32 log-domain scoring of Nc candidates (fp64 [Nc][D] row-major) against one prepared KDE
int hbx_kde_logpdf(const double* cand, int64_t Nc, int32_t D, const void* params, const float* table,
                   int32_t dc_pad, int32_t du_pad, int32_t variant, void* est_out, void* stream) {
  if ((!cand || !est_out) && Nc > 0) return hbx_fail(HBX_ERR_ARG, "hbx_kde_logpdf: null pointer");
  if (!params || !table) return hbx_fail(HBX_ERR_ARG, "hbx_kde_logpdf: null pointer");
  if (Nc <= 0) return HBX_OK;
  ScoreFns f = pick_logpdf(dc_pad, du_pad, variant);
  if (!f.main) return hbx_fail(HBX_ERR_UNSUPPORTED, "no kernel for dc_pad=%d du_pad=%d", dc_pad, du_pad);
  return launch_score(f, cand, Nc, D, params, table, (KdeEst*)est_out, (hipStream_t)stream);
}

// One acquisition: score every candidate against l (good) and g (bad), shortlist, exact re-score,
// argmin.  index_base offsets the reported index (candidate sharding across GPUs).  The result
// (AcqResult) stays in the workspace; hbx_kde_result_ptr() gives its device address.
int hbx_kde_acquire(const double* cand, int64_t Nc, int32_t D, int64_t index_base,
                    const void* params_good, const float* table_good, const double* X_good,
                    const int64_t* rows_good, int32_t variant_good,
                    const void* params_bad, const float* table_bad, const double* X_bad,
                    const int64_t* rows_bad, int32_t variant_bad, int32_t dc_pad, int32_t du_pad,
                    int64_t nmax, float* logl_out, float* logg_out, void* workspace, int64_t ws_bytes,
                    void* events, void* stream) {
  if ((!cand && Nc > 0) || !params_good || !table_good || !X_good || !rows_good || !params_bad || !table_bad ||
      !X_bad || !rows_bad || !workspace)
    return hbx_fail(HBX_ERR_ARG, "hbx_kde_acquire: null pointer");
  if (Nc < 0 || Nc > INT32_MAX) return hbx_fail(HBX_ERR_ARG, "Nc=%lld out of range", (long long)Nc);
  const WsLayout w = ws_layout(Nc, nmax);
  if ((size_t)ws_bytes < w.total)
    return hbx_fail(HBX_ERR_ARG, "workspace too small: %lld < %lld bytes", (long long)ws_bytes,
                    (long long)w.total);
  ScoreFns fg = pick_logpdf(dc_pad, du_pad, variant_good);
  ScoreFns fb = pick_logpdf(dc_pad, du_pad, variant_bad);
  if (!fg.main || !fb.main) return hbx_fail(HBX_ERR_UNSUPPORTED, "no kernel for dc_pad=%d du_pad=%d", dc_pad, du_pad);
  char* ws = (char*)workspace;
  uint32_t* U = (uint32_t*)(ws + w.U);
  int32_t* count = (int32_t*)(ws + w.count);
  int32_t* flags = (int32_t*)(ws + w.flags);
  AcqResult* res = (AcqResult*)(ws + w.res);
  KdeEst* el = (KdeEst*)(ws + w.est_l);
  KdeEst* eg = (KdeEst*)(ws + w.est_g);
  float* lo = (float*)(ws + w.lo);
  float* hi = (float*)(ws + w.hi);
  int32_t* list = (int32_t*)(ws + w.list);
  double* exact_l = (double*)(ws + w.exact_l);
  double* exact_g = (double*)(ws + w.exact_g);
  double* part = (double*)(ws + w.part);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(acq_init_kernel, dim3(1), dim3(64), 0, s, U, count, flags, res);
  HBX_LAUNCH_CHECK();
  if (Nc > 0) {
    const dim3 grid((unsigned)((Nc + 255) / 256));
    hipEvent_t* ev = (hipEvent_t*)events;  // optional: [before l, between, after g] for timing
    if (ev) HBX_HIP(hipEventRecord(ev[0], s));
    int rc = launch_score(fg, cand, Nc, D, params_good, table_good, el, s);
    if (rc) return rc;
    if (ev) HBX_HIP(hipEventRecord(ev[1], s));
    rc = launch_score(fb, cand, Nc, D, params_bad, table_bad, eg, s);
    if (rc) return rc;
    if (ev) HBX_HIP(hipEventRecord(ev[2], s));
    hipLaunchKernelGGL(kde_combine_kernel, grid, dim3(256), 0, s, el, eg, Nc, logl_out, logg_out, lo, hi, U,
                       flags);
    HBX_LAUNCH_CHECK();
    hipLaunchKernelGGL(kde_shortlist_kernel, grid, dim3(256), 0, s, lo, Nc, U, flags, list, count);
    HBX_LAUNCH_CHECK();
    const int nbuf = (int)((nmax + PW_BUF - 1) / PW_BUF);
    hipLaunchKernelGGL(kde_exact_kernel, dim3(EXACT_GRID), dim3(EXACT_THREADS), 0, s, cand, D,
                       (const KdeParams*)params_good, X_good, rows_good, (const KdeParams*)params_bad, X_bad,
                       rows_bad, list, count, nbuf, part, exact_l, exact_g);
    HBX_LAUNCH_CHECK();
    hipLaunchKernelGGL(kde_exact_combine_kernel, dim3((2 * EXACT_SPLIT_CAP + 255) / 256), dim3(256), 0, s,
                       (const KdeParams*)params_good, (const KdeParams*)params_bad, count, nbuf, part, exact_l,
                       exact_g);
    HBX_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(kde_final_kernel, dim3(1), dim3(256), 0, s, list, count, exact_l, exact_g, flags,
                     index_base, res);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}


// the exact pdf stages its per-observation terms in LDS: no global scratch is needed any more (the
// entry point keeps its scratch argument; 256 bytes keep callers' allocations non-empty)
int64_t hbx_kde_pdf_scratch_bytes(int64_t nmax) { return 256; }

// Exact fp64 pdf (reference arithmetic and operation order) of one prepared KDE at Np points
// (device fp64 [Np][D]) -> out (device fp64 [Np]).  KDEMultivariate.pdf as a batched GPU call.
int hbx_kde_pdf_exact(const double* pts, int64_t Np, int32_t D, const void* params, const double* X,
                      const int64_t* rows, int64_t n, double* out, void* scratch, int64_t scratch_bytes,
                      void* stream) {
  if (!pts || !params || !X || !rows || !out || !scratch) return hbx_fail(HBX_ERR_ARG, "hbx_kde_pdf_exact: null");
  if (scratch_bytes < hbx_kde_pdf_scratch_bytes(n)) return hbx_fail(HBX_ERR_ARG, "pdf scratch too small");
  if (Np <= 0) return HBX_OK;
  const unsigned grid = (unsigned)(Np < EXACT_GRID ? Np : EXACT_GRID);
  hipLaunchKernelGGL(kde_pdf_exact_kernel, dim3(grid), dim3(EXACT_THREADS), 0, (hipStream_t)stream, pts, Np, D,
                     (const KdeParams*)params, X, rows, out);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

// Timing events (hipEvent_t) for hbx_kde_acquire's `events` argument.
int hbx_event_create(void** ev) {
  HBX_HIP(hipEventCreate((hipEvent_t*)ev));
  return HBX_OK;
}
int hbx_event_destroy(void* ev) {
  HBX_HIP(hipEventDestroy((hipEvent_t)ev));
  return HBX_OK;
}
int hbx_event_elapsed_ms(void* start, void* stop, float* ms) {
  HBX_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
  return HBX_OK;
}

void* hbx_kde_result_ptr(void* workspace) { return (char*)workspace + ws_layout(0, 0).res; }

}  // extern "C"
