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
#define EXACT_GRID 128
#define SUM_BLOCK 32
#define LDS_ROWS 128  // observation rows per LDS chunk of the scoring kernel

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

static int table_stride(int dc_pad, int du_pad) { return (1 + dc_pad + du_pad + 3) & ~3; }

// Per continuous slot: mean of the KDE's data column (centre of the scaled coordinates).
__global__ void kde_center_kernel(const double* __restrict__ X, int32_t D, const int64_t* __restrict__ rows,
                                  KdeParams* __restrict__ P) {
  for (int k = threadIdx.x; k < P->dc; k += blockDim.x) {
    const int d = P->cont_dim[k];
    double acc = 0.0;
    for (int j = 0; j < P->n; ++j) acc += X[rows[j] * (int64_t)D + d];
    const double m = acc / (double)P->n;
    P->center[k] = (m == m && m - m == 0.0) ? m : 0.0;
  }
}

// Fill the per-observation fp32 table: [C_j, X'_1..X'_dcpad, code_1..code_dupad, pad].
// C_j = -sum_c X'_jc^2 + lb_sum - M0  (log2 units), X'_jc = s_c * (X_jc - mu_c).
__global__ __launch_bounds__(256) void kde_table_kernel(const double* __restrict__ X, int32_t D,
                                                        const int64_t* __restrict__ rows,
                                                        KdeParams* __restrict__ P,
                                                        float* __restrict__ table) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = P->n;
  const bool ok = j < n;
  const double* x = X + (ok ? rows[j] : rows[0]) * (int64_t)D;
  float* row = table + (int64_t)(ok ? j : 0) * P->stride;
  const int dc = P->dc, du = P->du, dcp = P->dc_pad, dup = P->du_pad;
  double C = 0.0;
  for (int k = 0; k < dcp; ++k) {
    float v = 0.f;
    if (k < dc) v = (float)(P->cont_scale[k] * (x[P->cont_dim[k]] - P->center[k]));
    C -= (double)v * (double)v;
    if (ok) row[1 + k] = v;
    float a = ok ? fabsf(v) : 0.f;
    for (int o = 32; o > 0; o >>= 1) a = fmaxf(a, __shfl_xor(a, o));
    if ((threadIdx.x & 63) == 0 && k < dc) atomicMax((unsigned int*)&P->xmax[k], __float_as_uint(a));
  }
  for (int u = 0; u < dup; ++u) {
    float v = (u < du) ? (float)x[P->cat_dim[u]] : -2.0f;
    if (ok) row[1 + dcp + u] = v;
  }
  for (int p = 1 + dcp + dup; p < P->stride; ++p)
    if (ok) row[p] = 0.f;
  C += P->lb_sum - P->m0_log2;
  const float Cf = (float)C;
  if (ok) row[0] = Cf;
  float a = ok ? fabsf(Cf) : 0.f;
  for (int o = 32; o > 0; o >>= 1) a = fmaxf(a, __shfl_xor(a, o));
  if ((threadIdx.x & 63) == 0) atomicMax((unsigned int*)&P->cmax, __float_as_uint(a));
  if (j == 0)
    for (int q = 0; q < P->nconst; ++q) P->const_level[q] = x[P->const_dim[q]];
}

// ------------------------------------------------------------------------------------------
// fp32 log-domain scoring: CPT candidates per lane, all observations of one KDE
//
// Per (candidate i, observation j), in log2 units and minus the static bound M0:
//   t_ij = c_i + C_j + sum_c x''_ic X'_jc + sum_u delta_u [x_iu == X_ju]
// with X' = s (X - mu), x'' = 2 s (x - mu), c_i = -|x'_i|^2, C_j = -|X'_j|^2 + lb_sum - M0
// (the expansion of -|x' - X'|^2: one FMA per continuous dim).  The observation row is wave-uniform
// and arrives through scalar loads (s_load_dwordx16) as SGPR operands of the FMAs.  Each lane keeps
// CPT candidates in registers: CPT independent dependency chains per observation, and every scalar
// load is amortised over CPT*64 candidates.  The categorical match uses m = clamp(1 - d*d) on the
// integer codes (d = x - X), which stays in the VALU (no VCC round trip).

__device__ __forceinline__ float cat_match(float a, float b) {
  const float d = a - b;
  return __builtin_amdgcn_fmed3f(fmaf(-d, d, 1.f), 0.f, 1.f);
}

template <int DCP, int DUP, bool SIGNED, int CPT>
__global__ __launch_bounds__(256) void kde_logpdf_kernel(const double* __restrict__ cand, int64_t Nc,
                                                         int32_t D, const KdeParams* __restrict__ P,
                                                         const float* __restrict__ table,
                                                         KdeEst* __restrict__ out) {
  constexpr int STRIDE = (1 + DCP + DUP + 3) & ~3;
  constexpr int NC = DCP > 0 ? DCP : 1;
  constexpr int NU = DUP > 0 ? DUP : 1;
  const int n = P->n;
  const int dc = P->dc, du = P->du;

  int64_t idx[CPT];
  bool valid[CPT], nan_c[CPT];
  float xs[CPT][NC], xu[CPT][NU], ci[CPT], bnd[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    idx[c] = (int64_t)blockIdx.x * (256 * CPT) + c * 256 + threadIdx.x;
    valid[c] = idx[c] < Nc;
    const double* x = cand + (valid[c] ? idx[c] : (Nc - 1)) * (int64_t)D;
    ci[c] = 0.f;
    bnd[c] = 0.f;
#pragma unroll
    for (int k = 0; k < DCP; ++k) {
      float v = 0.f;
      if (k < dc) v = (float)(P->cont_scale[k] * (x[P->cont_dim[k]] - P->center[k]));
      ci[c] = fmaf(-v, v, ci[c]);
      xs[c][k] = 2.f * v;
      if (k < dc) bnd[c] = fmaf(fabsf(xs[c][k]), P->xmax[k], bnd[c]);
    }
#pragma unroll
    for (int u = 0; u < DUP; ++u) {
      float v = -1.f;
      if (u < du) {
        const double xv = x[P->cat_dim[u]];
        // codes are integers; anything else (incl. NaN) never equals an observed code
        v = (xv == rint(xv) && fabs(xv) < 1e6) ? (float)xv : -1e9f;
      }
      xu[c][u] = v;
    }
    nan_c[c] = P->nan_all != 0;
    for (int q = 0; q < P->nconst; ++q)
      if (x[P->const_dim[q]] != P->const_level[q]) nan_c[c] = true;
  }
  float dl[NU], ng[NU];
#pragma unroll
  for (int u = 0; u < DUP; ++u) {
    dl[u] = (u < du) ? P->cat_delta[u] : 0.f;
    ng[u] = (u < du) ? P->cat_negf[u] : 0.f;
  }

  // t (log2 units, minus M0) of candidate slot c against observation row r; q = parity of
  // matches in dims whose Aitchison-Aitken match weight 1-h is negative
  auto pair_t = [&](const float* __restrict__ r, int c, float& q) -> float {
    float t = ci[c] + r[0];
#pragma unroll
    for (int k = 0; k < DCP; ++k) t = fmaf(xs[c][k], r[1 + k], t);
    q = 0.f;
#pragma unroll
    for (int u = 0; u < DUP; ++u) {
      const float m = cat_match(xu[c][u], r[1 + DCP + u]);
      t = fmaf(dl[u], m, t);
      if (SIGNED) q = fmaf(m, ng[u], -fabsf(q));
    }
    return t;
  };

  float S[CPT], Sn[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) S[c] = Sn[c] = 0.f;
  // observation rows are staged through LDS, LDS_ROWS at a time (whole block, 16-B loads), and
  // read back as wave-wide broadcasts; the sum over one chunk is a partial sum (blocked summation)
  __shared__ __align__(16) float rows_lds[LDS_ROWS * STRIDE];
  for (int j0 = 0; j0 < n; j0 += LDS_ROWS) {
    const int nr = min(LDS_ROWS, n - j0);
    {
      const float4* __restrict__ src = (const float4*)(table + (int64_t)j0 * STRIDE);
      float4* dst = (float4*)rows_lds;
      for (int q = threadIdx.x; q < nr * (STRIDE / 4); q += 256) dst[q] = src[q];
    }
    __syncthreads();
    float Sb[CPT], Snb[CPT];
#pragma unroll
    for (int c = 0; c < CPT; ++c) Sb[c] = Snb[c] = 0.f;
#pragma unroll 2
    for (int j = 0; j < nr; ++j) {
      float r[STRIDE];
      const float4* rp = (const float4*)(rows_lds + j * STRIDE);
#pragma unroll
      for (int q = 0; q < STRIDE / 4; ++q) {
        const float4 v = rp[q];
        r[4 * q] = v.x;
        r[4 * q + 1] = v.y;
        r[4 * q + 2] = v.z;
        r[4 * q + 3] = v.w;
      }
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        float q;
        const float t = pair_t(r, c, q);
        const float e = __builtin_amdgcn_exp2f(t);
        Sb[c] += e;
        if (SIGNED) Snb[c] = fmaf(fabsf(q), e, Snb[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      S[c] += Sb[c];
      if (SIGNED) Sn[c] += Snb[c];
    }
    __syncthreads();
  }

  // rescue: every term sits far below the static bound -> two-pass (max, then sum) for that slot
  float off[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    off[c] = 0.f;
    const bool need = valid[c] && !nan_c[c] && (S[c] < 0x1p-64f);
    if (__any(need)) {
      if (need) {
        float mx = -INFINITY, q;
        for (int j = 0; j < n; ++j) mx = fmaxf(mx, pair_t(table + (int64_t)j * STRIDE, c, q));
        float s = 0.f, sn = 0.f;
        if (mx > -INFINITY) {
          for (int jb = 0; jb < n; jb += SUM_BLOCK) {
            const int je = min(jb + SUM_BLOCK, n);
            float Sb = 0.f, Snb = 0.f;
            for (int j = jb; j < je; ++j) {
              const float t = pair_t(table + (int64_t)j * STRIDE, c, q);
              const float e = __builtin_amdgcn_exp2f(t - mx);
              Sb += e;
              if (SIGNED) Snb = fmaf(fabsf(q), e, Snb);
            }
            s += Sb;
            if (SIGNED) sn += Snb;
          }
          off[c] = mx;
        }
        S[c] = s;
        Sn[c] = sn;
      }
    }
  }

  const float lnorm = (float)P->log_norm;
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    if (!valid[c]) continue;
    KdeEst o;
    if (nan_c[c] || S[c] != S[c]) {
      o.lpos = NAN;
      o.lneg = -INFINITY;
      o.err = 0.f;
    } else {
      const float Sp = SIGNED ? (S[c] - Sn[c]) : S[c];
      o.lpos = (Sp > 0.f) ? (__log2f(Sp) + off[c]) * HBX_LN2f + lnorm : -INFINITY;
      o.lneg = (SIGNED && Sn[c] > 0.f) ? (__log2f(Sn[c]) + off[c]) * HBX_LN2f + lnorm : -INFINITY;
      const float u = 0x1p-24f;
      const float Mabs = fabsf(ci[c]) + P->cmax + bnd[c] + P->sum_abs_delta;
      const float dt = 3.f * (float)(dc + du + 4) * u * Mabs;  // |error of t|, log2 units
      const float es = ((float)LDS_ROWS + (float)n / (float)LDS_ROWS + 8.f) * u * (SIGNED ? 3.f : 1.f);
      o.err = 2.f * (dt * HBX_LN2f + es) + 16.f * u;
    }
    o.pad = 0.f;
    out[idx[c]] = o;
  }
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

// numpy's pairwise summation (umath loops: n < 8 plain, <= 128 eight accumulators, else split).
// dens.sum(axis=0) (SM:_kernel_base.py:516) runs it over the ufunc buffer chunks of 8192 elements,
// accumulated left to right from 0.0 -- see np_sum below.
__device__ double np_pairwise_sum(const double* a, int64_t n) {
  // explicit stack instead of recursion: (offset, len, state)
  struct Fr { int64_t off, len; double left; int st; };
  Fr stk[48];
  int sp = 0;
  stk[0] = {0, n, 0.0, 0};
  double ret = 0.0;
  while (sp >= 0) {
    Fr& f = stk[sp];
    if (f.len <= 128) {
      double res;
      const double* p = a + f.off;
      if (f.len < 8) {
        res = 0.0;
        for (int64_t i = 0; i < f.len; ++i) res += p[i];
      } else {
        double r0 = p[0], r1 = p[1], r2 = p[2], r3 = p[3], r4 = p[4], r5 = p[5], r6 = p[6], r7 = p[7];
        int64_t i;
        for (i = 8; i < f.len - (f.len % 8); i += 8) {
          r0 += p[i + 0]; r1 += p[i + 1]; r2 += p[i + 2]; r3 += p[i + 3];
          r4 += p[i + 4]; r5 += p[i + 5]; r6 += p[i + 6]; r7 += p[i + 7];
        }
        res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
        for (; i < f.len; ++i) res += p[i];
      }
      ret = res;
      --sp;
      // propagate into parent frames
      while (sp >= 0) {
        Fr& pf = stk[sp];
        if (pf.st == 1) {  // left child finished -> start right child
          pf.left = ret;
          pf.st = 2;
          int64_t n2 = pf.len / 2;
          n2 -= n2 % 8;
          stk[++sp] = {pf.off + n2, pf.len - n2, 0.0, 0};
          break;
        } else {  // st == 2: right child finished
          ret = pf.left + ret;
          --sp;
        }
      }
    } else {
      int64_t n2 = f.len / 2;
      n2 -= n2 % 8;
      f.st = 1;
      const int64_t off = f.off;
      stk[++sp] = {off, n2, 0.0, 0};
    }
  }
  return ret;
}

// exact fp64 pdf of one KDE at x (reference arithmetic); dens = scratch[n]; called by a whole block
__device__ double exact_pdf(const double* __restrict__ X, int32_t D, const int64_t* __restrict__ rows,
                            const KdeParams* __restrict__ P, const double* __restrict__ x,
                            double* __restrict__ dens, double* __restrict__ sh) {
  const int n = P->n;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    const double* xr = X + rows[j] * (int64_t)D;
    double p = 1.0;
    for (int d = 0; d < D; ++d) {
      const double h = P->bw[d];
      double k;
      if (P->vartype[d] == 0) {
        const double diff = xr[d] - x[d];
        k = HBX_INV_SQRT_2PI * exp(-(diff * diff) / ((h * h) * 2.));
      } else {
        k = (xr[d] == x[d]) ? (1. - h) : (h / (double)(P->nlev[d] - 1));
      }
      p = (d == 0) ? k : p * k;
    }
    dens[j] = p / P->prod_bw_c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double acc = 0.0;  // np.add.reduce: identity 0.0, then one pairwise sum per 8192-element buffer
    for (int64_t c = 0; c < n; c += 8192) acc = acc + np_pairwise_sum(dens + c, (n - c) < 8192 ? (n - c) : 8192);
    *sh = acc / (double)n;
  }
  __syncthreads();
  const double r = *sh;
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void kde_exact_kernel(
    const double* __restrict__ cand, int32_t D, int64_t index_base,
    const KdeParams* __restrict__ Pg, const double* __restrict__ Xg, const int64_t* __restrict__ rows_g,
    const KdeParams* __restrict__ Pb, const double* __restrict__ Xb, const int64_t* __restrict__ rows_b,
    const int32_t* __restrict__ list, const int32_t* __restrict__ count, double* __restrict__ exact,
    double* __restrict__ exact_l, double* __restrict__ exact_g, double* __restrict__ scratch, int64_t nmax) {
  __shared__ double sh;
  const int cnt = *count;
  double* dens = scratch + (int64_t)blockIdx.x * nmax;
  for (int p = blockIdx.x; p < cnt; p += gridDim.x) {
    const double* x = cand + (int64_t)list[p] * D;
    const double g = exact_pdf(Xb, D, rows_b, Pb, x, dens, &sh);
    const double l = exact_pdf(Xg, D, rows_g, Pg, x, dens, &sh);
    if (threadIdx.x == 0) {
      // bohb.py:129 with Python max(): max(1e-8, g) keeps 1e-8 unless g > 1e-8 (NaN -> 1e-8);
      // max(l, 1e-8) keeps l unless 1e-8 > l (NaN -> NaN)
      const double G = (g > 1e-8) ? g : 1e-8;
      const double L = (1e-8 > l) ? 1e-8 : l;
      exact[p] = G / L;
      exact_l[p] = l;
      exact_g[p] = g;
    }
  }
}


// exact fp64 pdf of one KDE at every row of pts (grid-stride over points, one block per point)
__global__ __launch_bounds__(256) void kde_pdf_exact_kernel(const double* __restrict__ pts, int64_t Np, int32_t D,
                                                            const KdeParams* __restrict__ P,
                                                            const double* __restrict__ X,
                                                            const int64_t* __restrict__ rows,
                                                            double* __restrict__ out, double* __restrict__ scratch,
                                                            int64_t nmax) {
  __shared__ double sh;
  double* dens = scratch + (int64_t)blockIdx.x * nmax;
  for (int64_t p = blockIdx.x; p < Np; p += gridDim.x) {
    const double v = exact_pdf(X, D, rows, P, pts + p * D, dens, &sh);
    if (threadIdx.x == 0) out[p] = v;
  }
}

__global__ __launch_bounds__(256) void kde_final_kernel(const int32_t* __restrict__ list,
                                                        const int32_t* __restrict__ count,
                                                        const double* __restrict__ exact,
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
    const double s = exact[p];
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

#define LOGPDF_CPT 2  // candidates per lane
template <int DCP, int DUP>
static logpdf_fn pick_signed(bool sgn) {
  return sgn ? kde_logpdf_kernel<DCP, DUP, true, LOGPDF_CPT> : kde_logpdf_kernel<DCP, DUP, false, LOGPDF_CPT>;
}

template <int DCP>
static logpdf_fn pick_du(int du_pad, bool sgn) {
  switch (du_pad) {
    case 0: return pick_signed<DCP, 0>(sgn);
    case 4: return pick_signed<DCP, 4>(sgn);
    case 8: return pick_signed<DCP, 8>(sgn);
    case 16: return pick_signed<DCP, 16>(sgn);
    case 32: return pick_signed<DCP, 32>(sgn);
  }
  return nullptr;
}

static logpdf_fn pick_logpdf(int dc_pad, int du_pad, bool sgn) {
  switch (dc_pad) {
    case 0: return pick_du<0>(du_pad, sgn);
    case 4: return pick_du<4>(du_pad, sgn);
    case 8: return pick_du<8>(du_pad, sgn);
    case 16: return pick_du<16>(du_pad, sgn);
    case 24: return pick_du<24>(du_pad, sgn);
    case 32: return pick_du<32>(du_pad, sgn);
    case 64: return pick_du<64>(du_pad, sgn);
  }
  return nullptr;
}

// workspace layout (bytes), shared by hbx_kde_workspace_bytes and hbx_kde_acquire
struct WsLayout {
  size_t U, count, flags, res, est_l, est_g, lo, hi, list, exact, exact_l, exact_g, scratch, total;
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
  w.exact = take(8 * Nc);
  w.exact_l = take(8 * Nc);
  w.exact_g = take(8 * Nc);
  w.scratch = take(8 * (size_t)EXACT_GRID * nmax);
  w.total = o;
  return w;
}

extern "C" {

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
// n * stride floats), info[8] (host): {has_neg, nan_all, unsupported, dc, du, nconst, dc_pad, du_pad}.
int hbx_kde_prepare(const double* X, int32_t D, const int64_t* rows, int32_t n, const int32_t* vartype,
                    const double* bw, const int32_t* nlev, void* params, float* table, int64_t table_floats,
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
  if (table_floats < (int64_t)n * P->stride) {
    free(P);
    return hbx_fail(HBX_ERR_ARG, "table too small: %lld < %lld floats", (long long)table_floats,
                    (long long)n * P->stride);
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
  info[0] = P->has_neg;
  info[1] = P->nan_all;
  info[2] = P->unsupported;
  info[3] = P->dc;
  info[4] = P->du;
  info[5] = P->nconst;
  info[6] = P->dc_pad;
  info[7] = P->du_pad;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemcpyAsync(params, P, sizeof(KdeParams), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  free(P);
  if (e != hipSuccess) return hbx_fail(HBX_ERR_HIP, "params upload: %s", hipGetErrorString(e));
  hipLaunchKernelGGL(kde_center_kernel, dim3(1), dim3(256), 0, s, X, D, rows, (KdeParams*)params);
  HBX_LAUNCH_CHECK();
  hipLaunchKernelGGL(kde_table_kernel, dim3((n + 255) / 256), dim3(256), 0, s, X, D, rows, (KdeParams*)params,
                     table);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

// fp32 log-domain scoring of Nc candidates (fp64 [Nc][D] row-major) against one prepared KDE
int hbx_kde_logpdf(const double* cand, int64_t Nc, int32_t D, const void* params, const float* table,
                   int32_t dc_pad, int32_t du_pad, int32_t signed_sum, void* est_out, void* stream) {
  if ((!cand || !est_out) && Nc > 0) return hbx_fail(HBX_ERR_ARG, "hbx_kde_logpdf: null pointer");
  if (!params || !table) return hbx_fail(HBX_ERR_ARG, "hbx_kde_logpdf: null pointer");
  if (Nc <= 0) return HBX_OK;
  logpdf_fn f = pick_logpdf(dc_pad, du_pad, signed_sum != 0);
  if (!f) return hbx_fail(HBX_ERR_UNSUPPORTED, "no kernel for dc_pad=%d du_pad=%d", dc_pad, du_pad);
  hipLaunchKernelGGL(f, dim3((unsigned)((Nc + 256 * LOGPDF_CPT - 1) / (256 * LOGPDF_CPT))), dim3(256), 0,
                     (hipStream_t)stream, cand, Nc, D,
                     (const KdeParams*)params, table, (KdeEst*)est_out);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

// One acquisition: score every candidate against l (good) and g (bad), shortlist, exact re-score,
// argmin.  index_base offsets the reported index (candidate sharding across GPUs).  The result
// (AcqResult) stays in the workspace; hbx_kde_result_ptr() gives its device address.
int hbx_kde_acquire(const double* cand, int64_t Nc, int32_t D, int64_t index_base,
                    const void* params_good, const float* table_good, const double* X_good,
                    const int64_t* rows_good, int32_t signed_good,
                    const void* params_bad, const float* table_bad, const double* X_bad,
                    const int64_t* rows_bad, int32_t signed_bad, int32_t dc_pad, int32_t du_pad,
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
  logpdf_fn fg = pick_logpdf(dc_pad, du_pad, signed_good != 0);
  logpdf_fn fb = pick_logpdf(dc_pad, du_pad, signed_bad != 0);
  if (!fg || !fb) return hbx_fail(HBX_ERR_UNSUPPORTED, "no kernel for dc_pad=%d du_pad=%d", dc_pad, du_pad);
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
  double* exact = (double*)(ws + w.exact);
  double* exact_l = (double*)(ws + w.exact_l);
  double* exact_g = (double*)(ws + w.exact_g);
  double* scratch = (double*)(ws + w.scratch);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(acq_init_kernel, dim3(1), dim3(64), 0, s, U, count, flags, res);
  HBX_LAUNCH_CHECK();
  if (Nc > 0) {
    const dim3 grid((unsigned)((Nc + 255) / 256));
    const dim3 grid_s((unsigned)((Nc + 256 * LOGPDF_CPT - 1) / (256 * LOGPDF_CPT)));
    hipEvent_t* ev = (hipEvent_t*)events;  // optional: [before l, between, after g] for timing
    if (ev) HBX_HIP(hipEventRecord(ev[0], s));
    hipLaunchKernelGGL(fg, grid_s, dim3(256), 0, s, cand, Nc, D, (const KdeParams*)params_good, table_good, el);
    HBX_LAUNCH_CHECK();
    if (ev) HBX_HIP(hipEventRecord(ev[1], s));
    hipLaunchKernelGGL(fb, grid_s, dim3(256), 0, s, cand, Nc, D, (const KdeParams*)params_bad, table_bad, eg);
    HBX_LAUNCH_CHECK();
    if (ev) HBX_HIP(hipEventRecord(ev[2], s));
    hipLaunchKernelGGL(kde_combine_kernel, grid, dim3(256), 0, s, el, eg, Nc, logl_out, logg_out, lo, hi, U,
                       flags);
    HBX_LAUNCH_CHECK();
    hipLaunchKernelGGL(kde_shortlist_kernel, grid, dim3(256), 0, s, lo, Nc, U, flags, list, count);
    HBX_LAUNCH_CHECK();
    hipLaunchKernelGGL(kde_exact_kernel, dim3(EXACT_GRID), dim3(256), 0, s, cand, D, index_base,
                       (const KdeParams*)params_good, X_good, rows_good, (const KdeParams*)params_bad, X_bad,
                       rows_bad, list, count, exact, exact_l, exact_g, scratch, nmax);
    HBX_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(kde_final_kernel, dim3(1), dim3(256), 0, s, list, count, exact, exact_l, exact_g, flags,
                     index_base, res);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}


int64_t hbx_kde_pdf_scratch_bytes(int64_t nmax) { return (int64_t)(8 * (size_t)EXACT_GRID * nmax); }

// Exact fp64 pdf (reference arithmetic and operation order) of one prepared KDE at Np points
// (device fp64 [Np][D]) -> out (device fp64 [Np]).  KDEMultivariate.pdf as a batched GPU call.
int hbx_kde_pdf_exact(const double* pts, int64_t Np, int32_t D, const void* params, const double* X,
                      const int64_t* rows, int64_t n, double* out, void* scratch, int64_t scratch_bytes,
                      void* stream) {
  if (!pts || !params || !X || !rows || !out || !scratch) return hbx_fail(HBX_ERR_ARG, "hbx_kde_pdf_exact: null");
  if (scratch_bytes < hbx_kde_pdf_scratch_bytes(n)) return hbx_fail(HBX_ERR_ARG, "pdf scratch too small");
  if (Np <= 0) return HBX_OK;
  const unsigned grid = (unsigned)(Np < EXACT_GRID ? Np : EXACT_GRID);
  hipLaunchKernelGGL(kde_pdf_exact_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, pts, Np, D,
                     (const KdeParams*)params, X, rows, out, (double*)scratch, n);
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
