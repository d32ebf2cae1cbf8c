// hbx_cv.hip -- the cross-validation bandwidth objectives of KDEMultivariate:
// least-squares CV (imse, bw='cv_ls') and leave-one-out likelihood (bw='cv_ml'), used by the
// reference's KernelDensityEstimator generator (kde.py:145-147) through statsmodels 0.12.2:
//   imse(bw) = F / n^2 - 2 L / (n (n-1))                      SM:kernel_density.py:246-332
//     F = sum_i F_i, F_i = sum_j prod_d kbar_d(X_jd, X_id) / prod_c bw_c     (convolution kernels)
//     L = sum_i L_i, L_i = sum_{j != i} prod_d k_d(X_jd, X_id) / prod_c bw_c (leave-one-out)
//   loo_likelihood(bw, log) = -sum_i log L_i                   SM:kernel_density.py:126-160
// with kbar = gaussian_convolution / aitchison_aitken_convolution and k = gaussian / aitchison_aitken
// (SM:kernels.py:23-65,108-174).  The two per-observation sums F_i, L_i are O(n D) each: one block per
// observation i computes them in the reference's operation order (per-dim kernel values, product in
// dim order, division by the continuous bandwidth product, numpy's pairwise sum over 8192-element
// buffers); the O(n) sequential sums over i and the Nelder-Mead search stay on the host.
#include <math.h>

#include "hbx_common.h"
#include "hbx_npexp.h"
#include "hbx_pairwise.h"

struct CvShared {
  double dens[PW_UNIT_MAX];
  double nsum[PW_LEVELS][128];
  double usum[PW_UNITS];
  // per dim: 4 h^2 (convolution) and 2 h^2 (kernel) for continuous dims; 1 - h, h / (c - 1) (full
  // column level count) and h / (c_i - 1) (level count without row i) for categorical dims
  double h4[HBX_MAX_D], h2[HBX_MAX_D], a1[HBX_MAX_D], a0[HBX_MAX_D], a0loo[HBX_MAX_D], xi[HBX_MAX_D];
  int32_t cont[HBX_MAX_D];
};

// F-term (convolution kernels) of observation j against observation i
__device__ __forceinline__ double cv_conv_term(const double* __restrict__ xj, int32_t D, const double* __restrict__ lev,
                                               const int32_t* __restrict__ lev_off, double c4, double bwprod,
                                               const CvShared* sh) {
  double p = 1.0;
  for (int d = 0; d < D; ++d) {
    double k;
    if (sh->cont[d]) {
      const double t = xj[d] - sh->xi[d];
      k = c4 * hbx_npexp::exp(-(t * t) / sh->h4[d]);
    } else {
      // sum over the column's levels (ascending order of the negated values, np.unique of -data)
      const double vj = -xj[d], vi = -sh->xi[d];
      double o = 0.0;
      for (int q = lev_off[d]; q < lev_off[d + 1]; ++q) {
        const double x = lev[q];
        o += ((vj == x) ? sh->a1[d] : sh->a0[d]) * ((vi == x) ? sh->a1[d] : sh->a0[d]);
      }
      k = o;
    }
    p = (d == 0) ? k : p * k;
  }
  return p / bwprod;
}

// L-term (kernels, leave-one-out level counts) of observation j != i against observation i
__device__ __forceinline__ double cv_loo_term(const double* __restrict__ xj, int32_t D, double c2, double bwprod,
                                              const CvShared* sh) {
  double p = 1.0;
  for (int d = 0; d < D; ++d) {
    double k;
    if (sh->cont[d]) {
      const double t = xj[d] - sh->xi[d];
      k = c2 * hbx_npexp::exp(-(t * t) / sh->h2[d]);
    } else {
      k = (xj[d] == sh->xi[d]) ? sh->a1[d] : sh->a0loo[d];
    }
    p = (d == 0) ? k : p * k;
  }
  return p / bwprod;
}

// sum over cnt terms in numpy's order (8192-element buffers, pairwise inside); term(k) fills dens
template <typename TERM>
__device__ double cv_np_sum(int cnt, CvShared* sh, TERM term) {
  double acc = 0.0;
  for (int c0 = 0; c0 < cnt; c0 += PW_BUF) {
    const int m = (cnt - c0) < PW_BUF ? (cnt - c0) : PW_BUF;
    for (int u = 0; u < PW_UNITS; ++u) {
      int off, len;
      if (!pw_unit(m, u, &off, &len)) continue;
      for (int k = threadIdx.x; k < len; k += blockDim.x) sh->dens[k] = term(c0 + off + k);
      __syncthreads();
      const double v = np_pairwise_block(sh->dens, len, sh->nsum);
      if (threadIdx.x == 0) sh->usum[u] = v;
      __syncthreads();
    }
    if (threadIdx.x == 0) acc = acc + pw_combine_units(m, sh->usum);
    __syncthreads();
  }
  return acc;  // valid in thread 0
}

__global__ __launch_bounds__(EXACT_THREADS) void kde_cv_kernel(
    const double* __restrict__ X, int64_t n, int32_t D, const int32_t* __restrict__ vartype,
    const double* __restrict__ bw, const double* __restrict__ lev, const int32_t* __restrict__ lev_off,
    const int32_t* __restrict__ loo_levels, double c4, double c2, double bwprod, double* __restrict__ F,
    double* __restrict__ L) {
  __shared__ CvShared sh;
  for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
      const double h = bw[d];
      const bool c = vartype[d] == 0;
      sh.cont[d] = c;
      sh.xi[d] = X[i * D + d];
      sh.h4[d] = (h * h) * 4.;
      sh.h2[d] = (h * h) * 2.;
      sh.a1[d] = 1. - h;
      sh.a0[d] = c ? 0. : h / (double)(lev_off[d + 1] - lev_off[d] - 1);
      sh.a0loo[d] = c ? 0. : h / (double)(loo_levels[i * D + d] - 1);
    }
    __syncthreads();
    if (F) {
      const double v = cv_np_sum((int)n, &sh, [&](int j) {
        return cv_conv_term(X + (int64_t)j * D, D, lev, lev_off, c4, bwprod, &sh);
      });
      if (threadIdx.x == 0) F[i] = v;
    }
    if (L) {
      const double v = cv_np_sum((int)n - 1, &sh, [&](int k) {
        const int64_t j = k < i ? k : k + 1;  // LeaveOneOut: the rows without row i, in order
        return cv_loo_term(X + j * D, D, c2, bwprod, &sh);
      });
      if (threadIdx.x == 0) L[i] = v;
    }
    __syncthreads();
  }
}

extern "C" {

int hbx_kde_cv_terms(const double* X, int64_t n, int32_t D, const int32_t* vartype, const double* bw,
                     const double* lev, const int32_t* lev_off, const int32_t* loo_levels, double c4, double c2,
                     double bwprod, double* F, double* L, void* stream) {
  if (n < 2 || D < 1 || D > HBX_MAX_D || n > INT32_MAX)
    return hbx_fail(HBX_ERR_ARG, "hbx_kde_cv_terms: n=%lld D=%d", (long long)n, D);
  if (!X || !vartype || !bw || !lev || !lev_off || !loo_levels || (!F && !L))
    return hbx_fail(HBX_ERR_ARG, "hbx_kde_cv_terms: null pointer");
  const unsigned grid = (unsigned)(n < 65536 ? n : 65536);
  hipLaunchKernelGGL(kde_cv_kernel, dim3(grid), dim3(EXACT_THREADS), 0, (hipStream_t)stream, X, n, D, vartype, bw,
                     lev, lev_off, loo_levels, c4, c2, bwprod, F, L);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

}  // extern "C"
