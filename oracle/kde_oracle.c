/* ORACLE -- test infrastructure only.
 *
 * Plain-C fp64 restatement of the reference KDE arithmetic, used as (a) a second checker in
 * tests/ and (b) the `cpu_baseline` leg of bench.py (OpenMP over candidates on the host cores).
 * Never linked into, loaded by or called from the engine (hpbandster_amd/).
 *
 * Follows, per (candidate, observation) pair:
 *   gaussian          statsmodels 0.12.2 nonparametric/kernels.py:108-125
 *                     (1/sqrt(2*pi)) * exp(-(Xi - x)**2 / (h**2 * 2.))
 *   aitchison_aitken  kernels.py:23-65: 1 - h if Xi == x else h / (num_levels - 1)
 *   gpke              _kernel_base.py:509-516: prod over dims / prod(bw[continuous]), sum over obs
 *   pdf               kernel_density.py:190-193: gpke / nobs
 *   minimize_me       hpbandster bohb.py:129 max(1e-8, g) / max(l, 1e-8) (Python max semantics)
 *   argmin            bohb.py:149-152 strict '<' against best = +inf (first index wins)
 * Two modes.  exact = 1: the reference's float64 arithmetic bit for bit -- numpy's exp as the pinned
 * numpy 1.26.4 evaluates it and numpy's pairwise summation (np_arith.h) -- the checker.  exact = 0:
 * libm exp and a sequential sum (values agree to rounding, ~1e-15 relative), the fast CPU baseline.
 *
 * Build: oracle/Makefile (gcc -O3 -fopenmp -shared) -> oracle/_build/libkde_oracle.so.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "np_arith.h"

static const double INV_SQRT_2PI = 0.3989422804014327; /* 1. / np.sqrt(2 * np.pi) */

/* pdf of one KDE (data [n][D]) at Np points (pts [Np][D]) -> out[Np].  vartype: 0 = 'c', 1 = 'u'. */
void oracle_kde_pdf_mode(const double* data, int64_t n, int32_t D, const int32_t* vartype, const double* bw,
                         const int32_t* nlev, const double* pts, int64_t Np, double* out, int32_t nthreads,
                         int32_t exact) {
  double prod_bw_c = 1.0;
  for (int d = 0; d < D; ++d)
    if (vartype[d] == 0) prod_bw_c *= bw[d];
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
  {
    double* dens = exact ? (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1)) : 0;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
    for (int64_t p = 0; p < Np; ++p) {
      const double* x = pts + p * D;
      double acc = 0.0;
      for (int64_t j = 0; j < n; ++j) {
        const double* xr = data + j * D;
        double prod = 1.0;
        for (int d = 0; d < D; ++d) {
          const double h = bw[d];
          double k;
          if (vartype[d] == 0) {
            const double diff = xr[d] - x[d];
            const double a = -(diff * diff) / ((h * h) * 2.);
            k = INV_SQRT_2PI * (exact ? np_exp(a) : exp(a));
          } else {
            k = (xr[d] == x[d]) ? (1. - h) : (h / (double)(nlev[d] - 1));
          }
          prod = (d == 0) ? k : prod * k;
        }
        if (exact) dens[j] = prod / prod_bw_c;
        else acc += prod / prod_bw_c;
      }
      if (exact) acc = np_sum(dens, n);
      out[p] = acc / (double)n;
    }
    free(dens);
  }
}

void oracle_kde_pdf(const double* data, int64_t n, int32_t D, const int32_t* vartype, const double* bw,
                    const int32_t* nlev, const double* pts, int64_t Np, double* out, int32_t nthreads) {
  oracle_kde_pdf_mode(data, n, D, vartype, bw, nlev, pts, Np, out, nthreads, 0);
}

/* Screening pdf for the full-size winner scans (tests/golden/gen_full_winners.py): the same density
 * with the continuous kernels' exponents summed first and ONE libm exp per pair,
 *   term_j = exp(sum_c a_jd) * INV_SQRT_2PI^Dc * prod_u k_jd / prod_bw_c,   a_jd as in the exact mode,
 * sequential sum over j.  Against the exact mode every term differs by a relative
 * |sum_c a_jd| * (Dc + 2) * 2^-52 + (D + 4) * 2^-52 at most (rounding of the exponent sum and of the
 * products; 4 ulp allowed per exp), and the sum of same-signed terms keeps the largest term's bound plus the
 * two summation orders' n ulp each; the bound is returned per point in rel_out (nullable).  Only for KDEs whose categorical kernels are all positive
 * (1 - h > 0, h > 0): returns -1 otherwise and writes nothing. */
int32_t oracle_kde_pdf_screen(const double* data, int64_t n, int32_t D, const int32_t* vartype, const double* bw,
                              const int32_t* nlev, const double* pts, int64_t Np, double* out, double* rel_out,
                              int32_t nthreads) {
  int dc = 0, du = 0;
  int cidx[512], uidx[512];
  if (D > 512) return -2;
  double prod_bw_c = 1.0, c_norm = 1.0, inv2h2[512], kmatch[512], kmis[512];
  for (int d = 0; d < D; ++d) {
    if (vartype[d] == 0) {
      prod_bw_c *= bw[d];
      c_norm *= INV_SQRT_2PI;
      inv2h2[dc] = (bw[d] * bw[d]) * 2.;
      cidx[dc++] = d;
    } else {
      if (!(bw[d] > 0.0 && 1. - bw[d] > 0.0) || nlev[d] < 2) return -1;
      kmatch[du] = 1. - bw[d];
      kmis[du] = bw[d] / (double)(nlev[d] - 1);
      uidx[du++] = d;
    }
  }
  const double scale = c_norm / prod_bw_c;
  const double eps = 2.220446049250313e-16;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
  for (int64_t p = 0; p < Np; ++p) {
    const double* x = pts + p * D;
    double acc = 0.0, worst = 0.0;
    for (int64_t j = 0; j < n; ++j) {
      const double* xr = data + j * D;
      double a = 0.0, aa = 0.0;
      for (int k = 0; k < dc; ++k) {
        const double diff = xr[cidx[k]] - x[cidx[k]];
        const double t = -(diff * diff) / inv2h2[k];
        a += t;
        aa -= t;
      }
      double prod = exp(a) * scale;
      for (int k = 0; k < du; ++k) prod *= (xr[uidx[k]] == x[uidx[k]]) ? kmatch[k] : kmis[k];
      acc += prod;
      if (aa > worst) worst = aa;
    }
    out[p] = acc / (double)n;
    /* exponent sum (dc terms) + exp (libm and numpy's, 4 ulp each allowed) + the products (D + 4 roundings)
       + sequential vs pairwise summation (n ulp each) */
    if (rel_out) rel_out[p] = worst * (dc + 2) * eps + 4.0 * (D + 4) * eps + 2.0 * (double)n * eps;
  }
  return 0;
}

/* numpy 1.26.4's exp (SVML), element-wise: for the oracle's own known-answer tests */
void oracle_np_exp(const double* x, int64_t n, double* y) {
  for (int64_t i = 0; i < n; ++i) y[i] = np_exp(x[i]);
}

/* first index of the minimum of max(1e-8, g)/max(l, 1e-8) over finite scores; -1 if none */
int64_t oracle_bohb_select(const double* pdf_l, const double* pdf_g, int64_t Np, double* best_out) {
  double best = INFINITY;
  int64_t bi = -1;
  for (int64_t i = 0; i < Np; ++i) {
    const double g = pdf_g[i], l = pdf_l[i];
    const double G = (g > 1e-8) ? g : 1e-8;  /* max(1e-8, g): NaN -> 1e-8 */
    const double L = (1e-8 > l) ? 1e-8 : l;  /* max(l, 1e-8): NaN -> NaN  */
    const double v = G / L;
    if (v < best) {
      best = v;
      bi = i;
    }
  }
  if (best_out) *best_out = best;
  return bi;
}

int32_t oracle_max_threads(void) {
#ifdef _OPENMP
  return (int32_t)omp_get_max_threads();
#else
  return 1;
#endif
}
