// hbx_sample.hip -- BOHB's candidate sampler on the GPU (bohb.py:133-147).
//
// Per candidate i: a good observation idx ~ U{0..n-1} (bohb.py:135), then per dim d of its row m:
//   continuous (levels[d] == 0): truncnorm.rvs(a=-m/bw, b=(1-m)/bw, loc=m, scale=bw_factor*bw)
//     (bohb.py:141).  The bounds are in units of bw while the scale is bw_factor*bw, so the sample
//     lies in [m - bw_factor*m, m + bw_factor*(1-m)] -- the reference's quirk, kept as is;
//   categorical (levels[d] = t): keep m with probability 1 - bw, else U{0..t-1} (bohb.py:143-146).
// The truncated normal is drawn by inversion, z = Phi^-1(p), p = Phi(a) + u (Phi(b) - Phi(a)) (Phi at
// the bounds in fp64; a > 0 is mirrored), Phi^-1 on the smaller tail min(p, 1 - p) in fp32
// (-sqrt(2) erfcinv(2 min(p, 1 - p)): ~1e-7 relative in z, far below what a distributional test can see;
// a branch-free fp32 erfinv polynomial measured 3 % slower in round 5).
// Random numbers: Philox4x32-10 keyed by the seed; counter = (candidate index, word, stream): word w of lane
// g's blocks (w = g + 8 i) gives the uniforms u of the lane's pairs g + 16 i and g + 8 + 16 i (32-bit words,
// u = (w + 1/2) 2^-32).  A categorical dim keeps m when
// u < 1 - h and otherwise takes level floor(t (u - (1 - h)) / h) -- the conditional uniform of the same draw
// (h >= 1: always resampled, level floor(t u)) -- the reference draws from numpy's global RNG, so parity is
// distributional (tests/test_gpu_sample.py).
//
// One lane per (candidate, pair of dims), 4 lanes per candidate (kde_sample_pair_kernel).  Phi at the
// bounds comes from a per-model table when many candidates are drawn (hbx_kde_sample_table).
// hbx_norm_ppf keeps the fp64 inverse normal CDF (Wichura's AS 241) as a library function.
#include <math.h>

#include "hbx_common.h"
#include "hbx_philox.h"
#include <string.h>
#include <stdlib.h>

#define SAMPLE_BLOCK 256
#define DATUM_WORD 0xFFFFFFFFu  // counter word of the per-candidate datum draw (dims use 0..D-1)

__device__ __forceinline__ HbxU32x4 draw(uint64_t seed, uint64_t i, uint32_t word, uint32_t stream) {
  HbxU32x4 c;
  c.x[0] = (uint32_t)i;
  c.x[1] = (uint32_t)(i >> 32);
  c.x[2] = word;
  c.x[3] = stream;
  return hbx_philox4x32_10_impl(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// Standardised bounds of a continuous dim around datum m, mirrored so that lo <= 0 side is used
// (a > 0 -> sample -z from [-b, -a]); false when scipy's a < b check fails.  rh = 1 / h: the bounds are
// within an ulp or two of scipy's -m / h, (1 - m) / h (a distributional difference of nothing), and the
// domain check agrees exactly (h = 0: +-inf, or NaN where m is 0 or 1, as with the divisions).
__device__ __forceinline__ bool tn_bounds(double m, double rh, double* lo, double* hi, bool* flip) {
  const double a = -m * rh, b = (1.0 - m) * rh;
  if (!(a < b)) return false;
  *flip = a > 0.0;
  *lo = *flip ? -b : a;
  *hi = *flip ? -a : b;
  return true;
}

// Phi^-1(p), p in (0, 1), in double precision: Wichura's algorithm AS 241 (PPND16, Applied Statistics
// 37, 1988) -- a 7/7 rational in (0.180625 - (p-0.5)^2) for |p - 0.5| <= 0.425, else in
// sqrt(-log(min(p, 1-p))) on two ranges; relative error ~1e-16 (<= 1.1e-15 against scipy's ndtri over
// 2.4e5 probe points, including 1e-300 and 1 - 1e-10).  One log and one sqrt in the tails, no erfc /
// exp refinement step (the former fp32 guess + fp64 Halley step spent most of the sampler's time in
// ocml's fp64 normcdf and exp).
__device__ __forceinline__ double as241_poly(const double (&c)[8], double x) {
  double r = c[7];
#pragma unroll
  for (int k = 6; k >= 0; --k) r = fma(r, x, c[k]);
  return r;
}

__device__ __forceinline__ double norm_ppf(double p) {
  constexpr double A[8] = {3.3871328727963666080e0, 1.3314166789178437745e+2, 1.9715909503065514427e+3,
                           1.3731693765509461125e+4, 4.5921953931549871457e+4, 6.7265770927008700853e+4,
                           3.3430575583588128105e+4, 2.5090809287301226727e+3};
  constexpr double B[8] = {1.0, 4.2313330701600911252e+1, 6.8718700749205790830e+2, 5.3941960214247511077e+3,
                           2.1213794301586595867e+4, 3.9307895800092710610e+4, 2.8729085735721942674e+4,
                           5.2264952788528545610e+3};
  constexpr double C[8] = {1.42343711074968357734e0, 4.63033784615654529590e0, 5.76949722146069140550e0,
                           3.64784832476320460504e0, 1.27045825245236838258e0, 2.41780725177450611770e-1,
                           2.27238449892691845833e-2, 7.74545014278341407640e-4};
  constexpr double D[8] = {1.0, 2.05319162663775882187e0, 1.67638483018380384940e0, 6.89767334985100004550e-1,
                           1.48103976427480074590e-1, 1.51986665636164571966e-2, 5.47593808499534494600e-4,
                           1.05075007164441684324e-9};
  constexpr double E[8] = {6.65790464350110377720e0, 5.46378491116411436990e0, 1.78482653991729133580e0,
                           2.96560571828504891230e-1, 2.65321895265761230930e-2, 1.24266094738807843860e-3,
                           2.71155556874348757815e-5, 2.01033439929228813265e-7};
  constexpr double F[8] = {1.0, 5.99832206555887937690e-1, 1.36929880922735805310e-1, 1.48753612908506148525e-2,
                           7.86869131145613259100e-4, 1.84631831751005468180e-5, 1.42151175831644588870e-7,
                           2.04426310338993978564e-15};
  const double q = p - 0.5;
  if (fabs(q) <= 0.425) {
    const double r = 0.180625 - q * q;
    return q * as241_poly(A, r) / as241_poly(B, r);
  }
  double r = q < 0.0 ? p : 1.0 - p;  // exact for p >= 0.5 (Sterbenz)
  r = sqrt(-log(r));
  double v;
  if (r <= 5.0) {
    r -= 1.6;
    v = as241_poly(C, r) / as241_poly(D, r);
  } else {
    r -= 5.0;
    v = as241_poly(E, r) / as241_poly(F, r);
  }
  return q < 0.0 ? -v : v;
}

__global__ void norm_ppf_kernel(const double* __restrict__ p, int64_t n, double* __restrict__ z) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) z[i] = norm_ppf(p[i]);
}

// Per (datum j, dim d) constants of the continuous dims: {Phi(lo), Phi(hi)} (NaN pair: domain error;
// the sign of Phi(hi) - Phi(lo) is unused).  A property of the good KDE, computed once per model when
// many candidates are drawn from it (the two normcdf calls dominate a draw otherwise).
__global__ __launch_bounds__(SAMPLE_BLOCK) void kde_sample_table_kernel(
    const double* __restrict__ X, int32_t D, const int64_t* __restrict__ rows, int64_t n,
    const double* __restrict__ bw, const int32_t* __restrict__ levels, double2* __restrict__ tab) {
  const int64_t total = n * (int64_t)D;
  for (int64_t e = (int64_t)blockIdx.x * SAMPLE_BLOCK + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * SAMPLE_BLOCK) {
    const int64_t j = e / D;
    const int d = (int)(e - j * D);
    double2 r = make_double2(0.0, 0.0);
    if (levels[d] == 0) {
      double lo, hi;
      bool flip;
      if (tn_bounds(X[rows[j] * (int64_t)D + d], 1.0 / bw[d], &lo, &hi, &flip))
        r = make_double2(normcdf(lo), normcdf(hi));
      else
        r = make_double2(NAN, NAN);
    }
    tab[e] = r;
  }
}

// z = Phi^-1(p) on the smaller tail in fp32, p = Phi(lo) + u (Phi(hi) - Phi(lo)) in fp64, clamped to [lo, hi]
// erfcinv(t), t in (0, 1], in single precision without the library's branches: M. Giles' single-precision erfinv
// polynomials ("Approximating the erfinv function", GPU Computing Gems Jade, 2011; relative error ~4e-7) at
// x = 1 - t, with w = -ln((1 - x)(1 + x)) formed from t itself (t (2 - t): exact in the tail where 1 - t rounds)
__device__ __forceinline__ float fast_erfcinvf(float t) {
  float w = -__logf(t * (2.0f - t));
  float p;
  if (w < 5.0f) {
    w = w - 2.5f;
    p = 2.81022636e-08f;
    p = fmaf(p, w, 3.43273939e-07f);
    p = fmaf(p, w, -3.5233877e-06f);
    p = fmaf(p, w, -4.39150654e-06f);
    p = fmaf(p, w, 0.00021858087f);
    p = fmaf(p, w, -0.00125372503f);
    p = fmaf(p, w, -0.00417768164f);
    p = fmaf(p, w, 0.246640727f);
    p = fmaf(p, w, 1.50140941f);
  } else {
    w = sqrtf(w) - 3.0f;
    p = -0.000200214257f;
    p = fmaf(p, w, 0.000100950558f);
    p = fmaf(p, w, 0.00134934322f);
    p = fmaf(p, w, -0.00367342844f);
    p = fmaf(p, w, 0.00573950773f);
    p = fmaf(p, w, -0.0076224613f);
    p = fmaf(p, w, 0.00943887047f);
    p = fmaf(p, w, 1.00167406f);
    p = fmaf(p, w, 2.83297682f);
  }
  return p * (1.0f - t);
}

__device__ __forceinline__ double tn_invert_f32(double plo, double phi, double lo, double hi, double u) {
  const double p = fma(u, phi - plo, plo);
  const bool up = p > 0.5;
  const float t = (float)(2.0 * (up ? 1.0 - p : p));        // in (0, 1]
  const float zt = -1.41421356237309505f * fast_erfcinvf(t);  // Phi^-1(min(p, 1 - p)) <= 0
  // (the library's erfcinvf: the same draws in distribution, 0.126 instead of 0.113 ms per 1e6 x 32 launch)
  const double z = (double)(up ? -zt : zt);
  return fmin(fmax(z, lo), hi);
}

// One draw of dim d of a candidate whose datum row is xr from the 32-bit uniform word w0.
// TAB: the Phi table is given (one instance each way: the table instance carries no inlined normcdf)
template <bool TAB>
__device__ __forceinline__ double sample_dim(const double* __restrict__ xr, int d, int32_t idx, int32_t D,
                                             const double* __restrict__ bw, const double* __restrict__ rbw,
                                             const int32_t* __restrict__ levels,
                                             const double2* __restrict__ tab, double bw_factor, uint32_t w0,
                                             bool* derr) {
  const double m = xr[d];
  const double h = bw[d];
  const int t = levels[d];
  const double u = ((double)w0 + 0.5) * 0x1p-32;  // open (0, 1)
  if (t != 0) {  // keep m with probability 1 - h, else a uniform level: both from the one uniform
    const double thr = 1.0 - h;
    if (u < thr) return m;
    const double v = thr > 0.0 ? (u - thr) * rbw[d] : u;  // ~uniform on [0, 1) given the resample (1 / h: LDS)
    const int lv = (int)(v * (double)t);
    return (double)(lv < t ? lv : t - 1);
  }
  double lo, hi;
  bool flip;
  if (!tn_bounds(m, rbw[d], &lo, &hi, &flip)) {  // scipy's argcheck fails: the reference call raises
    *derr = true;
    return NAN;
  }
  double plo, phi;
  if constexpr (TAB) {
    const double2 p = tab[(int64_t)idx * D + d];
    plo = p.x;
    phi = p.y;
  } else {
    plo = normcdf(lo);
    phi = normcdf(hi);
  }
  const double z = tn_invert_f32(plo, phi, lo, hi, u);
  return fma(bw_factor * h, flip ? -z : z, m);
}

// The draws with one (candidate, pair of dims) per lane: L = SAMPLE_LPC lanes per candidate, lane g of the
// group takes the pairs g, g + L, ...  A candidate's datum row and Phi-table row are then read by its L lanes
// as contiguous 16-byte pieces and its output row is written as contiguous 16-byte stores (a lane-per-
// candidate layout, 8-9 % slower with the same draws, was removed in round 5).  One Philox block per lane and
// two pairs (word g + L i for pairs g + 2 L i and g + L + 2 L i): the block's four words are the four dims'
// uniforms -- a categorical dim takes both its keep-or-resample decision and its level from its uniform --
// so a candidate costs D / 4 blocks (D before round 5: two words per dim, the generator half the work).
// Dim types and bandwidths vary across the lanes (loaded per lane; the categorical branch is the cheap
// one): with 4 lanes a 24c + 8u candidate's 16 pairs take three all-continuous steps and one all-categorical
// step, where 8 lanes ran a mixed step through both branches.  Counter (candidate, word, stream): the draws
// do not depend on the launch shape.
#ifndef SAMPLE_LPC
#define SAMPLE_LPC 4  // lanes per candidate (8: 0.130 ms, 2: 0.196 ms per 1e6 x 32 launch against 0.119 ms; lib_ab)
#endif
template <bool TAB>
__global__ __launch_bounds__(256) void kde_sample_pair_kernel(
    const double* __restrict__ X, int32_t D, const int64_t* __restrict__ rows, int64_t n,
    const double* __restrict__ bw, const int32_t* __restrict__ levels, const double2* __restrict__ tab,
    double bw_factor, uint64_t seed, uint64_t counter_base, uint32_t stream_id, int64_t Nc,
    double* __restrict__ cands, int64_t* __restrict__ datum, uint8_t* __restrict__ domain_err) {
  constexpr int CPB = 256 / SAMPLE_LPC;  // candidates per block
  __shared__ int32_t sdat[CPB];
  __shared__ double srh[HBX_MAX_D];  // 1 / bw per dim
  const int64_t c0 = (int64_t)blockIdx.x * CPB;
  const int nc = (int)(Nc - c0 < CPB ? Nc - c0 : CPB);
  for (int t = threadIdx.x; t < D; t += 256) srh[t] = 1.0 / bw[t];
  if (threadIdx.x < nc) {
    const int64_t i = c0 + threadIdx.x;
    const uint64_t rb = hbx_bits64(draw(seed, counter_base + (uint64_t)i, DATUM_WORD, stream_id), 0);
    const int32_t idx = (int32_t)__umul64hi(rb, (uint64_t)n);  // floor(u * n), u = rb / 2^64
    sdat[threadIdx.x] = idx;
    if (datum) datum[i] = idx;
  }
  __syncthreads();
  const int cl = threadIdx.x / SAMPLE_LPC, g = threadIdx.x % SAMPLE_LPC;
  if (cl >= nc) return;
  const int64_t i = c0 + cl;
  const int32_t idx = sdat[cl];
  const double* xr = X + rows[idx] * (int64_t)D;
  double* out = cands + i * (int64_t)D;
  const int D2 = (D + 1) >> 1;
  bool derr = false;
  HbxU32x4 r;
  for (int k = g; k < D2; k += SAMPLE_LPC) {
    const int q = (k - g) / SAMPLE_LPC;  // this lane's q-th pair: a new block every second pair
    if ((q & 1) == 0) r = draw(seed, counter_base + (uint64_t)i, (uint32_t)(g + SAMPLE_LPC * (q >> 1)), stream_id);
    const uint32_t w0 = (q & 1) ? r.x[2] : r.x[0], w1 = (q & 1) ? r.x[3] : r.x[1];
    const int d = 2 * k;
    const double v0 = sample_dim<TAB>(xr, d, idx, D, bw, srh, levels, tab, bw_factor, w0, &derr);
    if (d + 1 < D) {
      const double v1 = sample_dim<TAB>(xr, d + 1, idx, D, bw, srh, levels, tab, bw_factor, w1, &derr);
      if ((D & 1) == 0) {
        *(double2*)(out + d) = make_double2(v0, v1);
      } else {
        out[d] = v0;
        out[d + 1] = v1;
      }
    } else {
      out[d] = v0;
    }
  }
  if (derr && domain_err) domain_err[i] = 1;  // any of the candidate's lanes (same byte, same value)
}

extern "C" {

int hbx_philox4x32_10(const uint32_t* counter, const uint32_t* key, uint32_t* out) {
  if (!counter || !key || !out) return hbx_fail(HBX_ERR_ARG, "hbx_philox4x32_10: null pointer");
  HbxU32x4 c;
  for (int k = 0; k < 4; ++k) c.x[k] = counter[k];
  const HbxU32x4 r = hbx_philox4x32_10_impl(c, key[0], key[1]);
  for (int k = 0; k < 4; ++k) out[k] = r.x[k];
  return HBX_OK;
}

int hbx_norm_ppf(const double* p, int64_t n, double* z, void* stream) {
  if (n < 0 || (n > 0 && (!p || !z))) return hbx_fail(HBX_ERR_ARG, "hbx_norm_ppf: bad arguments");
  if (n == 0) return HBX_OK;
  hipLaunchKernelGGL(norm_ppf_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, p, n, z);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

int64_t hbx_kde_sample_table_bytes(int64_t n, int32_t D) { return n * (int64_t)D * 16; }

int hbx_kde_sample_table(const double* X, int32_t D, const int64_t* rows, int64_t n, const double* bw,
                         const int32_t* levels, double* tab, void* stream) {
  if (n < 1 || D < 1 || D > HBX_MAX_D) return hbx_fail(HBX_ERR_ARG, "hbx_kde_sample_table: n=%lld D=%d", (long long)n, D);
  if (!X || !rows || !bw || !levels || !tab) return hbx_fail(HBX_ERR_ARG, "hbx_kde_sample_table: null pointer");
  const int64_t blocks = (n * (int64_t)D + SAMPLE_BLOCK - 1) / SAMPLE_BLOCK;
  hipLaunchKernelGGL(kde_sample_table_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(SAMPLE_BLOCK),
                     0, (hipStream_t)stream, X, D, rows, n, bw, levels, (double2*)tab);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

int hbx_kde_sample(const double* X, int32_t D, const int64_t* rows, int64_t n, const double* bw,
                   const int32_t* levels, const double* tab, double bw_factor, uint64_t seed, uint64_t counter_base,
                   uint32_t stream_id, int64_t Nc, double* cands, int64_t* datum, uint8_t* domain_err, void* stream) {
  if (Nc < 0 || D < 1 || D > HBX_MAX_D) return hbx_fail(HBX_ERR_ARG, "hbx_kde_sample: Nc=%lld D=%d", (long long)Nc, D);
  if (Nc == 0) return HBX_OK;
  if (!X || !rows || !bw || !levels || !cands) return hbx_fail(HBX_ERR_ARG, "hbx_kde_sample: null pointer");
  if (n < 1 || n > INT32_MAX) return hbx_fail(HBX_ERR_ARG, "hbx_kde_sample: n=%lld observations", (long long)n);
  hipStream_t s = (hipStream_t)stream;
  if (domain_err) HBX_HIP(hipMemsetAsync(domain_err, 0, (size_t)Nc, s));
  if ((D & 1) == 0 && ((uintptr_t)cands & 15)) return hbx_fail(HBX_ERR_ARG, "hbx_kde_sample: cands not 16-byte aligned");
  constexpr int CPB = 256 / SAMPLE_LPC;
  const int64_t pb = (Nc + CPB - 1) / CPB;  // one (candidate, pair of dims) per lane
  if (pb > INT32_MAX) return hbx_fail(HBX_ERR_ARG, "hbx_kde_sample: Nc=%lld", (long long)Nc);
  hipLaunchKernelGGL(tab ? kde_sample_pair_kernel<true> : kde_sample_pair_kernel<false>, dim3((unsigned)pb), dim3(256),
                     0, s, X, D, rows, n, bw, levels, (const double2*)tab, bw_factor, seed, counter_base, stream_id,
                     Nc, cands, datum, domain_err);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

}  // extern "C"
