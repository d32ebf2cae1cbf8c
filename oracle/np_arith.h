/* ORACLE -- test infrastructure only (included by oracle/kde_oracle.c).
 *
 * The reference's own float64 arithmetic for the exact checks: exp as the pinned oracle interpreter's
 * numpy 1.26.4 evaluates it on AVX512_SKX hosts (Intel SVML __svml_exp8, the variant numpy vendors;
 * main path + the scalar "cout_rare" routine for |x| >= 707.70), restated from its algorithm with the
 * constants and tables numpy 1.26.4 ships; checked bit for bit against that numpy on 1.1e7 inputs
 * over [-750, 750].  And numpy's pairwise summation (np.add.reduce over a contiguous float64 array:
 * 8192-element buffers accumulated from 0.0, pairwise within each: < 8 plain, <= 128 eight
 * accumulators, else split at n/2 rounded down to a multiple of 8).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

static const double NPEXP_T16[16] = {0x1.0000000000000p+0,0x1.0b5586cf9890fp+0,0x1.172b83c7d517bp+0,0x1.2387a6e756238p+0,0x1.306fe0a31b715p+0,0x1.3dea64c123422p+0,0x1.4bfdad5362a27p+0,0x1.5ab07dd485429p+0,0x1.6a09e667f3bcdp+0,0x1.7a11473eb0187p+0,0x1.8ace5422aa0dbp+0,0x1.9c49182a3f090p+0,0x1.ae89f995ad3adp+0,0x1.c199bdd85529cp+0,0x1.d5818dcfba487p+0,0x1.ea4afa2a490dap+0};
static const double NPEXP_HA[128] = {0x1.0000000000000p+0,0x0.0p+0,0x1.02c9a3e778061p+0,-0x1.160139cd8dc5dp-56,0x1.059b0d3158574p+0,0x1.cd2523567f613p-55,0x1.0874518759bc8p+0,0x1.0f74e61e6c861p-57,0x1.0b5586cf9890fp+0,0x1.79aa65d837b6dp-54,0x1.0e3ec32d3d1a2p+0,0x1.ebe3d702f9cd1p-60,0x1.11301d0125b51p+0,-0x1.556522a2fbd0ep-54,0x1.1429aaea92de0p+0,-0x1.1c923b9d5f416p-54,0x1.172b83c7d517bp+0,-0x1.01b15eaa59348p-55,0x1.1a35beb6fcb75p+0,0x1.b898c3f1353bfp-55,0x1.1d4873168b9aap+0,0x1.aecf73e3a2f60p-54,0x1.2063b88628cd6p+0,0x1.a6f4144a6c38dp-55,0x1.2387a6e756238p+0,0x1.68efde3a8a894p-54,0x1.26b4565e27cddp+0,0x1.0472b981fe7f2p-55,0x1.29e9df51fdee1p+0,0x1.2f7e16d09ab31p-55,0x1.2d285a6e4030bp+0,0x1.b3782720c0ab4p-55,0x1.306fe0a31b715p+0,0x1.34d754db0abb6p-55,0x1.33c08b26416ffp+0,0x1.fdd395dd3f84ap-55,0x1.371a7373aa9cbp+0,-0x1.24aedcc4b5068p-54,0x1.3a7db34e59ff7p+0,-0x1.1d1e83e9436d2p-56,0x1.3dea64c123422p+0,0x1.59f48a72a4c6dp-55,0x1.4160a21f72e2ap+0,-0x1.8a78f4817895bp-58,0x1.44e086061892dp+0,0x1.363ed60c2ac11p-59,0x1.486a2b5c13cd0p+0,0x1.ecce1daa10379p-57,0x1.4bfdad5362a27p+0,0x1.690cebb7aafb0p-56,0x1.4f9b2769d2ca7p+0,-0x1.f94340071a38ep-55,0x1.5342b569d4f82p+0,-0x1.8dec6bd0f385fp-56,0x1.56f4736b527dap+0,0x1.3350518fdd78ep-54,0x1.5ab07dd485429p+0,0x1.063e1e21c5409p-54,0x1.5e76f15ad2148p+0,0x1.432e62b64c035p-54,0x1.6247eb03a5585p+0,-0x1.c33c53bef4da8p-55,0x1.6623882552225p+0,-0x1.3cedd78565858p-54,0x1.6a09e667f3bcdp+0,-0x1.3b3efbf5e2228p-54,0x1.6dfb23c651a2fp+0,-0x1.367efb86da9eep-57,0x1.71f75e8ec5f74p+0,-0x1.81f647e5a3ecfp-56,0x1.75feb564267c9p+0,-0x1.619321e55e68ap-55,0x1.7a11473eb0187p+0,-0x1.b32dcb94da51dp-56,0x1.7e2f336cf4e62p+0,0x1.5ebe1abd66c55p-57,0x1.82589994cce13p+0,-0x1.369b6f13b3734p-54,0x1.868d99b4492edp+0,-0x1.4d450d872576ep-54,0x1.8ace5422aa0dbp+0,0x1.db72fc1f0eab4p-55,0x1.8f1ae99157736p+0,0x1.bf68359f35f44p-56,0x1.93737b0cdc5e5p+0,-0x1.da9b88b6c1e29p-58,0x1.97d829fde4e50p+0,-0x1.2434322f4f9aap-54,0x1.9c49182a3f090p+0,0x1.1affc2b91ce27p-56,0x1.a0c667b5de565p+0,-0x1.7c50422622263p-55,0x1.a5503b23e255dp+0,-0x1.1bbd1d3bcbb15p-54,0x1.a9e6b5579fdbfp+0,0x1.469846e735ab3p-55,0x1.ae89f995ad3adp+0,0x1.c1a7792cb3387p-55,0x1.b33a2b84f15fbp+0,-0x1.5c3d956dcaebap-58,0x1.b7f76f2fb5e47p+0,-0x1.8d6f438ad9334p-57,0x1.bcc1e904bc1d2p+0,0x1.4ffd70a5fddcdp-56,0x1.c199bdd85529cp+0,0x1.36eae30af0cb3p-56,0x1.c67f12e57d14bp+0,0x1.4e08fd10959acp-55,0x1.cb720dcef9069p+0,0x1.76b2c6c921968p-57,0x1.d072d4a07897cp+0,-0x1.fad5d3ffffa6fp-55,0x1.d5818dcfba487p+0,0x1.4a385a63d07a7p-56,0x1.da9e603db3285p+0,0x1.e5a50d5c192acp-55,0x1.dfc97337b9b5fp+0,-0x1.2d52107b43e1fp-55,0x1.e502ee78b3ff6p+0,0x1.4b604603a88d3p-56,0x1.ea4afa2a490dap+0,-0x1.ff7128fd391f0p-55,0x1.efa1bee615a27p+0,0x1.ec3bc41aa2008p-55,0x1.f50765b6e4540p+0,0x1.a64a931d185eep-55,0x1.fa7c1819e90d8p+0,0x1.7893b4d91cd9dp-56};
static inline uint64_t npexp_bits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static inline double npexp_dbl(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static double npexp_rare(double x) {
  const uint64_t ux = npexp_bits(x);
  const int e = (int)((ux >> 52) & 0x7ff);
  if (e == 0x7ff) {
    if ((ux >> 63) && (ux & 0xfffffffffffffull) == 0) return 0.0;
    return x * x;
  }
  if (e <= 0x3ca) return x + 1.0;
  if (!(x <= 0x1.62e42fefa39efp+9)) return 0x1.fffffffffffffp+1023 * 0x1.fffffffffffffp+1023;
  if (x < -0x1.74910d52d3051p+9) return 0x1.0000000000001p-1022 * 0x1.0000000000001p-1022;
  const double t = x * 0x1.71547652b82fep+6;
  const double s = t + 0x1.8p52;
  const uint32_t ecx = (uint32_t)npexp_bits(s);
  const int j = ecx & 63;
  const double kN = s - 0x1.8p52;
  double r = x - kN * 0x1.62e42fefa0000p-7;
  r = r - kN * 0x1.cf79abc9e3b3ap-46;
  double p = 0x1.6c16a1c2a3ffdp-10 * r;
  p = p + 0x1.111123aaf20d3p-7;
  p = p * r;
  p = p + 0x1.5555555558fccp-5;
  p = p * r;
  p = p + 0x1.55555555548f8p-3;
  p = p * r;
  p = p + 0x1p-1;
  p = p * r;
  p = p * r;
  p = p + r;
  p = p + NPEXP_HA[2 * j + 1];
  p = p * NPEXP_HA[2 * j];
  if (!(x < -0x1.6232bdd7abcd2p+9)) {
    double res = p + NPEXP_HA[2 * j];
    uint32_t m = ((ecx >> 6) + 0x3ff) & 0x7ff;
    if (m <= 0x7fe) return res * npexp_dbl((uint64_t)m << 52);
    m = (m - 1) & 0x7ff;
    return res * npexp_dbl((uint64_t)m << 52) * 2.0;
  }
  const uint32_t m = ((ecx >> 6) + 0x43b) & 0x7ff;
  const double sc = npexp_dbl((uint64_t)m << 52);
  const double a2 = p * sc;
  const double a1 = sc * NPEXP_HA[2 * j];
  double a0 = a1 + a2;
  if (m <= 0x32) return a0 * 0x1p-60;
  double b = a1 - a0;
  b = b + a2;
  const double c = a0 * 0x1.8p32;
  const double d = a0 + c;
  const double hi = d - c;
  double lo = a0 - hi;
  lo = b + lo;
  return hi * 0x1p-60 + lo * 0x1p-60;
}
static double npexp_fma_rz(double a, double b, double c) {
  const double r = fma(a, b, c);
  const double e = fma(a, b, c - r);
  return e < 0.0 ? r - 0x1p-4 : r;
}
static double np_exp(double x) {
  if (x != x) return x + x;
  const double z = npexp_fma_rz(x, 0x1.71547652b82fep+0, 0x1.8000000003ff0p+48);
  const double N = z - 0x1.8000000003ff0p+48;
  const double T = NPEXP_T16[npexp_bits(z) & 15];
  double r = fma(-N, 0x1.62e42fefa39efp-1, x);
  r = fma(-0x1.abc9e3b39803fp-56, N, r);
  const double rr = npexp_dbl(npexp_bits(r) & 0xbfffffffffffffffull);
  const double r2 = rr * rr;
  double A = fma(0x1.72eb5ef0d213dp-10, rr, 0x1.1106603d97c00p-7);
  const double B = fma(0x1.555564bb4f5f0p-5, rr, 0x1.5555554b508a2p-3);
  const double r3 = r2 * rr;
  const double C = fma(r2, 0x1.0000000002622p-1, rr);
  A = fma(r2, A, B);
  A = fma(r3, A, C);
  A = fma(T, A, T);
  if (!(fabs(x) >= 0x1.61da04cbafe44p+9)) return ldexp(A, (int)floor(N));
  return npexp_rare(x);
}

static double np_pairwise(const double* a, int64_t n) {
  if (n < 8) {
    double res = 0.0;
    for (int64_t i = 0; i < n; ++i) res += a[i];
    return res;
  }
  if (n <= 128) {
    double r[8];
    for (int k = 0; k < 8; ++k) r[k] = a[k];
    int64_t i;
    for (i = 8; i < n - (n % 8); i += 8)
      for (int k = 0; k < 8; ++k) r[k] += a[i + k];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return np_pairwise(a, n2) + np_pairwise(a + n2, n - n2);
}

/* np.add.reduce of a contiguous float64 array */
static double np_sum(const double* a, int64_t n) {
  double acc = 0.0;
  for (int64_t c = 0; c < n; c += 8192) acc = acc + np_pairwise(a + c, (n - c) < 8192 ? (n - c) : 8192);
  return acc;
}
