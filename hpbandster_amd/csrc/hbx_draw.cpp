// hbx_draw.cpp -- host side of BOHB's candidate draws (bohb.py:133-147) on the caller's legacy numpy
// RandomState, in the reference's exact consumption order.
//
// The reference draws, per candidate i: idx = np.random.randint(0, len(data)); then per dim d of
// data[idx]: continuous -- sps.truncnorm.rvs(-m/bw, (1-m)/bw, loc=m, scale=bw_factor*bw), whose scipy
// implementation (rv_generic.rvs -> rv_continuous._rvs) checks a < b and scale >= 0 (ValueError before
// any draw), returns loc when scale == 0 (no draw), else draws ONE random_state.uniform() and returns
// truncnorm._ppf(U, a, b) * scale + loc; categorical -- np.random.rand() < 1 - bw keeps m, else
// np.random.randint(t).  What costs the reference ~0.2 ms per continuous element is scipy's argument
// handling around that one uniform, not the uniform.  This file makes every draw of one get_config call
// -- on the very MT19937 state numpy's RandomState holds, so the stream continues exactly as the
// reference's calls would leave it -- and returns the uniforms; the caller applies the (vectorised)
// truncnorm._ppf to them (config_generators/bohb.py).  No compute here is approximate: the draws are
// numpy's legacy MT19937 algorithms restated (numpy/random/src/mt19937/mt19937.{h,c},
// numpy/random/src/distributions/distributions.c: random_standard_uniform = next_double,
// random_bounded_uint64_fill with use_masked = true, the legacy RandomState.randint path).
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "hbx_common.h"

namespace {

constexpr int kN = 624;
constexpr int kM = 397;

struct MTState {  // numpy's mt19937_state: uint32_t key[624]; int pos;
  uint32_t key[kN];
  int pos;
};

void mt_gen(MTState* s) {  // the standard MT19937 twist (mt19937_gen)
  const uint32_t UPPER = 0x80000000u, LOWER = 0x7fffffffu, MATRIX_A = 0x9908b0dfu;
  int i;
  uint32_t y;
  for (i = 0; i < kN - kM; ++i) {
    y = (s->key[i] & UPPER) | (s->key[i + 1] & LOWER);
    s->key[i] = s->key[i + kM] ^ (y >> 1) ^ (-(y & 1) & MATRIX_A);
  }
  for (; i < kN - 1; ++i) {
    y = (s->key[i] & UPPER) | (s->key[i + 1] & LOWER);
    s->key[i] = s->key[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1) & MATRIX_A);
  }
  y = (s->key[kN - 1] & UPPER) | (s->key[0] & LOWER);
  s->key[kN - 1] = s->key[kM - 1] ^ (y >> 1) ^ (-(y & 1) & MATRIX_A);
  s->pos = 0;
}

inline uint32_t mt_next32(MTState* s) {
  if (s->pos == kN) mt_gen(s);
  uint32_t y = s->key[s->pos++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

inline double mt_double(MTState* s) {  // random_sample / rand / uniform(0, 1): 53-bit double
  int32_t a = (int32_t)(mt_next32(s) >> 5), b = (int32_t)(mt_next32(s) >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

// RandomState.randint(low, high) for the default int64 dtype: rng = high - 1 - low, masked rejection on
// 32-bit words when rng fits 32 bits (every range BOHB draws), nothing drawn when rng == 0
inline int64_t mt_randint(MTState* s, int64_t low, int64_t high) {
  uint64_t rng = (uint64_t)(high - 1 - low);
  if (rng == 0) return low;
  if (rng == 0xFFFFFFFFull) return low + (int64_t)mt_next32(s);
  uint64_t mask = rng;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  mask |= mask >> 32;
  uint32_t v;
  while ((v = (mt_next32(s) & (uint32_t)mask)) > rng) {
  }
  return low + (int64_t)v;
}

}  // namespace

extern "C" {

int64_t hbx_mt_state_bytes(void) { return (int64_t)sizeof(MTState); }

// Self-check hooks (tests, and BOHB's start-up check against numpy itself): draw from a raw state.
int hbx_mt_draw(void* state, int32_t kind, int64_t n, int64_t high, double* out) {
  if (!state || !out || n < 0) return hbx_fail(HBX_ERR_ARG, "hbx_mt_draw: bad arguments");
  MTState* s = (MTState*)state;
  if (s->pos < 0 || s->pos > kN) return hbx_fail(HBX_ERR_ARG, "hbx_mt_draw: state position %d", s->pos);
  for (int64_t i = 0; i < n; ++i) out[i] = kind == 0 ? mt_double(s) : (double)mt_randint(s, 0, high);
  return HBX_OK;
}

int hbx_bohb_draw(void* state, const double* data, int64_t n, int32_t D, const double* bw, const int64_t* levels,
                  double bw_factor, int64_t num_samples, double* vals, double* uni, uint8_t* need_ppf,
                  int64_t* datum, int64_t* stop, int64_t* compact, int64_t* n_compact) {
  if (!state || !data || !bw || !levels || !vals || !uni || (!need_ppf && !compact) || !stop || n <= 0 || D <= 0 ||
      num_samples < 0 || (compact && !n_compact))
    return hbx_fail(HBX_ERR_ARG, "hbx_bohb_draw: bad arguments");
  const int64_t cap = num_samples * (int64_t)D;
  int64_t nc = 0;
  MTState* s = (MTState*)state;
  if (s->pos < 0 || s->pos > kN) return hbx_fail(HBX_ERR_ARG, "hbx_bohb_draw: state position %d", s->pos);
  for (int64_t i = 0; i < num_samples; ++i) {
    const int64_t idx = mt_randint(s, 0, n);  // bohb.py:135
    if (datum) datum[i] = idx;
    const double* row = data + idx * (int64_t)D;
    for (int32_t d = 0; d < D; ++d) {
      const int64_t e = i * D + d;
      const double m = row[d], h = bw[d];
      if (need_ppf) need_ppf[e] = 0;
      if (levels[d] == 0) {  // bohb.py:141: truncnorm.rvs(-m/bw, (1-m)/bw, loc=m, scale=bw_factor*bw)
        const double a = -m / h, b = (1. - m) / h, scale = bw_factor * h;
        if (!(a < b) || !(scale >= 0.)) {  // scipy's domain check raises before drawing
          *stop = e;
          return 1;
        }
        if (scale == 0.) {
          vals[e] = m * 1.0;  // loc * ones(size): no draw
        } else {
          const double u = mt_double(s);  // random_state.uniform(size=()) = 0 + 1 * next_double
          vals[e] = m;
          if (compact) {  // the inversion's inputs packed: uniform, element index, term index (datum row, dim)
            uni[nc] = u;
            compact[nc] = e;
            compact[cap + nc] = idx * (int64_t)D + d;
            ++nc;
          } else {
            uni[e] = u;
            need_ppf[e] = 1;
          }
        }
      } else {  // bohb.py:144-147
        if (mt_double(s) < (1. - h))
          vals[e] = m;
        else
          vals[e] = (double)mt_randint(s, 0, levels[d]);
      }
    }
  }
  *stop = -1;
  if (n_compact) *n_compact = nc;
  return HBX_OK;
}

}  // extern "C"
