// hbx_combine.h -- a candidate's score interval from its two KDE estimates (bohb.py:129), shared by the
// combine kernel (hbx_kde.hip) and the fused tail of the 32x32 scoring pair kernel (hbx_score_h32.hip).
//
// Fused single acquisition: the pair kernel's two blocks of one candidate tile (the bad KDE's, the good
// KDE's) each publish their estimates; the SECOND to finish combines the tile -- the score interval of each
// candidate (lo, hi), the tile's minimum upper bound, its first exactly-clamped candidate and the overflow
// flag -- so no separate combine launch re-reads 32 B per candidate.  The acquisition's running minimum,
// first-clamped index and flags are 64-bit words tagged with the acquisition's sequence number in the high
// half (atomicMax of (seq << 32 | ~value) is a min of value within one acquisition, and any word left by an
// earlier acquisition -- a smaller seq -- loses): no initialisation launch before the scoring kernel.
#pragma once

#include "hbx_common.h"
#include "hbx_kde_impl.h"

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

// One candidate: a = its l (good KDE) estimate, b = its g (bad KDE) estimate.  ln-score interval
// [slo, shi] of max(1e-8, g) / max(l, 1e-8); h = the upper bound that enters the acquisition's minimum;
// one = l and g both certainly below 1e-8 (score exactly 1: the candidates tie, only the first can win);
// of = overflow risk (the acquisition re-scores everything); lpt / gpt the point estimates of ln l, ln g.
struct CandScore {
  float slo, shi, h, lpt, gpt;
  bool one, of;
};
__device__ __forceinline__ CandScore combine_one(const KdeEst a, const KdeEst b) {
  CandScore r;
  r.h = INFINITY;
  r.one = false;
  r.of = false;
  const float C = (float)HBX_LN_CLAMP;
  float llo, lhi, glo, ghi;
  if (a.lpos != a.lpos) {  // l NaN -> max(l, 1e-8) is NaN -> score NaN (never selected)
    r.slo = r.shi = NAN;
    r.lpt = NAN;
    est_interval(b, &glo, &ghi, &r.gpt);
    if (b.lpos != b.lpos) r.gpt = NAN;
  } else {
    est_interval(a, &llo, &lhi, &r.lpt);
    float Glo, Ghi;
    if (b.lpos != b.lpos) {  // g NaN -> max(1e-8, g) == 1e-8
      Glo = Ghi = C;
      r.gpt = NAN;
    } else {
      est_interval(b, &glo, &ghi, &r.gpt);
      Glo = fmaxf(glo, C);
      Ghi = fmaxf(ghi, C);
      r.of = ghi > 700.f;
    }
    r.of = r.of || lhi > 700.f;
    r.slo = Glo - fmaxf(lhi, C);
    r.shi = Ghi - fmaxf(llo, C);
    r.h = r.shi;
    const float C1 = C - 1e-4f;  // margin for the rounding of ln(1e-8) to float
    if (lhi < C1 && (b.lpos != b.lpos || ghi < C1)) {  // both clamped: score exactly 1 (ln 0)
      r.one = true;
      r.slo = NAN;  // excluded from the shortlist unless it is the segment's first exact tie
      r.shi = r.h = 0.f;
    }
  }
  return r;
}

// sequence-tagged words of a fused acquisition: [0] the minimum upper bound (ordered-float code), [1] the
// first exactly-clamped candidate, [2] the flags; value ~low (atomicMax picks the smallest low word)
__device__ __forceinline__ void fz_lower(uint64_t* w, uint32_t seq, uint32_t v) {
  const uint64_t k = ((uint64_t)seq << 32) | (uint64_t)(~v);
  if (k > __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax((unsigned long long*)w, k);
}
__device__ __forceinline__ uint32_t fz_read(const uint64_t* w, uint32_t seq, uint32_t dflt) {
  const uint64_t k = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (uint32_t)(k >> 32) == seq ? ~(uint32_t)k : dflt;
}
// flags are ORed: the overflow bit is the only one the fused tail sets (~1 as the low word)
#define FZ_U 0
#define FZ_FIRST1 1
#define FZ_FLAGS 2

// One candidate's interval into lo / hi and the acquisition's words (the rescue pass: per candidate)
__device__ __forceinline__ void fz_candidate(const CandScore& r, int64_t i, float* lo, float* hi, uint64_t* fz,
                                             uint32_t seq) {
  lo[i] = r.slo;
  hi[i] = r.shi;
  if (r.h < INFINITY) fz_lower(fz + FZ_U, seq, hbx_f2ord(r.h));
  if (r.one) fz_lower(fz + FZ_FIRST1, seq, (uint32_t)i);
  if (r.of) fz_lower(fz + FZ_FLAGS, seq, HBX_ACQ_OVERFLOW);
}

// The fused tail of one scoring block of the pair kernel (every thread of the block calls it after its
// estimates are stored): candidates [c0, c0 + cpb) of tile `tile`; est_l / est_g the two KDEs' estimates;
// scratch: >= 3 * 16 dwords of the block's LDS, free by now.  Candidates carrying a rescue marker in either
// estimate are left to the rescue pass.
__device__ __forceinline__ void fz_tile_tail(const KdePairArgs::AcqFuse& f, unsigned tile, int64_t c0, int cpb,
                                             int64_t Nc, const KdeEst* __restrict__ est_l,
                                             const KdeEst* __restrict__ est_g, float* scratch) {
  // publish this block's estimates (every thread's stores), then count the tile's arrivals
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  int32_t* flag = (int32_t*)scratch;
  if (threadIdx.x == 0) {
    uint64_t* w = f.tile + tile;
    uint64_t cur = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t nw;
    do {
      nw = (uint32_t)(cur >> 32) == f.seq ? cur + 1 : (((uint64_t)f.seq << 32) | 1ull);
    } while (!__hip_atomic_compare_exchange_strong(w, &cur, nw, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT));
    *flag = (uint32_t)nw == 2u;  // this block finished the tile second
  }
  __syncthreads();
  const bool second = *flag != 0;
  if (!second) return;  // uniform
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the other block's estimates (no stale L1 lines)
  float h = INFINITY;
  int32_t f1 = INT32_MAX;
  bool of = false;
  for (int t = threadIdx.x; t < cpb; t += blockDim.x) {
    const int64_t i = c0 + t;
    if (i >= Nc) break;
    const KdeEst a = est_l[i], b = est_g[i];
    if (a.err == -1.f || b.err == -1.f) continue;  // the rescue pass recomputes and combines it
    const CandScore r = combine_one(a, b);
    f.lo[i] = r.slo;
    f.hi[i] = r.shi;
    h = fminf(h, r.h);
    if (r.one && (int32_t)i < f1) f1 = (int32_t)i;
    of = of || r.of;
  }
  // block reduction (one entry per wave), one tagged atomic each
  for (int o = 32; o > 0; o >>= 1) {
    h = fminf(h, __shfl_xor(h, o));
    f1 = min(f1, __shfl_xor(f1, o));
  }
  const bool wof = __any(of);
  const int wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  float* rh = scratch + 16;
  int32_t* rf = (int32_t*)(scratch + 32);
  int32_t* ro = (int32_t*)(scratch + 48);
  __syncthreads();  // *flag read by every thread before the scratch is reused
  if ((threadIdx.x & 63) == 0) {
    rh[wv] = h;
    rf[wv] = f1;
    ro[wv] = wof;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float hb = rh[0];
    int32_t fb = rf[0];
    bool ob = ro[0] != 0;
    for (int k = 1; k < nw; ++k) {
      hb = fminf(hb, rh[k]);
      fb = min(fb, rf[k]);
      ob = ob || ro[k] != 0;
    }
    if (hb < INFINITY) fz_lower(f.words + FZ_U, f.seq, hbx_f2ord(hb));
    if (fb != INT32_MAX) fz_lower(f.words + FZ_FIRST1, f.seq, (uint32_t)fb);
    if (ob) fz_lower(f.words + FZ_FLAGS, f.seq, HBX_ACQ_OVERFLOW);
  }
}
