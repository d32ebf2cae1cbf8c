// hbx_pairwise.h -- numpy's pairwise summation order on the GPU (shared by the exact re-score in
// hbx_kde.hip and the cross-validation objectives in hbx_cv.hip).
#pragma once
#include "hbx_common.h"

// numpy's pairwise summation (umath loops: n < 8 plain, <= 128 eight accumulators, else split at
// n/2 rounded down to a multiple of 8).  dens.sum(axis=0) (SM:_kernel_base.py:516) runs it over the
// ufunc buffer chunks of 8192 elements, accumulated left to right from 0.0 -- see exact_pdf.
__device__ inline double pw_leaf_sum(const double* p, int len) {
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
// the acquisition's split re-score (one block per unit) cuts deeper: 32 units of <= 263 elements, whose
// own split trees have depth <= 2, so a buffer spreads over 4x the CUs
#define PW_SPLIT_CUT 5
#define PW_SPLIT_UNITS 32
#define PW_SPLIT_LEVELS 3
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

// Unit u (0..2^CUT - 1) of a buffer: the depth-CUT node at position u, or the shallower leaf whose
// leftmost depth-CUT position is u.  Returns false for positions covered by another unit.
template <int CUT = PW_CUT>
__device__ __forceinline__ bool pw_unit(int m, int u, int* off, int* len) {
  for (int lev = 0; lev <= CUT; ++lev) {
    const int sh = CUT - lev;
    if (!pw_node(m, lev, u >> sh, off, len)) return false;
    if (lev == CUT || *len <= 128) return (u & ((1 << sh) - 1)) == 0;
  }
  return false;
}

// Top of the tree (depth <= CUT) from the unit sums, numpy's order; one thread.  Bottom-up in place:
// node (lev, t) overwrites v[t] after its children v[2t], v[2t+1] of the level below were read.
template <int CUT = PW_CUT>
__device__ inline double pw_combine_units(int m, const double* us) {
  double v[1 << CUT];
  for (int lev = CUT; lev >= 0; --lev)
    for (int t = 0; t < (1 << lev); ++t) {
      int off, len;
      if (!pw_node(m, lev, t, &off, &len)) continue;
      v[t] = (lev == CUT || len <= 128) ? us[t << (CUT - lev)] : v[2 * t] + v[2 * t + 1];
    }
  return v[0];
}

// The same by one wave: lane t holds node (lev, t) of each level in turn, its children read from lanes 2t
// and 2t+1 of the level below -- the same additions in the same order; every lane returns the root.
template <int CUT>
__device__ inline double pw_combine_units_wave(int m, const double* us) {
  static_assert((1 << CUT) <= 64, "one node per lane");
  const int t = threadIdx.x & 63;
  double v = 0.0;
  for (int lev = CUT; lev >= 0; --lev) {
    const double c0 = __shfl(v, (2 * t) & 63), c1 = __shfl(v, (2 * t + 1) & 63);
    int off, len;
    if (t < (1 << lev) && pw_node(m, lev, t, &off, &len))
      v = (lev == CUT || len <= 128) ? us[t << (CUT - lev)] : c0 + c1;
  }
  return __shfl(v, 0);
}

// Pairwise sum of a[0:m] (m <= 1040, in LDS) in numpy's order, whole block, level-synchronous:
// a leaf (len <= 128) is summed by one thread, an inner node adds its two children of the level
// below.  Same additions, same order, as the recursive reference loop.
template <int LEVELS = PW_LEVELS>
__device__ inline double np_pairwise_block(const double* a, int m, double (*nsum)[128]) {
  for (int lev = LEVELS - 1; lev >= 0; --lev) {
    for (int t = threadIdx.x; t < (1 << lev); t += blockDim.x) {
      int off, len;
      if (pw_node(m, lev, t, &off, &len))
        nsum[lev][t] = (len <= 128) ? pw_leaf_sum(a + off, len) : nsum[lev + 1][2 * t] + nsum[lev + 1][2 * t + 1];
    }
    __syncthreads();
  }
  return nsum[0][0];
}

