// hbx_npsort.h -- numpy's np.argsort of float64 restated for one workgroup, so that TIED keys come out
// in the reference's order (device code).
//
// The reference splits BOHB's losses with np.argsort(losses) (bohb.py:229) and ranks a successive-halving
// stage with np.argsort(np.argsort(losses)) (HB_iteration.py:180,240): numpy's default sort, which is not
// stable.  Crashed runs all score +inf (bohb.py:189-192) and quantised losses tie, so which rows enter
// each KDE -- and in which order, which fixes np.std's summation order and the pdf's -- and which tied
// configurations advance depend on how that sort breaks ties.  Third-party pin: numpy 1.26.4 on an
// AVX-512 (AVX512_SKX) host dispatches aquicksort_double to the vendored x86-simd-sort
// avx512_argsort<double> (numpy/core/src/npysort/x86-simd-sort, src/avx512-64bit-argsort.hpp):
//   * a NaN present: std::sort of the indices with a NaN-last comparator (libstdc++ introsort);
//   * else quicksort on the index array: pivot = 5th smallest of 8 keys sampled at stride
//     (right-left)/8; partition_avx512 (ranges <= 256) / partition_avx512_unrolled<4> moves 8-index
//     vectors with compress-stores, keys >= pivot to the right, the first and last 8 (32) held back to
//     the end, the next vector taken from the side with less stored room; ranges <= 64 go to the bitonic
//     key/index networks argsort_{8,16,32,64}_64bit (padding lanes +inf / index 0; equal keys never
//     swap); std::sort once 2 floor(log2 n) levels are spent.
// Licences of the restated third-party algorithms: x86-simd-sort is BSD-3-Clause (Intel Corporation), as
// vendored by numpy (BSD-3-Clause); libstdc++'s std::sort / heap helpers are GPL-3.0 with the GCC Runtime
// Library Exception.  Only their published algorithms are restated here (no source text is copied); the
// restatement is what reproduces numpy's tie order, so it follows them step for step.
// oracle/np_argsort.py is the same restatement in Python, pinned by numpy 1.26.4's own outputs
// (tests/golden/np_argsort.npz).  Here every range is handled by one wave: the partition's sequential
// "which side next" walk runs on uniform scalars with the per-group counts held in lane windows, the
// compress-stores become one parallel scatter, the networks run on 64 lanes; the work list of ranges is
// level-synchronous over the workgroup's waves (ranges of one level are disjoint).
#pragma once

#include "hbx_common.h"

#define NPS_WAVES 4
#define NPS_THREADS (64 * NPS_WAVES)

#ifdef NPS_TIMING  // diagnostic builds only (tools/build_variant.sh): stage stamps of the last re-rank
__device__ unsigned long long nps_dbg[64];
#define NPS_STAMP(k) do { if ((threadIdx.x & 63) == 0 && (k) < 64) nps_dbg[(k)] = wall_clock64(); } while (0)
#else
#define NPS_STAMP(k) do { } while (0)
#endif

struct NpsRange {
  int32_t L, R, it;  // [L, R), remaining depth budget
};

// ---- libstdc++ std::sort (bits/stl_algo.h, bits/stl_heap.h) on one lane ----------------------------
// Elements T: positions (int32, keys read through x) or (key, position) pairs (NpsKV: the key travels
// with its position, so a comparison is one LDS read instead of two dependent ones).  The same
// comparisons in the same order either way, so the same arrangement of positions.
struct NpsLess {
  const double* x;
  bool nan_last;
  __device__ bool operator()(int32_t a, int32_t b) const { return less(x[a], x[b]); }
  __device__ bool less(double u, double v) const {
    if (!nan_last) return u < v;
    if (u == u && v == v) return u < v;
    if (u != u) return false;
    return true;
  }
};

struct NpsKV {
  double k;
  int32_t i, pad;
};

struct NpsKVLess {
  bool nan_last;
  __device__ bool operator()(const NpsKV& a, const NpsKV& b) const { return NpsLess{nullptr, nan_last}.less(a.k, b.k); }
};

template <class T>
__device__ inline void nps_swap(T* a, int i, int j) {
  const T t = a[i];
  a[i] = a[j];
  a[j] = t;
}

template <class T, class C>
__device__ inline void nps_move_median_to_first(T* a, int res, int p, int q, int r, const C& lt) {
  if (lt(a[p], a[q])) {
    if (lt(a[q], a[r])) nps_swap(a, res, q);
    else if (lt(a[p], a[r])) nps_swap(a, res, r);
    else nps_swap(a, res, p);
  } else if (lt(a[p], a[r])) {
    nps_swap(a, res, p);
  } else if (lt(a[q], a[r])) {
    nps_swap(a, res, r);
  } else {
    nps_swap(a, res, q);
  }
}

template <class T, class C>
__device__ inline int nps_unguarded_partition(T* a, int first, int last, int pivot, const C& lt) {
  while (true) {
    while (lt(a[first], a[pivot])) ++first;
    --last;
    while (lt(a[pivot], a[last])) --last;
    if (!(first < last)) return first;
    nps_swap(a, first, last);
    ++first;
  }
}

template <class T, class C>
__device__ inline void nps_adjust_heap(T* a, int first, int hole, int len, T value, const C& lt) {
  const int top = hole;
  int child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (lt(a[first + child], a[first + child - 1])) --child;
    a[first + hole] = a[first + child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    a[first + hole] = a[first + child - 1];
    hole = child - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && lt(a[first + parent], value)) {
    a[first + hole] = a[first + parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  a[first + hole] = value;
}

template <class T, class C>
__device__ inline void nps_heap_sort(T* a, int first, int last, const C& lt) {
  const int n = last - first;
  if (n >= 2)
    for (int parent = (n - 2) / 2;; --parent) {
      nps_adjust_heap(a, first, parent, n, a[first + parent], lt);
      if (parent == 0) break;
    }
  while (last - first > 1) {
    --last;
    const T value = a[last];
    a[last] = a[first];
    nps_adjust_heap(a, first, 0, last - first, value, lt);
  }
}

template <class T, class C>
__device__ inline void nps_insertion_sort(T* a, int first, int last, const C& lt) {
  if (first == last) return;
  for (int i = first + 1; i < last; ++i) {
    const T val = a[i];
    if (lt(val, a[first])) {
      for (int j = i; j > first; --j) a[j] = a[j - 1];
      a[first] = val;
    } else {
      int j = i;
      while (lt(val, a[j - 1])) {
        a[j] = a[j - 1];
        --j;
      }
      a[j] = val;
    }
  }
}

template <class T, class C>
__device__ inline void nps_unguarded_insertion_sort(T* a, int first, int last, const C& lt) {
  for (int i = first; i < last; ++i) {
    const T val = a[i];
    int j = i;
    while (lt(val, a[j - 1])) {
      a[j] = a[j - 1];
      --j;
    }
    a[j] = val;
  }
}

// std::sort(a + first, a + last, lt): __introsort_loop (threshold 16, depth 2 floor(log2 n)) made
// iterative -- the right part of each cut on a stack with its depth, the loop on the left part; the
// ranges are disjoint, so the order they are finished in does not matter -- then __final_insertion_sort
template <class T, class C>
__device__ inline void nps_std_sort(T* a, int first, int last, const C& lt) {
  if (last - first < 2) return;
  struct Fr {
    int f, l, d;
  } st[66];
  int sp = 0;
  st[sp++] = Fr{first, last, 2 * (31 - __clz(last - first))};
  while (sp > 0) {
    Fr fr = st[--sp];
    while (fr.l - fr.f > 16) {
      if (fr.d == 0) {
        nps_heap_sort(a, fr.f, fr.l, lt);
        break;
      }
      --fr.d;
      const int mid = fr.f + (fr.l - fr.f) / 2;
      nps_move_median_to_first(a, fr.f, fr.f + 1, mid, fr.l - 1, lt);
      const int cut = nps_unguarded_partition(a, fr.f + 1, fr.l, fr.f, lt);
      st[sp++] = Fr{cut, fr.l, fr.d};
      fr.l = cut;
    }
  }
  if (last - first > 16) {
    nps_insertion_sort(a, first, first + 16, lt);
    nps_unguarded_insertion_sort(a, first + 16, last, lt);
  } else {
    nps_insertion_sort(a, first, last, lt);
  }
}

// std::sort of the positions A[first, last) by keys x (NaN-free) with each key carried beside its
// position in kv (>= last - first pairs of LDS scratch): the wave stages the pairs, lane 0 sorts them, the
// wave writes the positions back.  Whole wave.
__device__ inline void nps_std_sort_staged(const double* __restrict__ x, int32_t* A, int first, int last, NpsKV* kv,
                                           int lane) {
  const int m = last - first;
  for (int j = lane; j < m; j += 64) {
    const int32_t p = A[first + j];
    kv[j] = NpsKV{x[p], p, 0};
  }
  __threadfence_block();
  if (lane == 0) nps_std_sort(kv, 0, m, NpsKVLess{false});
  __threadfence_block();
  for (int j = lane; j < m; j += 64) A[first + j] = kv[j].i;
  __threadfence_block();
}

// ---- the bitonic key/index networks (x86-simd-sort argsort_{8,16,32,64}_64bit) on one wave ----------
// lane t = 8 r + l holds lane l of register r.  A compare-exchange: a lane takes the min (max) of its key
// and its partner's and keeps its own index where the chosen key equals its own -- equal keys never move.
struct NpsLane {
  double k;
  int32_t i;
};

__device__ __forceinline__ void nps_cx(NpsLane& v, int partner, bool takemax) {
  const double kp = __shfl(v.k, partner);
  const int32_t ip = __shfl(v.i, partner);
  const double kn = takemax ? (kp > v.k ? kp : v.k) : (kp < v.k ? kp : v.k);
  if (!(kn == v.k)) v.i = ip;
  v.k = kn;
}

__device__ __forceinline__ void nps_perm(NpsLane& v, int src) {
  v.k = __shfl(v.k, src);
  v.i = __shfl(v.i, src);
}

// cmp_merge within every register: partner lane l ^ x, the lanes whose mask bit is set take the max
__device__ __forceinline__ void nps_in_reg(NpsLane& v, int lane, int x, int maskbit) {
  nps_cx(v, (lane & ~7) | ((lane & 7) ^ x), ((lane & 7) & maskbit) != 0);
}

__device__ __forceinline__ void nps_sort_zmm(NpsLane& v, int lane) {
  nps_in_reg(v, lane, 1, 1);  // SHUFFLE_MASK(1,1,1,1), 0xAA
  nps_in_reg(v, lane, 3, 2);  // NETWORK_64BIT_1, 0xCC
  nps_in_reg(v, lane, 1, 1);
  nps_in_reg(v, lane, 7, 4);  // NETWORK_64BIT_2 (reverse), 0xF0
  nps_in_reg(v, lane, 2, 2);  // NETWORK_64BIT_3, 0xCC
  nps_in_reg(v, lane, 1, 1);
}

__device__ __forceinline__ void nps_merge_zmm(NpsLane& v, int lane) {
  nps_in_reg(v, lane, 4, 4);  // NETWORK_64BIT_4, 0xF0
  nps_in_reg(v, lane, 2, 2);  // NETWORK_64BIT_3, 0xCC
  nps_in_reg(v, lane, 1, 1);
}

// reverse the registers whose bit is set in `regs` (permutexvar with NETWORK_64BIT_2)
__device__ __forceinline__ void nps_rev(NpsLane& v, int lane, unsigned regs) {
  const int r = lane >> 3;
  nps_perm(v, ((regs >> r) & 1u) ? (lane ^ 7) : lane);
}

// COEX of register pairs: partner[r] = the other register of r's pair (r itself: untouched); the lower
// register of a pair takes the min
__device__ __forceinline__ void nps_coex(NpsLane& v, int lane, const int (&partner)[8]) {
  const int r = lane >> 3, p = partner[r];
  if (p == r) {
    nps_perm(v, lane);  // every lane joins the shuffles
    return;
  }
  nps_cx(v, 8 * p + (lane & 7), p < r);
}

// argsort_n of the keys x[A[L .. L+N)], N <= 64, by one wave
__device__ inline void nps_leaf(const double* __restrict__ x, int32_t* A, int L, int N, int lane) {
  if (N <= 1) return;
  const int nreg = N <= 8 ? 1 : N <= 16 ? 2 : N <= 32 ? 4 : 8;
  NpsLane v;
  if (lane < N) {
    v.i = A[L + lane];
    v.k = x[v.i];
  } else {
    v.i = 0;
    v.k = __builtin_inf();
  }
  nps_sort_zmm(v, lane);
  if (nreg >= 2) {  // bitonic_merge_two_zmm_64bit on (0,1), (2,3), ...
    const unsigned odd = nreg == 2 ? 0x2u : nreg == 4 ? 0xAu : 0xAAu;
    nps_rev(v, lane, odd);
    const int pr[8] = {nreg > 1 ? 1 : 0, nreg > 1 ? 0 : 1, nreg > 2 ? 3 : 2, nreg > 2 ? 2 : 3,
                       nreg > 4 ? 5 : 4, nreg > 4 ? 4 : 5, nreg > 4 ? 7 : 6, nreg > 4 ? 6 : 7};
    nps_coex(v, lane, pr);
    nps_rev(v, lane, odd);
    nps_merge_zmm(v, lane);
  }
  if (nreg >= 4) {  // bitonic_merge_four_zmm_64bit on (0..3) (and (4..7))
    const unsigned hi2 = nreg == 4 ? 0xCu : 0xCCu;
    const bool two = nreg == 8;
    nps_rev(v, lane, hi2);
    const int p1[8] = {3, 2, 1, 0, two ? 7 : 4, two ? 6 : 5, two ? 5 : 6, two ? 4 : 7};
    nps_coex(v, lane, p1);
    nps_rev(v, lane, hi2);
    const int p2[8] = {1, 0, 3, 2, two ? 5 : 4, two ? 4 : 5, two ? 7 : 6, two ? 6 : 7};
    nps_coex(v, lane, p2);
    nps_merge_zmm(v, lane);
  }
  if (nreg == 8) {  // bitonic_merge_eight_zmm_64bit
    nps_rev(v, lane, 0xF0u);
    const int p1[8] = {7, 6, 5, 4, 3, 2, 1, 0};
    nps_coex(v, lane, p1);
    nps_rev(v, lane, 0xF0u);
    const int p2[8] = {2, 3, 0, 1, 6, 7, 4, 5};
    nps_coex(v, lane, p2);
    const int p3[8] = {1, 0, 3, 2, 5, 4, 7, 6};
    nps_coex(v, lane, p3);
    nps_merge_zmm(v, lane);
  }
  if (lane < N) A[L + lane] = v.i;
}

// ---- the quicksort partition of one range by one wave ----------------------------------------------

// lane `src` (wave-uniform) of v, through the scalar unit (v_readlane: no LDS round trip as __shfl takes)
__device__ __forceinline__ int32_t nps_rl(int32_t v, int src) { return __builtin_amdgcn_readlane(v, src); }
__device__ __forceinline__ double nps_rl(double v, int src) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, src);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), src);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// packed >= pivot counts of the U blocks of 8 of group g (4 bits per block): one lane's share of a window
__device__ __forceinline__ uint32_t nps_group_counts(const double* __restrict__ x, const int32_t* A, int Lp, int g,
                                                     int U, double pivot) {
  uint32_t pk = 0;
  for (int ii = 0; ii < U; ++ii) {
    const int32_t* blk = A + Lp + 8 * (g * U + ii);
    int c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) c += x[blk[j]] >= pivot;
    pk |= (uint32_t)c << (4 * ii);
  }
  return pk;
}

// Partition A[L, R) (R - L > 64) around the pivot as partition_avx512(_unrolled<4>) does; returns the
// pivot index, and the range's smallest / biggest key.  T (temp) and W (block destinations) are scratch
// over the same positions.
__device__ inline int nps_partition(const double* __restrict__ x, int32_t* A, int32_t* T, int32_t* W, int L, int R,
                                    int lane, double* pivot_out, double* smallest, double* biggest) {
  const int m = R - L;
  // get_pivot_64bit: the 5th smallest of x[A[L + k size]], k = 1..8, size = (right - left) / 8
  const int size = (R - 1 - L) / 8;
  const double sv = lane < 8 ? x[A[L + (lane + 1) * size]] : 0.0;
  int rank = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const double o = nps_rl(sv, q);
    rank += (o < sv) || (o == sv && q < lane);
  }
  const uint64_t at4 = __ballot(lane < 8 && rank == 4);
  const double pivot = nps_rl(sv, __ffsll((long long)at4) - 1);
  // the range's min / max (the recursion stops on a side whose extreme equals the pivot)
  double mn = __builtin_inf(), mx = -__builtin_inf();
  for (int i = L + lane; i < R; i += 64) {
    const double v = x[A[i]];
    mn = v < mn ? v : mn;
    mx = v > mx ? v : mx;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const double a = __shfl_xor(mn, o), b = __shfl_xor(mx, o);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  *pivot_out = pivot;
  *smallest = mn;
  *biggest = mx;
  const int U = m > 256 ? 4 : 1;  // partition_avx512_unrolled<4> falls back to partition_avx512 at <= 256
  const int p = m % (8 * U);
  int left = L, right = R;
  if (p) {
    // the scalar head loop: examines positions left.. (slots 0..31) and right-1.. (slots 32..63) only
    const int pos = lane < 32 ? L + lane : R - 64 + lane;
    int32_t id = A[pos];
    double kv = x[id];
    for (int t = 0; t < p; ++t) {
      const int sl = left - L;
      const double kl = nps_rl(kv, sl);
      if (!(kl < pivot)) {
        --right;
        const int sr = right - (R - 64);
        const double kr = nps_rl(kv, sr);
        const int32_t il = nps_rl(id, sl), ir = nps_rl(id, sr);
        if (lane == sl) {
          kv = kr;
          id = ir;
        } else if (lane == sr) {
          kv = kl;
          id = il;
        }
      } else {
        ++left;
      }
    }
    A[pos] = id;
    __threadfence_block();
  }
  const int Lp = left, Rp = right;
  const int nb = (Rp - Lp) / 8, G = nb / U;
  // the walk: groups 1 .. G-2 in the order the vector loop loads them, then group 0 and group G-1
  int l_store = Lp, r_store = Rp - 8, lft = Lp + 8 * U, rgt = Rp - 8 * U;
  int wl = 1, wr = G - 2;  // windows: lanes 0..31 hold group wl + lane, lanes 32..63 group wr - (lane - 32)
  auto fill = [&](bool left_half, int base) -> uint32_t {
    const int g = left_half ? base + lane : base - (lane - 32);
    const bool mine = left_half ? lane < 32 : lane >= 32;
    return (mine && g >= 0 && g < G) ? nps_group_counts(x, A, Lp, g, U, pivot) : 0u;
  };
  uint32_t win = 0;
  if (G > 2) {
    const uint32_t a = fill(true, wl), b = fill(false, wr);
    win = lane < 32 ? a : b;
  }
  auto store_group = [&](int g, uint32_t pk) {
    for (int ii = 0; ii < U; ++ii) {
      const int c = (int)((pk >> (4 * ii)) & 15u);
      const int bi = g * U + ii;
      if (lane == 0) {
        W[L + 2 * bi] = l_store;
        W[L + 2 * bi + 1] = r_store + 8;
      }
      l_store += 8 - c;
      r_store -= c;
    }
  };
  int gl = 1, gr = G - 2;
  for (int guard = 0; rgt - lft != 0 && guard < G; ++guard) {  // G - 2 groups: the guard never binds
    int g, slot;
    if ((r_store + 8) - rgt < lft - l_store) {
      rgt -= 8 * U;
      g = gr--;
      if (wr - g >= 32) {
        wr = g;
        const uint32_t b = fill(false, wr);
        if (lane >= 32) win = b;
      }
      slot = 32 + (wr - g);
    } else {
      g = gl++;
      lft += 8 * U;
      if (g - wl >= 32) {
        wl = g;
        const uint32_t a = fill(true, wl);
        if (lane < 32) win = a;
      }
      slot = g - wl;
    }
    store_group(g, (uint32_t)nps_rl((int32_t)win, slot));
  }
  {  // the held-back first and last groups
    uint32_t pk0 = 0, pk1 = 0;
    if (lane == 0) {
      pk0 = nps_group_counts(x, A, Lp, 0, U, pivot);
      pk1 = nps_group_counts(x, A, Lp, G - 1, U, pivot);
    }
    store_group(0, (uint32_t)nps_rl((int32_t)pk0, 0));
    store_group(G - 1, (uint32_t)nps_rl((int32_t)pk1, 0));
  }
  __threadfence_block();
  // the compress-stores, all at once: block b's keys >= pivot end at W[2b+1], the rest start at W[2b]
  for (int b0 = 0; b0 < nb; b0 += 8) {
    const int b = b0 + (lane >> 3), j = lane & 7;
    const bool act = b < nb;
    int32_t id = 0;
    bool ge = false;
    if (act) {
      id = A[Lp + 8 * b + j];
      ge = x[id] >= pivot;
    }
    const uint64_t bal = __ballot(ge);
    const uint32_t m8 = (uint32_t)(bal >> (lane & ~7)) & 0xffu;
    const int c = __popc(m8), gb = __popc(m8 & ((1u << j) - 1u));
    if (act) {
      const int dst = ge ? W[L + 2 * b + 1] - c + gb : W[L + 2 * b] + (j - gb);
      T[dst] = id;
    }
  }
  __threadfence_block();
  for (int i = Lp + lane; i < Rp; i += 64) A[i] = T[i];
  __threadfence_block();
  return l_store;
}

// ---- one segment, one workgroup ----------------------------------------------------------------------
// A[0..n) must hold the positions to sort (keys x[A[i]]); on return it holds numpy's argsort order.
// T, W: n int32 each; lists: 2 * cap NpsRange.  nan_any: some key is NaN (the std::sort path).
__device__ inline void nps_sort_segment(const double* __restrict__ x, int n, bool nan_any, int32_t* A, int32_t* T,
                                        int32_t* W, NpsRange* lists, int cap) {
  __shared__ int cnt[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (n <= 1) return;
  if (nan_any) {  // avx512_argsort: has_nan -> std_argsort_withnan
    if (tid == 0) nps_std_sort(A, 0, n, NpsLess{x, true});
    __threadfence_block();
    __syncthreads();
    return;
  }
  const int it0 = 2 * (31 - __clz(n));  // 2 * (int64_t)log2(arrsize)
  if (n <= 64) {
    if (wave == 0) nps_leaf(x, A, 0, n, lane);
    __threadfence_block();
    __syncthreads();
    return;
  }
  if (tid == 0) {
    lists[0] = NpsRange{0, n, it0};
    cnt[0] = 1;
    cnt[1] = 0;
  }
  __threadfence_block();
  __syncthreads();
  int cur = 0;
  for (int level = 0; level <= it0; ++level) {  // every level spends one unit of depth budget
    const int c = cnt[cur];
    if (c == 0) break;
    NpsRange* in = lists + cur * cap;
    NpsRange* out = lists + (cur ^ 1) * cap;
    for (int r = wave; r < c; r += NPS_WAVES) {
      const NpsRange rg = in[r];
      double pivot, sm, bg;
      const int pidx = nps_partition(x, A, T, W, rg.L, rg.R, lane, &pivot, &sm, &bg);
      const NpsRange kids[2] = {{rg.L, pidx, rg.it - 1}, {pidx, rg.R, rg.it - 1}};
      const bool want[2] = {pivot != sm, pivot != bg};
      for (int q = 0; q < 2; ++q) {
        if (!want[q]) continue;
        const NpsRange k = kids[q];
        const int len = k.R - k.L;
        if (len <= 1) continue;
        if (k.it <= 0) {  // depth budget spent: std_argsort on the range
          if (lane == 0) nps_std_sort(A, k.L, k.R, NpsLess{x, false});
        } else if (len <= 64) {
          nps_leaf(x, A, k.L, len, lane);
        } else if (lane == 0) {
          out[atomicAdd(&cnt[cur ^ 1], 1)] = k;
        }
        __threadfence_block();
      }
    }
    __threadfence_block();
    __syncthreads();
    if (tid == 0) cnt[cur] = 0;
    cur ^= 1;
    __syncthreads();
  }
}

// Which positions numpy's argsort puts first: the first kk of A[0..n) after the same quicksort, without
// finishing it -- after a partition only the child range holding the boundary between places kk - 1 and
// kk decides anything more (the other child's keys lie wholly before or after it, in whatever order), so
// the walk follows that one range, a quickselect along numpy's own partition sequence, and ends in its
// network, its std::sort (depth budget spent) or a partition point at the boundary.  One wave; NaN-free
// keys (the promotion's finite losses).  The whole workgroup calls it (a barrier at the end).
// kv (nullable): LDS scratch of kv_cap (key, position) pairs for a std::sort finish that fits
__device__ inline void nps_select_segment(const double* __restrict__ x, int n, int kk, int32_t* A, int32_t* T,
                                          int32_t* W, NpsKV* kv = nullptr, int kv_cap = 0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (wave == 0 && n > 1 && kk > 0 && kk < n) {
    int st = 1;
    NPS_STAMP(0);
    if (n <= 64) {
      nps_leaf(x, A, 0, n, lane);
    } else {
      int L = 0, R = n, it = 2 * (31 - __clz(n));  // 2 * (int64_t)log2(arrsize), as nps_sort_segment
      for (;;) {
        double pivot, sm, bg;
        const int pidx = nps_partition(x, A, T, W, L, R, lane, &pivot, &sm, &bg);
        NPS_STAMP(st);
        ++st;
        int cL, cR;
        bool want;
        if (kk < pidx) {
          cL = L, cR = pidx, want = pivot != sm;
        } else if (kk > pidx) {
          cL = pidx, cR = R, want = pivot != bg;
        } else {
          break;  // the boundary is the partition point
        }
        --it;
        if (!want || cR - cL <= 1) break;
        if (it <= 0) {  // depth budget spent: std_argsort on the range
          if (kv && cR - cL <= kv_cap) nps_std_sort_staged(x, A, cL, cR, kv, lane);
          else if (lane == 0) nps_std_sort(A, cL, cR, NpsLess{x, false});
          break;
        }
        if (cR - cL <= 64) {
          nps_leaf(x, A, cL, cR - cL, lane);
          break;
        }
        L = cL;
        R = cR;
      }
    }
    NPS_STAMP(st);
    NPS_STAMP(63);
  }
  __threadfence_block();
  __syncthreads();
}

// One segment re-ranked in numpy's order by the whole workgroup (the flagged segments of a stable order).
//   promote = 0 (argsort): every position is ranked; out_order[r] = the r-th position.
//   promote = 1 (SH promotion ranks, HB_iteration.py:179-182): the finite losses' positions, in position
//     order, are ranked; advance[pos] = rank < kk (kk = min(#finite, ceil(kb)), kb <= 0: none) for the
//     finite ones, and -- out_order non-null -- out_order = their order then the non-finite positions.
// A / T / W: n int32 of scratch each; Lst: n int32 (two range lists of n / 6).
__device__ inline void nps_order_segment(const double* __restrict__ x, int n, int promote, double kb, int32_t* A,
                                         int32_t* T, int32_t* W, int32_t* Lst, int64_t* __restrict__ out_order,
                                         uint8_t* __restrict__ advance, NpsKV* kv = nullptr, int kv_cap = 0) {
  __shared__ int nan_any, m_sh;
  const int tid = threadIdx.x;
  if (tid == 0) {
    nan_any = 0;
    m_sh = 0;
  }
  __syncthreads();
  if (!promote) {
    for (int i = tid; i < n; i += NPS_THREADS) {
      A[i] = i;
      if (x[i] != x[i]) nan_any = 1;
    }
  } else if (tid < 64) {  // the finite losses' positions, in position order (wave 0)
    int base = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
      const int i = i0 + tid;
      const bool f = i < n && x[i] - x[i] == 0.0;
      const uint64_t m = __ballot(f);
      if (f) A[base + __popcll(m & ((1ull << tid) - 1ull))] = i;
      base += __popcll(m);
    }
    if (tid == 0) m_sh = base;
  }
  __threadfence_block();
  __syncthreads();
  const int m = promote ? m_sh : n;
  const int kk = kb > 0.0 ? (kb >= (double)m ? m : (int)ceil(kb)) : 0;
  if (promote && !out_order)  // the mask alone: only which positions come first (finite keys: no NaN path)
    nps_select_segment(x, m, kk, A, T, W, kv, kv_cap);
  else
    nps_sort_segment(x, m, nan_any != 0, A, T, W, (NpsRange*)Lst, (n / 3) / 2);
  __threadfence_block();
  __syncthreads();
  if (!promote) {
    for (int i = tid; i < n; i += NPS_THREADS) out_order[i] = A[i];
  } else {
    for (int r = tid; r < m; r += NPS_THREADS) {
      advance[A[r]] = r < kk ? 1 : 0;
      if (out_order) out_order[r] = A[r];
    }
    if (out_order && tid < 64) {  // the non-finite positions after them, in position order
      int base = m;
      for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + tid;
        const bool nf = i < n && !(x[i] - x[i] == 0.0);
        const uint64_t mm = __ballot(nf);
        if (nf) out_order[base + __popcll(mm & ((1ull << tid) - 1ull))] = i;
        base += __popcll(mm);
      }
    }
  }
  __threadfence_block();
  __syncthreads();
}
