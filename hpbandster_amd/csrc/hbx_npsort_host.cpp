// hbx_npsort_host.cpp -- numpy 1.26.4's np.argsort of float64 on the HOST, for the successive-halving
// ranks of one bracket whose tied losses straddle the k-th place (HB_iteration.py:180,240:
// np.argsort(np.argsort(losses)) < k) -- the drop-in's one-bracket-per-call case, where a GPU round trip
// costs more than the sort.  Host code only (no device work); the device restatement for batched brackets
// is hbx_npsort.h.
//
// Third-party pin (as hbx_npsort.h): numpy 1.26.4 on an AVX-512 (AVX512_SKX) host dispatches
// aquicksort_double to the vendored x86-simd-sort avx512_argsort<double> (BSD-3-Clause, Intel;
// numpy/core/src/npysort/x86-simd-sort/src/avx512-64bit-argsort.hpp), whose std::sort fallbacks are
// libstdc++'s introsort (GPL-3.0 with the GCC Runtime Library Exception; bits/stl_algo.h, stl_heap.h).
// What follows is a restatement of their published algorithms -- the 8-lane register networks modelled
// lane by lane, the compress-store partition as its sequence of stores -- written from oracle/np_argsort.py
// (this repository's Python restatement, pinned by numpy 1.26.4's own outputs in
// tests/golden/np_argsort.npz); no code of either project is copied.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "hbx_common.h"

namespace {

struct Lane {
  double k;
  int64_t i;
};
struct Reg {
  Lane l[8];
};

// permutation tables: lane i of the result takes lane idx[i] (oracle/np_argsort.py NET*, SWAP1)
constexpr int NET1[8] = {3, 2, 1, 0, 7, 6, 5, 4};
constexpr int NET2[8] = {7, 6, 5, 4, 3, 2, 1, 0};
constexpr int NET3[8] = {2, 3, 0, 1, 6, 7, 4, 5};
constexpr int NET4[8] = {4, 5, 6, 7, 0, 1, 2, 3};
constexpr int SWAP1[8] = {1, 0, 3, 2, 5, 4, 7, 6};

// cmp_merge(v, permute(v), mask): masked lanes take the max, the others the min; a lane keeps its own
// index where the chosen key equals its own (equal keys never swap)
inline Reg cmp_merge(const Reg& v, const int* idx, unsigned mask) {
  Reg o;
  for (int i = 0; i < 8; ++i) {
    const Lane a = v.l[i], b = v.l[idx[i]];
    // max / min (no NaN reaches the networks); of equal keys the lane's own (own index below)
    const double k = ((mask >> i) & 1) ? (b.k > a.k ? b.k : a.k) : (b.k < a.k ? b.k : a.k);
    o.l[i].k = k;
    o.l[i].i = (k == a.k) ? a.i : b.i;
  }
  return o;
}

inline Reg sort_zmm(Reg v) {
  v = cmp_merge(v, SWAP1, 0xAA);
  v = cmp_merge(v, NET1, 0xCC);
  v = cmp_merge(v, SWAP1, 0xAA);
  v = cmp_merge(v, NET2, 0xF0);
  v = cmp_merge(v, NET3, 0xCC);
  v = cmp_merge(v, SWAP1, 0xAA);
  return v;
}

inline Reg merge_zmm(Reg v) {
  v = cmp_merge(v, NET4, 0xF0);
  v = cmp_merge(v, NET3, 0xCC);
  v = cmp_merge(v, SWAP1, 0xAA);
  return v;
}

inline Reg rev(const Reg& v) {
  Reg o;
  for (int i = 0; i < 8; ++i) o.l[i] = v.l[NET2[i]];
  return o;
}

// COEX lane by lane: x the min, y the max; ties keep their places
inline void coex(Reg& x, Reg& y) {
  for (int i = 0; i < 8; ++i) {
    if (y.l[i].k < x.l[i].k) {
      const Lane t = x.l[i];
      x.l[i] = y.l[i];
      y.l[i] = t;
    }
  }
}

void merge_two(Reg* r) {
  Reg a = r[0], b = rev(r[1]);
  coex(a, b);
  r[0] = merge_zmm(a);
  r[1] = merge_zmm(rev(b));
}

void merge_four(Reg* r) {
  Reg t1 = r[0], m1 = rev(r[3]);
  coex(t1, m1);
  Reg t2 = r[1], m2 = rev(r[2]);
  coex(t2, m2);
  Reg t3 = rev(m2), t4 = rev(m1);
  coex(t1, t2);
  coex(t3, t4);
  r[0] = merge_zmm(t1);
  r[1] = merge_zmm(t2);
  r[2] = merge_zmm(t3);
  r[3] = merge_zmm(t4);
}

void merge_eight(Reg* r) {
  Reg t[8], m[4];
  for (int q = 0; q < 4; ++q) {
    t[q] = r[q];
    m[q] = rev(r[7 - q]);
    coex(t[q], m[q]);
  }
  t[4] = rev(m[3]);
  t[5] = rev(m[2]);
  t[6] = rev(m[1]);
  t[7] = rev(m[0]);
  coex(t[0], t[2]);
  coex(t[1], t[3]);
  coex(t[4], t[6]);
  coex(t[5], t[7]);
  coex(t[0], t[1]);
  coex(t[2], t[3]);
  coex(t[4], t[5]);
  coex(t[6], t[7]);
  for (int q = 0; q < 8; ++q) r[q] = merge_zmm(t[q]);
}

// argsort_{8,16,32,64}_64bit on arg[lo, lo + N), N <= 64: padding lanes (+inf, 0), only N lanes stored
void argsort_small(const double* x, int64_t* arg, int64_t lo, int N) {
  const int nreg = N <= 8 ? 1 : N <= 16 ? 2 : N <= 32 ? 4 : 8;
  Reg r[8];
  for (int q = 0; q < nreg; ++q) {
    for (int l = 0; l < 8; ++l) {
      const int p = 8 * q + l;
      if (p < N) {
        const int64_t ix = arg[lo + p];
        r[q].l[l] = Lane{x[ix], ix};
      } else {
        r[q].l[l] = Lane{INFINITY, 0};
      }
    }
    r[q] = sort_zmm(r[q]);
  }
  if (nreg >= 2)
    for (int q = 0; q < nreg; q += 2) merge_two(r + q);
  if (nreg >= 4)
    for (int q = 0; q < nreg; q += 4) merge_four(r + q);
  if (nreg == 8) merge_eight(r);
  for (int p = 0; p < N; ++p) arg[lo + p] = r[p >> 3].l[p & 7].i;
}

// ---- libstdc++ std::sort (introsort) -------------------------------------------------------------
struct LessKey {
  const double* x;
  bool nan_last;
  bool operator()(int64_t a, int64_t b) const {
    const double u = x[a], v = x[b];
    if (!nan_last) return u < v;
    if (u == u && v == v) return u < v;
    if (u != u) return false;
    return true;
  }
};

inline void swp(int64_t* a, int64_t i, int64_t j) {
  const int64_t t = a[i];
  a[i] = a[j];
  a[j] = t;
}

void move_median_to_first(int64_t* a, int64_t res, int64_t p, int64_t q, int64_t r, const LessKey& lt) {
  if (lt(a[p], a[q])) {
    if (lt(a[q], a[r])) swp(a, res, q);
    else if (lt(a[p], a[r])) swp(a, res, r);
    else swp(a, res, p);
  } else if (lt(a[p], a[r])) {
    swp(a, res, p);
  } else if (lt(a[q], a[r])) {
    swp(a, res, r);
  } else {
    swp(a, res, q);
  }
}

int64_t unguarded_partition(int64_t* a, int64_t first, int64_t last, int64_t pivot, const LessKey& lt) {
  while (true) {
    while (lt(a[first], a[pivot])) ++first;
    --last;
    while (lt(a[pivot], a[last])) --last;
    if (!(first < last)) return first;
    swp(a, first, last);
    ++first;
  }
}

void adjust_heap(int64_t* a, int64_t first, int64_t hole, int64_t len, int64_t value, const LessKey& lt) {
  const int64_t top = hole;
  int64_t child = hole;
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
  int64_t parent = (hole - 1) / 2;
  while (hole > top && lt(a[first + parent], value)) {
    a[first + hole] = a[first + parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  a[first + hole] = value;
}

void partial_sort_heap(int64_t* a, int64_t first, int64_t last, const LessKey& lt) {
  const int64_t n = last - first;
  if (n >= 2) {
    for (int64_t parent = (n - 2) / 2;; --parent) {
      adjust_heap(a, first, parent, n, a[first + parent], lt);
      if (parent == 0) break;
    }
  }
  while (last - first > 1) {
    --last;
    const int64_t value = a[last];
    a[last] = a[first];
    adjust_heap(a, first, 0, last - first, value, lt);
  }
}

void introsort_loop(int64_t* a, int64_t first, int64_t last, int depth, const LessKey& lt) {
  while (last - first > 16) {
    if (depth == 0) {
      partial_sort_heap(a, first, last, lt);
      return;
    }
    --depth;
    const int64_t mid = first + (last - first) / 2;
    move_median_to_first(a, first, first + 1, mid, last - 1, lt);
    const int64_t cut = unguarded_partition(a, first + 1, last, first, lt);
    introsort_loop(a, cut, last, depth, lt);
    last = cut;
  }
}

void insertion_sort(int64_t* a, int64_t first, int64_t last, const LessKey& lt) {
  if (first == last) return;
  for (int64_t i = first + 1; i < last; ++i) {
    const int64_t val = a[i];
    if (lt(val, a[first])) {
      memmove(a + first + 1, a + first, sizeof(int64_t) * (size_t)(i - first));
      a[first] = val;
    } else {
      int64_t j = i;
      while (lt(val, a[j - 1])) {
        a[j] = a[j - 1];
        --j;
      }
      a[j] = val;
    }
  }
}

void unguarded_insertion_sort(int64_t* a, int64_t first, int64_t last, const LessKey& lt) {
  for (int64_t i = first; i < last; ++i) {
    const int64_t val = a[i];
    int64_t j = i;
    while (lt(val, a[j - 1])) {
      a[j] = a[j - 1];
      --j;
    }
    a[j] = val;
  }
}

inline int floor_log2(int64_t n) { return 63 - __builtin_clzll((unsigned long long)n); }

void std_sort(int64_t* a, int64_t first, int64_t last, const LessKey& lt) {
  if (first == last) return;
  introsort_loop(a, first, last, 2 * floor_log2(last - first), lt);
  if (last - first > 16) {
    insertion_sort(a, first, first + 16, lt);
    unguarded_insertion_sort(a, first + 16, last, lt);
  } else {
    insertion_sort(a, first, last, lt);
  }
}

// ---- x86-simd-sort quicksort --------------------------------------------------------------------
double get_pivot(const double* x, const int64_t* arg, int64_t left, int64_t right) {
  if (right - left >= 8) {
    const int64_t size = (right - left) / 8;
    double s[8];
    for (int k = 1; k <= 8; ++k) s[k - 1] = x[arg[left + k * size]];
    std::sort(s, s + 8);  // the 5th smallest of eight keys: any correct sort gives the same value
    return s[4];
  }
  return x[arg[right]];
}

// partition_vec: keys >= pivot compress-stored to end at r_end, the others from l_store, lane order;
// returns how many went right
inline int partition_vec(const double* x, int64_t* arg, int64_t l_store, int64_t r_end, const int64_t* vec,
                         double pivot) {
  int64_t lt[8], ge[8];
  int nl = 0, ng = 0;
  for (int l = 0; l < 8; ++l) {
    if (x[vec[l]] >= pivot) ge[ng++] = vec[l];
    else lt[nl++] = vec[l];
  }
  for (int q = 0; q < nl; ++q) arg[l_store + q] = lt[q];
  for (int q = 0; q < ng; ++q) arg[r_end - ng + q] = ge[q];
  return ng;
}

// partition_avx512 (unroll 1) / partition_avx512_unrolled<4> over arg[left, right): the pivot's index,
// the smallest and the biggest key seen
int64_t partition(const double* x, int64_t* arg, int64_t left, int64_t right, double pivot, int unroll,
                  double* smallest, double* biggest) {
  double sm = INFINITY, bg = -INFINITY;
  if (unroll > 1 && right - left <= 8 * unroll * 8) unroll = 1;
  const int U = 8 * unroll;
  for (int64_t t = (right - left) % U; t > 0; --t) {
    const double v = x[arg[left]];
    sm = v < sm ? v : sm;
    bg = v > bg ? v : bg;
    if (!(v < pivot)) {
      --right;
      swp(arg, left, right);
    } else {
      ++left;
    }
  }
  if (left == right) {
    *smallest = sm;
    *biggest = bg;
    return left;
  }
  for (int64_t p = left; p < right; ++p) {
    const double v = x[arg[p]];
    sm = v < sm ? v : sm;
    bg = v > bg ? v : bg;
  }
  *smallest = sm;
  *biggest = bg;
  if (unroll == 1 && right - left == 8) {
    int64_t v[8];
    memcpy(v, arg + left, sizeof(v));
    const int c = partition_vec(x, arg, left, left + 8, v, pivot);
    return left + (8 - c);
  }
  int64_t vl[4][8], vr[4][8], grp[4][8];
  for (int q = 0; q < unroll; ++q) {
    memcpy(vl[q], arg + left + 8 * q, sizeof(vl[q]));
    memcpy(vr[q], arg + right - 8 * (unroll - q), sizeof(vr[q]));
  }
  int64_t r_store = right - 8, l_store = left;
  left += U;
  right -= U;
  while (right - left != 0) {
    if ((r_store + 8) - right < left - l_store) {
      right -= U;
      for (int q = 0; q < unroll; ++q) memcpy(grp[q], arg + right + 8 * q, sizeof(grp[q]));
    } else {
      for (int q = 0; q < unroll; ++q) memcpy(grp[q], arg + left + 8 * q, sizeof(grp[q]));
      left += U;
    }
    for (int q = 0; q < unroll; ++q) {
      const int c = partition_vec(x, arg, l_store, r_store + 8, grp[q], pivot);
      l_store += 8 - c;
      r_store -= c;
    }
  }
  if (unroll == 1) {
    int c = partition_vec(x, arg, l_store, r_store + 8, vl[0], pivot);
    l_store += 8 - c;
    c = partition_vec(x, arg, l_store, l_store + 8, vr[0], pivot);
    l_store += 8 - c;
    return l_store;
  }
  for (int q = 0; q < 2 * unroll; ++q) {
    const int64_t* v = q < unroll ? vl[q] : vr[q - unroll];
    const int c = partition_vec(x, arg, l_store, r_store + 8, v, pivot);
    l_store += 8 - c;
    r_store -= c;
  }
  return l_store;
}

struct Rng {
  int64_t left, right;
  int it;
};

// kk < 0: the whole sort.  kk >= 0: only the SET of positions [0, kk) is wanted (the promotion mask):
// a range lying wholly before or wholly after the cut at kk is left unsorted -- sorting inside it never
// moves an element across the cut -- so only the ranges straddling it are followed (quickselect work)
void qsort64(const double* x, int64_t* arg, int64_t n, int64_t kk = -1) {
  std::vector<Rng> stack;
  stack.push_back(Rng{0, n - 1, 2 * floor_log2(n)});
  const LessKey lt{x, false};
  while (!stack.empty()) {
    const Rng r = stack.back();
    stack.pop_back();
    if (kk >= 0 && !(r.left < kk && r.right >= kk)) continue;
    if (r.it <= 0) {
      std_sort(arg, r.left, r.right + 1, lt);
      continue;
    }
    if (r.right + 1 - r.left <= 64) {
      argsort_small(x, arg, r.left, (int)(r.right + 1 - r.left));
      continue;
    }
    const double pivot = get_pivot(x, arg, r.left, r.right);
    double sm, bg;
    const int64_t pidx = partition(x, arg, r.left, r.right + 1, pivot, 4, &sm, &bg);
    if (pivot != sm) stack.push_back(Rng{r.left, pidx - 1, r.it - 1});
    if (pivot != bg) stack.push_back(Rng{pidx, r.right, r.it - 1});
  }
}

}  // namespace

extern "C" {

// np.argsort(x) of numpy 1.26.4 (AVX512_SKX), host arrays: order[n] (positions), ties in numpy's order
int hbx_np_argsort_host(const double* x, int64_t n, int64_t* order) {
  if (n < 0 || (n > 0 && (!x || !order))) return hbx_fail(HBX_ERR_ARG, "hbx_np_argsort_host: bad arguments");
  for (int64_t i = 0; i < n; ++i) order[i] = i;
  if (n <= 1) return HBX_OK;
  bool nan = false;
  for (int64_t i = 0; i < n && !nan; ++i) nan = x[i] != x[i];
  if (nan) {
    std_sort(order, 0, n, LessKey{x, true});
    return HBX_OK;
  }
  qsort64(x, order, n);
  return HBX_OK;
}

// HB_iteration.py:180-182 for one bracket on the host: advance[i] = (argsort(argsort(loss)) < k)[i], i.e.
// the first k positions of numpy's argsort (the same set; only the ranges straddling the k-th place are
// sorted); scratch: host i64[n]
int hbx_sh_advance_host(const double* loss, int64_t n, int64_t k, uint8_t* advance, int64_t* scratch) {
  if (n < 0 || (n > 0 && (!loss || !advance || !scratch)))
    return hbx_fail(HBX_ERR_ARG, "hbx_sh_advance_host: bad arguments");
  for (int64_t i = 0; i < n; ++i) scratch[i] = i;
  bool nan = false;
  for (int64_t i = 0; i < n && !nan; ++i) nan = loss[i] != loss[i];
  if (nan)
    std_sort(scratch, 0, n, LessKey{loss, true});
  else if (n > 1)
    qsort64(loss, scratch, n, k < 0 ? 0 : k);
  memset(advance, 0, (size_t)n);
  for (int64_t j = 0; j < n && j < k; ++j) advance[scratch[j]] = 1;
  return HBX_OK;
}

}  // extern "C"
