"""ORACLE -- test infrastructure only (see kde_oracle.py's header for who may import it).

numpy 1.26.4's default ``np.argsort`` of float64 data on an AVX-512 (AVX512_SKX) host, restated step
for step, so that its order among TIED keys can be reproduced.  The reference splits BOHB's losses
with ``np.argsort(losses)`` (bohb.py:229) and ranks a successive-halving stage with
``np.argsort(np.argsort(losses))`` (HB_iteration.py:180); both are numpy's default, unstable sort.
Crashed runs all have loss +inf (bohb.py:189-192) and quantised losses tie too, so the rows the
reference puts into each KDE -- and in which order -- depend on how this particular sort breaks ties.

Third-party pin: numpy 1.26.4 (the fixtures' interpreter, tests/golden/PROVENANCE.json) dispatches
``aquicksort_double`` to ``np::qsort_simd::ArgQSort_AVX512_SKX`` = the vendored x86-simd-sort
``avx512_argsort<double>`` (numpy/core/src/npysort/x86-simd-sort, src/avx512-64bit-argsort.hpp):

* NaN present -> ``std::sort`` of the indices with a NaN-last comparator (libstdc++ introsort);
* else ``argsort_64bit_(arr, arg, 0, n-1, 2*floor(log2 n))``: quicksort whose partition moves 8-index
  vectors with compress-stores (``partition_avx512``: keys >= pivot go right, in lane order), pivot =
  median (5th smallest) of 8 keys sampled at a stride of (right-left)/8, ranges of <= 64 sorted by
  the bitonic key/index networks ``argsort_{8,16,32,64}_64bit`` (padding lanes +inf, index 0; a
  compare-exchange never swaps equal keys), and ``std::sort`` once the depth budget is spent.

Pinned by ``tests/golden/np_argsort.npz`` (numpy 1.26.4 outputs on tie-heavy inputs, written by
``tests/golden/gen_np_argsort.py``) in ``tests/test_oracle_golden.py``.
"""

import math

import numpy as np

# --- 8-lane register model ------------------------------------------------------------------------
# A register is a list of 8 (key, index) lanes.  Permutations follow the intrinsics: permutexvar(idx, v)
# gives lane i = v[idx[i]]; _mm512_set_epi64 lists lanes from 7 down to 0.


def _seti(*hi_to_lo):
    return list(reversed(hi_to_lo))


NET1 = _seti(4, 5, 6, 7, 0, 1, 2, 3)   # reverse within each half
NET2 = _seti(0, 1, 2, 3, 4, 5, 6, 7)   # reverse
NET3 = _seti(5, 4, 7, 6, 1, 0, 3, 2)   # exchange at distance 2
NET4 = _seti(3, 2, 1, 0, 7, 6, 5, 4)   # exchange at distance 4
SWAP1 = [1, 0, 3, 2, 5, 4, 7, 6]       # shuffle<SHUFFLE_MASK(1,1,1,1)>: exchange neighbours


def _perm(v, idx):
    return [v[i] for i in idx]


def _cmp_merge(v, idx, mask):
    """cmp_merge(v, permuted v, mask): lanes with the mask bit take the max, the others the min; a lane
    keeps its own index where the chosen key equals its own key (so equal keys never swap)."""
    w = _perm(v, idx)
    out = []
    for i in range(8):
        a, b = v[i], w[i]
        if (mask >> i) & 1:
            k = max(a[0], b[0])
        else:
            k = min(a[0], b[0])
        out.append((k, a[1] if k == a[0] else b[1]))
    return out


def _coex(x, y):
    """COEX of two registers lane by lane: x gets the min, y the max; ties keep their places."""
    lo, hi = [], []
    for a, b in zip(x, y):
        if b[0] < a[0]:
            lo.append(b)
            hi.append(a)
        else:
            lo.append(a)
            hi.append(b)
    return lo, hi


def _sort_zmm(v):
    v = _cmp_merge(v, SWAP1, 0xAA)
    v = _cmp_merge(v, NET1, 0xCC)
    v = _cmp_merge(v, SWAP1, 0xAA)
    v = _cmp_merge(v, NET2, 0xF0)
    v = _cmp_merge(v, NET3, 0xCC)
    v = _cmp_merge(v, SWAP1, 0xAA)
    return v


def _merge_zmm(v):
    v = _cmp_merge(v, NET4, 0xF0)
    v = _cmp_merge(v, NET3, 0xCC)
    v = _cmp_merge(v, SWAP1, 0xAA)
    return v


def _rev(v):
    return _perm(v, NET2)


def _merge_two(r):
    a, b = _coex(r[0], _rev(r[1]))
    return [_merge_zmm(a), _merge_zmm(_rev(b))]


def _merge_four(r):
    t1, m1 = _coex(r[0], _rev(r[3]))
    t2, m2 = _coex(r[1], _rev(r[2]))
    t3, t4 = _rev(m2), _rev(m1)
    z0, z1 = _coex(t1, t2)
    z2, z3 = _coex(t3, t4)
    return [_merge_zmm(z) for z in (z0, z1, z2, z3)]


def _merge_eight(r):
    t1, m1 = _coex(r[0], _rev(r[7]))
    t2, m2 = _coex(r[1], _rev(r[6]))
    t3, m3 = _coex(r[2], _rev(r[5]))
    t4, m4 = _coex(r[3], _rev(r[4]))
    t5, t6, t7, t8 = _rev(m4), _rev(m3), _rev(m2), _rev(m1)
    t1, t3 = _coex(t1, t3)
    t2, t4 = _coex(t2, t4)
    t5, t7 = _coex(t5, t7)
    t6, t8 = _coex(t6, t8)
    t1, t2 = _coex(t1, t2)
    t3, t4 = _coex(t3, t4)
    t5, t6 = _coex(t5, t6)
    t7, t8 = _coex(t7, t8)
    return [_merge_zmm(z) for z in (t1, t2, t3, t4, t5, t6, t7, t8)]


def _argsort_small(arr, arg, lo, N):
    """argsort_{8,16,32,64}_64bit on arg[lo:lo+N] (N <= 64): registers of 8 lanes, full ones first,
    padding lanes (key +inf, index 0) in the masked tail registers; only the first N lanes are stored."""
    nreg = 1 if N <= 8 else 2 if N <= 16 else 4 if N <= 32 else 8
    regs = []
    for r in range(nreg):
        reg = []
        for l in range(8):
            p = 8 * r + l
            if p < N:
                ix = int(arg[lo + p])
                reg.append((arr[ix], ix))
            else:
                reg.append((math.inf, 0))
        regs.append(_sort_zmm(reg))
    if nreg >= 2:
        for r in range(0, nreg, 2):
            regs[r:r + 2] = _merge_two(regs[r:r + 2])
    if nreg >= 4:
        for r in range(0, nreg, 4):
            regs[r:r + 4] = _merge_four(regs[r:r + 4])
    if nreg == 8:
        regs = _merge_eight(regs)
    flat = [e for reg in regs for e in reg]
    for p in range(N):
        arg[lo + p] = flat[p][1]


# --- libstdc++ std::sort (introsort), the fallbacks ----------------------------------------------

def _std_sort(arg, first, last, less):
    """std::sort(arg + first, arg + last, less) as libstdc++ implements it (bits/stl_algo.h):
    __introsort_loop (threshold 16, depth 2*floor(log2 n), median-of-three pivot moved to first,
    unguarded partition, heap sort when the depth runs out) then __final_insertion_sort."""
    if first == last:
        return
    _introsort_loop(arg, first, last, 2 * (int(last - first).bit_length() - 1), less)
    _final_insertion_sort(arg, first, last, less)


def _move_median_to_first(arg, result, a, b, c, less):
    if less(arg[a], arg[b]):
        if less(arg[b], arg[c]):
            arg[result], arg[b] = arg[b], arg[result]
        elif less(arg[a], arg[c]):
            arg[result], arg[c] = arg[c], arg[result]
        else:
            arg[result], arg[a] = arg[a], arg[result]
    elif less(arg[a], arg[c]):
        arg[result], arg[a] = arg[a], arg[result]
    elif less(arg[b], arg[c]):
        arg[result], arg[c] = arg[c], arg[result]
    else:
        arg[result], arg[b] = arg[b], arg[result]


def _unguarded_partition(arg, first, last, pivot, less):
    while True:
        while less(arg[first], arg[pivot]):
            first += 1
        last -= 1
        while less(arg[pivot], arg[last]):
            last -= 1
        if not first < last:
            return first
        arg[first], arg[last] = arg[last], arg[first]
        first += 1


def _introsort_loop(arg, first, last, depth, less):
    while last - first > 16:
        if depth == 0:
            _partial_sort_heap(arg, first, last, less)
            return
        depth -= 1
        mid = first + (last - first) // 2
        _move_median_to_first(arg, first, first + 1, mid, last - 1, less)
        cut = _unguarded_partition(arg, first + 1, last, first, less)
        _introsort_loop(arg, cut, last, depth, less)
        last = cut


def _adjust_heap(arg, first, hole, length, value, less):
    top = hole
    child = hole
    while child < (length - 1) // 2:
        child = 2 * (child + 1)
        if less(arg[first + child], arg[first + child - 1]):
            child -= 1
        arg[first + hole] = arg[first + child]
        hole = child
    if (length & 1) == 0 and child == (length - 2) // 2:
        child = 2 * (child + 1)
        arg[first + hole] = arg[first + child - 1]
        hole = child - 1
    parent = (hole - 1) // 2
    while hole > top and less(arg[first + parent], value):
        arg[first + hole] = arg[first + parent]
        hole = parent
        parent = (hole - 1) // 2
    arg[first + hole] = value


def _partial_sort_heap(arg, first, last, less):
    """std::__partial_sort(first, last, last): make_heap then sort_heap."""
    n = last - first
    if n >= 2:
        parent = (n - 2) // 2
        while True:
            _adjust_heap(arg, first, parent, n, arg[first + parent], less)
            if parent == 0:
                break
            parent -= 1
    while last - first > 1:
        last -= 1
        value = arg[last]
        arg[last] = arg[first]
        _adjust_heap(arg, first, 0, last - first, value, less)


def _insertion_sort(arg, first, last, less):
    if first == last:
        return
    for i in range(first + 1, last):
        val = arg[i]
        if less(val, arg[first]):
            arg[first + 1:i + 1] = arg[first:i].copy()
            arg[first] = val
        else:
            j = i
            while less(val, arg[j - 1]):
                arg[j] = arg[j - 1]
                j -= 1
            arg[j] = val


def _unguarded_insertion_sort(arg, first, last, less):
    for i in range(first, last):
        val = arg[i]
        j = i
        while less(val, arg[j - 1]):
            arg[j] = arg[j - 1]
            j -= 1
        arg[j] = val


def _final_insertion_sort(arg, first, last, less):
    if last - first > 16:
        _insertion_sort(arg, first, first + 16, less)
        _unguarded_insertion_sort(arg, first + 16, last, less)
    else:
        _insertion_sort(arg, first, last, less)


# --- x86-simd-sort quicksort ----------------------------------------------------------------------

def _pivot(arr, arg, left, right):
    """get_pivot_64bit: the 5th smallest of the keys at left + k*size, k = 1..8 (size = (right-left)/8)."""
    if right - left >= 8:
        size = (right - left) // 8
        s = sorted(arr[arg[left + k * size]] for k in range(1, 9))
        return s[4]
    return arr[arg[right]]


def _partition_vec(arr, arg, l_store, r_end, vec):
    """partition_vec: keys >= pivot compress-stored ending at r_end, the rest from l_store, lane order."""
    ge = [ix for ix in vec if arr[ix] >= _partition_vec.pivot]
    lt = [ix for ix in vec if not arr[ix] >= _partition_vec.pivot]
    arg[l_store:l_store + len(lt)] = lt
    arg[r_end - len(ge):r_end] = ge
    return len(ge)


def _partition(arr, arg, left, right, pivot, unroll):
    """partition_avx512 (unroll 1) / partition_avx512_unrolled<4> over arg[left:right]; returns
    (pivot index, smallest, biggest)."""
    smallest, biggest = math.inf, -math.inf
    _partition_vec.pivot = pivot
    if unroll > 1 and right - left <= 8 * unroll * 8:
        unroll = 1
    U = 8 * unroll
    for _ in range((right - left) % U):
        v = arr[arg[left]]
        smallest = min(smallest, v)
        biggest = max(biggest, v)
        if not v < pivot:
            right -= 1
            arg[left], arg[right] = arg[right], arg[left]
        else:
            left += 1
    if left == right:
        return left, smallest, biggest
    seen = [arr[ix] for ix in arg[left:right]]
    smallest = min(smallest, min(seen))
    biggest = max(biggest, max(seen))
    if unroll == 1 and right - left == 8:
        c = _partition_vec(arr, arg, left, left + 8, list(arg[left:left + 8]))
        return left + (8 - c), smallest, biggest
    vl = [list(arg[left + 8 * i:left + 8 * i + 8]) for i in range(unroll)]
    vr = [list(arg[right - 8 * (unroll - i):right - 8 * (unroll - i) + 8]) for i in range(unroll)]
    r_store = right - 8
    l_store = left
    left += U
    right -= U
    while right - left != 0:
        if (r_store + 8) - right < left - l_store:
            right -= U
            grp = [list(arg[right + 8 * i:right + 8 * i + 8]) for i in range(unroll)]
        else:
            grp = [list(arg[left + 8 * i:left + 8 * i + 8]) for i in range(unroll)]
            left += U
        for vec in grp:
            c = _partition_vec(arr, arg, l_store, r_store + 8, vec)
            l_store += 8 - c
            r_store -= c
    if unroll == 1:
        c = _partition_vec(arr, arg, l_store, r_store + 8, vl[0])
        l_store += 8 - c
        c = _partition_vec(arr, arg, l_store, l_store + 8, vr[0])
        l_store += 8 - c
        return l_store, smallest, biggest
    for vec in vl + vr:
        c = _partition_vec(arr, arg, l_store, r_store + 8, vec)
        l_store += 8 - c
        r_store -= c
    return l_store, smallest, biggest


def _less_key(arr):
    return lambda a, b: arr[a] < arr[b]


def _less_nan_last(arr):
    def less(a, b):
        x, y = arr[a], arr[b]
        if x == x and y == y:
            return x < y
        if x != x:
            return False
        return True
    return less


def _qsort(arr, arg, left, right, max_iters, unroll):
    # explicit stack: disjoint ranges, so the processing order does not change the result
    stack = [(left, right, max_iters)]
    while stack:
        left, right, it = stack.pop()
        if it <= 0:
            _std_sort(arg, left, right + 1, _less_key(arr))
            continue
        if right + 1 - left <= 64:
            _argsort_small(arr, arg, left, right + 1 - left)
            continue
        pivot = _pivot(arr, arg, left, right)
        pidx, smallest, biggest = _partition(arr, arg, left, right + 1, pivot, unroll)
        if pivot != smallest:
            stack.append((left, pidx - 1, it - 1))
        if pivot != biggest:
            stack.append((pidx, right, it - 1))


UNROLL = 4  # partition_avx512_unrolled<vtype, 4> (ranges > 256 keys)


def argsort(a):
    """np.argsort(a) (kind='quicksort', the default) of a 1-D float64 array, numpy 1.26.4 AVX512_SKX."""
    arr = [float(v) for v in np.asarray(a, dtype=np.float64).reshape(-1)]
    n = len(arr)
    arg = np.arange(n, dtype=np.int64)
    if n <= 1:
        return arg
    if any(v != v for v in arr):
        _std_sort(arg, 0, n, _less_nan_last(arr))
        return arg
    _qsort(arr, arg, 0, n - 1, 2 * int(math.log2(n)), UNROLL)
    return arg


def ranks_advance(losses, k):
    """HB_iteration.py:180-182: argsort(argsort(losses)) < k -- the first k of the inner argsort."""
    o = argsort(losses)
    adv = np.zeros(len(o), dtype=bool)
    adv[o[:k]] = True
    return adv
