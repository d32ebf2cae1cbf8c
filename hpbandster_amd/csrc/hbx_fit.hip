// hbx_fit.hip -- batched BOHB KDE refit on MI355X: per-budget (segment) stable argsort of the
// losses, good/bad split and normal-reference bandwidths + observed level counts.
//
// Reference: bohb.py:220-246 (argsort, good = head, bad = tail, KDEMultivariate(..., 'normal_reference'))
// -> SM:_kernel_base.py:250-265 (bw = 1.06 * np.std(X, axis=0) * n**(-1/(4+D))) and
// SM:kernels.py:59-60 (num_levels = np.unique(column).size).
//
// Bit-exactness: np.std(X, axis=0) is reproduced operation for operation -- mean = sum / n,
// var = sum((x - mean)^2) / n, sqrt -- with numpy's reduction order: sequential down each column
// for D > 1, and (D == 1, where numpy reduces a contiguous vector) pairwise summation over
// 8192-element buffers.  The factor n**(-1/(4+D)) is a host-side glibc pow() per segment, passed in,
// because the device pow() is not guaranteed to round the same way.
#include "hbx_common.h"
#include "hbx_kde_impl.h"
#include "hbx_npsort.h"
#include "hbx_sort.h"
#include <stdlib.h>
#include <string.h>
#include <stddef.h>
#include <type_traits>

__device__ double np_pairwise_gather(const double* X, int32_t D, int32_t d, const int64_t* rows, int64_t n,
                                     double mean, bool sq);

// sum of (x) or ((x - mean)^2) over a gathered column, numpy pairwise order (one leaf <= 128)
__device__ double pw_leaf(const double* X, int32_t D, int32_t d, const int64_t* rows, int64_t n, double mean,
                          bool sq) {
  auto v = [&](int64_t i) -> double {
    const double x = X[rows[i] * (int64_t)D + d];
    if (!sq) return x;
    const double t = x - mean;
    return t * t;
  };
  if (n < 8) {
    double res = 0.0;
    for (int64_t i = 0; i < n; ++i) res += v(i);
    return res;
  }
  double r0 = v(0), r1 = v(1), r2 = v(2), r3 = v(3), r4 = v(4), r5 = v(5), r6 = v(6), r7 = v(7);
  int64_t i;
  for (i = 8; i < n - (n % 8); i += 8) {
    r0 += v(i + 0); r1 += v(i + 1); r2 += v(i + 2); r3 += v(i + 3);
    r4 += v(i + 4); r5 += v(i + 5); r6 += v(i + 6); r7 += v(i + 7);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += v(i);
  return res;
}

__device__ double np_pairwise_gather(const double* X, int32_t D, int32_t d, const int64_t* rows, int64_t n,
                                     double mean, bool sq) {
  if (n <= 128) return pw_leaf(X, D, d, rows, n, mean, sq);
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  // depth <= log2(8192/128) + 1 here (called per 8192 buffer) -> bounded recursion
  return np_pairwise_gather(X, D, d, rows, n2, mean, sq) +
         np_pairwise_gather(X, D, d, rows + n2, n - n2, mean, sq);
}

__device__ double np_sum_column(const double* X, int32_t D, int32_t d, const int64_t* rows, int64_t n,
                                double mean, bool sq) {
  if (D > 1) {  // axis-0 reduction of an (n, D) C-array: sequential down the column
    // the additions stay strictly in row order; only the (independent) gathers are batched, so 16
    // loads are in flight per round trip instead of one
    constexpr int U = 16;
    double acc = 0.0;
    int64_t i = 0;
    for (; i + U <= n; i += U) {
      int64_t rr[U];
      double v[U];
#pragma unroll
      for (int k = 0; k < U; ++k) rr[k] = rows[i + k];
#pragma unroll
      for (int k = 0; k < U; ++k) v[k] = X[rr[k] * (int64_t)D + d];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (sq) {
          const double t = v[k] - mean;
          acc = acc + t * t;
        } else {
          acc = acc + v[k];
        }
      }
    }
    for (; i < n; ++i) {
      const double x = X[rows[i] * (int64_t)D + d];
      if (sq) {
        const double t = x - mean;
        acc = acc + t * t;
      } else {
        acc = acc + x;
      }
    }
    return acc;
  }
  double acc = 0.0;  // contiguous vector: pairwise per 8192-element ufunc buffer
  for (int64_t c = 0; c < n; c += 8192)
    acc = acc + np_pairwise_gather(X, D, d, rows + c, (n - c) < 8192 ? (n - c) : 8192, mean, sq);
  return acc;
}

// one workgroup per segment: stable argsort of the segment's losses
__global__ __launch_bounds__(256) void seg_argsort_kernel(const double* __restrict__ loss,
                                                          const int64_t* __restrict__ seg_off, int tile,
                                                          uint64_t* gk, int32_t* gi, uint64_t* gk2, int32_t* gi2,
                                                          int64_t* __restrict__ order) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint64_t* lk = (uint64_t*)smem;
  int32_t* li = (int32_t*)(smem + sizeof(uint64_t) * tile);
  const int64_t b = blockIdx.x;
  const int64_t s = seg_off[b], e = seg_off[b + 1];
  block_sort_segment<false>(loss + s, e - s, tile, lk, li, gk + s, gi + s, gk2 + s, gi2 + s, order + s);
}

// segments of up to 1024 losses: one wave each, sorted in registers (wave_sort_1024).  list / count (numpy's
// tie order, nullable): a segment whose sorted keys hold two equal neighbours joins `list` -- the sorted keys
// are in the wave's registers, so the tie check reads no memory (seg_tie_flag_kernel re-gathered every key)
#ifndef SORT_WPE
#define SORT_WPE 4
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SORT_WPE))) void seg_argsort_wave_kernel(const double* __restrict__ loss,
                                                               const int64_t* __restrict__ seg_off, int64_t B,
                                                               int64_t* __restrict__ order, int32_t* list,
                                                               int32_t* count) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // whole wave
  const int64_t s = seg_off[b];
  const int n = (int)(seg_off[b + 1] - s);
  uint64_t key[PW_PER_LANE];
  int32_t pos[PW_PER_LANE];
  wave_sort_1024<false>(loss + s, n, lane, key, pos);
#pragma unroll
  for (int r = 0; r < PW_PER_LANE; ++r) {
    const int rank = lane * PW_PER_LANE + r;
    if (rank < n) order[s + rank] = pos[r];
  }
  if (list) {  // adjacent sorted ranks with equal keys (hbx_d2ord: -0.0 == 0.0, every NaN one key)
    bool tie = false;
#pragma unroll
    for (int r = 0; r + 1 < PW_PER_LANE; ++r) tie |= lane * PW_PER_LANE + r + 1 < n && key[r] == key[r + 1];
    const uint64_t nxt = __shfl_down(key[0], 1);  // the next lane's first rank
    tie |= lane < 63 && (lane + 1) * PW_PER_LANE < n && key[PW_PER_LANE - 1] == nxt;
    if (__ballot(tie) && lane == 0) list[atomicAdd(count, 1)] = (int32_t)b;
  }
}

// Segments of 1024 < n <= RANK_MAX_SEG: stable rank by counting, spread over many workgroups.
// rank(i) = #{j : (key_j, j) < (key_i, i)} -- a total order, so the ranks are a permutation and
// order[rank(i)] = i is the stable argsort.  Grid (i blocks of 256, j chunks of RANK_J, segment):
// each workgroup counts one j chunk (staged in LDS) for its 256 elements and adds the partial counts
// into rank[] (zeroed first); a second kernel scatters order[rank(i)] = i.  O(n^2) compares on every
// CU at once instead of one workgroup's merge passes.
#define RANK_J 512
#define RANK_MAX_SEG 65536
__global__ __launch_bounds__(256) void seg_rank_count_kernel(const double* __restrict__ loss,
                                                             const int64_t* __restrict__ seg_off,
                                                             int32_t* __restrict__ rank) {
  __shared__ uint64_t kt[RANK_J];
  const int64_t b = blockIdx.z;
  const int64_t s = seg_off[b];
  const int n = (int)(seg_off[b + 1] - s);
  const int j0 = blockIdx.y * RANK_J;
  if ((int)blockIdx.x * 256 >= n || j0 >= n) return;  // whole block
  const int m = (n - j0) < RANK_J ? (n - j0) : RANK_J;
  for (int t = threadIdx.x; t < m; t += 256) kt[t] = key_argsort(loss[s + j0 + t]);
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t ki = key_argsort(loss[s + i]);
  // j < i (j = j0 + t): equal keys count too; j >= i: only strictly smaller keys
  const int split = i - j0 < 0 ? 0 : (i - j0 > m ? m : i - j0);
  int c = 0;
#pragma unroll 8
  for (int t = 0; t < split; ++t) c += kt[t] <= ki;
#pragma unroll 8
  for (int t = split; t < m; ++t) c += kt[t] < ki;
  if (c) atomicAdd(rank + s + i, c);
}

__global__ __launch_bounds__(256) void seg_rank_scatter_kernel(const int64_t* __restrict__ seg_off,
                                                               const int32_t* __restrict__ rank,
                                                               int64_t* __restrict__ order) {
  const int64_t b = blockIdx.y;
  const int64_t s = seg_off[b];
  const int n = (int)(seg_off[b + 1] - s);
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) order[s + rank[s + i]] = i;
}

// ---- numpy's tie order (hbx_npsort.h) ------------------------------------------------------------
// One wave per segment: does the stable order hold tied keys?  -> the segment joins `list`.
//   promote = 0 (argsort): any two equal keys (hbx_d2ord: -0.0 == 0.0, every NaN one key);
//   promote = 1 (promotion ranks over the finite losses, which the stable order puts first): with the
//   order wanted, any two equal finite keys; for the mask alone, equal keys at ranks kk-1 and kk.
__global__ __launch_bounds__(256) void seg_tie_flag_kernel(const double* __restrict__ loss,
                                                           const int64_t* __restrict__ seg_off, int64_t B,
                                                           const int64_t* __restrict__ order,
                                                           const double* __restrict__ k, int promote,
                                                           int want_order, int32_t* __restrict__ list,
                                                           int32_t* __restrict__ count) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // whole wave
  const int64_t s = seg_off[b];
  const int n = (int)(seg_off[b + 1] - s);
  auto key = [&](int r) -> uint64_t {
    const double v = loss[s + order[s + r]];
    return promote ? key_promote(v) : key_argsort(v);
  };
  bool tie = false;
  if (!promote || want_order) {
    for (int i = lane; i + 1 < n; i += 64) {
      const uint64_t a = key(i), c = key(i + 1);
      tie |= a == c && (!promote || a != ~0ull);
    }
  } else {
    int nf = 0;
    for (int i = lane; i < n; i += 64) nf += key(i) != ~0ull;
    for (int o = 32; o > 0; o >>= 1) nf += __shfl_xor(nf, o);
    const double kb = k[b];
    const int kk = kb > 0.0 ? (kb >= (double)nf ? nf : (int)ceil(kb)) : 0;
    tie = lane == 0 && kk > 0 && kk < nf && key(kk - 1) == key(kk);
  }
  if (__ballot(tie) && lane == 0) list[atomicAdd(count, 1)] = (int32_t)b;
}

// Few segments (a single refit's split): one thread per adjacent pair of the sorted order over a 2-D
// grid (pair chunks x segments) -- one wave per segment would walk 1e4 dependent gathers in a row; the
// first block to see a tie in segment b claims flags[b] and appends b (flags: B <= 15 ints, zeroed)
__global__ __launch_bounds__(256) void seg_tie_flag_wide_kernel(const double* __restrict__ loss,
                                                                const int64_t* __restrict__ seg_off,
                                                                const int64_t* __restrict__ order,
                                                                int32_t* __restrict__ flags,
                                                                int32_t* __restrict__ list,
                                                                int32_t* __restrict__ count) {
  const int64_t b = blockIdx.y;
  const int64_t s = seg_off[b];
  const int n = (int)(seg_off[b + 1] - s);
  const int i = blockIdx.x * 256 + threadIdx.x;
  bool tie = false;
  if (i + 1 < n) tie = key_argsort(loss[s + order[s + i]]) == key_argsort(loss[s + order[s + i + 1]]);
  __shared__ int any;
  if (threadIdx.x == 0) any = 0;
  __syncthreads();
  if (__ballot(tie) && (threadIdx.x & 63) == 0) any = 1;
  __syncthreads();
  if (threadIdx.x == 0 && any && atomicCAS(flags + b, 0, 1) == 0) list[atomicAdd(count, 1)] = (int32_t)b;
}

// The flagged segments, one workgroup each (grid-stride over the list): A[0, m) = the positions to
// rank -- every position (argsort), or the finite losses' in position order (promotion) -- sorted in
// numpy's order.  Scratch arrays A/T/W/Lst are indexed by the segment's offset (slot_stride == 0) or
// by the block (slot_stride elements per block: a fixed pool).
__global__ __launch_bounds__(NPS_THREADS) void seg_np_order_kernel(
    const double* __restrict__ loss, const int64_t* __restrict__ seg_off, const double* __restrict__ k,
    const int32_t* __restrict__ list, const int32_t* __restrict__ count, int32_t* A0, int32_t* T0, int32_t* W0,
    int32_t* L0, int64_t slot_stride, int promote, int64_t* __restrict__ order, uint8_t* __restrict__ advance) {
  const int c = *count;
  for (int q = blockIdx.x; q < c; q += gridDim.x) {
    const int64_t b = list[q];
    const int64_t s = seg_off[b];
    const int n = (int)(seg_off[b + 1] - s);
    const int64_t o = slot_stride ? (int64_t)blockIdx.x * slot_stride : s;
    nps_order_segment(loss + s, n, promote, promote ? k[b] : 0.0, A0 + o, T0 + o, W0 + o, L0 + o,
                      order ? order + s : nullptr, advance ? advance + s : nullptr);
  }
}

// host: flag the segments of a stable order that hold ties, then re-rank them in numpy's order.
// arrays: int32 [A | T | W | Lst], `slots` entries each -- slot_stride 0: indexed by segment offset
// (slots = N), else a pool of slots / slot_stride blocks; cnt_list: int32 [16] counter + the list (<= B)
// (flagged: the list is filled already -- sh_select_kernel flags its tie-straddling brackets itself)
int hbx_np_order_fix(const double* loss, const int64_t* seg_off, int64_t B, int64_t max_seg, const int64_t* order_in,
                     const double* k, int promote, int want_order, int64_t* order_out, uint8_t* advance,
                     int32_t* arrays, int64_t slots, int64_t slot_stride, int32_t* cnt_list, bool flagged,
                     hipStream_t s) {
  int32_t* A = arrays;
  int32_t* T = A + slots;
  int32_t* W = T + slots;
  int32_t* L = W + slots;
  int32_t* cnt = cnt_list;
  int32_t* list = cnt_list + 16;
  if (!flagged) {
    // argsort mode, a few segments: the wide kernel (its per-segment claim flags sit in cnt_list[1..])
    const bool wide = !promote && B <= 15 && max_seg > 256;
    HBX_HIP(hipMemsetAsync(cnt, 0, sizeof(int32_t) * (wide ? 16 : 1), s));
    if (wide) {
      hipLaunchKernelGGL(seg_tie_flag_wide_kernel, dim3((unsigned)((max_seg + 255) / 256), (unsigned)B), dim3(256), 0,
                         s, loss, seg_off, order_in, cnt + 1, list, cnt);
    } else {
      hipLaunchKernelGGL(seg_tie_flag_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, loss, seg_off, B,
                         order_in, k, promote, want_order, list, cnt);
    }
    HBX_LAUNCH_CHECK();
  }
  const int64_t nblk = slot_stride ? slots / slot_stride : (B < 1024 ? B : 1024);
  hipLaunchKernelGGL(seg_np_order_kernel, dim3((unsigned)(nblk > 0 ? nblk : 1)), dim3(NPS_THREADS), 0, s, loss,
                     seg_off, k, list, cnt, A, T, W, L, slot_stride, promote, order_out, advance);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

// One refit of n <= REFIT_SORT_SMALL rows in one workgroup (hbx_kde_refit; bohb.py:211-229): append the
// n_new staged rows ([n_new][D] then n_new losses) at rows n - n_new .. n - 1, write the split metadata,
// sort the losses (wave 0: the register network, ties by position), and -- only when two sorted keys are
// equal -- re-rank the whole segment in numpy 1.26.4's order (hbx_npsort.h, every thread).  The same
// order as the metadata kernel + counting rank + scatter + tie check + numpy-order launches it replaces.
struct RefitSortArgs {
  double* X;
  double* loss;
  const double* staged;  // device rows to append (nullptr: the inline copy below)
  int64_t n_new;
  RefitMetaArgs a;
  RefitMeta* m;
  int64_t* order;
  int32_t* A0;
  double inl[REFIT_INLINE];  // the appended rows then their losses, when they fit (no host-to-device copy)
};

// SORT_STAMPS (diagnostic builds only): s_memtime at the phase boundaries of the one-launch refit sort (thread 0)
#ifdef SORT_STAMPS
__device__ unsigned long long sort_stamps[16];
#define SSTAMP(i) \
  if (threadIdx.x == 0) sort_stamps[i] = __builtin_amdgcn_s_memtime()
extern "C" int hbx_debug_sort_stamps(unsigned long long* out) {
  HBX_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(sort_stamps), sizeof(sort_stamps)));
  return HBX_OK;
}
#else
#define SSTAMP(i)
#endif

// PW losses per lane (runs of 64 PW): 2 while n <= 512 (the shorter network and searches), else 4
template <int PW>
__global__ __launch_bounds__(NPS_THREADS) void kde_refit_sort_small_kernel(RefitSortArgs g) {
  SSTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const RefitMetaArgs& a = g.a;
  double* __restrict__ X = g.X;
  double* __restrict__ loss = g.loss;
  RefitMeta* __restrict__ m = g.m;
  int64_t* __restrict__ order = g.order;
  int32_t* A0 = g.A0;
  const int64_t n_new = g.n_new;
  // the inline rows read in place from the kernel-argument segment (indexing the by-value argument would copy
  // it to scratch)
  const double* inl =
      (const double*)((const char*)__builtin_amdgcn_kernarg_segment_ptr() + offsetof(RefitSortArgs, inl));
  const int n = (int)a.n;
  const int64_t per = n_new * (int64_t)a.D;
  for (int64_t e = tid; e < per + n_new; e += NPS_THREADS) {
    const double v = g.staged ? g.staged[e] : inl[e];
    if (e < per) X[(a.n - n_new) * (int64_t)a.D + e] = v;
    else loss[a.n - n_new + (e - per)] = v;
  }
  for (int d = tid; d < a.D; d += NPS_THREADS) m->vt[d] = (a.vt[d >> 5] >> (d & 31)) & 1u;
  if (tid == 0) {
    m->seg[0] = 0;
    m->seg[1] = a.n;
    m->n_good = a.n_good;
    m->n_bad = a.n_bad;
    m->fac_good = a.fac_good;
    m->fac_bad = a.fac_bad;
  }
  __shared__ uint64_t rk[REFIT_SORT_SMALL];  // the four waves' sorted runs, then the keys by rank
  SSTAMP(1);
  __syncthreads();  // the appended losses are visible to every wave
  SSTAMP(2);
  // each wave sorts its run of 256 losses in registers (a quarter of one wave's 1024-network), the runs are
  // merged by rank: an element's rank is its place in its run plus, in each other run, the count of (key,
  // position) pairs below it (binary searches in LDS); positions are distinct, so the ranks are a permutation
  static_assert(PW * NPS_THREADS <= REFIT_SORT_SMALL, "runs beyond the LDS arrays");
  const int w = tid >> 6;
  uint64_t key[PW];
  int32_t pos[PW];
  wave_sort_run<false, PW>(loss, 64 * PW * w, n, lane, key, pos);
  SSTAMP(3);
#pragma unroll
  for (int r = 0; r < PW; ++r) {
    rk[64 * PW * w + PW * lane + r] = key[r];
  }
  __syncthreads();
  // count of entries of each other run below (key, pos).  Run v holds positions [RUN v, RUN v + RUN), so against
  // an earlier run (v < w) that is the count of keys <= key, against a later one the count of keys < key: the
  // keys alone decide.  A fixed-step search over the run's real entries (b = 256, 128, .., 1: step b adds b when
  // entry c + b - 1 counts), every (run, register) chain advanced together -- one LDS round trip per step for
  // all of them, not a dependent loop per element
  constexpr int NR = NPS_THREADS / 64, RUN = 64 * PW;
  int cnt[NR][PW];
#pragma unroll
  for (int v = 0; v < NR; ++v)
#pragma unroll
    for (int r = 0; r < PW; ++r) cnt[v][r] = 0;
#pragma unroll
  for (int b = RUN; b > 0; b >>= 1) {
#pragma unroll
    for (int v = 0; v < NR - 1; ++v) {
      const int vr = v < w ? v : v + 1;  // the other runs
      const int len = min(max(n - RUN * vr, 0), RUN);
#pragma unroll
      for (int r = 0; r < PW; ++r) {
        const int c = cnt[v][r] + b - 1;
        if (c < len) {
          const uint64_t e = rk[RUN * vr + c];
          if (vr < w ? e <= key[r] : e < key[r]) cnt[v][r] += b;
        }
      }
    }
  }
  int rank[PW];
#pragma unroll
  for (int r = 0; r < PW; ++r) {
    rank[r] = PW * lane + r;
#pragma unroll
    for (int v = 0; v < NR - 1; ++v) rank[r] += cnt[v][r];
  }
  SSTAMP(4);
  __syncthreads();  // every run read
#pragma unroll
  for (int r = 0; r < PW; ++r) {
    if (pos[r] != 0x7fffffff) {  // a real element: rank < n
      rk[rank[r]] = key[r];
      order[rank[r]] = pos[r];
    }
  }
  SSTAMP(5);
  __syncthreads();
  int t = 0;
  for (int i = tid; i + 1 < n; i += NPS_THREADS) t |= rk[i] == rk[i + 1];
  if (__syncthreads_or(t))  // tied losses: every position re-ranked in numpy's order
    nps_order_segment(loss, n, 0, 0.0, A0, A0 + n, A0 + 2 * n, A0 + 3 * n, order, nullptr);
  SSTAMP(6);
}

int refit_sort_small(double* X, double* loss, const double* staged, const double* staged_inline, int64_t n_new,
                     const RefitMetaArgs& a, RefitMeta* m, int64_t* order, int32_t* arrays, hipStream_t s) {
  if (a.n < 1 || a.n > REFIT_SORT_SMALL) return hbx_fail(HBX_ERR_ARG, "refit_sort_small: n=%lld", (long long)a.n);
  RefitSortArgs g;
  memset(&g, 0, offsetof(RefitSortArgs, inl));
  g.X = X;
  g.loss = loss;
  g.staged = staged;
  g.n_new = n_new;
  g.a = a;
  g.m = m;
  g.order = order;
  g.A0 = arrays;
  const int64_t nst = n_new * ((int64_t)a.D + 1);
  if (staged_inline) {
    if (nst > REFIT_INLINE) return hbx_fail(HBX_ERR_ARG, "refit_sort_small: %lld inline doubles", (long long)nst);
    g.staged = nullptr;
    memcpy(g.inl, staged_inline, 8 * (size_t)nst);
  }
  if (a.n <= 2 * NPS_THREADS)
    hipLaunchKernelGGL(kde_refit_sort_small_kernel<2>, dim3(1), dim3(NPS_THREADS), 0, s, g);
  else
    hipLaunchKernelGGL(kde_refit_sort_small_kernel<REFIT_SORT_SMALL / NPS_THREADS>, dim3(1), dim3(NPS_THREADS), 0, s, g);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

// one thread per (segment, set in {good, bad}, dim): bandwidth and observed level count
__global__ __launch_bounds__(128) void kde_fit_stats_kernel(
    const double* __restrict__ X, int32_t D, const int64_t* __restrict__ seg_off, int64_t B,
    const int64_t* __restrict__ order, const int64_t* __restrict__ n_good, const int64_t* __restrict__ n_bad,
    const double* __restrict__ fac_good, const double* __restrict__ fac_bad, const int32_t* __restrict__ vartype,
    double* __restrict__ bw_good, double* __restrict__ bw_bad, int32_t* __restrict__ nlev_good,
    int32_t* __restrict__ nlev_bad) {
  __shared__ uint32_t bits[128][33];  // 1024-level bitmap per thread (+1 pad: bank spread)
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = B * 2 * D;
  if (t >= total) return;
  const int32_t d = (int32_t)(t % D);
  const int64_t bs = t / D;
  const int64_t b = bs >> 1;
  const bool good = (bs & 1) == 0;
  const int64_t ns = good ? n_good[b] : n_bad[b];
  const int64_t s0 = seg_off[b], len = seg_off[b + 1] - s0;
  double* bwo = (good ? bw_good : bw_bad) + b * D + d;
  int32_t* nlo = (good ? nlev_good : nlev_bad) + b * D + d;
  if (ns <= 0 || ns > len) {  // segment not refit (host decided) -> leave a NaN marker
    *bwo = NAN;
    *nlo = 0;
    return;
  }
  // rows of the set: good = head of the argsort, bad = tail (bohb.py:231-232)
  const int64_t* ord = order + s0 + (good ? 0 : (len - ns));
  // order holds positions local to the segment -> shift X to the segment's first row
  const double* Xs = X + s0 * (int64_t)D;
  const double mean = np_sum_column(Xs, D, d, ord, ns, 0.0, false) / (double)ns;
  const double var = np_sum_column(Xs, D, d, ord, ns, mean, true) / (double)ns;
  const double sd = sqrt(var);
  *bwo = (1.06 * sd) * (good ? fac_good[b] : fac_bad[b]);
  if (vartype[d] == 0) {
    *nlo = 0;
    return;
  }
  uint32_t* bm = bits[threadIdx.x];
  for (int w = 0; w < 32; ++w) bm[w] = 0u;
  int32_t cnt = 0;
  constexpr int U = 16;  // gathers batched U at a time (the count is order-independent anyway)
  for (int64_t i0 = 0; i0 < ns && cnt >= 0; i0 += U) {
    double xv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) xv[k] = (i0 + k < ns) ? Xs[ord[i0 + k] * (int64_t)D + d] : 0.0;
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (i0 + k >= ns) break;  // past the set (the gather above loaded a dummy 0.0)
      const double x = xv[k];
      const int v = (int)x;
      if (!(x >= 0.0 && x < 1024.0) || (double)v != x) {
        cnt = -1;  // categorical codes must be integers in [0, 1024)
        break;
      }
      const uint32_t m = 1u << (v & 31);
      if (!(bm[v >> 5] & m)) {
        bm[v >> 5] |= m;
        ++cnt;
      }
    }
  }
  *nlo = cnt;
}

// One workgroup per (segment, set, dim) -- used when there are too few columns to fill the GPU with
// one thread each (a single BOHB refit: 2 x D columns).  The column is gathered into LDS by the whole
// block (once: up to FIT_TILE rows stay resident for both passes); thread 0 then adds strictly in row
// order (np.std's axis-0 reduction order, D > 1), so the result is bit-identical to the
// thread-per-column kernel.  Level counts come from a block-wide bitmap (order-independent).
#define FIT_TILE FIT_TILE_ROWS
// numpy's axis-0 order: one dependent add per row.  The LDS reads of the next 32 rows are issued
// before the adds of the current 32, so the read latency hides behind the add chain (same additions,
// same order).  SQ: add (v - mean)^2.
template <bool SQ>
__device__ __forceinline__ double fit_chain(const double* v, int m, double acc, double mean) {
  auto val = [&](double x) {
    if (SQ) {
      const double q = x - mean;
      return q * q;
    }
    return x;
  };
  const int m32 = m & ~31;
  if (m32 > 0) {
    double r[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) r[k] = v[k];
    for (int i = 32; i < m32; i += 32) {
      double nx[32];
#pragma unroll
      for (int k = 0; k < 32; ++k) nx[k] = v[i + k];
#pragma unroll
      for (int k = 0; k < 32; ++k) acc = acc + val(r[k]);
#pragma unroll
      for (int k = 0; k < 32; ++k) r[k] = nx[k];
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) acc = acc + val(r[k]);
  }
  for (int i = m32; i < m; ++i) acc = acc + val(v[i]);
  return acc;
}

// cs_good / cs_bad (a single segment's refit, both sets within one tile; nullable): the preparation's column
// statistics of each set (kde_colstats_kernel's values, its summation order) from the gathered column --
// one launch less
__global__ __launch_bounds__(256) void kde_fit_col_kernel(
    const double* __restrict__ X, int32_t D, const int64_t* __restrict__ seg_off,
    const int64_t* __restrict__ order, const int64_t* __restrict__ n_good, const int64_t* __restrict__ n_bad,
    const double* __restrict__ fac_good, const double* __restrict__ fac_bad, const int32_t* __restrict__ vartype,
    double* __restrict__ bw_good, double* __restrict__ bw_bad, int32_t* __restrict__ nlev_good,
    int32_t* __restrict__ nlev_bad, ColStats* __restrict__ cs_good, ColStats* __restrict__ cs_bad) {
  __shared__ double v[FIT_TILE];
  __shared__ uint32_t bits[32];
  __shared__ double red;
  __shared__ int bad_code;
  const int64_t t = blockIdx.x;
  const int32_t d = (int32_t)(t % D);
  const int64_t bs = t / D;
  const int64_t b = bs >> 1;
  const bool good = (bs & 1) == 0;
  const int64_t ns = good ? n_good[b] : n_bad[b];
  const int64_t s0 = seg_off[b], len = seg_off[b + 1] - s0;
  double* bwo = (good ? bw_good : bw_bad) + b * D + d;
  int32_t* nlo = (good ? nlev_good : nlev_bad) + b * D + d;
  if (ns <= 0 || ns > len) {
    if (threadIdx.x == 0) {
      *bwo = NAN;
      *nlo = 0;
    }
    return;
  }
  const int64_t* ord = order + s0 + (good ? 0 : (len - ns));
  const double* Xs = X + s0 * (int64_t)D;
  const bool cat = vartype[d] != 0;
  if (threadIdx.x < 32) bits[threadIdx.x] = 0u;
  if (threadIdx.x == 0) bad_code = 0;
  // gather rows [c, c + m) of the column into v (pass 0 also marks the codes; pass 1 re-gathers only
  // when the column exceeds one tile)
  auto gather = [&](int64_t c, int m, bool codes) {
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
      const double x = Xs[ord[c + i] * (int64_t)D + d];
      v[i] = x;
      if (codes && cat) {
        const int iv = (int)x;
        if (!(x >= 0.0 && x < 1024.0) || (double)iv != x) bad_code = 1;
        else atomicOr(&bits[iv >> 5], 1u << (iv & 31));
      }
    }
    __syncthreads();
  };
  double acc = 0.0;  // thread 0
  for (int64_t c = 0; c < ns; c += FIT_TILE) {
    const int m = (int)((ns - c) < FIT_TILE ? (ns - c) : FIT_TILE);
    gather(c, m, true);
    if (cs_good && ns <= FIT_TILE) {  // kde_colstats_kernel's statistic of this (set, dim), its order
      ColStats* cs = good ? cs_good : cs_bad;
      __shared__ double cred[4];
      __shared__ int mred[4];
      if (!cat) {
        double a = 0.0;
        for (int j = threadIdx.x; j < m; j += 256) a += v[j];
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
        if ((threadIdx.x & 63) == 0) cred[threadIdx.x >> 6] = a;
      } else {
        int mx = -1;
        for (int j = threadIdx.x; j < m; j += 256) {
          const double x = v[j];
          mx = max(mx, (!(x >= 0.0 && x < 1024.0) || x != floor(x)) ? 100000 : (int)x);
        }
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
        if ((threadIdx.x & 63) == 0) mred[threadIdx.x >> 6] = mx;
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        if (!cat) {
          cs->mean[d] = ((cred[0] + cred[1]) + (cred[2] + cred[3])) / (double)ns;
        } else {
          const int mm = max(max(mred[0], mred[1]), max(mred[2], mred[3]));
          cs->maxcode[d] = mm >= 100000 ? -1 : mm;
        }
      }
    }
    if (threadIdx.x == 0) acc = fit_chain<false>(v, m, acc, 0.0);
  }
  if (threadIdx.x == 0) red = acc;
  __syncthreads();
  const double mean = red / (double)ns;
  acc = 0.0;
  if (ns <= FIT_TILE) {  // the column is still in LDS: squared deviations in place, then the chain
    for (int i = threadIdx.x; i < ns; i += blockDim.x) {
      const double q = v[i] - mean;
      v[i] = q * q;
    }
    __syncthreads();
    if (threadIdx.x == 0) acc = fit_chain<false>(v, (int)ns, 0.0, 0.0);
  } else {
    for (int64_t c = 0; c < ns; c += FIT_TILE) {
      const int m = (int)((ns - c) < FIT_TILE ? (ns - c) : FIT_TILE);
      gather(c, m, false);
      if (threadIdx.x == 0) acc = fit_chain<true>(v, m, acc, mean);
    }
  }
  if (threadIdx.x == 0) {
    const double var = acc / (double)ns;
    *bwo = (1.06 * sqrt(var)) * (good ? fac_good[b] : fac_bad[b]);
    int cnt = 0;
    if (cat) {
      for (int w = 0; w < 32; ++w) cnt += __popc(bits[w]);
      if (bad_code) cnt = -1;
    }
    *nlo = cnt;
  }
}

// Many segments, one LANE per (set, segment, dim) chain, set-major (q = (set B + b) D + d): a wave's lanes are
// the D dims of one or more segments of the same set, so every step reads whole observation rows (D
// consecutive doubles: coalesced) and the wave's chains have one length (the set's size).  np.std's
// axis-0 reduction is one sequential add chain per column (the mean, then the squared deviations); with 64
// chains per wave instead of the LDS kernel's 8 per workgroup, the chains' add latency hides behind the
// other waves of the SIMD, and the kernel runs at the rate of its two HBM reads of the rows.  The order is
// read two batches ahead and the rows one batch ahead of the adds (U loads of each in flight per lane).
// Level counts: a 128-bit register mask per categorical lane in the mean pass; codes >= 128 (rare) take
// one more pass per 128-code window.
#ifndef FIT_WAVE_U
#define FIT_WAVE_U 12
#endif
__global__ __launch_bounds__(256) void kde_fit_wave_kernel(
    const double* __restrict__ X, int32_t D, const int64_t* __restrict__ seg_off, int64_t B,
    const int64_t* __restrict__ order, const int64_t* __restrict__ n_good, const int64_t* __restrict__ n_bad,
    const double* __restrict__ fac_good, const double* __restrict__ fac_bad, const int32_t* __restrict__ vartype,
    double* __restrict__ bw_good, double* __restrict__ bw_bad, int32_t* __restrict__ nlev_good,
    int32_t* __restrict__ nlev_bad) {
  constexpr int U = FIT_WAVE_U;
  const int64_t per_set = B * (int64_t)D;
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= 2 * per_set) return;  // (no barriers below)
#ifndef FIT_BAD_FIRST
#define FIT_BAD_FIRST 1
#endif
  // the bad sets' (long) chains first, the good sets' (short) ones filling the tail
  const int set = (q >= per_set) != (FIT_BAD_FIRST != 0) ? 1 : 0;
  const int64_t qq = q >= per_set ? q - per_set : q;
  const int64_t b = qq / D;
  const int32_t d = (int32_t)(qq - b * D);
  const int64_t ns = set ? n_bad[b] : n_good[b];
  const int64_t s0 = seg_off[b], len = seg_off[b + 1] - s0;
  double* bwo = (set ? bw_bad : bw_good) + b * D + d;
  int32_t* nlo = (set ? nlev_bad : nlev_good) + b * D + d;
  if (ns <= 0 || ns > len) {  // segment not refit (host decided): NaN marker
    *bwo = NAN;
    *nlo = 0;
    return;
  }
  const int64_t* ord = order + s0 + (set ? len - ns : 0);  // rows of the set: head / tail of the argsort
  const double* Xs = X + s0 * (int64_t)D + d;
  const bool cat = vartype[d] != 0;
  uint64_t m0 = 0, m1 = 0;
  bool badc = false, big = false;
  // one pass over the set's rows in rank order; SQ: squared deviations from mean, else the plain values
  // (and the level masks of a categorical column)
  auto pass = [&](auto sq_tag, double mean) __attribute__((always_inline)) -> double {
    constexpr bool SQ = decltype(sq_tag)::value;
    double acc = 0.0;
    // the order's entries are segment-local row indices (< 2^31): their low words, one register each
    const int32_t* ord32 = reinterpret_cast<const int32_t*>(ord);
    int32_t o1[U], o2[U];
    double v0[U];
#pragma unroll
    for (int k = 0; k < U; ++k) o1[k] = k < ns ? ord32[2 * k] : 0;  // (row 0 past the end: read, unused)
#pragma unroll
    for (int k = 0; k < U; ++k) v0[k] = Xs[o1[k] * (int64_t)D];
#pragma unroll
    for (int k = 0; k < U; ++k) o1[k] = U + k < ns ? ord32[2 * (U + k)] : 0;
#pragma unroll
    for (int k = 0; k < U; ++k) o2[k] = 2 * U + k < ns ? ord32[2 * (2 * U + k)] : 0;
    for (int64_t i = 0; i < ns; i += U) {
      double v1[U];
#pragma unroll
      for (int k = 0; k < U; ++k) v1[k] = Xs[o1[k] * (int64_t)D];  // ranks [i + U, i + 2U)
#pragma unroll
      for (int k = 0; k < U; ++k) {
        o1[k] = o2[k];
        o2[k] = i + 3 * U + k < ns ? ord32[2 * (i + 3 * U + k)] : 0;  // ranks [i + 3U, i + 4U)
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (i + k < ns) {
          const double x = v0[k];
          if constexpr (SQ) {
            const double t = x - mean;
            acc = acc + t * t;
          } else {
            acc = acc + x;
            if (cat) {
              const int iv = (int)x;
              if (!(x >= 0.0 && x < 1024.0) || (double)iv != x) badc = true;
              else if (iv < 64) m0 |= 1ull << iv;
              else if (iv < 128) m1 |= 1ull << (iv - 64);
              else big = true;
            }
          }
        }
      }
#pragma unroll
      for (int k = 0; k < U; ++k) v0[k] = v1[k];
    }
    return acc;
  };
  const double mean = pass(std::false_type{}, 0.0) / (double)ns;
  const double var = pass(std::true_type{}, mean) / (double)ns;
  *bwo = (1.06 * sqrt(var)) * (set ? fac_bad[b] : fac_good[b]);
  int32_t cnt = 0;
  if (cat) {
    cnt = __popcll(m0) + __popcll(m1);
    for (int w = 1; big && !badc && w < 8; ++w) {  // codes in [128 w, 128 w + 128): one pass per window
      uint64_t a = 0, c = 0;
      for (int64_t i = 0; i < ns; ++i) {
        const int iv = (int)Xs[ord[i] * (int64_t)D] - 128 * w;
        if (iv >= 0 && iv < 64) a |= 1ull << iv;
        else if (iv >= 64 && iv < 128) c |= 1ull << (iv - 64);
      }
      cnt += __popcll(a) + __popcll(c);
    }
    if (badc) cnt = -1;
  }
  *nlo = cnt;
}

extern "C" {

int hbx_seg_argsort_ex(const double* loss, const int64_t* seg_off, int64_t B, int64_t max_seg, int64_t N,
                       int64_t* order, void* scratch, int64_t scratch_bytes, int32_t order_mode, void* stream);

// Scratch bytes hbx_kde_fit / hbx_sh_promote need for N total rows.
// sort scratch: two (key, position) ping-pong arrays, then room for the promotion's sorted positions
// when its caller passes no `order` buffer (hbx_sh_promote, brackets > 1024)
int64_t hbx_sort_scratch_bytes(int64_t N) {
  return (int64_t)((2 * (sizeof(uint64_t) + sizeof(int32_t)) + sizeof(int64_t)) * N + 64);
}

static int sort_tile(int64_t max_seg) {
  int tile = 64;
  while (tile < max_seg && tile < 4096) tile <<= 1;
  return tile;
}

// Stable argsort of each segment's losses (np.argsort order; ties by position).  seg_off: device
// int64[B+1]; max_seg: host upper bound on segment length; order: device int64[N] (segment-local).
static int seg_argsort_stable(const double* loss, const int64_t* seg_off, int64_t B, int64_t max_seg, int64_t N,
                              int64_t* order, void* scratch, int64_t scratch_bytes, void* stream,
                              int32_t* cnt_list = nullptr, bool* flagged = nullptr);

int hbx_seg_argsort(const double* loss, const int64_t* seg_off, int64_t B, int64_t max_seg, int64_t N,
                    int64_t* order, void* scratch, int64_t scratch_bytes, void* stream) {
  return hbx_seg_argsort_ex(loss, seg_off, B, max_seg, N, order, scratch, scratch_bytes, HBX_ORDER_STABLE, stream);
}

// numpy mode: the stable sort, then the segments holding ties re-sorted in numpy's order; the scratch
// (32 N + 64 bytes) is free again after the stable sort: A/T/W/Lst take 4 N int32 (indexed by segment
// offset), the flagged list <= N / 2 + 16 more (only segments of >= 2 elements can tie)
int hbx_seg_argsort_ex(const double* loss, const int64_t* seg_off, int64_t B, int64_t max_seg, int64_t N,
                       int64_t* order, void* scratch, int64_t scratch_bytes, int32_t order_mode, void* stream) {
  if (order_mode != HBX_ORDER_NUMPY && order_mode != HBX_ORDER_STABLE)
    return hbx_fail(HBX_ERR_ARG, "hbx_seg_argsort_ex: order_mode %d", order_mode);
  int32_t* arrays = (int32_t*)scratch;
  const bool np = order_mode == HBX_ORDER_NUMPY && B > 0 && N >= 2;
  bool flagged = false;  // the wave sort flagged its tied segments itself (numpy mode)
  int rc = seg_argsort_stable(loss, seg_off, B, max_seg, N, order, scratch, scratch_bytes, stream,
                              np ? arrays + 4 * N : nullptr, &flagged);
  if (rc || !np) return rc;
  return hbx_np_order_fix(loss, seg_off, B, max_seg, order, nullptr, 0, 1, order, nullptr, arrays, N, 0, arrays + 4 * N,
                          flagged, (hipStream_t)stream);
}

static int seg_argsort_stable(const double* loss, const int64_t* seg_off, int64_t B, int64_t max_seg, int64_t N,
                              int64_t* order, void* scratch, int64_t scratch_bytes, void* stream, int32_t* cnt_list,
                              bool* flagged) {
  if (!loss || !seg_off || !order || (!scratch && N > 0)) return hbx_fail(HBX_ERR_ARG, "hbx_seg_argsort: null");
  if (B <= 0) return HBX_OK;
  if (scratch_bytes < hbx_sort_scratch_bytes(N)) return hbx_fail(HBX_ERR_ARG, "sort scratch too small");
  const bool rank_ok = max_seg <= RANK_MAX_SEG && B <= 65535;
  // many short segments: one wave each; a few (a single refit split): the counting rank spreads
  // each segment over many workgroups; longer segments or more of them: LDS tiles + merges
  if (max_seg <= 64 * PW_PER_LANE && (B >= 64 || !rank_ok)) {
    if (cnt_list) {  // numpy mode: the wave sort flags its tied segments (cnt_list: count, then the list)
      HBX_HIP(hipMemsetAsync(cnt_list, 0, sizeof(int32_t), (hipStream_t)stream));
      *flagged = true;
    }
    hipLaunchKernelGGL(seg_argsort_wave_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                       loss, seg_off, B, order, cnt_list ? cnt_list + 16 : nullptr, cnt_list);
    HBX_LAUNCH_CHECK();
    return HBX_OK;
  }
  if (rank_ok) {
    int32_t* rank = (int32_t*)scratch;  // N int32 of the (24 N + 64)-byte sort scratch
    HBX_HIP(hipMemsetAsync(rank, 0, sizeof(int32_t) * (size_t)N, (hipStream_t)stream));
    const unsigned gi = (unsigned)((max_seg + 255) / 256);
    hipLaunchKernelGGL(seg_rank_count_kernel, dim3(gi, (unsigned)((max_seg + RANK_J - 1) / RANK_J), (unsigned)B),
                       dim3(256), 0, (hipStream_t)stream, loss, seg_off, rank);
    HBX_LAUNCH_CHECK();
    hipLaunchKernelGGL(seg_rank_scatter_kernel, dim3(gi, (unsigned)B), dim3(256), 0, (hipStream_t)stream, seg_off,
                       rank, order);
    HBX_LAUNCH_CHECK();
    return HBX_OK;
  }
  const int tile = sort_tile(max_seg);
  char* sc = (char*)scratch;
  uint64_t* gk = (uint64_t*)sc;
  uint64_t* gk2 = gk + N;
  int32_t* gi = (int32_t*)(gk2 + N);
  int32_t* gi2 = gi + N;
  hipLaunchKernelGGL(seg_argsort_kernel, dim3((unsigned)B), dim3(256), (sizeof(uint64_t) + sizeof(int32_t)) * tile,
                     (hipStream_t)stream, loss, seg_off, tile, gk, gi, gk2, gi2, order);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

// Batched KDE refit.  X: device fp64 [N][D] (segment b = rows seg_off[b]..seg_off[b+1]);
// order: output of hbx_seg_argsort; n_good/n_bad: device int64[B] (0 = segment not refit);
// fac_good/fac_bad: device fp64[B] = n**(-1/(4+D)) from host pow(); vartype: device int32[D].
// Outputs: bw_good/bw_bad fp64[B][D], nlev_good/nlev_bad int32[B][D] (-1: code not an integer in [0,1024)).
int hbx_kde_fit(const double* X, int32_t D, const int64_t* seg_off, int64_t B, const int64_t* order,
                const int64_t* n_good, const int64_t* n_bad, const double* fac_good, const double* fac_bad,
                const int32_t* vartype, double* bw_good, double* bw_bad, int32_t* nlev_good, int32_t* nlev_bad,
                void* stream) {
  if (!X || !seg_off || !order || !n_good || !n_bad || !fac_good || !fac_bad || !vartype || !bw_good ||
      !bw_bad || !nlev_good || !nlev_bad)
    return hbx_fail(HBX_ERR_ARG, "hbx_kde_fit: null pointer");
  if (D < 1 || D > HBX_MAX_D) return hbx_fail(HBX_ERR_UNSUPPORTED, "D=%d outside [1, %d]", D, HBX_MAX_D);
  if (B <= 0) return HBX_OK;
  const int64_t total = B * 2 * D;
  if (D > 1 && total >= 16384) {  // many segments: one lane per column chain
    if ((total + 255) / 256 > 0x7fffffffLL) return hbx_fail(HBX_ERR_ARG, "hbx_kde_fit: too many segments");
    hipLaunchKernelGGL(kde_fit_wave_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       X, D, seg_off, B, order, n_good, n_bad, fac_good, fac_bad, vartype, bw_good, bw_bad,
                       nlev_good, nlev_bad);
  } else if (D > 1 && total < 16384) {  // few columns: one workgroup each (LDS-staged gathers)
    hipLaunchKernelGGL(kde_fit_col_kernel, dim3((unsigned)total), dim3(256), 0, (hipStream_t)stream, X, D, seg_off,
                       order, n_good, n_bad, fac_good, fac_bad, vartype, bw_good, bw_bad, nlev_good, nlev_bad,
                       (ColStats*)nullptr, (ColStats*)nullptr);
  } else {
    hipLaunchKernelGGL(kde_fit_stats_kernel, dim3((unsigned)((total + 127) / 128)), dim3(128), 0,
                       (hipStream_t)stream, X, D, seg_off, B, order, n_good, n_bad, fac_good, fac_bad, vartype,
                       bw_good, bw_bad, nlev_good, nlev_bad);
  }
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

}  // extern "C"

// A single refit's fit (B = 1, D > 1, both sets within one LDS tile) that also writes the preparation's column
// statistics of both sets (the colstats launch saved): hbx_kde_refit's path
int refit_fit_colstats(const double* X, int32_t D, const int64_t* seg_off, const int64_t* order, const int64_t* n_good,
                       const int64_t* n_bad, const double* fac_good, const double* fac_bad, const int32_t* vartype,
                       double* bw_good, double* bw_bad, int32_t* nlev_good, int32_t* nlev_bad, ColStats* cs_good,
                       ColStats* cs_bad, hipStream_t s) {
  hipLaunchKernelGGL(kde_fit_col_kernel, dim3((unsigned)(2 * D)), dim3(256), 0, s, X, D, seg_off, order, n_good, n_bad,
                     fac_good, fac_bad, vartype, bw_good, bw_bad, nlev_good, nlev_bad, cs_good, cs_bad);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}
