// hbx_sort.h -- per-segment stable sort of fp64 losses for one workgroup (device code).
//
// A segment (one budget's observations for the KDE refit, or one bracket's losses for the SH
// promotion) is sorted by (key, position): keys are order-preserving 64-bit images of the fp64
// losses, the position breaks ties, so the order is total and stable.  Segments up to `tile`
// elements are bitonic-sorted in LDS; longer segments are cut into LDS-sorted runs of `tile`
// elements that are merged pairwise through global scratch (every output element finds its slot
// with one binary search in the partner run -- no data-dependent control flow between threads).
#pragma once

#include "hbx_common.h"

// argsort order of numpy (np.argsort on fp64): -inf < finite < +inf < NaN
__device__ __forceinline__ uint64_t key_argsort(double v) { return hbx_d2ord(v); }
// promotion order: finite losses ranked, every non-finite loss (CRASHED) after them
__device__ __forceinline__ uint64_t key_promote(double v) {
  return (v - v == 0.0) ? hbx_d2ord(v) : ~0ull;
}

__device__ __forceinline__ bool kv_less(uint64_t ka, int32_t ia, uint64_t kb, int32_t ib) {
  return ka < kb || (ka == kb && ia < ib);
}

// The value of lane `lane ^ lm` (lm a power of two known after unrolling) without the LDS crossbar where the
// pattern allows: xor 1 / 2 by a quad permutation, xor 4 / 8 by row rotations (row_ror:n gives lane i the
// value of lane i - n within its 16-lane row), xor 16 by ds_swizzle's bit mode; xor 32 by ds_bpermute
__device__ __forceinline__ uint32_t lane_xor_u32(uint32_t v, int lm, int lane) {
  switch (lm) {
    case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xb1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4e, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
    case 4: {
      const uint32_t a = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xf, 0xf, false);  // row_ror:4  (i - 4)
      const uint32_t b = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x12c, 0xf, 0xf, false);  // row_ror:12 (i + 4)
      return (lane & 4) ? a : b;
    }
    case 8: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
    case 16: return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401f);  // and 0x1f, xor 0x10
    default: return (uint32_t)__shfl_xor((int)v, lm);
  }
}
__device__ __forceinline__ uint64_t lane_xor_u64(uint64_t v, int lm, int lane) {
  return (uint64_t)lane_xor_u32((uint32_t)v, lm, lane) | ((uint64_t)lane_xor_u32((uint32_t)(v >> 32), lm, lane) << 32);
}

// Bitonic sort of P (power of two) pairs in LDS, whole block participates.
__device__ void block_bitonic(uint64_t* k, int32_t* ix, int P) {
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const bool gt = kv_less(k[j], ix[j], k[i], ix[i]);
          if (gt == up) {
            const uint64_t tk = k[i];
            k[i] = k[j];
            k[j] = tk;
            const int32_t ti = ix[i];
            ix[i] = ix[j];
            ix[j] = ti;
          }
        }
      }
      __syncthreads();
    }
  }
}

// Sort one segment of n losses; writes the sorted positions (0..n-1) to `order` (int64) and, if
// `sorted_keys` is non-null, the keys.  lds_k / lds_i hold `tile` entries; gk/gi (and gk2/gi2) are
// global scratch of n entries each, needed only when n > tile.  PROMOTE selects the key order.
template <bool PROMOTE>
__device__ void block_sort_segment(const double* __restrict__ loss, int64_t n, int tile, uint64_t* lds_k,
                                   int32_t* lds_i, uint64_t* gk, int32_t* gi, uint64_t* gk2, int32_t* gi2,
                                   int64_t* __restrict__ order) {
  if (n <= 0) return;
  if (n <= tile) {
    int P = 1;
    while (P < n) P <<= 1;
    for (int i = threadIdx.x; i < P; i += blockDim.x) {
      if (i < n) {
        lds_k[i] = PROMOTE ? key_promote(loss[i]) : key_argsort(loss[i]);
        lds_i[i] = i;
      } else {
        lds_k[i] = ~0ull;
        lds_i[i] = 0x7fffffff;
      }
    }
    __syncthreads();
    block_bitonic(lds_k, lds_i, P);
    for (int i = threadIdx.x; i < n; i += blockDim.x) order[i] = lds_i[i];
    __syncthreads();
    return;
  }
  // 1) LDS-sorted runs of `tile`
  for (int64_t base = 0; base < n; base += tile) {
    const int len = (int)((n - base) < tile ? (n - base) : tile);
    for (int i = threadIdx.x; i < tile; i += blockDim.x) {
      if (i < len) {
        lds_k[i] = PROMOTE ? key_promote(loss[base + i]) : key_argsort(loss[base + i]);
        lds_i[i] = (int32_t)(base + i);
      } else {
        lds_k[i] = ~0ull;
        lds_i[i] = 0x7fffffff;
      }
    }
    __syncthreads();
    block_bitonic(lds_k, lds_i, tile);
    for (int i = threadIdx.x; i < len; i += blockDim.x) {
      gk[base + i] = lds_k[i];
      gi[base + i] = lds_i[i];
    }
    __syncthreads();
  }
  // 2) pairwise merges of runs (width doubles each pass); ping-pong gk/gi <-> gk2/gi2
  uint64_t *sk = gk, *dk = gk2;
  int32_t *si = gi, *di = gi2;
  for (int64_t width = tile; width < n; width <<= 1) {
    for (int64_t e = threadIdx.x; e < n; e += blockDim.x) {
      const int64_t run = e / width;
      const int64_t lstart = (run & ~1ll) * width;
      const int64_t rstart = lstart + width;
      const bool left = (run & 1) == 0;
      const int64_t o_start = left ? rstart : lstart;              // partner run
      const int64_t o_end = left ? (rstart + width < n ? rstart + width : n) : rstart;
      const uint64_t k = sk[e];
      const int32_t ix = si[e];
      int64_t lo = o_start, hi = o_end;  // count partner elements less than (k, ix)
      if (!left || rstart < n) {
        while (lo < hi) {
          const int64_t mid = (lo + hi) >> 1;
          if (kv_less(sk[mid], si[mid], k, ix)) lo = mid + 1; else hi = mid;
        }
      } else {
        lo = o_start;
      }
      const int64_t mine = e - (left ? lstart : rstart);
      const int64_t pos = lstart + mine + (lo - o_start);
      dk[pos] = k;
      di[pos] = ix;
    }
    __threadfence_block();
    __syncthreads();
    uint64_t* tk = sk; sk = dk; dk = tk;
    int32_t* ti = si; si = di; di = ti;
  }
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) order[i] = si[i];
  __syncthreads();
}

// Segments of up to 1024 elements, one wave: logical element i = 16 lane + r lives in register r of
// lane `lane`; the bitonic network runs in registers -- strides < 16 compare registers of one lane,
// strides >= 16 exchange with lane ^ (stride / 16) through cross-lane shuffles.  No LDS, no barriers.
// On return register r of lane `lane` holds rank 16 lane + r: its key and position (padding past n:
// key ~0, position 0x7fffffff, after every real element).  Same (key, position) order as
// block_sort_segment.
#define PW_PER_LANE 16
template <bool PROMOTE>
__device__ __forceinline__ void wave_sort_1024(const double* __restrict__ loss, int n, int lane,
                                               uint64_t (&key)[PW_PER_LANE], int32_t (&pos)[PW_PER_LANE]) {
#pragma unroll
  for (int r = 0; r < PW_PER_LANE; ++r) {
    const int i = lane * PW_PER_LANE + r;
    key[r] = i < n ? (PROMOTE ? key_promote(loss[i]) : key_argsort(loss[i])) : ~0ull;
    pos[r] = i < n ? i : 0x7fffffff;
  }
#pragma unroll
  for (int size = 2; size <= 64 * PW_PER_LANE; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= PW_PER_LANE) {
        const int lm = stride / PW_PER_LANE;
        const bool lower = (lane & lm) == 0;
#pragma unroll
        for (int r = 0; r < PW_PER_LANE; ++r) {
          // (ds_bpermute: the DPP exchanges of wave_sort_run measured 1.48 -> 2.04 ms on config #5's refit
          // of 1e4 brackets in this 16-per-lane network)
          const uint64_t ok = __shfl_xor(key[r], lm);
          const int32_t op = __shfl_xor(pos[r], lm);
          const bool up = ((lane * PW_PER_LANE + r) & size) == 0;
          const bool other_less = kv_less(ok, op, key[r], pos[r]);
          // ascending run: the lower index keeps the smaller element; descending: the larger
          const bool take = (lower == up) ? other_less : !other_less;
          if (take) {
            key[r] = ok;
            pos[r] = op;
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < PW_PER_LANE; ++r) {
          if (r & stride) continue;
          const int q = r | stride;
          const bool up = ((lane * PW_PER_LANE + r) & size) == 0;
          const bool gt = kv_less(key[q], pos[q], key[r], pos[r]);
          if (gt == up) {
            const uint64_t tk = key[r];
            key[r] = key[q];
            key[q] = tk;
            const int32_t tp = pos[r];
            pos[r] = pos[q];
            pos[q] = tp;
          }
        }
      }
    }
  }
}

// The same network over 64 PW elements starting at position base of loss (register r of lane `lane` =
// element base + PW lane + r; padding past n: key ~0, position 0x7fffffff): one wave's run of a
// multi-wave sort (kde_refit_sort_small_kernel: four runs of 256, merged by rank).
template <bool PROMOTE, int PW>
__device__ __forceinline__ void wave_sort_run(const double* __restrict__ loss, int base, int n, int lane,
                                              uint64_t (&key)[PW], int32_t (&pos)[PW]) {
#pragma unroll
  for (int r = 0; r < PW; ++r) {
    const int i = base + lane * PW + r;
    key[r] = i < n ? (PROMOTE ? key_promote(loss[i]) : key_argsort(loss[i])) : ~0ull;
    pos[r] = i < n ? i : 0x7fffffff;
  }
#pragma unroll
  for (int size = 2; size <= 64 * PW; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= PW) {
        const int lm = stride / PW;
        const bool lower = (lane & lm) == 0;
#pragma unroll
        for (int r = 0; r < PW; ++r) {
          const uint64_t ok = lane_xor_u64(key[r], lm, lane);
          const int32_t op = (int32_t)lane_xor_u32((uint32_t)pos[r], lm, lane);
          const bool up = ((lane * PW + r) & size) == 0;
          const bool other_less = kv_less(ok, op, key[r], pos[r]);
          const bool take = (lower == up) ? other_less : !other_less;
          if (take) {
            key[r] = ok;
            pos[r] = op;
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < PW; ++r) {
          if (r & stride) continue;
          const int q = r | stride;
          const bool up = ((lane * PW + r) & size) == 0;
          const bool gt = kv_less(key[q], pos[q], key[r], pos[r]);
          if (gt == up) {
            const uint64_t tk = key[r];
            key[r] = key[q];
            key[q] = tk;
            const int32_t tp = pos[r];
            pos[r] = pos[q];
            pos[q] = tp;
          }
        }
      }
    }
  }
}
