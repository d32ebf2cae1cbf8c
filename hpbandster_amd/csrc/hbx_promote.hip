// hbx_promote.hip -- batched successive-halving promotion on MI355X.
//
// Reference: HB_iteration.py:179-182 (SuccessiveHalving.process_results)
//     ranks = np.argsort(np.argsort(losses)); advance = ranks < num_configs[SH_iter]
// and HB_iteration.py:240-242 (SuccessiveResampling: ranks < max(1, n * (1 - 0.5))).
// Only REVIEW configurations (finite losses) are ranked; CRASHED ones (non-finite, register_result
// HB_iteration.py:102-106) never advance.  Mask only (the drop-in's need): a radix select of the k-th
// (key, position) per bracket (sh_select_kernel).  With the sorted order requested: a stable sort of
// the losses (hbx_sort.h; one wave per bracket <= 1024, else one workgroup), then
// advance[position] = (rank < k).  Ties are ranked by position (stable);
// numpy's argsort is unstable, so on tied losses the reference's choice is platform dependent.
#include "hbx_common.h"
#include "hbx_sort.h"
#include <stdlib.h>

__global__ __launch_bounds__(256) void sh_promote_kernel(const double* __restrict__ loss,
                                                         const int64_t* __restrict__ seg_off,
                                                         const double* __restrict__ k, int tile, uint64_t* gk,
                                                         int32_t* gi, uint64_t* gk2, int32_t* gi2,
                                                         int64_t* __restrict__ order,
                                                         uint8_t* __restrict__ advance,
                                                         int64_t* __restrict__ n_advance) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint64_t* lk = (uint64_t*)smem;
  int32_t* li = (int32_t*)(smem + sizeof(uint64_t) * tile);
  __shared__ int cnt;
  const int64_t b = blockIdx.x;
  const int64_t s = seg_off[b], e = seg_off[b + 1], n = e - s;
  if (threadIdx.x == 0) cnt = 0;
  block_sort_segment<true>(loss + s, n, tile, lk, li, gk + s, gi + s, gk2 + s, gi2 + s, order + s);
  const double kb = k[b];
  int mine = 0;
  for (int64_t r = threadIdx.x; r < n; r += blockDim.x) {
    const int64_t p = order[s + r];
    const double v = loss[s + p];
    const bool adv = (v - v == 0.0) && ((double)r < kb);
    advance[s + p] = adv ? 1 : 0;
    mine += adv;
  }
  for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(&cnt, mine);
  __syncthreads();
  if (threadIdx.x == 0 && n_advance) n_advance[b] = cnt;
}

// Brackets of up to 1024 configurations (every SH bracket of a realistic ladder): one wave per
// bracket, sorted in registers (wave_sort_1024, hbx_sort.h).  Same (key, position) order as
// sh_promote_kernel, so order / advance / n_advance are identical.
__global__ __launch_bounds__(256) void sh_promote_wave_kernel(const double* __restrict__ loss,
                                                              const int64_t* __restrict__ seg_off, int64_t B,
                                                              const double* __restrict__ k,
                                                              int64_t* __restrict__ order,
                                                              uint8_t* __restrict__ advance,
                                                              int64_t* __restrict__ n_advance) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // whole wave
  const int64_t s = seg_off[b];
  const int n = (int)(seg_off[b + 1] - s);
  uint64_t key[PW_PER_LANE];
  int32_t pos[PW_PER_LANE];
  wave_sort_1024<true>(loss + s, n, lane, key, pos);
  const double kb = k[b];
  int mine = 0;
#pragma unroll
  for (int r = 0; r < PW_PER_LANE; ++r) {
    const int rank = lane * PW_PER_LANE + r;
    if (rank < n) {
      order[s + rank] = pos[r];
      const bool adv = key[r] != ~0ull && (double)rank < kb;  // finite loss (key_promote) and rank < k
      advance[s + pos[r]] = adv ? 1 : 0;
      mine += adv;
    }
  }
  for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o);
  if (lane == 0 && n_advance) n_advance[b] = mine;
}

// Brackets of up to 1024 configurations without a sorted order requested: the mask needs only the
// k-th smallest (key, position) of the bracket, found by a bitwise radix select in registers -- O(n)
// per bracket instead of the O(n log^2 n) sort.  One wave per bracket; element i = 64 r + lane sits in
// register r of lane `lane` (coalesced loads, 64 consecutive mask bytes per store).  Each lane keeps
// its 16 elements' state as bit masks (bit r): `alive` = still in the bucket holding the k-th element,
// `less` = known to rank below it.  Bits are resolved from the highest bit where the finite keys
// differ downwards; a pass counts the bucket's elements with a 0 at that bit (one wave sum) and keeps
// the half that holds the k-th.  It stops as soon as the whole bucket advances; keys equal in all 64
// bits are ranked by position (stable), as sh_promote_wave_kernel / sh_promote_kernel rank them.
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ uint32_t wave_and(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v &= (uint32_t)__shfl_xor((int)v, o);
  return v;
}
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o);
  return v;
}

__global__ __launch_bounds__(256) void sh_select_kernel(const double* __restrict__ loss,
                                                        const int64_t* __restrict__ seg_off, int64_t B,
                                                        const double* __restrict__ k,
                                                        uint8_t* __restrict__ advance,
                                                        int64_t* __restrict__ n_advance) {
  constexpr int R = PW_PER_LANE;  // 16 registers x 64 lanes = 1024 elements
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // whole wave
  const int64_t s = seg_off[b];
  const int n = (int)(seg_off[b + 1] - s);
  uint32_t khi[R], klo[R];
  uint32_t alive = 0;
  uint32_t andh = ~0u, andl = ~0u, orh = 0u, orl = 0u;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = 64 * r + lane;
    const double v = i < n ? loss[s + i] : 0.0;
    const bool fin = i < n && (v - v == 0.0);  // CRASHED (non-finite) entries are never ranked
    const uint64_t key = fin ? hbx_d2ord(v) : 0ull;
    khi[r] = (uint32_t)(key >> 32);
    klo[r] = (uint32_t)key;
    if (fin) {
      alive |= 1u << r;
      andh &= khi[r];
      andl &= klo[r];
      orh |= khi[r];
      orl |= klo[r];
    }
  }
  const int nfin = wave_sum(__popc(alive));
  // rank < k advances: the first kk ranks, kk = min(nfin, ceil(k)) (k > 0; NaN or k <= 0: none)
  const double kb = k[b];
  const int kk = kb > 0.0 ? (kb >= (double)nfin ? nfin : (int)ceil(kb)) : 0;
  uint32_t adv;
  if (kk == nfin) {
    adv = alive;
  } else if (kk == 0) {
    adv = 0u;
  } else {
    uint32_t less = 0u;
    int need = kk, cnt = nfin;
    // bits above the highest one where the finite keys differ are common to all of them
    const uint32_t dh = wave_or(orh) ^ wave_and(andh), dl = wave_or(orl) ^ wave_and(andl);
    const int top = dh ? 63 - __clz((int)dh) : (dl ? 31 - __clz((int)dl) : -1);
    for (int bit = top; bit >= 0 && cnt != need; --bit) {
      uint32_t ones = 0u;
      const int sh = bit & 31;
#pragma unroll
      for (int r = 0; r < R; ++r) ones |= (((bit >= 32 ? khi[r] : klo[r]) >> sh) & 1u) << r;
      const uint32_t zero = alive & ~ones;
      const int c0 = wave_sum(__popc(zero));
      if (need <= c0) {
        alive = zero;
        cnt = c0;
      } else {
        less |= zero;
        alive &= ones;
        need -= c0;
        cnt -= c0;
      }
    }
    // the `need` first bucket elements by position (all of them when cnt == need)
    adv = less;
    int taken = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t m = __ballot((alive >> r) & 1u);
      const int before = __popcll(m & ((1ull << lane) - 1ull));
      if (((alive >> r) & 1u) && taken + before < need) adv |= 1u << r;
      taken += __popcll(m);
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = 64 * r + lane;
    if (i < n) advance[s + i] = (uint8_t)((adv >> r) & 1u);
  }
  if (lane == 0 && n_advance) n_advance[b] = kk;
}

extern "C" {

int64_t hbx_sort_scratch_bytes(int64_t N);

// loss: device fp64[N] (non-finite = not ranked); seg_off: device int64[B+1]; k: device fp64[B];
// max_seg: host bound on the longest bracket; order: device int64[N] (sorted positions per bracket) or
// NULL when only the mask is wanted; advance: device uint8[N]; n_advance: device int64[B] (nullable).
int hbx_sh_promote(const double* loss, const int64_t* seg_off, int64_t B, int64_t max_seg, int64_t N,
                   const double* k, int64_t* order, uint8_t* advance, int64_t* n_advance, void* scratch,
                   int64_t scratch_bytes, void* stream) {
  if (!loss || !seg_off || !k || !advance) return hbx_fail(HBX_ERR_ARG, "hbx_sh_promote: null pointer");
  if (B <= 0) return HBX_OK;
  if (max_seg <= 64 * PW_PER_LANE && !order) {  // mask only: O(n) selection, no scratch
    hipLaunchKernelGGL(sh_select_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, (hipStream_t)stream, loss,
                       seg_off, B, k, advance, n_advance);
    HBX_LAUNCH_CHECK();
    return HBX_OK;
  }
  if (!scratch || scratch_bytes < hbx_sort_scratch_bytes(N)) return hbx_fail(HBX_ERR_ARG, "sort scratch too small");
  char* sc = (char*)scratch;
  uint64_t* gk = (uint64_t*)sc;
  uint64_t* gk2 = gk + N;
  int32_t* gi = (int32_t*)(gk2 + N);
  int32_t* gi2 = gi + N;
  if (!order) order = (int64_t*)(sc + ((2 * (sizeof(uint64_t) + sizeof(int32_t)) * N + 7) & ~(size_t)7));
  const char* wenv = getenv("HBX_PROMOTE_WAVE");  // 0: the block-per-bracket kernel for every size
  if (max_seg <= 64 * PW_PER_LANE && !(wenv && atoi(wenv) == 0)) {
    hipLaunchKernelGGL(sh_promote_wave_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, (hipStream_t)stream, loss,
                       seg_off, B, k, order, advance, n_advance);
    HBX_LAUNCH_CHECK();
    return HBX_OK;
  }
  int tile = 64;
  while (tile < max_seg && tile < 4096) tile <<= 1;
  hipLaunchKernelGGL(sh_promote_kernel, dim3((unsigned)B), dim3(256), (sizeof(uint64_t) + sizeof(int32_t)) * tile,
                     (hipStream_t)stream, loss, seg_off, k, tile, gk, gi, gk2, gi2, order, advance, n_advance);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

}  // extern "C"
