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
// k-th smallest (key, position) of the bracket, found by a bitwise radix select -- O(n) per bracket
// instead of the O(n log^2 n) sort.  One wave per bracket; element i = 64 r + lane sits in register r
// of lane `lane` (coalesced buffer loads issued together, 64 consecutive mask bytes per store).
//   Bits are resolved from the highest bit where the finite keys differ downwards: a pass counts the
// bucket's elements (those matching every bit resolved so far) with a 0 at the bit and keeps the half
// holding the k-th.  While the bucket is large each lane tracks its 16 elements as a bit mask and a
// pass costs 16 bit extractions and one DPP wave sum; once it holds <= 64 keys they are compacted into
// one per lane (LDS, position order) and a pass is one compare and one ballot.  It stops as soon as
// the whole bucket advances.  The mask is then one masked 64-bit compare per element against the
// resolved prefix; keys equal in all 64 bits are ranked by position (stable), as sh_promote_wave_kernel
// and sh_promote_kernel rank them.

constexpr int kBufDword3 = 0x00020000;  // gfx9 buffer resource word 3 (raw 32-bit data, range checked)

__global__ __launch_bounds__(256) void sh_select_kernel(const double* __restrict__ loss,
                                                        const int64_t* __restrict__ seg_off, int64_t B,
                                                        const double* __restrict__ k,
                                                        uint8_t* __restrict__ advance,
                                                        int64_t* __restrict__ n_advance) {
  constexpr int R = PW_PER_LANE;  // 16 registers x 64 lanes = 1024 elements
  __shared__ uint64_t cbuf[4][64];  // per wave: the compacted bucket
  // the wave index made visibly uniform: the bracket's bounds, k and buffer resources live in SGPRs
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t b = (int64_t)blockIdx.x * 4 + wv;
  if (b >= B) return;  // whole wave
  const int64_t s = seg_off[b];
  const int n = (int)(seg_off[b + 1] - s);
  if (n <= 0) {
    if (lane == 0 && n_advance) n_advance[b] = 0;
    return;
  }
  // the bracket as buffer resources: loads past n return 0 and stores past n are dropped by the
  // hardware range check, so all 16 loads (and stores) are unconditional, one address VGPR each
  const __amdgpu_buffer_rsrc_t lrs = __builtin_amdgcn_make_buffer_rsrc((void*)(loss + s), (short)0, n * 8, kBufDword3);
  const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc((void*)(advance + s), (short)0, n, kBufDword3);
  double v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) v[r] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(lrs, 8 * lane, 512 * r, 0));
  // order-preserving keys (hbx_d2ord; -0.0 + 0.0 = +0.0 merges the zeros) and the min / max of the
  // high words over the bracket (rows past n skipped, the partial row masked: uniform branches).
  // Finite keys have high words in [0x00100000, 0xFFEFFFFF]; a bracket without CRASHED (non-finite)
  // entries -- the common case -- then needs no per-element finite mask at all.
  const int nrow = (n + 63) >> 6;  // rows holding elements
  uint64_t key[R];
  uint32_t mnh = ~0u, mxh = 0u;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const double z = v[r] + 0.0;
    const uint32_t hi = (uint32_t)(__double_as_longlong(z) >> 32), lo = (uint32_t)__double_as_longlong(z);
    const uint32_t sg = (uint32_t)((int32_t)hi >> 31);
    const uint32_t kh = hi ^ (sg | 0x80000000u);
    key[r] = ((uint64_t)kh << 32) | (lo ^ sg);
    if (64 * r + 64 <= n) {
      mnh = min(mnh, kh);
      mxh = max(mxh, kh);
    } else if (r < nrow) {
      const bool ok = 64 * r + lane < n;
      mnh = min(mnh, ok ? kh : ~0u);
      mxh = max(mxh, ok ? kh : 0u);
    }
  }
  mnh = ~wave_reduce_dpp(~mnh, OpMax());
  mxh = wave_reduce_dpp(mxh, OpMax());
  const bool allfin = mnh >= 0x00100000u && mxh <= 0xFFEFFFFFu;  // uniform
  // per-lane element mask: bit r = element 64 r + lane exists (and, with CRASHED entries, is finite)
  const int nr = min(max((n - lane + 63) >> 6, 0), R);
  uint32_t fin = (1u << nr) - 1u;
  int nfin = n;
  uint32_t ph, pl = 0u, dh, dl = 0u;  // resolved prefix of the k-th key; bits where the keys differ
  if (allfin) {
    dh = mnh ^ mxh;
    ph = mnh;
    if (dh == 0u) {  // equal high words: the low words decide (rare)
      uint32_t mnl = ~0u, mxl = 0u;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const bool f = (fin >> r) & 1u;
        mnl = min(mnl, f ? (uint32_t)key[r] : ~0u);
        mxl = max(mxl, f ? (uint32_t)key[r] : 0u);
      }
      mnl = ~wave_reduce_dpp(~mnl, OpMax());
      mxl = wave_reduce_dpp(mxl, OpMax());
      dl = mnl ^ mxl;
      pl = mnl;
    }
  } else {  // CRASHED entries present: finite mask, AND / OR of the finite keys
    uint32_t andh = ~0u, orh = 0u;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t kh = (uint32_t)(key[r] >> 32);
      const bool f = ((fin >> r) & 1u) && kh >= 0x00100000u && kh <= 0xFFEFFFFFu;  // finite
      fin &= ~((f ? 0u : 1u) << r);
      andh &= f ? kh : ~0u;
      orh |= f ? kh : 0u;
    }
    nfin = (int)wave_reduce_dpp((uint32_t)__popc(fin), OpAdd());
    ph = wave_reduce_dpp(andh, OpAnd());
    dh = wave_reduce_dpp(orh, OpOr()) ^ ph;
    if (dh == 0u) {
      uint32_t andl = ~0u, orl = 0u;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const bool f = (fin >> r) & 1u;
        andl &= f ? (uint32_t)key[r] : ~0u;
        orl |= f ? (uint32_t)key[r] : 0u;
      }
      pl = wave_reduce_dpp(andl, OpAnd());
      dl = wave_reduce_dpp(orl, OpOr()) ^ pl;
    }
  }
  // rank < k advances: the first kk ranks, kk = min(nfin, ceil(k)) (k > 0; NaN or k <= 0: none)
  const double kb = k[b];
  const int kk = kb > 0.0 ? (kb >= (double)nfin ? nfin : (int)ceil(kb)) : 0;
  if (kk == nfin || kk == 0) {  // all the finite entries, or none
#pragma unroll
    for (int r = 0; r < R; ++r)
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(kk ? (fin >> r) & 1u : 0u), ars, lane, 64 * r, 0);
    if (lane == 0 && n_advance) n_advance[b] = kk;
    return;
  }
  // bits above the highest one where the finite keys differ are common to all of them: resolved
  int bit = dh ? 63 - __clz((int)dh) : (dl ? 31 - __clz((int)dl) : -1);
  if (bit >= 32) {  // the prefix keeps only the bits above `bit`
    ph &= ~((2u << (bit - 32)) - 1u);
    pl = 0u;
  } else if (bit >= 0) {
    pl &= ~((2u << bit) - 1u);
  }
  int need = kk, cnt = nfin;
  uint32_t alive = fin;
  // phase 1: the bucket as per-lane bit masks
  for (; bit >= 0 && cnt != need && cnt > 64; --bit) {
    uint32_t ones = 0u;
    if (bit >= 32) {
#pragma unroll
      for (int r = 0; r < R; ++r) ones |= __builtin_amdgcn_ubfe((uint32_t)(key[r] >> 32), (uint32_t)(bit - 32), 1u) << r;
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) ones |= __builtin_amdgcn_ubfe((uint32_t)key[r], (uint32_t)bit, 1u) << r;
    }
    const uint32_t zero = alive & ~ones;
    const int c0 = (int)wave_reduce_dpp((uint32_t)__popc(zero), OpAdd());
    if (need <= c0) {
      alive = zero;
      cnt = c0;
    } else {
      alive &= ones;
      need -= c0;
      cnt -= c0;
      if (bit >= 32) ph |= 1u << (bit - 32); else pl |= 1u << bit;
    }
  }
  if (bit >= 0 && cnt != need) {
    // phase 2: compact the <= 64 bucket keys into one per lane, in position order
    int base = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool a = (alive >> r) & 1u;
      const uint64_t m = __ballot(a);
      if (a) cbuf[wv][base + __popcll(m & ((1ull << lane) - 1ull))] = key[r];
      base += __popcll(m);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t key1 = cbuf[wv][lane < cnt ? lane : 0];
    bool a1 = lane < cnt;
    for (; bit >= 0 && cnt != need; --bit) {
      const bool one = (key1 >> bit) & 1ull;
      const int c0 = __popcll(__ballot(a1 && !one));
      if (need <= c0) {
        a1 = a1 && !one;
        cnt = c0;
      } else {
        a1 = a1 && one;
        need -= c0;
        cnt -= c0;
        if (bit >= 32) ph |= 1u << (bit - 32); else pl |= 1u << bit;
      }
    }
  }
  // bits > bit are resolved (prefix P): an element advances iff its key's resolved part is below P,
  // or equal and either the whole bucket advances (cnt == need: key < P + 2^(bit+1), one 64-bit
  // compare) or -- keys equal in all 64 bits -- it is among the first `need` of them by position
  const uint64_t P = ((uint64_t)ph << 32) | pl;
  if (cnt == need) {
    // bit <= 62 (at least one pass ran); -1 when all 64 bits were resolved.  No overflow: finite keys
    // stay below 0xFFF0000000000000
    const uint64_t T = P + (bit >= 0 ? (2ull << bit) : 1ull);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool adv = key[r] < T && (allfin || ((fin >> r) & 1u));
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(adv ? 1 : 0), ars, lane, 64 * r, 0);
    }
  } else {
    int taken = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool f = (fin >> r) & 1u;
      const bool eq = f && key[r] == P;
      const uint64_t m = __ballot(eq);
      const bool take = (f && key[r] < P) || (eq && taken + __popcll(m & ((1ull << lane) - 1ull)) < need);
      taken += __popcll(m);
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(take ? 1 : 0), ars, lane, 64 * r, 0);
    }
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
