// hbx_promote.hip -- batched successive-halving promotion on MI355X.
//
// Reference: HB_iteration.py:179-182 (SuccessiveHalving.process_results)
//     ranks = np.argsort(np.argsort(losses)); advance = ranks < num_configs[SH_iter]
// and HB_iteration.py:240-242 (SuccessiveResampling: ranks < max(1, n * (1 - 0.5))).
// Only REVIEW configurations (finite losses) are ranked; CRASHED ones (non-finite, register_result
// HB_iteration.py:102-106) never advance.  Mask only (the drop-in's need): a selection of the k-th
// (key, position) per bracket (sh_select_kernel: interpolation, then bisection of the key range).  With the sorted order requested: a stable sort of
// the losses (hbx_sort.h; one wave per bracket <= 1024, else one workgroup), then
// advance[position] = (rank < k).  Ties are ranked by position (stable), or -- HBX_ORDER_NUMPY, what the
// drop-in uses -- as numpy 1.26.4's unstable argsort ranks them (hbx_npsort.h): brackets whose tied
// losses straddle the k-th place are re-ranked on the device in numpy's order.
#include <cstring>

#include "hbx_common.h"
#include <hip/hip_ext.h>
#include "hbx_npsort.h"
#include "hbx_sort.h"
#include <stdlib.h>

int hbx_np_order_fix(const double* loss, const int64_t* seg_off, int64_t B, int64_t max_seg, const int64_t* order_in,
                     const double* k, int promote, int want_order, int64_t* order_out, uint8_t* advance,
                     int32_t* arrays, int64_t slots, int64_t slot_stride, int32_t* cnt_list, bool flagged,
                     hipStream_t s);
#define NPS_POOL 64  // workgroups (scratch slots) re-ranking flagged brackets after the selection

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
// k-th smallest (loss, position) of the bracket -- a selection, O(n) per bracket instead of a sort.
// One wave per bracket; element i = 64 r + lane sits in register r of lane `lane` (coalesced buffer
// loads issued together, 64 consecutive mask bytes per store).  Non-finite losses (CRASHED) and lanes
// past n hold NaN, which no comparison counts.
//   The search keeps a bracket [Lk, Hk) of order-preserving 64-bit keys (hbx_d2ord's order, -0.0 and
// 0.0 one key) with cL = #{keys < Lk} < kk <= cH = #{keys < Hk}; it starts from the high key words of
// the minimum and the maximum, and its ends live in scalar registers.  A key threshold K is compared in
// the loss domain (key(x) < K  <=>  x < val(K) for finite x), so counting the losses below it is one
// f64 compare and one carry-add per register plus one wave sum.  Rounds: (1) up to two interpolation
// rounds -- two thresholds around the k-th loss's position estimated linearly between the bracket ends
// (+-1.5 sigma of its rank, + 2), which isolate <= 64 keys in one round on smooth data; (2) bisection of
// the key range at its highest differing bit while the bracket holds > 64 keys (any data: at most 64
// rounds); (3) the <= 64 bracket losses compacted into one key per lane (LDS, position order) and the
// bisection finished with one compare and one ballot per round.  It ends when kk losses lie below one
// end of the bracket -- the mask is then one compare per element -- or when the bracket is a single key
// value: its copies are ranked by position (stable), as sh_promote_wave_kernel / sh_promote_kernel
// rank them.

constexpr int kBufDword3 = 0x00020000;  // gfx9 buffer resource word 3 (raw 32-bit data, range checked)

// finite x -> order-preserving key (-0.0 and 0.0 map to one key); val() inverts it on keys of finite
// values and of the thresholds between them (key(x) < K  <=>  x < val(K))
__device__ __forceinline__ uint64_t sel_key(double x) {
  const uint64_t u = (uint64_t)__double_as_longlong(x + 0.0);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double sel_val(uint64_t k) {
  return __longlong_as_double((long long)((k >> 63) ? (k ^ 0x8000000000000000ull) : ~k));
}
// a uniform 64-bit value into scalar registers (the bracket ends: the loops over them run in SALU)
__device__ __forceinline__ uint64_t sel_uniform(uint64_t x) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}

// One bracket (n <= 1024) by one wave: the mask written through `advp`, the count to *nadvp (nullable).
// Returns true (uniform) when tied losses straddle the k-th place: the copies of that key were taken by
// position, and numpy's order may take others (HBX_ORDER_NUMPY re-ranks the bracket afterwards).
__device__ __forceinline__ bool sh_select_wave(const double* __restrict__ lossp, int n, double kb,
                                               uint8_t* __restrict__ advp, int64_t* __restrict__ nadvp,
                                               double* __restrict__ cb, int lane) {
  constexpr int R = PW_PER_LANE;  // 16 registers x 64 lanes = 1024 elements
  if (n <= 0) {
    if (lane == 0 && nadvp) *nadvp = 0;
    return false;
  }
  // the bracket as buffer resources: loads past n return 0 and stores past n are dropped by the
  // hardware range check, so all 16 loads (and stores) are unconditional; the row offset goes in the
  // vector offset, whose constant part the compiler folds into the 12-bit immediate (no per-row SGPR)
  const __amdgpu_buffer_rsrc_t lrs = __builtin_amdgcn_make_buffer_rsrc((void*)lossp, (short)0, n * 8, kBufDword3);
  const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc((void*)advp, (short)0, n, kBufDword3);
  double v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) v[r] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(lrs, 8 * lane + 512 * r, 0, 0));
  // fz = sum of x * 0: NaN iff some loss is not finite (the loads past n returned 0.0)
  double fz = 0.0;
#pragma unroll
  for (int r = 0; r < R; ++r) fz = fma(v[r], 0.0, fz);
  // lanes past n become NaN (the partial row and the absent rows), then min / max: one vector compare
  // of floor((lane - n) / 64) against -r (lane + 64 r < n) and a select of the high dword per row (a
  // uniform row test would become per-row scalar mask arithmetic on the CU's shared scalar unit)
  const int nl = (lane - n) >> 6;
  const double qnan = __builtin_nan("");
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v[r]);
    const uint32_t hi = nl < -r ? (uint32_t)(u >> 32) : 0x7ff80000u;
    v[r] = __builtin_bit_cast(double, ((uint64_t)hi << 32) | (uint32_t)u);
  }
  double mn = __builtin_inf(), mx = -__builtin_inf();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    mn = fmin(mn, v[r]);
    mx = fmax(mx, v[r]);
  }
  int nfin = n;
  if (__builtin_amdgcn_ballot_w64(fz != fz)) {  // CRASHED entries present (uniform): they become NaN
    mn = __builtin_inf();
    mx = -__builtin_inf();
    nfin = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool f = v[r] - v[r] == 0.0;
      v[r] = f ? v[r] : qnan;
      mn = fmin(mn, v[r]);
      mx = fmax(mx, v[r]);
      nfin += (int)__popcll(__builtin_amdgcn_ballot_w64(f));
    }
  }
  // rank < k advances: the first kk ranks, kk = min(nfin, ceil(k)) (k > 0; NaN or k <= 0: none)
  const int kk = __builtin_amdgcn_readfirstlane(kb > 0.0 ? (kb >= (double)nfin ? nfin : (int)ceil(kb)) : 0);
  if (kk == nfin || kk == 0) {  // all the finite entries, or none
#pragma unroll
    for (int r = 0; r < R; ++r) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(kk && v[r] == v[r] ? 1u : 0u), ars, lane + 64 * r, 0, 0);
    if (lane == 0 && nadvp) *nadvp = kk;
    return false;
  }
  // the bracket: the high key words of the minimum and the maximum (a lane without a finite loss
  // contributes key(+inf) / key(-inf)); exact bounds only when the two coincide
  const uint32_t mnh = ~wave_reduce_dpp(~(uint32_t)(sel_key(mn) >> 32), OpMax());
  const uint32_t mxh = wave_reduce_dpp((uint32_t)(sel_key(mx) >> 32), OpMax());
  uint64_t Lk = (uint64_t)mnh << 32, Hk = ((uint64_t)mxh + 1ull) << 32;
  if (mnh == mxh) {
    Lk = ((uint64_t)mnh << 32) | ~wave_reduce_dpp(~(uint32_t)sel_key(mn), OpMax());
    Hk = (((uint64_t)mxh << 32) | wave_reduce_dpp((uint32_t)sel_key(mx), OpMax())) + 1ull;
  }
  int cL = 0, cH = nfin;
#define HBX_SEL_OPEN (cL != kk && cH != kk && ((Hk - Lk) >> 1) != 0ull)
  // (1) interpolation rounds
  for (int it = 0; it < 2 && HBX_SEL_OPEN && cH - cL > 64; ++it) {
    const double Ld = sel_val(Lk), Hd = sel_val(Hk), rng = Hd - Ld;
    if (!(rng - rng == 0.0)) break;  // range beyond the doubles: bisection only
    const double span = (double)(cH - cL);
    const double tm = fma(((double)(kk - cL) - 0.5) / span, rng, Ld);
    const double de = (1.5 * sqrt((double)(kk - cL) * (double)(cH - kk) / span) + 2.0) / span * rng;
    uint64_t klo = sel_key(tm - de), khi = sel_key(tm + de);
    klo = klo < Lk ? Lk : (klo > Hk ? Hk : klo);
    khi = khi < Lk ? Lk : (khi > Hk ? Hk : khi);
    if (klo <= Lk && khi >= Hk) break;  // the window covers the bracket
    const double lo = sel_val(klo), hi = sel_val(khi);
    uint32_t alo = 0, ahi = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      alo += v[r] < lo;
      ahi += v[r] < hi;
    }
    const uint32_t both = wave_reduce_dpp(alo | (ahi << 16), OpAdd());  // counts <= 1024
    const int clo = (int)(both & 0xffffu), chi = (int)(both >> 16);
    if (clo >= kk) {
      Hk = klo;
      cH = clo;
    } else if (chi < kk) {
      Lk = khi;
      cL = chi;
    } else {
      Lk = klo;
      cL = clo;
      Hk = khi;
      cH = chi;
    }
    Lk = sel_uniform(Lk);
    Hk = sel_uniform(Hk);
  }
  // (2) bisection at the highest bit where the bracket's keys can differ, while it holds > 64 keys
  while (HBX_SEL_OPEN && cH - cL > 64) {
    Lk = sel_uniform(Lk);
    Hk = sel_uniform(Hk);
    const int bt = 63 - __clzll((long long)(Lk ^ (Hk - 1ull)));
    const uint64_t M = (Lk & ~((2ull << bt) - 1ull)) | (1ull << bt);  // bt = 63: 2 << 63 = 0
    const double Md = sel_val(M);
    uint32_t a = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) a += v[r] < Md;
    const int cM = (int)wave_reduce_dpp(a, OpAdd());
    if (cM >= kk) {
      Hk = M;
      cH = cM;
    } else {
      Lk = M;
      cL = cM;
    }
  }
  if (HBX_SEL_OPEN) {
    // (3) compact the <= 64 bracket losses into one per lane, in position order, and finish there
    const double Ld = sel_val(Lk), Hd = sel_val(Hk);
    int base = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      // branchless: a lane outside the bracket writes its own dummy slot 64 + lane
      const uint64_t m = __builtin_amdgcn_ballot_w64(v[r] < Hd) & ~__builtin_amdgcn_ballot_w64(v[r] < Ld);
      const int at = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      cb[__builtin_amdgcn_inverse_ballot_w64(m) ? at : 64 + lane] = v[r];
      base += (int)__popcll(m);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int c0 = cL;
    const uint64_t key1 = lane < cH - cL ? sel_key(cb[lane]) : ~0ull;
    Lk = sel_uniform(Lk);
    Hk = sel_uniform(Hk);
    while (HBX_SEL_OPEN) {
      const int bt = 63 - __clzll((long long)(Lk ^ (Hk - 1ull)));
      const uint64_t M = (Lk & ~((2ull << bt) - 1ull)) | (1ull << bt);
      const int cM = c0 + (int)__popcll(__builtin_amdgcn_ballot_w64(key1 < M));
      if (cM >= kk) {
        Hk = M;
        cH = cM;
      } else {
        Lk = M;
        cL = cM;
      }
    }
  }
#undef HBX_SEL_OPEN
  bool tie = false;
  if (cL == kk || cH == kk) {  // exactly kk keys below T
    const double T = sel_val(cL == kk ? Lk : Hk);
#pragma unroll
    for (int r = 0; r < R; ++r) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v[r] < T ? 1u : 0u), ars, lane + 64 * r, 0, 0);
  } else {  // Hk = Lk + 1: the bracket holds copies of one key, the first kk - cL of them by position advance
    const double P = sel_val(Lk);
    const int need = kk - cL;
    int taken = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool eq = v[r] == P;
      const uint64_t m = __builtin_amdgcn_ballot_w64(eq);
      const int at = taken + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      const bool take = v[r] < P || (eq && at < need);
      taken += (int)__popcll(m);
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(take ? 1u : 0u), ars, lane + 64 * r, 0, 0);
    }
    tie = true;  // tied losses straddle the k-th place: numpy's order decides which copies advance
  }
  if (lane == 0 && nadvp) *nadvp = kk;
  return tie;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(10))) void sh_select_kernel(const double* __restrict__ loss,
                                                        const int64_t* __restrict__ seg_off, int64_t B,
                                                        const double* __restrict__ k,
                                                        uint8_t* __restrict__ advance,
                                                        int64_t* __restrict__ n_advance,
                                                        int32_t* __restrict__ tie_list,
                                                        int32_t* __restrict__ tie_count) {
  __shared__ double cbuf[4][128];  // per wave: the compacted bracket, then one dummy slot per lane
  // the wave index made visibly uniform: the bracket's bounds, k and buffer resources live in SGPRs
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t b = (int64_t)blockIdx.x * 4 + wv;
  if (b >= B) return;  // whole wave
  const int64_t s = seg_off[b];
  const int n = (int)(seg_off[b + 1] - s);
  const bool tie = sh_select_wave(loss + s, n, k[b], advance + s, n_advance ? n_advance + b : nullptr, cbuf[wv], lane);
  if (tie && tie_list && lane == 0) tie_list[atomicAdd(tie_count, 1)] = (int32_t)b;  // re-ranked after
}

// One bracket of n <= 1024 (the drop-in's process_results: HpBandSter ranks one bracket per call), ONE
// wave: the selection, no private segment (a kernel with scratch costs more to dispatch).  flag (device,
// nullable): 1 when tied losses straddle the k-th place (numpy's order must then re-rank the bracket,
// sh_rerank_one_kernel), else 0.  done (mapped, nullable): after every mask byte, `seq` -- or -seq when
// neg_on_tie and the bracket needs the re-rank (the host then launches it).  loss / advance may be mapped
// host memory (no copies).
__global__ __launch_bounds__(64) void sh_promote_one_kernel(const double* __restrict__ loss, int n, double kb,
                                                            uint8_t* __restrict__ advance, int32_t* flag,
                                                            int32_t* done, int32_t seq, int neg_on_tie) {
  __shared__ double cbuf[128];
  const int lane = threadIdx.x;
  const bool tie = sh_select_wave(loss, n, kb, advance, nullptr, cbuf, lane);
  if (flag && lane == 0) *flag = tie ? 1 : 0;
  if (done) {  // every mask byte is out (system scope) before the word the host polls for
    __threadfence_system();
    if (lane == 0) __hip_atomic_store(done, tie && neg_on_tie ? -seq : seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The numpy-order re-rank of that bracket (scratch: 4 x n int32, the flag in its first word): a no-op when
// the selection found no straddling tie (force: the host already knows it did).  done as above (seq).
__global__ __launch_bounds__(NPS_THREADS) void sh_rerank_one_kernel(const double* __restrict__ loss, int n, double kb,
                                                                     uint8_t* __restrict__ advance, int32_t* __restrict__ scr,
                                                                     int force, int32_t* done, int32_t seq) {
  constexpr int NM = 64 * PW_PER_LANE;  // n <= 1024
  __shared__ int go;
  __shared__ double xl[NM];              // the bracket's losses
  __shared__ int32_t wk[4 * NM];         // the sort's position arrays and range lists
  __shared__ NpsKV kv[NM];                // a std::sort finish's (key, position) pairs
  if (threadIdx.x == 0) go = force || scr[0];
  __syncthreads();
  if (go) {  // uniform
    // the sort reads and rewrites its keys and positions at random, many times over: all of it in LDS --
    // the losses may be mapped host memory (the drop-in's), the scratch is global memory; reading them in
    // place made a 1000-config bracket of quantised losses cost 0.43-0.5 ms
    NPS_STAMP(40);
    for (int i = threadIdx.x; i < n; i += blockDim.x) xl[i] = loss[i];
    __syncthreads();
    NPS_STAMP(41);
    nps_order_segment(xl, n, 1, kb, wk, wk + n, wk + 2 * n, wk + 3 * n, nullptr, advance, kv, NM);
    NPS_STAMP(42);
  }
  if (done) {
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

extern "C" {

#ifdef NPS_TIMING
int hbx_debug_nps(void* host) { return hipMemcpyFromSymbol(host, HIP_SYMBOL(nps_dbg), sizeof(nps_dbg)) == hipSuccess ? 0 : 1; }
#endif

int64_t hbx_sort_scratch_bytes(int64_t N);

// loss: device fp64[N] (non-finite = not ranked); seg_off: device int64[B+1]; k: device fp64[B];
// max_seg: host bound on the longest bracket; order: device int64[N] (sorted positions per bracket) or
// NULL when only the mask is wanted; advance: device uint8[N]; n_advance: device int64[B] (nullable).
int64_t hbx_sh_promote_scratch_bytes(int64_t B, int64_t max_seg, int64_t N, int32_t order_requested,
                                     int32_t order_mode) {
  const int64_t listb = 64 + 4 * (B + 1);
  if (max_seg <= 64 * PW_PER_LANE && !order_requested)  // selection: a pool of NPS_POOL re-ranking slots
    return order_mode == HBX_ORDER_NUMPY ? 16 * NPS_POOL * max_seg + listb : 0;
  return hbx_sort_scratch_bytes(N) + (order_mode == HBX_ORDER_NUMPY ? listb : 0);
}

int hbx_sh_promote(const double* loss, const int64_t* seg_off, int64_t B, int64_t max_seg, int64_t N,
                   const double* k, int64_t* order, uint8_t* advance, int64_t* n_advance, void* scratch,
                   int64_t scratch_bytes, void* stream) {
  return hbx_sh_promote_ex(loss, seg_off, B, max_seg, N, k, order, advance, n_advance, scratch, scratch_bytes,
                           HBX_ORDER_STABLE, nullptr, stream);
}

int hbx_sh_promote_ex(const double* loss, const int64_t* seg_off, int64_t B, int64_t max_seg, int64_t N,
                      const double* k, int64_t* order, uint8_t* advance, int64_t* n_advance, void* scratch,
                      int64_t scratch_bytes, int32_t order_mode, void* events, void* stream) {
  if (((!loss || !advance) && N > 0) || !seg_off || (!k && B > 0)) return hbx_fail(HBX_ERR_ARG, "hbx_sh_promote: null pointer");
  if (order_mode != HBX_ORDER_NUMPY && order_mode != HBX_ORDER_STABLE)
    return hbx_fail(HBX_ERR_ARG, "hbx_sh_promote_ex: order_mode %d", order_mode);
  if (B <= 0) return HBX_OK;
  hipStream_t st = (hipStream_t)stream;
  if (N <= 0) {  // every bracket empty: nothing advances (process_results over no results)
    if (n_advance) HBX_HIP(hipMemsetAsync(n_advance, 0, sizeof(int64_t) * B, st));
    return HBX_OK;
  }
  const bool np = order_mode == HBX_ORDER_NUMPY;
  const bool want_order = order != nullptr;
  const int64_t need = hbx_sh_promote_scratch_bytes(B, max_seg, N, want_order, order_mode);
  if (need > 0 && (!scratch || scratch_bytes < need))
    return hbx_fail(HBX_ERR_ARG, "promotion scratch too small: %lld < %lld bytes", (long long)scratch_bytes,
                    (long long)need);
  if (max_seg <= 64 * PW_PER_LANE && !order) {  // mask only: O(n) selection
    int32_t* pool = (int32_t*)scratch;
    const int64_t slots = (int64_t)NPS_POOL * max_seg;
    int32_t* cnt_list = np ? pool + 4 * slots : nullptr;
    if (np) HBX_HIP(hipMemsetAsync(cnt_list, 0, sizeof(int32_t), st));
    hipEvent_t* ev = (hipEvent_t*)events;  // optional: stamped at the selection kernel's start and end
    if (ev)
      hipExtLaunchKernelGGL(sh_select_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, ev[0], ev[1], 0, loss,
                            seg_off, B, k, advance, n_advance, np ? cnt_list + 16 : (int32_t*)nullptr, cnt_list);
    else
      hipLaunchKernelGGL(sh_select_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, loss, seg_off, B, k,
                         advance, n_advance, np ? cnt_list + 16 : (int32_t*)nullptr, cnt_list);
    HBX_LAUNCH_CHECK();
    if (!np) return HBX_OK;
    return hbx_np_order_fix(loss, seg_off, B, max_seg, nullptr, k, 1, 0, nullptr, advance, pool, slots, max_seg,
                            cnt_list, true, st);
  }
  char* sc = (char*)scratch;
  uint64_t* gk = (uint64_t*)sc;
  uint64_t* gk2 = gk + N;
  int32_t* gi = (int32_t*)(gk2 + N);
  int32_t* gi2 = gi + N;
  int64_t* ord = order ? order : (int64_t*)(sc + ((2 * (sizeof(uint64_t) + sizeof(int32_t)) * N + 7) & ~(size_t)7));
  if (max_seg <= 64 * PW_PER_LANE) {  // one wave per bracket; longer brackets: a block each
    hipLaunchKernelGGL(sh_promote_wave_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, loss, seg_off, B, k,
                       ord, advance, n_advance);
  } else {
    int tile = 64;
    while (tile < max_seg && tile < 4096) tile <<= 1;
    hipLaunchKernelGGL(sh_promote_kernel, dim3((unsigned)B), dim3(256), (sizeof(uint64_t) + sizeof(int32_t)) * tile,
                       st, loss, seg_off, k, tile, gk, gi, gk2, gi2, ord, advance, n_advance);
  }
  HBX_LAUNCH_CHECK();
  if (!np || N < 2) return HBX_OK;
  // the sort's key / position arrays are free again: [A | T | W | Lst] over the first 16 N bytes (indexed
  // by bracket offset; the order stays at 24 N), the flagged list after the sort scratch
  return hbx_np_order_fix(loss, seg_off, B, max_seg, ord, k, 1, want_order ? 1 : 0, order, advance, (int32_t*)sc, N, 0,
                          (int32_t*)(sc + hbx_sort_scratch_bytes(N)), false, st);
}

// One bracket (sh_promote_one_kernel, then -- numpy's order only -- sh_rerank_one_kernel, which re-ranks when
// the first one flagged a straddling tie): loss / advance device or mapped host pointers, n <= 1024, k by
// value; scratch: device int32[4 n] (HBX_ORDER_NUMPY only, else NULL).  Stream-ordered; done = seq last.
int hbx_sh_promote_one(const double* loss, int64_t n, double k, uint8_t* advance, void* scratch, int32_t order_mode,
                       int32_t* done, int32_t seq, void* stream) {
  if (!loss || !advance) return hbx_fail(HBX_ERR_ARG, "hbx_sh_promote_one: null pointer");
  if (n < 0 || n > 64 * PW_PER_LANE) return hbx_fail(HBX_ERR_ARG, "hbx_sh_promote_one: n=%lld", (long long)n);
  const bool np = order_mode == HBX_ORDER_NUMPY;
  if (np && !scratch) return hbx_fail(HBX_ERR_ARG, "hbx_sh_promote_one: scratch");
  int32_t* scr = (int32_t*)scratch;
  hipLaunchKernelGGL(sh_promote_one_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, loss, (int)n, k, advance,
                     np ? scr : (int32_t*)nullptr, np ? (int32_t*)nullptr : done, seq, 0);
  HBX_LAUNCH_CHECK();
  if (np) {
    hipLaunchKernelGGL(sh_rerank_one_kernel, dim3(1), dim3(NPS_THREADS), 0, (hipStream_t)stream, loss, (int)n, k,
                       advance, scr, 0, done, seq);
    HBX_LAUNCH_CHECK();
  }
  return HBX_OK;
}

// The drop-in's whole ranking step in ONE host call: the losses copied into the mapped buffer `pin`, the
// selection kernel, a spin on the word it stores last (bounded: then the stream is synchronised); only when
// it reports a tie that straddles the k-th place (numpy's order) does a second launch re-rank the bracket,
// then the mask is copied out of `pout` into `mask` (host uint8[n]).
static int spin_done(int32_t* done, int32_t a, int32_t b, hipStream_t stream, int32_t* seen_out) {
  // ~0.1 ms of polling covers the launch and the kernel; past it, block on the stream instead
  int32_t v = 0;
  bool seen = false;
  for (int i = 0; i < 200000 && !seen; ++i) {
    v = __atomic_load_n(done, __ATOMIC_ACQUIRE);
    seen = v == a || v == b;
  }
  if (!seen) {
    HBX_HIP(hipStreamSynchronize(stream));
    v = __atomic_load_n(done, __ATOMIC_ACQUIRE);
    if (v != a && v != b)
      return hbx_fail(HBX_ERR_HIP, "hbx_sh_advance_mapped: the kernel did not store its completion word");
  }
  *seen_out = v;
  return HBX_OK;
}

int hbx_sh_advance_mapped(const double* losses, int64_t n, double k, uint8_t* mask, double* pin, uint8_t* pout,
                          int32_t* done, int32_t seq, void* scratch, int32_t order_mode, void* stream) {
  if (!losses || !mask || !pin || !pout || !done) return hbx_fail(HBX_ERR_ARG, "hbx_sh_advance_mapped: null pointer");
  if (n <= 0) return HBX_OK;
  if (n > 64 * PW_PER_LANE) return hbx_fail(HBX_ERR_ARG, "hbx_sh_advance_mapped: n=%lld", (long long)n);
  if (seq <= 0) return hbx_fail(HBX_ERR_ARG, "hbx_sh_advance_mapped: seq must be positive");
  const bool np = order_mode == HBX_ORDER_NUMPY;
  if (np && !scratch) return hbx_fail(HBX_ERR_ARG, "hbx_sh_advance_mapped: scratch");
  if (losses != pin) memcpy(pin, losses, sizeof(double) * (size_t)n);  // (the caller may have filled pin itself)
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(sh_promote_one_kernel, dim3(1), dim3(64), 0, st, (const double*)pin, (int)n, k, pout,
                     (int32_t*)nullptr, done, seq, np ? 1 : 0);
  HBX_LAUNCH_CHECK();
  int32_t v = 0;
  int rc = spin_done(done, seq, -seq, st, &v);
  if (rc) return rc;
  if (v == -seq) {  // tied losses straddle the k-th place: numpy's order decides which copies advance
    hipLaunchKernelGGL(sh_rerank_one_kernel, dim3(1), dim3(NPS_THREADS), 0, st, (const double*)pin, (int)n, k, pout,
                       (int32_t*)scratch, 1, done, seq);
    HBX_LAUNCH_CHECK();
    rc = spin_done(done, seq, seq, st, &v);
    if (rc) return rc;
  }
  if (mask != pout) memcpy(mask, pout, (size_t)n);
  return HBX_OK;
}

int hbx_sh_advance_state(int64_t* state, int64_t n, double k, void* stream) {
  if (!state) return hbx_fail(HBX_ERR_ARG, "hbx_sh_advance_state: null state");
  const int32_t seq = (int32_t)(state[5] % 0x7ffffffe) + 1;
  state[5] = seq;
  double* pin = (double*)(intptr_t)state[0];
  uint8_t* pout = (uint8_t*)(intptr_t)state[1];
  const int dev = (int)state[6];
  int cur = dev;
  HBX_HIP(hipGetDevice(&cur));  // a dispatcher thread's current device may be another GPU
  if (cur != dev) HBX_HIP(hipSetDevice(dev));
  const int rc = hbx_sh_advance_mapped(pin, n, k, pout, pin, pout, (int32_t*)(intptr_t)state[2], seq,
                                       (void*)(intptr_t)state[3], (int32_t)state[4], stream);
  if (cur != dev) HBX_HIP(hipSetDevice(cur));
  return rc;
}

// pinned host memory the device reads and writes directly (coherent, mapped): the drop-in promotion's
// losses and mask travel with the kernel's own loads and stores, no copies.  Portable: mapped for every
// device of the process, whichever is current when it is allocated
int hbx_host_alloc(int64_t bytes, void** out) {
  if (!out || bytes <= 0) return hbx_fail(HBX_ERR_ARG, "hbx_host_alloc: %lld bytes", (long long)bytes);
  HBX_HIP(hipHostMalloc(out, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
  void* dp = nullptr;  // the engine passes the host address itself to kernels: it must be the device's too
  HBX_HIP(hipHostGetDevicePointer(&dp, *out, 0));
  if (dp != *out) {
    (void)hipHostFree(*out);
    *out = nullptr;
    return hbx_fail(HBX_ERR_UNSUPPORTED, "mapped host memory has a different device address");
  }
  return HBX_OK;
}

int hbx_host_free(void* p) {
  if (p) HBX_HIP(hipHostFree(p));
  return HBX_OK;
}

}  // extern "C"
