// hbx_kde.hip -- KDE acquisition on MI355X (gfx950): l(x)/g(x) scoring of candidates against the
// good/bad product-kernel KDEs of BOHB, and the exact argmin.
//
// Reference path: bohb.py:124-152 calls statsmodels KDEMultivariate.pdf
// (SM:kernel_density.py:162-196 -> SM:_kernel_base.py:456-518 gpke -> SM:kernels.py:23-65,108-125)
// twice per candidate and keeps the first candidate with the smallest max(1e-8,g)/max(l,1e-8).
//
// Engine structure (one acquisition, all on one HIP stream, no host round trip until the result):
//   acq_init         U = +inf, counters = 0
//   kde_logpdf<..>   x2 (good, bad): fp32 log-domain sum over observations, one candidate per lane,
//                    observations broadcast through the scalar path; per candidate ln S+, ln S-, bound
//   kde_combine      per-candidate score interval [lo, hi] (ln units) + block min of hi -> U
//   kde_shortlist    every candidate with lo <= U (the only ones that can be the argmin)
//   kde_exact        fp64 re-score of the shortlist in the reference's arithmetic/operation order
//   kde_final        strict-'<', first-index argmin over the exact scores
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stddef.h>

#include <atomic>
#include <mutex>
#include <new>
#include <vector>

#include "hbx_common.h"
#include <hip/hip_ext.h>
#include "hbx_kde_impl.h"
#include "hbx_npsort.h"
#include "hbx_sort.h"
#include <type_traits>

// ------------------------------------------------------------------------------------------
// model preparation

__host__ __device__ static void bucket_dims(int dc, int du, int* dc_pad, int* du_pad) {
  const int dcb[] = {0, 4, 8, 16, 24, 32, 64};
  const int dub[] = {0, 4, 8, 16, 32};
  *dc_pad = -1;
  *du_pad = -1;
  for (int b : dcb)
    if (dc <= b) { *dc_pad = b; break; }
  for (int b : dub)
    if (du <= b) { *du_pad = b; break; }
}

__host__ __device__ static int table_stride(int dc_pad, int du_pad) { return chunk_floats(dc_pad, du_pad); }
static int64_t n_chunks(int64_t n) { return (n + OBS_CHUNK - 1) / OBS_CHUNK; }
__device__ __forceinline__ int64_t n_chunks_dev(int64_t n) { return (n + OBS_CHUNK - 1) / OBS_CHUNK; }
// capacity of a table: the largest layout hbx_kde_prepare may choose for this bucket (exact-only KDEs,
// outside every bucket, keep no table: one float)
static int64_t table_floats(int64_t n, int dc_pad, int du_pad) {
  if (dc_pad < 0 || du_pad < 0) return 1;
  int a = chunk_floats(dc_pad, du_pad, 0, 0), b = chunk_floats(dc_pad, du_pad, OH_MAX_KC, 1);
  const int c = h_chunk_floats(dc_pad, OH_MAX_KC, 1), d = h32_chunk_floats(nsc_of(dc_pad), OH_MAX_KC, 1);
  a = a > b ? a : b;
  a = a > d ? a : d;
  // + the coarse h32 table (hbx_kde_impl.h), after the main one
  const int e = h32c_chunk_floats(nsc_of(dc_pad), 2);
  return n_chunks(n) * (int64_t)((a > c ? a : c) + e);
}

// Model preparation runs on the device from (data rows, bandwidths, level counts), so a refit needs
// no host round trip until its single read-back (hbx_kde_refit).  One or two KDEs per launch
// (PrepSet): block / block range k belongs to KDE k.
struct PrepArgs {
  const double* X;      // device f64[*][D]
  const int64_t* rows;  // device i64[n]
  const double* bw;     // device f64[D]
  const int32_t* nlev;  // device i32[D]
  KdeParams* P;
  int32_t* info;        // device i32[8]
  int32_t n, D;
  int32_t hm_allowed;   // HBX_HMODE not 0
  int32_t h32_allowed;  // HBX_H32 not 0
  int32_t co_allowed;   // HBX_COARSE not 0: the coarse h32 table beside the precise one
  int32_t nblk_table;   // blocks of this KDE in the table launches
  uint32_t vt[HBX_MAX_D / 32];  // bit d: dim d categorical ('u')
};
// The refit's output block published to device-mapped host memory (hbx_kde_refit_sync), every 32-bit word of it
// as one flagged 8-byte word (seq << 32 | word): the split's rows (n words: indices < 2^31), each KDE's
// bandwidths (2 D words: the doubles' low then high halves) and level counts (D words) by the parameter
// launch, then the two info records (16 words, `ll`) by the finishing blocks.  The host accepts a word only when
// it carries the call's sequence number, so it needs no ordering between the launches' stores and the host
// (dst == nullptr: nothing published)
struct PrepPub {
  uint64_t* dst;        // mapped flagged words: order [0, n), bw KDE k [n + 2 D k, + 2 D), nlev KDE k [n + 4 D + D k, + D)
  const uint32_t* src;  // the device output block
  uint64_t* ll;         // the two info records as 16 flagged words
  int32_t seq;
  int32_t n;            // rows of the split
  int32_t bw_off[2], nl_off[2], info_off[2];  // word offsets of KDE k's pieces in src
  int32_t D;
};
struct PrepSet {
  PrepArgs k[2];
  int32_t nk;
  PrepPub pub;
};

// The split's rows (KDE 0) and KDE k's bandwidths and level counts -- written by the launches before the
// parameter launch -- published by the parameter launch's block k (thread t of nt) as flagged words: the rows
// of a 400-observation refit are ~2 stores per thread, not 14 dependent load/store pairs of one wave
__device__ __forceinline__ void prep_publish_rows(const PrepPub& q, int k, int t, int nt) {
  const uint64_t tag = (uint64_t)(uint32_t)q.seq << 32;
  auto put = [&](int64_t i, uint32_t w) {
    __hip_atomic_store(q.dst + i, tag | w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  };
  if (k == 0) {
    const int64_t* order = (const int64_t*)q.src;  // (the order sits at word 0 of the block)
    for (int i = t; i < q.n; i += nt) put(i, (uint32_t)order[i]);
  }
  const int64_t bw0 = (int64_t)q.n + 2 * (int64_t)q.D * k, nl0 = (int64_t)q.n + 4 * (int64_t)q.D + (int64_t)q.D * k;
  for (int i = t; i < 2 * q.D; i += nt) put(bw0 + i, q.src[q.bw_off[k] + i]);
  for (int i = t; i < q.D; i += nt) put(nl0 + i, q.src[q.nl_off[k] + i]);
}
// KDE k's info record (from registers) as flagged 8-byte words: (prep_publish_info below reads it back)
__device__ __forceinline__ void prep_publish_vals(const PrepPub& q, const int32_t (&vals)[8], int k) {
  for (int i = 0; i < 8; ++i)
    __hip_atomic_store(q.ll + 8 * k + i, ((uint64_t)(uint32_t)q.seq << 32) | (uint32_t)vals[i], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}
// KDE k's info record (thread 0's own stores of prep_finish_one, read back by it) as flagged 8-byte words:
// each carries the call's sequence number beside its value, so the host knows every word from the word itself
// and no store has to wait for the others' acknowledgement (a completion word after an acknowledged record
// cost ~12k cycles of round trip to host memory).  The host reads the block only once the flags match AND
// the stream has completed (hbx_kde_refit_sync), so the parameter launch's unflagged words come from launches
// that have ended.
__device__ __forceinline__ void prep_publish_info(const PrepPub& q, const PrepArgs& A, int k) {
  for (int i = 0; i < 8; ++i)
    __hip_atomic_store(q.ll + 8 * k + i, ((uint64_t)(uint32_t)q.seq << 32) | (uint32_t)A.info[i], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ bool prep_cat(const PrepArgs& A, int d) { return (A.vt[d >> 5] >> (d & 31)) & 1u; }

__host__ __device__ __forceinline__ ColStats* col_stats(KdeParams* P) { return (ColStats*)((char*)P + HBX_COLSTATS_OFF); }

// Column statistics of every (KDE, dim), one workgroup each (blocks [k*D, (k+1)*D) belong to KDE k):
// the mean of a continuous column (the centre of the scaled coordinates: any finite centre is correct
// -- table and candidates use the same one -- it only keeps the fp32 expansion well conditioned, so the
// summation order is free) and the largest code of a categorical column.
__global__ __launch_bounds__(256) void kde_colstats_kernel(PrepSet ps) {
  const PrepArgs& A = (int)blockIdx.x >= ps.k[0].D ? ps.k[1] : ps.k[0];
  const int d = blockIdx.x % ps.k[0].D;
  const int n = A.n, D = A.D;
  ColStats* cs = col_stats(A.P);
  __shared__ double red[4];
  __shared__ int mred[4];
  if (!prep_cat(A, d)) {
    double acc = 0.0;
    for (int j = threadIdx.x; j < n; j += 256) acc += A.X[A.rows[j] * (int64_t)D + d];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) cs->mean[d] = ((red[0] + red[1]) + (red[2] + red[3])) / (double)n;
  } else {
    int m = -1;
    for (int j = threadIdx.x; j < n; j += 256) {
      const double v = A.X[A.rows[j] * (int64_t)D + d];
      m = max(m, (!(v >= 0.0 && v < 1024.0) || v != floor(v)) ? 100000 : (int)v);
    }
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) mred[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int mm = max(max(mred[0], mred[1]), max(mred[2], mred[3]));
      cs->maxcode[d] = mm >= 100000 ? -1 : mm;
    }
  }
}

// the table launch's block counter of a KDE (in its parameter buffer's staging area, after the info
// record; zeroed by kde_params_kernel)
__device__ __forceinline__ int32_t* prep_counter(KdeParams* P) {
  return (int32_t*)((char*)P + HBX_PARAM_STAGE + 8 * HBX_MAX_D + 4 * HBX_MAX_D + 32);
}

// PREP_STAMPS (diagnostic builds only): s_memtime at the phase boundaries of the parameter build (block 0) and of
// the table launch (block 1's and the finishing block's thread 0) into a buffer of their own, read back by
// hbx_debug_prep_stamps; no stamp executes in the product build
#ifdef PREP_STAMPS
__device__ unsigned long long prep_stamps[32];
#define PSTAMP(i) \
  if (threadIdx.x == 0) prep_stamps[i] = __builtin_amdgcn_s_memtime()
#else
#define PSTAMP(i)
#endif

// LDS of the parameter build
struct ParamsScratch {
  double t0[HBX_MAX_D], t1[HBX_MAX_D], h[HBX_MAX_D], mean[HBX_MAX_D];
  int32_t c[HBX_MAX_D], maxc[HBX_MAX_D], cm[HBX_MAX_D], cd[HBX_MAX_D];
  int32_t ix[HBX_MAX_D];   // index of dim d within its class (continuous slot k, categorical slot u, constant dim)
  uint8_t kind[HBX_MAX_D]; // 0 continuous, 1 active categorical, 2 constant (one level, h = 0), 3 unsupported
  int32_t ohs[HBX_MAX_D];  // first one-hot position of each active categorical dim's block
  int32_t du, dcp, dup, exo, neg, dc_tot, du_tot, dc, nconst, kc, tot;
};

// The parameter block P of one KDE (the whole workgroup calls it; P in global memory or in LDS): the per-dim
// transcendentals and fields in parallel (each dim's slot within its class from one wave's ballots), the
// sums by thread 0 in dim order, the one-hot layout and the kernel mode.
__device__ __forceinline__ void kde_params_body(const PrepArgs& A, KdeParams* P, const ColStats* cs, ParamsScratch& S) {
  const int D = A.D, n = A.n;
  const int tid = threadIdx.x;
  uint32_t* pz = (uint32_t*)P;
  for (int i = tid; i < (int)(sizeof(KdeParams) / 4); i += blockDim.x) pz[i] = 0u;
  if (tid == 0) S.neg = 0;
  // per dim: continuous -> ln h and the scale; categorical -> log2 of the match / mismatch factors, and its class
  const double LOG2E = 1.4426950408889634;
  if (blockIdx.x == 0) PSTAMP(0);
  for (int d = tid; d < D; d += blockDim.x) {
    const double h = A.bw[d];
    const int c = A.nlev[d];
    S.h[d] = h;
    S.c[d] = c;
    S.mean[d] = cs->mean[d];
    S.maxc[d] = cs->maxcode[d];
    if (!prep_cat(A, d)) {
      S.kind[d] = 0;
      S.t0[d] = (h > 0.0) ? log(h) : 0.0;
      S.t1[d] = (h > 0.0) ? sqrt(LOG2E / 2.0) / h : 0.0;
    } else {
      // single observed level: match -> 1, mismatch -> 0/0 = NaN (a constant dim); c < 2 otherwise, h <= 0 or
      // NaN (c == -1: codes not integers in [0, 1024)): not modelled
      S.kind[d] = (c == 1 && h == 0.0) ? 2 : ((c < 2 || !(h > 0.0) || h != h) ? 3 : 1);
      const double a = 1.0 - h, b = h / (double)(c - 1);
      S.t0[d] = log2(b);
      S.t1[d] = (a == 0.0) ? -INFINITY : log2(fabs(a));
    }
  }
  __syncthreads();
  if (blockIdx.x == 0) PSTAMP(1);
  if (tid < 64) {  // each dim's slot within its class: ballots over 64-dim groups, in dim order
    const uint64_t below = (1ull << tid) - 1ull;
    int bc = 0, bu = 0, bk = 0, nu = 0;
    for (int g = 0; g < D; g += 64) {
      const int d = g + tid;
      const int kd = d < D ? S.kind[d] : -1;
      const uint64_t mc = __ballot(kd == 0), mu = __ballot(kd == 1), mk = __ballot(kd == 2), ma = __ballot(kd >= 1);
      if (d < D) S.ix[d] = kd == 0 ? bc + __popcll(mc & below) : kd == 1 ? bu + __popcll(mu & below)
                                                                         : bk + __popcll(mk & below);
      bc += __popcll(mc);
      bu += __popcll(mu);
      bk += __popcll(mk);
      nu += __popcll(ma);
    }
    if (tid == 0) {
      S.dc_tot = bc;  // every continuous dim has a slot
      S.du_tot = nu;  // every categorical dim, active or not
      S.du = bu;
      S.nconst = bk;
    }
  }
  __syncthreads();
  for (int d = tid; d < D; d += blockDim.x) {
    const double h = S.h[d];
    const int kd = S.kind[d], ix = S.ix[d];
    P->vartype[d] = kd != 0 ? 1 : 0;
    P->nlev[d] = S.c[d];
    P->bw[d] = h;
    if (kd == 0) {
      P->cont_dim[ix] = d;
      const double m = S.mean[d];
      P->center[ix] = (m == m && m - m == 0.0) ? m : 0.0;
      if (!(h > 0.0)) {
        P->nan_all = 1;  // exp(-0/0) * ... / 0 -> NaN for every candidate
        P->cont_scale[ix] = 0.0;
      } else {
        P->cont_scale[ix] = S.t1[d];
      }
    } else if (kd == 2) {
      P->const_dim[ix] = d;
    } else if (kd == 3) {
      P->unsupported = 1;
    } else {
      const double a = 1.0 - h;
      P->cat_dim[ix] = d;
      P->cat_maxcode[ix] = S.maxc[d];
      S.cm[ix] = S.maxc[d];
      S.cd[ix] = d;
      P->cat_delta[ix] = (a == 0.0) ? -1e30f : (float)(S.t1[d] - S.t0[d]);
      P->cat_negf[ix] = (a < 0.0) ? 1.f : 0.f;
      if (a < 0.0) {
        P->has_neg = 1;
        S.neg = 1;
      }
    }
  }
  if (tid == 0) {  // the sums in dim order (np.prod(bw[iscontinuous]) sequential: the reference's order)
    double sum_ln_h = 0.0, m0 = 0.0, lb_sum = 0.0, prod_bw_c = 1.0;
    float sad = 0.f;
    // branch-free (a factor 1 or a term +0.0 where a dim does not count: exact), so the loads of several dims
    // are in flight at once
#pragma unroll 4
    for (int d = 0; d < D; ++d) {
      const int kd = S.kind[d];
      const double h = S.h[d], lb = S.t0[d], la = S.t1[d];
      prod_bw_c *= (kd == 0) ? h : 1.0;
      sum_ln_h += (kd == 0 && h > 0.0) ? lb : 0.0;
      m0 += (kd == 1) ? ((la > lb) ? la : lb) : 0.0;
      lb_sum += (kd == 1) ? lb : 0.0;
      sad += (kd == 1 && 1.0 - h != 0.0) ? fabsf((float)(la - lb)) : 0.f;
    }
    int dcp, dup;
    bucket_dims(S.dc_tot, S.du_tot, &dcp, &dup);
    P->n = n;
    P->D = D;
    P->dc_pad = dcp;
    P->du_pad = dup;
    const int exo = (dcp < 0 || dup < 0) ? 1 : 0;
    P->exact_only = exo;
    P->stride = exo ? 0 : table_stride(dcp, dup);
    const int dc = S.dc_tot;
    P->dc = dc;
    P->du = S.du;
    S.dcp = dcp;
    S.dup = dup;
    S.exo = exo;
    P->nconst = S.nconst;
    P->m0_log2 = m0;
    P->lb_sum = lb_sum;
    P->prod_bw_c = prod_bw_c;
    P->sum_abs_delta = sad;
    P->log_norm = -log((double)n) - sum_ln_h - 0.5 * (double)dc * log(2.0 * M_PI) + m0 * M_LN2;
    P->X = A.X;
    P->rows = A.rows;
  }
  __syncthreads();  // (S.neg and the slot arrays from every thread)
  if (blockIdx.x == 0) PSTAMP(2);
  for (int t = tid; t < 64; t += blockDim.x) {  // padding read branch-free by the scoring prologue: never a match
    P->oh_col[t] = 0;
    P->oh_val[t] = NAN;
  }
  // categorical mode: one-hot on the f16 matrix cores when every active dim has integer codes in
  // [0, 1024) and the one-hot width sum(max code + 1) fits OH_MAX_KC K-steps; else VALU matching.
  // One-hot positions: every dim's block starts at an even position (a padding position, level -1,
  // never matches) -- the sparse matrix-core kernel relies on adjacent pairs never spanning dims.
  // Thread 0 places the blocks (each dim's first level position), then one thread per dim fills its block.
  const int du = S.du;
  if (tid == 0) {
    int tot = 0;
    bool ok = true;
    for (int u = 0; u < du; ++u) {
      if (S.cm[u] < 0) {
        ok = false;
      } else {
        S.ohs[u] = (tot + 1) & ~1;
        tot = S.ohs[u] + S.cm[u] + 1;
      }
    }
    S.kc = (!S.exo && du > 0 && ok && 2 * tot <= 32 * OH_MAX_KC && tot <= 64) ? (2 * tot + 31) / 32 : 0;
    S.tot = tot;
  }
  __syncthreads();
  const int kc = S.kc;
  if (kc > 0) {
    for (int u = tid; u < du; u += blockDim.x) {
      int t = S.ohs[u];
      P->oh_start[u] = t;
      if (t > 0 && (u == 0 || t != S.ohs[u - 1] + S.cm[u - 1] + 1)) {  // the padding position before the block
        P->oh_dim[t - 1] = u;
        P->oh_level[t - 1] = -1;
      }
      for (int l = 0; l <= S.cm[u]; ++l, ++t) {
        P->oh_dim[t] = u;
        P->oh_level[t] = l;
        P->oh_col[t] = S.cd[u];
        P->oh_val[t] = (double)l;
      }
    }
  }
  if (threadIdx.x != 0) return;
  // (read back from LDS, not from the P just written: see above)
  const int dcp = S.dcp, dup = S.dup, has_neg = S.neg;
  if (S.exo) {  // no table, no fp32 scoring: the acquisition re-scores every candidate
    P->hmode = 0;
    P->nsc = 0;
    P->chunk_floats = 0;
    return;
  }
  if (kc > 0) {
    P->kc = kc;
    P->oh_total = S.tot;
  }
  // continuous product on the f16 matrix cores (hi/lo split) when it has >= 8 dims (one full
  // 32-wide K-step; the C_j pieces ride in dims 0-2) and the categorical part is one-hot (or absent);
  // otherwise the exact f32 MFMA product.  |C_j| beyond the f16 range is caught after the table.
  const bool hm_ok = (du == 0 || kc > 0) && dcp >= 8;
  int hmode = (hm_ok && A.hm_allowed) ? 1 : 0;
  // the 32x32-tile kernel (hbx_score_h32.hip) in the buckets it is built for
  if (hmode && A.h32_allowed && h32_ok(nsc_of(dcp), h32_kp(kc), has_neg)) hmode = 2;
  P->hmode = hmode;
  P->nsc = nsc_of(dcp);
  P->chunk_floats = hmode == 2 ? h32_chunk_floats(nsc_of(dcp), h32_kp(kc), has_neg)
                               : (hmode ? h_chunk_floats(dcp, kc, has_neg) : chunk_floats(dcp, dup, kc, kc ? has_neg : 0));
  // the coarse pre-screen table (unsigned h32 KDEs): after the main table in the same buffer
  const bool co = hmode == 2 && !has_neg && A.co_allowed;
  P->coarse_chunk_floats = co ? h32c_chunk_floats(nsc_of(dcp), h32_kp(kc)) : 0;
  P->coarse_off = co ? (int32_t)(n_chunks_dev(n) * P->chunk_floats) : 0;
  if (blockIdx.x == 0) PSTAMP(3);
}

__global__ __launch_bounds__(256) void kde_params_kernel(PrepSet ps) {
  const PrepArgs& A = blockIdx.x ? ps.k[1] : ps.k[0];  // (no dynamic index into the kernel arguments)
  __shared__ ParamsScratch S;
  if (threadIdx.x == 0) *prep_counter(A.P) = 0;  // the table launch's block counter (finish by the last block)
  if (ps.pub.dst) prep_publish_rows(ps.pub, blockIdx.x ? 1 : 0, threadIdx.x, blockDim.x);
  kde_params_body(A, A.P, col_stats(A.P), S);
  // the published words acknowledged before the launch ends: the finishing blocks' flagged info words follow them
  if (ps.pub.dst) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Fill the chunked observation table (layout in hbx_kde_impl.h).  X'_jc = s_c * (X_jc - mu_c),
// C_j = -sum_c X'_jc^2 + lb_sum - M0 (log2 units).  One thread per observation row (a serial walk over
// its dims), 64-thread blocks so a 1e4-row table spreads over ~150 CUs.  `hm` / `chunk_f` select the
// layout; |C_j| and |X'| maxima go to *cmax_acc / P->xmax.
// The one-hot positions observation row x matches, as a bit mask: position oh_start[u] + l for each active
// categorical dim u whose code is the integer l in [0, max code] -- exactly the positions t where
// x[oh_col[t]] == oh_val[t] (padding positions hold NaN: never), found with du loads instead of oh_total.
__device__ __forceinline__ uint64_t onehot_hits(const double* x, const KdeParams* P, bool ok) {
  uint64_t hit = 0;
  if (!ok) return hit;
  for (int u = 0; u < P->du; ++u) {
    const double v = x[P->cat_dim[u]];
    if (v >= 0.0 && v <= (double)P->cat_maxcode[u]) {
      const int l = (int)v;
      if (v == (double)l) hit |= 1ull << (P->oh_start[u] + l);
    }
  }
  return hit;
}

__device__ __forceinline__ void kde_table_body(const double* __restrict__ x, const KdeParams* __restrict__ P,
                                               KdeParams* __restrict__ Pw, float* __restrict__ table, int j,
                                               int hm, int chunk_f, float* cmax_acc, _Float16* hst) {
  // hst: this thread's LDS row (H32_ROW_MAX halves) where the h32 layout's dense slots are assembled
  // P: the parameters as read (an LDS copy); Pw: the global block, written (xmax, cmax / cmax2,
  // const_level) -- fields disjoint from every one read here
  const int n = P->n;
  const int nslots = ((n + OBS_CHUNK - 1) / OBS_CHUNK) * OBS_CHUNK;
  const bool ok = j < n;
  const bool slot = j < nslots;
  const int dc = P->dc, du = P->du, dcp = P->dc_pad, dup = P->du_pad;
  const int KP = kp_of(dcp);
  float* ch = table + (int64_t)(j / OBS_CHUNK) * chunk_f;
  const int jj = j % OBS_CHUNK;
  // hm: 0 = f32 layout, 1 = hmode (16x16 kernel), 2 = h32 (32x32 kernel, no chunk header)
  const int KTP = hm == 2 ? h32_ktp(P->nsc, h32_kp(P->kc), P->has_neg) : h_ktp(dcp, P->kc);
  _Float16* hrow = (_Float16*)(hm == 2 ? ch : ch + OBS_CHUNK) + jj * KTP;
  // the coarse pre-screen row (h32 KDEs with a coarse table; hbx_kde_impl.h): dense C pieces, ones, Xh
  _Float16* crow = (hm == 2 && P->coarse_off > 0 && slot)
                       ? (_Float16*)(table + P->coarse_off + (int64_t)(j / OBS_CHUNK) * P->coarse_chunk_floats) +
                             jj * h32c_ktp(P->nsc, h32_kp(P->kc))
                       : nullptr;
  double C = 0.0;
  // hmode rows are written 16 bytes (8 halves) at a time: two dims' h, l, h, l per store
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  h8 grp = {};
  const int nd32 = h32_nd(P->nsc);
  if (hm == 2) {
    for (int q = 0; q < 2 * nd32; ++q) *(h8*)(hst + 8 * q) = h8{};
    // eight dims at a time with no branch between them: their loads in flight together, then the stores and
    // the eight |X'| maxima (independent reductions); C accumulates in dim order as below
    for (int k0 = 0; k0 < dcp; k0 += 8) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int k = k0 + i;
        const bool live = ok && k < dc;
        const double xv = x[live ? P->cont_dim[k] : 0];
        v[i] = live ? (float)(P->cont_scale[k] * (xv - P->center[k])) : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int k = k0 + i;
        C -= (double)v[i] * (double)v[i];
        if (slot && k < dcp) {  // slots 6 + 3k: Xh, Xl, Xh
          const float vc = fminf(fmaxf(v[i], -60000.f), 60000.f);
          const _Float16 h = (_Float16)vc;
          const _Float16 l = (_Float16)(vc - (float)h);
          hst[6 + 3 * k] = h;
          hst[7 + 3 * k] = l;
          hst[8 + 3 * k] = h;
        }
      }
      // the eight |X'| maxima over the wave's 64 rows at once: every lane writes its eight, then lane (i, p)
      // takes dim i's rows 8p..8p+7 and the 8 lanes of dim i combine by lane exchanges (eight serial wave
      // reductions cost ~5k cycles per block); non-negative floats order as their bit patterns
      __shared__ __align__(16) uint32_t vab[8][64];
      const int ln = threadIdx.x & 63;
#pragma unroll
      for (int i = 0; i < 8; ++i) vab[i][ln] = __float_as_uint(fabsf(v[i]));
      __syncthreads();
      {
        const int i = ln >> 3, p8 = ln & 7;
        const uint4 q0 = *(const uint4*)&vab[i][8 * p8], q1 = *(const uint4*)&vab[i][8 * p8 + 4];
        uint32_t mx = max(max(max(q0.x, q0.y), max(q0.z, q0.w)), max(max(q1.x, q1.y), max(q1.z, q1.w)));
        mx = max(mx, lane_xor_u32(mx, 1, ln));
        mx = max(mx, lane_xor_u32(mx, 2, ln));
        mx = max(mx, lane_xor_u32(mx, 4, ln));
        if (p8 == 0 && k0 + i < dc) atomicMax((unsigned int*)&Pw->xmax[k0 + i], mx);
      }
      __syncthreads();  // (vab is rewritten by the next eight dims)
    }
  }
#pragma unroll 8
  for (int k = 0; k < (hm == 2 ? 0 : hm ? dcp : KP - 2); ++k) {
    float v = 0.f;
    if (ok && k < dc) v = (float)(P->cont_scale[k] * (x[P->cont_dim[k]] - P->center[k]));
    C -= (double)v * (double)v;
    if (slot) {
      if (hm) {
        const float vc = fminf(fmaxf(v, -60000.f), 60000.f);
        const _Float16 h = (_Float16)vc;
        const _Float16 l = (_Float16)(vc - (float)h);
        const int o = 4 * (k & 1);
        grp[o + 0] = h;
        grp[o + 1] = l;
        grp[o + 2] = h;
        grp[o + 3] = l;
        if (k & 1) *(h8*)(hrow + 4 * (k - 1)) = grp;
      } else {
        ch[(2 + k) * KROW + jj] = v;
      }
    }
    // |X'| maximum of the wave (non-negative floats order as their bit patterns)
    const uint32_t a = wave_reduce_dpp(__float_as_uint(fabsf(v)), OpMax());
    if ((threadIdx.x & 63) == 0 && k < dc) atomicMax((unsigned int*)&Pw->xmax[k], a);
  }
  if (blockIdx.x == 1) PSTAMP(14);
  const h8 z8 = {};
  if (hm == 1 && slot) {  // dc_pad is a multiple of 8: the dims filled whole groups
    for (int k = 4 * dcp; k < 32 * P->nsc; k += 8) *(h8*)(hrow + k) = z8;
    for (int k = 32 * (P->nsc + P->kc); k < KTP; k += 8) *(h8*)(hrow + k) = z8;
  }
  if (hm == 2 && slot)  // row padding past the index words (rows are 16-byte aligned, KTP % 8 == 0); the
    // parity block of a signed KDE is rewritten below
    for (int k = (16 * nd32 + 32 * h32_kp(P->kc) + 2 * h32_ixw(h32_kp(P->kc))) & ~7; k < KTP; k += 8)
      *(h8*)(hrow + k) = z8;
  if (P->kc == 0) {
    // the f32 layout's code block only: a matrix-core layout with kc == 0 has no active categorical dim (hm_ok),
    // and du_pad > 0 there means single-level dims alone -- writing their codes would overwrite row data
    if (hm == 0)
      for (int u = 0; u < dup; ++u) {
        const float v = (ok && u < du) ? (float)x[P->cat_dim[u]] : -2.0f;
        if (slot) ch[KP * KROW + jj * dup + u] = v;
      }
  } else if (slot && hm == 2) {
    // 2:4-compressed one-hot (h32 layout, hbx_kde_impl.h): per step s and group g (positions t0 = 32s + 4g
    // .. t0 + 3) the f16 hi / lo of delta_u for the observation's level in the pair (t0, t0+1) and in
    // (t0+2, t0+3), and the index nibble i0 | i1 << 2 (i0: 0 or 1, i1: 2 or 3); index dword ksp h + s
    // holds groups 4h..4h+3 of step s
    const int kp = h32_kp(P->kc);
    _Float16* cz = hrow + 16 * nd32;
    _Float16* cp = hrow + h32_par(P->nsc, kp);  // parity block (signed KDEs)
    _Float16* cc = crow ? crow + 16 * h32c_nd(P->nsc) : nullptr;
    const int ksp = h32_ksp(kp);
    if (blockIdx.x == 1) PSTAMP(17);
    // the matched position t of dim u (at most one per dim, never two in one pair: every dim's block starts at
    // an even position) puts delta_u's hi / lo (and the parity 1/2) at half t >> 1 of its part; every other
    // half is 0: zero-filled first, then one scattered half per matched dim (this thread's own row, in order)
    for (int q = 0; q < 2 * kp; ++q) {
      *(h8*)(cz + 8 * q) = z8;
      *(h8*)(cz + 16 * kp + 8 * q) = z8;
      if (cc) *(h8*)(cc + 8 * q) = z8;
      if (P->has_neg) *(h8*)(cp + 8 * q) = z8;
    }
    if (blockIdx.x == 1) PSTAMP(18);
    // eight dims at a time, every load of the eight issued before the first use (the positions matched are
    // those of onehot_hits: x[oh_col[t]] == oh_val[t])
    uint64_t hit = 0;
    for (int u0 = 0; u0 < (ok ? du : 0); u0 += 8) {
      int cd[8], cm[8], os[8];
      float dlt[8], ngf[8];
      double v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {  // (indices < du + 8 <= 72: inside the HBX_MAX_D arrays)
        cd[i] = P->cat_dim[u0 + i];
        cm[i] = u0 + i < du ? P->cat_maxcode[u0 + i] : -1;
        os[i] = P->oh_start[u0 + i];
        dlt[i] = P->cat_delta[u0 + i];
        ngf[i] = P->cat_negf[u0 + i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = x[u0 + i < du ? cd[i] : 0];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (!(v[i] >= 0.0 && v[i] <= (double)cm[i]) || v[i] != (double)(int)v[i]) continue;
        const int t = os[i] + (int)v[i], h = t >> 1;
        hit |= 1ull << t;
        const float dl = fminf(fmaxf(dlt[i], -60000.f), 60000.f);
        const float hi = (float)(_Float16)dl;
        cz[h] = (_Float16)hi;
        cz[16 * kp + h] = (_Float16)(fabsf(dl) < 60000.f ? dl - hi : 0.f);
        if (cc) cc[h] = (_Float16)hi;
        if (P->has_neg && ngf[i] != 0.f) cp[h] = (_Float16)0.5f;
      }
    }
    if (blockIdx.x == 1) PSTAMP(19);
    if (blockIdx.x == 1) PSTAMP(20);
    // index nibble of group g (positions t0 = 32 s + 4 g .. t0 + 3): i0 | i1 << 2 with i0 = 0 or 1, i1 = 2 or 3
    // (1 / 3 where the odd position of the pair matched); dword ksp h + s holds groups 4h..4h+3 of step s
    uint32_t iw[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int hh = q / ksp, st = q - hh * ksp, sh = 32 * st + 16 * hh;
      const uint32_t win = (st < kp && hh < 2 && sh < 64) ? (uint32_t)(hit >> sh) & 0xFFFFu : 0u;
      iw[q] = (st < kp && hh < 2) ? 0x8888u | ((win & 0xAAAAu) >> 1) : 0u;
    }
    for (int w = 0; w < (crow ? 2 : 1); ++w) {  // index words of the precise row, then of the coarse row
      uint32_t* ix = w == 0 ? (uint32_t*)(hrow + 16 * nd32 + 32 * kp) : (uint32_t*)(crow + 16 * h32c_nd(P->nsc) + 16 * kp);
      if (kp == 1) {  // dwords 2b + h, b = bit 4 of the row (bank spread of the kernel's b64 reads)
        const int b = (jj >> 4) & 1;
        for (int q = 0; q < 4; ++q) ix[q] = (q >> 1) == b ? iw[q & 1] : 0u;
      } else {
        for (int q = 0; q < 2 * ksp; ++q) ix[q] = iw[q];
      }
    }
  } else if (slot) {
    const int W = P->kc * 32;  // one-hot halves per observation
    _Float16* oh;
    _Float16* par;
    if (hm == 1) {
      oh = hrow + 32 * P->nsc;
      par = (_Float16*)(ch + OBS_CHUNK + OBS_CHUNK * KTP / 2) + jj * h_kpp(P->kc);
    } else {
      oh = (_Float16*)(ch + KP * KROW) + jj * W;
      par = (_Float16*)(ch + KP * KROW) + OBS_CHUNK * W + jj * W;
    }
    const uint64_t hit = onehot_hits(x, P, ok);
    h8 og = {}, pg = {};
#pragma unroll 8
    for (int k = 0; k < W; ++k) {
      const int t = k >> 1, p = k & 1;
      float v = 0.f, pv = 0.f;
      if (t < P->oh_total) {
        const int u = P->oh_dim[t];
        if ((hit >> t) & 1u) {
          const float dl = fminf(fmaxf(P->cat_delta[u], -60000.f), 60000.f);
          const float hi = (float)(_Float16)dl;
          v = (p == 0) ? hi : (fabsf(dl) < 60000.f ? dl - hi : 0.f);
          pv = (p == 0 && P->cat_negf[u] != 0.f) ? 1.f : 0.f;
        }
      }
      og[k & 7] = (_Float16)v;
      pg[k & 7] = (_Float16)pv;
      if ((k & 7) == 7) {  // W is a multiple of 32 and every row 16-byte aligned
        *(h8*)(oh + k - 7) = og;
        if (P->has_neg) *(h8*)(par + k - 7) = pg;
      }
    }
    if (hm == 1 && P->has_neg)
      for (int k = W; k < h_kpp(P->kc); k += 8) *(h8*)(par + k) = z8;
  }
  if (blockIdx.x == 1) PSTAMP(15);
  C += P->lb_sum - P->m0_log2;
  const float Cf = ok ? (float)C : -1e30f;
  if (slot) {
    if (hm) {
      if (hm == 1) ch[jj] = Cf;
      // C_j as three f16 pieces in the lo.lo slots 4c+3 of dims c = 0, 1, 2 (A side = 1 there);
      // padding rows get -60000, so their terms underflow to 0 (c_i <= 0, the rest of the row is 0;
      // h32: the shifted c_i stays below H32_CMAX = 30000)
      const float cv = ok ? fmaxf(Cf, -H_CMAX) : -H_CMAX;
      const _Float16 c0 = (_Float16)cv;
      const float r1 = cv - (float)c0;
      const _Float16 c1 = (_Float16)r1;
      const _Float16 c2 = (_Float16)(r1 - (float)c1);
      if (hm == 2) {  // slots 0-2: the C_j pieces; 3-5: 1 against the candidate's c_i pieces
        hst[0] = c0;
        hst[1] = c1;
        hst[2] = c2;
        hst[3] = hst[4] = hst[5] = (_Float16)1.f;
        for (int q = 0; q < 2 * nd32; ++q) *(h8*)(hrow + 8 * q) = *(const h8*)(hst + 8 * q);
        if (crow) {  // coarse dense slots: the same six, then Xh of continuous dim c at 6 + c; row padding
          const int ndc = h32c_nd(P->nsc), kpc = h32_kp(P->kc), ktpc = h32c_ktp(P->nsc, kpc);
          for (int q = 0; q < 2 * ndc; ++q) {
            h8 g;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const int k = 8 * q + e;
              g[e] = k < 6 ? hst[k] : (k - 6 < dcp ? hst[6 + 3 * (k - 6)] : (_Float16)0.f);
            }
            *(h8*)(crow + 8 * q) = g;
          }
          for (int k = (16 * ndc + 16 * kpc + 2 * h32_ixw(kpc) + 7) & ~7; k < ktpc; k += 8) *(h8*)(crow + k) = z8;
        }
      } else {
        hrow[3] = c0;
        hrow[7] = c1;
        hrow[11] = c2;
      }
    } else {
      ch[0 * KROW + jj] = Cf;
      ch[1 * KROW + jj] = 1.f;
      if (jj < KROW - OBS_CHUNK)  // zero the pad columns of every k-row once per chunk
        for (int k = 0; k < KP; ++k) ch[k * KROW + OBS_CHUNK + jj] = 0.f;
    }
  }
  if (blockIdx.x == 1) PSTAMP(16);
  const uint32_t a = wave_reduce_dpp(__float_as_uint(ok ? fabsf(Cf) : 0.f), OpMax());
  if ((threadIdx.x & 63) == 0) atomicMax((unsigned int*)cmax_acc, a);
  if (j == 0)
    for (int q = 0; q < P->nconst; ++q) Pw->const_level[q] = x[P->const_dim[q]];
}

// f32-MFMA layout of an hmode KDE whose C_j left the f16 range of the three-piece split
__device__ __forceinline__ bool table_needs_rebuild(const KdeParams* P) { return P->hmode && !(P->cmax <= H_CMAX); }
// variant bit 8: at most 8 categorical slots and every active categorical dim's codes in [0, 3] -- the
// direct-difference ln-pdf pass then matches codes through two-bit fields and 256-entry tables (DD_LUT)
__device__ __forceinline__ int small_codes(const KdeParams* P) {
  if (P->du_pad != 4 && P->du_pad != 8) return 0;
  for (int u = 0; u < P->du; ++u)
    if (P->cat_maxcode[u] < 0 || P->cat_maxcode[u] > 3) return 0;
  return 1;
}

// Final mode of each KDE and its info record {variant, nan_all, unsupported, dc, du, nconst, dc_pad,
// du_pad}; variant = has_neg | kc << 1 | (hmode != 0) << 4 | exact_only << 5 | (hmode == 2) << 6 |
// (coarse table) << 7 | small_codes << 8 selects the scoring kernel.  rebuild: the table needed its f32 rebuild.
__device__ __forceinline__ void prep_finish_p(KdeParams* P, int32_t* info, bool rebuild) {
  if (rebuild) {
    P->hmode = 0;
    P->chunk_floats = chunk_floats(P->dc_pad, P->du_pad, P->kc, P->kc ? P->has_neg : 0);
    P->cmax = P->cmax2;
    P->coarse_off = 0;
  }
  info[0] = P->has_neg | (P->kc << 1) | ((P->hmode != 0) << 4) | (P->exact_only << 5) | ((P->hmode == 2) << 6) |
            ((P->hmode == 2 && P->coarse_off > 0) << 7) | (small_codes(P) << 8);
  info[1] = P->nan_all;
  info[2] = P->unsupported;
  info[3] = P->dc;
  info[4] = P->du;
  info[5] = P->nconst;
  info[6] = P->dc_pad;
  info[7] = P->du_pad;
}
__device__ __forceinline__ void prep_finish_one(const PrepArgs& A, bool rebuild) { prep_finish_p(A.P, A.info, rebuild); }
// The same from R, the table launch's LDS copy of the block (every field read here is final before that
// launch), the rebuild's changes written to W, the record kept in vals: no global reads on the finishing
// block's path (cmax2: the rebuild's maximum, read by the caller)
__device__ __forceinline__ void prep_finish_lds(const KdeParams* R, KdeParams* W, int32_t* info, bool rebuild,
                                                float cmax2, int32_t (&vals)[8]) {
  int hmode = R->hmode, coarse = R->coarse_off;
  if (rebuild) {
    hmode = 0;
    coarse = 0;
    W->hmode = 0;
    W->chunk_floats = chunk_floats(R->dc_pad, R->du_pad, R->kc, R->kc ? R->has_neg : 0);
    W->cmax2 = cmax2;
    W->cmax = cmax2;
    W->coarse_off = 0;
  }
  vals[0] = R->has_neg | (R->kc << 1) | ((hmode != 0) << 4) | (R->exact_only << 5) | ((hmode == 2) << 6) |
            ((hmode == 2 && coarse > 0) << 7) | (small_codes(R) << 8);
  vals[1] = R->nan_all;
  vals[2] = R->unsupported;
  vals[3] = R->dc;
  vals[4] = R->du;
  vals[5] = R->nconst;
  vals[6] = R->dc_pad;
  vals[7] = R->du_pad;
#pragma unroll
  for (int i = 0; i < 8; ++i) info[i] = vals[i];
}

// pass 0: the layout the parameter kernel chose; pass 1: the f32 rebuild where it is needed (every
// block of a KDE that needs none exits at once)
// The block's 64 observation rows are staged in LDS first (all loads in flight at once, coalesced
// within each row) when D <= 64; the per-dim walk then reads LDS instead of waiting on one dependent
// global load per dim.
// finish (pass 0 only): the KDE's last block to finish -- told by the counter its add returns, after every
// wave's stores and maxima atomics have been acknowledged -- rebuilds the table in the f32 layout when its
// C_j left the f16 range (rare: every row, in this block) and writes the final mode and the info record:
// the rebuild and finish launches saved.
#define TABLE_STAGE_D 64
// LDS row stride (halves) of the table launch's h32 rows: a 16-byte multiple >= H32_ROW_MAX whose dword count
// is not a multiple of 8 (112 halves = 56 dwords put lanes i and i + 8 on one bank: 8-way conflicts on the
// per-dim half stores; 120 = 60 dwords: 4-way)
#ifndef H32_ROW_STRIDE
#define H32_ROW_STRIDE 120
#endif
__global__ __launch_bounds__(64) void kde_table_kernel(PrepSet ps, float* table0, float* table1, int pass, int finish) {
  const bool second = ps.nk > 1 && (int)blockIdx.x >= ps.k[0].nblk_table;
  const PrepArgs& A = ps.k[second ? 1 : 0];
  KdeParams* P = A.P;
  const int j0 = (int)(blockIdx.x - (second ? ps.k[0].nblk_table : 0)) * 64;
  if (pass != 0 && !table_needs_rebuild(P)) return;
  if (blockIdx.x == 1) PSTAMP(8);
  // the parameter block is copied to LDS: loads from the global block the kernel also writes (atomics)
  // would be vector loads, one memory latency each along the per-dim walk
  // (every load issued before the first store: one memory latency for the whole block, not one per 1 KiB)
  constexpr int NPL = (int)((sizeof(KdeParams) + 15) / 16);
  __shared__ uint4 pl[NPL];
  for (int i0 = 0; i0 < NPL; i0 += 8 * 64) {
    uint4 t[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = min(i0 + (int)threadIdx.x + 64 * q, NPL - 1);  // past the end: the last entry again
      t[q] = ((const uint4*)P)[i];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) pl[min(i0 + (int)threadIdx.x + 64 * q, NPL - 1)] = t[q];
  }
  __shared__ double xs[64 * (TABLE_STAGE_D + 1)];
  __shared__ __align__(16) _Float16 h32s[64 * H32_ROW_STRIDE];  // h32 rows assembled here
  const int D = A.D, n = A.n;
  const KdeParams* Pl = (const KdeParams*)pl;
  float* tab = second ? table1 : table0;
  // one block's 64 rows [r0, r0 + 64) of pass ps_: two inlined copies of the body, rows read from LDS
  // (every load a ds_read) or from global memory (a generic pointer would make each row read wait for the
  // outstanding table stores as well)
  auto rows64 = [&](int r0, int ps_) {
    const int j = r0 + threadIdx.x;
    auto run = [&](const double* x) {
      if (ps_ == 0)
        kde_table_body(x, Pl, P, tab, j, Pl->hmode, Pl->chunk_floats, &P->cmax, h32s + threadIdx.x * H32_ROW_STRIDE);
      else
        kde_table_body(x, Pl, P, tab, j, 0, chunk_floats(Pl->dc_pad, Pl->du_pad, Pl->kc, Pl->kc ? Pl->has_neg : 0),
                       &P->cmax2, h32s + threadIdx.x * H32_ROW_STRIDE);
    };
    if (D <= TABLE_STAGE_D) {
      const int DS = D | 1;  // odd row stride: the 64 threads' reads of one dim hit distinct banks
      __shared__ int64_t rs[64];
      __syncthreads();  // the parameter copy; the previous rows' readers done
      rs[threadIdx.x] = A.rows[j < n ? j : 0];
      __syncthreads();
      // 16 independent loads in flight per thread per batch (coalesced within each row); past the end
      // the last element is re-read and re-stored (same value, same place)
      const int tot = 64 * D;
      for (int e0 = 0; e0 < tot; e0 += 16 * 64) {
        double t[16];
        int at[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int e = min(e0 + q * 64 + (int)threadIdx.x, tot - 1);
          const int i = e / D, c = e - i * D;
          at[q] = i * DS + c;
          t[q] = A.X[rs[i] * (int64_t)D + c];
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) xs[at[q]] = t[q];
      }
      __syncthreads();
      if (blockIdx.x == 1 && ps_ == 0) PSTAMP(9);
      run(xs + threadIdx.x * DS);
      if (blockIdx.x == 1 && ps_ == 0) PSTAMP(10);
    } else {
      __syncthreads();  // the parameter copy
      run(A.X + A.rows[j < n ? j : 0] * (int64_t)D);
    }
  };
  rows64(j0, pass);
  if (pass != 0 || !finish) return;
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's table stores and maxima atomics are done
  __syncthreads();
  if (blockIdx.x == 1) PSTAMP(11);
  __shared__ int last;
  if (threadIdx.x == 0) last = atomicAdd(prep_counter(P), 1) == A.nblk_table - 1;
  __syncthreads();
  if (!last) return;
  PSTAMP(12);
  // every block's |C_j| maximum is in (atomics at the device level; read past this CU's cache)
  const float cmax = __hip_atomic_load(&P->cmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool rebuild = Pl->hmode && !(cmax <= H_CMAX);
  if (rebuild) {
    for (int r0 = 0; r0 < A.nblk_table * 64; r0 += 64) rows64(r0, 1);
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float cm2 = rebuild ? __hip_atomic_load(&P->cmax2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
    int32_t vals[8];
    prep_finish_lds(Pl, P, A.info, rebuild, cm2, vals);
    // the refit's output block to the host (hbx_kde_refit_sync): the rest went out with the parameter launch
    if (ps.pub.dst) prep_publish_vals(ps.pub, vals, second ? 1 : 0);
  }
  PSTAMP(13);
}

// Final mode of each KDE and its info record (the separate launch of hbx_kde_prepare's path)
__global__ void kde_prep_finish_kernel(PrepSet ps) {
  const int k = threadIdx.x;
  if (k >= ps.nk) return;
  const PrepArgs& A = k ? ps.k[1] : ps.k[0];
  prep_finish_one(A, table_needs_rebuild(A.P));
  if (ps.pub.dst) prep_publish_info(ps.pub, A, k);
}

static int64_t prep_table_blocks(int64_t n) { return (((n + OBS_CHUNK - 1) / OBS_CHUNK) * OBS_CHUNK + 63) / 64; }

// host: fill a PrepArgs (vartype from host memory), checking the table capacity
static int prep_args(PrepArgs* A, const double* X, int32_t D, const int64_t* rows, int32_t n, const int32_t* vartype,
                     const double* bw, const int32_t* nlev, void* params, int32_t* info, int64_t table_floats_) {
  if (D < 1 || D > HBX_MAX_D) return hbx_fail(HBX_ERR_UNSUPPORTED, "D=%d outside [1, %d]", D, HBX_MAX_D);
  if (n < 1) return hbx_fail(HBX_ERR_ARG, "KDE with n=%d observations", n);
  memset(A, 0, sizeof(*A));
  int dc = 0, du = 0;
  for (int d = 0; d < D; ++d) {
    if (vartype[d] != 0) {
      A->vt[d >> 5] |= 1u << (d & 31);
      ++du;
    } else {
      ++dc;
    }
  }
  int dcp, dup;
  bucket_dims(dc, du, &dcp, &dup);  // outside every bucket: an exact-only KDE (no table)
  if (table_floats_ < table_floats(n, dcp, dup))
    return hbx_fail(HBX_ERR_ARG, "table too small: %lld < %lld floats", (long long)table_floats_,
                    (long long)table_floats(n, dcp, dup));
  const char* hm_env = getenv("HBX_HMODE");  // 0: the f32-MFMA kernels everywhere (tests)
  A->X = X;
  A->rows = rows;
  A->bw = bw;
  A->nlev = nlev;
  A->P = (KdeParams*)params;
  A->info = info;
  A->n = n;
  A->D = D;
  A->hm_allowed = !(hm_env && hm_env[0] == '0');
  const char* h32_env = getenv("HBX_H32");  // 0: the 16x16-tile hmode kernel instead of the 32x32 one
  A->h32_allowed = !(h32_env && h32_env[0] == '0');
  const char* co_env = getenv("HBX_COARSE");  // 0: no coarse pre-screen table (the FAST instance scores)
  A->co_allowed = !(co_env && co_env[0] == '0');
  A->nblk_table = (dcp < 0 || dup < 0) ? 0 : (int32_t)prep_table_blocks(n);
  return HBX_OK;
}

// enqueue the preparation of ps.nk KDEs (no host synchronisation).  colstats_done: the fit wrote the column
// statistics already (refit_fit_colstats).  Every KDE with a table: the table launch's last block per KDE
// does the rare f32 rebuild and writes the final mode (3 launches; 5 before round 5)
static int prep_launch(PrepSet& ps, float* table0, float* table1, hipStream_t s, bool colstats_done = false) {
  if (!colstats_done) {
    hipLaunchKernelGGL(kde_colstats_kernel, dim3(ps.nk * ps.k[0].D), dim3(256), 0, s, ps);
    HBX_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(kde_params_kernel, dim3(ps.nk), dim3(256), 0, s, ps);
  HBX_LAUNCH_CHECK();
  const bool all_tables = ps.k[0].nblk_table > 0 && (ps.nk < 2 || ps.k[1].nblk_table > 0);
  const unsigned tb = (unsigned)(ps.k[0].nblk_table + (ps.nk > 1 ? ps.k[1].nblk_table : 0));
  if (tb > 0) {
    hipLaunchKernelGGL(kde_table_kernel, dim3(tb), dim3(64), 0, s, ps, table0, table1, 0, all_tables ? 1 : 0);
    HBX_LAUNCH_CHECK();
  }
  if (!all_tables) {  // an exact-only KDE (no table) in the set: the separate passes
    if (tb > 0) {
      hipLaunchKernelGGL(kde_table_kernel, dim3(tb), dim3(64), 0, s, ps, table0, table1, 1, 0);
      HBX_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(kde_prep_finish_kernel, dim3(1), dim3(64), 0, s, ps);
    HBX_LAUNCH_CHECK();
  }
  return HBX_OK;
}

// Rescue (rare): candidates whose every term sits far below the static bound M0 are recomputed
// with a true maximum (two passes over the observations), one candidate per thread on the VALU.
// Continuous coordinates come from the table's f32 part, categorical codes straight from the data.
// LOWREG (the combine kernel's copy): the same operations in the same order over k < dc only (the padded
// k >= dc terms add exact zeros), candidate and observation coordinates recomputed per pair instead of held
// in DCP-long register arrays -- the combine kernel keeps its occupancy (29-32 VGPRs, not up to 170)
template <int DCP, bool SIGNED, bool LOWREG = false>
__device__ __forceinline__ KdeEst kde_rescue_one(const double* __restrict__ cand, int64_t i, int32_t D,
                                                 const KdeParams* __restrict__ P) {
  constexpr int NC = DCP > 0 && !LOWREG ? DCP : 1;
  const double* x = cand + i * (int64_t)D;
  const int n = P->n, dc = P->dc, du = P->du;
  const double* __restrict__ Xo = P->X;
  const int64_t* __restrict__ rows = P->rows;
  float xs[NC], ci = 0.f, bnd = 0.f;
  auto coord = [&](const double* r, int k) { return (float)(P->cont_scale[k] * (r[P->cont_dim[k]] - P->center[k])); };
  if constexpr (LOWREG) {
#pragma unroll 1
    for (int k = 0; k < dc; ++k) {
      const float v = coord(x, k);
      ci = fmaf(-v, v, ci);
      bnd = fmaf(fabsf(2.f * v), P->xmax[k], bnd);
    }
  }
#pragma unroll
  for (int k = 0; k < (LOWREG ? 0 : DCP); ++k) {
    float v = 0.f;
    if (k < dc) v = (float)(P->cont_scale[k] * (x[P->cont_dim[k]] - P->center[k]));
    ci = fmaf(-v, v, ci);
    xs[k] = 2.f * v;
    if (k < dc) bnd = fmaf(fabsf(xs[k]), P->xmax[k], bnd);
  }
  auto pair_t = [&](int j, float& par) -> float {
    // observation row rebuilt exactly as kde_table_kernel writes it (f32 X', f64 C_j rounded once)
    const double* xo = Xo + rows[j] * (int64_t)D;
    float Xp[NC];
    double Cd = 0.0;
    if constexpr (LOWREG) {
#pragma unroll 1
      for (int k = 0; k < dc; ++k) {
        const float v = coord(xo, k);
        Cd -= (double)v * (double)v;
      }
    }
#pragma unroll
    for (int k = 0; k < (LOWREG ? 0 : DCP); ++k) {
      float v = 0.f;
      if (k < dc) v = (float)(P->cont_scale[k] * (xo[P->cont_dim[k]] - P->center[k]));
      Cd -= (double)v * (double)v;
      Xp[k] = v;
    }
    const float Cj = (float)(Cd + P->lb_sum - P->m0_log2);
    float t = fmaf(1.f, Cj, 0.f);
    t = fmaf(ci, 1.f, t);
    if constexpr (LOWREG) {
#pragma unroll 1
      for (int k = 0; k < dc; ++k) t = fmaf(2.f * coord(x, k), coord(xo, k), t);
    }
#pragma unroll
    for (int k = 0; k < (LOWREG ? 0 : DCP); ++k) t = fmaf(xs[k], Xp[k], t);
    par = 0.f;
    for (int u = 0; u < du; ++u) {
      const int d = P->cat_dim[u];
      const float m = (x[d] == xo[d]) ? 1.f : 0.f;
      t = fmaf(P->cat_delta[u], m, t);
      if (SIGNED) par = fmaf(m, P->cat_negf[u], -fabsf(par));
    }
    return t;
  };
  float mx = -INFINITY, par;
  for (int j = 0; j < n; ++j) mx = fmaxf(mx, pair_t(j, par));
  float S = 0.f, Sn = 0.f;
  if (mx > -INFINITY) {
    for (int j0 = 0; j0 < n; j0 += OBS_CHUNK) {
      float Sb = 0.f, Snb = 0.f;
      for (int j = j0; j < min(n, j0 + OBS_CHUNK); ++j) {
        const float e = __builtin_amdgcn_exp2f(pair_t(j, par) - mx);
        Sb += e;
        if (SIGNED) Snb = fmaf(fabsf(par), e, Snb);
      }
      S += Sb;
      Sn += Snb;
    }
  } else {
    mx = 0.f;
  }
  return finish_est(P, S, Sn, mx, false, ci, bnd, SIGNED, OBS_CHUNK);
}

template <int DCP, bool SIGNED>
__device__ __forceinline__ void kde_rescue_body(const double* __restrict__ cand, int64_t Nc, int32_t D,
                                                const KdeParams* __restrict__ P, const float* __restrict__ table,
                                                KdeEst* __restrict__ out, const unsigned blk,
                                                const int nsplit = 1) {
  const int64_t i = (int64_t)blk * 256 + threadIdx.x;
  bool need = false;  // a marker in any observation split's partial estimate
  if (i < Nc)
    for (int r = 0; r < nsplit; ++r) need = need || out[(int64_t)r * Nc + i].err == -1.f;
  if (!__any(need)) return;
  if (!need) return;
  out[i] = kde_rescue_one<DCP, SIGNED>(cand, i, D, P);  // the whole sum in split 0
  for (int r = 1; r < nsplit; ++r) out[(int64_t)r * Nc + i] = kde_est_neutral();
}

template <int DCP, bool SIGNED>
__global__ __launch_bounds__(256) void kde_rescue_kernel(const double* __restrict__ cand, int64_t Nc, int32_t D,
                                                         const KdeParams* __restrict__ P,
                                                         const float* __restrict__ table,
                                                         KdeEst* __restrict__ out) {
  kde_rescue_body<DCP, SIGNED>(cand, Nc, D, P, table, out, blockIdx.x);
}


// both KDEs' rescue passes in one launch (blocks [0, nblk0) KDE 0, the rest KDE 1)
// grid-stride over the 2 nblk0 logical blocks; with the scoring kernel's marker count available and 0
// (the common case) every workgroup exits after one load; its first
// workgroup also initialises a single acquisition's state (acq_init's work)
template <int DCP, bool SIGNED>
__global__ __launch_bounds__(256) void kde_rescue_pair_kernel(const double* __restrict__ cand, int64_t Nc, int32_t D,
                                                              KdePairArgs a) {
  if (a.init.U && blockIdx.x == 0 && threadIdx.x == 0)  // a single acquisition's state (acq_init's work)
    acq_init_state(a.init.U, a.init.count, a.init.flags, a.init.first1, a.init.res);
  if (a.rescue && __hip_atomic_load(a.rescue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  for (unsigned b = blockIdx.x; b < 2 * a.nblk0; b += gridDim.x) {
    const bool second = b >= a.nblk0;
    kde_rescue_body<DCP, SIGNED>(cand, Nc, D, second ? a.P1 : a.P0, second ? a.table1 : a.table0,
                                 second ? a.out1 : a.out0, second ? b - a.nblk0 : b, second ? a.nsplit1 : a.nsplit0);
  }
}

// ------------------------------------------------------------------------------------------
// score intervals, shortlist, exact re-score, final argmin

__global__ void acq_init_kernel(uint32_t* U, int32_t* count, int32_t* flags, int32_t* first1, AcqResult* res) {
  if (threadIdx.x == 0 && blockIdx.x == 0) acq_init_state(U, count, flags, first1, res);
}

// batched acquisition: per-segment bound, flags, shortlist count, best score and (index, position) key
__global__ void acq_init_batch_kernel(int64_t B, uint32_t* __restrict__ U, int32_t* __restrict__ flags,
                                      int32_t* __restrict__ segcnt, uint64_t* __restrict__ best,
                                      uint64_t* __restrict__ key, int32_t* __restrict__ first1,
                                      int32_t* __restrict__ count, int32_t* __restrict__ segnear) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b == 0) *count = 0;
  if (b < B) {
    U[b] = hbx_f2ord(INFINITY);
    flags[b] = 0;
    segcnt[b] = 0;
    segnear[b] = 0;
    first1[b] = INT32_MAX;
    best[b] = ~0ull;
    key[b] = ~0ull;
  }
}

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

// Candidates [b*seg, (b+1)*seg) form acquisition b (seg = Nc: one acquisition).  U[b] = min over the
// segment of the upper score bound, flags[b] bit 0 = overflow risk (re-score the whole segment).
// Candidates whose l and g are both certainly below 1e-8 score exactly 1e-8/1e-8 = 1 (bohb.py:129):
// they tie, so only the first of them per segment (first1[b]) can win and needs the exact re-score
// (BOHB's own sampler puts most candidates there at D = 32: the truncnorm scale is 3 bw).
#define OBS_SPLIT_MAX 16  // observation splits of one scoring launch at most (obs_splits)

// Candidate i's estimate merged over its nsplit observation-split partials (hbx_score_h32.hip): the sums
// add (log domain, fp32); each partial's relative bound holds for the total too (sums of positive terms),
// plus per merge its own rounding: 2^-18 for the fp32 exp / log / addition, and the rounding of the merged
// ln S to fp32 (<= |ln S| 2^-23 absolute, counted as 2^-22 |ln S| relative on S)
__device__ __forceinline__ KdeEst merge_splits(const KdeEst* __restrict__ e, int64_t Nc, int64_t i, int nsplit) {
  // every partial's load issued before the first merge (a load per dependent merge step cost 14 us for 16
  // splits of 64 candidates); fixed-size and fully unrolled, so the partials stay in registers
  KdeEst p[OBS_SPLIT_MAX];
#pragma unroll
  for (int r = 0; r < OBS_SPLIT_MAX; ++r) p[r] = r < nsplit ? e[(int64_t)r * Nc + i] : kde_est_neutral();
  auto lae = [](float x, float y) {
    const float m = fmaxf(x, y);
    return m == -INFINITY ? m : m + __logf(__expf(x - m) + __expf(y - m));
  };
  KdeEst a = p[0];
#pragma unroll
  for (int r = 1; r < OBS_SPLIT_MAX; ++r) {
    if (r < nsplit) {
      const KdeEst b = p[r];
      if (a.lpos != a.lpos || b.lpos != b.lpos) {  // structural NaN (every split carries it)
        a.lpos = NAN;
      } else {
        a.lpos = lae(a.lpos, b.lpos);
        a.lneg = lae(a.lneg, b.lneg);
        const float ml = fmaxf(a.lpos > -INFINITY ? fabsf(a.lpos) : 0.f, a.lneg > -INFINITY ? fabsf(a.lneg) : 0.f);
        a.err = fmaxf(a.err, b.err) + 0x1p-18f + ml * 0x1p-22f;
      }
    }
  }
  return a;
}

// observation splits: each candidate's partial estimates merged into its first slot, for the combine and
// every later step (one thread per candidate and KDE; launched only when the scoring launch split)
__global__ __launch_bounds__(256) void kde_merge_splits_kernel(KdeEst* __restrict__ el, KdeEst* __restrict__ eg,
                                                               int64_t Nc, int32_t ns_l, int32_t ns_g) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= 2 * Nc) return;
  const bool g = t >= Nc;
  const int64_t i = g ? t - Nc : t;
  const int ns = g ? ns_g : ns_l;
  if (ns > 1) (g ? eg : el)[i] = merge_splits(g ? eg : el, Nc, i, ns);
}

#ifndef COMBINE_SUB
#define COMBINE_SUB 2  // 256-candidate sub-blocks per block of kde_combine_kernel (2: 13-15 us at 1e6, 4: 15-17, 8: 19)
#endif
// RESCUE: the rescue pass done here (a single acquisition scored by a 32x32 pair launch without splits):
// with the scoring launch's marker count non-zero, a thread re-scores its own marked candidates before
// combining them (kde_rescue_one, the rescue kernel's arithmetic) and stores them for the later steps --
// one launch less per acquisition (a rescue launch took 4.8 us even when it exited at once)
struct CombineRescue {
  const double* cand;
  int32_t D;
  const KdeParams* Pl;  // the KDEs behind el / eg
  const KdeParams* Pg;
  const int32_t* cnt;   // the scoring launch's marker count
};
template <bool SIGNED, bool RESCUE>
__global__ __launch_bounds__(256) void kde_combine_kernel(KdeEst* __restrict__ el, KdeEst* __restrict__ eg,
                                                          int64_t Nc, uint32_t seg, float* __restrict__ logl,
                                                          float* __restrict__ logg, float* __restrict__ lo,
                                                          uint32_t* __restrict__ U, int32_t* __restrict__ flags,
                                                          int32_t* __restrict__ first1, CombineRescue rs) {
  // COMBINE_SUB consecutive 256-candidate sub-blocks per block: every sub-block's loads are issued first
  // (the kernel is latency-bound with one candidate per thread), then each runs as its own block would
  // the marker count, final since the scoring launch ended: a plain (scalar) load, like the estimates'
  int32_t nres = 0;
  if constexpr (RESCUE) nres = *rs.cnt;
  KdeEst ea[COMBINE_SUB], eb[COMBINE_SUB];
#pragma unroll
  for (int r = 0; r < COMBINE_SUB; ++r) {
    const int64_t i = ((int64_t)blockIdx.x * COMBINE_SUB + r) * 256 + threadIdx.x;
    if (i < Nc) {
      ea[r] = el[i];
      eb[r] = eg[i];
    }
  }
  if constexpr (RESCUE) {
    if (nres != 0) {  // rare
#pragma unroll
      for (int r = 0; r < COMBINE_SUB; ++r) {
        const int64_t i = ((int64_t)blockIdx.x * COMBINE_SUB + r) * 256 + threadIdx.x;
        if (i < Nc && ea[r].err == -1.f) {
          ea[r] = kde_rescue_one<0, SIGNED, true>(rs.cand, i, rs.D, rs.Pl);
          el[i] = ea[r];
        }
        if (i < Nc && eb[r].err == -1.f) {
          eb[r] = kde_rescue_one<0, SIGNED, true>(rs.cand, i, rs.D, rs.Pg);
          eg[i] = eb[r];
        }
      }
    }
  }
  __shared__ float rh[COMBINE_SUB][4];
  __shared__ int32_t rf[COMBINE_SUB][4];
  // thread 0: the whole-block sub-blocks' minima of one segment, lowered into U / first1 once per segment
  // (an atomic round trip per sub-block made thread 0 -- and the next sub-block's barrier -- wait 4x)
  uint32_t acc_sg = ~0u;
  float acc_h = INFINITY;
  int32_t acc_f = INT32_MAX;
#pragma unroll
  for (int r = 0; r < COMBINE_SUB; ++r) {
    const int64_t blkr = (int64_t)blockIdx.x * COMBINE_SUB + r;
    if (blkr * 256 >= Nc) break;  // uniform
    const int64_t i = blkr * 256 + threadIdx.x;
    float h = INFINITY;
    bool one = false;
    const uint32_t sg = (uint32_t)(i < Nc ? i : Nc - 1) / seg;
    if (i < Nc) {
      const KdeEst a = ea[r], b = eb[r];
      const float C = (float)HBX_LN_CLAMP;
      float slo, shi;
      bool of = false;
      float llo, lhi, lpt, glo, ghi, gpt;
      if (a.lpos != a.lpos) {  // l NaN -> max(l, 1e-8) is NaN -> score NaN (never selected)
        slo = shi = NAN;
        lpt = NAN;
        est_interval(b, &glo, &ghi, &gpt);
        if (b.lpos != b.lpos) gpt = NAN;
      } else {
        est_interval(a, &llo, &lhi, &lpt);
        float Glo, Ghi;
        if (b.lpos != b.lpos) {  // g NaN -> max(1e-8, g) == 1e-8
          Glo = Ghi = C;
          gpt = NAN;
        } else {
          est_interval(b, &glo, &ghi, &gpt);
          Glo = fmaxf(glo, C);
          Ghi = fmaxf(ghi, C);
          of = ghi > 700.f;
        }
        of = of || lhi > 700.f;
        slo = Glo - fmaxf(lhi, C);
        shi = Ghi - fmaxf(llo, C);
        h = shi;
        const float C1 = C - 1e-4f;  // margin for the rounding of ln(1e-8) to float
        if (lhi < C1 && (b.lpos != b.lpos || ghi < C1)) {  // both clamped: score exactly 1 (ln 0)
          one = true;
          slo = NAN;  // excluded from the shortlist unless it is the segment's first exact tie
          shi = h = 0.f;
        }
      }
      if (logl) logl[i] = lpt;
      if (logg) logg[i] = gpt;
      lo[i] = slo;  // (the upper bound only enters the segment minimum below)
      if (of) atomicOr(flags + sg, 1);
    }
    // min of hi and first exact tie per segment.  Same-address atomics serialise in L2 (~10 ns each),
    // so: block reduction when the block lies in one segment (the common case), one wave-level atomic
    // when the wave does, per lane otherwise; and an atomic only when it can still lower the value.
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t blk0 = blkr * 256;
    const int64_t blk1 = (blk0 + 255 < Nc ? blk0 + 255 : Nc - 1);
    auto lower_u = [&](uint32_t sgi, float hv) {
      const uint32_t o = hbx_f2ord(hv);
      if (hv < INFINITY && o < __hip_atomic_load(U + sgi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(U + sgi, o);
    };
    auto lower_first = [&](uint32_t sgi, int32_t iv) {
      if (iv < __hip_atomic_load(first1 + sgi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(first1 + sgi, iv);
    };
    const uint32_t s0 = __shfl(sg, 0), s63 = __shfl(sg, 63);
    if (s0 == s63) {
      for (int o = 32; o > 0; o >>= 1) h = fminf(h, __shfl_xor(h, o));
      const uint64_t ones = __ballot(one);
      const int32_t f1 = ones ? (int32_t)(blk0 + 64 * wv + __ffsll((long long)ones) - 1) : INT32_MAX;
      if ((uint32_t)(blk0 / seg) == (uint32_t)(blk1 / seg)) {
        if (lane == 0) {
          rh[r][wv] = h;
          rf[r][wv] = f1;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
          const float hb = fminf(fminf(rh[r][0], rh[r][1]), fminf(rh[r][2], rh[r][3]));
          const int32_t fb = min(min(rf[r][0], rf[r][1]), min(rf[r][2], rf[r][3]));
          if (sg != acc_sg) {
            if (acc_sg != ~0u) {
              lower_u(acc_sg, acc_h);
              if (acc_f != INT32_MAX) lower_first(acc_sg, acc_f);
            }
            acc_sg = sg;
            acc_h = hb;
            acc_f = fb;
          } else {
            acc_h = fminf(acc_h, hb);
            acc_f = min(acc_f, fb);
          }
        }
      } else if (lane == 0) {
        lower_u(sg, h);
        if (f1 != INT32_MAX) lower_first(sg, f1);
      }
    } else {
      lower_u(sg, h);
      if (one) lower_first(sg, (int32_t)i);
    }
  }  // sub-block
  if (threadIdx.x == 0 && acc_sg != ~0u) {
    const uint32_t o = hbx_f2ord(acc_h);
    if (acc_h < INFINITY && o < __hip_atomic_load(U + acc_sg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMin(U + acc_sg, o);
    if (acc_f != INT32_MAX &&
        acc_f < __hip_atomic_load(first1 + acc_sg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMin(first1 + acc_sg, acc_f);
  }
}

typedef void (*combine_fn)(KdeEst*, KdeEst*, int64_t, uint32_t, float*, float*, float*, uint32_t*, int32_t*,
                           int32_t*, CombineRescue);

__global__ __launch_bounds__(256) void kde_shortlist_kernel(const float* __restrict__ lo, int64_t Nc, uint32_t seg,
                                                            const uint32_t* __restrict__ U,
                                                            const int32_t* __restrict__ flags,
                                                            int32_t* __restrict__ list,
                                                            int32_t* __restrict__ count,
                                                            int32_t* __restrict__ segcnt,
                                                            const int32_t* __restrict__ first1,
                                                            int32_t* __restrict__ rescue_cnt) {
  // the rescue of this acquisition is done (its pass or the combine): the marker count starts the next at 0
  if (rescue_cnt && blockIdx.x == 0 && threadIdx.x == 0) *rescue_cnt = 0;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= Nc) return;
  const uint32_t sg = (uint32_t)i / seg;
  const float u = hbx_ord2f(U[sg]);
  const bool all = (flags[sg] & 1) != 0;
  const float l = lo[i];
  if ((l == l && (all || l <= u)) || (int32_t)i == first1[sg]) {
    const int pos = atomicAdd(count, 1);
    list[pos] = (int32_t)i;
    if (segcnt) atomicAdd(segcnt + sg, 1);
  }
}

#include "hbx_npexp.h"
#include "hbx_pairwise.h"

struct ExactShared {
  double dens[PW_UNIT_MAX];
  double nsum[PW_LEVELS][128];
  double usum[PW_UNITS];
  // per-dim constants of the reference kernels (SM:kernels.py:62-64,125): continuous -> (h*h)*2 in
  // c0, categorical -> 1-h in c0 and h/(c-1) in c1; the point's coordinates in xd
  double c0[HBX_MAX_D], c1[HBX_MAX_D], xd[HBX_MAX_D];
  int32_t cont[HBX_MAX_D];
};

// Per-dim constants + the point's coordinates into LDS (whole block).
__device__ void exact_setup(const KdeParams* __restrict__ P, int32_t D, const double* __restrict__ x,
                            ExactShared* sh) {
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    const double h = P->bw[d];
    const bool c = P->vartype[d] == 0;
    sh->cont[d] = c;
    sh->c0[d] = c ? (h * h) * 2. : 1. - h;
    sh->c1[d] = c ? 0. : h / (double)(P->nlev[d] - 1);
    sh->xd[d] = x[d];
  }
  __syncthreads();
}

// Sum of the per-observation terms Kval.prod(1) / prod(bw_c) (SM:_kernel_base.py:509-516) over
// the observations [first, first+len) -- one unit of one buffer, pairwise order; whole block.
template <int LEVELS = PW_LEVELS>
__device__ double exact_unit(const double* __restrict__ X, int32_t D, const int64_t* __restrict__ rows,
                             const KdeParams* __restrict__ P, int first, int len, ExactShared* sh) {
  const double pbc = P->prod_bw_c;
  for (int j = threadIdx.x; j < len; j += blockDim.x) {
    const double* xr = X + rows[first + j] * (int64_t)D;
    double p = 1.0;
#pragma unroll 8
    for (int d = 0; d < D; ++d) {
      const double v = xr[d], xv = sh->xd[d];
      double k;
      if (sh->cont[d]) {
        const double diff = v - xv;
        k = HBX_INV_SQRT_2PI * hbx_npexp::exp(-(diff * diff) / sh->c0[d]);  // numpy's exp, bit for bit
      } else {
        k = (v == xv) ? sh->c0[d] : sh->c1[d];
      }
      p = (d == 0) ? k : p * k;
    }
    sh->dens[j] = p / pbc;
  }
  __syncthreads();
  return np_pairwise_block<LEVELS>(sh->dens, len, sh->nsum);
}

// exact fp64 pdf of one KDE at the point staged by exact_setup, one block, all units in turn
__device__ double exact_pdf(const double* __restrict__ X, int32_t D, const int64_t* __restrict__ rows,
                            const KdeParams* __restrict__ P, ExactShared* sh) {
  const int n = P->n;
  double acc = 0.0;  // np.add.reduce: identity 0.0, then one pairwise sum per 8192-element buffer
  for (int c = 0; c < n; c += PW_BUF) {
    const int m = (n - c) < PW_BUF ? (n - c) : PW_BUF;
    for (int u = 0; u < PW_UNITS; ++u) {
      int off, len;
      if (!pw_unit(m, u, &off, &len)) continue;
      const double v = exact_unit(X, D, rows, P, c + off, len, sh);
      if (threadIdx.x == 0) sh->usum[u] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) acc = acc + pw_combine_units(m, sh->usum);
  }
  return acc / (double)n;  // valid in thread 0
}

// Exact re-score of the shortlist.  Small shortlists (<= EXACT_SPLIT_CAP): one work item per
// (candidate, KDE, 8192-buffer, unit) so one candidate spreads over many CUs; the unit sums go to
// `part` and kde_final combines them.  Larger: one item per (candidate, KDE), all units in turn.
// threads per block of the acquisition's exact re-score: one unit (<= 263 observations) per block, one
// observation per thread (one wave per SIMD; the 32 units of a buffer run on 32 CUs)
#ifndef EXACT_ACQ_THREADS
#define EXACT_ACQ_THREADS 256
#endif
// SCAN (a single acquisition of <= EXACT_SCAN_MAX candidates): no shortlist launch before this one -- every
// block restates kde_shortlist_kernel's predicate over the whole candidate set itself, in index order (a
// ballot prefix per wave), into its own LDS list; block 0 stores the list, its length and the zeroed marker
// count for the later kernels.  The final pick does not depend on the list's order (the atomics of the
// shortlist kernel give none).
#define EXACT_SCAN_MAX 1024
struct ExactScan {
  const float* lo;
  int64_t Nc;
  const uint32_t* U;
  const int32_t* flags;
  const int32_t* first1;
  int32_t* list;
  int32_t* count;
  int32_t* rescue_cnt;
};
template <bool SCAN>
__global__ __launch_bounds__(EXACT_ACQ_THREADS) void kde_exact_kernel(
    const double* __restrict__ cand, int32_t D,
    const KdeParams* __restrict__ Pg, const double* __restrict__ Xg, const int64_t* __restrict__ rows_g,
    const KdeParams* __restrict__ Pb, const double* __restrict__ Xb, const int64_t* __restrict__ rows_b,
    const int32_t* __restrict__ list_in, const int32_t* __restrict__ count, int32_t nbuf, double* __restrict__ part,
    double* __restrict__ exact_l, double* __restrict__ exact_g, ExactScan sc) {
  __shared__ ExactShared sh;
  __shared__ int32_t slist[SCAN ? EXACT_SCAN_MAX : 1];
  __shared__ int32_t swc[EXACT_ACQ_THREADS / 64];
  int cnt;
  const int32_t* list = list_in;
  if constexpr (SCAN) {
    const float u = hbx_ord2f(sc.U[0]);
    const bool all = (sc.flags[0] & 1) != 0;
    const int32_t f1 = sc.first1[0];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int base = 0;
    for (int64_t c0 = 0; c0 < sc.Nc; c0 += EXACT_ACQ_THREADS) {
      const int64_t i = c0 + threadIdx.x;
      bool in = false;
      if (i < sc.Nc) {
        const float l = sc.lo[i];
        in = (l == l && (all || l <= u)) || (int32_t)i == f1;
      }
      const uint64_t b = __ballot(in);
      if (lane == 0) swc[wv] = __popcll(b);
      __syncthreads();
      int off = base, tot = 0;
#pragma unroll
      for (int w = 0; w < EXACT_ACQ_THREADS / 64; ++w) {
        off += w < wv ? swc[w] : 0;
        tot += swc[w];
      }
      if (in) slist[off + __popcll(b & ((1ull << lane) - 1))] = (int32_t)i;
      base += tot;
      __syncthreads();
    }
    cnt = base;
    list = slist;
    if (blockIdx.x == 0) {
      for (int k = threadIdx.x; k < cnt; k += EXACT_ACQ_THREADS) sc.list[k] = slist[k];
      if (threadIdx.x == 0) {
        *sc.count = cnt;
        if (sc.rescue_cnt) *sc.rescue_cnt = 0;
      }
    }
  } else {
    cnt = *count;
  }
  const bool split = cnt <= EXACT_SPLIT_CAP;
  const int per = split ? nbuf * PW_SPLIT_UNITS : 1;  // items per (candidate, KDE)
  const int64_t items = (int64_t)cnt * 2 * per;
  for (int64_t item = blockIdx.x; item < items; item += gridDim.x) {
    const int64_t pk = item / per;  // (candidate, KDE)
    const int p = (int)(pk >> 1);
    const bool isl = pk & 1;
    const KdeParams* P = isl ? Pg : Pb;
    const double* X = isl ? Xg : Xb;
    const int64_t* rows = isl ? rows_g : rows_b;
    if (split) {
      const int r = (int)(item % per), b = r / PW_SPLIT_UNITS, u = r % PW_SPLIT_UNITS;
      const int n = P->n, c = b * PW_BUF;
      if (c >= n) continue;
      const int m = (n - c) < PW_BUF ? (n - c) : PW_BUF;
      int off, len;
      if (!pw_unit<PW_SPLIT_CUT>(m, u, &off, &len)) continue;
      exact_setup(P, D, cand + (int64_t)list[p] * D, &sh);
      const double v = exact_unit<PW_SPLIT_LEVELS>(X, D, rows, P, c + off, len, &sh);
      if (threadIdx.x == 0) part[pk * per + r] = v;
    } else {
      exact_setup(P, D, cand + (int64_t)list[p] * D, &sh);
      const double v = exact_pdf(X, D, rows, P, &sh);
      if (threadIdx.x == 0) (isl ? exact_l : exact_g)[p] = v;
    }
    __syncthreads();
  }
}

// split mode: pdf of every (shortlisted candidate, KDE) from its unit sums; one thread each
__global__ __launch_bounds__(256) void kde_exact_combine_kernel(const KdeParams* __restrict__ Pg,
                                                                const KdeParams* __restrict__ Pb,
                                                                const int32_t* __restrict__ count, int32_t nbuf,
                                                                const double* __restrict__ part,
                                                                double* __restrict__ exact_l,
                                                                double* __restrict__ exact_g) {
  const int cnt = *count;
  if (cnt > EXACT_SPLIT_CAP) return;
  // one wave per (candidate, KDE)
  const int64_t pk = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pk >= 2 * (int64_t)cnt) return;  // whole wave
  const bool isl = pk & 1;
  const int n = (isl ? Pg : Pb)->n;
  const double* us = part + pk * nbuf * PW_SPLIT_UNITS;
  double acc = 0.0;
  for (int c = 0, b = 0; c < n; c += PW_BUF, ++b) {
    const int m = (n - c) < PW_BUF ? (n - c) : PW_BUF;
    acc = acc + pw_combine_units_wave<PW_SPLIT_CUT>(m, us + b * PW_SPLIT_UNITS);
  }
  if ((threadIdx.x & 63) == 0) (isl ? exact_l : exact_g)[pk >> 1] = acc / (double)n;
}

// exact fp64 pdf of one KDE at every row of pts (grid-stride over points, one block per point)
// list (nullable): only the points list[0 .. *count), written at their own index; take_log: ln of the
// pdf, and only for KDEs the fp64 log-space kernel does not cover (negative factors, structural NaN)
__global__ __launch_bounds__(EXACT_THREADS) void kde_pdf_exact_kernel(const double* __restrict__ pts, int64_t Np,
                                                                      int32_t D, const KdeParams* __restrict__ P,
                                                                      const double* __restrict__ X,
                                                                      const int64_t* __restrict__ rows,
                                                                      double* __restrict__ out,
                                                                      const int32_t* __restrict__ list,
                                                                      const int32_t* __restrict__ count,
                                                                      int take_log) {
  __shared__ ExactShared sh;
  if (take_log && !(P->has_neg || P->nan_all || P->nconst)) return;
  const int64_t np = list ? (int64_t)*count : Np;
  for (int64_t p = blockIdx.x; p < np; p += gridDim.x) {
    const int64_t q = list ? (int64_t)list[p] : p;
    exact_setup(P, D, pts + q * D, &sh);
    const double v = exact_pdf(X, D, rows, P, &sh);
    if (threadIdx.x == 0) out[q] = take_log ? log(v) : v;
    __syncthreads();
  }
}

// ln pdf of one KDE at Np points in fp64 log space (one block per point): per observation j the
// log kernel product t_j = sum_c -(x_c - X_jc)^2 / (2 h_c^2) + sum_u ln K_u (SM:kernels.py:62-64,125
// with the constants pulled out), then ln pdf = logsumexp_j(t_j) - ln n - sum_c ln(h_c sqrt(2 pi)).
// No expansion and no fp64 underflow: accurate to ~1e-15 where the reference's own pdf is positive
// and still finite where the reference's fp64 pdf underflows to 0.  KDEs with negative categorical
// factors (bandwidth > 1 - 1/c) or structural NaNs are not handled here (NaN out): callers use the
// exact pdf there.  The mathematically exact counterpart of hbx_kde_logpdf's fp32 estimate.
__global__ __launch_bounds__(256) void kde_logpdf_exact_kernel(const double* __restrict__ pts, int64_t Np, int32_t D,
                                                              const KdeParams* __restrict__ P,
                                                              const double* __restrict__ X,
                                                              const int64_t* __restrict__ rows,
                                                              double* __restrict__ out,
                                                              const int32_t* __restrict__ list,
                                                              const int32_t* __restrict__ count) {
  __shared__ double c0[HBX_MAX_D], c1[HBX_MAX_D], xd[HBX_MAX_D];
  __shared__ int32_t cont[HBX_MAX_D];
  __shared__ double rm[4], rs[4];
  __shared__ double lconst;
  const int n = P->n;
  const int64_t np = list ? (int64_t)*count : Np;  // list: only those points, written at their own index
  for (int64_t pi = blockIdx.x; pi < np; pi += gridDim.x) {
    const int64_t p = list ? (int64_t)list[pi] : pi;
    const double* x = pts + p * D;
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
      const double h = P->bw[d];
      const bool c = P->vartype[d] == 0;
      cont[d] = c;
      c0[d] = c ? 1.0 / ((h * h) * 2.) : log(1. - h);          // continuous: 1/(2h^2); categorical: ln(1-h)
      c1[d] = c ? 0.0 : log(h / (double)(P->nlev[d] - 1));     // categorical mismatch: ln(h/(c-1))
      xd[d] = x[d];
    }
    if (threadIdx.x == 0) {
      double lc = -log((double)n);
      for (int d = 0; d < D; ++d)
        if (P->vartype[d] == 0) lc -= log(P->bw[d]) + 0.91893853320467274178;  // ln(h sqrt(2 pi))
      lconst = lc;
    }
    __syncthreads();
    double m = -INFINITY, sm = 0.0;  // this thread's running logsumexp
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
      const double* xr = X + rows[j] * (int64_t)D;
      double t = 0.0;
      for (int d = 0; d < D; ++d) {
        const double v = xr[d];
        if (cont[d]) {
          const double diff = v - xd[d];
          t -= diff * diff * c0[d];
        } else {
          t += (v == xd[d]) ? c0[d] : c1[d];
        }
      }
      if (t > m) {
        sm = sm * exp(m - t) + 1.0;
        m = t;
      } else if (t > -INFINITY) {
        sm += exp(t - m);
      } else if (t != t) {
        m = NAN;
      }
    }
    // block logsumexp of the (m, sm) pairs
    for (int o = 32; o > 0; o >>= 1) {
      const double m2 = __shfl_xor(m, o), s2 = __shfl_xor(sm, o);
      const double mm = fmax(m, m2);
      if (m != m || m2 != m2) {
        m = NAN;
      } else if (mm > -INFINITY) {
        sm = (m > -INFINITY ? sm * exp(m - mm) : 0.0) + (m2 > -INFINITY ? s2 * exp(m2 - mm) : 0.0);
        m = mm;
      }
    }
    if ((threadIdx.x & 63) == 0) {
      rm[threadIdx.x >> 6] = m;
      rs[threadIdx.x >> 6] = sm;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double M = -INFINITY, Sx = 0.0;
      bool nan = false;
      for (int w = 0; w < 4; ++w) {
        if (rm[w] != rm[w]) nan = true;
        else if (rm[w] > -INFINITY) {
          const double mm = fmax(M, rm[w]);
          Sx = (M > -INFINITY ? Sx * exp(M - mm) : 0.0) + rs[w] * exp(rm[w] - mm);
          M = mm;
        }
      }
      out[p] = (nan || P->has_neg || P->nan_all || P->nconst) ? NAN : (M > -INFINITY ? M + log(Sx) + lconst : -INFINITY);
    }
    __syncthreads();
  }
}

// Bound of |exact pdf here - pdf in numpy's arithmetic| / pdf for one KDE at one candidate.  Both run
// the same IEEE operations in the same order (SM:_kernel_base.py:509-516: per-dim kernels, dim-ordered
// product, / prod(bw_c), numpy's pairwise sum, / n) except exp, where ocml's and numpy's results may
// differ by ulps: per term <= (6 D + 4) u, plus 2 u per level of the summation tree (<= 40 levels up
// to 1e5 observations) -- (8 D + 160) 2^-52 leaves a margin over both.  Sums with negative terms
// (categorical bandwidth > 1) scale by their condition number sum|t| / |sum t|, taken pessimistically
// from the fp32 estimate (inf when its sign is not certain).
__device__ __forceinline__ double exact_rel(const KdeParams* __restrict__ P, const KdeEst e) {
  const double base = (8.0 * (double)P->D + 160.0) * 0x1p-52;
  if (!P->has_neg) return base;
  if (e.err < -1.5f) return INFINITY;  // exact-only acquisition: no fp32 estimate of the condition
  const float m = fmaxf(e.lpos, e.lneg);
  if (!(m > -INFINITY)) return base;
  const float a = __expf(e.lpos - m), b = __expf(e.lneg - m);
  const float den = fabsf(a - b) - (e.err + 1e-6f) * (a + b);
  if (!(den > 0.f)) return INFINITY;
  return base * (double)((a + b) / den) * 1.01;
}

// relative bound of one candidate's score (bohb.py:129: g clamped, / l clamped): both pdfs' bounds
// plus the division's rounding
__device__ __forceinline__ double score_rel(const KdeParams* __restrict__ Pg, const KdeParams* __restrict__ Pb,
                                            const KdeEst* __restrict__ el, const KdeEst* __restrict__ eg,
                                            int64_t i) {
  return exact_rel(Pg, el[i]) + exact_rel(Pb, eg[i]) + 0x1p-51;
}

// p may beat the winner in numpy's arithmetic only if s_p (1 - R_p) <= s_best (1 + R_best)
__device__ __forceinline__ bool near_best(double s, double rp, double best, double rb) {
  return s < INFINITY && s <= best * (1.0 + 1.0001 * (rp + rb));
}

// A get_config pick published to device-mapped host memory by the final argmin (hbx_kde_acquire_bound with err /
// row_out): the record, whether any of the call's candidates hit a sampler domain error, the winning row (as
// tagged 8-byte words: kde_final_body)
struct PickOut {
  const double* cand;
  const uint8_t* err;  // nullable
  int64_t Nc;
  int32_t D;
  char* out;  // null: no pick
};

// the final argmin of one acquisition (256 threads): the split re-score's unit sums -> pdfs, strict '<'
// first-index argmin over the shortlist, the near set, the result record
__device__ void kde_final_body(const int32_t* __restrict__ list, const int32_t* __restrict__ count,
                               const double* exact_l,  // (written here through exact_lw / _gw)
                               const double* exact_g, const int32_t* __restrict__ flags, int64_t index_base,
                               const KdeParams* __restrict__ Pg, const KdeParams* __restrict__ Pb,
                               const KdeEst* __restrict__ el, const KdeEst* __restrict__ eg,
                               int32_t* __restrict__ near_list, AcqResult* __restrict__ res, int32_t nbuf,
                               const double* part, double* exact_lw, double* exact_gw, AcqResult* host_res,
                               int32_t* done, int32_t seq, PickOut pick = PickOut{}) {
  __shared__ double bs[256];
  __shared__ AcqResult rec_sh;
  __shared__ int64_t bi[256];
  __shared__ int32_t bp[256];
  __shared__ double exl[256], exg[256];  // the exact pdfs of a shortlist of <= 256 (no global re-read)
  __shared__ double rb_sh;
  __shared__ int32_t nnear;
  const int cnt = *count;
  int err_any = 0;
  if (pick.out && pick.err) {  // uniform
    bool e = false;
    for (int64_t i = threadIdx.x; i < pick.Nc; i += 256) e = e || pick.err[i] != 0;
    err_any = __syncthreads_or(e);
  }
  // shortlists of <= 256 (the common case): thread p owns candidate p -- its index and bound are loaded
  // first, beside the unit sums' combination, and its pdfs come back through LDS
  const bool small = cnt <= 256;
  const int tp = threadIdx.x;
  const int64_t my_idx = (small && tp < cnt) ? list[tp] : 0;
  const double my_rel = (small && tp < cnt) ? score_rel(Pg, Pb, el, eg, my_idx) : 0.0;
  if (part && cnt <= EXACT_SPLIT_CAP) {  // the split re-score's unit sums -> pdfs (kde_exact_combine's work)
    for (int pk = threadIdx.x >> 6; pk < 2 * cnt; pk += 4) {  // one wave per (candidate, KDE)
      const bool isl = pk & 1;
      const int n = (isl ? Pg : Pb)->n;
      const double* us = part + (int64_t)pk * nbuf * PW_SPLIT_UNITS;
      double acc = 0.0;
      for (int c = 0, b = 0; c < n; c += PW_BUF, ++b) {
        const int m = (n - c) < PW_BUF ? (n - c) : PW_BUF;
        acc = acc + pw_combine_units_wave<PW_SPLIT_CUT>(m, us + b * PW_SPLIT_UNITS);
      }
      if ((threadIdx.x & 63) == 0) {
        const double pdf = acc / (double)n;
        (isl ? exact_lw : exact_gw)[pk >> 1] = pdf;
        if (small) (isl ? exl : exg)[pk >> 1] = pdf;
      }
    }
    __threadfence_block();
    __syncthreads();
  } else if (small) {  // pdfs written by another kernel: one global read each
    if (tp < cnt) {
      exl[tp] = exact_l[tp];
      exg[tp] = exact_g[tp];
    }
    __syncthreads();
  }
  double best = INFINITY;
  int64_t bidx = INT64_MAX;
  int32_t bpos = -1;
  if (threadIdx.x == 0) nnear = 0;
  for (int p = threadIdx.x; p < cnt; p += 256) {
    // bohb.py:129 with Python max(): max(1e-8, g) keeps 1e-8 unless g > 1e-8 (NaN -> 1e-8);
    // max(l, 1e-8) keeps l unless 1e-8 > l (NaN -> NaN)
    const double g = small ? exg[p] : exact_g[p], l = small ? exl[p] : exact_l[p];
    const double s = ((g > 1e-8) ? g : 1e-8) / ((1e-8 > l) ? 1e-8 : l);
    const int64_t idx = small ? my_idx : list[p];
    // valid iff s < +inf (bohb.py:150 'val < best' with best = inf); strict '<', first index wins
    if (s < INFINITY && (s < best || (s == best && idx < bidx))) {
      best = s;
      bidx = idx;
      bpos = p;
    }
  }
  bs[threadIdx.x] = best;
  bi[threadIdx.x] = bidx;
  bp[threadIdx.x] = bpos;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      const double s2 = bs[threadIdx.x + w];
      const int64_t i2 = bi[threadIdx.x + w];
      if (s2 < bs[threadIdx.x] || (s2 == bs[threadIdx.x] && i2 < bi[threadIdx.x])) {
        bs[threadIdx.x] = s2;
        bi[threadIdx.x] = i2;
        bp[threadIdx.x] = bp[threadIdx.x + w];
      }
    }
    __syncthreads();
  }
  // the near set: every re-scored candidate the winner cannot be told apart from by these bounds
  const int32_t wp = bp[0];
  double rb = 0.0;
  if (small) {  // the winner's thread holds its bound
    if (tp == wp) rb_sh = my_rel;
    __syncthreads();
    if (wp >= 0) rb = rb_sh;
  }
  if (wp >= 0) {
    const double sb = bs[0];
    if (!small) rb = score_rel(Pg, Pb, el, eg, list[wp]);
    for (int p = threadIdx.x; p < cnt; p += 256) {
      const double g = small ? exg[p] : exact_g[p], l = small ? exl[p] : exact_l[p];
      const double s = ((g > 1e-8) ? g : 1e-8) / ((1e-8 > l) ? 1e-8 : l);
      const int64_t ip = small ? my_idx : list[p];
      if (p == wp || near_best(s, small ? my_rel : score_rel(Pg, Pb, el, eg, ip), sb, rb))
        near_list[atomicAdd(&nnear, 1)] = (int32_t)ip;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    AcqResult r;  // acq_init_state's record when nothing is finite
    r.index = -1;
    r.score = r.pdf_l = r.pdf_g = NAN;
    r.shortlist = cnt;
    r.flags = *flags | (nnear > 1 ? HBX_ACQ_NEAR_TIE : 0);
    r.near = nnear;
    r.rel = (float)rb;
    if (wp >= 0) {
      r.index = bi[0] + index_base;
      r.score = bs[0];
      r.pdf_l = small ? exl[wp] : exact_l[wp];
      r.pdf_g = small ? exg[wp] : exact_g[wp];
    }
    *res = r;
    rec_sh = r;
  }
  if (host_res || pick.out) {  // uniform: the record (and a pick's flag and row) to mapped host memory
    static_assert(sizeof(AcqResult) % 4 == 0, "record of whole words");
    __syncthreads();
    // every 32-bit word as one 8-byte system-scope store tagged with the call's sequence number (seq << 32 |
    // word): the host takes each word only once its tag is the call's, so there is no acknowledgement wait
    // and no completion word (hbx_pub_wait)
    uint64_t* out = (uint64_t*)(pick.out ? pick.out : (char*)host_res);
    const uint64_t tag = (uint64_t)(uint32_t)seq << 32;
    constexpr int RW = (int)(sizeof(AcqResult) / 4);
    if (threadIdx.x < RW) hbx_publish_store64(out + threadIdx.x, tag | ((const uint32_t*)&rec_sh)[threadIdx.x]);
    if (pick.out) {  // a pick: + the domain-error flag (word RW) and the winning row (words RW + 1 ..)
      if (threadIdx.x == 0) hbx_publish_store64(out + RW, tag | (err_any ? 1u : 0u));
      const int64_t idx = rec_sh.index - index_base;
      if (rec_sh.index >= 0 && idx < pick.Nc)
        for (int w = threadIdx.x; w < 2 * pick.D; w += 256)
          hbx_publish_store64(out + RW + 1 + w, tag | ((const uint32_t*)(pick.cand + idx * pick.D))[w]);
    }
    (void)done;
  }
}

__global__ __launch_bounds__(256) void kde_final_kernel(const int32_t* __restrict__ list,
                                                        const int32_t* __restrict__ count, const double* exact_l,
                                                        const double* exact_g, const int32_t* __restrict__ flags,
                                                        int64_t index_base, const KdeParams* __restrict__ Pg,
                                                        const KdeParams* __restrict__ Pb,
                                                        const KdeEst* __restrict__ el, const KdeEst* __restrict__ eg,
                                                        int32_t* __restrict__ near_list, AcqResult* __restrict__ res,
                                                        int32_t nbuf, const double* __restrict__ part,
                                                        double* exact_lw, double* exact_gw, AcqResult* host_res,
                                                        int32_t* done, int32_t seq, PickOut pick) {
  kde_final_body(list, count, exact_l, exact_g, flags, index_base, Pg, Pb, el, eg, near_list, res, nbuf, part,
                 exact_lw, exact_gw, host_res, done, seq, pick);
}

// Batched argmin, three passes over the shortlist: (1) per-segment minimum of the exact score,
// (2) among the entries reaching it the smallest index (strict '<', first index -- bohb.py:149-152),
// (3) one thread per segment writes its record.  Scores are > 0 or NaN (both factors are clamped
// to >= 1e-8), so the bits of a finite score order like the score.
__device__ __forceinline__ double bohb_score(double g, double l) {
  return ((g > 1e-8) ? g : 1e-8) / ((1e-8 > l) ? 1e-8 : l);  // Python max() semantics, see kde_final
}

__global__ __launch_bounds__(256) void kde_batch_min_kernel(const int32_t* __restrict__ list,
                                                            const int32_t* __restrict__ count, uint32_t seg,
                                                            const double* __restrict__ exact_l,
                                                            const double* __restrict__ exact_g,
                                                            uint64_t* __restrict__ best) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= *count) return;
  const double s = bohb_score(exact_g[p], exact_l[p]);
  if (s < INFINITY) atomicMin((unsigned long long*)best + (uint32_t)list[p] / seg,
                              (unsigned long long)__double_as_longlong(s));
}

__global__ __launch_bounds__(256) void kde_batch_key_kernel(const int32_t* __restrict__ list,
                                                            const int32_t* __restrict__ count, uint32_t seg,
                                                            const double* __restrict__ exact_l,
                                                            const double* __restrict__ exact_g,
                                                            const uint64_t* __restrict__ best,
                                                            uint64_t* __restrict__ key) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= *count) return;
  const double s = bohb_score(exact_g[p], exact_l[p]);
  const uint32_t i = (uint32_t)list[p], sg = i / seg;
  if (s < INFINITY && (uint64_t)__double_as_longlong(s) == best[sg])
    atomicMin((unsigned long long*)key + sg, ((unsigned long long)(i - sg * seg) << 32) | (uint32_t)p);
}

// per shortlist entry: 1 in near_flag (and counted in segnear) when its segment's winner cannot be
// told apart from it by the error bounds (kde_final_kernel's near set, per segment)
__global__ __launch_bounds__(256) void kde_batch_near_kernel(const int32_t* __restrict__ list,
                                                             const int32_t* __restrict__ count, uint32_t seg,
                                                             const double* __restrict__ exact_l,
                                                             const double* __restrict__ exact_g,
                                                             const uint64_t* __restrict__ key,
                                                             const KdeParams* __restrict__ Pg,
                                                             const KdeParams* __restrict__ Pb,
                                                             const KdeEst* __restrict__ el,
                                                             const KdeEst* __restrict__ eg,
                                                             int32_t* __restrict__ near_flag,
                                                             int32_t* __restrict__ segnear) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= *count) return;
  const uint32_t i = (uint32_t)list[p], sg = i / seg;
  const uint64_t k = key[sg];
  int f = 0;
  if (k != ~0ull) {
    const int wp = (int)(uint32_t)k;
    const double sb = bohb_score(exact_g[wp], exact_l[wp]);
    const double rb = score_rel(Pg, Pb, el, eg, list[wp]);
    const double s = bohb_score(exact_g[p], exact_l[p]);
    f = (p == wp || near_best(s, score_rel(Pg, Pb, el, eg, i), sb, rb)) ? 1 : 0;
  }
  near_flag[p] = f;
  if (f) atomicAdd(segnear + sg, 1);
}

__global__ __launch_bounds__(256) void kde_batch_final_kernel(int64_t B, const uint64_t* __restrict__ key,
                                                              const int32_t* __restrict__ segcnt,
                                                              const int32_t* __restrict__ flags,
                                                              const int32_t* __restrict__ segnear,
                                                              const int32_t* __restrict__ list,
                                                              const double* __restrict__ exact_l,
                                                              const double* __restrict__ exact_g,
                                                              const KdeParams* __restrict__ Pg,
                                                              const KdeParams* __restrict__ Pb,
                                                              const KdeEst* __restrict__ el,
                                                              const KdeEst* __restrict__ eg,
                                                              int64_t index_base, AcqResult* __restrict__ res) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  AcqResult r;
  r.shortlist = segcnt[b];
  r.near = segnear[b];
  r.flags = flags[b] | (r.near > 1 ? HBX_ACQ_NEAR_TIE : 0);
  r.rel = 0.f;
  const uint64_t k = key[b];
  if (k == ~0ull) {
    r.index = -1;
    r.score = NAN;
    r.pdf_l = NAN;
    r.pdf_g = NAN;
  } else {
    const int p = (int)(uint32_t)k;
    r.index = (int64_t)(k >> 32) + index_base;
    r.pdf_l = exact_l[p];
    r.pdf_g = exact_g[p];
    r.score = bohb_score(r.pdf_g, r.pdf_l);
    r.rel = (float)score_rel(Pg, Pb, el, eg, list[p]);
  }
  res[b] = r;
}

// Exact-only acquisition (KDEs outside every fp32 scoring bucket): every candidate joins the fp64
// re-score -- no estimate (err = -2 marks it), each segment flagged so the shortlist takes it whole.
__global__ __launch_bounds__(256) void kde_exact_only_init_kernel(int64_t Nc, uint32_t seg, KdeEst* __restrict__ el,
                                                                  KdeEst* __restrict__ eg, float* __restrict__ lo,
                                                                  int32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= Nc) return;
  const KdeEst e = {0.f, -INFINITY, -2.f, 0.f};
  el[i] = e;
  eg[i] = e;
  lo[i] = 0.f;
  if ((uint32_t)i % seg == 0) flags[(uint32_t)i / seg] = HBX_ACQ_OVERFLOW;
}

// ln of the exact pdfs for the logl/logg outputs of an exact-only acquisition
__global__ __launch_bounds__(256) void kde_exact_logs_kernel(const int32_t* __restrict__ list,
                                                             const int32_t* __restrict__ count,
                                                             const double* __restrict__ exact_l,
                                                             const double* __restrict__ exact_g,
                                                             float* __restrict__ logl, float* __restrict__ logg) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= *count) return;
  const int i = list[p];
  if (logl) logl[i] = (float)log(exact_l[p]);
  if (logg) logg[i] = (float)log(exact_g[p]);
}

// ------------------------------------------------------------------------------------------
// launch-side dispatch over the (dc_pad, du_pad, signed) template buckets

struct ScoreFns {
  logpdf_fn main, rescue;
  int cands_per_block;
  int threads;
  logpdf_pair_fn pair;  // the same kernel over both KDEs in one grid (hmode 16x16 only), or nullptr
  logpdf_pair_fn rescue_pair;
  bool split_ok = false;  // the pair kernel takes observation splits and initialises a single acquisition's
                          // state (the 32x32-tile instances)
  combine_fn combine_rescue = nullptr;  // the combine kernel doing the rescue pass of this instance
  logpdf_pair_fn pair1 = nullptr;       // the coarse pair kernel with one column tile per wave (launch_score2)
};

// Observation splits of a pair launch with `tiles` candidate tiles per KDE over <= nmax observations: a
// few candidates against many observations would otherwise be a handful of blocks each walking every
// chunk (64 candidates x 1e4 observations: 2 blocks, 123 us); while both KDEs' tiles are at most one block
// per CU, split until they fill the chip about twice, each range >= 4 chunks, at most 16 (the combine
// kernel merges the partial sums).
// HBX_OBS_SPLIT=0: no splits (read per call).  ws_sizing: the workspace's bound (no switch, the largest
// tile size).
static bool obs_split_enabled() {
  const char* e = getenv("HBX_OBS_SPLIT");
  return !(e && atoi(e) == 0);
}
static int obs_splits(unsigned tiles, int64_t nmax, bool ws_sizing = false) {
  if (!ws_sizing && !obs_split_enabled()) return 1;
  const int64_t nch = (nmax + OBS_CHUNK - 1) / OBS_CHUNK;
  if (2 * (int64_t)tiles > 256) return 1;  // one block per CU or more already (config #2: 392 blocks; both
                                           // KDEs split in two measured 4 us slower: a second round)
  int64_t sp = (512 + 2 * (int64_t)tiles - 1) / (2 * (int64_t)(tiles > 0 ? tiles : 1));
  if (sp > nch / 4) sp = nch / 4;
  if (sp > OBS_SPLIT_MAX) sp = OBS_SPLIT_MAX;
  return sp < 1 ? 1 : (int)sp;
}

// l and g scored by one launch of the pair kernel when both KDEs run the same hmode instance;
// HBX_SCORE_PAIR=0 keeps two launches (read per call: tests switch it in-process)
static bool pair_enabled() {
  const char* e = getenv("HBX_SCORE_PAIR");
  return !(e && atoi(e) == 0);
}

// the coarse pair launch with one column tile per wave where it fits one round (launch_score2); HBX_PAIR1=0:
// always the H32C_CT-tile kernel (read per call: tests switch it in-process)
static bool pair1_enabled() {
  const char* e = getenv("HBX_PAIR1");
  return !(e && atoi(e) == 0);
}

template <bool SG>
static logpdf_pair_fn pick_rescue_pair(int dc_pad) {
  switch (dc_pad) {
    case 0: return kde_rescue_pair_kernel<0, SG>;
    case 4: return kde_rescue_pair_kernel<4, SG>;
    case 8: return kde_rescue_pair_kernel<8, SG>;
    case 16: return kde_rescue_pair_kernel<16, SG>;
    case 24: return kde_rescue_pair_kernel<24, SG>;
    case 32: return kde_rescue_pair_kernel<32, SG>;
    case 64: return kde_rescue_pair_kernel<64, SG>;
  }
  return nullptr;
}

template <bool SG>
static logpdf_fn pick_rescue(int dc_pad) {
  switch (dc_pad) {
    case 0: return kde_rescue_kernel<0, SG>;
    case 4: return kde_rescue_kernel<4, SG>;
    case 8: return kde_rescue_kernel<8, SG>;
    case 16: return kde_rescue_kernel<16, SG>;
    case 24: return kde_rescue_kernel<24, SG>;
    case 32: return kde_rescue_kernel<32, SG>;
    case 64: return kde_rescue_kernel<64, SG>;
  }
  return nullptr;
}

// variant code of a prepared KDE (hbx_kde_prepare info[0]): bit 0 = signed sums, bits 1-3 = kc,
// bit 4 = hmode (whole exponent on the f16 matrix cores), bit 6 = its 32x32-tile kernel (h32 table)
// fast: the acquisition's instance where one exists (the 32x32 kernel without the one-hot lo steps,
// their bound added) -- its ln-pdf estimates are looser than 1e-5, so calls that report them do not use it
static ScoreFns pick_logpdf(int dc_pad, int du_pad, int variant, bool fast = false) {
  const bool sg = variant & 1;
  const int kc = du_pad == 0 ? 0 : (variant >> 1) & 7;  // no categorical dims: kc irrelevant
  const bool hm = (variant >> 4) & 1;
  int dcp, dup;
  bucket_dims(dc_pad, du_pad, &dcp, &dup);
  if (dcp != dc_pad || dup != du_pad) return {nullptr, nullptr, 0, 0, nullptr, nullptr};  // not a bucket
  const logpdf_fn r = sg ? pick_rescue<true>(dc_pad) : pick_rescue<false>(dc_pad);
  if (hm && ((variant >> 6) & 1)) {
    if (dc_pad < 8) return {nullptr, nullptr, 0, 0, nullptr, nullptr};
    const int kp = h32_kp(kc);
    const bool co = fast && !sg && ((variant >> 7) & 1);  // the acquisition's coarse pre-screen instance
    const bool fa = fast && kp > 0;
    const int hw = co ? H32C_WAVES : H16_WAVES;
    ScoreFns f{hbx_pick_h32(nsc_of(dc_pad), kp, sg, fa, co), r, 32 * hw * (co ? H32C_CT : 1), 64 * hw,
               hbx_pick_h32_pair(nsc_of(dc_pad), kp, sg, fa, co),
               sg ? pick_rescue_pair<true>(dc_pad) : pick_rescue_pair<false>(dc_pad), true,
               sg ? kde_combine_kernel<true, true> : kde_combine_kernel<false, true>};
    if (co && H32C_CT > 1) f.pair1 = hbx_pick_h32_pair1(nsc_of(dc_pad), kp);
    return f;
  }
  if (hm) {
    if (dc_pad < 8) return {nullptr, nullptr, 0, 0, nullptr, nullptr};
    return {hbx_pick_h(nsc_of(dc_pad), kc, sg), r, 16 * H16_WAVES * H_ROW_TILES, 64 * H16_WAVES,
            hbx_pick_h_pair(nsc_of(dc_pad), kc, sg), sg ? pick_rescue_pair<true>(dc_pad) : pick_rescue_pair<false>(dc_pad)};
  }
  if (kc == 0) return {hbx_pick_f32(dc_pad, du_pad, sg), r, 16 * MFMA_WAVES, 64 * MFMA_WAVES, nullptr, nullptr};
  return {hbx_pick_oh(dc_pad, kc, sg), r, 16 * MFMA_WAVES, 64 * MFMA_WAVES, nullptr, nullptr};
}

// launch main + rescue scoring for one KDE
static int launch_score(ScoreFns f, const double* cand, int64_t Nc, int32_t D, const void* params, const float* table,
                        KdeEst* est, hipStream_t s) {
  const unsigned gm = (unsigned)((Nc + f.cands_per_block - 1) / f.cands_per_block);
  hipLaunchKernelGGL(f.main, dim3(gm), dim3(f.threads), 0, s, cand, Nc, D, (const KdeParams*)params, table, est);
  HBX_LAUNCH_CHECK();
  hipLaunchKernelGGL(f.rescue, dim3((unsigned)((Nc + 255) / 256)), dim3(256), 0, s, cand, Nc, D,
                     (const KdeParams*)params, table, est);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

// launch main + rescue scoring for both KDEs of an acquisition: one pair launch when both run the
// same hmode instance (KDE 1 -- the bad one, normally the larger -- first), else two single launches.
// Events (optional): [0] before, [1] after KDE 0's launches, [2] after KDE 1's; a pair launch
// records [0] and [1] only ([1] after everything).
static int launch_score2(ScoreFns f0, const void* params0, const float* table0, KdeEst* est0, ScoreFns f1,
                         const void* params1, const float* table1, KdeEst* est1, const double* cand, int64_t Nc,
                         int32_t D, hipEvent_t* ev, int32_t* rescue_cnt, hipStream_t s,
                         KdePairArgs::AcqInitPtrs init = {}, bool* inited = nullptr, int64_t nmax = 0,
                         int32_t* nsplit_out = nullptr, bool* rescue_inline = nullptr) {
  if (nsplit_out) nsplit_out[0] = nsplit_out[1] = 1;
  if (rescue_inline) *rescue_inline = false;
  const bool pair = f0.pair && f0.main == f1.main && f0.rescue_pair && f0.rescue == f1.rescue && pair_enabled();
  if (ev && !pair) HBX_HIP(hipEventRecord(ev[0], s));
  if (pair) {
    unsigned gm = (unsigned)((Nc + f0.cands_per_block - 1) / f0.cands_per_block);
    logpdf_pair_fn pk = f0.pair;
    // both KDEs' blocks within one round of the chip's slots (two per CU): one column tile per wave instead,
    // twice the waves (config #2: 52 instead of 53.5 us per acquisition; profiles/r06/ct1/)
    if (f0.pair1 && f0.pair1 == f1.pair1 && 2 * gm <= 512 && pair1_enabled()) {
      pk = f0.pair1;
      gm = (unsigned)((Nc + f0.cands_per_block / H32C_CT - 1) / (f0.cands_per_block / H32C_CT));
    }
    const unsigned gr = (unsigned)((Nc + 255) / 256);
    if ((uint64_t)gr * 2 > 0x7fffffffu) return hbx_fail(HBX_ERR_ARG, "too many candidates for one pair launch");
    const bool can = f0.split_ok && nsplit_out && nmax > 0;
    // segment 0 = params1 (the bad KDE), 1 = params0.  (At about one block per CU -- config #2, 2 x 196
    // blocks -- splitting only the bad KDE's longer walks in two measured 3-5 us slower, like splitting
    // both: each range repeats the block's prologue, and the merge reads twice the estimates.)
    const int ns0 = can ? obs_splits(gm, nmax) : 1, ns1 = ns0;
    KdePairArgs a{(const KdeParams*)params1, (const KdeParams*)params0, table1, table0, est1, est0, gm * ns0,
                  rescue_cnt, {}};
    a.tiles = gm;
    a.nsplit0 = ns0;
    a.nsplit1 = ns1;
    if (nsplit_out) {
      nsplit_out[0] = ns1;  // params0's (the first KDE argument's) splits
      nsplit_out[1] = ns0;
    }
    const unsigned grid = gm * (unsigned)(ns0 + ns1);
    const bool pinit = f0.split_ok && HBX_PAIR_INIT;
    if (pinit) a.init = init;  // the 32x32 pair kernel's first workgroup sets the acquisition state
    if (ev)  // events stamped by the dispatch itself at the kernel's start and end (rocprof's duration)
      hipExtLaunchKernelGGL(pk, dim3(grid), dim3(f0.threads), 0, s, ev[0], ev[1], 0, cand, Nc, D, a);
    else
      hipLaunchKernelGGL(pk, dim3(grid), dim3(f0.threads), 0, s, cand, Nc, D, a);
    HBX_LAUNCH_CHECK();
    a.nblk0 = gr;
    a.init = pinit ? KdePairArgs::AcqInitPtrs{} : init;  // else set by the rescue pass's first workgroup
    if (inited) *inited = init.U != nullptr;
    if (rescue_inline && pinit && f0.combine_rescue && rescue_cnt && ns0 == 1 && ns1 == 1) {
      *rescue_inline = true;  // the combine kernel re-scores the marked candidates
      return HBX_OK;
    }
    // the rescue pass: grid-stride, exits at once unless the scoring kernel counted a marker
    const unsigned grr = rescue_cnt ? (2 * gr < 1024u ? 2 * gr : 1024u) : 2 * gr;
    hipLaunchKernelGGL(f0.rescue_pair, dim3(grr), dim3(256), 0, s, cand, Nc, D, a);
    HBX_LAUNCH_CHECK();
    return HBX_OK;
  }
  int rc = launch_score(f0, cand, Nc, D, params0, table0, est0, s);
  if (rc) return rc;
  if (ev) HBX_HIP(hipEventRecord(ev[1], s));
  rc = launch_score(f1, cand, Nc, D, params1, table1, est1, s);
  if (rc) return rc;
  if (ev) HBX_HIP(hipEventRecord(ev[2], s));
  return HBX_OK;
}

// workspace layout (bytes), shared by the *_workspace_bytes helpers and the acquisitions; B = number
// of acquisitions (segments) of a batched call (1 for hbx_kde_acquire).  The single result record
// comes first so its offset does not depend on the sizes.
struct WsLayout {
  size_t res, U, count, flags, segcnt, segnear, best, key, first1, rescue, est_l, est_g, lo, list, near, exact_l,
      exact_g, part, total;
};

static WsLayout ws_layout(int64_t Nc, int64_t nmax, int64_t B = 1) {
  WsLayout w;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    size_t r = o;
    o += (bytes + 255) & ~(size_t)255;
    return r;
  };
  w.res = take(sizeof(AcqResult));
  w.count = take(4);
  w.U = take(4 * B);
  w.flags = take(4 * B);
  w.segcnt = take(4 * B);
  w.segnear = take(4 * B);
  w.best = take(8 * B);
  w.key = take(8 * B);
  w.first1 = take(4 * B);
  w.rescue = take(4);
  // estimates: one per candidate and observation split (the launch's splits never exceed this bound).  The
  // allowance is non-decreasing in Nc -- a workspace sized for a larger candidate count serves every smaller
  // one: splits happen only up to 65536 candidates (128 tiles), where Nc x sp <= min(16 Nc, 196608)
  const int sp = obs_splits((unsigned)((Nc + 511) / 512), nmax, true);
  const int64_t cap16 = 16 * Nc < 196608 ? 16 * Nc : 196608;
  const int64_t nest = Nc * sp > cap16 ? Nc * sp : cap16;
  w.est_l = take(sizeof(KdeEst) * nest);
  w.est_g = take(sizeof(KdeEst) * nest);
  w.lo = take(4 * Nc);
  w.list = take(4 * Nc);
  w.near = take(4 * Nc);
  w.exact_l = take(8 * Nc);
  w.exact_g = take(8 * Nc);
  w.part = take(8 * (size_t)2 * EXACT_SPLIT_CAP * PW_SPLIT_UNITS * ((nmax + PW_BUF - 1) / PW_BUF));
  w.total = o;
  return w;
}

extern "C" {

int64_t hbx_kde_table_floats(int32_t n, int32_t dc_pad, int32_t du_pad) { return table_floats(n, dc_pad, du_pad); }

int hbx_kde_bucket(int32_t dc, int32_t du, int32_t* dc_pad, int32_t* du_pad, int32_t* stride) {
  int a, b;
  bucket_dims(dc, du, &a, &b);
  if (a < 0 || b < 0) {  // outside every fp32 scoring bucket: exact-only KDEs
    *dc_pad = *du_pad = -1;
    *stride = 0;
    return hbx_fail(HBX_ERR_UNSUPPORTED, "no fp32 scoring kernel for %d continuous / %d categorical dims "
                    "(max 64 / 32): the KDE is exact-only (every candidate re-scored in fp64)", dc, du);
  }
  *dc_pad = a;
  *du_pad = b;
  *stride = table_stride(a, b);
  return HBX_OK;
}

int64_t hbx_kde_workspace_bytes(int64_t Nc, int64_t nmax) { return (int64_t)ws_layout(Nc, nmax).total; }

// Build one KDE (good or bad) for scoring.  Host arrays: vartype[D] (0='c', 1='u'), bw[D], nlev[D].
// Device arrays: X[N][D] fp64 (rows of the whole budget), rows[n] int64 (this KDE's rows, in the
// reference's order).  Outputs: params (device, hbx_kde_param_bytes()), table (device fp32,
// hbx_kde_table_floats(n, dc_pad, du_pad) floats), info[8] (host): {variant, nan_all, unsupported, dc, du,
// nconst, dc_pad, du_pad}.  The host inputs go to the parameter buffer's staging area; the parameters
// are derived on the device (kde_params_kernel); one synchronisation for the info record.
int hbx_kde_prepare(const double* X, int32_t D, const int64_t* rows, int32_t n, const int32_t* vartype,
                    const double* bw, const int32_t* nlev, void* params, float* table, int64_t table_floats_,
                    int32_t* info, void* stream) {
  if (!X || !rows || !vartype || !bw || !nlev || !params || !table || !info)
    return hbx_fail(HBX_ERR_ARG, "hbx_kde_prepare: null pointer");
  char* stage = (char*)params + HBX_PARAM_STAGE;
  double* bw_d = (double*)stage;
  int32_t* nlev_d = (int32_t*)(stage + 8 * HBX_MAX_D);
  int32_t* info_d = nlev_d + HBX_MAX_D;
  PrepSet ps;
  memset(&ps, 0, sizeof(ps));
  ps.nk = 1;
  int rc = prep_args(&ps.k[0], X, D, rows, n, vartype, bw_d, nlev_d, params, info_d, table_floats_);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  HBX_HIP(hipMemcpyAsync(bw_d, bw, 8 * (size_t)D, hipMemcpyHostToDevice, s));
  HBX_HIP(hipMemcpyAsync(nlev_d, nlev, 4 * (size_t)D, hipMemcpyHostToDevice, s));
  rc = prep_launch(ps, table, table, s);
  if (rc) return rc;
  HBX_HIP(hipMemcpyAsync(info, info_d, 8 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HBX_HIP(hipStreamSynchronize(s));
  return HBX_OK;
}

}  // extern "C"

// ---- one-call refit (BOHB.new_result, bohb.py:211-251) ------------------------------------------
// Split metadata hbx_seg_argsort / hbx_kde_fit read from device memory, written by a kernel from its
// arguments (no host copy).
static size_t refit_meta_bytes() { return (sizeof(RefitMeta) + 255) & ~(size_t)255; }

// Append the n_new staged rows ([n_new][D] then n_new losses) at rows n - n_new .. n - 1 of X / loss,
// and write the split metadata (block 0).
__global__ __launch_bounds__(256) void kde_refit_meta_kernel(double* __restrict__ X, double* __restrict__ loss,
                                                             const double* __restrict__ staged, int64_t n_new,
                                                             RefitMetaArgs a, RefitMeta* __restrict__ m) {
  const int64_t per = n_new * (int64_t)a.D;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < per + n_new; e += (int64_t)gridDim.x * 256) {
    if (e < per) X[(a.n - n_new) * (int64_t)a.D + e] = staged[e];
    else loss[a.n - n_new + (e - per)] = staged[e];
  }
  if (blockIdx.x == 0) {
    for (int d = threadIdx.x; d < a.D; d += 256) m->vt[d] = (a.vt[d >> 5] >> (d & 31)) & 1u;
    if (threadIdx.x == 0) {
      m->seg[0] = 0;
      m->seg[1] = a.n;
      m->n_good = a.n_good;
      m->n_bad = a.n_bad;
      m->fac_good = a.fac_good;
      m->fac_bad = a.fac_bad;
    }
  }
}

// output block of hbx_kde_refit: order i64[n] | bw_good f64[D] | bw_bad f64[D] | nlev_good i32[D] |
// nlev_bad i32[D] | info_good i32[8] | info_bad i32[8]
struct RefitOut {
  size_t order, bw_good, bw_bad, nlev_good, nlev_bad, info_good, info_bad, total;
};
static RefitOut refit_out_layout(int64_t n, int32_t D) {
  RefitOut o;
  o.order = 0;
  o.bw_good = 8 * (size_t)n;
  o.bw_bad = o.bw_good + 8 * (size_t)D;
  o.nlev_good = o.bw_bad + 8 * (size_t)D;
  o.nlev_bad = o.nlev_good + 4 * (size_t)D;
  o.info_good = o.nlev_bad + 4 * (size_t)D;
  o.info_bad = o.info_good + 32;
  o.total = o.info_bad + 32;
  return o;
}

extern "C" {

int64_t hbx_kde_refit_out_bytes(int64_t n, int32_t D) { return (int64_t)refit_out_layout(n, D).total; }
int64_t hbx_kde_refit_scratch_bytes(int64_t n, int32_t D) {
  // metadata | sort scratch | host rows staged to the device (hbx_kde_refit_sync, beyond the inline copy)
  return (int64_t)refit_meta_bytes() + ((hbx_sort_scratch_bytes(n) + 15) & ~(int64_t)15) + 8 * n * ((int64_t)D + 1);
}

}  // extern "C"

static int refit_impl(double* X, double* loss, int64_t n, int32_t D, const int32_t* vartype, const double* staged,
                      bool staged_host, int64_t n_new, int64_t n_good, int64_t n_bad, double fac_good, double fac_bad,
                      void* params_good, float* table_good, int64_t table_good_floats, void* params_bad,
                      float* table_bad, int64_t table_bad_floats, void* out, void* scratch, int64_t scratch_bytes,
                      void* stream, const PrepPub* pub = nullptr);

extern "C" {

// The whole refit of one budget in one call, enqueued without host synchronisation: append the staged
// rows, stable argsort of the losses, normal-reference bandwidths and level counts of the good (head
// n_good) and bad (tail n_bad) rows, and both KDEs prepared for scoring.  The caller reads `out` back
// once (its info records say which scoring kernel each KDE runs).
int hbx_kde_refit(double* X, double* loss, int64_t n, int32_t D, const int32_t* vartype, const double* staged,
                  int64_t n_new, int64_t n_good, int64_t n_bad, double fac_good, double fac_bad, void* params_good,
                  float* table_good, int64_t table_good_floats, void* params_bad, float* table_bad,
                  int64_t table_bad_floats, void* out, void* scratch, int64_t scratch_bytes, void* stream) {
  return refit_impl(X, loss, n, D, vartype, staged, false, n_new, n_good, n_bad, fac_good, fac_bad, params_good,
                    table_good, table_good_floats, params_bad, table_bad, table_bad_floats, out, scratch, scratch_bytes,
                    stream);
}

}  // extern "C"

// Device-mapped coherent host buffers for refit output blocks: `cap` bytes of data, then the 16 flagged info
// words.  A thread holds one while it refits (grown on demand); when the thread ends, its buffer goes back to a
// process-wide pool for the next thread (no HIP call from a thread-exit destructor, no pinned memory lost per
// short-lived result thread).  The sequence number travels with the buffer, so a pooled buffer's old flags
// never match a new owner's next call.
static std::atomic<int64_t> g_mapped_live{0};  // device-mapped host buffers allocated (hbx_mapped_host_buffers)
struct RefitMapped {
  char* p = nullptr;
  int64_t cap = 0;
  int32_t seq = 0;
  bool pending = false;  // a call failed with its launches possibly still writing into the buffer
};
static std::mutex* refit_pool_mu = new std::mutex;                       // never destroyed: thread exits at
static std::vector<RefitMapped>* refit_pool = new std::vector<RefitMapped>;  // process end may still return buffers
struct RefitMappedHolder {
  RefitMapped b;
  ~RefitMappedHolder() {
    if (b.p && !b.pending) {
      std::lock_guard<std::mutex> g(*refit_pool_mu);
      refit_pool->push_back(b);
    }  // (a pending buffer is left to the process: its words may still be in flight)
  }
};
thread_local RefitMappedHolder t_refit;
static int refit_mapped_buffer(int64_t bytes, RefitMapped** out) {
  RefitMapped& b = t_refit.b;
  if (b.pending) {  // the last call failed after its launches: let them land before the buffer is reused
    HBX_HIP(hipDeviceSynchronize());
    b.pending = false;
  }
  if (bytes > b.cap) {
    RefitMapped nb;
    {
      std::lock_guard<std::mutex> g(*refit_pool_mu);
      for (size_t i = 0; i < refit_pool->size(); ++i)
        if ((*refit_pool)[i].cap >= bytes) {
          nb = (*refit_pool)[i];
          refit_pool->erase(refit_pool->begin() + i);
          break;
        }
    }
    if (!nb.p) {
      int64_t cap = b.cap > 0 ? b.cap : 16384;
      while (cap < bytes) cap *= 2;
      void* p = nullptr;
      HBX_HIP(hipHostMalloc(&p, (size_t)cap + 256, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
      void* dp = nullptr;
      HBX_HIP(hipHostGetDevicePointer(&dp, p, 0));
      if (dp != p) {
        (void)hipHostFree(p);
        return hbx_fail(HBX_ERR_UNSUPPORTED, "mapped host memory has a different device address");
      }
      nb.p = (char*)p;
      nb.cap = cap;
      g_mapped_live.fetch_add(1, std::memory_order_relaxed);
      for (int i = 0; i < 16; ++i) ((volatile uint64_t*)(nb.p + cap))[i] = 0;  // flagged info words
    }
    if (b.p) {  // the smaller buffer (every call on it completed) back to the pool
      std::lock_guard<std::mutex> g(*refit_pool_mu);
      refit_pool->push_back(b);
    }
    b = nb;
  }
  *out = &b;
  return HBX_OK;
}

extern "C" {

// hbx_kde_refit with the appended rows in HOST memory (rows then losses, n_new (D + 1) doubles: up to 256
// doubles ride in the first launch's kernel arguments, no copy; more go through the scratch), then the output
// block in host memory (out_host, hbx_kde_refit_out_bytes) when the
// call returns: the preparation's launches publish it to a device-mapped host buffer, every 32-bit word as a
// flagged word carrying the call's sequence number (the parameter launch the rows, bandwidths and level counts,
// the finishing blocks the info records; PrepPub), and the call spins until every word carries it -- no copy
// launch, no stream synchronisation, and no reliance on the order in which the launches' stores reach the host
// (bounded spin: then the stream is synchronised and the words checked once more).  The prepared parameter
// blocks and tables are complete for work on the refit's stream; another stream orders itself after the refit
// with hbx_stream_order (KDEPair does it when the calling stream is not the refit's)
int hbx_kde_refit_sync(double* X, double* loss, int64_t n, int32_t D, const int32_t* vartype,
                       const double* staged_host, int64_t n_new, int64_t n_good, int64_t n_bad, double fac_good,
                       double fac_bad, void* params_good, float* table_good, int64_t table_good_floats,
                       void* params_bad, float* table_bad, int64_t table_bad_floats, void* out, void* scratch,
                       int64_t scratch_bytes, void* stream, void* out_host) {
  if (!out_host) return hbx_fail(HBX_ERR_ARG, "hbx_kde_refit_sync: null host output");
  if (n < 1 || n > INT32_MAX || D < 1 || D > HBX_MAX_D) return hbx_fail(HBX_ERR_ARG, "hbx_kde_refit_sync: n, D");
  const int64_t words = n + 6 * (int64_t)D;  // flagged words before the info records
  RefitMapped* mb = nullptr;
  int rc = refit_mapped_buffer(8 * words, &mb);
  if (rc) return rc;
  uint64_t* w = (uint64_t*)mb->p;
  uint64_t* ll = (uint64_t*)(mb->p + mb->cap);
  const int32_t seq = mb->seq = mb->seq == INT32_MAX ? 1 : mb->seq + 1;
  PrepPub pub;
  memset(&pub, 0, sizeof(pub));
  pub.dst = w;
  pub.ll = ll;
  pub.seq = seq;
  mb->pending = true;
  rc = refit_impl(X, loss, n, D, vartype, staged_host, true, n_new, n_good, n_bad, fac_good, fac_bad, params_good,
                  table_good, table_good_floats, params_bad, table_bad, table_bad_floats, out, scratch, scratch_bytes,
                  stream, &pub);
  if (rc) return rc;
  auto tagged = [&](const uint64_t* p, int64_t cnt) {
    for (int64_t i = 0; i < cnt; ++i)
      if ((int32_t)(__atomic_load_n(p + i, __ATOMIC_ACQUIRE) >> 32) != seq) return false;
    return true;
  };
  // the info records come last: spin on them, then every other word (bounded: ~0.1 s, then the stream is
  // synchronised and every word checked once more)
  bool seen = false;
  for (int64_t i = 0; i < 5000000 && !seen; ++i) seen = tagged(ll, 16) && tagged(w, words);
  if (!seen) {
    HBX_HIP(hipStreamSynchronize((hipStream_t)stream));
    if (!tagged(ll, 16) || !tagged(w, words))
      return hbx_fail(HBX_ERR_HIP, "hbx_kde_refit_sync: the device did not publish the output block");
  }
  mb->pending = false;
  const RefitOut o = refit_out_layout(n, D);
  int64_t* order = (int64_t*)out_host;
  for (int64_t i = 0; i < n; ++i) order[i] = (int64_t)(uint32_t)w[i];
  uint32_t* rest = (uint32_t*)((char*)out_host + o.bw_good);  // bw good | bw bad | nlev good | nlev bad
  for (int64_t j = 0; j < 6 * (int64_t)D; ++j) rest[j] = (uint32_t)w[n + j];
  for (int k = 0; k < 2; ++k)
    for (int i = 0; i < 8; ++i)
      ((int32_t*)((char*)out_host + (k ? o.info_bad : o.info_good)))[i] = (int32_t)(uint32_t)ll[8 * k + i];
  const int32_t* nl = (const int32_t*)((const char*)out_host + o.nlev_good);  // good then bad
  for (int32_t d = 0; d < 2 * D; ++d)
    if (nl[d] < 0) return hbx_fail(HBX_ERR_ARG, "categorical codes must be integers in [0, 1024)");
  return HBX_OK;
}

// Order stream `waiter` after everything enqueued on stream `signaller` so far (an event recorded on the
// signaller, waited for by the waiter; no host wait): a model refit or prepared on one stream and used from
// another (KDEPair / DeviceKDE call it when the calling stream is not the model's)
int hbx_stream_order(void* waiter, void* signaller) {
  if (waiter == signaller) return HBX_OK;
  thread_local hipEvent_t ev = nullptr;
  if (!ev) HBX_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HBX_HIP(hipEventRecord(ev, (hipStream_t)signaller));
  HBX_HIP(hipStreamWaitEvent((hipStream_t)waiter, ev, 0));
  return HBX_OK;
}

}  // extern "C"


// hbx_kde_refit / hbx_kde_refit_sync (staged_host: the appended rows are in host memory)
static int refit_impl(double* X, double* loss, int64_t n, int32_t D, const int32_t* vartype, const double* staged,
                      bool staged_host, int64_t n_new, int64_t n_good, int64_t n_bad, double fac_good, double fac_bad,
                      void* params_good, float* table_good, int64_t table_good_floats, void* params_bad,
                      float* table_bad, int64_t table_bad_floats, void* out, void* scratch, int64_t scratch_bytes,
                      void* stream, const PrepPub* pub) {
  if (!X || !loss || !vartype || !params_good || !table_good || !params_bad || !table_bad || !out || !scratch ||
      (n_new > 0 && !staged))
    return hbx_fail(HBX_ERR_ARG, "hbx_kde_refit: null pointer");
  if (D < 1 || D > HBX_MAX_D) return hbx_fail(HBX_ERR_UNSUPPORTED, "D=%d outside [1, %d]", D, HBX_MAX_D);
  if (n < 1 || n > INT32_MAX || n_new < 0 || n_new > n)
    return hbx_fail(HBX_ERR_ARG, "hbx_kde_refit: n=%lld, n_new=%lld", (long long)n, (long long)n_new);
  if (n_good < 1 || n_good > n || n_bad < 1 || n_bad > n)
    return hbx_fail(HBX_ERR_ARG, "hbx_kde_refit: split %lld / %lld of %lld rows", (long long)n_good,
                    (long long)n_bad, (long long)n);
  if (scratch_bytes < hbx_kde_refit_scratch_bytes(n, D)) return hbx_fail(HBX_ERR_ARG, "refit scratch too small");
  hipStream_t s = (hipStream_t)stream;
  const RefitOut o = refit_out_layout(n, D);
  char* ob = (char*)out;
  int64_t* order = (int64_t*)(ob + o.order);
  double* bw_g = (double*)(ob + o.bw_good);
  double* bw_b = (double*)(ob + o.bw_bad);
  int32_t* nl_g = (int32_t*)(ob + o.nlev_good);
  int32_t* nl_b = (int32_t*)(ob + o.nlev_bad);
  PrepSet ps;
  memset(&ps, 0, sizeof(ps));
  ps.nk = 2;
  int rc = prep_args(&ps.k[0], X, D, order, (int32_t)n_good, vartype, bw_g, nl_g, params_good,
                     (int32_t*)(ob + o.info_good), table_good_floats);
  if (rc) return rc;
  rc = prep_args(&ps.k[1], X, D, order + (n - n_bad), (int32_t)n_bad, vartype, bw_b, nl_b, params_bad,
                 (int32_t*)(ob + o.info_bad), table_bad_floats);
  if (rc) return rc;
  if (pub) {  // the finishing blocks publish the output block (word offsets of the layout above)
    ps.pub = *pub;
    ps.pub.src = (const uint32_t*)out;
    ps.pub.n = (int32_t)n;
    ps.pub.bw_off[0] = (int32_t)(o.bw_good / 4);
    ps.pub.bw_off[1] = (int32_t)(o.bw_bad / 4);
    ps.pub.nl_off[0] = (int32_t)(o.nlev_good / 4);
    ps.pub.nl_off[1] = (int32_t)(o.nlev_bad / 4);
    ps.pub.info_off[0] = (int32_t)(o.info_good / 4);
    ps.pub.info_off[1] = (int32_t)(o.info_bad / 4);
    ps.pub.D = D;
  }
  RefitMetaArgs ma;
  memset(&ma, 0, sizeof(ma));
  ma.n = n;
  ma.n_good = n_good;
  ma.n_bad = n_bad;
  ma.fac_good = fac_good;
  ma.fac_bad = fac_bad;
  ma.D = D;
  memcpy(ma.vt, ps.k[0].vt, sizeof(ma.vt));
  RefitMeta* m = (RefitMeta*)scratch;
  char* sort_scratch = (char*)scratch + refit_meta_bytes();
  double* stage_dev = (double*)(sort_scratch + ((hbx_sort_scratch_bytes(n) + 15) & ~(int64_t)15));
  const int64_t nst = n_new * ((int64_t)D + 1);  // staged doubles: the rows, then their losses
  // host rows: carried in the sort launch's arguments when they fit (no copy), else copied through the scratch
  const bool inl = staged_host && n <= REFIT_SORT_SMALL && nst <= REFIT_INLINE;
  if (staged_host && !inl && nst > 0) {
    HBX_HIP(hipMemcpyAsync(stage_dev, staged, 8 * (size_t)nst, hipMemcpyHostToDevice, s));
    staged = stage_dev;
  }
  // numpy's argsort order (bohb.py:229): tied losses -- crashed +inf runs, quantised losses -- give the
  // reference's rows in the reference's order
  if (n <= REFIT_SORT_SMALL) {  // one launch: rows appended, metadata, sort, numpy's tie order
    rc = refit_sort_small(X, loss, inl ? nullptr : staged, inl ? staged : nullptr, n_new, ma, m, order,
                          (int32_t*)sort_scratch, s);
    if (rc) return rc;
  } else {
    const int64_t per = n_new * (int64_t)(D + 1);
    const unsigned gmeta = (unsigned)(per > 0 ? ((per + 255) / 256 < 1024 ? (per + 255) / 256 : 1024) : 1);
    hipLaunchKernelGGL(kde_refit_meta_kernel, dim3(gmeta), dim3(256), 0, s, X, loss, staged, n_new, ma, m);
    HBX_LAUNCH_CHECK();
    rc = hbx_seg_argsort_ex(loss, m->seg, 1, n, n, order, sort_scratch, hbx_sort_scratch_bytes(n), HBX_ORDER_NUMPY,
                            stream);
    if (rc) return rc;
  }
  // both sets within one LDS tile: the fit also writes the preparation's column statistics (one launch less)
  const bool fused = D > 1 && n_good <= FIT_TILE_ROWS && n_bad <= FIT_TILE_ROWS;
  if (fused)
    rc = refit_fit_colstats(X, D, m->seg, order, &m->n_good, &m->n_bad, &m->fac_good, &m->fac_bad, m->vt, bw_g, bw_b,
                            nl_g, nl_b, col_stats((KdeParams*)params_good), col_stats((KdeParams*)params_bad), s);
  else
    rc = hbx_kde_fit(X, D, m->seg, 1, order, &m->n_good, &m->n_bad, &m->fac_good, &m->fac_bad, m->vt, bw_g, bw_b,
                     nl_g, nl_b, stream);
  if (rc) return rc;
  return prep_launch(ps, table_good, table_bad, s, fused);
}



extern "C" {

// fp32 log-domain scoring of Nc candidates (fp64 [Nc][D] row-major) against one prepared KDE
int hbx_kde_logpdf(const double* cand, int64_t Nc, int32_t D, const void* params, const float* table,
                   int32_t dc_pad, int32_t du_pad, int32_t variant, void* est_out, void* stream) {
  if ((!cand || !est_out) && Nc > 0) return hbx_fail(HBX_ERR_ARG, "hbx_kde_logpdf: null pointer");
  if (!params || !table) return hbx_fail(HBX_ERR_ARG, "hbx_kde_logpdf: null pointer");
  if (Nc <= 0) return HBX_OK;
  ScoreFns f = pick_logpdf(dc_pad, du_pad, variant);
  if (!f.main) return hbx_fail(HBX_ERR_UNSUPPORTED, "no kernel for dc_pad=%d du_pad=%d", dc_pad, du_pad);
  return launch_score(f, cand, Nc, D, params, table, (KdeEst*)est_out, (hipStream_t)stream);
}

}  // extern "C"

// Shared body of hbx_kde_acquire (batch_res == nullptr: one acquisition over all Nc candidates, the
// record stays in the workspace) and hbx_kde_acquire_batch (B = ceil(Nc/seg) acquisitions over
// consecutive segments of seg candidates, one record each into batch_res).
static int acquire_impl(const char* who, const double* cand, int64_t Nc, int64_t seg, int32_t D, int64_t index_base,
                        const void* params_good, const float* table_good, const double* X_good,
                        const int64_t* rows_good, int32_t variant_good, const void* params_bad,
                        const float* table_bad, const double* X_bad, const int64_t* rows_bad, int32_t variant_bad,
                        int32_t dc_pad, int32_t du_pad, int64_t nmax, float* logl_out, float* logg_out,
                        AcqResult* batch_res, void* workspace, int64_t ws_bytes, void* events, void* stream,
                        AcqResult* host_res = nullptr, int32_t* done = nullptr, int32_t seq = 0,
                        PickOut pick = PickOut{}) {
  if ((!cand && Nc > 0) || !params_good || !table_good || !X_good || !rows_good || !params_bad || !table_bad ||
      !X_bad || !rows_bad || !workspace)
    return hbx_fail(HBX_ERR_ARG, "%s: null pointer", who);
  if (Nc < 0 || Nc > INT32_MAX) return hbx_fail(HBX_ERR_ARG, "Nc=%lld out of range", (long long)Nc);
  if (seg < 1) return hbx_fail(HBX_ERR_ARG, "%s: segment length %lld", who, (long long)seg);
  const int64_t B = batch_res ? (Nc + seg - 1) / seg : 1;
  const WsLayout w = ws_layout(Nc, nmax, B);
  if ((size_t)ws_bytes < w.total)
    return hbx_fail(HBX_ERR_ARG, "workspace too small: %lld < %lld bytes", (long long)ws_bytes,
                    (long long)w.total);
  const bool exact_only = ((variant_good | variant_bad) >> 5) & 1;
  // no ln-pdf estimates returned: the fast scoring instances (their looser bounds only widen the shortlist
  // the exact re-score resolves)
  const bool fast = !logl_out && !logg_out;
  ScoreFns fg = pick_logpdf(dc_pad, du_pad, variant_good, fast);
  ScoreFns fb = pick_logpdf(dc_pad, du_pad, variant_bad, fast);
  if (!exact_only && (!fg.main || !fb.main))
    return hbx_fail(HBX_ERR_UNSUPPORTED, "no kernel for dc_pad=%d du_pad=%d", dc_pad, du_pad);
  char* ws = (char*)workspace;
  uint32_t* U = (uint32_t*)(ws + w.U);
  int32_t* count = (int32_t*)(ws + w.count);
  int32_t* flags = (int32_t*)(ws + w.flags);
  int32_t* segcnt = (int32_t*)(ws + w.segcnt);
  int32_t* segnear = (int32_t*)(ws + w.segnear);
  int32_t* near = (int32_t*)(ws + w.near);
  uint64_t* best = (uint64_t*)(ws + w.best);
  uint64_t* key = (uint64_t*)(ws + w.key);
  int32_t* first1 = (int32_t*)(ws + w.first1);
  AcqResult* res = (AcqResult*)(ws + w.res);
  KdeEst* el = (KdeEst*)(ws + w.est_l);
  KdeEst* eg = (KdeEst*)(ws + w.est_g);
  float* lo = (float*)(ws + w.lo);
  int32_t* list = (int32_t*)(ws + w.list);
  double* exact_l = (double*)(ws + w.exact_l);
  double* exact_g = (double*)(ws + w.exact_g);
  double* part = (double*)(ws + w.part);
  hipStream_t s = (hipStream_t)stream;
  const uint32_t sg = (uint32_t)(batch_res ? seg : (Nc > 0 ? Nc : 1));
  if (B == 0) return HBX_OK;  // batched call without candidates: no records
  // the scoring launch goes first (it touches none of the per-acquisition state), so the GPU starts on
  // it while the host is still enqueueing the rest
  const bool scored = Nc > 0 && !exact_only;
  bool inited = false;  // a single acquisition's pair launch: its rescue pass initialises the state
  int32_t nsplit[2] = {1, 1};  // the scoring launch's observation splits, good / bad (merged before the combine)
  bool rescue_inline = false;  // the rescue pass left to the combine kernel
  if (scored) {
    hipEvent_t* ev = (hipEvent_t*)events;  // optional: [before l, between, after g] for timing
    KdePairArgs::AcqInitPtrs ip{};
    if (!batch_res) ip = KdePairArgs::AcqInitPtrs{U, count, flags, first1, res};
    const int rc = launch_score2(fg, params_good, table_good, el, fb, params_bad, table_bad, eg, cand, Nc, D, ev,
                                 (int32_t*)(ws + w.rescue), s, ip, &inited,
                                 fast ? nmax : 0,  // splits for the pick only: reported ln-pdfs stay unsplit
                                 nsplit, batch_res ? nullptr : &rescue_inline);
    if (rc) return rc;
  }
  if (batch_res) {
    hipLaunchKernelGGL(acq_init_batch_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, B, U, flags,
                       segcnt, best, key, first1, count, segnear);
    HBX_LAUNCH_CHECK();
  } else if (!inited) {
    hipLaunchKernelGGL(acq_init_kernel, dim3(1), dim3(64), 0, s, U, count, flags, first1, res);
    HBX_LAUNCH_CHECK();
  }
  const dim3 grid((unsigned)((Nc + 255) / 256));
  bool fuse_combine = false;
  if (Nc > 0) {
    if (exact_only) {
      hipLaunchKernelGGL(kde_exact_only_init_kernel, grid, dim3(256), 0, s, Nc, sg, el, eg, lo, flags);
      HBX_LAUNCH_CHECK();
    } else {
      if (nsplit[0] > 1 || nsplit[1] > 1) {  // the scoring launch's observation splits merged first
        hipLaunchKernelGGL(kde_merge_splits_kernel, dim3((unsigned)((2 * Nc + 255) / 256)), dim3(256), 0, s, el, eg,
                           Nc, nsplit[0], nsplit[1]);
        HBX_LAUNCH_CHECK();
      }
      const CombineRescue rs{cand, D, (const KdeParams*)params_good, (const KdeParams*)params_bad,
                             (const int32_t*)(ws + w.rescue)};
      const combine_fn cf = rescue_inline ? fg.combine_rescue : kde_combine_kernel<false, false>;
      hipLaunchKernelGGL(cf, dim3((unsigned)((Nc + 256 * COMBINE_SUB - 1) / (256 * COMBINE_SUB))), dim3(256), 0, s, el,
                         eg, Nc, sg, logl_out, logg_out, lo, U, flags, first1, rs);
      HBX_LAUNCH_CHECK();
    }
    // a single acquisition of few candidates: the exact re-score's blocks shortlist for themselves
    const bool scan = !batch_res && Nc <= EXACT_SCAN_MAX;
    if (!scan) {
      hipLaunchKernelGGL(kde_shortlist_kernel, grid, dim3(256), 0, s, lo, Nc, sg, U, flags, list, count,
                         batch_res ? segcnt : (int32_t*)nullptr, first1, (int32_t*)(ws + w.rescue));
      HBX_LAUNCH_CHECK();
    }
    const int nbuf = (int)((nmax + PW_BUF - 1) / PW_BUF);
    const ExactScan esc{lo, Nc, U, flags, first1, list, count, (int32_t*)(ws + w.rescue)};
    auto ek = scan ? kde_exact_kernel<true> : kde_exact_kernel<false>;
    hipLaunchKernelGGL(ek, dim3(EXACT_GRID), dim3(EXACT_ACQ_THREADS), 0, s, cand, D,
                       (const KdeParams*)params_good, X_good, rows_good, (const KdeParams*)params_bad, X_bad,
                       rows_bad, list, count, nbuf, part, exact_l, exact_g, esc);
    HBX_LAUNCH_CHECK();
    // single acquisition: the final kernel combines the unit sums itself (one launch less)
    fuse_combine = !batch_res && !(exact_only && (logl_out || logg_out));
    if (!fuse_combine) {
      hipLaunchKernelGGL(kde_exact_combine_kernel, dim3((2 * EXACT_SPLIT_CAP + 3) / 4), dim3(256), 0, s,
                         (const KdeParams*)params_good, (const KdeParams*)params_bad, count, nbuf, part, exact_l,
                         exact_g);
      HBX_LAUNCH_CHECK();
    }
    if (exact_only && (logl_out || logg_out)) {
      hipLaunchKernelGGL(kde_exact_logs_kernel, grid, dim3(256), 0, s, list, count, exact_l, exact_g, logl_out,
                         logg_out);
      HBX_LAUNCH_CHECK();
    }
  }
  if (!batch_res) {
    hipLaunchKernelGGL(kde_final_kernel, dim3(1), dim3(256), 0, s, list, count, exact_l, exact_g, flags,
                       index_base, (const KdeParams*)params_good, (const KdeParams*)params_bad, el, eg, near, res,
                       (int32_t)((nmax + PW_BUF - 1) / PW_BUF), fuse_combine ? part : (const double*)nullptr,
                       exact_l, exact_g, host_res, done, seq, pick);
    HBX_LAUNCH_CHECK();
    return HBX_OK;
  }
  if (Nc > 0) {
    hipLaunchKernelGGL(kde_batch_min_kernel, grid, dim3(256), 0, s, list, count, sg, exact_l, exact_g, best);
    HBX_LAUNCH_CHECK();
    hipLaunchKernelGGL(kde_batch_key_kernel, grid, dim3(256), 0, s, list, count, sg, exact_l, exact_g, best, key);
    HBX_LAUNCH_CHECK();
    hipLaunchKernelGGL(kde_batch_near_kernel, grid, dim3(256), 0, s, list, count, sg, exact_l, exact_g, key,
                       (const KdeParams*)params_good, (const KdeParams*)params_bad, el, eg, near, segnear);
    HBX_LAUNCH_CHECK();
    hipLaunchKernelGGL(kde_batch_final_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, B, key, segcnt,
                       flags, segnear, list, exact_l, exact_g, (const KdeParams*)params_good,
                       (const KdeParams*)params_bad, el, eg, index_base, batch_res);
    HBX_LAUNCH_CHECK();
  }
  return HBX_OK;
}

extern "C" {

// One acquisition: score every candidate against l (good) and g (bad), shortlist, exact re-score,
// argmin.  index_base offsets the reported index (candidate sharding across GPUs).  The result
// (AcqResult) stays in the workspace; hbx_kde_result_ptr() gives its device address.
int hbx_kde_acquire(const double* cand, int64_t Nc, int32_t D, int64_t index_base,
                    const void* params_good, const float* table_good, const double* X_good,
                    const int64_t* rows_good, int32_t variant_good,
                    const void* params_bad, const float* table_bad, const double* X_bad,
                    const int64_t* rows_bad, int32_t variant_bad, int32_t dc_pad, int32_t du_pad,
                    int64_t nmax, float* logl_out, float* logg_out, void* workspace, int64_t ws_bytes,
                    void* events, void* stream) {
  return acquire_impl("hbx_kde_acquire", cand, Nc, Nc > 0 ? Nc : 1, D, index_base, params_good, table_good, X_good,
                      rows_good, variant_good, params_bad, table_bad, X_bad, rows_bad, variant_bad, dc_pad, du_pad,
                      nmax, logl_out, logg_out, nullptr, workspace, ws_bytes, events, stream);
}

int64_t hbx_kde_batch_workspace_bytes(int64_t Nc, int64_t seg, int64_t nmax) {
  if (seg < 1) return -1;
  return (int64_t)ws_layout(Nc, nmax, (Nc + seg - 1) / seg).total;
}

// Batched acquisition: candidates [b*seg, min((b+1)*seg, Nc)) are the num_samples candidates of
// get_config call b; every segment gets its own exact argmin (index relative to the segment start,
// plus index_base) in results[b].  Same kernels as hbx_kde_acquire, one pass for all segments.
int hbx_kde_acquire_batch(const double* cand, int64_t Nc, int64_t seg, int32_t D, int64_t index_base,
                          const void* params_good, const float* table_good, const double* X_good,
                          const int64_t* rows_good, int32_t variant_good,
                          const void* params_bad, const float* table_bad, const double* X_bad,
                          const int64_t* rows_bad, int32_t variant_bad, int32_t dc_pad, int32_t du_pad,
                          int64_t nmax, float* logl_out, float* logg_out, void* results, void* workspace,
                          int64_t ws_bytes, void* stream) {
  if (!results) return hbx_fail(HBX_ERR_ARG, "hbx_kde_acquire_batch: null results");
  return acquire_impl("hbx_kde_acquire_batch", cand, Nc, seg, D, index_base, params_good, table_good, X_good,
                      rows_good, variant_good, params_bad, table_bad, X_bad, rows_bad, variant_bad, dc_pad, du_pad,
                      nmax, logl_out, logg_out, (AcqResult*)results, workspace, ws_bytes, nullptr, stream);
}

// the exact pdf stages its per-observation terms in LDS: no global scratch is needed any more (the
// entry point keeps its scratch argument; 256 bytes keep callers' allocations non-empty)
int64_t hbx_kde_pdf_scratch_bytes(int64_t nmax) { return 256; }

// Exact fp64 pdf (reference arithmetic and operation order) of one prepared KDE at Np points
// (device fp64 [Np][D]) -> out (device fp64 [Np]).  KDEMultivariate.pdf as a batched GPU call.
int hbx_kde_pdf_exact(const double* pts, int64_t Np, int32_t D, const void* params, const double* X,
                      const int64_t* rows, int64_t n, double* out, void* scratch, int64_t scratch_bytes,
                      void* stream) {
  if (((!pts || !out) && Np > 0) || !params || !X || !rows || !scratch)
    return hbx_fail(HBX_ERR_ARG, "hbx_kde_pdf_exact: null");
  if (scratch_bytes < hbx_kde_pdf_scratch_bytes(n)) return hbx_fail(HBX_ERR_ARG, "pdf scratch too small");
  if (Np <= 0) return HBX_OK;
  const unsigned grid = (unsigned)(Np < EXACT_GRID ? Np : EXACT_GRID);
  hipLaunchKernelGGL(kde_pdf_exact_kernel, dim3(grid), dim3(EXACT_THREADS), 0, (hipStream_t)stream, pts, Np, D,
                     (const KdeParams*)params, X, rows, out, (const int32_t*)nullptr, (const int32_t*)nullptr, 0);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

// ln pdf in fp64 log space (kde_logpdf_exact_kernel): the accurate log-domain value, NaN where the
// KDE has negative categorical factors or structural NaNs (use hbx_kde_pdf_exact there).
int hbx_kde_logpdf_exact(const double* pts, int64_t Np, int32_t D, const void* params, const double* X,
                         const int64_t* rows, double* out, void* stream) {
  if (((!pts || !out) && Np > 0) || !params || !X || !rows) return hbx_fail(HBX_ERR_ARG, "hbx_kde_logpdf_exact: null");
  if (D < 1 || D > HBX_MAX_D) return hbx_fail(HBX_ERR_ARG, "hbx_kde_logpdf_exact: D=%d", D);
  if (Np <= 0) return HBX_OK;
  const unsigned grid = (unsigned)(Np < EXACT_GRID ? Np : EXACT_GRID);
  hipLaunchKernelGGL(kde_logpdf_exact_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, pts, Np, D,
                     (const KdeParams*)params, X, rows, out, (const int32_t*)nullptr, (const int32_t*)nullptr);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

}  // extern "C"

int hbx_logpdf_estimate(const double* cand, int64_t Nc, int32_t D, const void* params, const float* table,
                        int32_t dc_pad, int32_t du_pad, int32_t variant, KdeEst* est, hipStream_t s) {
  ScoreFns f = pick_logpdf(dc_pad, du_pad, variant);
  if (!f.main) return hbx_fail(HBX_ERR_UNSUPPORTED, "no kernel for dc_pad=%d du_pad=%d", dc_pad, du_pad);
  return launch_score(f, cand, Nc, D, params, table, est, s);
}

int hbx_logpdf_exact_listed(const double* cand, int64_t Nc, int32_t D, const KdeParams* P, const double* X,
                            const int64_t* rows, double* out, const int32_t* list, const int32_t* count,
                            bool per_point, hipStream_t s) {
  const unsigned grid = (unsigned)(Nc < EXACT_GRID ? Nc : EXACT_GRID);
  if (per_point) {
    hipLaunchKernelGGL(kde_logpdf_exact_kernel, dim3(grid), dim3(256), 0, s, cand, Nc, D, P, X, rows, out, list, count);
    HBX_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(kde_pdf_exact_kernel, dim3(grid), dim3(EXACT_THREADS), 0, s, cand, Nc, D, P, X, rows, out, list,
                     count, 1);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

extern "C" {

// Timing events (hipEvent_t) for hbx_kde_acquire's `events` argument.
int hbx_event_create(void** ev) {
  HBX_HIP(hipEventCreate((hipEvent_t*)ev));
  return HBX_OK;
}
int hbx_event_destroy(void* ev) {
  HBX_HIP(hipEventDestroy((hipEvent_t)ev));
  return HBX_OK;
}
int hbx_event_elapsed_ms(void* start, void* stop, float* ms) {
  HBX_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
  return HBX_OK;
}

void* hbx_kde_result_ptr(void* workspace) { return (char*)workspace + ws_layout(0, 0).res; }

// A small device buffer (an acquisition's result record) to the host with no copy engine and no blocking
// synchronisation: one wave copies it into this thread's device-mapped coherent host buffer, then stores a
// completion word last (system scope, after a system fence); the host spins on that word (bounded: then
// the stream is synchronised) and copies the bytes out.  A DMA copy + stream synchronisation of the
// 48-byte record cost ~28 us per acquisition (tools/step_breakdown.py)
__global__ void fetch_publish_kernel(const uint32_t* __restrict__ src, int32_t words, uint32_t* dst, int32_t* done,
                                     int32_t seq) {
  for (int i = threadIdx.x; i < words; i += 64) hbx_publish_store(dst + i, src[i]);
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every lane's words acknowledged (one wave)
  if (threadIdx.x == 0) hbx_publish_done(done, seq);
}

#define FETCH_MAPPED_BYTES 4096
// the final kernel's tagged words (hbx_kde_acquire_bound) live past the completion word, apart from hbx_fetch's
// untagged bytes (whose words could otherwise pass for a later call's tags)
#define PUB_OFF (FETCH_MAPPED_BYTES + 64)
#define PUB_BYTES (8 * (16 + 2 * HBX_MAX_D))
// this thread's device-mapped coherent host buffer: FETCH_MAPPED_BYTES of data, the completion word, then the
// tagged region.  Held for the thread's lifetime and then pooled for the next thread, like the refit buffers
// (short-lived result threads do not each leave one behind); its sequence number travels with it, so a pooled
// buffer's old completion word and tags never match a new owner's calls.
struct AcqMapped {
  char* p = nullptr;
  int32_t seq = 0;
};
static std::mutex* acq_pool_mu = new std::mutex;                     // never destroyed (as refit_pool)
static std::vector<AcqMapped>* acq_pool = new std::vector<AcqMapped>;
struct AcqMappedHolder {
  AcqMapped b;
  ~AcqMappedHolder() {
    if (b.p) {
      std::lock_guard<std::mutex> g(*acq_pool_mu);
      acq_pool->push_back(b);
    }
  }
};
thread_local AcqMappedHolder t_acq;
// the buffer and this call's sequence number (>= 1)
static int mapped_buffer(char** out, int32_t* seq) {
  AcqMapped& b = t_acq.b;
  if (!b.p) {
    {
      std::lock_guard<std::mutex> g(*acq_pool_mu);
      if (!acq_pool->empty()) {
        b = acq_pool->back();
        acq_pool->pop_back();
      }
    }
    if (!b.p) {
      void* p = nullptr;
      HBX_HIP(hipHostMalloc(&p, PUB_OFF + PUB_BYTES,
                            hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
      memset(p, 0, PUB_OFF + PUB_BYTES);  // (no stale tag can match: sequence numbers start at 1)
      void* dp = nullptr;
      HBX_HIP(hipHostGetDevicePointer(&dp, p, 0));
      if (dp != p) {
        (void)hipHostFree(p);
        return hbx_fail(HBX_ERR_UNSUPPORTED, "mapped host memory has a different device address");
      }
      b.p = (char*)p;
      b.seq = 0;
      g_mapped_live.fetch_add(1, std::memory_order_relaxed);
    }
  }
  b.seq = b.seq == INT32_MAX ? 1 : b.seq + 1;
  *out = b.p;
  *seq = b.seq;
  return HBX_OK;
}

// spin on the completion word (bounded: ~0.1 s, then the stream is synchronised)
static int wait_done(int32_t* done, int32_t seq, hipStream_t s, const char* who) {
  bool seen = false;
  for (int64_t i = 0; i < 20000000 && !seen; ++i) seen = __atomic_load_n(done, __ATOMIC_ACQUIRE) == seq;
  if (!seen) {
    HBX_HIP(hipStreamSynchronize(s));
    if (__atomic_load_n(done, __ATOMIC_ACQUIRE) != seq)
      return hbx_fail(HBX_ERR_HIP, "%s: the device did not store its completion word", who);
  }
  return HBX_OK;
}

// spin until `n` tagged words (seq << 32 | word, 8 bytes each, stored by the device in any order) all carry
// this call's sequence number, then take their words (bounded like wait_done)
static int hbx_pub_wait(const volatile uint64_t* w, int n, int32_t seq, uint32_t* out, hipStream_t s, const char* who) {
  const uint32_t sq = (uint32_t)seq;
  int i = 0;
  for (int64_t it = 0; it < 20000000 && i < n; ++it) {
    while (i < n) {
      const uint64_t v = __atomic_load_n((const uint64_t*)(w + i), __ATOMIC_ACQUIRE);
      if ((uint32_t)(v >> 32) != sq) break;
      out[i++] = (uint32_t)v;
    }
  }
  if (i < n) {
    HBX_HIP(hipStreamSynchronize(s));
    for (; i < n; ++i) {
      const uint64_t v = __atomic_load_n((const uint64_t*)(w + i), __ATOMIC_ACQUIRE);
      if ((uint32_t)(v >> 32) != sq) return hbx_fail(HBX_ERR_HIP, "%s: the device did not publish word %d", who, i);
      out[i] = (uint32_t)v;
    }
  }
  return HBX_OK;
}

int64_t hbx_mapped_host_buffers(void) { return g_mapped_live.load(std::memory_order_relaxed); }

int hbx_fetch(void* host_dst, const void* dev_src, int64_t bytes, void* stream) {
  if (bytes < 0 || (bytes > 0 && (!host_dst || !dev_src))) return hbx_fail(HBX_ERR_ARG, "hbx_fetch: bad arguments");
  const hipStream_t s = (hipStream_t)stream;
  const bool small = bytes <= FETCH_MAPPED_BYTES && (bytes & 3) == 0 && ((uintptr_t)dev_src & 3) == 0;
  char* mapped = nullptr;
  int32_t seq = 0;
  if (small) {
    const int rc = mapped_buffer(&mapped, &seq);
    if (rc) return rc;
  }
  if (!small) {  // larger or unaligned: a copy, then the stream polled to completion
    if (bytes > 0) HBX_HIP(hipMemcpyAsync(host_dst, dev_src, (size_t)bytes, hipMemcpyDeviceToHost, s));
    hipError_t e;
    while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
    }
    if (e != hipSuccess) return hbx_fail(HBX_ERR_HIP, "hbx_fetch: %s", hipGetErrorString(e));
    return HBX_OK;
  }
  int32_t* done = (int32_t*)(mapped + FETCH_MAPPED_BYTES);
  hipLaunchKernelGGL(fetch_publish_kernel, dim3(1), dim3(64), 0, s, (const uint32_t*)dev_src, (int32_t)(bytes / 4),
                     (uint32_t*)mapped, done, seq);
  HBX_LAUNCH_CHECK();
  const int rc = wait_done(done, seq, s, "hbx_fetch");
  if (rc) return rc;
  memcpy(host_dst, mapped, (size_t)bytes);
  return HBX_OK;
}

struct KdePairBinding {
  int32_t D;
  const void* params_good;
  const float* table_good;
  const double* X_good;
  const int64_t* rows_good;
  int32_t variant_good;
  const void* params_bad;
  const float* table_bad;
  const double* X_bad;
  const int64_t* rows_bad;
  int32_t variant_bad, dc_pad, du_pad;
  int64_t nmax;
};

void* hbx_kde_pair_bind(int32_t D, const void* params_good, const float* table_good, const double* X_good,
                        const int64_t* rows_good, int32_t variant_good, const void* params_bad,
                        const float* table_bad, const double* X_bad, const int64_t* rows_bad, int32_t variant_bad,
                        int32_t dc_pad, int32_t du_pad, int64_t nmax) {
  if (D <= 0 || D > HBX_MAX_D || !params_good || !params_bad || nmax < 0) {
    hbx_fail(HBX_ERR_ARG, "hbx_kde_pair_bind: bad arguments (D=%d, nmax=%lld)", D, (long long)nmax);
    return nullptr;
  }
  KdePairBinding* b = new (std::nothrow) KdePairBinding{D, params_good, table_good, X_good, rows_good, variant_good,
                                                        params_bad, table_bad, X_bad, rows_bad, variant_bad, dc_pad,
                                                        du_pad, nmax};
  if (!b) hbx_fail(HBX_ERR_ARG, "hbx_kde_pair_bind: out of host memory");
  return b;
}

// The drop-in's synchronous acquisition on a bound pair: the final kernel stores the 48-byte record into this
// thread's mapped host buffer and a completion word last; the call spins on that word and copies the record to
// rec_out -- the acquisition and its pick on the host in one call, no copy kernel, no blocking synchronisation.
// err (nullable, device u8[Nc]: the GPU sampler's domain-error flags) sets HBX_ACQ_DOMAIN_ERR in the record
// when any is set; row_out (nullable, host f64[D]) receives the winning candidate's row -- both published by
// the same final kernel with the record (one wait for the draws' check, the pick and its row).
int hbx_kde_acquire_bound(const void* pair, const double* cand, int64_t Nc, int64_t index_base, void* workspace,
                          int64_t ws_bytes, const uint8_t* err, void* events, void* stream, void* rec_out,
                          double* row_out) {
  if (!pair || !rec_out || Nc < 0) return hbx_fail(HBX_ERR_ARG, "hbx_kde_acquire_bound: bad arguments");
  const KdePairBinding& b = *(const KdePairBinding*)pair;
  char* mapped = nullptr;
  int32_t seq = 0;
  int rc = mapped_buffer(&mapped, &seq);
  if (rc) return rc;
  const bool pick = err || row_out;  // (8 (13 + 2 D) <= PUB_BYTES for D <= HBX_MAX_D)
  rc = acquire_impl("hbx_kde_acquire_bound", cand, Nc, Nc > 0 ? Nc : 1, b.D, index_base, b.params_good, b.table_good,
                    b.X_good, b.rows_good, b.variant_good, b.params_bad, b.table_bad, b.X_bad, b.rows_bad, b.variant_bad,
                    b.dc_pad, b.du_pad, b.nmax, nullptr, nullptr, nullptr, workspace, ws_bytes, events, stream,
                    pick ? nullptr : (AcqResult*)(mapped + PUB_OFF), nullptr, seq,
                    pick ? PickOut{cand, err, Nc, b.D, mapped + PUB_OFF} : PickOut{});
  if (rc) return rc;
  // the final kernel's tagged words: the record, then (a pick) the flag, then the row when there is a winner
  constexpr int RW = (int)(sizeof(AcqResult) / 4);
  const volatile uint64_t* w = (const volatile uint64_t*)(mapped + PUB_OFF);
  uint32_t words[RW];
  rc = hbx_pub_wait(w, RW, seq, words, (hipStream_t)stream, "hbx_kde_acquire_bound");
  if (rc) return rc;
  AcqResult r;
  memcpy(&r, words, sizeof(AcqResult));
  if (pick) {
    uint32_t e = 0;
    rc = hbx_pub_wait(w + RW, 1, seq, &e, (hipStream_t)stream, "hbx_kde_acquire_bound");
    if (rc) return rc;
    if (e) r.flags |= HBX_ACQ_DOMAIN_ERR;
    if (row_out && r.index >= 0 && r.index - index_base < Nc) {
      rc = hbx_pub_wait(w + RW + 1, 2 * b.D, seq, (uint32_t*)row_out, (hipStream_t)stream, "hbx_kde_acquire_bound");
      if (rc) return rc;
    }
  }
  memcpy(rec_out, &r, sizeof(AcqResult));
  return HBX_OK;
}

void hbx_kde_pair_free(void* pair) { delete (KdePairBinding*)pair; }

// numpy's float64 exp (hbx_npexp.h) element-wise: the known-answer check of the exact re-score's exp
__global__ void np_exp_kernel(const double* __restrict__ x, int64_t n, double* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) y[i] = hbx_npexp::exp(x[i]);
}

int hbx_np_exp(const double* x, int64_t n, double* y, void* stream) {
  if ((!x || !y) && n > 0) return hbx_fail(HBX_ERR_ARG, "hbx_np_exp: null pointer");
  if (n <= 0) return HBX_OK;
  hipLaunchKernelGGL(np_exp_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, n, y);
  HBX_LAUNCH_CHECK();
  return HBX_OK;
}

// Byte offsets inside an acquisition workspace of (Nc, seg, nmax) -- hbx_kde_acquire: seg = Nc -- of
// what a host re-resolution of a near tie reads: out[0] shortlist count (i32), [1] shortlist (i32
// candidate indices), [2] near list (hbx_kde_acquire: the near set's candidate indices, res.near of
// them; batched: a 0/1 flag per shortlist entry), [3] exact l, [4] exact g (f64 per shortlist entry).
int hbx_kde_ws_offsets(int64_t Nc, int64_t seg, int64_t nmax, int64_t* out) {
  if (!out || seg < 1) return hbx_fail(HBX_ERR_ARG, "hbx_kde_ws_offsets: bad arguments");
  const WsLayout w = ws_layout(Nc, nmax, seg >= Nc ? 1 : (Nc + seg - 1) / seg);
  out[0] = (int64_t)w.count;
  out[1] = (int64_t)w.list;
  out[2] = (int64_t)w.near;
  out[3] = (int64_t)w.exact_l;
  out[4] = (int64_t)w.exact_g;
  return HBX_OK;
}

}  // extern "C"

#ifdef PREP_STAMPS
extern "C" int hbx_debug_prep_stamps(unsigned long long* out) {
  HBX_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(prep_stamps), sizeof(prep_stamps)));
  return HBX_OK;
}
#endif
