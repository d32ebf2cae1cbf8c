// hbx_common.h -- shared definitions for the MI355X (gfx950) KDE-acquisition / SH-promotion engine.
//
// Everything in this directory is compiled by hipcc --offload-arch=gfx950 into ONE shared library
// (hpbandster_amd/_lib/libhbx.so) whose extern "C" entry points are declared in include/hbx.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define HBX_MAX_D 256          // largest configuration-space dimension the engine accepts
#define HBX_WAVE 64            // CDNA wavefront width

#include "hbx.h"  // the public C ABI (include/hbx.h): every definition here must match it

// Sets the thread-local error message returned by hbx_last_error(); returns `code`.
int hbx_fail(int code, const char* fmt, ...);

#define HBX_HIP(call)                                                                 \
  do {                                                                                \
    hipError_t _e = (call);                                                           \
    if (_e != hipSuccess)                                                             \
      return hbx_fail(HBX_ERR_HIP, "%s failed: %s (%s:%d)", #call, hipGetErrorString(_e), \
                      __FILE__, __LINE__);                                            \
  } while (0)

#define HBX_LAUNCH_CHECK()                                                            \
  do {                                                                                \
    hipError_t _e = hipGetLastError();                                                \
    if (_e != hipSuccess)                                                             \
      return hbx_fail(HBX_ERR_HIP, "kernel launch failed: %s (%s:%d)",               \
                      hipGetErrorString(_e), __FILE__, __LINE__);                    \
  } while (0)

// ------------------------------------------------------------------------------------------
// KDE model parameters, one block per KDE (good or bad).  Written on the device by
// kde_params_kernel from (data rows, bandwidths, level counts); read by the scoring kernels.
// Python never looks inside: it only allocates hbx_kde_param_bytes() bytes.
struct KdeParams {
  int32_t n;          // observations in this KDE
  int32_t D;          // total dims
  int32_t dc;         // continuous dims
  int32_t du;         // active categorical dims (num_levels > 1)
  int32_t nconst;     // categorical dims with a single observed level (bw == 0)
  int32_t nan_all;    // a continuous bandwidth is 0 -> reference pdf is NaN everywhere
  int32_t has_neg;    // some active categorical dim has 1 - h < 0 (signed sums needed)
  int32_t unsupported;// bandwidth/level combination the engine does not model (error)
  int32_t stride;     // floats per observation row of the fp32 table
  int32_t dc_pad;     // continuous slots in the table (template bucket)
  int32_t du_pad;     // categorical slots in the table (template bucket)
  int32_t exact_only; // no fp32 scoring bucket fits (> 64 continuous / > 32 categorical dims): every
                      // candidate is re-scored in fp64 (variant bit 5)
  double log_norm;    // ln pdf = ln(S) + log_norm  (S = sum of 2^(t - M0))
  double m0_log2;     // M0: upper bound of the per-pair log2 kernel product
  double lb_sum;      // sum over active categorical dims of log2(h/(c-1))
  double prod_bw_c;   // sequential product of continuous bandwidths (reference op order)
  float cmax;         // max_j |C_j| over the table (error bound)
  float sum_abs_delta;// sum |delta_u| over finite deltas (error bound)
  float cmax2;        // max_j |C_j| of the f32-layout rebuild (hmode table out of the f16 range)
  int32_t pad1;
  int32_t kc;         // categorical mode: 0 = VALU match on codes, k >= 1 = one-hot on f16 MFMA,
                      // k steps of K=32 (2 * oh_total <= 32 k)
  int32_t hmode;      // 1: continuous product on f16 matrix cores too (hi/lo split coordinates)
  int32_t nsc;        // hmode: f16 K-steps (of 32) of the continuous product = ceil(4 dc_pad / 32)
  int32_t chunk_floats; // floats per 64-observation chunk of this KDE's table (layout depends on kc)
  int32_t oh_total;   // one-hot width: sum over active categorical dims of (max observed code + 1)
  int32_t coarse_off; // floats into the table where the coarse h32 layout starts (0: none)
  int32_t coarse_chunk_floats; // floats per 64-observation chunk of the coarse table
  const double* X;    // the KDE's data (device): X[rows[j]] is observation j (rescue / exact paths)
  const int64_t* rows;
  int32_t oh_dim[64];   // one-hot slot -> active categorical dim u
  int32_t oh_level[64]; // one-hot slot -> code level
  int32_t oh_col[64];   // one-hot slot -> candidate column (cat_dim[oh_dim[t]])
  double oh_val[64];    // one-hot slot -> code level as the fp64 value a matching column holds
  int32_t oh_start[64]; // active categorical dim u -> one-hot slot of its level 0 (one-hot mode only)
  int32_t cat_maxcode[HBX_MAX_D]; // per active categorical dim: max observed code (-1: not an integer code)
  int32_t cont_dim[HBX_MAX_D];
  double cont_scale[HBX_MAX_D];     // s_c = sqrt(log2(e) / 2) / h_c
  double center[HBX_MAX_D];         // per continuous slot: mean of the KDE's data (coordinates are
                                    // centred before scaling so the fp32 expansion keeps precision)
  float xmax[HBX_MAX_D];            // max_j |X'_jc| (error bound)
  int32_t cat_dim[HBX_MAX_D];
  float cat_delta[HBX_MAX_D];       // log2|1-h| - log2(h/(c-1)); -1e30 when 1-h == 0
  float cat_negf[HBX_MAX_D];        // 1.0 when 1-h < 0
  int32_t const_dim[HBX_MAX_D];
  double const_level[HBX_MAX_D];
  // exact fp64 re-score (reference arithmetic)
  int32_t vartype[HBX_MAX_D];       // 0 = continuous 'c', 1 = unordered categorical 'u'
  int32_t nlev[HBX_MAX_D];
  double bw[HBX_MAX_D];
};

// A parameter buffer (hbx_kde_param_bytes()) is the KdeParams block followed by a staging area for
// hbx_kde_prepare's host inputs (bandwidths, level counts) and its info record.
// After the staging area: per-dim column statistics of the KDE's observations (ColStats), written by
// the first preparation kernel and read by the parameter kernel.
#define HBX_PARAM_STAGE ((sizeof(KdeParams) + 255) & ~(size_t)255)
#define HBX_COLSTATS_OFF (HBX_PARAM_STAGE + 8 * HBX_MAX_D + 4 * HBX_MAX_D + 64)
#define HBX_PARAM_BYTES (HBX_COLSTATS_OFF + 8 * HBX_MAX_D + 4 * HBX_MAX_D)
struct ColStats {
  double mean[HBX_MAX_D];      // continuous dim: mean of the column (any summation order)
  int32_t maxcode[HBX_MAX_D];  // categorical dim: largest code, -1 when a code is not an integer in [0, 1024)
};

// Per-candidate output of the fp32 log-domain scoring kernel, one per KDE.
struct KdeEst {
  float lpos;   // ln(sum of positive terms) + log_norm   (NaN: structural NaN pdf)
  float lneg;   // ln(sum of negative terms) + log_norm   (-inf when none)
  float err;    // relative error bound on each sum
  float pad;
};

// Result of one acquisition on one device.  The first 24 bytes (index, score, rel, flags) are what a
// multi-GPU winner exchange needs.
struct AcqResult {
  int64_t index;     // winning candidate (global index), -1 when no finite score exists
  double score;      // its exact fp64 score max(1e-8, g) / max(l, 1e-8)
  float rel;         // bound of |score - score in numpy's arithmetic| / score (exp may differ by ulps)
  int32_t flags;     // HBX_ACQ_* bits
  int32_t shortlist; // candidates re-scored in fp64
  int32_t near;      // candidates whose score is within the bounds of the winner's (1: certified)
  double pdf_l;      // exact fp64 l(x) of the winner
  double pdf_g;      // exact fp64 g(x) of the winner
};
// flags: HBX_ACQ_OVERFLOW / HBX_ACQ_NEAR_TIE / HBX_ACQ_RESOLVED (include/hbx.h)

// Publish `words` 32-bit words of this thread (or, called by every lane, of this wave) to device-mapped
// coherent host memory, then the completion word the host polls.  The words go out as system-scope relaxed
// stores (coherent, not held in the L2), the wave waits until every one is acknowledged, then stores the
// completion word.  A system-scope fence would do the same ordering by writing back every dirty line of the
// L2 first -- whatever earlier kernels of the acquisition left there (config #3: ~8 MB of score bounds).
__device__ __forceinline__ void hbx_publish_store(uint32_t* dst, uint32_t v) {
  __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void hbx_publish_store64(uint64_t* dst, uint64_t v) {
  __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void hbx_publish_done(int32_t* done, int32_t seq) {
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// float <-> order-preserving uint32 (for atomicMin on floats of either sign)
__device__ __forceinline__ uint32_t hbx_f2ord(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float hbx_ord2f(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// double -> order-preserving uint64 with every NaN mapped past +inf; -0.0 and 0.0 map to one key
// (numpy's comparison sorts treat them as equal: ties, ranked by position)
__device__ __forceinline__ uint64_t hbx_d2ord(double d) {
  if (d != d) return ~0ull;
  if (d == 0.0) d = 0.0;
  uint64_t u = (uint64_t)__double_as_longlong(d);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

// Wave-wide reduction of a 32-bit value (DPP within rows of 16 lanes, then the four rows combined in
// scalar registers): every lane gets the result.
template <typename Op>
__device__ __forceinline__ uint32_t wave_reduce_dpp(uint32_t v, Op op) {
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false));   // quad_perm [1,0,3,2]
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false));   // quad_perm [2,3,0,1]
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false));  // row_half_mirror
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, false));  // row_mirror
  // every lane of a 16-lane row now holds the row's value: combine the four rows (scalar, uniform)
  return op(op((uint32_t)__builtin_amdgcn_readlane((int)v, 0), (uint32_t)__builtin_amdgcn_readlane((int)v, 16)),
            op((uint32_t)__builtin_amdgcn_readlane((int)v, 32), (uint32_t)__builtin_amdgcn_readlane((int)v, 48)));
}
struct OpAdd { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; } };
struct OpAnd { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a & b; } };
struct OpOr { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a | b; } };
struct OpMax { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; } };
