// hbx_logpdf.hip -- the north-star ln-pdf contract on MI355X (gfx950): ln pdf of one prepared KDE at Nc
// candidates within rtol * max(1, |ln p|) of the reference's KDEMultivariate.pdf (bohb.py:124-152 ->
// SM:kernel_density.py:162-196 -> SM:kernels.py:23-65,108-125), the entry point hbx_kde_logpdf_rtol.
//
//   kde_dd_stage       (SG path) the observation rows scaled to fp32, staged once for every block
//   kde_logpdf_dd      fp32 direct differences per pair, rigorous per-candidate bound; writes what the bound
//                      accepts, lists the rest (two instances per call: rows from SGPRs or from LDS)
//   kde_logpdf_classify  (signed / unbucketed KDEs) the same split over the MFMA scoring estimate
//   kde_logpdf_tiled   fp64 log-space evaluation of the listed candidates, rows staged in LDS
//   (hbx_kde.hip)      the per-point fp64 kernels for buckets without a tiled instance and for KDEs with
//                      negative categorical factors or structural NaN
// Split from hbx_kde.hip, whose acquisition engine shares the KDE parameter block and the scoring instances.
#include <math.h>
#include <stdlib.h>

#include "hbx_common.h"
#include "hbx_kde_impl.h"

// ln pdf within rtol * max(1, |ln p|) of the reference's (the north-star contract), per candidate: the
// fp32 estimate where its rigorous bound guarantees it, else queued for an fp64 evaluation
// ln pdf in fp64 log space, tiled: the same value as kde_logpdf_exact_kernel (per pair the direct
// differences -((x - X) / (h sqrt 2))^2 per continuous dim, ln(1 - h) or ln(h / (c - 1)) per categorical
// dim, SM:kernels.py:23-65 in log form), but one candidate per thread and the observations staged in LDS
// 64 at a time for the whole block -- each observation row is read once per 256 candidates, where the
// per-point kernel re-read every row for every candidate (2.6 TB of L2 traffic for 1e6 x 1e4 at D = 32).
// Per thread the pair terms go into a running logsumexp: the running maximum m and S = sum 2^(t' - m')
// (t' = t log2 e), each term 2^(t' - m') evaluated by v_exp_f32 on the fp32-rounded exponent.  Error of a
// term <= ln2 |t' - m'| 2^-24 + 2^-22 relative: below 3e-6 for the terms with |t' - m'| <= 60 and a
// contribution < 1e4 x 2^-60 for the rest, so |ln S_est - ln S| < 4e-6 -- inside rtol for rtol >= 1e-5
// (EXP64: fp64 exp2 for tighter rtol).  The sums, the maximum and the pair terms are fp64.
// DC / DU: continuous / categorical slots (the KDE's dims padded with zero terms); candidates list[0, *count)
// (or all Np), outputs at their own index.  Only for KDEs without negative categorical factors, structural
// NaN or single-level categorical dims (kde_pdf_exact_kernel takes those).
template <int DC, int DU, bool EXP64>
__global__ __launch_bounds__(256) void kde_logpdf_tiled_kernel(const double* __restrict__ pts, int64_t Np,
                                                              int32_t D, const KdeParams* __restrict__ P,
                                                              const double* __restrict__ X,
                                                              const int64_t* __restrict__ rows,
                                                              double* __restrict__ out,
                                                              const int32_t* __restrict__ list,
                                                              const int32_t* __restrict__ count) {
  constexpr int OB = 64;  // observations per staged chunk
  constexpr int DUS = DU > 0 ? DU : 1;
  __shared__ double xs_c[2][OB][DC];
  __shared__ double xs_u[2][OB][DUS];
  __shared__ double sa[DC], sdl[DUS];
  __shared__ int32_t scol[DC + DUS];
  __shared__ double lconst;
  const int n = P->n, dc = P->dc, du = P->du;
  const int64_t np = list ? (int64_t)*count : Np;
  const int64_t i0 = (int64_t)blockIdx.x * 256;
  if (i0 >= np) return;  // uniform
  const int tid = threadIdx.x;
  if (P->has_neg || P->nan_all || P->nconst) {  // kde_pdf_exact_kernel writes these (ln of the exact pdf)
    if (i0 + tid < np) out[list ? (int64_t)list[i0 + tid] : i0 + tid] = NAN;
    return;
  }
  // per-dim constants: a_c = 1 / (h sqrt 2) (finite: a zero bandwidth is nan_all); categorical: the term is
  // ln(h / (c - 1)) + [match] (ln(1 - h) - ln(h / (c - 1))), the first part summed into the constant
  if (tid < DC) {
    const bool act = tid < dc;
    const int d = act ? P->cont_dim[tid] : 0;
    sa[tid] = act ? 1.0 / (P->bw[d] * 1.4142135623730951) : 0.0;
    scol[tid] = d;
  }
  if (tid < DU) {
    const bool act = tid < du;
    const int d = act ? P->cat_dim[tid] : 0;
    const double h = act ? P->bw[d] : 0.0;
    sdl[tid] = act ? log(1. - h) - log(h / (double)(P->nlev[d] - 1)) : 0.0;
    scol[DC + tid] = d;
  }
  if (tid == 0) {
    double lc = -log((double)n);
    for (int k = 0; k < dc; ++k) lc -= log(P->bw[P->cont_dim[k]]) + 0.91893853320467274178;  // ln(h sqrt(2 pi))
    for (int k = 0; k < du; ++k) {
      const int d = P->cat_dim[k];
      lc += log(P->bw[d] / (double)(P->nlev[d] - 1));
    }
    lconst = lc;
  }
  __syncthreads();
  const int64_t pi = i0 + tid;
  const bool valid = pi < np;
  const int64_t p = valid ? (list ? (int64_t)list[pi] : pi) : 0;
  const double* x = pts + p * (int64_t)D;
  double xc[DC], xu[DUS];  // the candidate: scaled continuous coordinates, categorical codes
#pragma unroll
  for (int k = 0; k < DC; ++k) xc[k] = (k < dc && valid) ? x[scol[k]] * sa[k] : 0.0;
#pragma unroll
  for (int k = 0; k < DUS; ++k) xu[k] = (k < du && valid) ? x[scol[DC + k]] : 0.0;
  // stage chunk c into buffer b: scaled coordinates and codes of 64 observations (padding dims 0; an
  // observation past n gets an infinite first coordinate: its term is exp(-inf) = 0)
  auto stage = [&](int c, int b) {
    const int j0 = c * OB;
    for (int e = tid; e < OB * (DC + DU); e += 256) {
      const int jj = e / (DC + DU), k = e - jj * (DC + DU);
      const int j = j0 + jj;
      double v = 0.0;
      if (j < n) {
        if (k < DC) {
          if (k < dc) v = X[rows[j] * (int64_t)D + scol[k]] * sa[k];
        } else if (k - DC < du) {
          v = X[rows[j] * (int64_t)D + scol[k]];
        }
      } else if (k == 0) {
        v = __builtin_inf();
      }
      if (k < DC) xs_c[b][jj][k] = v;
      else xs_u[b][jj][k - DC] = v;
    }
  };
  const int nch = (n + OB - 1) / OB;
  double m = -INFINITY, S = 0.0;
  bool nan = false;
  stage(0, 0);
  for (int c = 0; c < nch; ++c) {
    __syncthreads();  // chunk c staged; every thread done with chunk c - 1's buffer
    if (c + 1 < nch) stage(c + 1, (c + 1) & 1);
    const int b = c & 1;
    const int jn = min(OB, n - c * OB);
    for (int jj = 0; jj < jn; ++jj) {
      double t = 0.0;
#pragma unroll
      for (int k = 0; k < DC; ++k) {
        const double d = xc[k] - xs_c[b][jj][k];
        t = fma(-d, d, t);
      }
#pragma unroll
      for (int k = 0; k < DU; ++k) t += (xu[k] == xs_u[b][jj][k]) ? sdl[k] : 0.0;
      const double tl = t * 1.4426950408889634;  // log2 units
      if (tl > m) {
        S = (m > -INFINITY ? S * (EXP64 ? exp2(m - tl) : (double)__builtin_amdgcn_exp2f((float)(m - tl))) : 0.0) + 1.0;
        m = tl;
      } else if (tl > -INFINITY) {
        S += EXP64 ? exp2(tl - m) : (double)__builtin_amdgcn_exp2f((float)(tl - m));
      } else if (tl != tl) {
        nan = true;
      }
    }
  }
  if (valid)
    out[p] = nan ? NAN : (m > -INFINITY ? (m + log2(S)) * 0.69314718055994531 + lconst : -INFINITY);
}

// ln pdf within rtol by DIRECT DIFFERENCES in fp32 (the ln-pdf contract's first pass, hbx_kde_logpdf_rtol):
// per pair t' = -sum_k (x'_k - X'_jk)^2 + sum_u delta_u [x_u == X_ju] (log2 units, x' = s (x - mu) as the
// scoring kernels scale it, s = sqrt(log2 e / 2) / h; SM:kernels.py:23-65,108-125 in log2 form), S' =
// sum_j 2^(t'_j - m) (m: the largest exponent of the first chunk, raised when a group of terms would
// overflow), ln p = ln2 (m + log2 S' + lb_sum - M0) + log_norm.  No expansion -|x'|^2 - |X'|^2 + 2 x'X': its
// terms of ~100 log2 units cancel, and a bound relative to them (the matrix-core estimates') never reaches
// 1e-5 at D = 32; here every rounding is relative to the pair's own distance.  Packed fp32 VALU: the
// differences and their squares two dims per v_pk_add_f32 / v_pk_fma_f32, the categorical match as
// clamp(1 - e^2) of the integer code difference e (v_pk_fma_f32 ... clamp) times delta; observations staged
// in LDS 64 at a time and read as broadcasts; CPT candidates per thread share each read.
// Rigorous per-candidate bound of |ln p_est - ln p| (log2 units first):
//   coordinates: x', X' rounded to fp32, d = fl(x' - X'): |d~ - d| <= dl_k = 2^-23 (1 + 2^-20)(|x'_k| + xmax_k);
//   squares: |d~^2 - d^2| summed <= 2 sqrt(Q) |dl| + |dl|^2 over the terms that matter (t' >= t'_max - 64,
//     Q = -m + 64 + sum_u max(delta_u, 0) + slack bounds their sum_k d_k^2; the others add <= n 2^-63);
//   the accumulation: chains of NCH fma / add steps, each rounding <= 2^-24 (Q + sum|delta|);
//   delta_u in fp32: <= 2^-24 sum|delta|; the exponent t' - m: 2^-24 (64 + 1);
//   exp2: v_exp_f32 within 2 ulp (2^-22 relative); sums: (DD_G - 1) 2^-24 (fp32 groups) + n 2^-52 (fp64).
// Candidates whose bound stays within 0.99 rtol max(1, |ln p|) are written; the rest go to `list` for the
// fp64 pass.  KDEs with negative categorical factors, structural NaN or single-level dims: all to `list`.
// LUT (variant bit 8: <= 8 categorical slots, codes in [0, 3]): the categorical part of a pair is two table
// reads instead of 1.5 packed instructions per dim -- the candidate's and the observation's codes packed as
// two-bit fields (dims 0-3 at bits 2..9, dims 4-7 at bits 12..19), their xor's two 8-bit field groups index
// 256-entry LDS tables whose entry is sum_u delta_u [field u == 0] (summed in fp64, rounded once: within
// 2^-24 sum|delta|, the bound's delta term); a candidate whose code is not an integer in [0, 3] goes to `list`.
#ifndef DD_WPE
#define DD_WPE(w) ((w) <= 16 ? 4 : (w) <= 40 ? 3 : 2)  // waves per SIMD the register budget is sized for
#endif
// SG (scalar-staged rows): the observation rows are staged ONCE per call into global memory by
// kde_dd_stage_kernel (the same fp32 values the LDS staging computes, padded with +inf rows to a multiple of
// DD_G) and read by each wave through the scalar cache into SGPRs, which the packed VALU instructions take as
// operands: no per-block staging, no barrier per chunk, and no LDS broadcast reads (4 LDS cycles per
// ds_read_b128) competing with the table reads.  `sg_flag` (scratch header): the stage kernel sets it when the
// table fit the scratch; the SG kernel runs only then, the LDS kernel of the same call only otherwise.
#ifndef DD_G
#define DD_G 4  // terms per fp32 group (its sum's rounding: (DD_G - 1) 2^-24 in the bound)
#endif
#ifndef DD_WPE_SG
#define DD_WPE_SG 4  // the SG kernel: its rows live in SGPRs, so more waves fit
#endif
template <int DC, int DU, int CPT, bool LUT = false, bool SG = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SG ? DD_WPE_SG : DD_WPE(DC + DU)))) void kde_logpdf_dd_kernel(const double* __restrict__ pts, int64_t Np, int32_t D,
                                                           const KdeParams* __restrict__ P,
                                                           const double* __restrict__ X,
                                                           const int64_t* __restrict__ rows, double rtol,
                                                           double* __restrict__ out, int32_t* __restrict__ list,
                                                           int32_t* __restrict__ count,
                                                           const float* __restrict__ stg,
                                                           const int32_t* __restrict__ sg_flag) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  constexpr int OB = 64;      // observations per staged chunk
  constexpr int G = DD_G;
  static_assert(OB % G == 0, "groups within a chunk");
  // floats per staged row: DC scaled coordinates, then DU codes (LUT: the packed code word and 3 pad slots)
  constexpr int W = LUT ? DC + 4 : DC + DU;
  static_assert(!SG || W <= 32, "SG: a row in at most 32 SGPRs");
  if (sg_flag && ((*sg_flag != 0) != SG)) return;  // uniform: the other kernel of the call runs
  constexpr int WC = LUT ? DC : W;  // staged elements per row written by the element loop
  constexpr int NB = DC / 2, NU = DU / 2;  // packed pairs
  static_assert(DC % 4 == 0 && DU % 4 == 0, "pairs of pairs");
  static_assert(!LUT || DU == 4 || DU == 8, "LUT: 4 or 8 categorical slots");
  __shared__ __align__(16) float xs[SG ? 1 : 2][SG ? 1 : OB][W];
  __shared__ double s_scale[DC > 0 ? DC : 1], s_mu[DC > 0 ? DC : 1];
  __shared__ int32_t s_col[DC + DU > 0 ? DC + DU : 1];
  __shared__ float s_dl[DU > 0 ? DU : 1];
  __shared__ float s_lut[LUT ? 512 : 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int n = P->n, dc = P->dc, du = P->du;
  const int64_t i0 = (int64_t)blockIdx.x * 256 * CPT;
  if (i0 >= Np) return;  // uniform
  int64_t cid[CPT];
  bool valid[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    cid[c] = i0 + c * 256 + tid;
    valid[c] = cid[c] < Np;
  }
  const bool unsupported = P->has_neg || P->nan_all || P->nconst || n <= 0;
  auto to_list = [&](bool f, int64_t p) __attribute__((always_inline)) {  // one atomic per wave
    const uint64_t bal = __ballot(f);
    if (!bal) return;
    int32_t base = 0;
    if (lane == __ffsll((long long)bal) - 1) base = atomicAdd(count, __popcll(bal));
    base = __shfl(base, __ffsll((long long)bal) - 1);
    if (f) list[base + __popcll(bal & ((1ull << lane) - 1ull))] = (int32_t)p;
  };
  if (unsupported) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) to_list(valid[c], cid[c]);
    return;
  }
  for (int k = tid; k < DC + DU; k += 256) {
    if (k < DC) {
      const bool act = k < dc;
      s_scale[k] = act ? P->cont_scale[k] : 0.0;
      s_mu[k] = act ? P->center[k] : 0.0;
      s_col[k] = act ? P->cont_dim[k] : -1;
    } else {
      const int u = k - DC;
      const bool act = u < du;
      s_dl[u] = act ? P->cat_delta[u] : 0.f;
      s_col[k] = act ? P->cat_dim[u] : -1;
    }
  }
  __syncthreads();
  if constexpr (LUT) {  // table k, entry i: the deltas of the dims 4k..4k+3 whose two-bit field of i is 0
#pragma unroll
    for (int k = 0; k < DU / 4; ++k) {
      double v = 0.0;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (((tid >> (2 * u)) & 3) == 0) v += (double)s_dl[4 * k + u];
      s_lut[256 * k + tid] = (float)v;
    }
  }
  // the candidates: scaled continuous coordinates and codes in registers, pairs of dims packed
  f2 xc[CPT][NB > 0 ? NB : 1], xu[CPT][(NU > 0 && !LUT) ? NU : 1];
  uint32_t cw[CPT], cw1[CPT];  // LUT: the candidate's packed codes; dims 4-7's field group alone
  bool cbad[CPT];    // LUT: a code outside [0, 3] (or not an integer): the candidate goes to the fp64 pass
  float nx2[CPT];  // sum_k (|x'_k| + xmax_k)^2
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const double* x = pts + (valid[c] ? cid[c] : 0) * (int64_t)D;
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      float v[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = 2 * q + h;
        v[h] = s_col[k] >= 0 ? (float)(s_scale[k] * (x[s_col[k]] - s_mu[k])) : 0.f;
        const float a = fabsf(v[h]) + (k < dc ? P->xmax[k] : 0.f);
        acc = fmaf(a, a, acc);
      }
      xc[c][q] = f2{v[0], v[1]};
    }
    cw[c] = cw1[c] = 0u;
    cbad[c] = false;
    if constexpr (LUT) {
#pragma unroll
      for (int u = 0; u < DU; ++u) {
        const int k = DC + u;
        const double v = s_col[k] >= 0 ? x[s_col[k]] : 0.0;
        const bool ok = v == rint(v) && v >= 0.0 && v <= 3.0;
        cbad[c] = cbad[c] || !ok;
        cw[c] |= (ok ? (uint32_t)v : 0u) << (u < 4 ? 2 + 2 * u : 12 + 2 * (u - 4));
      }
      cw1[c] = (cw[c] >> 10) & 0x3FFu;
    } else {
#pragma unroll
      for (int q = 0; q < NU; ++q) {
        float v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int k = DC + 2 * q + h;
          v[h] = s_col[k] >= 0 ? cand_code(x[s_col[k]]) : 0.f;
        }
        xu[c][q] = f2{v[0], v[1]};
      }
    }
    nx2[c] = acc;
  }
  f2 dl2[(NU > 0 && !LUT) ? NU : 1];
  if constexpr (!LUT) {
#pragma unroll
    for (int q = 0; q < NU; ++q) dl2[q] = f2{s_dl[2 * q], s_dl[2 * q + 1]};
  }
  // stage chunk cc into buffer b (padding dims 0 -- codes 0 against the candidate's 0: a match of delta 0;
  // an observation past n: first coordinate +inf, its term 2^-inf = 0)
  // the loads of a chunk are issued into registers before the previous chunk's math and stored after it
  constexpr int PER = (OB * WC + 255) / 256;
  double pre[PER];
  uint32_t prc[LUT ? DU : 1];  // LUT, threads < OB: row tid's codes (the high words of the f64 values)
  auto fetch = [&](int cc) __attribute__((always_inline)) {
    const int j0 = cc * OB;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = tid + 256 * q;
      const int jj = e / WC, k = e - jj * WC;
      const int j = j0 + jj;
      pre[q] = (e < OB * WC && j < n && s_col[k] >= 0) ? X[rows[j] * (int64_t)D + s_col[k]] : 0.0;
    }
    if constexpr (LUT) {
      const int j = j0 + tid;
#pragma unroll
      for (int u = 0; u < DU; ++u) {
        const int k = DC + u;
        prc[u] = (tid < OB && j < n && s_col[k] >= 0)
                     ? reinterpret_cast<const uint32_t*>(X + rows[j] * (int64_t)D + s_col[k])[1] : 0u;
      }
    }
  };
  auto store = [&](int cc, int b) __attribute__((always_inline)) {
    const int j0 = cc * OB;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = tid + 256 * q;
      if (e >= OB * WC) break;
      const int jj = e / WC, k = e - jj * WC;
      float v = 0.f;
      if (j0 + jj < n) {
        if (s_col[k] >= 0) v = k < DC ? (float)(s_scale[k] * (pre[q] - s_mu[k])) : cand_code(pre[q]);
      } else if (k == 0) {
        v = __builtin_inf();
      }
      xs[b][jj][k] = v;
    }
    if constexpr (LUT) {
      if (tid < OB) {  // the codes are integers in [0, 3] (variant bit 8): exact from the f64 high word
        uint32_t w = 0u;
#pragma unroll
        for (int u = 0; u < DU; ++u)
          w |= (uint32_t)__hiloint2double((int)prc[u], 0) << (u < 4 ? 2 + 2 * u : 12 + 2 * (u - 4));
        xs[b][tid][DC] = __uint_as_float(w);
        xs[b][tid][DC + 1] = __uint_as_float((w >> 10) & 0x3FFu);  // dims 4-7's group alone: one xor per pair
        xs[b][tid][DC + 2] = xs[b][tid][DC + 3] = 0.f;
      }
    }
  };
  auto stage = [&](int cc, int b) __attribute__((always_inline)) {
    fetch(cc);
    store(cc, b);
  };
  // exponents t' of the pairs (every candidate c of the thread, staged row r) into t[c]: two packed accumulators
  // per candidate (four fma chains), the candidates' steps interleaved so consecutive packed instructions are
  // independent (each chain's order is that of one candidate alone)
  auto terms = [&](const float* r, float (&t)[CPT]) __attribute__((always_inline)) {
    f2 a0[CPT], a1[CPT];
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      a0[c] = f2{0.f, 0.f};
      a1[c] = f2{0.f, 0.f};
      if constexpr (LUT) {  // the categorical part: two table reads of the codes' xor
        const uint32_t x0 = (cw[c] ^ __float_as_uint(r[DC])) & 0x3FFu;  // (one v_bitop3)
        const float l0 = *(const float*)((const char*)s_lut + x0);
        const float l1 =
            DU > 4 ? *(const float*)((const char*)s_lut + 1024 + (cw1[c] ^ __float_as_uint(r[DC + 1]))) : 0.f;
        a0[c] = f2{l0, l1};
      }
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const f2 X2 = f2{r[2 * q], r[2 * q + 1]};
      f2 d[CPT];
#pragma unroll
      for (int c = 0; c < CPT; ++c) d[c] = xc[c][q] - X2;
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        if (q < NB / 2) a0[c] = __builtin_elementwise_fma(-d[c], d[c], a0[c]);
        else a1[c] = __builtin_elementwise_fma(-d[c], d[c], a1[c]);
      }
    }
#pragma unroll
    for (int q = 0; q < (LUT ? 0 : NU); ++q) {
      const f2 E2 = f2{r[DC + 2 * q], r[DC + 2 * q + 1]};
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        const f2 e = xu[c][q] - E2;
        f2 m;  // [x_u == X_u] = clamp(1 - e^2) for integer code differences e
        asm("v_pk_fma_f32 %0, %1, %2, 1.0 op_sel_hi:[1,1,0] neg_lo:[1,0,0] neg_hi:[1,0,0] clamp" : "=v"(m) : "v"(e), "v"(e));
        if (q < NU / 2) a0[c] = __builtin_elementwise_fma(dl2[q], m, a0[c]);
        else a1[c] = __builtin_elementwise_fma(dl2[q], m, a1[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const f2 a = a0[c] + a1[c];
      t[c] = a.x + a.y;
    }
  };
  const int nch = (n + OB - 1) / OB;
  if constexpr (!SG) {
    stage(0, 0);
    __syncthreads();
  }
  // m: the largest exponent of chunk 0 (every candidate's sum then has a term 2^0)
  float m[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) m[c] = -INFINITY;
  const int jn0 = min(OB, n);
  for (int jj = 0; jj < jn0; ++jj) {
    const float* r0 = SG ? stg + (int64_t)jj * W : &xs[0][SG ? 0 : jj][0];
    float t[CPT];
    terms(r0, t);
#pragma unroll
    for (int c = 0; c < CPT; ++c) m[c] = fmaxf(m[c], t[c]);
  }
  double S[CPT];
  float s4[CPT];
  bool ref0[CPT];  // chunk 0 had a finite term: the bound's reference point (S' >= 1/2) holds
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    S[c] = 0.0;
    s4[c] = 0.f;
    // an integer reference point (rescales are exact ldexps); no finite term in chunk 0 (or NaN): m = 0, and
    // the candidate goes to the fp64 pass (the bound assumes a term at or above m - 1)
    ref0[c] = m[c] > -INFINITY;
    m[c] = ref0[c] ? ceilf(m[c]) : 0.f;
  }
  // one group of G rows (rowp(q, r): row q of the group into r): terms summed in fp32, the group into the fp64
  // sums (a chunk's last group: rows past n are the padding rows, whose first coordinate is +inf: exact zeros)
  auto group = [&](auto rowp) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < G; ++q) {
      float r[W], t[CPT];
      rowp(q, r);
      terms(r, t);
#pragma unroll
      for (int c = 0; c < CPT; ++c) s4[c] += __builtin_amdgcn_exp2f(t[c] - m[c]);
    }
    // rare: a term far above the reference point, or NaN (one test per candidate and group): the reference
    // point moves up to ceil of the group's largest exponent (an integer: the rescale is an exact ldexp) and the
    // group is summed again (a wave-uniform branch; the lanes that need it)
    bool redo[CPT];
    bool any = false;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      redo[c] = !(s4[c] < 0x1p100f);
      any = any || redo[c];
    }
    if (__builtin_expect(__ballot(any) != 0, 0)) {
      float tmx[CPT];  // the group's largest exponent per candidate (NaN terms left out)
#pragma unroll
      for (int c = 0; c < CPT; ++c) tmx[c] = -INFINITY;
      for (int q = 0; q < G; ++q) {
        float r[W], t[CPT];
        rowp(q, r);
        terms(r, t);
#pragma unroll
        for (int c = 0; c < CPT; ++c) tmx[c] = fmaxf(tmx[c], t[c]);
      }
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        const float mn = ceilf(tmx[c]);
        if (redo[c] && mn > m[c]) {
          S[c] = ldexp(S[c], (int)(m[c] - mn));
          m[c] = mn;
        }
        if (redo[c]) s4[c] = 0.f;
      }
      for (int q = 0; q < G; ++q) {
        float r[W], t[CPT];
        rowp(q, r);
        terms(r, t);
#pragma unroll
        for (int c = 0; c < CPT; ++c) {
          const float e = __builtin_amdgcn_exp2f(t[c] - m[c]);
          if (redo[c]) s4[c] += e;
        }
      }
    }
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      S[c] += (double)s4[c];
      s4[c] = 0.f;
    }
  };
  if constexpr (SG) {
    const int ngr = (n + G - 1) / G;
    for (int g = 0; g < ngr; ++g) {
      const float* base = stg + (int64_t)g * (G * W);  // uniform: scalar loads
      group([&](int q, float (&r)[W]) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < W; ++k) r[k] = base[q * W + k];
      });
    }
  } else {
    for (int cc = 0; cc < nch; ++cc) {
      const int b = cc & 1;
      if (cc + 1 < nch) fetch(cc + 1);
      const int jn = min(OB, n - cc * OB);
      const int jg = (jn + G - 1) & ~(G - 1);
      for (int j4 = 0; j4 < jg; j4 += G) {
        group([&](int q, float (&r)[W]) __attribute__((always_inline)) {  // 16-byte vectors (ds_read_b128)
#pragma unroll
          for (int v = 0; v < W / 4; ++v) {
            const float4 f = reinterpret_cast<const float4*>(&xs[SG ? 0 : b][SG ? 0 : j4 + q][0])[v];
            r[4 * v] = f.x;
            r[4 * v + 1] = f.y;
            r[4 * v + 2] = f.z;
            r[4 * v + 3] = f.w;
          }
        });
      }
      // the other buffer is free since the barrier after chunk cc - 1
      if (cc + 1 < nch) store(cc + 1, b ^ 1);
      __syncthreads();  // chunk cc + 1 staged; every thread done with chunk cc's buffer
    }
  }
  // the bound (log2 units) and the result
  float sdp = 0.f, sda = 0.f;
  for (int u = 0; u < du; ++u) {
    const float dlt = s_dl[u];
    if (dlt > -1e29f) {  // a 1 - h == 0 factor's match: 2^-inf, no rounding
      sdp += fmaxf(dlt, 0.f);
      sda += fabsf(dlt);
    }
  }
  const double log_c = P->lb_sum - P->m0_log2;
  const float u24 = 0x1p-24f;
  constexpr int NCH = (NB + NU) / 2 + 3;  // fma / add steps per chain, with the combining adds
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const float Q = fmaxf(-m[c], 0.f) + 64.f + sdp + 1.f;
    const float dln = 0x1p-23f * (1.f + 0x1p-20f) * __builtin_sqrtf(nx2[c]) * (1.f + 0x1p-20f);
    const float Et = 2.f * __builtin_sqrtf(Q) * dln + dln * dln + (float)NCH * u24 * (Q + sda) + u24 * sda +
                     65.f * u24 + 0x1p-48f * Q;
    // relative bound of S': 2^Et - 1 per term, the exp, the sums, the terms left out
    const double rel = exp2((double)Et * (1.0 + 0x1p-20)) - 1.0 + 0x1p-22 + (G - 1) * 0x1p-24 + (double)n * 0x1p-52 +
                       (double)n * 0x1p-63;
    const double lnS = log(S[c]) + (double)m[c] * 0.69314718055994531;
    const double lp = lnS + log_c * 0.69314718055994531 + P->log_norm;
    const double bound = rel / (1.0 - rel) + 0x1p-50 * fabs(lp);
    const bool ok = valid[c] && ref0[c] && !cbad[c] && S[c] > 0.0 && lp - lp == 0.0 && rel < 0.5 && bound <= 0.99 * rtol * fmax(1.0, fabs(lp));
    if (ok) out[cid[c]] = lp;
    to_list(valid[c] && !ok, cid[c]);
  }
}

typedef void (*logpdf_dd_fn)(const double*, int64_t, int32_t, const KdeParams*, const double*, const int64_t*, double,
                             double*, int32_t*, int32_t*, const float*, const int32_t*);
typedef void (*dd_stage_fn)(const KdeParams*, const double*, const int64_t*, int32_t, int64_t, float*, int32_t*);

// the SG kernel's staged rows: row j < n as kde_logpdf_dd_kernel's LDS staging writes it (the DC scaled
// coordinates in fp32; LUT: the packed two-bit code word, its dims 4-7 group alone, two zeros; else the DU codes),
// rows n .. n_pad - 1 padding (first coordinate +inf, the rest 0).  Writes only when n_pad W floats fit `cap`
// bytes, and sets *sg_flag to say so (read by both dd kernels of the call); grid-stride (n is on the device).
template <int DC, int DU, bool LUT>
__global__ __launch_bounds__(256) void kde_dd_stage_kernel(const KdeParams* __restrict__ P, const double* __restrict__ X,
                                                           const int64_t* __restrict__ rows, int32_t D, int64_t cap,
                                                           float* __restrict__ stg, int32_t* __restrict__ sg_flag) {
  constexpr int W = LUT ? DC + 4 : DC + DU;
  const int n = P->n, dc = P->dc, du = P->du;
  const int64_t n_pad = ((int64_t)n + DD_G - 1) / DD_G * DD_G;
  const bool fits = n > 0 && n_pad * W * 4 <= cap && !(P->has_neg || P->nan_all || P->nconst);
  if (blockIdx.x == 0 && threadIdx.x == 0) *sg_flag = fits ? 1 : 0;
  if (!fits) return;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n_pad * W; e += (int64_t)gridDim.x * 256) {
    const int j = (int)(e / W), k = (int)(e - (int64_t)j * W);
    float v = 0.f;
    if (j < n) {
      const double* x = X + rows[j] * (int64_t)D;
      if (k < DC) {
        if (k < dc) v = (float)(P->cont_scale[k] * (x[P->cont_dim[k]] - P->center[k]));
      } else if constexpr (LUT) {
        if (k < DC + 2) {  // codes are integers in [0, 3] (variant bit 8)
          uint32_t w = 0u;
#pragma unroll
          for (int u = 0; u < DU; ++u)
            if (u < du) w |= (uint32_t)x[P->cat_dim[u]] << (u < 4 ? 2 + 2 * u : 12 + 2 * (u - 4));
          v = __uint_as_float(k == DC ? w : (w >> 10) & 0x3FFu);
        }
      } else {
        const int u = k - DC;
        if (u < du) v = cand_code(x[P->cat_dim[u]]);
      }
    } else if (k == 0) {
      v = __builtin_inf();
    }
    stg[e] = v;
  }
}

// candidates per thread: two share each staged row where both fit the register budget
#ifndef DD_CPT
#define DD_CPT 2
#endif
constexpr int dd_cpt(int dc, int du) { return DD_CPT; }
#ifndef DD_CPT_LUT
#define DD_CPT_LUT 2
#endif

struct DdFns {
  logpdf_dd_fn lds = nullptr, sg = nullptr;
  dd_stage_fn stage = nullptr;
};
template <int DC, int DU, int CPT, bool LUT>
static DdFns dd_fns() {
  DdFns f;
  f.lds = kde_logpdf_dd_kernel<DC, DU, CPT, LUT>;
  if constexpr ((LUT ? DC + 4 : DC + DU) <= 32) {
    f.sg = kde_logpdf_dd_kernel<DC, DU, CPT, LUT, true>;
    f.stage = kde_dd_stage_kernel<DC, DU, LUT>;
  }
  return f;
}

template <int DC>
static DdFns pick_dd_du(int du_pad, int* cpt, bool lut) {
  if (lut && du_pad == 4) {
    *cpt = DD_CPT_LUT;
    return dd_fns<DC, 4, DD_CPT_LUT, true>();
  }
  if (lut && du_pad == 8) {
    *cpt = DD_CPT_LUT;
    return dd_fns<DC, 8, DD_CPT_LUT, true>();
  }
  switch (du_pad) {
    case 0: *cpt = dd_cpt(DC, 0); return dd_fns<DC, 0, dd_cpt(DC, 0), false>();
    case 4: *cpt = dd_cpt(DC, 4); return dd_fns<DC, 4, dd_cpt(DC, 4), false>();
    case 8: *cpt = dd_cpt(DC, 8); return dd_fns<DC, 8, dd_cpt(DC, 8), false>();
    case 16: *cpt = dd_cpt(DC, 16); return dd_fns<DC, 16, dd_cpt(DC, 16), false>();
    case 32: *cpt = dd_cpt(DC, 32); return dd_fns<DC, 32, dd_cpt(DC, 32), false>();
  }
  return DdFns{};
}

static DdFns pick_logpdf_dd(int dc_pad, int du_pad, int* cpt, bool lut) {
  switch (dc_pad) {
    case 0:
    case 4: return pick_dd_du<4>(du_pad, cpt, lut);
    case 8: return pick_dd_du<8>(du_pad, cpt, lut);
    case 16: return pick_dd_du<16>(du_pad, cpt, lut);
    case 24: return pick_dd_du<24>(du_pad, cpt, lut);
    case 32: return pick_dd_du<32>(du_pad, cpt, lut);
  }
  return DdFns{};  // 64 continuous slots: the estimate + fp64 path
}

__global__ __launch_bounds__(256) void kde_logpdf_classify_kernel(const KdeEst* __restrict__ est, int64_t Nc,
                                                                 double rtol, int exact_all, double* __restrict__ out,
                                                                 int32_t* __restrict__ list,
                                                                 int32_t* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= Nc) return;
  bool ok = false;
  if (!exact_all) {
    const KdeEst e = est[i];
    const double lp = e.lpos, ln = e.lneg, er = e.err;
    const double m = fmax(lp, ln);
    const double a = exp(lp - m), b = exp(ln - m), S = a - b;
    const double pt = S > 0.0 ? m + log(S) : -INFINITY;
    const double rel = er * (a + b) / S;  // relative bound of the sum: |ln S_est - ln S| <= -ln(1 - rel)
    const double bound = -log1p(-fmin(rel, 0.5)) + 4e-7 * fmax(1.0, fabs(m));  // + fp32 rounding of the logs
    ok = pt - pt == 0.0 && er >= 0.0 && rel < 0.5 && bound <= 0.5 * rtol * fmax(1.0, fabs(pt));
    if (ok) out[i] = pt;
  }
  if (!ok) list[atomicAdd(count, 1)] = (int32_t)i;
}

typedef void (*logpdf_tiled_fn)(const double*, int64_t, int32_t, const KdeParams*, const double*, const int64_t*,
                                double*, const int32_t*, const int32_t*);

template <int DC, bool E64>
static logpdf_tiled_fn pick_tiled_du(int du_pad) {
  switch (du_pad) {
    case 0: return kde_logpdf_tiled_kernel<DC, 0, E64>;
    case 4:
    case 8: return kde_logpdf_tiled_kernel<DC, 8, E64>;
    case 16: return kde_logpdf_tiled_kernel<DC, 16, E64>;
    case 32: return kde_logpdf_tiled_kernel<DC, 32, E64>;
  }
  return nullptr;
}

template <bool E64>
static logpdf_tiled_fn pick_tiled_e(int dc_pad, int du_pad) {
  switch (dc_pad) {
    case 0:
    case 4:
    case 8: return pick_tiled_du<8, E64>(du_pad);
    case 16: return pick_tiled_du<16, E64>(du_pad);
    case 24: return pick_tiled_du<24, E64>(du_pad);
    case 32: return pick_tiled_du<32, E64>(du_pad);
  }
  return nullptr;  // 64 continuous slots: the per-point kernel
}

// the tiled fp64 log-space kernel of a bucket (dc_pad, du_pad), fp64 exponentials for rtol < 1e-5
static logpdf_tiled_fn pick_logpdf_tiled(int dc_pad, int du_pad, bool exp64) {
  return exp64 ? pick_tiled_e<true>(dc_pad, du_pad) : pick_tiled_e<false>(dc_pad, du_pad);
}

extern "C" {

int64_t hbx_kde_logpdf_rtol_scratch_bytes(int64_t Nc) { return 16 * Nc + 4 * Nc + 256; }

int hbx_kde_logpdf_rtol(const double* cand, int64_t Nc, int32_t D, const void* params, const float* table,
                        const double* X, const int64_t* rows, int32_t dc_pad, int32_t du_pad, int32_t variant,
                        double rtol, double* out, void* scratch, int64_t scratch_bytes, void* stream) {
  if ((!cand || !out) && Nc > 0) return hbx_fail(HBX_ERR_ARG, "hbx_kde_logpdf_rtol: null pointer");
  if (!params || !X || !rows || !scratch) return hbx_fail(HBX_ERR_ARG, "hbx_kde_logpdf_rtol: null pointer");
  if (D < 1 || D > HBX_MAX_D) return hbx_fail(HBX_ERR_ARG, "hbx_kde_logpdf_rtol: D=%d", D);
  if (!(rtol > 0.0)) return hbx_fail(HBX_ERR_ARG, "hbx_kde_logpdf_rtol: rtol %g", rtol);
  if (scratch_bytes < hbx_kde_logpdf_rtol_scratch_bytes(Nc)) return hbx_fail(HBX_ERR_ARG, "logpdf scratch too small");
  if (Nc <= 0) return HBX_OK;
  hipStream_t s = (hipStream_t)stream;
  char* sc = (char*)scratch;
  int32_t* count = (int32_t*)sc;
  KdeEst* est = (KdeEst*)(sc + 256);
  int32_t* list = (int32_t*)(sc + 256 + 16 * Nc);
  const bool exact_only = (variant >> 5) & 1;
  // unsigned KDEs of a bucket with <= 32 continuous slots: the direct-difference fp32 pass writes every
  // candidate its bound accepts and lists the rest (its kernel lists all of a KDE it does not model)
  int cpt = 1;
  const char* lut_env = getenv("HBX_DD_LUT");  // 0: the packed-match categorical path everywhere (tests)
  const bool lut = ((variant >> 8) & 1) && !(lut_env && atoi(lut_env) == 0);
  const DdFns dd = (!exact_only && !(variant & 1)) ? pick_logpdf_dd(dc_pad, du_pad, &cpt, lut) : DdFns{};
  const char* sg_env = getenv("HBX_DD_SG");  // 0: the LDS-staged dd kernel everywhere (tests)
  // (small calls: the LDS-staged kernel alone -- the staging launch and a second dd launch would cost more than
  // the SG kernel saves, and the scratch of a few thousand candidates rarely holds the rows)
  const bool sg = dd.sg && Nc >= 8192 && !(sg_env && atoi(sg_env) == 0);
  HBX_HIP(hipMemsetAsync(count, 0, sizeof(int32_t), s));
  if (dd.lds) {
    const dim3 g((unsigned)((Nc + 256 * cpt - 1) / (256 * cpt)));
    int32_t* flag = sg ? count + 1 : nullptr;
    if (sg) {  // rows staged into the (unused here) estimate area when they fit; the flag picks the kernel
      hipLaunchKernelGGL(dd.stage, dim3(256), dim3(256), 0, s, (const KdeParams*)params, X, rows, D, 16 * Nc,
                         (float*)est, flag);
      HBX_LAUNCH_CHECK();
      hipLaunchKernelGGL(dd.sg, g, dim3(256), 0, s, cand, Nc, D, (const KdeParams*)params, X, rows, rtol, out, list,
                         count, (const float*)est, (const int32_t*)flag);
      HBX_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(dd.lds, g, dim3(256), 0, s, cand, Nc, D, (const KdeParams*)params, X, rows, rtol, out, list,
                       count, (const float*)nullptr, (const int32_t*)flag);
    HBX_LAUNCH_CHECK();
  } else {
    if (!exact_only) {  // the estimate (the precise instance: hbx_kde_logpdf's)
      if (!table) return hbx_fail(HBX_ERR_ARG, "hbx_kde_logpdf_rtol: null table");
      const int rc = hbx_logpdf_estimate(cand, Nc, D, params, table, dc_pad, du_pad, variant, est, s);
      if (rc) return rc;
    }
    hipLaunchKernelGGL(kde_logpdf_classify_kernel, dim3((unsigned)((Nc + 255) / 256)), dim3(256), 0, s, est, Nc, rtol,
                       exact_only ? 1 : 0, out, list, count);
    HBX_LAUNCH_CHECK();
  }
  // the rest in fp64 log space (positive factors): tiled over candidates where the bucket has an instance,
  // else one block per point (its kernel exits for KDEs the tiled one would mis-handle: see below) ...
  const logpdf_tiled_fn tf = exact_only ? nullptr : pick_logpdf_tiled(dc_pad, du_pad, rtol < 1e-5);
  if (tf) {
    hipLaunchKernelGGL(tf, dim3((unsigned)((Nc + 255) / 256)), dim3(256), 0, s, cand, Nc, D, (const KdeParams*)params,
                       X, rows, out, list, count);
    HBX_LAUNCH_CHECK();
  }
  // ... or ln of the exact pdf (negative categorical factors, structural NaN: every block exits otherwise)
  return hbx_logpdf_exact_listed(cand, Nc, D, (const KdeParams*)params, X, rows, out, list, count, !tf, s);
}

}  // extern "C"
