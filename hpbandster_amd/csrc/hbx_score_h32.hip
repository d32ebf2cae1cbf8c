// hbx_score_h32.hip -- hmode scoring on 32x32 matrix tiles (unsigned sums).
//
// Same exponent as kde_logpdf_h_kernel (hbx_score_h.hip): continuous hi/lo products, C_j as three f16
// pieces against A = 1, c_i as the accumulator input, the one-hot product on the sparse matrix cores
// -- but on v_mfma_f32_32x32x16_f16 / v_smfmac_f32_32x32x32_f16.  Why: the kernel is bound by the
// SIMD's vector ISSUE port, not by the matrix pipe.  Per 256 pairs the 16x16x32 form spends 4 MFMAs
// x 8 issue cycles + 4 v_exp_f32 x 8 + 4 v_add_f32 x 4 = 80 cycles against 64 cycles of matrix pipe;
// a 32x32x16 MFMA holds the issue port for 8 of its 32 cycles, so the same work costs 16 + 32 + 16 = 64
// issue cycles: the exp2/sum epilogue of one tile fits in the gaps of the next tile's 8 MFMAs.
// The sparse form also takes any number of one-hot steps (K = 32 per instruction).
//
// Operand layouts (gfx950, established by tools/mfma32_probe.hip, profiles/r01/mfma32_probe.txt):
//   A (dense): lane l holds row l%32, K = 8(l/32) + 0..7;  B: K = 8(l/32) + 0..7 of column l%32;
//   D: register r of lane l = row 8(r/4) + 4(l/32) + r%4, column l%32;
//   sparse A: lane l covers row l%32, dense K [16(l/32), +16) as four 2-of-4 groups (index nibbles);
//   sparse B: lane half h holds K = 8h..8h+7 and 16+8h..16+8h+7 of column l%32.
// Table layout: the hmode chunk of hbx_kde_impl.h, unchanged (rows are K-contiguous, so a lane half's
// 8 halves of a dense 16-step are one ds_read_b128).
//
// Pipeline per 64-observation chunk c (two 32-observation tiles T0, T1), one basic block:
//   LDS-DMA of chunk c+2 | MFMAs of T1(c) beside exp2/sum of T0(c) | wait chunk c+1 + barrier |
//   MFMAs of T0(c+1) beside exp2/sum of T1(c)
// (the last iteration's T0(c+1) runs on the re-loaded last chunk and is discarded).
#include "hbx_common.h"
#include "hbx_kde_impl.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

// sched_group_barrier pattern: NM times {1 MFMA, then a share of NV VALU ops}
template <int I, int NM, int NV>
struct SgbAlt32 {
  static __device__ __forceinline__ void run() {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    constexpr int n = NV / NM + (I < NV % NM ? 1 : 0);
    if constexpr (n > 0) __builtin_amdgcn_sched_group_barrier(0x002, n, 0);
    SgbAlt32<I + 1, NM, NV>::run();
  }
};
template <int NM, int NV>
struct SgbAlt32<NM, NM, NV> {
  static __device__ __forceinline__ void run() {}
};

template <int NSC, int KC>
__global__ __launch_bounds__(64 * H32_WAVES) __attribute__((amdgpu_waves_per_eu(2))) void kde_logpdf_h32_kernel(
    const double* __restrict__ cand, int64_t Nc, int32_t D, const KdeParams* __restrict__ P,
    const float* __restrict__ table, KdeEst* __restrict__ out) {
  constexpr int ND = 2 * NSC;               // dense 16-wide K-steps (continuous + C_j pieces)
  constexpr int KS = KC;                    // sparse 32-wide K-steps (one-hot)
  constexpr int NMT = ND + KS;              // matrix instructions per 32x32 tile
  constexpr int KTP = h_ktp(NSC * 8, KC);   // halves per observation row
  constexpr int CHF = h_chunk_floats(NSC * 8, KC, 0);
  constexpr int AUXF = H32_WAVES * 32 * 3;  // per candidate: c_i, bound term, shift
  // two blocks per CU (their waves share the SIMDs out of phase) when three ring buffers fit in half
  // the LDS, else one block with as many buffers as fit (at most 4)
  constexpr int NHALF = (80 * 1024 / 4 - AUXF) / CHF;
  constexpr int NFIT = (160 * 1024 / 4 - AUXF) / CHF;
  constexpr int NBUF = NHALF >= 3 ? 3 : (NFIT < 4 ? NFIT : 4);
  static_assert((NBUF * CHF + AUXF) * 4 <= 160 * 1024, "observation chunk too large for LDS");
  constexpr int G = CHF * 4 / (1024 * H32_WAVES);  // 1-KB LDS-DMA pieces per wave per chunk
  static_assert(G * 1024 * H32_WAVES == CHF * 4, "chunk must be a multiple of 8 KB");
  static_assert(NBUF >= 2, "observation chunk too large for LDS");
  __shared__ __align__(16) float lds[NBUF * CHF + AUXF];  // the kernel's only LDS object
  float* aux = lds + NBUF * CHF;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int64_t cbase = ((int64_t)blockIdx.x * H32_WAVES + wave) * 32;
  const int n = P->n, dc = P->dc;

  struct ContPrm { double scale, center; float xmax; int32_t col; };
  struct OhPrm { double val; int32_t col, pad; };
  constexpr int PRM_BYTES = 8 * NSC * (int)sizeof(ContPrm) + 16 * (KC > 0 ? KC : 1) * (int)sizeof(OhPrm);
  const int DS = D | 1;  // staged row stride (odd number of doubles: conflict-free)
  const int64_t rows_bytes = (int64_t)H32_WAVES * 32 * DS * 8;
  const bool rows_fit = rows_bytes + PRM_BYTES <= (int64_t)NBUF * CHF * 4;
  ContPrm* cprm = (ContPrm*)((char*)lds + (rows_fit ? rows_bytes : 0));
  OhPrm* oprm = (OhPrm*)(cprm + 8 * NSC);
  const int tid = threadIdx.x;
  if (tid < 8 * NSC) {
    const bool act = tid < dc;
    cprm[tid] = ContPrm{act ? P->cont_scale[tid] : 0.0, act ? P->center[tid] : 0.0, act ? P->xmax[tid] : 0.f,
                        act ? P->cont_dim[tid] : 0};
  }
  if (tid < 16 * KC) oprm[tid] = OhPrm{P->oh_val[tid], P->oh_col[tid], 0};  // padding: NaN, never equal
  const bool staged = rows_fit && cbase < Nc;
  const int64_t nv = (Nc - cbase) < 32 ? (Nc - cbase) : 32;
  double* xs = (double*)lds + (int64_t)wave * 32 * DS;
  if (staged) {
    const double* src = cand + cbase * (int64_t)D;
    if (D <= 64) {
      const int rpi = 64 / D, lr = lane / D, lc = lane - lr * D;
      if (lr < rpi)
        for (int row = lr; row < nv; row += rpi) xs[row * DS + lc] = src[row * D + lc];
    } else {
      for (int row = 0; row < nv; ++row)
        for (int cc = lane; cc < D; cc += 64) xs[row * DS + cc] = src[row * D + cc];
    }
  }
  __syncthreads();

  // A operands of candidate row c: dense step s covers continuous dims 4s + 2h + {0,1} (four halves
  // each: hi, hi, lo, lo -- or 1 against a C_j piece in the last slot of dims 0-2); sparse step s
  // covers one-hot positions 16s + 8h + 0..7
  f16x8 ah[ND];
  f16x8 asp[KS > 0 ? KS : 1];
  int aidx[KS > 0 ? KS : 1];
  float ci = 0.f, bnd = 0.f;
  auto build = [&](const double* x) {
#pragma unroll
    for (int s = 0; s < ND; ++s) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int dim = 4 * s + 2 * h + e;
        const ContPrm q = cprm[dim];
        const float v0 = (float)(q.scale * (x[q.col] - q.center));
        const float v = dim < dc ? v0 : 0.f;
        ci = fmaf(-v, v, ci);
        bnd = fmaf(2.f * fabsf(v), q.xmax, bnd);
        const float xc = fminf(fmaxf(2.f * v, -60000.f), 60000.f);
        const _Float16 hi = (_Float16)xc;
        const _Float16 lo = (_Float16)(xc - (float)hi);
        ah[s][4 * e + 0] = hi;
        ah[s][4 * e + 1] = hi;
        ah[s][4 * e + 2] = lo;
        ah[s][4 * e + 3] = dim < 3 ? (_Float16)1.f : lo;
      }
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      int idx = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int t0 = 16 * s + 8 * h + 2 * q;
        const OhPrm o0 = oprm[t0], o1 = oprm[t0 + 1];
        const bool m0 = x[o0.col] == o0.val, m1 = x[o1.col] == o1.val;
        const _Float16 one = (m0 || m1) ? (_Float16)1.f : (_Float16)0.f;
        asp[s][2 * q + 0] = one;
        asp[s][2 * q + 1] = one;
        idx |= (m1 ? 0xE : 0x4) << (4 * q);  // slots (2,3) of the group if t0+1 matches, else (0,1)
      }
      aidx[s] = idx;
    }
  };
  {
    const int loc = c < nv ? c : (int)nv - 1;
    if (staged) {
      build(xs + loc * DS);
    } else {
      int64_t ii = cbase + c;
      if (ii >= Nc) ii = Nc - 1;
      build(cand + ii * (int64_t)D);
    }
  }
  ci += __shfl_xor(ci, 32);
  bnd += __shfl_xor(bnd, 32);
  // accumulator input: register r of this lane is candidate row 8(r/4) + 4h + r%4
  f32x16 ciq;
#pragma unroll
  for (int r = 0; r < 16; ++r) ciq[r] = __shfl(ci, 8 * (r >> 2) + 4 * h + (r & 3));

  const int nchunks = (n + OBS_CHUNK - 1) / OBS_CHUNK;
  auto issue = [&](int cc, int slot) {
    const float* src = table + (int64_t)(cc < nchunks ? cc : nchunks - 1) * CHF;
    float* dst = lds + slot * CHF;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int piece = wave + g * H32_WAVES;
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) const void*)(src + piece * 256 + lane * 4),
                                       (__attribute__((address_space(3))) void*)(dst + piece * 256), 16, 0, 0);
    }
  };
  constexpr int PD = NBUF - 1;
  __syncthreads();  // staged rows and parameters consumed: the ring may be overwritten
#pragma unroll
  for (int i = 0; i < PD; ++i) issue(i, i);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G * (PD - 1)) : "memory");  // chunk 0 landed
  __builtin_amdgcn_s_barrier();

  // B fragments of one 32-observation tile (observations 32 jt .. 32 jt + 31 of the chunk in buf) and
  // the ND + KS matrix instructions of that 32x32 tile
  struct Frag {
    f16x8 b[ND];
    f16x16 bs[KS > 0 ? KS : 1];
  };
  auto load = [&](const float* buf, int jt, Frag& f) {
    const _Float16* hb = (const _Float16*)(buf + OBS_CHUNK) + (32 * jt + c) * KTP + 8 * h;
#pragma unroll
    for (int s = 0; s < ND; ++s) f.b[s] = *(const f16x8*)(hb + 16 * s);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const f16x8 lo = *(const f16x8*)(hb + 32 * NSC + 32 * s);
      const f16x8 hi = *(const f16x8*)(hb + 32 * NSC + 32 * s + 16);
      f.bs[s] = f16x16{lo[0], lo[1], lo[2], lo[3], lo[4], lo[5], lo[6], lo[7],
                       hi[0], hi[1], hi[2], hi[3], hi[4], hi[5], hi[6], hi[7]};
    }
  };
  // matrix instruction s (0 .. NMT-1) of a tile: dense steps first (the first one takes the
  // accumulator input), then the sparse one-hot steps
  auto mma_step = [&](const Frag& f, int s, const f32x16& cin, f32x16& acc) {
    if (s == 0)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[0], f.b[0], cin, 0, 0, 0);
    else if (s < ND)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s], f.b[s], acc, 0, 0, 0);
    else
      acc = __builtin_amdgcn_smfmac_f32_32x32x32_f16(asp[s - ND], f.bs[s - ND], acc, aidx[s - ND], 0, 0);
  };
  auto mma = [&](const Frag& f, const f32x16& cin, f32x16& acc) {
#pragma unroll
    for (int s = 0; s < NMT; ++s) mma_step(f, s, cin, acc);
  };
  auto tile = [&](const float* buf, int jt, const f32x16& cin, f32x16& acc) {
    Frag f;
    load(buf, jt, f);
    mma(f, cin, acc);
  };

  // Per-candidate shift (see hbx_score_h.hip): the exponent's maximum over chunk 0 moves to 0
  {
    f32x16 a0, a1;
    tile(lds, 0, ciq, a0);
    tile(lds, 1, ciq, a1);
    float mx[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      mx[r] = fmaxf(a0[r], a1[r]);
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], o));
      const float d = rintf(-mx[r]);
      const float dl = (d > 0.f && d < 1e30f) ? d : 0.f;  // NaN rows: no shift
      ciq[r] += dl;
      if (c == 0) aux[(wave * 32 + 8 * (r >> 2) + 4 * h + (r & 3)) * 3 + 2] = dl;
    }
    if (h == 0) {
      aux[(wave * 32 + c) * 3 + 0] = ci;
      aux[(wave * 32 + c) * 3 + 1] = bnd;
    }
  }

  // Two phases per chunk c, fenced with sched_barrier so the compiler keeps them apart; fragments are
  // read one phase ahead of their MFMAs (LDS latency under the previous tile's MFMAs), the exp2/sum of
  // a tile runs one phase behind its MFMAs (beside the next tile's):
  //   P1(c): MFMA T0(c) [f0] | exp2/add T1(c-1) (chunk c-1 complete) | read f1 <- T1(c)
  //   P2(c): wait chunk c+1 + barrier | MFMA T1(c) [f1] | S += chunk c-1, exp2 T0(c) | read f0 <- T0(c+1)
  // (per phase 8 MFMAs = 256 matrix-pipe cycles beside 64 + 16 x 8 + 16 x 4 = 256 issue cycles)
  float S[16], Sb[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) S[r] = Sb[r] = 0.f;
  f32x16 accA, accB;
#pragma unroll
  for (int r = 0; r < 16; ++r) accB[r] = -INFINITY;  // "T1(-1)": exp2 -> 0
  Frag f0, f1;
  load(lds, 0, f0);
  // the two waves of a SIMD run the same phases in lockstep; a static priority for the second half of
  // the block breaks the tie in VALU arbitration (MI355X_MICROARCH "two waves per SIMD", item 4)
#ifndef HBX_H32_PRIO
#define HBX_H32_PRIO 1
#endif
  if (HBX_H32_PRIO && H32_WAVES > 4 && wave >= H32_WAVES / 2) __builtin_amdgcn_s_setprio(1);
  // explicit instruction order inside each phase: matrix instruction s, then its share of the
  // 16 epilogue registers, fenced (the scheduler does not keep the interleave by itself)
  constexpr int RPS = (16 + NMT - 1) / NMT;  // epilogue registers per matrix instruction
  for (int cc = 0; cc < nchunks; ++cc) {
    const float* buf = lds + (cc % NBUF) * CHF;
    const float* nbuf = lds + ((cc + 1) % NBUF) * CHF;
    issue(cc + PD, (cc + PD) % NBUF);  // its buffer was last read before the previous barrier
    __builtin_amdgcn_sched_barrier(0);
    // P1: f0 was read a phase ago; f1's reads go out behind the first MFMA
#pragma unroll
    for (int s = 0; s < NMT; ++s) {
      mma_step(f0, s, ciq, accA);
      if (s == 0) {
        __builtin_amdgcn_sched_barrier(0);  // the reads must not go out before the first MFMA
        load(buf, 1, f1);
      }
#pragma unroll
      for (int r = s * RPS; r < (s + 1) * RPS && r < 16; ++r) Sb[r] += __builtin_amdgcn_exp2f(accB[r]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // P2: chunk cc+1 landed for this wave and its reads of the ring retired; the barrier publishes
    // chunk cc+1 to every wave
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(G * (PD - 1)) : "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < NMT; ++s) {
      mma_step(f1, s, ciq, accB);
      if (s == 0) {
        __builtin_amdgcn_sched_barrier(0);
        load(nbuf, 0, f0);
      }
#pragma unroll
      for (int r = s * RPS; r < (s + 1) * RPS && r < 16; ++r) {
        S[r] += Sb[r];  // chunk cc-1 complete
        Sb[r] = __builtin_amdgcn_exp2f(accA[r]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) S[r] += Sb[r] + __builtin_amdgcn_exp2f(accB[r]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup

  // sum over the 32 observation columns of each lane half; lane c < 16 of half h then writes row
  // 8(c/4) + 4h + c%4 (register c)
#pragma unroll
  for (int r = 0; r < 16; ++r)
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) S[r] += __shfl_xor(S[r], o);
  float Sq = S[0];
#pragma unroll
  for (int r = 1; r < 16; ++r) Sq = (c == r) ? S[r] : Sq;  // select chain (no runtime register index)
  if (c < 16) {
    const int row = 8 * (c >> 2) + 4 * h + (c & 3);
    const int64_t ii = cbase + row;
    if (ii < Nc) {
      const float ci_q = aux[(wave * 32 + row) * 3 + 0];
      const float bnd_q = aux[(wave * 32 + row) * 3 + 1];
      const float dq = aux[(wave * 32 + row) * 3 + 2];
      const double* x = cand + ii * (int64_t)D;
      bool nq = P->nan_all != 0;
      for (int k = 0; k < P->nconst; ++k)
        if (x[P->const_dim[k]] != P->const_level[k]) nq = true;
      // rounding of the sums: 2 terms per lane per chunk, n/64 chunk partials, 5 butterfly levels
      KdeEst o = finish_est_terms(P, Sq, 0.f, -dq, nq, ci_q - dq, bnd_q, false,
                                  (float)(2 + nchunks + 5 + 8));
      // f16 hi/lo representation error and the three lo.lo products given up to the C_j pieces
      if (o.err > 0.f) o.err += (6.f * 0x1p-22f * bnd_q + 0x1p-20f) * HBX_LN2f;
      if (!nq && Sq == Sq && (Sq < 0x1p-64f || Sq > 0x1p100f)) o.err = -1.f;  // rescue marker
      out[ii] = o;
    }
  }
}

template <int NSC>
static logpdf_fn pick_kc32(int kc) {
  switch (kc) {
    case 0: return kde_logpdf_h32_kernel<NSC, 0>;
    case 1: return kde_logpdf_h32_kernel<NSC, 1>;
    case 2: return kde_logpdf_h32_kernel<NSC, 2>;
    case 3: return kde_logpdf_h32_kernel<NSC, 3>;
    case 4: return kde_logpdf_h32_kernel<NSC, 4>;
  }
  return nullptr;
}

logpdf_fn hbx_pick_h32(int nsc, int kc) {
  switch (nsc) {  // nsc_of(dc_pad) for dc_pad in {16, 24, 32, 64}
    case 2: return pick_kc32<2>(kc);
    case 3: return pick_kc32<3>(kc);
    case 4: return pick_kc32<4>(kc);
    case 8: return pick_kc32<8>(kc);
  }
  return nullptr;
}
