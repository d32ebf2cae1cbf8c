// hbx_score_h32.hip -- hmode scoring on 32x32 matrix tiles, observations on the A side (hmode 2).
//
// Same exponent as hbx_score_h.hip (continuous hi/lo f16 products, C_j as three exact f16 pieces, the
// one-hot product on the sparse matrix cores), on v_mfma_f32_32x32x16_f16 / v_smfmac_f32_32x32x32_f16.
// Why: the 16x16 kernel is bound by the SIMD's vector ISSUE port, not by the matrix pipe.  Per 1024
// pairs it spends 16 MFMAs x 8 issue cycles + 16 v_exp_f32 x 8 + 16 v_add_f32 x 4 = 320 cycles against
// 256 cycles of matrix pipe; a 32x32x16 MFMA holds the issue port for 8 of its 32 cycles, so the same
// work costs 8 x 8 + 128 + 64 = 256: two exp2 and two adds (24 cycles) hide in each MFMA's gap
// (MI355X_MICROARCH, 'vector-instruction ISSUE cost').
//
// Roles: A = observations (32 rows per tile, read from the LDS ring; the one-hot part 2:4-compressed
// in the table, hbx_kde_impl.h h32 layout), B = candidates (32 columns per wave, resident in registers).
// One-hot part: KP steps of 32 positions, the deltas' f16 hi parts then their lo parts against the same
// candidate fragments and index words; the FAST instance (acquisition) multiplies the hi parts only and
// widens the bound by the lo parts (every term, of either sign, is off by a factor within 2^+-L): 6
// matrix instructions per 1024 pairs at 24c + 8u instead of 7 (signed sums: + KP parity products).
// The output column of a lane is ONE candidate, so a lane's 16 accumulator registers are 16
// observations of the same candidate: the exp2 sum is an in-register tree and a lane carries one
// running sum (the 16x16 kernel's A = candidates layout needs 16 per lane here).  The candidate's
// c_i cannot then be the accumulator input (it would take 16 registers): it rides as three exact f16
// pieces in the lo.lo slots of dims 3-5 against 1 on the observation side, like C_j in dims 0-2.
//
// Operand layouts (gfx950, tools/mfma32_probe.hip, profiles/r01/mfma32_probe.txt):
//   dense A: lane l holds row l%32, K = 8(l/32) + 0..7;  dense B: K = 8(l/32) + 0..7 of column l%32;
//   D: register r of lane l = row 8(r/4) + 4(l/32) + r%4, column l%32;
//   sparse A: lane l covers row l%32, dense K [16(l/32), +16) as four 2-of-4 groups (index nibbles);
//   sparse B: lane half h holds K = 8h..8h+7 and 16+8h..16+8h+7 of column l%32.
//
// Pipeline per 64-observation chunk c (tiles T0, T1 of 32 observations), one basic block per phase:
//   LDS-DMA of chunk c+3 (part 0) | MFMAs of T0(c), each A fragment re-read for T1(c) right behind
//   its MFMA | exp2/sum of T1(c-1) beside them | LDS-DMA part 1 | wait chunk c+1 + barrier |
//   MFMAs of T1(c), fragments re-read for T0(c+1) | exp2/sum of T0(c) beside them.
#include "hbx_common.h"
#include "hbx_kde_impl.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define H32_CMAX 30000.f    // |shifted c_i| limit of the three-piece split (else: rescue pass)

// sparse index words of one tile: KS dwords (one ds_read).  KS = 1: both lane halves read the row's two
// dwords and take theirs (ds_read_b64 banks over 64 dwords, b32 over 32: 4-way on these rows)
template <int KS> struct H32Idx { typedef u32x4 T; };
template <> struct H32Idx<1> { typedef u32x2 T; };
template <> struct H32Idx<2> { typedef u32x2 T; };
template <int KS, typename T> __device__ __forceinline__ int h32_idx(const T& v, int s, int h) {
  if constexpr (KS == 1) return (int)(h ? v[1] : v[0]);
  else return (int)v[s];
}

// sched_group_barrier pattern of one phase: NM times {1 MFMA, its fragment re-read(s), a share of the
// NV VALU ops} (the last matrix instruction re-reads its fragment and the index words)
template <int I, int NM, int NV, int NRL, bool RD = true>
struct SgbH32 {
  static __device__ __forceinline__ void run() {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    constexpr int nr = !RD ? 0 : I == NM - 1 ? NRL : 1;
    if constexpr (nr > 0) __builtin_amdgcn_sched_group_barrier(0x100, nr, 0);
    constexpr int n = NV / NM + (I < NV % NM ? 1 : 0);
    if constexpr (n > 0) __builtin_amdgcn_sched_group_barrier(0x002, n, 0);
    SgbH32<I + 1, NM, NV, NRL, RD>::run();
  }
};
template <int NM, int NV, int NRL, bool RD>
struct SgbH32<NM, NM, NV, NRL, RD> {
  static __device__ __forceinline__ void run() {}
};

template <int NSC, int KP, bool SG, bool FAST, bool CO = false, int CT = 1>
__device__ __forceinline__ void kde_logpdf_h32_body(const double* __restrict__ cand, int64_t Nc, int32_t D,
                                                    const KdeParams* __restrict__ P,
                                                    const float* __restrict__ table, KdeEst* __restrict__ out,
                                                    const unsigned blk, int32_t* __restrict__ rescue_cnt = nullptr,
                                                    const int split = 0, const int nsplit = 1) {
  // CO: the coarse pre-screen (hbx_kde_impl.h coarse layout): one product per continuous dim, no lo parts
  constexpr int ND = CO ? h32c_nd(NSC) : h32_nd(NSC);  // dense 16-wide K-steps (C_j / c_i pieces + per dim)
  constexpr int KS = KP;                     // sparse 32-wide K-steps (one-hot positions), hi parts
  constexpr int KL = (FAST || CO) ? 0 : KP;  // ... and lo parts
  constexpr int NMT = ND + KS + KL;          // matrix instructions per 32x32 tile
  constexpr int KTP = CO ? h32c_ktp(NSC, KP) : h32_ktp(NSC, KP, SG);
  constexpr int CHF = CO ? h32c_chunk_floats(NSC, KP) : h32_chunk_floats(NSC, KP, SG);
  constexpr int PAR = h32_par(NSC, KP);  // signed: the parity block (halves into the row)
  static_assert(!SG || KP > 0, "signed sums come from categorical dims");
  static_assert(!FAST || KP > 0, "the fast instance drops the one-hot lo parts");
  static_assert(!CO || !SG, "the coarse instance is built for unsigned sums");
  static_assert(CT == 1 || (CT == 2 && CO), "two candidate column tiles per wave: the coarse instance");
  constexpr int HW = CO ? H32C_WAVES : H16_WAVES;  // waves per block, 32 CT candidates each
  constexpr int AUXF = HW * 32 * CT * 4;  // per candidate: c_i, bound term, shift, rescue flag
  // LDS ring: 4 buffers (3 chunks in flight) when two blocks' rings fit in the 160 KB, else 3
  constexpr int NBUF = 2 * (4 * CHF + AUXF) * 4 <= 160 * 1024 ? 4 : 3;
  static_assert(2 * (NBUF * CHF + AUXF) * 4 <= 160 * 1024, "two blocks per CU");
  constexpr int GP = CHF * 4 / 1024;  // 1-KB LDS-DMA pieces per chunk: GL per wave, one more for NX waves
  constexpr int GL = GP / HW, NX = GP % HW;
  static_assert(GP * 1024 == CHF * 4, "chunk must be a multiple of 1 KB");
  __shared__ __align__(16) float lds[NBUF * CHF + AUXF];  // the kernel's only LDS object
  float* aux = lds + NBUF * CHF;
  if constexpr (CO) table += P->coarse_off;  // the coarse layout follows the precise table
  // observation split: this block's chunk range, its partial estimates at out + split Nc
  int c0 = 0, nchunks = (P->n + OBS_CHUNK - 1) / OBS_CHUNK;
  if (nsplit > 1) {
    obs_split_range(nchunks, split, nsplit, &c0, &nchunks);
    out += (int64_t)split * Nc;
    if (nchunks <= 0) {  // more splits than chunks: this range is empty
      const int64_t cb = (int64_t)blk * HW * 32 * CT;
      for (int k = threadIdx.x; k < HW * 32 * CT; k += blockDim.x)
        if (cb + k < Nc) out[cb + k] = kde_est_neutral();
      return;
    }
    table += (int64_t)c0 * CHF;
  }

  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 31, h = lane >> 5;
  const int64_t cbase = ((int64_t)blk * HW + wave) * 32 * CT;
  const bool xpiece = wave < NX;
  const int dc = P->dc;

  // per-dim parameters and the block's candidate rows staged in the (not yet used) ring
  struct ContPrm { double scale, center; float xmax; int32_t col; };
  struct OhPrm { double val; int32_t col, pad; };
  constexpr int PRM_BYTES = 8 * NSC * (int)sizeof(ContPrm) + 32 * (KP > 0 ? KP : 1) * (int)sizeof(OhPrm);
  static_assert(PRM_BYTES <= NBUF * CHF * 4, "parameters must fit in the ring");
  const int DS = D | 1;  // odd row stride in doubles: conflict-free
  const int64_t rows_bytes = (int64_t)HW * 32 * CT * DS * 8;
  const bool rows_fit = rows_bytes + PRM_BYTES <= (int64_t)NBUF * CHF * 4;
  ContPrm* cprm = (ContPrm*)((char*)lds + (rows_fit ? rows_bytes : 0));
  OhPrm* oprm = (OhPrm*)(cprm + 8 * NSC);
  const int tid = threadIdx.x;
  if (tid < 8 * NSC) {
    const bool act = tid < dc;  // padding: never read unmasked
    cprm[tid] = ContPrm{act ? P->cont_scale[tid] : 0.0, act ? P->center[tid] : 0.0, act ? P->xmax[tid] : 0.f,
                        act ? P->cont_dim[tid] : 0};
  }
  if (tid < 32 * KP) oprm[tid] = OhPrm{P->oh_val[tid], P->oh_col[tid], 0};  // padding: NaN, never equal
  const bool staged = rows_fit && cbase < Nc;
  const int64_t nv = (Nc - cbase) < 32 * CT ? (Nc - cbase) : 32 * CT;  // valid rows of this wave
  double* xs = (double*)lds + (int64_t)wave * 32 * CT * DS;
  if (staged) stage_rows(cand + cbase * (int64_t)D, nv, D, DS, xs, lane);
  __syncthreads();

  // B operands of candidate column c.  Dense step s, half j of the lane: slot k = 16s + 8h + j -- slots
  // 0-2: 1 (against the C_j pieces), 3-5: the pieces of the shifted c_i (against 1; 0 in the probe),
  // 6 + 3d + {0,1,2}: (hi, hi, lo) of x''_d against the observation's (Xh, Xl, Xh).  Sparse step s:
  // one-hot positions 32s + 8h + j (half j) and 32s + 16 + 8h + j (half 8 + j), 1 on a match.
  f16x8 bd[CT][ND];
  f16x16 bsp[CT][KS > 0 ? KS : 1];
  float ci[CT], bnd[CT], cer[CT];  // cer: the coarse instance's dropped products (log2 units)
  auto build = [&](const double* x, const int t) {
    ci[t] = bnd[t] = cer[t] = 0.f;
    auto coord = [&](int d) {  // 2 x'_d (0 past the continuous dims), clamped to the f16 range
      const ContPrm q = cprm[d];
      const float v0 = (float)(q.scale * (x[q.col] - q.center));
      return d < dc ? v0 : 0.f;
    };
#pragma unroll
    for (int s = 0; s < ND; ++s) bd[t][s] = f16x8{};
    if (h == 0) bd[t][0][0] = bd[t][0][1] = bd[t][0][2] = (_Float16)1.f;
    if constexpr (CO) {
      // coarse: slot k = 6 + d, so element j of a lane half's B fragments is slot 16 (j / 8) + 8 h + j % 8 --
      // the two halves walk DIFFERENT dims with the same register index: each dim is built once per
      // candidate, the sums (c_i, bound terms) are half sums added across the halves below
#pragma unroll
      for (int j = 0; j < 8 * ND; ++j) {
        const int d = 16 * (j >> 3) + 8 * h + (j & 7) - 6;  // per lane half
        if (d < 0) continue;  // slots 0-5 (set above / after the probe)
        const bool act = d < 8 * NSC;
        const ContPrm q = cprm[act ? d : 0];
        const float v0 = (float)(q.scale * (x[q.col] - q.center));
        const float v = (act && d < dc) ? v0 : 0.f;
        ci[t] = fmaf(-v, v, ci[t]);
        const float xm = act ? q.xmax : 0.f;
        bnd[t] = fmaf(2.f * fabsf(v), xm, bnd[t]);
        const float xc = fminf(fmaxf(2.f * v, -60000.f), 60000.f);
        const _Float16 hi = (_Float16)xc;
        bd[t][j >> 3][j & 7] = hi;  // |x''.X' - xh.Xh| <= |xh| |Xl| + |xl| |X'|
        cer[t] = fmaf(fabsf((float)hi), fmaf(0x1p-11f, xm, 0x1p-25f), cer[t]);
        cer[t] = fmaf(fabsf(xc - (float)hi), xm, cer[t]);
      }
      ci[t] += __shfl_xor(ci[t], 32);
      bnd[t] += __shfl_xor(bnd[t], 32);
      cer[t] += __shfl_xor(cer[t], 32);
    } else {
      // every lane walks all dims (compile-time slot positions; each lane keeps its half's slots)
#pragma unroll
      for (int d = 0; d < 8 * NSC; ++d) {
        const float v = coord(d);
        ci[t] = fmaf(-v, v, ci[t]);
        bnd[t] = fmaf(2.f * fabsf(v), cprm[d].xmax, bnd[t]);
        const float xc = fminf(fmaxf(2.f * v, -60000.f), 60000.f);
        const _Float16 hi = (_Float16)xc;
        const _Float16 lo = (_Float16)(xc - (float)hi);
#pragma unroll
        for (int comp = 0; comp < 3; ++comp) {
          const int k = 6 + 3 * d + comp;
          if (h == ((k >> 3) & 1)) bd[t][k >> 4][k & 7] = comp < 2 ? hi : lo;
        }
      }
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const OhPrm o0 = oprm[32 * s + 8 * h + j], o1 = oprm[32 * s + 16 + 8 * h + j];
        bsp[t][s][j] = (x[o0.col] == o0.val) ? (_Float16)1.f : (_Float16)0.f;
        bsp[t][s][8 + j] = (x[o1.col] == o1.val) ? (_Float16)1.f : (_Float16)0.f;
      }
    }
  };
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    const int loc = 32 * t + c < nv ? 32 * t + c : (int)nv - 1;
    if (staged) {
      build(xs + loc * DS, t);
    } else {
      int64_t ii = cbase + 32 * t + c;
      if (ii >= Nc) ii = Nc - 1;
      build(cand + ii * (int64_t)D, t);
    }
    // the next tile's build re-reads the parameters (no values kept live across the builds: no spills)
    asm volatile("" ::: "memory");
  }

  // LDS-DMA of chunk cc into ring slot `slot`; part p issues the pieces g with g % 2 == p.  Every wave
  // issues GL + 1 pieces when GP is not a multiple of HW: the waves without an extra piece load their
  // first one again (same bytes to the same place), so the loop body has no branch -- a branch would
  // split the phases' scheduling regions -- and every wave's counted vmcnt is the same.
  auto issue = [&](int cc, int slot, int part) {
    const float* src = table + (int64_t)(cc < nchunks ? cc : nchunks - 1) * CHF;
    float* dst = lds + slot * CHF;
#pragma unroll
    for (int g = 0; g < GL + (NX ? 1 : 0); ++g) {
      const int piece = (g < GL || xpiece) ? wave + g * HW : wave % GP;
      if (g % 2 == part)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) const void*)(src + piece * 256 + lane * 4),
                                         (__attribute__((address_space(3))) void*)(dst + piece * 256), 16, 0, 0);
    }
  };
  constexpr int GW = GL + (NX ? 1 : 0);  // pieces per wave per chunk
  constexpr int PD = NBUF - 1;  // chunks in flight ahead of the one being read
  __syncthreads();  // every wave has read its staged rows and the parameters: the ring may be overwritten
#pragma unroll
  for (int i = 0; i < PD; ++i) {
    issue(i, i, 0);
    issue(i, i, 1);
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GW * (PD - 1)) : "memory");
  __builtin_amdgcn_s_barrier();

  // A fragments of one 32-observation tile: row 32 jt + c, halves 8h.. of every step, and the lane
  // half's index words (at 2 ksp h halves past the compressed one-hot part)
  f16x8 ad[ND];
  f16x8 asp[KS > 0 ? KS : 1];
  f16x8 asl[KL > 0 ? KL : 1];  // the lo parts (precise instance)
  f16x8 apar[SG ? KS : 1];  // signed: parity fragments (the one-hot part's positions, 0.5 per negative dim)
  typename H32Idx<KS>::T aix;
  // index words relative to arow (KP = 1: dwords 2b, 2b + 1, b = bit 4 of the row -- hbx_kde_impl.h)
  const int ixo = 16 * ND + (CO ? 16 : 32) * KP + (KP == 1 ? 4 * ((c >> 4) & 1) : 2 * h32_ksp(KP) * h) - 8 * h;
  auto arow = [&](const float* buf, int jt) { return (const _Float16*)buf + (32 * jt + c) * KTP + 8 * h; };
  auto readA = [&](const float* buf, int jt) {
    const _Float16* a = arow(buf, jt);
#pragma unroll
    for (int s = 0; s < ND; ++s) ad[s] = *(const f16x8*)(a + 16 * s);
#pragma unroll
    for (int s = 0; s < KS; ++s) asp[s] = *(const f16x8*)(a + 16 * ND + 16 * s);
#pragma unroll
    for (int s = 0; s < KL; ++s) asl[s] = *(const f16x8*)(a + 16 * ND + 16 * KP + 16 * s);
    if constexpr (SG)
#pragma unroll
      for (int s = 0; s < KS; ++s) apar[s] = *(const f16x8*)(a + PAR + 16 * s);
    if constexpr (KS > 0) aix = *(const typename H32Idx<KS>::T*)(a + ixo);
  };
  const f32x16 zero16 = {};
  // the tile's matrix instructions
  auto mma = [&](f32x16& acc, const int t) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ad[0], bd[t][0], zero16, 0, 0, 0);
#pragma unroll
    for (int s = 1; s < ND; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ad[s], bd[t][s], acc, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < KS; ++s)
      acc = __builtin_amdgcn_smfmac_f32_32x32x32_f16(asp[s], bsp[t][s], acc, h32_idx<KS>(aix, s, h), 0, 0);
#pragma unroll
    for (int s = 0; s < KL; ++s)
      acc = __builtin_amdgcn_smfmac_f32_32x32x32_f16(asl[s], bsp[t][s], acc, h32_idx<KS>(aix, s, h), 0, 0);
  };
  // the same, every fragment re-read (tile jt of nb) right behind the instruction that consumed it; a
  // signed KDE's parity product (the same index words) follows into accp
  auto mma_rd = [&](f32x16& acc, f32x16& accp, const float* nb, int jt, const int t = CT - 1) {
    const _Float16* a = arow(nb, jt);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ad[0], bd[t][0], zero16, 0, 0, 0);
    ad[0] = *(const f16x8*)a;
#pragma unroll
    for (int s = 1; s < ND; ++s) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ad[s], bd[t][s], acc, 0, 0, 0);
      ad[s] = *(const f16x8*)(a + 16 * s);
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      acc = __builtin_amdgcn_smfmac_f32_32x32x32_f16(asp[s], bsp[t][s], acc, h32_idx<KS>(aix, s, h), 0, 0);
      asp[s] = *(const f16x8*)(a + 16 * ND + 16 * s);
      if (!SG && KL == 0 && s == KS - 1) aix = *(const typename H32Idx<KS>::T*)(a + ixo);
    }
#pragma unroll
    for (int s = 0; s < KL; ++s) {
      acc = __builtin_amdgcn_smfmac_f32_32x32x32_f16(asl[s], bsp[t][s], acc, h32_idx<KS>(aix, s, h), 0, 0);
      asl[s] = *(const f16x8*)(a + 16 * ND + 16 * KP + 16 * s);
      if (!SG && s == KL - 1) aix = *(const typename H32Idx<KS>::T*)(a + ixo);
    }
    if constexpr (SG) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        accp = __builtin_amdgcn_smfmac_f32_32x32x32_f16(apar[s], bsp[t][s], s == 0 ? zero16 : accp, h32_idx<KS>(aix, s, h),
                                                        0, 0);
        apar[s] = *(const f16x8*)(a + PAR + 16 * s);
        if (s == KS - 1) aix = *(const typename H32Idx<KS>::T*)(a + ixo);
      }
    }
  };
  // Per-candidate shift (see hbx_score_h.hip): the exponent's maximum over chunk 0 is moved to 0.  The
  // probe runs without c_i (its B slots are 0); the maximum with it is c_i + the probe's maximum.
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    f32x16 a0, a1;
    readA(lds, 0);
    mma(a0, t);
    readA(lds, 1);
    mma(a1, t);
    float mx = fmaxf(a0[0], a1[0]);
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, fmaxf(a0[r], a1[r]));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float d = rintf(-(ci[t] + mx));
    const float dl = (d > 0.f && d < 1e30f) ? d : 0.f;  // NaN rows: no shift
    const float cs = ci[t] + dl;                        // the shifted c_i (its rounding is in the bound)
    const bool big = fabsf(cs) > H32_CMAX;              // beyond the split: the rescue pass
    const float cv = big ? 0.f : cs;
    const _Float16 p0 = (_Float16)cv;
    const float r1 = cv - (float)p0;
    const _Float16 p1 = (_Float16)r1;
    const _Float16 p2 = (_Float16)(r1 - (float)p1);
    // slots 3-5 = step 0, lane half 0, halves 3-5
    if (h == 0) {
      bd[t][0][3] = p0;
      bd[t][0][4] = p1;
      bd[t][0][5] = p2;
    }
    if (h == 0) {
      float* ax = aux + ((wave * CT + t) * 32 + c) * 4;
      ax[0] = ci[t];
      ax[1] = bnd[t];
      ax[2] = dl;
      ax[3] = big ? -1.f : cer[t] * (1.f + 0x1p-18f);  // rescue flag, else the coarse bound (rounded up)
    }
  }

  // exp2 of a tile's 16 terms and their pairwise sum (depth 4); signed: also the odd-parity terms'
  // sum, halved (fract of 0.5 x count is 0.5 for an odd count, else 0), in register order
  auto tile_sum = [&](const f32x16& a, const f32x16& ap, float& sn) -> float {
    float e[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) e[r] = __builtin_amdgcn_exp2f(a[r]);
    if constexpr (SG) {
      sn = __builtin_amdgcn_fractf(ap[0]) * e[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) sn = fmaf(__builtin_amdgcn_fractf(ap[r]), e[r], sn);
    }
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
      for (int r = 0; r < w; ++r) e[r] = e[2 * r] + e[2 * r + 1];
    return e[0];
  };
  auto schedule = [&]() {
    SgbH32<0, NMT, 32, (KS > 0 ? 2 : 1)>::run();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto schedule_nr = [&]() {  // a phase without fragment re-reads (two column tiles: the first tile's)
    SgbH32<0, NMT, 32, (KS > 0 ? 2 : 1), false>::run();
    __builtin_amdgcn_sched_barrier(0);
  };

  // Main loop.  Sums: a tile's 16 terms pairwise (depth 4), the chunk's two tiles (1), the chunks in
  // order (nchunks), the two lane halves (1).
  float S[CT], Sb[CT], Sn = 0.f, Snb = 0.f;
#pragma unroll
  for (int t = 0; t < CT; ++t) S[t] = Sb[t] = 0.f;
  f32x16 accA, accB, accpA, accpB;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    accB[r] = -INFINITY;  // "T1(-1)": exp2 -> 0
    accpB[r] = 0.f;
  }
  readA(lds, 0);
  // one chunk; b = cc % NBUF.  The main loop is unrolled over the ring so that b is a constant there: the
  // fragment addresses are then one lane base plus ds_read immediates (no address arithmetic per tile)
  auto chunk1 = [&](int cc, int b) {
    const float* buf = lds + b * CHF;
    const float* nbuf = lds + ((b + 1) % NBUF) * CHF;
    // chunk cc+PD's buffer was last read before the previous iteration's barrier
    issue(cc + PD, (b + PD) % NBUF, 0);
    mma_rd(accA, accpA, buf, 1);  // T0(cc); fragments of T1(cc)
    float tn;
    Sb[0] += tile_sum(accB, accpB, tn);  // T1(cc-1): chunk cc-1 complete
    S[0] += Sb[0];
    if constexpr (SG) {
      Snb += tn;
      Sn += Snb;
    }
    schedule();
    issue(cc + PD, (b + PD) % NBUF, 1);
    // chunk cc+1 complete for this wave (PD-1 chunks stay in flight), every read of the ring retired;
    // the barrier makes chunk cc+1 visible to every wave
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(GW * (PD - 1)) : "memory");
    __builtin_amdgcn_s_barrier();
    mma_rd(accB, accpB, nbuf, 0);  // T1(cc); fragments of T0(cc+1)
    Sb[0] = tile_sum(accA, accpA, tn);  // T0(cc)
    if constexpr (SG) Snb = tn;
    schedule();
  };
  // two column tiles (unsigned sums): four phases per chunk, each one tile x one column tile, in "snake"
  // order (T0, 0), (T0, 1), (T1, 1), (T1, 0), so every matrix instruction group shares one operand with
  // the group before it (the A fragments, or the column tile's B operands); the fragments of a tile feed
  // both column tiles, the second one's instructions re-reading them for the next tile.  accA: the odd
  // phases, accB: the even ones; each phase sums the accumulator the previous phase filled, and per
  // column tile the sums keep chunk1's association.  Column tile 0's T1 is summed in the next chunk's
  // first phase
  auto chunk2s = [&](int cc, int b) {
    const float* buf = lds + b * CHF;
    const float* nbuf = lds + ((b + 1) % NBUF) * CHF;
    float tn;
    issue(cc + PD, (b + PD) % NBUF, 0);
    mma(accA, 0);                       // (T0(cc), 0)
    Sb[0] += tile_sum(accB, accpB, tn);  // (T1(cc-1), 0): chunk cc-1 complete for column tile 0
    S[0] += Sb[0];
    schedule_nr();
    mma_rd(accB, accpB, buf, 1, 1);     // (T0(cc), 1); fragments of T1(cc)
    Sb[0] = tile_sum(accA, accpA, tn);  // (T0(cc), 0)
    schedule();
    issue(cc + PD, (b + PD) % NBUF, 1);
    mma(accA, 1);                           // (T1(cc), 1)
    Sb[CT - 1] = tile_sum(accB, accpB, tn);  // (T0(cc), 1)
    schedule_nr();
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(GW * (PD - 1)) : "memory");
    __builtin_amdgcn_s_barrier();
    mma_rd(accB, accpB, nbuf, 0, 0);          // (T1(cc), 0); fragments of T0(cc+1)
    Sb[CT - 1] += tile_sum(accA, accpA, tn);  // (T1(cc), 1): chunk cc complete for column tile 1
    S[CT - 1] += Sb[CT - 1];
    schedule();
  };
  auto chunk = [&](int cc, int b) {
    if constexpr (CT == 1) chunk1(cc, b);
    else chunk2s(cc, b);
  };
  int cc = 0;
  for (; cc + NBUF <= nchunks; cc += NBUF) {
    chunk(cc, 0);
    chunk(cc + 1, 1);
    chunk(cc + 2, 2);
    if constexpr (NBUF == 4) chunk(cc + 3, 3);
  }
  for (; cc < nchunks; ++cc) chunk(cc, cc % NBUF);
  {
    float tn;
    constexpr int tl = 0;  // the column tile of the last phase (CT = 2: snake order ends on column tile 0)
    Sb[tl] += tile_sum(accB, accpB, tn);  // T1(last)
    S[tl] += Sb[tl];
    if constexpr (SG) Sn += Snb + tn;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup
#pragma unroll
  for (int t = 0; t < CT; ++t) S[t] += __shfl_xor(S[t], 32);
  if constexpr (SG) Sn = 2.f * (Sn + __shfl_xor(Sn, 32));  // the odd-parity terms' sum (exact doubling)
#pragma unroll
  for (int t = 0; t < CT; ++t) {
  if (h == 0) {
    const int64_t ii = cbase + 32 * t + c;
    if (ii < Nc) {
      const float* ax = aux + ((wave * CT + t) * 32 + c) * 4;
      const float ci_q = ax[0], bnd_q = ax[1], dq = ax[2];
      const bool big = ax[3] < 0.f;
      const float cer_q = big ? 0.f : ax[3];
      const double* x = cand + ii * (int64_t)D;
      bool nq = P->nan_all != 0;
      for (int k = 0; k < P->nconst; ++k)
        if (x[P->const_dim[k]] != P->const_level[k]) nq = true;
      // S carries the factor 2^dq; |c_i| + dq bounds the rounding of the shifted c_i
      // sums: a tile's terms pairwise (depth 4; signed: its odd-parity terms in order, 16), the chunk's
      // two tiles, the chunks in order, the two lane halves
      KdeEst o = finish_est_terms(P, S[t], Sn, -dq, nq, ci_q - dq, bnd_q, SG, (float)(nchunks + (SG ? 18 : 6) + 24));
      // f16 hi/lo representation error of both coordinates (2 x 2^-22 sum|x''X'|) and the lo.lo products
      // given up (together <= 2^-22 sum|x''X'|), plus the C_j / c_i pieces' subnormal rounding
      if (o.err > 0.f) o.err += (6.f * 0x1p-22f * bnd_q + 0x1p-19f) * HBX_LN2f;
      if constexpr (FAST || CO) {  // the one-hot lo parts left out: |sum_u lo_u m_u| <= sum_u |lo_u| (log2)
        float lo_err = CO ? cer_q : 0.f;  // coarse: the dropped continuous products as well
        for (int u = 0; u < P->du; ++u) {
          const float dl = fminf(fmaxf(P->cat_delta[u], -60000.f), 60000.f);
          if (fabsf(dl) < 60000.f) lo_err += fabsf(dl - (float)(_Float16)dl);
        }
        // every term is off by a factor in [2^-L, 2^L], L = lo_err: the sums' relative bound e becomes
        // (1 + e) 2^L - 1 (rounded up)
        if (o.err > 0.f) o.err = (1.f + o.err) * exp2f(lo_err * (1.f + 0x1p-20f)) * (1.f + 0x1p-20f) - 1.f;
      }
      if (!nq && S[t] == S[t] && (big || S[t] < 0x1p-64f || S[t] > 0x1p100f)) {  // rescue marker
        o.err = -1.f;
        if (rescue_cnt) atomicAdd(rescue_cnt, 1);
      }
      out[ii] = o;
    }
  }
  }
}

// unsigned sums: 128 VGPRs, 4 waves per SIMD (two blocks per CU); the coarse instance: H32C_WAVES-wave
// blocks at >= H32C_EU waves per SIMD
template <int NSC, int KP, bool FAST, bool CO>
__global__ __launch_bounds__(64 * (CO ? H32C_WAVES : H16_WAVES)) __attribute__((amdgpu_waves_per_eu(CO ? H32C_EU : 4))) void kde_logpdf_h32_kernel(
    const double* __restrict__ cand, int64_t Nc, int32_t D, const KdeParams* __restrict__ P,
    const float* __restrict__ table, KdeEst* __restrict__ out) {
  kde_logpdf_h32_body<NSC, KP, false, FAST, CO, CO ? H32C_CT : 1>(cand, Nc, D, P, table, out, blockIdx.x);
}

// both KDEs of an acquisition in one grid (see kde_logpdf_h_pair_kernel)
template <int NSC, int KP, bool FAST, bool CO>
__global__ __launch_bounds__(64 * (CO ? H32C_WAVES : H16_WAVES)) __attribute__((amdgpu_waves_per_eu(CO ? H32C_EU : 4))) void kde_logpdf_h32_pair_kernel(
    const double* __restrict__ cand, int64_t Nc, int32_t D, KdePairArgs a) {
#if HBX_PAIR_INIT
  if (a.init.U && blockIdx.x == 0 && threadIdx.x == 0)  // a single acquisition's state (acq_init's work)
    acq_init_state(a.init.U, a.init.count, a.init.flags, a.init.first1, a.init.res);
#endif
  const bool second = blockIdx.x >= a.nblk0;  // uniform per block: scalar selects
  const unsigned loc = second ? blockIdx.x - a.nblk0 : blockIdx.x;
  const int ns = second ? a.nsplit1 : a.nsplit0;
  const unsigned tile = ns > 1 ? loc % a.tiles : loc;  // blocks of one chunk range are consecutive
  const int split = ns > 1 ? (int)(loc / a.tiles) : 0;
  kde_logpdf_h32_body<NSC, KP, false, FAST, CO, CO ? H32C_CT : 1>(cand, Nc, D, second ? a.P1 : a.P0, second ? a.table1 : a.table0,
                                                second ? a.out1 : a.out0, tile, a.rescue, split, ns);
}

// the coarse pair kernel with ONE candidate column tile per wave (32 candidates, half a block's): for launches
// whose two KDEs' H32C_CT-tile blocks fit one round of the chip's block slots (config #2: 2 x 196 blocks), twice
// the waves, each walking its chunks with half the matrix work -- more waves per SIMD to hide the ring refills
template <int NSC, int KP>
__global__ __launch_bounds__(64 * H32C_WAVES) __attribute__((amdgpu_waves_per_eu(H32C_EU))) void kde_logpdf_h32_pair1_kernel(
    const double* __restrict__ cand, int64_t Nc, int32_t D, KdePairArgs a) {
#if HBX_PAIR_INIT
  if (a.init.U && blockIdx.x == 0 && threadIdx.x == 0)
    acq_init_state(a.init.U, a.init.count, a.init.flags, a.init.first1, a.init.res);
#endif
  const bool second = blockIdx.x >= a.nblk0;
  const unsigned loc = second ? blockIdx.x - a.nblk0 : blockIdx.x;
  const int ns = second ? a.nsplit1 : a.nsplit0;
  const unsigned tile = ns > 1 ? loc % a.tiles : loc;
  const int split = ns > 1 ? (int)(loc / a.tiles) : 0;
  kde_logpdf_h32_body<NSC, KP, false, false, true, 1>(cand, Nc, D, second ? a.P1 : a.P0, second ? a.table1 : a.table0,
                                                       second ? a.out1 : a.out0, tile, a.rescue, split, ns);
}

// signed sums (the parity product and its accumulators): one 8-wave block per CU, so 2 waves per SIMD
// and a 256-register budget
template <int NSC, int KP, bool FAST>
__global__ __launch_bounds__(64 * H16_WAVES) __attribute__((amdgpu_waves_per_eu(2))) void kde_logpdf_h32s_kernel(
    const double* __restrict__ cand, int64_t Nc, int32_t D, const KdeParams* __restrict__ P,
    const float* __restrict__ table, KdeEst* __restrict__ out) {
  kde_logpdf_h32_body<NSC, KP, true, FAST>(cand, Nc, D, P, table, out, blockIdx.x);
}

template <int NSC, int KP, bool FAST>
__global__ __launch_bounds__(64 * H16_WAVES) __attribute__((amdgpu_waves_per_eu(2))) void kde_logpdf_h32s_pair_kernel(
    const double* __restrict__ cand, int64_t Nc, int32_t D, KdePairArgs a) {
#if HBX_PAIR_INIT
  if (a.init.U && blockIdx.x == 0 && threadIdx.x == 0)
    acq_init_state(a.init.U, a.init.count, a.init.flags, a.init.first1, a.init.res);
#endif
  const bool second = blockIdx.x >= a.nblk0;
  const unsigned loc = second ? blockIdx.x - a.nblk0 : blockIdx.x;
  const int ns = second ? a.nsplit1 : a.nsplit0;
  const unsigned tile = ns > 1 ? loc % a.tiles : loc;
  const int split = ns > 1 ? (int)(loc / a.tiles) : 0;
  kde_logpdf_h32_body<NSC, KP, true, FAST>(cand, Nc, D, second ? a.P1 : a.P0, second ? a.table1 : a.table0,
                                           second ? a.out1 : a.out0, tile, a.rescue, split, ns);
}

// instances: h32_ok (hbx_kde_impl.h); FAST where there is a one-hot part; CO (coarse) for unsigned sums
template <int NSC, int KP, bool SG, bool PAIR, bool FAST, bool CO>
static constexpr auto h32_inst() {
  if constexpr (PAIR) {
    if constexpr (SG) return (logpdf_pair_fn)kde_logpdf_h32s_pair_kernel<NSC, KP, FAST>;
    else return (logpdf_pair_fn)kde_logpdf_h32_pair_kernel<NSC, KP, FAST, CO>;
  } else {
    if constexpr (SG) return (logpdf_fn)kde_logpdf_h32s_kernel<NSC, KP, FAST>;
    else return (logpdf_fn)kde_logpdf_h32_kernel<NSC, KP, FAST, CO>;
  }
}

template <int NSC, int KP, bool SG, bool PAIR>
static auto pick32_fast(bool fast, bool coarse) {
  if constexpr (!SG)
    if (coarse) return h32_inst<NSC, KP, SG, PAIR, false, true>();
  if constexpr (KP > 0)
    if (fast) return h32_inst<NSC, KP, SG, PAIR, true, false>();
  return h32_inst<NSC, KP, SG, PAIR, false, false>();
}

template <int NSC, bool SG, bool PAIR>
static auto pick32_kp(int kp, bool fast, bool coarse) {
  switch (kp) {
    case 0: if constexpr (h32_ok(NSC, 0, SG)) return pick32_fast<NSC, 0, SG, PAIR>(fast, coarse); break;
    case 1: if constexpr (h32_ok(NSC, 1, SG)) return pick32_fast<NSC, 1, SG, PAIR>(fast, coarse); break;
    case 2: if constexpr (h32_ok(NSC, 2, SG)) return pick32_fast<NSC, 2, SG, PAIR>(fast, coarse); break;
  }
  return decltype(h32_inst<NSC, 1, SG, PAIR, false, false>())(nullptr);
}

template <bool SG, bool PAIR>
static auto pick32(int nsc, int kp, bool fast, bool coarse) {
  switch (nsc) {  // nsc_of(dc_pad) for dc_pad in {8, 16, 24, 32}
    case 1: return pick32_kp<1, SG, PAIR>(kp, fast, coarse);
    case 2: return pick32_kp<2, SG, PAIR>(kp, fast, coarse);
    case 3: return pick32_kp<3, SG, PAIR>(kp, fast, coarse);
    case 4: return pick32_kp<4, SG, PAIR>(kp, fast, coarse);
  }
  return decltype(pick32_kp<1, SG, PAIR>(0, false, false))(nullptr);
}

logpdf_fn hbx_pick_h32(int nsc, int kp, bool sg, bool fast, bool coarse) {
  return sg ? pick32<true, false>(nsc, kp, fast, false) : pick32<false, false>(nsc, kp, fast, coarse);
}

logpdf_pair_fn hbx_pick_h32_pair(int nsc, int kp, bool sg, bool fast, bool coarse) {
  return sg ? pick32<true, true>(nsc, kp, fast, false) : pick32<false, true>(nsc, kp, fast, coarse);
}

template <int NSC>
static logpdf_pair_fn pick32_pair1_kp(int kp) {
  switch (kp) {
    case 0: if constexpr (h32_ok(NSC, 0, false)) return kde_logpdf_h32_pair1_kernel<NSC, 0>; break;
    case 1: if constexpr (h32_ok(NSC, 1, false)) return kde_logpdf_h32_pair1_kernel<NSC, 1>; break;
    case 2: if constexpr (h32_ok(NSC, 2, false)) return kde_logpdf_h32_pair1_kernel<NSC, 2>; break;
  }
  return nullptr;
}

logpdf_pair_fn hbx_pick_h32_pair1(int nsc, int kp) {
  switch (nsc) {
    case 1: return pick32_pair1_kp<1>(kp);
    case 2: return pick32_pair1_kp<2>(kp);
    case 3: return pick32_pair1_kp<3>(kp);
    case 4: return pick32_pair1_kp<4>(kp);
  }
  return nullptr;
}
