// hbx_score_h.hip -- scoring kernel, whole exponent on the f16 matrix cores (hmode).
#include "hbx_common.h"
#include "hbx_kde_impl.h"

// hmode: the whole exponent is one f16 matrix product.  Continuous coordinates are split into f16
// hi + lo parts and the cross products are summed (every f16 x f16 product is exact in fp32; the
// representation error of each coordinate, 2^-22 relative, and the three lo.lo products given up to
// the C_j pieces are in the bound); C_j rides along as three exact f16 pieces against A = 1 and the
// one-hot categorical product follows in the same K loop.  c_i is the accumulator input of the first
// MFMA.  VALU work per pair: exp2 and one add.

// sched_group_barrier pattern: NM times {1 MFMA, then a share of NV VALU ops}, the remainder spread
// over the first MFMAs (LLVM SchedGroupMask: MFMA = 0x8, VALU = 0x2)
template <int I, int NM, int NV>
struct SgbAlternate {
  static __device__ __forceinline__ void run() {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    constexpr int n = NV / NM + (I < NV % NM ? 1 : 0);
    if constexpr (n > 0) __builtin_amdgcn_sched_group_barrier(0x002, n, 0);
    SgbAlternate<I + 1, NM, NV>::run();
  }
};
template <int NM, int NV>
struct SgbAlternate<NM, NM, NV> {
  static __device__ __forceinline__ void run() {}
};

// The same with the in-place B-fragment re-reads of a prefetching phase: after the last of the RT
// MFMAs of K-step s, its fragment reads (1 for a dense step, 2 for a sparse one: s >= NDENSE)
template <int I, int NM, int NV, int RT, int NDENSE>
struct SgbPrefetch {
  static __device__ __forceinline__ void run() {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    constexpr int n = NV / NM + (I < NV % NM ? 1 : 0);
    if constexpr (I % RT == RT - 1) __builtin_amdgcn_sched_group_barrier(0x100, (I / RT) < NDENSE ? 1 : 2, 0);
    if constexpr (n > 0) __builtin_amdgcn_sched_group_barrier(0x002, n, 0);
    SgbPrefetch<I + 1, NM, NV, RT, NDENSE>::run();
  }
};
template <int NM, int NV, int RT, int NDENSE>
struct SgbPrefetch<NM, NM, NV, RT, NDENSE> {
  static __device__ __forceinline__ void run() {}
};

// The kernel body, for block `blk` of one KDE's grid (the single-KDE kernel and the l+g pair kernel
// below both run it).
template <int NSC, int KC, bool SIGNED>
__device__ __forceinline__ void kde_logpdf_h_body(const double* __restrict__ cand, int64_t Nc, int32_t D,
                                                  const KdeParams* __restrict__ P,
                                                  const float* __restrict__ table, KdeEst* __restrict__ out,
                                                  const unsigned blk, int32_t* __restrict__ rescue_cnt = nullptr) {
  constexpr int RT = H_ROW_TILES;           // 16-candidate row tiles per wave
  constexpr int NSH = NSC + KC;             // f16 K-steps of 32
  // one-hot product on the sparse matrix cores (v_smfmac_f32_16x16x64_f16, 2:4 structured sparsity:
  // the candidate side has at most one match per pair of adjacent one-hot positions) -- one sparse
  // 64-wide step replaces two dense 32-wide steps
  constexpr bool SP = !SIGNED && KC > 0 && (KC % 2 == 0);
  constexpr int KS = SP ? KC / 2 : 1;       // sparse 64-wide steps
  constexpr int NMT = SP ? NSC + KC / 2 : NSH;  // matrix instructions per row tile and 16-obs tile
  constexpr int KTP = h_ktp(NSC * 8, KC);   // halves per observation row (padded); nsc_of(8 NSC) = NSC
  constexpr int KPP = h_kpp(KC);
  constexpr int CHF = h_chunk_floats(NSC * 8, KC, SIGNED ? 1 : 0);
  // LDS ring: 3 buffers (chunk c+2 in flight while c is used) when they fit in the 160 KB, else 2
  constexpr int HW = H16_WAVES;             // waves per block (16 candidates x RT each)
  static_assert(HW == 8, "only the 8-wave block is validated");
  // LDS ring: with 8-wave blocks (two per CU) 3 buffers when they fit, else 2; with 16-wave blocks (one
  // per CU) as many as fit, at most 6 (the staged candidate rows of 16 waves need the room)
  constexpr int NMAX = 160 * 1024 / (CHF * 4);
  constexpr int NBUF = HW > 8 ? (NMAX < 6 ? NMAX : 6) : (NMAX >= 3 ? 3 : 2);
  static_assert(NBUF >= 2 && NBUF * CHF * 4 <= 160 * 1024, "observation chunk too large for LDS");
  // 1-KB LDS-DMA pieces per chunk: GL per wave, one more for the first NX waves.  The issue cost of an
  // LDS-DMA instruction (~60-100 cycles) is per instruction, so larger blocks (more candidates sharing
  // one chunk load) issue fewer of them per pair.
  constexpr int GP = CHF * 4 / 1024;
  constexpr int GL = GP / HW, NX = GP % HW;
  static_assert(GP * 1024 == CHF * 4, "chunk must be a multiple of 1 KB");
  // after the ring: per (wave, row tile) the candidates' c_i, bound term and probe shift (read by the
  // epilogue only, so they need no registers across the main loop)
  constexpr int AUXF = HW * RT * 48;
  static_assert(NBUF * CHF * 4 + AUXF * 4 <= 160 * 1024, "ring + epilogue values exceed the LDS");
  __shared__ __align__(16) float lds[NBUF * CHF + AUXF];   // the kernel's only LDS object

  // wave made visibly uniform: LDS-DMA addresses, m0 and row bases are then SGPR arithmetic
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t cbase = ((int64_t)blk * HW + wave) * 16 * RT;
  const bool xpiece = wave < NX;  // this wave issues GL + 1 pieces per chunk
  const int n = P->n, dc = P->dc;
  const int ia = lane & 15, kq = lane >> 4;

  // A operands (candidate side).  Lane group kq owns, per K-step s, continuous dims
  // c = 8s + 2kq + {0,1} (halves 4e+{0,1} = hi, 4e+{2,3} = lo of x''_c) and one-hot slots
  // t = 16(s-NSC) + 4kq + q (halves 2q+{0,1}).  The per-dim parameters and the wave's candidate
  // rows (contiguous in HBM: one coalesced copy) are staged in LDS first, so every lane touches only
  // its own dims.  c_i = -|x'_i|^2 and the bound term are summed over the four lane groups with a
  // butterfly (bitwise identical in all four).  Rows fall back to global reads when the rows of all
  // waves do not fit in the (not yet used) LDS ring (large D).
  // All of it lives in the one LDS array (a second __shared__ object beside the LDS-DMA ring makes
  // hipcc wait vmcnt(0) before every ds_read of the main loop): staged rows first, parameters after.
  struct ContPrm { double scale, center; float xmax; int32_t col; };
  struct OhPrm { double val; int32_t col, pad; };
  constexpr int PRM_BYTES = 8 * NSC * (int)sizeof(ContPrm) + 16 * (KC > 0 ? KC : 1) * (int)sizeof(OhPrm);
  static_assert(PRM_BYTES <= NBUF * CHF * 4, "parameters must fit in the ring");
  // staged rows are DS = D|1 doubles apart (odd): the 16 rows a lane group reads hit distinct banks
  const int DS = D | 1;
  const int64_t rows_bytes = (int64_t)HW * 16 * RT * DS * 8;
  const bool rows_fit = rows_bytes + PRM_BYTES <= (int64_t)NBUF * CHF * 4;
  ContPrm* cprm = (ContPrm*)((char*)lds + (rows_fit ? rows_bytes : 0));
  OhPrm* oprm = (OhPrm*)(cprm + 8 * NSC);
  const int tid = threadIdx.x;
  if (tid < 8 * NSC) {
    const bool act = tid < dc;  // padding: never read unmasked
    cprm[tid] = ContPrm{act ? P->cont_scale[tid] : 0.0, act ? P->center[tid] : 0.0, act ? P->xmax[tid] : 0.f,
                        act ? P->cont_dim[tid] : 0};
  }
  if (tid < 16 * KC) oprm[tid] = OhPrm{P->oh_val[tid], P->oh_col[tid], 0};  // padding: NaN, never equal
  const bool staged = rows_fit && cbase < Nc;
  const int64_t nv = (Nc - cbase) < 16 * RT ? (Nc - cbase) : 16 * RT;  // valid rows of this wave
  double* xs = (double*)lds + (int64_t)wave * 16 * RT * DS;
  if (staged) stage_rows(cand + cbase * (int64_t)D, nv, D, DS, xs, lane);
  __syncthreads();
  f16x8 ah[RT][NSH];
  f16x8 asp[RT][KS];  // SP: compressed one-hot A (two nonzeros per group of four K slots)
  int aidx[RT][KS];   // SP: their positions, one nibble per group (first | second << 2)
  float ci_a[RT], bnd_a[RT];
  // row tile r of the A operands from candidate row x (LDS or global; inlined once for each)
  auto build = [&](int r, const double* x) {
    float ci = 0.f, bnd = 0.f;
#pragma unroll
    for (int s = 0; s < NSC; ++s) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int c = 8 * s + 2 * kq + e;
        const ContPrm q = cprm[c];
        const float v0 = (float)(q.scale * (x[q.col] - q.center));
        const float v = c < dc ? v0 : 0.f;
        ci = fmaf(-v, v, ci);
        bnd = fmaf(2.f * fabsf(v), q.xmax, bnd);
        const float xc = fminf(fmaxf(2.f * v, -60000.f), 60000.f);
        const _Float16 hi = (_Float16)xc;
        const _Float16 lo = (_Float16)(xc - (float)hi);
        ah[r][s][4 * e + 0] = hi;
        ah[r][s][4 * e + 1] = hi;
        ah[r][s][4 * e + 2] = lo;
        ah[r][s][4 * e + 3] = c < 3 ? (_Float16)1.f : lo;  // dims 0-2: against a C_j piece
      }
    }
    ci += __shfl_xor(ci, 16);
    ci += __shfl_xor(ci, 32);
    bnd += __shfl_xor(bnd, 16);
    bnd += __shfl_xor(bnd, 32);
    ci_a[r] = ci;
    bnd_a[r] = bnd;
    if constexpr (SP) {
      // lane group kq covers dense K [16kq, 16kq+16) of each 64-wide step: one-hot positions
      // t0 = 32 s + 8 kq + 2q and t0+1 (slots 2t, 2t+1 each); prepare pads every dim's positions to
      // start even, so the two never belong to different dims and at most one of them matches
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        int idx = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const OhPrm o0 = oprm[32 * s + 8 * kq + 2 * q], o1 = oprm[32 * s + 8 * kq + 2 * q + 1];
          const bool m0 = x[o0.col] == o0.val, m1 = x[o1.col] == o1.val;
          const _Float16 h = (m0 || m1) ? (_Float16)1.f : (_Float16)0.f;
          asp[r][s][2 * q + 0] = h;
          asp[r][s][2 * q + 1] = h;
          idx |= (m1 ? 0xE : 0x4) << (4 * q);  // slots (2,3) of the group if t0+1 matches, else (0,1)
        }
        aidx[r][s] = idx;
      }
    } else {
#pragma unroll
      for (int s = 0; s < KC; ++s) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const OhPrm o = oprm[16 * s + 4 * kq + q];
          const _Float16 h = (x[o.col] == o.val) ? (_Float16)1.f : (_Float16)0.f;
          ah[r][NSC + s][2 * q + 0] = h;
          ah[r][NSC + s][2 * q + 1] = h;
        }
      }
    }
  };
  if (staged) {
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const int loc = (16 * r + ia) < nv ? (16 * r + ia) : (int)nv - 1;
      build(r, xs + loc * DS);
    }
  } else {
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      int64_t ii = cbase + 16 * r + ia;
      if (ii >= Nc) ii = Nc - 1;
      build(r, cand + ii * (int64_t)D);
    }
  }
  // accumulator rows of this lane: candidates cbase + 16 r + 4 kq + q
  f32x4 ciq[RT];
  float* aux = lds + NBUF * CHF + wave * RT * 48;
#pragma unroll
  for (int r = 0; r < RT; ++r) {
#pragma unroll
    for (int q = 0; q < 4; ++q) ciq[r][q] = __shfl(ci_a[r], 4 * kq + q);
    if (kq == 0) {  // lane ia holds candidate 16 r + ia's values
      aux[r * 48 + ia] = ci_a[r];
      aux[r * 48 + 16 + ia] = bnd_a[r];
    }
  }

  float S[RT][4], Sn[RT][4];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q) S[r][q] = Sn[r][q] = 0.f;
  const int nchunks = (n + OBS_CHUNK - 1) / OBS_CHUNK;
  // LDS-DMA (global_load_lds_dwordx4): each wave copies its G 1-KB pieces of a chunk straight into
  // the ring; completion is tracked by a counted vmcnt + one raw barrier per chunk
  // part < 0: all pieces; else only pieces g with g % 3 == part (the main loop spreads a chunk's
  // LDS-DMA instructions over its first three phases)
  auto issue = [&](int c, int slot, int part = -1) {
    const float* src = table + (int64_t)(c < nchunks ? c : nchunks - 1) * CHF;
    float* dst = lds + slot * CHF;
#pragma unroll
    for (int g = 0; g < GL + (NX ? 1 : 0); ++g) {
      const int piece = wave + g * HW;
      if ((part < 0 || g % 3 == part) && (g < GL || xpiece))
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) const void*)(src + piece * 256 + lane * 4),
                                         (__attribute__((address_space(3))) void*)(dst + piece * 256), 16, 0, 0);
    }
  };
  // The loads of every iteration are unconditional (past the last chunk the last chunk is re-loaded
  // into the free buffer and never read), so the counted vmcnt is the same in every iteration and the
  // loop body is one basic block the scheduler can interleave.
  constexpr int PD = NBUF - 1;  // chunks in flight ahead of the one being read
  __syncthreads();  // every wave has read its staged rows: the ring may be overwritten
#pragma unroll
  for (int i = 0; i < PD; ++i) issue(i, i);
  // chunk 0 landed (the waves' piece counts differ: GL or GL + 1 per chunk)
  if (NX && xpiece)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((GL + 1) * (PD - 1)) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL * (PD - 1)) : "memory");
  __builtin_amdgcn_s_barrier();

  // B fragments of one 16-observation column tile (and, signed, its parity fragments)
  constexpr int KPF = (SIGNED && KC > 0) ? KC : 1;
  auto readb = [&](const float* buf, int jt, f16x8 (&b)[NSH], f16x8 (&bp)[KPF]) {
    const int jo = jt * 16 + ia;
    const _Float16* hb = (const _Float16*)(buf + OBS_CHUNK) + jo * KTP + 8 * kq;
#pragma unroll
    for (int s = 0; s < NSH; ++s) b[s] = *(const f16x8*)(hb + 32 * s);
    if constexpr (SIGNED) {
      const _Float16* pb = (const _Float16*)(buf + OBS_CHUNK + OBS_CHUNK * KTP / 2) + jo * KPP + 8 * kq;
#pragma unroll
      for (int s = 0; s < KC; ++s) bp[s] = *(const f16x8*)(pb + 32 * s);
    }
  };
  // MFMAs of one column tile for every row tile
  auto mfmas = [&](const f16x8 (&b)[NSH], const f16x8 (&bp)[KPF], f32x4* acc, f32x4* accp) {
#pragma unroll
    for (int r = 0; r < RT; ++r) acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[r][0], b[0], ciq[r], 0, 0, 0);
    constexpr int NDENSE = SP ? NSC : NSH;
#pragma unroll
    for (int s = 1; s < NDENSE; ++s)
#pragma unroll
      for (int r = 0; r < RT; ++r) acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[r][s], b[s], acc[r], 0, 0, 0);
    if constexpr (SP) {
      // B of the sparse step: lane group g holds K = 8g .. 8g+7 and 32 + 8g .. 32 + 8g + 7 of the
      // 64-wide step, i.e. the two dense fragments already read
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const f16x8 lo = b[NSC + 2 * s], hi = b[NSC + 2 * s + 1];
        const f16x16 b16 = {lo[0], lo[1], lo[2], lo[3], lo[4], lo[5], lo[6], lo[7],
                            hi[0], hi[1], hi[2], hi[3], hi[4], hi[5], hi[6], hi[7]};
#pragma unroll
        for (int r = 0; r < RT; ++r)
          acc[r] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(asp[r][s], b16, acc[r], aidx[r][s], 0, 0);
      }
    }
    if constexpr (SIGNED) {
#pragma unroll
      for (int r = 0; r < RT; ++r) accp[r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KC; ++s)
#pragma unroll
        for (int r = 0; r < RT; ++r)
          accp[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[r][NSC + s], bp[s], accp[r], 0, 0, 0);
    }
  };

  // The MFMAs of one column tile, each B fragment re-read in place (from tile jt of `nb`) right after
  // the last MFMA that consumes it: one register set, and every read has the rest of the phase to land.
  auto mfmas_rd = [&](f16x8 (&b)[NSH], f16x8 (&bp)[KPF], f32x4* acc, f32x4* accp, const float* nb, int jt) {
    const int jo = jt * 16 + ia;
    const _Float16* hb = (const _Float16*)(nb + OBS_CHUNK) + jo * KTP + 8 * kq;
#pragma unroll
    for (int r = 0; r < RT; ++r) acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[r][0], b[0], ciq[r], 0, 0, 0);
    constexpr int NDENSE = SP ? NSC : NSH;
    b[0] = *(const f16x8*)(hb);
#pragma unroll
    for (int s = 1; s < NDENSE; ++s) {
#pragma unroll
      for (int r = 0; r < RT; ++r) acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[r][s], b[s], acc[r], 0, 0, 0);
      b[s] = *(const f16x8*)(hb + 32 * s);
    }
    if constexpr (SP) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const f16x8 lo = b[NSC + 2 * s], hi = b[NSC + 2 * s + 1];
        const f16x16 b16 = {lo[0], lo[1], lo[2], lo[3], lo[4], lo[5], lo[6], lo[7],
                            hi[0], hi[1], hi[2], hi[3], hi[4], hi[5], hi[6], hi[7]};
#pragma unroll
        for (int r = 0; r < RT; ++r)
          acc[r] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(asp[r][s], b16, acc[r], aidx[r][s], 0, 0);
        b[NSC + 2 * s] = *(const f16x8*)(hb + 32 * (NSC + 2 * s));
        b[NSC + 2 * s + 1] = *(const f16x8*)(hb + 32 * (NSC + 2 * s + 1));
      }
    }
    if constexpr (SIGNED) {
      const _Float16* pb = (const _Float16*)(nb + OBS_CHUNK + OBS_CHUNK * KTP / 2) + jo * KPP + 8 * kq;
#pragma unroll
      for (int r = 0; r < RT; ++r) accp[r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KC; ++s) {
#pragma unroll
        for (int r = 0; r < RT; ++r)
          accp[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[r][NSC + s], bp[s], accp[r], 0, 0, 0);
        bp[s] = *(const f16x8*)(pb + 32 * s);
      }
    }
  };

  // Per-candidate shift: the exponent's maximum over chunk 0 (a lower bound of the maximum over all
  // observations) is moved to 0 through the accumulator input.  Without it candidates far from every
  // observation -- most of what BOHB's own sampler proposes at D = 32, where the truncnorm scale is
  // 3 bw -- would underflow fp32 against the static bound M0 and need the slow rescue pass.  Terms of
  // later chunks can exceed the probe's maximum; a sum that leaves [2^-64, 2^100] still takes the
  // rescue.  Costs one chunk of MFMAs (no exp2) per block.
  float dl[RT][4];
  f16x8 bA[NSH], bpA[KPF];
  {
    f32x4 acc[RT], accp[RT];
    float mx[RT][4];
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) mx[r][q] = -INFINITY;
#pragma unroll
    for (int jt = 0; jt < OBS_CHUNK / 16; ++jt) {
      readb(lds, jt, bA, bpA);
      mfmas(bA, bpA, acc, accp);
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) mx[r][q] = fmaxf(mx[r][q], acc[r][q]);
    }
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) mx[r][q] = fmaxf(mx[r][q], __shfl_xor(mx[r][q], o));
        const float d = rintf(-mx[r][q]);
        dl[r][q] = (d > 0.f && d < 1e30f) ? d : 0.f;  // NaN rows: no shift
        ciq[r][q] += dl[r][q];
        if (ia == 0) aux[r * 48 + 32 + 4 * kq + q] = dl[r][q];
      }
  }

  // Main loop, software-pipelined across tiles and chunks.  Phase t of iteration c runs the MFMAs of
  // tile t of chunk c on B fragments read one phase earlier, issues the LDS reads of the next tile
  // (tile 0 of chunk c+1 in phase 3) and, beside the MFMAs, the exp2/sum epilogue of the previous tile
  // (tile 3 of chunk c-1 in phase 0).  Every MFMA thus waits on LDS reads issued a whole phase
  // before, and every exp2 sits between MFMAs.  The chunk c+1 barrier comes before phase 3 (whose
  // reads need chunk c+1); at that point all reads of buffer c have retired, so the LDS-DMA issued at
  // the top of iteration c+1 into that buffer is safe.  Per-chunk partial sums (Sb: four terms) and
  // their order into S are those of the unpipelined loop.
  f32x4 accA[RT], accB[RT], accpA[RT], accpB[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    accB[r] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};  // exp2 -> 0: the first epilogue adds nothing
    accpB[r] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float Sb[RT][4], Snb[RT][4];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q) Sb[r][q] = Snb[r][q] = 0.f;
  // epilogue of one tile: first = the tile opens a chunk's partial sum
  // (all exp2s first, then the adds: in program order the sched groups then never put an add right
  // behind the exp2 it waits for)
  auto epi = [&](const f32x4* cur, const f32x4* curp, bool first) {
    float e[RT][4];
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) e[r][q] = __builtin_amdgcn_exp2f(cur[r][q]);
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        Sb[r][q] = first ? e[r][q] : Sb[r][q] + e[r][q];
        if (SIGNED)
          Snb[r][q] = fmaf(2.f * __builtin_amdgcn_fractf(0.5f * curp[r][q]), e[r][q], first ? 0.f : Snb[r][q]);
      }
  };
  auto close_chunk = [&]() {
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        S[r][q] += Sb[r][q];
        if (SIGNED) Sn[r][q] += Snb[r][q];
      }
  };
  // fragment prefetch where the register budget allows (small buckets); the large ones read each
  // tile's fragments right before its MFMAs
  constexpr bool PREF = (NSH + (SIGNED ? KC : 0)) <= 8;
  // one MFMA, then one or two VALU (an exp2 or an add), alternating; the B-fragment reads first
  auto schedule = [&]() {
    if constexpr (!SIGNED) {
      if constexpr (PREF) {  // fragment re-reads right behind their last MFMA
        SgbPrefetch<0, NMT * RT, 8 * RT, RT, (SP ? NSC : NSH)>::run();
      } else {  // this tile's fragments first
        __builtin_amdgcn_sched_group_barrier(0x100, NSH, 0);
        SgbAlternate<0, NMT * RT, 8 * RT>::run();  // exp2 + add of the previous tile
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto phase = [&](const float* cb, int t, const float* nb, int tn, f32x4* acc, f32x4* accp) {
    if constexpr (PREF) {
      mfmas_rd(bA, bpA, acc, accp, nb, tn);
    } else {
      readb(cb, t, bA, bpA);
      mfmas(bA, bpA, acc, accp);
    }
  };
  if (PREF) readb(lds, 0, bA, bpA);  // tile 0 of chunk 0 (buffer 0)
  for (int c = 0; c < nchunks; ++c) {
    const float* buf = lds + (c % NBUF) * CHF;
    const float* nbuf = lds + ((c + 1) % NBUF) * CHF;
    // chunk c+PD's LDS-DMA, spread over phases 0-2 (its buffer's reads all retired before the previous
    // barrier; all pieces are in flight before this iteration's barrier, so its counted vmcnt holds)
    issue(c + PD, (c + PD) % NBUF, 0);
    // phase 0: MFMAs of tile 0, then its fragments re-read for tile 1; epilogue of tile 3 of chunk c-1
    phase(buf, 0, buf, 1, accA, accpA);
    epi(accB, accpB, false);
    close_chunk();
    schedule();
    // phase 1
    issue(c + PD, (c + PD) % NBUF, 1);
    phase(buf, 1, buf, 2, accB, accpB);
    epi(accA, accpA, true);
    schedule();
    // phase 2
    issue(c + PD, (c + PD) % NBUF, 2);
    phase(buf, 2, buf, 3, accA, accpA);
    epi(accB, accpB, false);
    schedule();
    // chunk c+1 complete for this wave (PD-1 chunks stay in flight) and every read of buffer c
    // retired; the barrier makes chunk c+1 visible to every wave
    if (NX && xpiece)
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((GL + 1) * (PD - 1)) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(GL * (PD - 1)) : "memory");
    __builtin_amdgcn_s_barrier();
    // phase 3: MFMAs of tile 3; fragments of tile 0 of chunk c+1 read
    phase(buf, 3, nbuf, 0, accB, accpB);
    epi(accA, accpA, false);
    schedule();
  }
  epi(accB, accpB, false);  // tile 3 of the last chunk
  close_chunk();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        S[r][q] += __shfl_xor(S[r][q], o);
        if (SIGNED) Sn[r][q] += __shfl_xor(Sn[r][q], o);
      }
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    if (ia < 4) {
      const int cq = 4 * kq + ia;  // this lane's candidate within the row tile
      const float ci_q = aux[r * 48 + cq], bnd_q = aux[r * 48 + 16 + cq], dq = aux[r * 48 + 32 + cq];
      const int q = ia;
      const int64_t ii = cbase + 16 * r + 4 * kq + q;
      // select tree on named values (a runtime index into S would put S in scratch memory)
      const bool b0 = (ia & 1) != 0, b1 = (ia & 2) != 0;
      const float s0 = S[r][0], s1 = S[r][1], s2 = S[r][2], s3 = S[r][3];
      const float n0 = Sn[r][0], n1 = Sn[r][1], n2 = Sn[r][2], n3 = Sn[r][3];
      const float Sq = b1 ? (b0 ? s3 : s2) : (b0 ? s1 : s0);
      const float Snq = b1 ? (b0 ? n3 : n2) : (b0 ? n1 : n0);
      if (ii < Nc) {
        const double* x = cand + ii * (int64_t)D;
        bool nq = P->nan_all != 0;
        for (int cc = 0; cc < P->nconst; ++cc)
          if (x[P->const_dim[cc]] != P->const_level[cc]) nq = true;
        // S carries the factor 2^dq; |c_i| + dq bounds the rounding of the shifted accumulator input
        KdeEst o = finish_est(P, Sq, Snq, -dq, nq, ci_q - dq, bnd_q, SIGNED, OBS_CHUNK / 16);
        // f16 hi/lo representation error of both coordinates and the three lo.lo products given up
        // to the C_j pieces (each <= 2^-22 sum|x''X'|), plus the pieces' subnormal rounding
        if (o.err > 0.f) o.err += (6.f * 0x1p-22f * bnd_q + 0x1p-20f) * HBX_LN2f;
        if (!nq && Sq == Sq && (Sq < 0x1p-64f || Sq > 0x1p100f)) {
          o.err = -1.f;  // rescue marker
          if (rescue_cnt) atomicAdd(rescue_cnt, 1);
        }
        out[ii] = o;
      }
    }
  }
}

template <int NSC, int KC, bool SIGNED>
__global__ __launch_bounds__(64 * H16_WAVES) __attribute__((amdgpu_waves_per_eu(H_WAVES_PER_EU))) void kde_logpdf_h_kernel(
    const double* __restrict__ cand, int64_t Nc, int32_t D, const KdeParams* __restrict__ P,
    const float* __restrict__ table, KdeEst* __restrict__ out) {
  kde_logpdf_h_body<NSC, KC, SIGNED>(cand, Nc, D, P, table, out, blockIdx.x);
}

// Both KDEs of an acquisition in one launch: blocks [0, nblk0) score KDE 0, the rest KDE 1 over the
// same candidates.  The launcher puts the larger KDE first, so the short KDE's blocks fill the tail
// of the long one's last wave of blocks (and one launch gap goes away).
template <int NSC, int KC, bool SIGNED>
__global__ __launch_bounds__(64 * H16_WAVES) __attribute__((amdgpu_waves_per_eu(H_WAVES_PER_EU))) void kde_logpdf_h_pair_kernel(
    const double* __restrict__ cand, int64_t Nc, int32_t D, KdePairArgs a) {
  const bool second = blockIdx.x >= a.nblk0;  // uniform per block: scalar selects
  kde_logpdf_h_body<NSC, KC, SIGNED>(cand, Nc, D, second ? a.P1 : a.P0, second ? a.table1 : a.table0,
                                     second ? a.out1 : a.out0, second ? blockIdx.x - a.nblk0 : blockIdx.x, a.rescue);
}

template <int NSC, bool SG>
static logpdf_pair_fn pick_pair_kc(int kc) {
  switch (kc) {
    case 0: return kde_logpdf_h_pair_kernel<NSC, 0, SG>;
    case 1: return kde_logpdf_h_pair_kernel<NSC, 1, SG>;
    case 2: return kde_logpdf_h_pair_kernel<NSC, 2, SG>;
    case 3: return kde_logpdf_h_pair_kernel<NSC, 3, SG>;
    case 4: return kde_logpdf_h_pair_kernel<NSC, 4, SG>;
  }
  return nullptr;
}

template <bool SG>
static logpdf_pair_fn pick_pair_nsc(int nsc, int kc) {
  switch (nsc) {
    case 1: return pick_pair_kc<1, SG>(kc);
    case 2: return pick_pair_kc<2, SG>(kc);
    case 3: return pick_pair_kc<3, SG>(kc);
    case 4: return pick_pair_kc<4, SG>(kc);
    case 8: return pick_pair_kc<8, SG>(kc);
  }
  return nullptr;
}

logpdf_pair_fn hbx_pick_h_pair(int nsc, int kc, bool sg) {
  return sg ? pick_pair_nsc<true>(nsc, kc) : pick_pair_nsc<false>(nsc, kc);
}

template <int NSC, bool SG>
static logpdf_fn pick_kc(int kc) {
  switch (kc) {
    case 0: return kde_logpdf_h_kernel<NSC, 0, SG>;
    case 1: return kde_logpdf_h_kernel<NSC, 1, SG>;
    case 2: return kde_logpdf_h_kernel<NSC, 2, SG>;
    case 3: return kde_logpdf_h_kernel<NSC, 3, SG>;
    case 4: return kde_logpdf_h_kernel<NSC, 4, SG>;
  }
  return nullptr;
}

template <bool SG>
static logpdf_fn pick_nsc(int nsc, int kc) {
  switch (nsc) {  // nsc_of(dc_pad) for dc_pad in {8, 16, 24, 32, 64}
    case 1: return pick_kc<1, SG>(kc);
    case 2: return pick_kc<2, SG>(kc);
    case 3: return pick_kc<3, SG>(kc);
    case 4: return pick_kc<4, SG>(kc);
    case 8: return pick_kc<8, SG>(kc);
  }
  return nullptr;
}

logpdf_fn hbx_pick_h(int nsc, int kc, bool sg) { return sg ? pick_nsc<true>(nsc, kc) : pick_nsc<false>(nsc, kc); }
