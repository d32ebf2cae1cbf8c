// hbx_score_oh.hip -- scoring kernel, f32 matrix-core continuous product + f16 one-hot categorical product.
#include "hbx_common.h"
#include "hbx_kde_impl.h"

// One-hot mode: the categorical sum  sum_u delta_u [x_u == X_u]  is a second matrix product,
// (candidate one-hot) x (delta-weighted observation one-hot), on the f16 matrix cores: operands are
// 0/1 and the f16 hi+lo parts of delta_u, so every product is exact and only the fp32 accumulation
// rounds.  It continues the same accumulator as the f32 continuous product, leaving the VALU only
// exp2 and the running sums.  Signed KDEs add one more f16 product that counts matches in dims with
// a negative match weight (the sign of the term is (-1)^count).

template <int DCP, int KC, bool SIGNED>
__global__ __launch_bounds__(64 * MFMA_WAVES) void kde_logpdf_oh_kernel(const double* __restrict__ cand,
                                                                       int64_t Nc, int32_t D,
                                                                       const KdeParams* __restrict__ P,
                                                                       const float* __restrict__ table,
                                                                       KdeEst* __restrict__ out) {
  constexpr int KP = kp_of(DCP);
  constexpr int NS = KP / 4;
  constexpr int W = KC * 32;  // one-hot halves per observation
  constexpr int CHF = chunk_floats(DCP, 0, KC, SIGNED ? 1 : 0);
  __shared__ __align__(16) float lds[2 * CHF];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t cbase = ((int64_t)blockIdx.x * MFMA_WAVES + wave) * 16;
  const int n = P->n, dc = P->dc;
  const int ia = lane & 15, kq = lane >> 4;

  float a[NS];
  f16x8 ah[KC];
  float ci_a = 0.f, bnd_a = 0.f;
  {
    int64_t ii = cbase + ia;
    if (ii >= Nc) ii = Nc - 1;
    const double* x = cand + ii * (int64_t)D;
    for (int k = 0; k < dc; ++k) {
      const float v = (float)(P->cont_scale[k] * (x[P->cont_dim[k]] - P->center[k]));
      ci_a = fmaf(-v, v, ci_a);
      bnd_a = fmaf(2.f * fabsf(v), P->xmax[k], bnd_a);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int k = 4 * s + kq;
      float v = 0.f;
      if (k == 0) {
        v = 1.f;
      } else if (k == 1) {
        v = ci_a;
      } else if (k - 2 < dc) {
        const int c = k - 2;
        v = 2.f * (float)(P->cont_scale[c] * (x[P->cont_dim[c]] - P->center[c]));
      }
      a[s] = v;
    }
    // candidate one-hot: lane holds A[row ia][k = 32 s + 8 kq + j]
    const int tot = P->oh_total;
#pragma unroll
    for (int s = 0; s < KC; ++s) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int t = (32 * s + 8 * kq + j) >> 1;
        float v = 0.f;
        if (t < tot && x[P->cat_dim[P->oh_dim[t]]] == (double)P->oh_level[t]) v = 1.f;
        ah[s][j] = (_Float16)v;
      }
    }
  }
  bool nanc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    int64_t ii = cbase + 4 * kq + q;
    if (ii >= Nc) ii = Nc - 1;
    const double* x = cand + ii * (int64_t)D;
    bool nn = P->nan_all != 0;
    for (int c = 0; c < P->nconst; ++c)
      if (x[P->const_dim[c]] != P->const_level[c]) nn = true;
    nanc[q] = nn;
  }

  float S[4] = {0.f, 0.f, 0.f, 0.f}, Sn[4] = {0.f, 0.f, 0.f, 0.f};
  const int nchunks = (n + OBS_CHUNK - 1) / OBS_CHUNK;
  constexpr int NT = 64 * MFMA_WAVES;
  constexpr int NV4 = CHF / 4;
  constexpr int PER = (NV4 + NT - 1) / NT;
  float4 pre[PER];
  {
    const float4* __restrict__ src = (const float4*)table;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int v = threadIdx.x + q * NT;
      if (v < NV4) ((float4*)lds)[v] = src[v];
    }
  }
  __syncthreads();

  // accumulate one 16x16 tile: f32 continuous product, then the f16 one-hot product
  auto tile = [&](const float* buf, int jt, f32x4& acc, f32x4& accp) {
    const _Float16* ohb = (const _Float16*)(buf + KP * KROW);
    acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; ++s)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], buf[(4 * s + kq) * KROW + jt * 16 + ia], acc, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      const f16x8 b = *(const f16x8*)(ohb + (jt * 16 + ia) * W + 32 * s + 8 * kq);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[s], b, acc, 0, 0, 0);
    }
    if (SIGNED) {
      accp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KC; ++s) {
        const f16x8 b = *(const f16x8*)(ohb + OBS_CHUNK * W + (jt * 16 + ia) * W + 32 * s + 8 * kq);
        accp = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[s], b, accp, 0, 0, 0);
      }
    }
  };
  auto epilogue = [&](const f32x4& acc, const f32x4& accp, float* Sb, float* Snb) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float e = __builtin_amdgcn_exp2f(acc[q]);
      Sb[q] += e;
      if (SIGNED) {
        const float odd = 2.f * __builtin_amdgcn_fractf(0.5f * accp[q]);  // count mod 2
        Snb[q] = fmaf(odd, e, Snb[q]);
      }
    }
  };

  for (int c = 0; c < nchunks; ++c) {
    float* buf = lds + (c & 1) * CHF;
    const bool more = c + 1 < nchunks;
    if (more) {
      const float4* __restrict__ src = (const float4*)(table + (int64_t)(c + 1) * CHF);
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int v = threadIdx.x + q * NT;
        if (v < NV4) pre[q] = src[v];
      }
    }
    float Sb[4] = {0.f, 0.f, 0.f, 0.f}, Snb[4] = {0.f, 0.f, 0.f, 0.f};
    f32x4 acc0, acc1, ap0, ap1;
    tile(buf, 0, acc0, ap0);
    tile(buf, 1, acc1, ap1);
#pragma unroll
    for (int p = 0; p < OBS_CHUNK / 32; ++p) {
      const f32x4 n0 = acc0, n1 = acc1, m0 = ap0, m1 = ap1;
      if (p + 1 < OBS_CHUNK / 32) {
        tile(buf, 2 * p + 2, acc0, ap0);
        tile(buf, 2 * p + 3, acc1, ap1);
      }
      epilogue(n0, m0, Sb, Snb);
      epilogue(n1, m1, Sb, Snb);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      S[q] += Sb[q];
      if (SIGNED) Sn[q] += Snb[q];
    }
    if (more) {
      float4* dst = (float4*)(lds + ((c + 1) & 1) * CHF);
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int v = threadIdx.x + q * NT;
        if (v < NV4) dst[v] = pre[q];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      S[q] += __shfl_xor(S[q], o);
      if (SIGNED) Sn[q] += __shfl_xor(Sn[q], o);
    }
  }
  const int src_lane = (4 * kq + (ia & 3)) & 15;
  const float ci_q = __shfl(ci_a, src_lane);
  const float bnd_q = __shfl(bnd_a, src_lane);
  if (ia < 4) {
    const int q = ia;
    const int64_t ii = cbase + 4 * kq + q;
    float Sq = S[0], Snq = Sn[0];
    bool nq = nanc[0];
    if (q == 1) { Sq = S[1]; Snq = Sn[1]; nq = nanc[1]; }
    if (q == 2) { Sq = S[2]; Snq = Sn[2]; nq = nanc[2]; }
    if (q == 3) { Sq = S[3]; Snq = Sn[3]; nq = nanc[3]; }
    if (ii < Nc) {
      KdeEst o = finish_est(P, Sq, Snq, 0.f, nq, ci_q, bnd_q, SIGNED, OBS_CHUNK / 16);
      if (!nq && Sq == Sq && Sq < 0x1p-64f) o.err = -1.f;
      out[ii] = o;
    }
  }
}

template <int DCP, bool SG>
static logpdf_fn pick_kc(int kc) {
  switch (kc) {
    case 1: return kde_logpdf_oh_kernel<DCP, 1, SG>;
    case 2: return kde_logpdf_oh_kernel<DCP, 2, SG>;
    case 3: return kde_logpdf_oh_kernel<DCP, 3, SG>;
    case 4: return kde_logpdf_oh_kernel<DCP, 4, SG>;
  }
  return nullptr;
}

template <bool SG>
static logpdf_fn pick_dc(int dc_pad, int kc) {
  switch (dc_pad) {
    case 0: return pick_kc<0, SG>(kc);
    case 4: return pick_kc<4, SG>(kc);
    case 8: return pick_kc<8, SG>(kc);
    case 16: return pick_kc<16, SG>(kc);
    case 24: return pick_kc<24, SG>(kc);
    case 32: return pick_kc<32, SG>(kc);
    case 64: return pick_kc<64, SG>(kc);
  }
  return nullptr;
}

logpdf_fn hbx_pick_oh(int dc_pad, int kc, bool sg) { return sg ? pick_dc<true>(dc_pad, kc) : pick_dc<false>(dc_pad, kc); }
