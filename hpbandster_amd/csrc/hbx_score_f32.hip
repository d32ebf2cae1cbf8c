// hbx_score_f32.hip -- scoring kernel, f32 matrix-core continuous product + VALU categorical match
// (buckets with fewer than 16 continuous dims or non-integer categorical codes).
#include "hbx_common.h"
#include "hbx_kde_impl.h"

template <int DCP, int DUP, bool SIGNED>
__global__ __launch_bounds__(64 * MFMA_WAVES) void kde_logpdf_kernel(const double* __restrict__ cand, int64_t Nc,
                                                                    int32_t D, const KdeParams* __restrict__ P,
                                                                    const float* __restrict__ table,
                                                                    KdeEst* __restrict__ out) {
  constexpr int KP = kp_of(DCP);
  constexpr int NS = KP / 4;
  constexpr int CHF = chunk_floats(DCP, DUP);
  constexpr int NU = DUP > 0 ? DUP : 1;
  __shared__ __align__(16) float lds[2 * CHF];  // double-buffered observation chunks

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t cbase = ((int64_t)blockIdx.x * MFMA_WAVES + wave) * 16;  // this wave's 16 candidates
  const int n = P->n, dc = P->dc, du = P->du;
  const int ia = lane & 15, kq = lane >> 4;

  // A fragments: lane holds A[i = ia][k = 4s + kq]; A[i][0] = 1 (x C_j), A[i][1] = c_i, A[i][2+c] = x''_ic
  float a[NS];
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
  }
  // epilogue rows: the accumulator of lane holds candidates 4*kq + q (q = 0..3), observation ia
  float xu[4][NU];
  bool nanc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    int64_t ii = cbase + 4 * kq + q;
    if (ii >= Nc) ii = Nc - 1;
    const double* x = cand + ii * (int64_t)D;
#pragma unroll
    for (int u = 0; u < DUP; ++u) xu[q][u] = (u < du) ? cand_code(x[P->cat_dim[u]]) : -1.f;
    bool nn = P->nan_all != 0;
    for (int c = 0; c < P->nconst; ++c)
      if (x[P->const_dim[c]] != P->const_level[c]) nn = true;
    nanc[q] = nn;
  }
  float dl[NU], ng[NU];
#pragma unroll
  for (int u = 0; u < DUP; ++u) {
    dl[u] = (u < du) ? P->cat_delta[u] : 0.f;
    ng[u] = (u < du) ? P->cat_negf[u] : 0.f;
  }

  float S[4] = {0.f, 0.f, 0.f, 0.f}, Sn[4] = {0.f, 0.f, 0.f, 0.f};
  const int nchunks = (n + OBS_CHUNK - 1) / OBS_CHUNK;
  constexpr int NT = 64 * MFMA_WAVES;                 // threads per block
  constexpr int NV4 = CHF / 4;                        // float4 per chunk
  constexpr int PER = (NV4 + NT - 1) / NT;            // float4 per thread per chunk
  float4 pre[PER];
  // stage chunk 0; later chunks are prefetched into registers during the previous chunk's math
  {
    const float4* __restrict__ src = (const float4*)table;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int v = threadIdx.x + q * NT;
      if (v < NV4) ((float4*)lds)[v] = src[v];
    }
  }
  __syncthreads();

  // one 16x16 tile: B fragments and categorical codes of observation column jt*16 + ia
  auto load_tile = [&](const float* buf, int jt, float* b, float* xo) {
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2) b[s2] = buf[(4 * s2 + kq) * KROW + jt * 16 + ia];
#pragma unroll
    for (int u = 0; u < DUP; ++u) xo[u] = buf[KP * KROW + (jt * 16 + ia) * DUP + u];
  };
  auto epilogue = [&](const f32x4& acc, const float* xo, float* Sb, float* Snb) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float t = acc[q];
      float par = 0.f;
#pragma unroll
      for (int u = 0; u < DUP; ++u) {
        const float m = cat_match(xu[q][u], xo[u]);
        t = fmaf(dl[u], m, t);
        if (SIGNED) par = fmaf(m, ng[u], -fabsf(par));
      }
      const float e = __builtin_amdgcn_exp2f(t);
      Sb[q] += e;
      if (SIGNED) Snb[q] = fmaf(fabsf(par), e, Snb[q]);
    }
  };

  for (int c = 0; c < nchunks; ++c) {
    float* buf = lds + (c & 1) * CHF;
    const bool more = c + 1 < nchunks;
    if (more) {  // prefetch the next chunk into registers (lands during this chunk's math)
      const float4* __restrict__ src = (const float4*)(table + (int64_t)(c + 1) * CHF);
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int v = threadIdx.x + q * NT;
        if (v < NV4) pre[q] = src[v];
      }
    }
    float Sb[4] = {0.f, 0.f, 0.f, 0.f}, Snb[4] = {0.f, 0.f, 0.f, 0.f};
    // software pipeline over tile pairs: MFMAs of pair p+1 are issued before the VALU epilogue of p
    float b0[NS], b1[NS], xo0[NU], xo1[NU];
    f32x4 acc0, acc1;
    load_tile(buf, 0, b0, xo0);
    load_tile(buf, 1, b1, xo1);
    acc0 = f32x4{0.f, 0.f, 0.f, 0.f};
    acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s2], b0[s2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s2], b1[s2], acc1, 0, 0, 0);
    }
#pragma unroll
    for (int p = 0; p < OBS_CHUNK / 32; ++p) {
      f32x4 n0 = acc0, n1 = acc1;
      float c0[NU], c1[NU];
#pragma unroll
      for (int u = 0; u < DUP; ++u) {
        c0[u] = xo0[u];
        c1[u] = xo1[u];
      }
      if (p + 1 < OBS_CHUNK / 32) {
        load_tile(buf, 2 * p + 2, b0, xo0);
        load_tile(buf, 2 * p + 3, b1, xo1);
        acc0 = f32x4{0.f, 0.f, 0.f, 0.f};
        acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s2], b0[s2], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s2], b1[s2], acc1, 0, 0, 0);
        }
      }
      epilogue(n0, c0, Sb, Snb);
      epilogue(n1, c1, Sb, Snb);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      S[q] += Sb[q];
      if (SIGNED) Sn[q] += Snb[q];
    }
    if (more) {  // publish the prefetched chunk into the other buffer
      float4* dst = (float4*)(lds + ((c + 1) & 1) * CHF);
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int v = threadIdx.x + q * NT;
        if (v < NV4) dst[v] = pre[q];
      }
    }
    __syncthreads();
  }
  // reduce over the 16 lanes (observation columns) that share kq
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      S[q] += __shfl_xor(S[q], o);
      if (SIGNED) Sn[q] += __shfl_xor(Sn[q], o);
    }
  }
  // lane ia = q of group kq writes candidate 4*kq + q; c_i / bound of that candidate live in lane
  // (4*kq + q) & 15 + 16*anything of the A layout -> fetch with a shuffle
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
      if (!nq && Sq == Sq && Sq < 0x1p-64f) o.err = -1.f;  // rescue marker (kde_rescue_kernel)
      out[ii] = o;
    }
  }
}

template <int DCP, bool SG>
static logpdf_fn pick_du(int du_pad) {
  switch (du_pad) {
    case 0: return kde_logpdf_kernel<DCP, 0, SG>;
    case 4: return kde_logpdf_kernel<DCP, 4, SG>;
    case 8: return kde_logpdf_kernel<DCP, 8, SG>;
    case 16: return kde_logpdf_kernel<DCP, 16, SG>;
    case 32: return kde_logpdf_kernel<DCP, 32, SG>;
  }
  return nullptr;
}

template <bool SG>
static logpdf_fn pick_dc(int dc_pad, int du_pad) {
  switch (dc_pad) {
    case 0: return pick_du<0, SG>(du_pad);
    case 4: return pick_du<4, SG>(du_pad);
    case 8: return pick_du<8, SG>(du_pad);
    case 16: return pick_du<16, SG>(du_pad);
    case 24: return pick_du<24, SG>(du_pad);
    case 32: return pick_du<32, SG>(du_pad);
    case 64: return pick_du<64, SG>(du_pad);
  }
  return nullptr;
}

logpdf_fn hbx_pick_f32(int dc_pad, int du_pad, bool sg) {
  return sg ? pick_dc<true>(dc_pad, du_pad) : pick_dc<false>(dc_pad, du_pad);
}
