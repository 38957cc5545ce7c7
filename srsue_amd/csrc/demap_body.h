// demap_body.h -- equalisation + max-log soft demapping arithmetic shared by demap_kernel (demap.hip)
// and the fused demap -> rate de-matching path of rm_combine_kernel (rm.hip), so both produce the
// same LLRs (srslte_predecoding_single / _diversity + srslte_demod_soft_demodulate with sigma^2 = 0.5 +
// srslte_scrambling_f, inside srslte_pdsch_decode_rnti, /root/reference/ue/src/phy/phch_worker.cc:347).
#pragma once
#include "dl_common.h"

namespace mi {

// Equalisation, shared by every path that forms LLRs (demap_kernel, the fused staging and the direct form of
// rate de-matching, the single-LLR repetition path), so that all give the same floats.  Floating-point
// contraction is off here: the default (fast) lets the compiler fuse a multiply into an add or not depending
// on the surrounding code, which made two of these paths differ in the last bits; uncontracted, the
// arithmetic is also the oracle's (plain C, no FMA).
#if defined(__clang__)
#define MI_FP_EXACT _Pragma("clang fp contract(off)")
#else
#define MI_FP_EXACT
#endif
// TM1 MMSE: y h* / (|h|^2 + noise)
__device__ __forceinline__ float2 eq_single(float2 y, float2 h, float noise) {
  MI_FP_EXACT
  const float den = h.x * h.x + h.y * h.y + noise;
  return make_float2((y.x * h.x + y.y * h.y) / den, (y.y * h.x - y.x * h.y) / den);
}
// TM2 SFBC (Alamouti) pair: symbols x0 (k = 0) and x1 (k = 1) of REs ra / rb
__device__ __forceinline__ void eq_sfbc(float2 r0, float2 r1, float2 h00, float2 h01, float2 h10, float2 h11,
                                       float2* x0, float2* x1) {
  MI_FP_EXACT
  float hh = h00.x * h00.x + h00.y * h00.y + h11.x * h11.x + h11.y * h11.y;
  if (hh <= 0.f) hh = 1e-9f;
  const float sc = 1.41421356237309504880f / hh;
  *x0 = make_float2(sc * ((h00.x * r0.x + h00.y * r0.y) + (h11.x * r1.x + h11.y * r1.y)),
                    sc * ((h00.x * r0.y - h00.y * r0.x) + (h11.y * r1.x - h11.x * r1.y)));
  *x1 = make_float2(sc * (-(h10.x * r0.x + h10.y * r0.y) + (h01.x * r1.x + h01.y * r1.y)),
                    sc * (-(h10.y * r0.x - h10.x * r0.y) + (h01.x * r1.y - h01.y * r1.x)));
}

template <int QM>
__device__ __forceinline__ float pam_level(int lab) {
  // lab: this dimension's bits, MSB first (36.211 7.1 Gray mapping, separable I/Q)
  if constexpr (QM == 2) {
    return (1 - 2 * (lab & 1)) * 0.70710678118654752440f;
  } else if constexpr (QM == 4) {
    const int b0 = (lab >> 1) & 1, b1 = lab & 1;
    return (float)((1 - 2 * b0) * (1 + 2 * b1)) * 0.31622776601683793320f;
  } else {
    const int b0 = (lab >> 2) & 1, b1 = (lab >> 1) & 1, b2 = lab & 1;
    return (float)((1 - 2 * b0) * (4 - (1 - 2 * b1) * (2 - (1 - 2 * b2)))) * 0.15430334996209191026f;
  }
}

// writes the QM/2 LLRs of one dimension at llr[0], llr[2], llr[4] (I at even, Q at odd slots)
template <int QM>
__device__ __forceinline__ void demap_dim(float x, float* llr) {
  MI_FP_EXACT
  constexpr int NB = QM / 2, NL = 1 << NB;
  float d2[NL];
#pragma unroll
  for (int lab = 0; lab < NL; lab++) {
    const float d = x - pam_level<QM>(lab);
    d2[lab] = d * d;
  }
#pragma unroll
  for (int j = 0; j < NB; j++) {
    float m0 = 3.0e38f, m1 = 3.0e38f;
#pragma unroll
    for (int lab = 0; lab < NL; lab++) {
      if ((lab >> (NB - 1 - j)) & 1) m1 = fminf(m1, d2[lab]); else m0 = fminf(m0, d2[lab]);
    }
    llr[2 * j] = (m0 - m1) * 2.0f;   // / sigma^2, sigma^2 = 0.5
  }
}

// LLR of bit j (MSB first) of one dimension: demap_dim's arithmetic for that bit alone (no dynamic
// register-array index)
template <int QM>
__device__ __forceinline__ float demap_bit(float x, uint32_t j) {
  MI_FP_EXACT
  constexpr int NB = QM / 2, NL = 1 << NB;
  float d2[NL];
#pragma unroll
  for (int lab = 0; lab < NL; lab++) {
    const float d = x - pam_level<QM>(lab);
    d2[lab] = d * d;
  }
  float out = 0.0f;
#pragma unroll
  for (int jj = 0; jj < NB; jj++) {
    float m0 = 3.0e38f, m1 = 3.0e38f;
#pragma unroll
    for (int lab = 0; lab < NL; lab++) {
      if ((lab >> (NB - 1 - jj)) & 1) m1 = fminf(m1, d2[lab]); else m0 = fminf(m0, d2[lab]);
    }
    out = (uint32_t)jj == j ? (m0 - m1) * 2.0f : out;
  }
  return out;
}

// one LLR of a PDSCH subframe: bit `gi` of the subframe's LLR stream (after descrambling), computed
// from the grid and channel estimates exactly as demap_kernel computes it (TM1: one RE per Qm bits; TM2:
// one SFBC RE pair per 2 Qm bits)
template <int QM>
__device__ __forceinline__ float demap_llr(const MiPdschDesc& pd, uint32_t gi, const float2* __restrict__ g,
                                           const float2* __restrict__ c0, const float2* __restrict__ c1,
                                           const uint32_t* __restrict__ re, const uint32_t* __restrict__ scr,
                                           float noise) {
  const uint32_t s = gi / QM, b = gi - s * QM;   // data symbol, bit within it
  float2 x;
  if (pd.tm != 2) {
    const uint32_t r = re[s];
    x = eq_single(g[r], c0[r], noise);
  } else {
    const uint32_t u = s >> 1, ra = re[2 * u], rb = re[2 * u + 1];
    float2 x0, x1;
    eq_sfbc(g[ra], g[rb], c0[ra], c0[rb], c1[ra], c1[rb], &x0, &x1);
    x = (s & 1) == 0 ? x0 : x1;
  }
  const float v = demap_bit<QM>((b & 1) ? x.y : x.x, b >> 1);   // I: even bits, Q: odd bits
  return ((scr[gi >> 5] >> (gi & 31)) & 1u) ? -v : v;
}

}  // namespace mi
