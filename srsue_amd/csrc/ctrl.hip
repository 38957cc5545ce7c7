// ctrl.hip -- DL control channels on the GPU: PCFICH -> CFI, PDCCH soft-bit
// extraction, DCI blind search (rate de-matching + tail-biting Viterbi + RNTI-masked CRC16), PHICH.
//
// Replaces the host work behind srslte_pdcch_extract_llr (/root/reference/ue/src/phy/
// phch_worker.cc:260) and srslte_ue_dl_find_dl_dci_type / _find_ul_dci (:293, :426); the arithmetic
// contract is oracle/o_ctrl.c's (Viterbi: float metrics, same operation order and tie rules, so
// decisions are bit-identical on identical soft bits).
//
// MI355X layout:
//   * pcfich_kernel: one wavefront per subframe (16 REs, 32 soft bits, 3 code-word correlations);
//   * pdcch_llr_kernel: one thread per REG (4 REs -> 8 soft bits), REG -> logical quadruplet and the
//     scrambling words from per-(cell, sf, cfi) tables; writes the soft bits in logical CCE order;
//   * dci_search_kernel: one wavefront per (candidate, DCI size) job.  Lanes own coded-bit positions
//     for the rate de-matching (each position sums its e_k in increasing k, as the serial loop), then
//     the 64 lanes ARE the 64 trellis states: predecessor metrics by cross-lane shuffles, survivor
//     bits by ballot into LDS, best final state by a (metric, index) butterfly, traceback and CRC16
//     by one lane.
#include "ctrl.h"
#include "kernels.h"

namespace mi {

__device__ __forceinline__ void eq_tm1(float2 y, float2 h, float noise, float2& x) {
  const float den = h.x * h.x + h.y * h.y + noise;
  x.x = (y.x * h.x + y.y * h.y) / den;
  x.y = (y.y * h.x - y.x * h.y) / den;
}

// Alamouti / SFBC combining of an RE pair (the PDSCH demapper's arithmetic, demap.hip)
__device__ __forceinline__ void eq_tm2(float2 r0, float2 r1, float2 h00, float2 h01, float2 h10, float2 h11, float2& x0,
                                       float2& x1) {
  float hh = h00.x * h00.x + h00.y * h00.y + h11.x * h11.x + h11.y * h11.y;
  if (hh <= 0.f) hh = 1e-9f;
  const float s = 1.41421356237f / hh;
  x0.x = s * ((h00.x * r0.x + h00.y * r0.y) + (h11.x * r1.x + h11.y * r1.y));
  x0.y = s * ((h00.x * r0.y - h00.y * r0.x) + (h11.y * r1.x - h11.x * r1.y));
  x1.x = s * (-(h10.x * r0.x + h10.y * r0.y) + (h01.x * r1.x + h01.y * r1.y));
  x1.y = s * (-(h10.y * r0.x - h10.x * r0.y) + (h01.x * r1.y - h01.y * r1.x));
}

// QPSK max-log soft bits, LLR > 0 => bit 1 (same scale as the PDSCH demapper)
__device__ __forceinline__ void qpsk_llr(float2 x, float* l) {
  const float a = 0.70710678118f;
  l[0] = ((x.x - a) * (x.x - a) - (x.x + a) * (x.x + a)) * 2.0f;
  l[1] = ((x.y - a) * (x.y - a) - (x.y + a) * (x.y + a)) * 2.0f;
}

// 4 REs of one REG / PCFICH quadruplet -> 4 equalised symbols
__device__ __forceinline__ void eq_quad(const float2* g, const float2* c0, const float2* c1, const uint32_t* re,
                                        bool tm2, float noise, float2 (&x)[4]) {
  if (!tm2) {
#pragma unroll
    for (int j = 0; j < 4; j++) eq_tm1(g[re[j]], c0[re[j]], noise, x[j]);
  } else {
#pragma unroll
    for (int j = 0; j < 4; j += 2)
      eq_tm2(g[re[j]], g[re[j + 1]], c0[re[j]], c0[re[j + 1]], c1[re[j]], c1[re[j + 1]], x[j], x[j + 1]);
  }
}

__global__ __launch_bounds__(64) void pcfich_kernel(const float2* __restrict__ grid, const float2* __restrict__ ce,
                                                   const MiCtrlSf* __restrict__ sfs,
                                                   const uint32_t* __restrict__ cdata, uint32_t* __restrict__ cfi) {
  __shared__ float llr[32];
  const MiCtrlSf d = sfs[blockIdx.x];
  const uint32_t t = threadIdx.x;
  const float2* g = grid + d.grid_off;
  const float2* c0 = ce + d.ce_off;
  const float2* c1 = c0 + d.plane;
  const uint32_t* k16 = cdata + d.pcfich_off;
  const uint32_t sc = cdata[d.pcfich_off + 16];   // 32 scrambling bits
  if (t < 4) {
    float2 x[4];
    eq_quad(g, c0, c1, k16 + 4 * t, d.ports == 2, 0.0f, x);
#pragma unroll
    for (int j = 0; j < 4; j++) {
      float l[2];
      qpsk_llr(x[j], l);
      const uint32_t b = 8 * t + 2 * j;
      llr[b] = ((sc >> b) & 1u) ? -l[0] : l[0];
      llr[b + 1] = ((sc >> (b + 1)) & 1u) ? -l[1] : l[1];
    }
  }
  __syncthreads();
  if (t == 0) {
    // CFI code words (36.212 Table 5.3.4-1): 32 bits repeating <0,1,1>, <1,0,1>, <1,1,0>
    int best = 0;
    float bs = -3.0e38f;
    for (int c = 1; c <= 3; c++) {
      float s = 0.0f;
      for (int i = 0; i < 32; i++) {
        const int bit = (c == 1) ? (i % 3 != 0) : (c == 2) ? (i % 3 != 1) : (i % 3 != 2);
        s = s + (bit ? llr[i] : -llr[i]);
      }
      if (s > bs) { bs = s; best = c; }
    }
    cfi[blockIdx.x] = (uint32_t)best;
  }
}

__global__ __launch_bounds__(256) void pdcch_llr_kernel(const float2* __restrict__ grid, const float2* __restrict__ ce,
                                                       const MiCtrlSf* __restrict__ sfs,
                                                       const uint32_t* __restrict__ cdata, float* __restrict__ llr,
                                                       float noise) {
  const MiCtrlSf d = sfs[blockIdx.y];
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= d.M) return;
  const float2* g = grid + d.grid_off;
  const float2* c0 = ce + d.ce_off;
  const float2* c1 = c0 + d.plane;
  const uint32_t* re = cdata + d.reg_off + 4 * i;
  const uint32_t lg = cdata[d.reg_off + 4 * d.M + i];
  float2 x[4];
  eq_quad(g, c0, c1, re, d.ports == 2, noise, x);
  const uint32_t sw = cdata[d.scr_off + lg / 4] >> (8 * (lg % 4));   // 8 scrambling bits of quadruplet lg
  float* o = llr + d.llr_off + 8 * lg;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    float l[2];
    qpsk_llr(x[j], l);
    o[2 * j] = ((sw >> (2 * j)) & 1u) ? -l[0] : l[0];
    o[2 * j + 1] = ((sw >> (2 * j + 1)) & 1u) ? -l[1] : l[1];
  }
}

// generators 133, 171, 165 (octal): bit 6 <-> c_k, bit 0 <-> c_{k-6}
__device__ __forceinline__ int par7(uint32_t x) { return __popc(x) & 1; }

__global__ __launch_bounds__(64) void dci_search_kernel(const float* __restrict__ llr,
                                                       const MiDciJob* __restrict__ jobs,
                                                       const uint32_t* __restrict__ cdata,
                                                       MiDciRes* __restrict__ res) {
  constexpr int DMAX = DCI_MAX_BITS + 16;
  __shared__ float d[3 * DMAX];
  __shared__ uint64_t surv[3 * DMAX];
  __shared__ uint8_t c[DMAX];
  const MiDciJob j = jobs[blockIdx.x];
  const uint32_t t = threadIdx.x, D = j.D, E = 72 * j.L;
  const float* e = llr + j.llr_off + 72 * j.ncce;
  const uint32_t* rank = cdata + j.rank_off;
  // rate de-matching: coded bit p receives e_k for k = rank(p), rank(p) + 3D, ... < E
  for (uint32_t p = t; p < 3 * D; p += 64) {
    float s = 0.0f;
    for (uint32_t k = rank[p]; k < E; k += 3 * D) s = s + e[k];
    d[p] = s;
  }
  __syncthreads();
  // Viterbi over three circular copies; lane t = state t
  const uint32_t u = t >> 5;
  const uint32_t s0 = (t << 1) & 63u, s1 = s0 | 1u;
  const uint32_t r0 = (u << 6) | s0, r1 = (u << 6) | s1;
  const int o00 = par7(r0 & 0133u), o01 = par7(r0 & 0171u), o02 = par7(r0 & 0165u);
  const int o10 = par7(r1 & 0133u), o11 = par7(r1 & 0171u), o12 = par7(r1 & 0165u);
  float pm = 0.0f;
  for (uint32_t k = 0, kk = 0; k < 3 * D; k++) {
    const float v0 = d[kk], v1 = d[D + kk], v2 = d[2 * D + kk];
    float bm0 = 0.0f, bm1 = 0.0f;
    bm0 = bm0 + (o00 ? v0 : -v0); bm0 = bm0 + (o01 ? v1 : -v1); bm0 = bm0 + (o02 ? v2 : -v2);
    bm1 = bm1 + (o10 ? v0 : -v0); bm1 = bm1 + (o11 ? v1 : -v1); bm1 = bm1 + (o12 ? v2 : -v2);
    const float m0 = __shfl(pm, (int)s0, 64) + bm0;
    const float m1 = __shfl(pm, (int)s1, 64) + bm1;
    const bool pick = m1 > m0;
    pm = pick ? m1 : m0;
    const uint64_t b = __ballot(pick);
    if (t == 0) surv[k] = b;
    if (++kk == D) kk = 0;
  }
  // best final state: largest metric, lowest index on ties
  float bv = pm;
  uint32_t bi = t;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const uint32_t oi = __shfl_xor(bi, o, 64);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  __syncthreads();
  if (t == 0) {
    uint32_t st = bi;
    for (int k = (int)(3 * D) - 1; k >= 0; k--) {
      if ((uint32_t)k >= D && (uint32_t)k < 2 * D) c[k - D] = (uint8_t)(st >> 5);
      st = ((st << 1) & 63u) | (uint32_t)((surv[k] >> st) & 1u);
    }
    // CRC16 (g = 0x1021, zero init) over the payload; the attached bits are CRC ^ RNTI
    const uint32_t A = j.A;
    uint32_t reg = 0;
    for (uint32_t i = 0; i < A; i++) {
      const uint32_t fb = ((reg >> 15) ^ c[i]) & 1u;
      reg = ((reg << 1) & 0xFFFFu) ^ (fb ? 0x1021u : 0u);
    }
    uint32_t rx = 0;
    for (uint32_t i = 0; i < 16; i++) rx = (rx << 1) | c[A + i];
    MiDciRes r;
    r.found = ((reg ^ rx) & 0xFFFFu) == j.rnti;
    r.bits[0] = r.bits[1] = 0;
    for (uint32_t i = 0; i < A; i++) r.bits[i >> 5] |= (uint32_t)c[i] << (31 - (i & 31));
    res[blockIdx.x] = r;
  }
}

// PHICH (36.211 6.9): one wavefront per subframe; lanes equalise the group's 12 REs (SFBC: 6 pairs),
// lane 0 despreads them in order i = 0..11 (oracle or_phich_soft's contract, in fp32):
// s = sum_i Re(conj(w(i mod 4)) (1 - 2 c(i)) x(i) (1 - j) / sqrt2), soft HI = -s (> 0 favours ACK)
__global__ __launch_bounds__(64) void phich_kernel(const float2* __restrict__ grid, const float2* __restrict__ ce,
                                                  const MiCtrlSf* __restrict__ sfs,
                                                  const uint32_t* __restrict__ cdata, float* __restrict__ soft) {
  __shared__ float2 x[12];
  const MiCtrlSf d = sfs[blockIdx.x];
  const uint32_t t = threadIdx.x;
  const float2* g = grid + d.grid_off;
  const float2* c0 = ce + d.ce_off;
  const float2* c1 = c0 + d.plane;
  const uint32_t* re = cdata + d.phich_off;
  if (d.ports == 2) {
    if (t < 6) {
      float2 a, b;
      const uint32_t r0 = re[2 * t], r1 = re[2 * t + 1];
      eq_tm2(g[r0], g[r1], c0[r0], c0[r1], c1[r0], c1[r1], a, b);
      x[2 * t] = a;
      x[2 * t + 1] = b;
    }
  } else if (t < 12) {
    const float2 h = c0[re[t]];
    float den = h.x * h.x + h.y * h.y;
    if (den <= 0.f) den = 1e-9f;
    const float2 y = g[re[t]];
    x[t] = make_float2((y.x * h.x + y.y * h.y) / den, (y.y * h.x - y.x * h.y) / den);
  }
  __syncthreads();
  if (t == 0) {
    const uint32_t cs = re[12], seq = re[13];
    float s = 0.0f;
    for (int i = 0; i < 12; i++) {
      // w(i mod 4) of Table 6.9.1-2: sign pattern by seq & 3, times j for seq >= 4
      const int c = i & 3, m = (int)(seq & 3);
      const float sw = ((m == 1 && (c & 1)) || (m == 2 && c >= 2) || (m == 3 && (c == 1 || c == 2))) ? -1.f : 1.f;
      const float wr = seq < 4 ? sw : 0.f, wi = seq < 4 ? 0.f : sw;
      const float yr = wr * x[i].x + wi * x[i].y, yi = wr * x[i].y - wi * x[i].x;
      const float sg = ((cs >> i) & 1u) ? -1.f : 1.f;
      s = s + sg * (yr + yi) * 0.70710678118654752f;
    }
    soft[blockIdx.x] = -s;
  }
}

void launch_phich(const float2* grid, const float2* ce, const MiCtrlSf* sfs, const uint32_t* cdata, float* soft,
                  uint32_t n_sf, hipStream_t st) {
  if (!n_sf) return;
  hipLaunchKernelGGL(phich_kernel, dim3(n_sf), dim3(64), 0, st, grid, ce, sfs, cdata, soft);
}

void launch_pcfich(const float2* grid, const float2* ce, const MiCtrlSf* sfs, const uint32_t* cdata, uint32_t* cfi,
                   uint32_t n_sf, hipStream_t st) {
  if (!n_sf) return;
  hipLaunchKernelGGL(pcfich_kernel, dim3(n_sf), dim3(64), 0, st, grid, ce, sfs, cdata, cfi);
}
void launch_pdcch_llr(const float2* grid, const float2* ce, const MiCtrlSf* sfs, const uint32_t* cdata, float* llr,
                      uint32_t n_sf, uint32_t max_regs, float noise, hipStream_t st) {
  if (!n_sf || !max_regs) return;
  hipLaunchKernelGGL(pdcch_llr_kernel, dim3((max_regs + 255) / 256, n_sf), dim3(256), 0, st, grid, ce, sfs, cdata, llr,
                     noise);
}
void launch_dci_search(const float* llr, const MiDciJob* jobs, const uint32_t* cdata, MiDciRes* res, uint32_t n_jobs,
                       hipStream_t st) {
  if (!n_jobs) return;
  hipLaunchKernelGGL(dci_search_kernel, dim3(n_jobs), dim3(64), 0, st, llr, jobs, cdata, res);
}

}  // namespace mi
