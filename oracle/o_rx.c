/*
 * o_rx.c -- PDSCH receive chain of the oracle (TEST INFRASTRUCTURE ONLY).
 *
 * Restates what srsUE reaches through
 *   srslte_ue_dl_decode_fft_estimate  (/root/reference/ue/src/phy/phch_worker.cc:254)
 *     = ofdm_rx_sf -> chest_dl_estimate -> PCFICH (CFI)
 *   srslte_pdsch_decode_rnti          (phch_worker.cc:347-348, noise_estimate = 0.01 at :340)
 *     = RE gather -> predecoding (single / diversity) -> demod_soft -> descramble -> dlsch decode
 * with the conventions of SURVEY.md 8a.  Computation in double, outputs float.
 *
 * Conventions that the GPU path matches (all [X]-tagged in SURVEY.md, i.e. parity unpinned):
 *   OFDM RX : unnormalised forward DFT, CP skipped, subcarrier k -> bin k-6N_RB (k<6N_RB) else
 *             k-6N_RB+1 (DC skipped); grid row-major [symbol][subcarrier].
 *   chest   : LS p = y conj(r); 3-tap smoothing [0.1 0.8 0.1] (edge taps renormalised);
 *             linear interpolation in frequency (edge extrapolation) on pilot symbols
 *             {0,4,7,11}, then linear interpolation / extrapolation in time.
 *             noise = mean |p - p_smooth|^2, rsrp = mean |p|^2 (port 0), rssi = mean over
 *             pilot symbols of sum_k |y|^2, rsrq = N_RB rsrp / rssi, snr = rsrp / noise.
 *   TM1     : x = y conj(h) / (|h|^2 + noise)
 *   TM2     : x0 = sqrt2 (h00* r0 + h11 r1*) / hh, x1 = sqrt2 (-h10 r0* + h01* r1) / hh,
 *             hh = |h00|^2 + |h11|^2 (srsLTE predecoding_diversity, 2 ports)
 *   demod   : max-log, LLR = (min_{b=0} d^2 - min_{b=1} d^2) / sigma^2, sigma^2 = 0.5 (LLR>0 => 1)
 */
#include "oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

double or_pam_level(const uint8_t *b, uint32_t Qm);
void or_pcfich_k(const or_cell_t *c, uint32_t *k_out);
uint32_t or_pcfich_cinit(const or_cell_t *c, uint32_t sf);
void or_cfi_codeword(uint32_t cfi, uint8_t *b);

int or_ofdm_rx(const or_cell_t *c, const float *iq, float *grid) {
  const int N = or_symbol_sz(c->nof_prb);
  const uint32_t W = 12 * c->nof_prb;
  if (N < 0) return -1;
  double *x = (double *)malloc(sizeof(double) * 2 * N), *X = (double *)malloc(sizeof(double) * 2 * N);
  size_t pos = 0;
  for (uint32_t l = 0; l < OR_NSYMB; l++) {
    pos += (size_t)or_cp_len((uint32_t)N, l % 7);
    for (int n = 0; n < N; n++) { x[2 * n] = iq[2 * (pos + n)]; x[2 * n + 1] = iq[2 * (pos + n) + 1]; }
    pos += (size_t)N;
    or_dft(x, X, N, 0);
    for (uint32_t k = 0; k < W; k++) {
      int bin = (k < W / 2) ? (int)(N - W / 2 + k) : (int)(k - W / 2 + 1);
      grid[2 * (l * W + k)] = (float)X[2 * bin];
      grid[2 * (l * W + k) + 1] = (float)X[2 * bin + 1];
    }
  }
  free(x); free(X);
  return 0;
}

static const uint32_t PILOT_L[4] = {0, 4, 7, 11};
#define SMOOTH_W1 0.1
#define SMOOTH_W0 0.8

int or_chest(const or_cell_t *c, uint32_t sf, const float *grid, float *ce, float *metrics) {
  const uint32_t W = 12 * c->nof_prb, NP = 2 * c->nof_prb;
  double *hp = (double *)malloc(sizeof(double) * 2 * NP), *hs = (double *)malloc(sizeof(double) * 2 * NP);
  double *hf = (double *)malloc(sizeof(double) * 2 * 4 * W);
  float rs[4 * OR_NRB_MAX];
  double noise_acc = 0, rsrp_acc = 0, rssi_acc = 0;
  uint32_t noise_n = 0, rsrp_n = 0;
  for (uint32_t p = 0; p < c->nof_ports; p++) {
    for (int i = 0; i < 4; i++) {
      uint32_t l = PILOT_L[i], lp = l % 7;
      uint32_t v = (p == 0) ? (lp == 0 ? 0 : 3) : (lp == 0 ? 3 : 0);
      uint32_t off = (v + c->id % 6) % 6;
      or_crs_seq(c->id, 2 * sf + l / 7, lp, rs);
      for (uint32_t m = 0; m < NP; m++) {
        uint32_t mp = m + OR_NRB_MAX - c->nof_prb, k = 6 * m + off;
        double yr = grid[2 * (l * W + k)], yi = grid[2 * (l * W + k) + 1];
        double rr = rs[2 * mp], ri = rs[2 * mp + 1];
        hp[2 * m] = yr * rr + yi * ri;          /* y * conj(r) */
        hp[2 * m + 1] = yi * rr - yr * ri;
        if (p == 0) { rsrp_acc += hp[2 * m] * hp[2 * m] + hp[2 * m + 1] * hp[2 * m + 1]; rsrp_n++; }
      }
      for (uint32_t m = 0; m < NP; m++) {
        for (int q = 0; q < 2; q++) {
          double s;
          if (m == 0) s = (SMOOTH_W0 * hp[q] + SMOOTH_W1 * hp[2 + q]) / (SMOOTH_W0 + SMOOTH_W1);
          else if (m == NP - 1) s = (SMOOTH_W1 * hp[2 * (m - 1) + q] + SMOOTH_W0 * hp[2 * m + q]) / (SMOOTH_W0 + SMOOTH_W1);
          else s = SMOOTH_W1 * hp[2 * (m - 1) + q] + SMOOTH_W0 * hp[2 * m + q] + SMOOTH_W1 * hp[2 * (m + 1) + q];
          hs[2 * m + q] = s;
        }
        double dr = hp[2 * m] - hs[2 * m], di = hp[2 * m + 1] - hs[2 * m + 1];
        noise_acc += dr * dr + di * di; noise_n++;
      }
      /* frequency interpolation */
      for (uint32_t k = 0; k < W; k++) {
        int m = ((int)k - (int)off) / 6;
        if ((int)k < (int)off) m = 0;
        if (m > (int)NP - 2) m = (int)NP - 2;
        double frac = ((double)k - (double)(6 * m + off)) / 6.0;
        hf[2 * (i * W + k)] = hs[2 * m] + frac * (hs[2 * (m + 1)] - hs[2 * m]);
        hf[2 * (i * W + k) + 1] = hs[2 * m + 1] + frac * (hs[2 * (m + 1) + 1] - hs[2 * m + 1]);
      }
    }
    /* time interpolation onto all 14 symbols */
    float *cp = ce + (size_t)p * OR_NSYMB * W * 2;
    for (uint32_t l = 0; l < OR_NSYMB; l++) {
      int ia, ib;
      if (l <= 4) { ia = 0; ib = 1; } else if (l <= 7) { ia = 1; ib = 2; } else { ia = 2; ib = 3; }
      double t = ((double)l - PILOT_L[ia]) / (double)(PILOT_L[ib] - PILOT_L[ia]);
      for (uint32_t k = 0; k < W; k++) {
        double ar = hf[2 * (ia * W + k)], ai = hf[2 * (ia * W + k) + 1];
        double br = hf[2 * (ib * W + k)], bi = hf[2 * (ib * W + k) + 1];
        cp[2 * (l * W + k)] = (float)(ar + t * (br - ar));
        cp[2 * (l * W + k) + 1] = (float)(ai + t * (bi - ai));
      }
    }
  }
  for (int i = 0; i < 4; i++) {
    uint32_t l = PILOT_L[i];
    double s = 0;
    for (uint32_t k = 0; k < W; k++) {
      double yr = grid[2 * (l * W + k)], yi = grid[2 * (l * W + k) + 1];
      s += yr * yr + yi * yi;
    }
    rssi_acc += s;
  }
  if (metrics) {
    double rsrp = rsrp_acc / rsrp_n, rssi = rssi_acc / 4.0, noise = noise_acc / noise_n;
    metrics[0] = (float)rsrp; metrics[1] = (float)rssi;
    metrics[2] = (float)(rssi > 0 ? c->nof_prb * rsrp / rssi : 0);
    metrics[3] = (float)noise; metrics[4] = (float)(noise > 0 ? rsrp / noise : 0);
  }
  free(hp); free(hs); free(hf);
  return 0;
}

/* max-log soft demapper of one complex symbol into Qm LLRs: per bit, the smallest squared distance to a
 * PAM level whose label has the bit 0 / 1 (exhaustive over the levels).  Each level's squared distance is
 * formed once per dimension and shared by the nb bits' minima (the same values and comparisons as one
 * search per bit, so the LLRs are unchanged; the CPU baseline runs this). */
static void pam_levels(uint32_t Qm, double *lev) {
  uint32_t nb = Qm / 2, nl = 1u << nb;
  for (uint32_t lab = 0; lab < nl; lab++) {
    uint8_t bits[3];
    for (uint32_t q = 0; q < nb; q++) bits[q] = (lab >> (nb - 1 - q)) & 1;
    lev[lab] = or_pam_level(bits, Qm);
  }
}
static void demod_symbol(double xr, double xi, uint32_t Qm, const double *lev, float *llr) {
  const double inv_s2 = 1.0 / 0.5;
  uint32_t nb = Qm / 2, nl = 1u << nb;
  for (int dim = 0; dim < 2; dim++) {
    double x = dim ? xi : xr;
    double d2[8];
    for (uint32_t lab = 0; lab < nl; lab++) {
      double d = x - lev[lab];
      d2[lab] = d * d;
    }
    for (uint32_t j = 0; j < nb; j++) {
      double m0 = 1e300, m1 = 1e300;
      for (uint32_t lab = 0; lab < nl; lab++) {
        if ((lab >> (nb - 1 - j)) & 1) { if (d2[lab] < m1) m1 = d2[lab]; } else { if (d2[lab] < m0) m0 = d2[lab]; }
      }
      llr[2 * j + dim] = (float)((m0 - m1) * inv_s2);
    }
  }
}

static void equalize(const float *grid, const float *ce, uint32_t plane, const uint32_t *re, int nre,
                     uint32_t tm, double noise, double *sym) {
  for (int i = 0; i < nre; i += (tm == 2 ? 2 : 1)) {
    if (tm != 2) {
      double yr = grid[2 * re[i]], yi = grid[2 * re[i] + 1];
      double hr = ce[2 * re[i]], hi = ce[2 * re[i] + 1];
      double den = hr * hr + hi * hi + noise;
      sym[2 * i] = (yr * hr + yi * hi) / den;
      sym[2 * i + 1] = (yi * hr - yr * hi) / den;
    } else {
      const float *c0 = ce, *c1 = ce + plane * 2;
      double r0r = grid[2 * re[i]], r0i = grid[2 * re[i] + 1];
      double r1r = grid[2 * re[i + 1]], r1i = grid[2 * re[i + 1] + 1];
      double h00r = c0[2 * re[i]], h00i = c0[2 * re[i] + 1];
      double h01r = c0[2 * re[i + 1]], h01i = c0[2 * re[i + 1] + 1];
      double h10r = c1[2 * re[i]], h10i = c1[2 * re[i] + 1];
      double h11r = c1[2 * re[i + 1]], h11i = c1[2 * re[i + 1] + 1];
      double hh = h00r * h00r + h00i * h00i + h11r * h11r + h11i * h11i;
      if (hh <= 0) hh = 1e-9;
      double s = sqrt(2.0) / hh;
      /* x0 = (conj(h00) r0 + h11 conj(r1)) */
      double x0r = (h00r * r0r + h00i * r0i) + (h11r * r1r + h11i * r1i);
      double x0i = (h00r * r0i - h00i * r0r) + (h11i * r1r - h11r * r1i);
      /* x1 = (-h10 conj(r0) + conj(h01) r1) */
      double x1r = -(h10r * r0r + h10i * r0i) + (h01r * r1r + h01i * r1i);
      double x1i = -(h10i * r0r - h10r * r0i) + (h01r * r1i - h01i * r1r);
      sym[2 * i] = s * x0r; sym[2 * i + 1] = s * x0i;
      sym[2 * i + 2] = s * x1r; sym[2 * i + 3] = s * x1i;
    }
  }
}

int or_pdsch_llr(const or_cell_t *c, uint32_t cfi, uint32_t sf, const uint8_t *prb_mask, uint32_t Qm,
                 uint32_t rnti, uint32_t tm, float noise, const float *grid, const float *ce, float *llr,
                 uint32_t *G_out, float *symbols_out) {
  const uint32_t W = 12 * c->nof_prb;
  uint32_t *re = (uint32_t *)malloc(sizeof(uint32_t) * OR_NSYMB * W);
  int nre = or_pdsch_re_list(c, cfi, sf, prb_mask, re);
  if (tm == 2 && (nre & 1)) { free(re); return -1; }
  double *sym = (double *)malloc(sizeof(double) * 2 * (nre + 1));
  equalize(grid, ce, OR_NSYMB * W, re, nre, tm, noise, sym);
  uint32_t G = (uint32_t)nre * Qm;
  uint8_t *cs = (uint8_t *)malloc(G + 8);
  or_gold((rnti << 14) | (sf << 9) | c->id, cs, G);
  double lev[8];
  pam_levels(Qm, lev);
  for (int i = 0; i < nre; i++) {
    demod_symbol(sym[2 * i], sym[2 * i + 1], Qm, lev, llr + (size_t)i * Qm);
    if (symbols_out) { symbols_out[2 * i] = (float)sym[2 * i]; symbols_out[2 * i + 1] = (float)sym[2 * i + 1]; }
  }
  for (uint32_t i = 0; i < G; i++) if (cs[i]) llr[i] = -llr[i];
  if (G_out) *G_out = G;
  free(re); free(sym); free(cs);
  return 0;
}

int or_pcfich(const or_cell_t *c, uint32_t sf, const float *grid, const float *ce) {
  uint32_t kk[16];
  or_pcfich_k(c, kk);   /* symbol 0 -> RE index == k */
  double sym[32];
  uint32_t tm = c->nof_ports == 2 ? 2 : 1;
  equalize(grid, ce, OR_NSYMB * 12 * c->nof_prb, kk, 16, tm, 0.0, sym);
  float llr[32];
  double lev[8];
  pam_levels(2, lev);
  for (int i = 0; i < 16; i++) demod_symbol(sym[2 * i], sym[2 * i + 1], 2, lev, llr + 2 * i);
  uint8_t sc[32];
  or_gold(or_pcfich_cinit(c, sf), sc, 32);
  for (int i = 0; i < 32; i++) if (sc[i]) llr[i] = -llr[i];
  int best = 0;
  double best_s = -1e300;
  for (uint32_t cfi = 1; cfi <= 3; cfi++) {
    uint8_t cw[32];
    or_cfi_codeword(cfi, cw);
    double s = 0;
    for (int i = 0; i < 32; i++) s += llr[i] * (cw[i] ? 1.0 : -1.0);
    if (s > best_s) { best_s = s; best = (int)cfi; }
  }
  return best;
}

int or_dlsch_decode(const float *llr, uint32_t G, uint32_t tbs, uint32_t Qm, uint32_t NL, uint32_t rv,
                    int new_tb, float *sb, uint32_t sb_stride, uint32_t max_its, uint8_t *payload,
                    uint32_t *noi_out, uint32_t *cb_crc_ok_out) {
  return or_dlsch_decode_cbits(llr, G, tbs, Qm, NL, rv, new_tb, sb, sb_stride, max_its, payload, noi_out,
                               cb_crc_ok_out, NULL);
}

int or_dlsch_decode_cbits(const float *llr, uint32_t G, uint32_t tbs, uint32_t Qm, uint32_t NL, uint32_t rv,
                          int new_tb, float *sb, uint32_t sb_stride, uint32_t max_its, uint8_t *payload,
                          uint32_t *noi_out, uint32_t *cb_crc_ok_out, uint32_t *cb_its_out) {
  or_cbsegm_t sg;
  if (or_cbsegm(tbs, &sg)) return -1;
  /* per-call decoder state: or_dlsch_decode / or_decode_subframe are called from several threads
     by the CPU baseline */
  int mode = or_get_tdec_mode();
  if (mode == OR_TDEC_AVX2 && !or_avx2_available()) mode = OR_TDEC_SIMD;
  void *h = malloc(mode == OR_TDEC_GEN ? sizeof(or_tdec_t)
                   : mode == OR_TDEC_I16 ? sizeof(or_tdec16_t)
                   : mode == OR_TDEC_AVX2 ? or_avx2_tdec_size() : or_simd_tdec_size());
  if (mode == OR_TDEC_SIMD) or_simd_tdec_init(h);   /* empty QPP-table cache: built once for the TB's K */
  if (mode == OR_TDEC_AVX2) or_avx2_tdec_init(h);
  float *din = (float *)malloc(sizeof(float) * 2 * 3 * (OR_TCOD_MAX_K + 4));
  float *din2 = din + 3 * (OR_TCOD_MAX_K + 4);
  uint8_t *bits = (uint8_t *)malloc(2 * OR_TCOD_MAX_K), *b = (uint8_t *)malloc(sg.B + 8);
  uint8_t *bits2 = bits + OR_TCOD_MAX_K;
  uint32_t pos = 0, pb = 0, noi = 0, ncb_ok = 0;
  for (uint32_t r = 0; r < sg.C; r++) {
    uint32_t K = (r < sg.Cm) ? sg.Km : sg.Kp, F = (r == 0) ? sg.F : 0;
    uint32_t E = (uint32_t)or_rm_E(G, sg.C, Qm, NL, r);
    or_rm_rx(llr + pos, E, K, F, rv, new_tb, sb + (size_t)r * sb_stride, din);
    pos += E;
    int ok, ok2 = 0, its, its2 = 0;
    /* AVX2: code blocks r and r + 1 of equal K decoded together (two per __m256i) */
    const int pair = mode == OR_TDEC_AVX2 && r + 1 < sg.C && ((r + 1 < sg.Cm) ? sg.Km : sg.Kp) == K;
    if (pair) {
      const uint32_t E2 = (uint32_t)or_rm_E(G, sg.C, Qm, NL, r + 1);
      or_rm_rx(llr + pos, E2, K, 0, rv, new_tb, sb + (size_t)(r + 1) * sb_stride, din2);
      pos += E2;
    }
    if (mode == OR_TDEC_AVX2)
      or_avx2_decode_pair(h, din, pair ? din2 : NULL, K, max_its, 1, sg.C == 1, bits, pair ? bits2 : NULL, &ok, &ok2,
                          &its, &its2);
    else
      its = mode == OR_TDEC_I16    ? or_decode_cb16((or_tdec16_t *)h, din, K, max_its, 1, sg.C == 1, bits, &ok)
            : mode == OR_TDEC_SIMD ? or_simd_decode_cb(h, din, K, max_its, 1, sg.C == 1, bits, &ok)
                                   : or_decode_cb((or_tdec_t *)h, din, K, max_its, 1, sg.C == 1, bits, &ok);
    for (int q = 0; q < 1 + pair; q++) {
      const uint32_t rr = r + (uint32_t)q, Fq = q ? 0 : F;
      const int itq = q ? its2 : its, okq = q ? ok2 : ok;
      const uint8_t *bq = q ? bits2 : bits;
      if ((uint32_t)itq > noi) noi = (uint32_t)itq;
      if (cb_its_out) cb_its_out[rr] = (uint32_t)itq;
      ncb_ok += okq ? 1 : 0;
      uint32_t L = sg.C > 1 ? 24 : 0;
      for (uint32_t k = Fq; k < K - L; k++) b[pb++] = bq[k];
    }
    r += (uint32_t)pair;
  }
  int tb_ok = (or_crc24a(b, sg.B) == 0);
  memset(payload, 0, (tbs + 7) / 8);
  for (uint32_t i = 0; i < tbs; i++) payload[i / 8] |= (uint8_t)(b[i] << (7 - i % 8));
  if (noi_out) *noi_out = noi;
  if (cb_crc_ok_out) *cb_crc_ok_out = ncb_ok;
  free(din); free(bits); free(b); free(h);
  return tb_ok ? 0 : -1;
}

int or_decode_subframe(const or_cell_t *c, uint32_t sf, uint32_t cfi, const uint8_t *prb_mask, uint32_t tbs,
                       uint32_t Qm, uint32_t rv, uint32_t rnti, uint32_t tm, uint32_t nl_td, const float *iq,
                       float *sb, uint32_t sb_stride, int new_tb, uint32_t max_its, uint8_t *payload,
                       uint32_t *noi_out) {
  const uint32_t W = 12 * c->nof_prb;
  float *grid = (float *)malloc(sizeof(float) * 2 * OR_NSYMB * W);
  float *ce = (float *)malloc(sizeof(float) * 2 * OR_NSYMB * W * c->nof_ports);
  float *llr = (float *)malloc(sizeof(float) * OR_NSYMB * W * 6);
  uint32_t G;
  or_ofdm_rx(c, iq, grid);
  or_chest(c, sf, grid, ce, NULL);
  int ret = or_pdsch_llr(c, cfi, sf, prb_mask, Qm, rnti, tm, 0.01f, grid, ce, llr, &G, NULL);
  if (!ret)
    ret = or_dlsch_decode(llr, G, tbs, Qm, tm == 2 ? (nl_td ? nl_td : 2) : 1, rv, new_tb, sb, sb_stride,
                          max_its, payload, noi_out, NULL);
  free(grid); free(ce); free(llr);
  return ret;
}
