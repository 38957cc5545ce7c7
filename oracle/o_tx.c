/*
 * o_tx.c -- synthetic PDSCH subframe transmitter (TEST INFRASTRUCTURE ONLY: ground truth).
 *
 * Generates the IQ that srsUE's radio would hand to phch_worker (/root/reference/ue/src/phy/
 * phch_recv.cc:321-322 -> phch_worker.cc:254) for a known transport block: CRC24A -> segmentation
 * -> CRC24B -> turbo code -> rate matching -> scrambling -> QAM -> (SFBC) -> RE mapping + CRS +
 * PCFICH -> IFFT (1/sqrt(N)) + CP -> flat channel + AWGN.  36.211 / 36.212 throughout.
 */
#include "oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

static uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static double urand(uint64_t *s) { return ((double)(splitmix64(s) >> 11) + 0.5) * (1.0 / 9007199254740992.0); }

/* 36.211 7.1: per-dimension PAM level of a Gray QAM symbol (bits of one dimension, MSB first) */
double or_pam_level(const uint8_t *b, uint32_t Qm) {
  switch (Qm) {
    case 2: return (1 - 2 * (int)b[0]) / sqrt(2.0);
    case 4: return (1 - 2 * (int)b[0]) * (1 + 2 * (int)b[1]) / sqrt(10.0);
    case 6: return (1 - 2 * (int)b[0]) * (4 - (1 - 2 * (int)b[1]) * (2 - (1 - 2 * (int)b[2]))) / sqrt(42.0);
  }
  return 0;
}
static void qam(const uint8_t *bits, uint32_t Qm, double *re, double *im) {
  uint8_t bi[3], bq[3];
  for (uint32_t j = 0; j < Qm / 2; j++) { bi[j] = bits[2 * j]; bq[j] = bits[2 * j + 1]; }
  *re = or_pam_level(bi, Qm);
  *im = or_pam_level(bq, Qm);
}

/* PCFICH resource elements (36.211 6.7.4 + REG definition 6.2.4): 16 subcarriers of symbol 0 */
void or_pcfich_k(const or_cell_t *c, uint32_t *k_out) {
  uint32_t W = 12 * c->nof_prb, kbar = 6 * (c->id % (2 * c->nof_prb)), vs3 = (c->id % 6) % 3;
  int n = 0;
  for (uint32_t i = 0; i < 4; i++) {
    uint32_t kreg = (kbar + (i * c->nof_prb / 2) * 6) % W;
    for (uint32_t k = kreg; k < kreg + 6; k++) if (k % 3 != vs3) k_out[n++] = k;
  }
}
uint32_t or_pcfich_cinit(const or_cell_t *c, uint32_t sf) { return (sf + 1) * (2 * c->id + 1) * 512 + c->id; }
/* 36.212 Table 5.3.4-1 CFI code words */
void or_cfi_codeword(uint32_t cfi, uint8_t *b) {
  static const uint8_t pat[3][3] = {{0, 1, 1}, {1, 0, 1}, {1, 1, 0}};
  for (int i = 0; i < 32; i++) b[i] = (cfi >= 1 && cfi <= 3) ? pat[cfi - 1][i % 3] : 0;
}

/* SFBC precoding of a symbol pair onto two ports (36.211 6.3.4.3) */
static void sfbc(double x0r, double x0i, double x1r, double x1i, double *p0a, double *p1a, double *p0b,
                 double *p1b) {
  const double s = 1.0 / sqrt(2.0);
  p0a[0] = s * x0r;  p0a[1] = s * x0i;    /* y0(2i)   =  x0 / sqrt2     */
  p1a[0] = -s * x1r; p1a[1] = s * x1i;    /* y1(2i)   = -x1* / sqrt2    */
  p0b[0] = s * x1r;  p0b[1] = s * x1i;    /* y0(2i+1) =  x1 / sqrt2     */
  p1b[0] = s * x0r;  p1b[1] = -s * x0i;   /* y1(2i+1) =  x0* / sqrt2    */
}

int or_tx_subframe(const or_tx_cfg_t *cfg, const uint8_t *tb, float *iq, uint32_t *G_out) {
  const or_cell_t *c = &cfg->cell;
  const int N = or_symbol_sz(c->nof_prb);
  const uint32_t W = 12 * c->nof_prb, P = c->nof_ports;
  uint32_t Qm = cfg->qm, itbs, nalloc = 0;
  for (uint32_t p = 0; p < c->nof_prb; p++) nalloc += cfg->prb_mask[p] ? 1 : 0;
  if (or_mcs(cfg->mcs, &Qm, &itbs) && !cfg->qm) return -1;
  if (cfg->qm) Qm = cfg->qm;
  int tbs = cfg->tbs ? (int)cfg->tbs : or_tbs(itbs, nalloc);
  if (tbs <= 0 || N < 0) return -1;
  if (cfg->tm == 2 && P != 2) return -1;

  /* ---- transport channel: 36.212 5.3.2 ---- */
  uint32_t A = (uint32_t)tbs;
  uint8_t *b = (uint8_t *)malloc(A + 24);
  for (uint32_t i = 0; i < A; i++) b[i] = (tb[i / 8] >> (7 - i % 8)) & 1;
  uint32_t crc = or_crc24a(b, A);
  for (int i = 0; i < 24; i++) b[A + i] = (crc >> (23 - i)) & 1;
  or_cbsegm_t sg;
  or_cbsegm(A, &sg);

  uint32_t *re = (uint32_t *)malloc(sizeof(uint32_t) * OR_NSYMB * W);
  int nre = or_pdsch_re_list(c, cfg->cfi, cfg->sf_idx, cfg->prb_mask, re);
  if (cfg->tm == 2 && (nre & 1)) { free(b); free(re); return -1; }
  uint32_t G = (uint32_t)nre * Qm;
  uint32_t NL = (cfg->tm == 2) ? (cfg->nl_td ? cfg->nl_td : 2) : 1;
  uint8_t *f = (uint8_t *)malloc(G + 8);
  uint8_t *cb = (uint8_t *)malloc(OR_TCOD_MAX_K), *d = (uint8_t *)malloc(3 * (OR_TCOD_MAX_K + 4));
  uint32_t pos_b = 0, pos_f = 0;
  for (uint32_t r = 0; r < sg.C; r++) {
    uint32_t K = (r < sg.Cm) ? sg.Km : sg.Kp, F = (r == 0) ? sg.F : 0;
    uint32_t L = (sg.C > 1) ? 24 : 0;
    for (uint32_t k = 0; k < K - L; k++) cb[k] = (k < F) ? 0 : b[pos_b++];
    if (L) {
      uint32_t cc = or_crc24b(cb, K - L);
      for (int i = 0; i < 24; i++) cb[K - L + i] = (cc >> (23 - i)) & 1;
    }
    or_tcod(cb, K, F, d);
    uint32_t E = (uint32_t)or_rm_E(G, sg.C, Qm, NL, r);
    or_rm_tx(d, K, E, cfg->rv, f + pos_f);
    pos_f += E;
  }
  /* scrambling, 36.211 6.3.1 (q = 0) */
  uint8_t *cs = (uint8_t *)malloc(G + 8);
  or_gold((cfg->rnti << 14) | (cfg->sf_idx << 9) | c->id, cs, G);
  for (uint32_t i = 0; i < G; i++) f[i] ^= cs[i];

  /* ---- grid per port ---- */
  double *grid = (double *)calloc((size_t)P * OR_NSYMB * W * 2, sizeof(double));
  uint32_t nsym = G / Qm;
  for (uint32_t i = 0; i < nsym; i += (cfg->tm == 2 ? 2 : 1)) {
    double xr, xi;
    qam(f + i * Qm, Qm, &xr, &xi);
    if (cfg->tm != 2) {
      grid[2 * re[i]] = xr; grid[2 * re[i] + 1] = xi;
    } else {
      double yr, yi;
      qam(f + (i + 1) * Qm, Qm, &yr, &yi);
      double *g0 = grid, *g1 = grid + (size_t)OR_NSYMB * W * 2;
      sfbc(xr, xi, yr, yi, g0 + 2 * re[i], g1 + 2 * re[i], g0 + 2 * re[i + 1], g1 + 2 * re[i + 1]);
    }
  }
  /* CRS, 36.211 6.10.1 */
  float rs[4 * OR_NRB_MAX];
  for (uint32_t p = 0; p < P; p++) {
    for (uint32_t l = 0; l < OR_NSYMB; l++) {
      uint32_t lp = l % 7;
      if (lp != 0 && lp != 4) continue;
      uint32_t v = (p == 0) ? (lp == 0 ? 0 : 3) : (lp == 0 ? 3 : 0);
      uint32_t off = (v + c->id % 6) % 6;
      or_crs_seq(c->id, 2 * cfg->sf_idx + l / 7, lp, rs);
      for (uint32_t m = 0; m < 2 * c->nof_prb; m++) {
        uint32_t mp = m + OR_NRB_MAX - c->nof_prb;
        double *gp = grid + ((size_t)p * OR_NSYMB * W + l * W + 6 * m + off) * 2;
        gp[0] = rs[2 * mp]; gp[1] = rs[2 * mp + 1];
      }
    }
  }
  /* PCFICH, 36.211 6.7 */
  if (cfg->cfi >= 1 && cfg->cfi <= 3) {
    uint8_t cw[32], sc[32];
    uint32_t kk[16];
    or_cfi_codeword(cfg->cfi, cw);
    or_gold(or_pcfich_cinit(c, cfg->sf_idx), sc, 32);
    for (int i = 0; i < 32; i++) cw[i] ^= sc[i];
    or_pcfich_k(c, kk);
    for (int i = 0; i < 16; i += (P == 2 ? 2 : 1)) {
      double xr, xi;
      qam(cw + 2 * i, 2, &xr, &xi);
      if (P == 1) { grid[2 * kk[i]] = xr; grid[2 * kk[i] + 1] = xi; }
      else {
        double yr, yi;
        qam(cw + 2 * (i + 1), 2, &yr, &yi);
        double *g0 = grid, *g1 = grid + (size_t)OR_NSYMB * W * 2;
        sfbc(xr, xi, yr, yi, g0 + 2 * kk[i], g1 + 2 * kk[i], g0 + 2 * kk[i + 1], g1 + 2 * kk[i + 1]);
      }
    }
  }
  /* ---- OFDM modulation + channel + AWGN ---- */
  double *X = (double *)malloc(sizeof(double) * 2 * N), *x = (double *)malloc(sizeof(double) * 2 * N);
  const double nrm = 1.0 / sqrt((double)N);
  const int SF = or_sf_len(c->nof_prb);
  double *acc = (double *)calloc((size_t)SF * 2, sizeof(double));
  for (uint32_t p = 0; p < P; p++) {
    double hr = cfg->h_re[p], hi = cfg->h_im[p];
    if (hr == 0 && hi == 0 && p == 0 && P == 1) hr = 1.0;
    size_t pos = 0;
    for (uint32_t l = 0; l < OR_NSYMB; l++) {
      memset(X, 0, sizeof(double) * 2 * N);
      const double *gl = grid + ((size_t)p * OR_NSYMB * W + l * W) * 2;
      for (uint32_t k = 0; k < W; k++) {
        int bin = (k < W / 2) ? (int)(N - W / 2 + k) : (int)(k - W / 2 + 1);
        X[2 * bin] = gl[2 * k]; X[2 * bin + 1] = gl[2 * k + 1];
      }
      or_dft(X, x, N, 1);
      int cp = or_cp_len((uint32_t)N, l % 7);
      for (int n = 0; n < cp + N; n++) {
        int src = (n < cp) ? (N - cp + n) : (n - cp);
        double sr = x[2 * src] * nrm, si = x[2 * src + 1] * nrm;
        acc[2 * pos] += hr * sr - hi * si;
        acc[2 * pos + 1] += hr * si + hi * sr;
        pos++;
      }
    }
  }
  uint64_t seed = cfg->noise_seed;
  double sigma = (cfg->snr_db >= 200.0f) ? 0.0 : sqrt(pow(10.0, -cfg->snr_db / 10.0) / 2.0);
  for (int n = 0; n < SF; n++) {
    double nr = 0, ni = 0;
    if (sigma > 0) {
      double u1 = urand(&seed), u2 = urand(&seed), rr = sqrt(-2.0 * log(u1));
      nr = rr * cos(2 * M_PI * u2) * sigma; ni = rr * sin(2 * M_PI * u2) * sigma;
    }
    iq[2 * n] = (float)(acc[2 * n] + nr);
    iq[2 * n + 1] = (float)(acc[2 * n + 1] + ni);
  }
  if (G_out) *G_out = G;
  free(b); free(re); free(f); free(cb); free(d); free(cs); free(grid); free(X); free(x); free(acc);
  return 0;
}
