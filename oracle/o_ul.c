/*
 * o_ul.c -- UL PUSCH transmit chain (TEST INFRASTRUCTURE ONLY): SURVEY.md 8f row f4, what srsUE reaches
 * through srslte_ue_ul_cfg_grant + srslte_ue_ul_pusch_encode_rnti_softbuffer
 * (/root/reference/ue/src/phy/phch_worker.cc:551-560).  srsLTE is not in the container: parity against
 * it is unpinned; this restates 3GPP TS 36.212 / 36.211 Rel-8 and is pinned by properties (DMRS
 * constant amplitude / ZC structure, interleaver permutation) and by round trips (the coded bits
 * through the DL-SCH decoder, the SC-FDMA symbols through a DFT receiver).
 *
 *   UL-SCH (36.212 5.2.2): CRC24A, segmentation, CRC24B, turbo code, rate matching with the full
 *          circular buffer (the DL-SCH chain of o_tx.c with N_L = 1), G = 12 M_sc Q_m (normal CP, no
 *          SRS, no UCI);
 *   channel interleaver (5.2.2.8, no UCI): Q_m-bit symbols written row by row into M_sc rows x 12
 *          columns, read column by column -> SC-FDMA data symbol l takes rows 0..M_sc-1 of column l;
 *   scrambling (36.211 5.3.1): c_init = n_RNTI 2^14 + sf 2^9 + N_ID; modulation as the DL (7.1);
 *   transform precoding (5.3.3): z = (1/sqrt M) DFT_M per data symbol;
 *   DMRS (5.5.2.1, M_sc >= 36 only -- the L_prb = 1, 2 base sequences are tables this restatement
 *          does not carry): ZC root q of N_ZC = largest prime < M_sc, group hopping f_gh, sequence
 *          hopping v (M_sc >= 72), f_ss = (N_ID + delta_ss) mod 30, alpha = 2 pi n_cs / 12 with
 *          n_cs = (n1_DMRS[cyclic_shift] + n2_DMRS[dci field] + n_PRS(n_s)) mod 12, symbol 3 of each slot;
 *   mapping (5.3.4): PRBs n_prb .. n_prb + L - 1 of symbols 0-2, 4-6 of slot 0, and of slot 1 unless
 *          frequency hopping moves slot 1 to n_prb1 .. n_prb1 + L - 1 (36.213 8.4, computed by the caller);
 *   SC-FDMA (5.6): s[n] = (1/sqrt N) sum_k a_k exp(j 2 pi (k - 6 N_RB + 1/2) n / N), n = -N_CP .. N-1.
 */
#include "oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

static const uint32_t N1_DMRS[8] = {0, 2, 3, 4, 6, 8, 9, 10};   /* Table 5.5.2.1.1-2 (cyclicShift) */
static const uint32_t N2_DMRS[8] = {0, 6, 3, 4, 2, 8, 10, 9};   /* Table 5.5.2.1.1-1 (DCI 0 field) */

uint32_t or_pusch_G(const or_ul_cfg_t *c) { return 12 * 12 * c->L_prb * c->Qm; }

/* 36.213 Table 8.6.3-1: beta_offset^HARQ-ACK x 8 for I_offset^HARQ-ACK = 0..14 */
static const uint32_t BETA8_ACK[15] = {16, 20, 25, 32, 40, 50, 64, 80, 101, 127, 160, 248, 400, 640, 1008};

uint32_t or_ack_qprime(const or_ul_cfg_t *c) {
  if (!c->ack_len) return 0;
  or_cbsegm_t sg;
  if (or_cbsegm(c->tbs, &sg)) return 0;
  const uint64_t sumK = (uint64_t)sg.Cm * sg.Km + (uint64_t)(sg.C - sg.Cm) * sg.Kp, M = 12 * c->L_prb;
  const uint64_t num = (uint64_t)c->ack_len * M * 12 * BETA8_ACK[c->I_offset_ack > 14 ? 14 : c->I_offset_ack];
  const uint64_t q = (num + 8 * sumK - 1) / (8 * sumK);
  return (uint32_t)(q < 4 * M ? q : 4 * M);
}

/* 36.212 Tables 5.2.2.6-1 / -2 (placeholders: 2 = x, 3 = y) */
uint32_t or_ack_block(const or_ul_cfg_t *c, uint8_t *blk) {
  const uint32_t Qm = c->Qm, o0 = c->ack & 1, o1 = (c->ack >> 1) & 1, o2 = o0 ^ o1;
  if (c->ack_len == 1) {
    blk[0] = (uint8_t)o0;
    blk[1] = 3;
    for (uint32_t b = 2; b < Qm; b++) blk[b] = 2;
    return Qm;
  }
  const uint8_t seq[3][2] = {{(uint8_t)o0, (uint8_t)o1}, {(uint8_t)o2, (uint8_t)o0}, {(uint8_t)o1, (uint8_t)o2}};
  for (uint32_t s = 0; s < 3; s++) {   /* Qm = 2: o0 o1 o2 o0 o1 o2; else each pair padded with x */
    blk[s * Qm] = seq[s][0];
    blk[s * Qm + 1] = seq[s][1];
    for (uint32_t b = 2; b < Qm; b++) blk[s * Qm + b] = 2;
  }
  return 3 * Qm;
}

int or_ulsch_encode(const or_ul_cfg_t *c, const uint8_t *tb, uint8_t *f) {
  const uint32_t A = c->tbs, G = or_pusch_G(c);
  if (A == 0 || (c->Qm != 2 && c->Qm != 4 && c->Qm != 6)) return -1;
  uint8_t *b = (uint8_t *)malloc(A + 24);
  for (uint32_t i = 0; i < A; i++) b[i] = (tb[i / 8] >> (7 - i % 8)) & 1;
  const uint32_t crc = or_crc24a(b, A);
  for (int i = 0; i < 24; i++) b[A + i] = (crc >> (23 - i)) & 1;
  or_cbsegm_t sg;
  if (or_cbsegm(A, &sg)) { free(b); return -1; }
  uint8_t *cb = (uint8_t *)malloc(OR_TCOD_MAX_K), *d = (uint8_t *)malloc(3 * (OR_TCOD_MAX_K + 4));
  uint32_t pos_b = 0, pos_f = 0;
  for (uint32_t r = 0; r < sg.C; r++) {
    const uint32_t K = (r < sg.Cm) ? sg.Km : sg.Kp, F = (r == 0) ? sg.F : 0, L = sg.C > 1 ? 24 : 0;
    for (uint32_t k = 0; k < K - L; k++) cb[k] = (k < F) ? 0 : b[pos_b++];
    if (L) {
      const uint32_t cc = or_crc24b(cb, K - L);
      for (int i = 0; i < 24; i++) cb[K - L + i] = (cc >> (23 - i)) & 1;
    }
    or_tcod(cb, K, F, d);
    const uint32_t E = (uint32_t)or_rm_E(G, sg.C, c->Qm, 1, r);
    or_rm_tx(d, K, E, c->rv, f + pos_f);
    pos_f += E;
  }
  free(b); free(cb); free(d);
  return (int)G;
}

int or_pusch_mod(const or_ul_cfg_t *c, const uint8_t *f, float *x) {
  const uint32_t M = 12 * c->L_prb, Qm = c->Qm, G = or_pusch_G(c);
  uint8_t *cs = (uint8_t *)malloc(G), *h = (uint8_t *)malloc(G);
  for (uint32_t l = 0; l < 12; l++)          /* interleaver: output symbol l M + m <- input m 12 + l */
    for (uint32_t m = 0; m < M; m++)
      memcpy(h + (size_t)(l * M + m) * Qm, f + (size_t)(m * 12 + l) * Qm, Qm);
  /* HARQ-ACK symbols overwrite the matrix from the last row up, columns ColumnSet(j), j = 0, 3, 2, 1, ... */
  static const uint32_t COLSET[4] = {2, 3, 8, 9};
  uint8_t blk[18];
  const uint32_t nq = or_ack_qprime(c), nb = c->ack_len ? or_ack_block(c, blk) : Qm;
  for (uint32_t i = 0, j = 0; i < nq; i++, j = (j + 3) % 4) {
    const uint32_t r = M - 1 - i / 4, col = COLSET[j];
    for (uint32_t b = 0; b < Qm; b++) h[(size_t)(col * M + r) * Qm + b] = blk[(i * Qm + b) % nb];
  }
  or_gold((c->rnti << 14) | (c->sf_idx << 9) | c->cell_id, cs, G);
  for (uint32_t i = 0; i < G; i++)            /* 36.211 5.3.1 with the UCI placeholders */
    h[i] = h[i] == 2 ? 1 : h[i] == 3 ? h[i - 1] : (uint8_t)(h[i] ^ cs[i]);
  for (uint32_t s = 0; s < 12 * M; s++) {
    uint8_t bi[3], bq[3];
    for (uint32_t j = 0; j < Qm / 2; j++) { bi[j] = h[s * Qm + 2 * j]; bq[j] = h[s * Qm + 2 * j + 1]; }
    x[2 * s] = (float)or_pam_level(bi, Qm);
    x[2 * s + 1] = (float)or_pam_level(bq, Qm);
  }
  free(cs); free(h);
  return 0;
}

void or_dft_m(const float *in, uint32_t M, float *out, int inverse) {
  const double sg = inverse ? 1.0 : -1.0, nrm = 1.0 / sqrt((double)M);
  for (uint32_t k = 0; k < M; k++) {
    double re = 0, im = 0;
    for (uint32_t i = 0; i < M; i++) {
      const double ph = sg * 2.0 * M_PI * (double)((uint64_t)i * k % M) / (double)M, cc = cos(ph), ss = sin(ph);
      re += in[2 * i] * cc - in[2 * i + 1] * ss;
      im += in[2 * i] * ss + in[2 * i + 1] * cc;
    }
    out[2 * k] = (float)(re * nrm);
    out[2 * k + 1] = (float)(im * nrm);
  }
}

static int is_prime(uint32_t n) {
  if (n < 2) return 0;
  for (uint32_t d = 2; d * d <= n; d++) if (n % d == 0) return 0;
  return 1;
}

int or_dmrs_params(const or_ul_cfg_t *c, uint32_t ns, uint32_t *u, uint32_t *v, uint32_t *ncs) {
  const uint32_t M = 12 * c->L_prb, fss = (c->cell_id + c->delta_ss) % 30;
  uint32_t fgh = 0;
  if (c->group_hopping) {
    uint8_t g[160];
    or_gold(c->cell_id / 30, g, 160);
    for (int i = 0; i < 8; i++) fgh += (uint32_t)g[8 * ns + i] << i;
    fgh %= 30;
  }
  *u = (fgh + fss) % 30;
  *v = 0;
  uint8_t s[8 * 7 * 20];   /* n_PRS reads c(8 N_symb^UL n_s + i), n_s < 20 */
  or_gold((c->cell_id / 30) * 32 + fss, s, 8 * 7 * 20);
  if (M >= 72 && !c->group_hopping && c->sequence_hopping) *v = s[ns];
  uint32_t prs = 0;
  for (int i = 0; i < 8; i++) prs += (uint32_t)s[8 * 7 * ns + i] << i;   /* n_PRS(n_s), N_symb^UL = 7 */
  *ncs = (N1_DMRS[c->cyclic_shift & 7] + N2_DMRS[c->n_dmrs2 & 7] + prs) % 12;
  return M >= 36 ? 0 : -1;
}

int or_dmrs_pusch(const or_ul_cfg_t *c, uint32_t ns, float *r) {
  const uint32_t M = 12 * c->L_prb;
  uint32_t u, v, ncs;
  if (or_dmrs_params(c, ns, &u, &v, &ncs)) return -1;
  uint32_t Nzc = M - 1;
  while (!is_prime(Nzc)) Nzc--;
  const double qb = (double)Nzc * (u + 1) / 31.0;
  const uint32_t q = (uint32_t)floor(qb + 0.5) + v * (((uint32_t)floor(2.0 * qb) & 1) ? (uint32_t)-1 : 1u);
  for (uint32_t n = 0; n < M; n++) {
    const uint32_t m = n % Nzc;
    /* x_q(m) exp(j alpha n): phase -pi q m (m+1) / Nzc + 2 pi ncs n / 12 */
    const double ph = -M_PI * (double)((uint64_t)q * m * (m + 1) % (2ull * Nzc)) / Nzc + 2.0 * M_PI * (double)((ncs * n) % 12) / 12.0;
    r[2 * n] = (float)cos(ph);
    r[2 * n + 1] = (float)sin(ph);
  }
  return 0;
}

int or_pusch_grid(const or_ul_cfg_t *c, const uint8_t *tb, float *grid) {
  const uint32_t W = 12 * c->nof_prb, M = 12 * c->L_prb, G = or_pusch_G(c);
  if (c->n_prb + c->L_prb > c->nof_prb || M < 36) return -1;
  if (c->hop && c->n_prb1 + c->L_prb > c->nof_prb) return -1;
  uint8_t *f = (uint8_t *)malloc(G);
  float *x = (float *)malloc(sizeof(float) * 2 * 12 * M), *z = (float *)malloc(sizeof(float) * 2 * M);
  if (or_ulsch_encode(c, tb, f) < 0) { free(f); free(x); free(z); return -1; }
  or_pusch_mod(c, f, x);
  memset(grid, 0, sizeof(float) * 2 * OR_NSYMB * W);
  uint32_t ds = 0;
  for (uint32_t l = 0; l < OR_NSYMB; l++) {
    const uint32_t n0 = (c->hop && l >= 7) ? c->n_prb1 : c->n_prb;
    float *g = grid + 2 * ((size_t)l * W + 12 * n0);
    if (l % 7 == 3) {
      or_dmrs_pusch(c, 2 * c->sf_idx + l / 7, z);
    } else {
      or_dft_m(x + 2 * (size_t)ds * M, M, z, 0);
      ds++;
    }
    memcpy(g, z, sizeof(float) * 2 * M);
  }
  free(f); free(x); free(z);
  return 0;
}

int or_scfdma_tx(uint32_t nof_prb, const float *grid, float *iq) {
  const int N = or_symbol_sz(nof_prb);
  const uint32_t W = 12 * nof_prb;
  if (N < 0) return -1;
  double *X = (double *)malloc(sizeof(double) * 2 * N), *t = (double *)malloc(sizeof(double) * 2 * N);
  const double nrm = 1.0 / sqrt((double)N);
  size_t pos = 0;
  for (uint32_t l = 0; l < OR_NSYMB; l++) {
    const int cp = or_cp_len((uint32_t)N, l % 7);
    memset(X, 0, sizeof(double) * 2 * N);
    for (uint32_t k = 0; k < W; k++) {   /* frequency (k - W/2 + 1/2) df: bin (k - W/2) mod N, then the 1/2 shift */
      const uint32_t b = (uint32_t)(((int)k - (int)(W / 2) + N) % N);
      X[2 * b] = grid[2 * ((size_t)l * W + k)];
      X[2 * b + 1] = grid[2 * ((size_t)l * W + k) + 1];
    }
    or_dft(X, t, N, 1);
    for (int n = -cp; n < N; n++) {
      const uint32_t src = (uint32_t)((n + N) % N);
      const double ph = M_PI * (double)n / (double)N, cc = cos(ph), ss = sin(ph);
      const double vr = t[2 * src] * nrm, vi = t[2 * src + 1] * nrm;
      iq[2 * (pos + (size_t)(n + cp))] = (float)(vr * cc - vi * ss);
      iq[2 * (pos + (size_t)(n + cp)) + 1] = (float)(vr * ss + vi * cc);
    }
    pos += (size_t)(N + cp);
  }
  free(X); free(t);
  return 0;
}

int or_pusch_encode(const or_ul_cfg_t *c, const uint8_t *tb, float *iq) {
  const uint32_t W = 12 * c->nof_prb;
  float *grid = (float *)malloc(sizeof(float) * 2 * OR_NSYMB * W);
  int rc = or_pusch_grid(c, tb, grid);
  if (!rc) rc = or_scfdma_tx(c->nof_prb, grid, iq);
  free(grid);
  return rc;
}
