/*
 * o_ul.c -- UL PUSCH transmit chain (TEST INFRASTRUCTURE ONLY): SURVEY.md 8f row f4, what srsUE reaches
 * through srslte_ue_ul_cfg_grant + srslte_ue_ul_pusch_encode_rnti_softbuffer
 * (/root/reference/ue/src/phy/phch_worker.cc:551-560).  srsLTE is not in the container: parity against
 * it is unpinned; this restates 3GPP TS 36.212 / 36.211 Rel-8 and is pinned by properties (DMRS
 * constant amplitude / ZC structure, interleaver permutation) and by round trips (the coded bits
 * through the DL-SCH decoder, the SC-FDMA symbols through a DFT receiver).
 *
 *   UL-SCH (36.212 5.2.2): CRC24A, segmentation, CRC24B, turbo code, rate matching with the full
 *          circular buffer (the DL-SCH chain of o_tx.c with N_L = 1), G = 12 M_sc Q_m - Q_CQI - Q_RI
 *          (normal CP, no SRS);
 *   UCI (5.2.2.6): HARQ-ACK and RI blocks of Tables 5.2.2.6-1..-4 with placeholders, Q'_ACK / Q'_RI /
 *          Q'_CQI from the beta_offsets of 36.213 Tables 8.6.3-1..-3; CQI O <= 11 bits by the (32, O)
 *          block code of Table 5.2.2.6.4-1, O > 11 by CRC8 + the tail-biting convolutional code + 5.1.4.2;
 *   multiplexing (5.2.2.7): g = CQI symbols then data symbols;
 *   channel interleaver (5.2.2.8): a matrix of M_sc rows x 12 columns of Q_m-bit cells; RI cells first,
 *          from the last row up in ColumnSet {1, 4, 7, 10} (j = 0, 3, 2, 1, ...), then g row by row over
 *          the remaining cells, then HARQ-ACK overwriting from the last row up in {2, 3, 8, 9}; read
 *          column by column -> SC-FDMA data symbol l takes the rows of column l;
 *   scrambling (36.211 5.3.1): c_init = n_RNTI 2^14 + sf 2^9 + N_ID; modulation as the DL (7.1);
 *   transform precoding (5.3.3): z = (1/sqrt M) DFT_M per data symbol;
 *   DMRS (5.5.2.1): for M_sc = 12 / 24 (L_prb = 1, 2) the base sequences of Tables 5.5.1.2-1 / -2
 *          (transcribed; their low-PAPR design property is checked per row in the CPU suite, so this is
 *          pinned by the tables' defining property, not by a reference implementation), for M_sc >= 36 the
 *          ZC root q of N_ZC = largest prime < M_sc; group hopping f_gh, sequence
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

/* 36.213 Table 8.6.3-2 (RI, I 0..12) and Table 8.6.3-3 (CQI, I 2..15; 0, 1 reserved), x 8 */
static const uint32_t BETA8_RI[13] = {10, 13, 16, 20, 25, 32, 40, 50, 64, 80, 101, 127, 160};
static const uint32_t BETA8_CQI[16] = {0, 0, 9, 10, 11, 13, 14, 16, 18, 20, 23, 25, 28, 32, 40, 50};

static uint64_t ul_sum_k(const or_ul_cfg_t *c) {
  or_cbsegm_t sg;
  if (or_cbsegm(c->tbs, &sg)) return 0;
  return (uint64_t)sg.Cm * sg.Km + (uint64_t)(sg.C - sg.Cm) * sg.Kp;
}

uint32_t or_ri_qprime(const or_ul_cfg_t *c) {
  if (!c->ri_len) return 0;
  const uint64_t sk = ul_sum_k(c), M = 12 * c->L_prb;
  if (!sk || c->ri_len > 2 || c->I_offset_ri > 12) return (uint32_t)-1;
  const uint64_t q = ((uint64_t)c->ri_len * M * 12 * BETA8_RI[c->I_offset_ri] + 8 * sk - 1) / (8 * sk);
  return (uint32_t)(q < 4 * M ? q : 4 * M);
}

uint32_t or_cqi_qprime(const or_ul_cfg_t *c) {
  if (!c->cqi_len) return 0;
  const uint64_t sk = ul_sum_k(c), M = 12 * c->L_prb, L = c->cqi_len > 11 ? 8 : 0;
  const uint32_t qri = or_ri_qprime(c);
  if (!sk || c->cqi_len > 64 || c->I_offset_cqi < 2 || c->I_offset_cqi > 15 || qri == (uint32_t)-1)
    return (uint32_t)-1;
  const uint64_t q = ((c->cqi_len + L) * M * 12 * BETA8_CQI[c->I_offset_cqi] + 8 * sk - 1) / (8 * sk);
  const uint64_t cap = 12 * M - qri;
  return (uint32_t)(q < cap ? q : cap);
}

/* 36.212 Table 5.2.2.6.4-1: basis sequences M_{i,n} of the (32, O) code, row i, column n = 0..10 */
static const uint8_t RM32[32][11] = {
  {1,1,0,0,0,0,0,0,0,0,1}, {1,1,1,0,0,0,0,0,0,1,1}, {1,0,0,1,0,0,1,0,1,1,1}, {1,0,1,1,0,0,0,0,1,0,1},
  {1,1,1,1,0,0,0,1,0,0,1}, {1,1,0,0,1,0,1,1,1,0,1}, {1,0,1,0,1,0,1,0,1,1,1}, {1,0,0,1,1,0,0,1,1,0,1},
  {1,1,0,1,1,0,0,1,0,1,1}, {1,0,1,1,1,0,1,0,0,1,1}, {1,0,1,0,0,1,1,1,0,1,1}, {1,1,1,0,0,1,1,0,1,0,1},
  {1,0,0,1,0,1,0,1,1,1,1}, {1,1,0,1,0,1,0,1,0,1,1}, {1,0,0,0,1,1,0,1,0,0,1}, {1,1,0,0,1,1,1,1,0,1,1},
  {1,1,1,0,1,1,1,0,0,1,0}, {1,0,0,1,1,1,0,0,1,0,0}, {1,1,0,1,1,1,1,1,0,0,0}, {1,0,0,0,0,1,1,0,0,0,0},
  {1,0,1,0,0,0,1,0,0,0,1}, {1,1,0,1,0,0,0,0,0,1,1}, {1,0,0,0,1,0,0,1,1,0,1}, {1,1,1,0,1,0,0,0,1,1,1},
  {1,1,1,1,1,0,1,1,1,1,0}, {1,1,0,0,0,1,1,1,0,0,1}, {1,0,1,1,0,1,0,0,1,1,0}, {1,1,1,1,0,1,0,1,1,1,0},
  {1,0,1,0,1,1,1,0,1,0,0}, {1,0,1,1,1,1,1,1,1,0,0}, {1,1,1,1,1,1,1,1,1,1,1}, {1,0,0,0,0,0,0,0,0,0,0}};

uint32_t or_cqi_rm32(const uint8_t *o, uint32_t O) {
  uint32_t w = 0;
  for (uint32_t i = 0; i < 32; i++) {
    uint32_t b = 0;
    for (uint32_t n = 0; n < O && n < 11; n++) b ^= (uint32_t)(o[n] & RM32[i][n]);
    w = (w << 1) | b;
  }
  return w;
}

int or_cqi_encode(const or_ul_cfg_t *c, uint8_t *q) {
  const uint32_t qp = or_cqi_qprime(c);
  if (qp == (uint32_t)-1) return -1;
  const uint32_t Q = qp * c->Qm, O = c->cqi_len;
  if (!Q) return 0;
  if (O <= 11) {   /* q_i = b_(i mod 32) */
    const uint32_t w = or_cqi_rm32(c->cqi, O);
    for (uint32_t i = 0; i < Q; i++) q[i] = (uint8_t)((w >> (31 - i % 32)) & 1u);
    return (int)Q;
  }
  /* 36.212 5.2.2.6.4 O > 11: CRC8 (g_CRC8 = D^8 + D^7 + D^4 + D^3 + D + 1), tail-biting convolutional
     code (5.1.3.1), rate matching to Q bits (5.1.4.2) */
  const uint32_t D = O + 8;
  uint8_t a[72], d[3 * 72];
  memcpy(a, c->cqi, O);
  const uint32_t crc = or_crc(c->cqi, O, 0x9Bu, 8);
  for (uint32_t i = 0; i < 8; i++) a[O + i] = (uint8_t)((crc >> (7 - i)) & 1u);
  or_conv_encode_tb(a, D, d);
  or_conv_rm_tx(d, D, Q, q);
  return (int)Q;
}

/* Tables 5.2.2.6-1..-4: the HARQ-ACK / RI block of `len` bits `v` (placeholders: 2 = x, 3 = y) */
static uint32_t uci_block(uint32_t len, uint32_t v, uint32_t Qm, uint8_t *blk) {
  const uint32_t o0 = v & 1, o1 = (v >> 1) & 1, o2 = o0 ^ o1;
  if (len == 1) {
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

uint32_t or_ack_block(const or_ul_cfg_t *c, uint8_t *blk) { return uci_block(c->ack_len, c->ack, c->Qm, blk); }
uint32_t or_ri_block(const or_ul_cfg_t *c, uint8_t *blk) { return uci_block(c->ri_len, c->ri, c->Qm, blk); }

int or_ulsch_encode(const or_ul_cfg_t *c, const uint8_t *tb, uint8_t *g) {
  const uint32_t A = c->tbs, qri = or_ri_qprime(c), qcqi = or_cqi_qprime(c);
  if (A == 0 || (c->Qm != 2 && c->Qm != 4 && c->Qm != 6)) return -1;
  if (qri == (uint32_t)-1 || qcqi == (uint32_t)-1) return -1;
  const uint32_t Qcqi = qcqi * c->Qm, G = or_pusch_G(c) - Qcqi - qri * c->Qm;
  if (or_cqi_encode(c, g) != (int)Qcqi) return -1;
  uint8_t *f = g + Qcqi;
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
  return (int)(Qcqi + G);
}

int or_pusch_mod(const or_ul_cfg_t *c, const uint8_t *g, float *x) {
  const uint32_t M = 12 * c->L_prb, Qm = c->Qm, G = or_pusch_G(c), R = M, NC = 12;
  const uint32_t qri = or_ri_qprime(c), qack = or_ack_qprime(c);
  if (qri == (uint32_t)-1 || qri > 4 * M) return -1;
  /* the interleaver matrix: R rows x 12 columns of Qm-bit cells (codes 0/1, 2 = x, 3 = y); ri[] marks RI */
  uint8_t *y = (uint8_t *)malloc((size_t)R * NC * Qm), *ri = (uint8_t *)calloc((size_t)R * NC, 1);
  uint8_t *cs = (uint8_t *)malloc(G), *h = (uint8_t *)malloc(G);
  static const uint32_t RI_COLS[4] = {1, 4, 7, 10}, ACK_COLS[4] = {2, 3, 8, 9};
  uint8_t blk[18];
  /* 1. RI from the last row up */
  uint32_t nb = c->ri_len ? or_ri_block(c, blk) : Qm;
  for (uint32_t i = 0, j = 0; i < qri; i++, j = (j + 3) % 4) {
    const uint32_t r = R - 1 - i / 4, col = RI_COLS[j];
    ri[r * NC + col] = 1;
    for (uint32_t b = 0; b < Qm; b++) y[(size_t)(r * NC + col) * Qm + b] = blk[(i * Qm + b) % nb];
  }
  /* 2. g (CQI then data) row by row over the cells RI left free */
  uint32_t k = 0;
  for (uint32_t r = 0; r < R; r++)
    for (uint32_t col = 0; col < NC; col++) {
      if (ri[r * NC + col]) continue;
      memcpy(y + (size_t)(r * NC + col) * Qm, g + (size_t)k * Qm, Qm);
      k++;
    }
  /* 3. HARQ-ACK overwrites from the last row up */
  nb = c->ack_len ? or_ack_block(c, blk) : Qm;
  for (uint32_t i = 0, j = 0; i < qack; i++, j = (j + 3) % 4) {
    const uint32_t r = R - 1 - i / 4, col = ACK_COLS[j];
    for (uint32_t b = 0; b < Qm; b++) y[(size_t)(r * NC + col) * Qm + b] = blk[(i * Qm + b) % nb];
  }
  /* 4. read column by column: SC-FDMA data symbol l = column l */
  for (uint32_t col = 0; col < NC; col++)
    for (uint32_t r = 0; r < R; r++) memcpy(h + (size_t)(col * R + r) * Qm, y + (size_t)(r * NC + col) * Qm, Qm);
  or_gold((c->rnti << 14) | (c->sf_idx << 9) | c->cell_id, cs, G);
  for (uint32_t i = 0; i < G; i++)            /* 36.211 5.3.1 with the UCI placeholders */
    h[i] = h[i] == 2 ? 1 : h[i] == 3 ? h[i - 1] : (uint8_t)(h[i] ^ cs[i]);
  for (uint32_t s = 0; s < 12 * M; s++) {
    uint8_t bi[3], bq[3];
    for (uint32_t jj = 0; jj < Qm / 2; jj++) { bi[jj] = h[s * Qm + 2 * jj]; bq[jj] = h[s * Qm + 2 * jj + 1]; }
    x[2 * s] = (float)or_pam_level(bi, Qm);
    x[2 * s + 1] = (float)or_pam_level(bq, Qm);
  }
  free(y); free(ri); free(cs); free(h);
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

/* 36.211 Tables 5.5.1.2-1 / 5.5.1.2-2: phi(n) of the base sequences for M_sc = 12 / 24, u = 0..29 */
static const int8_t PHI12[30][12] = {
    {-1,  1,  3, -3,  3,  3,  1,  1,  3,  1, -3,  3},
    { 1,  1,  3,  3,  3, -1,  1, -3, -3,  1, -3,  3},
    { 1,  1, -3, -3, -3, -1, -3, -3,  1, -3,  1, -1},
    {-1,  1,  1,  1,  1, -1, -3, -3,  1, -3,  3, -1},
    {-1,  3,  1, -1,  1, -1, -3, -1,  1, -1,  1,  3},
    { 1, -3,  3, -1, -1,  1,  1, -1, -1,  3, -3,  1},
    {-1,  3, -3, -3, -3,  3,  1, -1,  3,  3, -3,  1},
    {-3, -1, -1, -1,  1, -3,  3, -1,  1, -3,  3,  1},
    { 1, -3,  3,  1, -1, -1, -1,  1,  1,  3, -1,  1},
    { 1, -3, -1,  3,  3, -1, -3,  1,  1,  1,  1,  1},
    {-1,  3, -1,  1,  1, -3, -3, -1, -3, -3,  3, -1},
    { 3,  1, -1, -1,  3,  3, -3,  1,  3,  1,  3,  3},
    { 1, -3,  1,  1, -3,  1,  1,  1, -3, -3, -3,  1},
    { 3,  3, -3,  3, -3,  1,  1,  3, -1, -3,  3,  3},
    {-3,  1, -1, -3, -1,  3,  1,  3,  3,  3, -1,  1},
    { 3, -1,  1, -3, -1, -1,  1,  1,  3,  1, -1, -3},
    { 1,  3,  1, -1,  1,  3,  3,  3, -1, -1,  3, -1},
    {-3,  1,  1,  3, -3,  3, -3, -3,  3,  1,  3, -1},
    {-3,  3,  1,  1, -3,  1, -3, -3, -1, -1,  1, -3},
    {-1,  3,  1,  3,  1, -1, -1,  3, -3, -1, -3, -1},
    {-1, -3,  1,  1,  1,  1,  3,  1, -1,  1, -3, -1},
    {-1,  3, -1,  1, -3, -3, -3, -3, -3,  1, -1, -3},
    { 1,  1, -3, -3, -3, -3, -1,  3, -3,  1, -3,  3},
    { 1,  1, -1, -3, -1, -3,  1, -1,  1,  3, -1,  1},
    { 1,  1,  3,  1,  3,  3, -1,  1, -1, -3, -3,  1},
    { 1, -3,  3,  3,  1,  3,  3,  1, -3, -1, -1,  3},
    { 1,  3, -3, -3,  3, -3,  1, -1, -1,  3, -1, -3},
    {-3, -1, -3, -1, -3,  3,  1, -1,  1,  3, -3, -3},
    {-1,  3, -3,  3, -1,  3,  3, -3,  3,  3, -1, -1},
    { 3, -3, -3, -1, -1, -3, -1,  3, -3,  3,  1, -1}};
static const int8_t PHI24[30][24] = {
    {-1,  3,  1, -3,  3, -1,  1,  3, -3,  3,  1,  3, -3,  3,  1,  1, -1,  1,  3, -3,  3, -3, -1, -3},
    {-3,  3, -3, -3, -3,  1, -3, -3,  3, -1,  1,  1,  1,  3,  1, -1,  3, -3, -3,  1,  3,  1,  1, -3},
    { 3, -1,  3,  3,  1,  1, -3,  3,  3,  3,  3,  1, -1,  3, -1,  1,  1, -1, -3, -1, -1,  1,  3,  3},
    {-1, -3,  1,  1,  3, -3,  1,  1, -3, -1, -1,  1,  3,  1,  3,  1, -1,  3,  1,  1, -3, -1, -3, -1},
    {-1, -1, -1, -3, -3, -1,  1,  1,  3,  3, -1,  3, -1,  1, -1, -3,  1, -1, -3, -3,  1, -3, -1, -1},
    {-3,  1,  1,  3, -1,  1,  3,  1, -3,  1, -3,  1,  1, -1, -1,  3, -1, -3,  3, -3, -3, -3,  1,  1},
    { 1,  1, -1, -1,  3, -3, -3,  3, -3,  1, -1, -1,  1, -1,  1,  1, -1, -3, -1,  1, -1,  3, -1, -3},
    {-3,  3,  3, -1, -1, -3, -1,  3,  1,  3,  1,  3,  1,  1, -1,  3,  1, -1,  1,  3, -3, -1, -1,  1},
    {-3,  1,  3, -3,  1, -1, -3,  3, -3,  3, -1, -1, -1, -1,  1, -3, -3, -3,  1, -3, -3, -3,  1, -3},
    { 1,  1, -3,  3,  3, -1, -3, -1,  3, -3,  3,  3,  3, -1,  1,  1, -3,  1, -1,  1,  1, -3,  1,  1},
    {-1,  1, -3, -3,  3, -1,  3, -1, -1, -3, -3, -3, -1, -3, -3,  1, -1,  1,  3,  3, -1,  1, -1,  3},
    { 1,  3,  3, -3, -3,  1,  3,  1, -1, -3, -3, -3,  3,  3, -3,  3,  3, -1, -3,  3, -1,  1, -3,  1},
    { 1,  3,  3,  1,  1,  1, -1, -1,  1, -3,  3, -1,  1,  1, -3,  3,  3, -1, -3,  3, -3, -1, -3, -1},
    { 3, -1, -1, -1, -1, -3, -1,  3,  3,  1, -1,  1,  3,  3,  3, -1,  1,  1, -3,  1,  3, -1, -3,  3},
    {-3, -3,  3,  1,  3,  1, -3,  3,  1,  3,  1,  1,  3,  3, -1, -1, -3,  1, -3, -1,  3,  1,  1,  3},
    {-1, -1,  1, -3,  1,  3, -3,  1, -1, -3, -1,  3,  1,  3,  1, -1, -3, -3, -1, -1, -3, -3, -3, -1},
    {-1, -3,  3, -1, -1, -1, -1,  1,  1, -3,  3,  1,  3,  3,  1, -1,  1, -3,  1, -3,  1,  1, -3, -1},
    { 1,  3, -1,  3,  3, -1, -3,  1, -1, -3,  3,  3,  3, -1,  1,  1,  3, -1, -3, -1,  3, -1, -1, -1},
    { 1,  1,  1,  1,  1, -1,  3, -1, -3,  1,  1,  3, -3,  1, -3, -1,  1,  1, -3, -3,  3,  1,  1, -3},
    { 1,  3,  3,  1, -1, -3,  3, -1,  3,  3,  3, -3,  1, -1,  1, -1, -3, -1,  1,  3, -1,  3, -3, -3},
    {-1, -3,  3, -3, -3, -3, -1, -1, -3, -1, -3,  3,  1,  3, -3, -1,  3, -1,  1, -1,  3, -3,  1, -1},
    {-3, -3,  1,  1, -1,  1, -1,  1, -1,  3,  1, -3, -1,  1, -1,  1, -1, -1,  3,  3, -3, -1,  1, -3},
    {-3, -1, -3,  3,  1, -1, -3, -1, -3, -3,  3, -3,  3, -3, -1,  1,  3,  1, -3,  1,  3,  3, -1, -3},
    {-1, -1, -1, -1,  3,  3,  3,  1,  3,  3, -3,  1,  3, -1,  3, -1,  3,  3, -3,  3,  1, -1,  3,  3},
    { 1, -1,  3,  3, -1, -3,  3, -3, -1, -1,  3, -1,  3, -1, -1,  1,  1,  1,  1, -1, -1, -3, -1,  3},
    { 1, -1,  1, -1,  3, -1,  3,  1,  1, -1, -1, -3,  1,  1, -3,  1,  3, -3,  1,  1, -3, -3, -1, -1},
    {-3, -1,  1,  3,  1,  1, -3, -1, -1, -3,  3, -3,  3,  1, -3,  3, -3,  1, -1,  1, -3,  1,  1,  1},
    {-1, -3,  3,  3,  1,  1,  3, -1, -3, -1, -1, -1,  3,  1, -3, -3, -1,  3, -3, -1, -3, -1, -3, -1},
    {-1, -3, -1, -1,  1, -3, -1, -1,  1, -1, -3,  1,  1, -3,  1, -3, -3,  3,  1,  1, -1,  3, -1, -1},
    { 1,  1, -1, -1, -3, -1,  3, -1,  3, -1,  1,  3,  1, -1,  3,  1,  3, -3, -3,  1, -1, -1,  1,  3}};

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
  return M == 12 || M == 24 || M >= 36 ? 0 : -1;
}

int or_dmrs_pusch(const or_ul_cfg_t *c, uint32_t ns, float *r) {
  const uint32_t M = 12 * c->L_prb;
  uint32_t u, v, ncs;
  if (or_dmrs_params(c, ns, &u, &v, &ncs)) return -1;
  if (M < 36) {   /* 5.5.1.2: r_u(n) = exp(j phi(n) pi / 4), tabulated for M_sc = 12 and 24 */
    for (uint32_t n = 0; n < M; n++) {
      const double ph = M_PI * (M == 12 ? PHI12[u][n] : PHI24[u][n]) / 4.0 + 2.0 * M_PI * (double)((ncs * n) % 12) / 12.0;
      r[2 * n] = (float)cos(ph);
      r[2 * n + 1] = (float)sin(ph);
    }
    return 0;
  }
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
  if (c->n_prb + c->L_prb > c->nof_prb || M < 12) return -1;
  if (c->hop && c->n_prb1 + c->L_prb > c->nof_prb) return -1;
  uint8_t *f = (uint8_t *)malloc(G);
  float *x = (float *)malloc(sizeof(float) * 2 * 12 * M), *z = (float *)malloc(sizeof(float) * 2 * M);
  if (or_ulsch_encode(c, tb, f) < 0 || or_pusch_mod(c, f, x)) { free(f); free(x); free(z); return -1; }
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

/* ---- PUSCH frequency hopping type 2 (36.211 5.3.4) ------------------------------------------------------
 * Restated per VRB: n~_PRB(n_s) = (n~_VRB + f_hop(i) N_RB^sb + ((N_RB^sb - 1) - 2 (n~_VRB mod N_RB^sb)) f_m(i))
 * mod (N_RB^sb N_sb), i = n_s (intra- and inter-subframe hopping) or floor(n_s / 2) (inter-subframe), with the
 * pseudo-random c(k) of 7.2 initialised with N_ID^cell at the start of each frame; the hopping region is shifted
 * by N~_RB^HO / 2 when N_sb > 1.  Writes the slot's PRB of every VRB (prb[L]); returns the lowest, or -1. */
static uint32_t hop_fhop(const uint8_t *c, uint32_t i, uint32_t nsb) {
  if (nsb == 1) return 0;
  uint32_t f = 0;                            /* f_hop(-1) = 0 */
  for (uint32_t j = 0; j <= i; j++) {
    uint32_t x = 0;
    for (uint32_t b = 0; b < 9; b++) x |= (uint32_t)c[10 * j + 1 + b] << b;
    f = (nsb == 2) ? (f + x) % nsb : (f + (x % (nsb - 1)) + 1) % nsb;
  }
  return f;
}

int or_pusch_hop_type2(uint32_t nof_prb, uint32_t n_ho, uint32_t n_sb, int intra, uint32_t cell_id, uint32_t n_vrb,
                       uint32_t L, uint32_t ns, uint32_t current_tx_nb, uint32_t *prb) {
  uint8_t c[220];
  if (n_sb < 1 || n_sb > 4 || ns > 19 || L < 1) return -1;
  or_gold(cell_id, c, 220);
  const uint32_t hot = (n_ho % 2) ? n_ho + 1 : n_ho;
  uint32_t nrb_sb, off;
  if (n_sb == 1) {
    nrb_sb = nof_prb;
    off = 0;
  } else {
    const int32_t w = (int32_t)nof_prb - (int32_t)hot - (int32_t)(nof_prb % 2);
    if (w <= 0) return -1;
    nrb_sb = (uint32_t)w / n_sb;
    off = hot / 2;
  }
  if (!nrb_sb) return -1;
  const uint32_t i = intra ? ns : ns / 2;
  const uint32_t fhop = hop_fhop(c, i, n_sb);
  const uint32_t fm = (n_sb > 1) ? c[10 * i] : (intra ? i % 2 : current_tx_nb % 2);
  int lo = -1;
  for (uint32_t l = 0; l < L; l++) {
    const int32_t vt = (int32_t)(n_vrb + l) - (int32_t)off;
    if (vt < 0 || (uint32_t)vt >= nrb_sb * n_sb) return -1;
    const uint32_t mirror = (nrb_sb - 1) - 2 * ((uint32_t)vt % nrb_sb);   /* may wrap: modular arithmetic below */
    const uint32_t pt = ((uint32_t)vt + fhop * nrb_sb + mirror * fm) % (nrb_sb * n_sb);
    prb[l] = pt + off;
    if (lo < 0 || (int)prb[l] < lo) lo = (int)prb[l];
  }
  /* a slot's allocation must stay one contiguous PRB run (SC-FDMA, 36.211 5.3.4): an allocation crossing a
     subband edge under mirroring maps to a split set, which is rejected (as the product's mi_ul_hop_type2) */
  uint32_t hi = 0;
  for (uint32_t l = 0; l < L; l++) {
    if (prb[l] >= nof_prb) return -1;
    if (prb[l] > hi) hi = prb[l];
  }
  if (hi - (uint32_t)lo + 1 != L) return -1;
  return lo;
}
