/*
 * o_ctrl.c -- DL control channels: PHICH/PCFICH REG allocation, PDCCH (REG/CCE mapping, LLR
 * extraction), DCI channel coding and blind search (TEST INFRASTRUCTURE ONLY).  SURVEY.md 8f row f1.
 *
 * Restates what srsUE calls through srsLTE for the PDCCH (reference call sites):
 *   srslte_pdcch_extract_llr(&ue_dl.pdcch, sf_symbols, ce, 0, sf, cfi)      phch_worker.cc:260
 *   srslte_ue_dl_find_dl_dci_type(&ue_dl, &msg, cfi, sf, rnti, type)       phch_worker.cc:293
 *   srslte_ue_dl_find_ul_dci(&ue_dl, &msg, cfi, sf, rnti)                   phch_worker.cc:426
 *   srslte_dci_msg_to_dl_grant(&msg, rnti, nof_prb, &dci, &grant)            phch_worker.cc:297
 * from 3GPP TS 36.211 (6.2.4 REGs, 6.7.4 PCFICH, 6.8 PDCCH, 6.9.3 PHICH), 36.212 (5.1.3.1 tail-
 * biting convolutional code, 5.1.4.2 its rate matching, 5.3.3 DCI) and 36.213 (9.1.1 search spaces,
 * 7.1.6.3 RIV).  srsLTE is not in the container: parity against it is unpinned; the transmit side
 * below is the ground truth (a DCI put on the air must be found with the same bits, CCE and L).
 *
 * Decoder contract (the GPU kernels in srsue_amd/csrc/ctrl.hip reproduce it operation by operation):
 *   soft bits  LLR > 0 => bit 1; QPSK max-log (sigma^2 = 0.5 scale, as the PDSCH demapper), ZF/MMSE
 *              equalisation with the noise srsUE passes (0), descrambling by sign flips
 *   rate de-matching  every e_k is added into its circular-buffer position in increasing k
 *   Viterbi    64 states s = (c_{k-1} .. c_{k-6}) (bit 5 = most recent); tail biting decoded by three
 *              circular copies of the D steps from all-zero metrics; branch metric
 *              sum_i (o_i ? d_i : -d_i) added in order i = 0, 1, 2; ACS keeps predecessor
 *              ((t << 1) & 63) | b with b = 1 only if strictly better; traceback from the best
 *              final state (lowest index on ties); the middle copy's decisions are the output
 */
#include "oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* 36.212 Table 5.1.4-2: inter-column permutation of the convolutional-code sub-block interleaver */
static const uint8_t P_CONV[32] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                   0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};

uint32_t or_phich_ngroups(uint32_t nof_prb, uint32_t ng) {
  /* N_group = ceil(Ng (N_RB / 8)), Ng in {1/6, 1/2, 1, 2} (normal CP) */
  static const uint32_t num[4] = {1, 3, 6, 12}, den = 6;   /* Ng = num/6 */
  return (num[ng & 3] * nof_prb + 8 * den - 1) / (8 * den);
}

/* Symbol-0 REG starts are k0 = 6 m; later control symbols k0 = 4 m (<= 2 ports: no CRS there). */
static void reg_res(const or_cell_t *c, uint32_t l, uint32_t k0, uint32_t *re) {
  const uint32_t W = 12 * c->nof_prb;
  if (l == 0) {
    const uint32_t vs3 = (c->id % 6) % 3;   /* CRS of ports 0 and 1 assumed present (6.2.4) */
    int n = 0;
    for (uint32_t k = k0; k < k0 + 6; k++) if (k % 3 != vs3) re[n++] = k;
  } else {
    for (uint32_t i = 0; i < 4; i++) re[i] = l * W + k0 + i;
  }
}

int or_pdcch_regs(const or_ctrl_t *q, uint32_t *re4, uint32_t *n_cce) {
  const or_cell_t *c = &q->cell;
  const uint32_t W = 12 * c->nof_prb, L = (uint32_t)or_ctrl_symbols(c, q->cfi);
  const uint32_t n0 = 2 * c->nof_prb;
  uint8_t *used0 = (uint8_t *)calloc(n0, 1);   /* symbol-0 REGs taken by PCFICH / PHICH */
  /* PCFICH: 4 REGs at k = kbar + floor(i N_RB / 2) N_sc / 2 (6.7.4) */
  const uint32_t kbar = 6 * (c->id % (2 * c->nof_prb));
  for (uint32_t i = 0; i < 4; i++) used0[((kbar + (i * c->nof_prb / 2) * 6) % W) / 6] = 1;
  /* PHICH (6.9.3, normal duration): REG n_i of the symbol-0 REGs not used by PCFICH, in frequency
     order, n_i = (N_ID + m' + floor(i n0' / 3)) mod n0' */
  uint32_t free0[2 * OR_NRB_MAX], nf = 0;
  for (uint32_t r = 0; r < n0; r++) if (!used0[r]) free0[nf++] = r;
  const uint32_t ng = or_phich_ngroups(c->nof_prb, q->ng);
  for (uint32_t m = 0; m < ng; m++)
    for (uint32_t i = 0; i < 3; i++) used0[free0[(c->id + m + (i * nf) / 3) % nf]] = 2;
  /* PDCCH REGs in mapping order (6.8.5): for k' in frequency, for l' in the control symbols */
  uint32_t n = 0;
  for (uint32_t k = 0; k < W; k++)
    for (uint32_t l = 0; l < L; l++) {
      const int start = l == 0 ? (k % 6 == 0) : (k % 4 == 0);
      if (!start || (l == 0 && used0[k / 6])) continue;
      if (re4) reg_res(c, l, k, re4 + 4 * n);
      n++;
    }
  free(used0);
  if (n_cce) *n_cce = n / 9;
  return (int)n;
}

/* quadruplet interleaver (36.212 5.1.4.2.1 on quadruplets, dummies removed) + cyclic shift by
   N_ID: physical REG i carries logical quadruplet log[i] */
void or_pdcch_quad_perm(uint32_t M, uint32_t cell_id, uint32_t *log_of_reg) {
  const uint32_t R = (M + 31) / 32, ND = 32 * R - M;
  uint32_t *w = (uint32_t *)malloc(sizeof(uint32_t) * M), n = 0;
  for (uint32_t col = 0; col < 32; col++)
    for (uint32_t r = 0; r < R; r++) {
      const uint32_t y = r * 32 + P_CONV[col];
      if (y >= ND) w[n++] = y - ND;
    }
  for (uint32_t i = 0; i < M; i++) log_of_reg[i] = w[(i + cell_id) % M];
  free(w);
}

/* QPSK max-log soft bits of one symbol (same scale as the PDSCH demapper: (m0 - m1) / 0.5) */
static void qpsk_llr(double xr, double xi, float *l) {
  const double a = 1.0 / sqrt(2.0);
  double d0 = (xr - a) * (xr - a), d1 = (xr + a) * (xr + a);
  l[0] = (float)((d0 - d1) / 0.5);
  d0 = (xi - a) * (xi - a); d1 = (xi + a) * (xi + a);
  l[1] = (float)((d0 - d1) / 0.5);
}

int or_pdcch_llr(const or_ctrl_t *q, const float *grid, const float *ce, float noise, float *llr, uint32_t *n_cce) {
  const or_cell_t *c = &q->cell;
  const uint32_t W = 12 * c->nof_prb, plane = OR_NSYMB * W;
  const uint32_t M = (uint32_t)or_pdcch_regs(q, NULL, n_cce);
  uint32_t *re = (uint32_t *)malloc(sizeof(uint32_t) * 4 * M), *lg = (uint32_t *)malloc(sizeof(uint32_t) * M);
  or_pdcch_regs(q, re, NULL);
  or_pdcch_quad_perm(M, c->id, lg);
  uint8_t *cs = (uint8_t *)malloc(8 * M);
  or_gold(q->sf * 512 + c->id, cs, 8 * M);
  const int tm2 = c->nof_ports == 2;
  for (uint32_t i = 0; i < M; i++) {
    const uint32_t *r = re + 4 * i;
    double x[8];
    for (int j = 0; j < 4; j += tm2 ? 2 : 1) {
      if (!tm2) {
        double yr = grid[2 * r[j]], yi = grid[2 * r[j] + 1], hr = ce[2 * r[j]], hi = ce[2 * r[j] + 1];
        double den = hr * hr + hi * hi + noise;
        x[2 * j] = (yr * hr + yi * hi) / den;
        x[2 * j + 1] = (yi * hr - yr * hi) / den;
      } else {
        const float *c0 = ce, *c1 = ce + 2 * plane;
        double r0r = grid[2 * r[j]], r0i = grid[2 * r[j] + 1], r1r = grid[2 * r[j + 1]], r1i = grid[2 * r[j + 1] + 1];
        double h00r = c0[2 * r[j]], h00i = c0[2 * r[j] + 1], h01r = c0[2 * r[j + 1]], h01i = c0[2 * r[j + 1] + 1];
        double h10r = c1[2 * r[j]], h10i = c1[2 * r[j] + 1], h11r = c1[2 * r[j + 1]], h11i = c1[2 * r[j + 1] + 1];
        double hh = h00r * h00r + h00i * h00i + h11r * h11r + h11i * h11i;
        if (hh <= 0) hh = 1e-9;
        double s = sqrt(2.0) / hh;
        x[2 * j] = s * ((h00r * r0r + h00i * r0i) + (h11r * r1r + h11i * r1i));
        x[2 * j + 1] = s * ((h00r * r0i - h00i * r0r) + (h11i * r1r - h11r * r1i));
        x[2 * j + 2] = s * (-(h10r * r0r + h10i * r0i) + (h01r * r1r + h01i * r1i));
        x[2 * j + 3] = s * (-(h10i * r0r - h10r * r0i) + (h01r * r1i - h01i * r1r));
      }
    }
    float *o = llr + 8 * (size_t)lg[i];
    for (int j = 0; j < 4; j++) qpsk_llr(x[2 * j], x[2 * j + 1], o + 2 * j);
    for (int j = 0; j < 8; j++) if (cs[8 * lg[i] + j]) o[j] = -o[j];
  }
  free(re); free(lg); free(cs);
  return (int)M;
}

/* ---- 36.212 5.1.3.1 tail-biting convolutional code, K = 7, G = 133, 171, 165 (octal) ---- */
static const uint8_t G_CONV[3] = {0133, 0171, 0165};   /* bit 6 <-> c_k, bit 0 <-> c_{k-6} */
static int parity7(uint32_t x) { x ^= x >> 4; x ^= x >> 2; x ^= x >> 1; return (int)(x & 1); }

void or_conv_encode_tb(const uint8_t *c, uint32_t D, uint8_t *d) {
  for (uint32_t k = 0; k < D; k++) {
    uint32_t reg = 0;   /* bit 6 - j = c_{k-j} */
    for (uint32_t j = 0; j <= 6; j++) reg |= (uint32_t)c[(k + 7 * D - j) % D] << (6 - j);
    for (int i = 0; i < 3; i++) d[i * D + k] = (uint8_t)parity7(reg & G_CONV[i]);
  }
}

/* 36.212 5.1.4.2: sub-block interleaving of each stream (dummies at the front) -> w = v0 v1 v2;
   wmap[j] = i*D + position in stream i, or -1 for a dummy */
static int conv_wmap(uint32_t D, int32_t *wmap) {
  const uint32_t R = (D + 31) / 32, KP = 32 * R, ND = KP - D;
  for (uint32_t i = 0; i < 3; i++)
    for (uint32_t col = 0, n = 0; col < 32; col++)
      for (uint32_t r = 0; r < R; r++, n++) {
        const uint32_t y = r * 32 + P_CONV[col];
        wmap[i * KP + n] = y >= ND ? (int32_t)(i * D + (y - ND)) : -1;
      }
  return (int)(3 * KP);
}

int or_conv_rm_tx(const uint8_t *d, uint32_t D, uint32_t E, uint8_t *e) {
  int32_t *wm = (int32_t *)malloc(sizeof(int32_t) * 3 * 32 * ((D + 31) / 32));
  const int Kw = conv_wmap(D, wm);
  for (uint32_t k = 0, j = 0; k < E; j++) {
    const int32_t s = wm[j % Kw];
    if (s >= 0) e[k++] = d[s];
  }
  free(wm);
  return 0;
}

void or_conv_rm_rx(const float *e, uint32_t E, uint32_t D, float *d) {
  int32_t *wm = (int32_t *)malloc(sizeof(int32_t) * 3 * 32 * ((D + 31) / 32));
  const int Kw = conv_wmap(D, wm);
  for (uint32_t i = 0; i < 3 * D; i++) d[i] = 0.0f;
  for (uint32_t k = 0, j = 0; k < E; j++) {
    const int32_t s = wm[j % Kw];
    if (s >= 0) { d[s] = d[s] + e[k]; k++; }
  }
  free(wm);
}

void or_viterbi_tb(const float *d, uint32_t D, uint8_t *c) {
  const uint32_t T = 3 * D;
  float pm[64], np[64];
  uint64_t *surv = (uint64_t *)malloc(sizeof(uint64_t) * T);
  for (int s = 0; s < 64; s++) pm[s] = 0.0f;
  for (uint32_t k = 0; k < T; k++) {
    const uint32_t kk = k % D;
    uint64_t sv = 0;
    for (uint32_t t = 0; t < 64; t++) {
      const uint32_t u = t >> 5;
      float m[2];
      for (uint32_t b = 0; b < 2; b++) {
        const uint32_t s = ((t << 1) & 63) | b;
        const uint32_t reg = (u << 6) | s;   /* bit 6 = c_k, bits 5..0 = c_{k-1} .. c_{k-6} */
        float bm = 0.0f;
        for (int i = 0; i < 3; i++) {
          const float v = d[i * D + kk];
          bm = bm + (parity7(reg & G_CONV[i]) ? v : -v);
        }
        m[b] = pm[s] + bm;
      }
      const int pick = m[1] > m[0];
      np[t] = pick ? m[1] : m[0];
      sv |= (uint64_t)pick << t;
    }
    surv[k] = sv;
    memcpy(pm, np, sizeof(pm));
  }
  uint32_t t = 0;
  for (uint32_t s = 1; s < 64; s++) if (pm[s] > pm[t]) t = s;
  for (int k = (int)T - 1; k >= 0; k--) {
    if ((uint32_t)k >= D && (uint32_t)k < 2 * D) c[k - D] = (uint8_t)(t >> 5);
    const uint32_t b = (uint32_t)((surv[k] >> t) & 1u);
    t = ((t << 1) & 63) | b;
  }
  free(surv);
}

/* ---- 36.212 5.3.3: DCI sizes, CRC attachment with RNTI mask, coding ---- */
static uint32_t ceil_log2(uint32_t x) { uint32_t n = 0; while ((1u << n) < x) n++; return n; }
static int ambiguous(uint32_t n) {
  static const uint32_t a[10] = {12, 14, 16, 20, 24, 26, 32, 40, 44, 56};
  for (int i = 0; i < 10; i++) if (a[i] == n) return 1;
  return 0;
}
uint32_t or_dci_size(uint32_t format, uint32_t nof_prb) {
  const uint32_t rba = ceil_log2(nof_prb * (nof_prb + 1) / 2);
  uint32_t s0 = 14 + rba, s1a = 15 + rba;            /* FDD, no carrier indicator */
  uint32_t n01a = s0 > s1a ? s0 : s1a;
  if (ambiguous(n01a)) n01a++;
  if (format == OR_DCI_0 || format == OR_DCI_1A) return n01a;
  if (format == OR_DCI_1C) return or_dci1c_size(nof_prb);
  /* format 1: [RA header if N_RB > 10] [RBG bitmap] MCS 5, HARQ 3, NDI 1, RV 2, TPC 2 */
  const uint32_t P = nof_prb <= 10 ? 1 : nof_prb <= 26 ? 2 : nof_prb <= 63 ? 3 : 4;
  uint32_t s1 = (nof_prb > 10 ? 1 : 0) + (nof_prb + P - 1) / P + 13;
  /* 36.212 5.3.3.1.2: pad until neither the 0/1A size nor one of Table 5.3.3.1.2-1 */
  while (s1 == n01a || ambiguous(s1)) s1++;
  return s1;
}

static void put_bits(uint8_t *b, uint32_t *pos, uint32_t v, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) b[(*pos)++] = (uint8_t)((v >> (n - 1 - i)) & 1u);
}
static uint32_t get_bits(const uint8_t *b, uint32_t *pos, uint32_t n) {
  uint32_t v = 0;
  for (uint32_t i = 0; i < n; i++) v = (v << 1) | b[(*pos)++];
  return v;
}
uint32_t or_riv(uint32_t nof_prb, uint32_t rb_start, uint32_t L) {   /* 36.213 7.1.6.3 */
  return (L - 1 <= nof_prb / 2) ? nof_prb * (L - 1) + rb_start : nof_prb * (nof_prb - L + 1) + (nof_prb - 1 - rb_start);
}
int or_dci1a_pack(uint32_t nof_prb, const or_dci1a_t *g, uint8_t *bits) {
  const uint32_t n = or_dci_size(OR_DCI_1A, nof_prb), rba = ceil_log2(nof_prb * (nof_prb + 1) / 2);
  uint32_t p = 0;
  memset(bits, 0, n);
  put_bits(bits, &p, 1, 1);                    /* format 0 / 1A flag: 1 = 1A */
  put_bits(bits, &p, 0, 1);                    /* localized VRB */
  put_bits(bits, &p, or_riv(nof_prb, g->rb_start, g->L_crb), rba);
  put_bits(bits, &p, g->mcs, 5);
  put_bits(bits, &p, g->harq, 3);
  put_bits(bits, &p, g->ndi, 1);
  put_bits(bits, &p, g->rv, 2);
  put_bits(bits, &p, g->tpc, 2);
  return (int)n;
}
int or_dci1a_unpack(uint32_t nof_prb, const uint8_t *bits, uint32_t nbits, or_dci1a_t *g) {
  const uint32_t rba = ceil_log2(nof_prb * (nof_prb + 1) / 2);
  if (nbits != or_dci_size(OR_DCI_1A, nof_prb) || bits[0] != 1 || bits[1] != 0) return -1;
  uint32_t p = 2;
  const uint32_t riv = get_bits(bits, &p, rba);
  /* invert the RIV: L - 1 = riv / N, start = riv % N; if that overflows, the mirrored branch */
  uint32_t a = riv / nof_prb, b = riv % nof_prb;
  if (a + b < nof_prb) { g->L_crb = a + 1; g->rb_start = b; }
  else { g->L_crb = nof_prb - a + 1; g->rb_start = nof_prb - 1 - b; }
  g->mcs = get_bits(bits, &p, 5);
  g->harq = get_bits(bits, &p, 3);
  g->ndi = get_bits(bits, &p, 1);
  g->rv = get_bits(bits, &p, 2);
  g->tpc = get_bits(bits, &p, 2);
  return 0;
}

/* CRC16 over the payload, XOR with the RNTI (MSB first), appended */
static void dci_attach_crc(const uint8_t *a, uint32_t A, uint16_t rnti, uint8_t *c) {
  memcpy(c, a, A);
  const uint32_t p = or_crc16(a, A);
  for (uint32_t i = 0; i < 16; i++) c[A + i] = (uint8_t)(((p >> (15 - i)) ^ (rnti >> (15 - i))) & 1u);
}

int or_dci_encode(const uint8_t *a, uint32_t A, uint16_t rnti, uint32_t L, uint8_t *e) {
  const uint32_t D = A + 16;
  uint8_t *c = (uint8_t *)malloc(D), *d = (uint8_t *)malloc(3 * D);
  dci_attach_crc(a, A, rnti, c);
  or_conv_encode_tb(c, D, d);
  or_conv_rm_tx(d, D, 72 * L, e);
  free(c); free(d);
  return 0;
}

int or_dci_decode(const float *e, uint32_t L, uint32_t A, uint16_t rnti, uint8_t *a) {
  const uint32_t D = A + 16;
  float *d = (float *)malloc(sizeof(float) * 3 * D);
  uint8_t *c = (uint8_t *)malloc(D);
  or_conv_rm_rx(e, 72 * L, D, d);
  or_viterbi_tb(d, D, c);
  const uint32_t p = or_crc16(c, A);
  uint32_t rx = 0;
  for (uint32_t i = 0; i < 16; i++) rx = (rx << 1) | c[A + i];
  const int ok = ((p ^ rx) & 0xFFFFu) == rnti;
  if (a) memcpy(a, c, A);
  free(d); free(c);
  return ok;
}

/* ---- 36.213 9.1.1 search spaces; candidates in search order ---- */
int or_search_space(uint32_t n_cce, uint32_t sf, uint16_t rnti, int common, uint32_t *Ls, uint32_t *ncce) {
  static const uint32_t LU[4] = {1, 2, 4, 8}, MU[4] = {6, 6, 2, 2}, LC[2] = {4, 8}, MC[2] = {4, 2};
  uint32_t Y = 0;
  if (!common) {
    Y = rnti;
    for (uint32_t k = 0; k <= sf; k++) Y = (39827u * Y) % 65537u;
  }
  int n = 0;
  for (int li = 0; li < (common ? 2 : 4); li++) {
    const uint32_t L = common ? LC[li] : LU[li], M = common ? MC[li] : MU[li];
    const uint32_t nl = n_cce / L;
    if (!nl) continue;
    for (uint32_t m = 0; m < M; m++) {
      Ls[n] = L;
      ncce[n] = L * ((Y + m) % nl);
      n++;
    }
  }
  return n;
}

/* blind search (srslte_ue_dl_find_dl_dci_type / _find_ul_dci semantics, srsLTE's dci_blind_search: one
   format over all candidates of a space at a time, the first CRC match wins).  mode 0 (C-RNTI, DL):
   UE-specific space (L = 1, 2, 4, 8) with the 1A size then format 1, then the common space (L = 4, 8)
   with the 1A size.  mode 1 (UL): the same spaces with the 0/1A size, flag 0.  mode 2 (SI/RA/P-RNTI):
   the common space only, the 1A size then format 1C.  The 0/1A flag separates 1A (1) from 0 (0). */
int or_find_dci_mode(const float *llr, uint32_t n_cce, uint32_t nof_prb, uint32_t sf, uint16_t rnti, int mode,
                     or_dci_found_t *out) {
  uint32_t Ls[32], nc[32];
  for (int common = (mode == 2); common < 2; common++) {
    const int n = or_search_space(n_cce, sf, rnti, common, Ls, nc);
    uint32_t fmts[2] = {mode == 1 ? OR_DCI_0 : OR_DCI_1A, mode == 2 ? OR_DCI_1C : OR_DCI_1};
    const int nf = (mode == 1 || (common && mode == 0)) ? 1 : 2;
    for (int f = 0; f < nf; f++)
      for (int i = 0; i < n; i++) {
        const uint32_t A = or_dci_size(fmts[f], nof_prb);
        uint8_t a[OR_DCI_MAX_BITS];
        if (!or_dci_decode(llr + 72 * nc[i], Ls[i], A, rnti, a)) continue;
        if ((fmts[f] == OR_DCI_0 || fmts[f] == OR_DCI_1A) && a[0] != (mode == 1 ? 0 : 1)) continue;
        out->format = fmts[f];
        out->nbits = A;
        out->L = Ls[i];
        out->ncce = nc[i];
        memcpy(out->bits, a, A);
        return 1;
      }
  }
  return 0;
}
int or_find_dci(const float *llr, uint32_t n_cce, uint32_t nof_prb, uint32_t sf, uint16_t rnti, int ul,
                or_dci_found_t *out) {
  return or_find_dci_mode(llr, n_cce, nof_prb, sf, rnti, ul ? 1 : 0, out);
}

/* ---- transmit side (ground truth): one DCI on the air, noiseless, added to iq ---- */
/* OFDM modulation of the first Lc symbols of a per-port grid (double, [P][14][W] complex) through the
   flat per-port channel h (NULL: port 0 only, h = 1), added to the subframe IQ */
static void add_ctrl_grid(const or_cell_t *c, uint32_t Lc, const double *grid, const float *h_re_im, float *iq) {
  const uint32_t W = 12 * c->nof_prb, N = (uint32_t)or_symbol_sz(c->nof_prb), P = c->nof_ports;
  double *X = (double *)malloc(sizeof(double) * 2 * N), *x = (double *)malloc(sizeof(double) * 2 * N);
  const double nrm = 1.0 / sqrt((double)N);
  for (uint32_t p = 0; p < P; p++) {
    double hr = h_re_im ? h_re_im[2 * p] : (p == 0 ? 1.0 : 0.0), hi = h_re_im ? h_re_im[2 * p + 1] : 0.0;
    size_t pos = 0;
    for (uint32_t l = 0; l < OR_NSYMB; l++) {
      const uint32_t cp = (uint32_t)or_cp_len(N, l % 7);
      if (l < Lc) {
        memset(X, 0, sizeof(double) * 2 * N);
        const double *gl = grid + ((size_t)p * OR_NSYMB * W + l * W) * 2;
        for (uint32_t k = 0; k < W; k++) {
          const uint32_t bin = (k < W / 2) ? (N - W / 2 + k) : (k - W / 2 + 1);
          X[2 * bin] = gl[2 * k]; X[2 * bin + 1] = gl[2 * k + 1];
        }
        or_dft(X, x, N, 1);
        for (uint32_t t = 0; t < N + cp; t++) {
          const uint32_t src = (t + N - cp) % N;
          const double vr = x[2 * src] * nrm, vi = x[2 * src + 1] * nrm;
          iq[2 * (pos + t)] += (float)(vr * hr - vi * hi);
          iq[2 * (pos + t) + 1] += (float)(vr * hi + vi * hr);
        }
      }
      pos += N + cp;
    }
  }
  free(X); free(x);
}

/* SFBC (36.211 6.3.4.3) of one RE pair (r0, r1) of the control region onto ports 0 / 1 */
static void sfbc_put(double *grid, size_t plane, uint32_t r0, uint32_t r1, double x0r, double x0i, double x1r,
                     double x1i) {
  const double s2 = 1.0 / sqrt(2.0);
  double *g0 = grid, *g1 = grid + 2 * plane;
  g0[2 * r0] += s2 * x0r;  g0[2 * r0 + 1] += s2 * x0i;
  g1[2 * r0] += -s2 * x1r; g1[2 * r0 + 1] += s2 * x1i;
  g0[2 * r1] += s2 * x1r;  g0[2 * r1 + 1] += s2 * x1i;
  g1[2 * r1] += s2 * x0r;  g1[2 * r1 + 1] += -s2 * x0i;
}

int or_tx_pdcch(const or_ctrl_t *q, uint16_t rnti, uint32_t L, uint32_t ncce, const uint8_t *a, uint32_t A,
                const float *h_re_im, float *iq) {
  const or_cell_t *c = &q->cell;
  const uint32_t W = 12 * c->nof_prb, P = c->nof_ports;
  uint32_t n_cce;
  const uint32_t M = (uint32_t)or_pdcch_regs(q, NULL, &n_cce);
  if (ncce + L > n_cce) return -1;
  uint32_t *re = (uint32_t *)malloc(sizeof(uint32_t) * 4 * M), *lg = (uint32_t *)malloc(sizeof(uint32_t) * M);
  or_pdcch_regs(q, re, NULL);
  or_pdcch_quad_perm(M, c->id, lg);
  uint8_t *b = (uint8_t *)calloc(8 * M, 1), *on = (uint8_t *)calloc(M, 1), *cs = (uint8_t *)malloc(8 * M);
  or_dci_encode(a, A, rnti, L, b + 72 * ncce);
  for (uint32_t qd = 9 * ncce; qd < 9 * (ncce + L); qd++) on[qd] = 1;
  or_gold(q->sf * 512 + c->id, cs, 8 * M);
  for (uint32_t i = 0; i < 8 * M; i++) b[i] ^= cs[i];
  double *grid = (double *)calloc((size_t)2 * P * OR_NSYMB * W, sizeof(double));
  const double s2 = 1.0 / sqrt(2.0);
  for (uint32_t i = 0; i < M; i++) {
    const uint32_t qd = lg[i];
    if (!on[qd]) continue;   /* <NIL> quadruplets carry no power */
    double xr[4], xi[4];
    for (int j = 0; j < 4; j++) {
      xr[j] = (1 - 2 * (int)b[8 * qd + 2 * j]) * s2;
      xi[j] = (1 - 2 * (int)b[8 * qd + 2 * j + 1]) * s2;
    }
    const uint32_t *r = re + 4 * i;
    if (P == 1) {
      for (int j = 0; j < 4; j++) { grid[2 * r[j]] = xr[j]; grid[2 * r[j] + 1] = xi[j]; }
    } else {
      double *g0 = grid, *g1 = grid + (size_t)2 * OR_NSYMB * W;
      for (int j = 0; j < 4; j += 2) {   /* SFBC (6.3.4.3) on the REG's RE pairs */
        g0[2 * r[j]] = s2 * xr[j];          g0[2 * r[j] + 1] = s2 * xi[j];
        g1[2 * r[j]] = -s2 * xr[j + 1];     g1[2 * r[j] + 1] = s2 * xi[j + 1];
        g0[2 * r[j + 1]] = s2 * xr[j + 1];  g0[2 * r[j + 1] + 1] = s2 * xi[j + 1];
        g1[2 * r[j + 1]] = s2 * xr[j];      g1[2 * r[j + 1] + 1] = -s2 * xi[j];
      }
    }
  }
  add_ctrl_grid(c, (uint32_t)or_ctrl_symbols(c, q->cfi), grid, h_re_im, iq);
  free(re); free(lg); free(b); free(on); free(cs); free(grid);
  return 0;
}

/* ---- PHICH (36.211 6.9, 36.212 5.3.5, 36.213 9.1.2) ------------------------------------------
   srsUE: *ack = srslte_ue_dl_decode_phich(&ue_dl, tti % 10, I_lowest, n_dmrs)  (phch_worker.cc:381)
   Resource (FDD, I_PHICH = 0): group = (I_lowest + n_dmrs) mod N_group,
                                seq = (floor(I_lowest / N_group) + n_dmrs) mod 2 N_SF (N_SF = 4).
   HI (1 = ACK) -> 3 repeated bits -> BPSK z (bit 0 -> (1+j)/sqrt2) -> d(i) = w_seq(i mod 4) (1 - 2 c(i))
   z(floor(i / 4)), i < 12, c_init = (sf + 1)(2 N_ID + 1) 2^9 + N_ID; quadruplet i of the group on
   REG n_i of symbol 0 (normal duration); 2 ports: SFBC per RE pair as the PDCCH.
   Receiver contract (the GPU's phich_kernel): equalise as the PDCCH (noise 0), despread
   s = sum_i Re(conj(w(i mod 4)) (1 - 2 c(i)) x(i) (1 - j) / sqrt2) over i = 0..11 in order;
   hi_soft = -s (> 0 favours ACK); ACK iff hi_soft > 0 (maximum likelihood; no erasure threshold). */
static const int8_t PHICH_W[8][4][2] = {   /* Table 6.9.1-2 (normal CP): (re, im) */
    {{1, 0}, {1, 0}, {1, 0}, {1, 0}},  {{1, 0}, {-1, 0}, {1, 0}, {-1, 0}},
    {{1, 0}, {1, 0}, {-1, 0}, {-1, 0}}, {{1, 0}, {-1, 0}, {-1, 0}, {1, 0}},
    {{0, 1}, {0, 1}, {0, 1}, {0, 1}},  {{0, 1}, {0, -1}, {0, 1}, {0, -1}},
    {{0, 1}, {0, 1}, {0, -1}, {0, -1}}, {{0, 1}, {0, -1}, {0, -1}, {0, 1}}};

void or_phich_calc(uint32_t nof_prb, uint32_t ng, uint32_t I_lowest, uint32_t n_dmrs, uint32_t *group,
                   uint32_t *seq) {
  const uint32_t N = or_phich_ngroups(nof_prb, ng);
  *group = (I_lowest + n_dmrs) % N;
  *seq = (I_lowest / N + n_dmrs) % 8;
}

uint32_t or_phich_cinit(uint32_t cell_id, uint32_t sf) { return (sf + 1) * (2 * cell_id + 1) * 512 + cell_id; }

int or_phich_res(const or_ctrl_t *q, uint32_t group, uint32_t *re12) {
  const or_cell_t *c = &q->cell;
  const uint32_t W = 12 * c->nof_prb, n0 = 2 * c->nof_prb;
  if (group >= or_phich_ngroups(c->nof_prb, q->ng)) return -1;
  uint8_t used0[2 * OR_NRB_MAX] = {0};
  const uint32_t kbar = 6 * (c->id % (2 * c->nof_prb));
  for (uint32_t i = 0; i < 4; i++) used0[((kbar + (i * c->nof_prb / 2) * 6) % W) / 6] = 1;
  uint32_t free0[2 * OR_NRB_MAX], nf = 0;
  for (uint32_t r = 0; r < n0; r++) if (!used0[r]) free0[nf++] = r;
  for (uint32_t i = 0; i < 3; i++) reg_res(c, 0, 6 * free0[(c->id + group + (i * nf) / 3) % nf], re12 + 4 * i);
  return 0;
}

float or_phich_soft(const or_ctrl_t *q, const float *grid, const float *ce, uint32_t group, uint32_t seq) {
  const or_cell_t *c = &q->cell;
  const uint32_t plane = OR_NSYMB * 12 * c->nof_prb;
  uint32_t re[12];
  if (or_phich_res(q, group, re) || seq > 7) return 0.0f;
  uint8_t cs[12];
  or_gold(or_phich_cinit(c->id, q->sf), cs, 12);
  double x[24];
  const int tm2 = c->nof_ports == 2;
  for (int j = 0; j < 12; j += tm2 ? 2 : 1) {
    if (!tm2) {
      double yr = grid[2 * re[j]], yi = grid[2 * re[j] + 1], hr = ce[2 * re[j]], hi = ce[2 * re[j] + 1];
      double den = hr * hr + hi * hi;
      if (den <= 0) den = 1e-9;
      x[2 * j] = (yr * hr + yi * hi) / den;
      x[2 * j + 1] = (yi * hr - yr * hi) / den;
    } else {
      const float *c0 = ce, *c1 = ce + 2 * plane;
      const uint32_t a = re[j], b = re[j + 1];
      double r0r = grid[2 * a], r0i = grid[2 * a + 1], r1r = grid[2 * b], r1i = grid[2 * b + 1];
      double h00r = c0[2 * a], h00i = c0[2 * a + 1], h01r = c0[2 * b], h01i = c0[2 * b + 1];
      double h10r = c1[2 * a], h10i = c1[2 * a + 1], h11r = c1[2 * b], h11i = c1[2 * b + 1];
      double hh = h00r * h00r + h00i * h00i + h11r * h11r + h11i * h11i;
      if (hh <= 0) hh = 1e-9;
      double s = sqrt(2.0) / hh;
      x[2 * j] = s * ((h00r * r0r + h00i * r0i) + (h11r * r1r + h11i * r1i));
      x[2 * j + 1] = s * ((h00r * r0i - h00i * r0r) + (h11i * r1r - h11r * r1i));
      x[2 * j + 2] = s * (-(h10r * r0r + h10i * r0i) + (h01r * r1r + h01i * r1i));
      x[2 * j + 3] = s * (-(h10i * r0r - h10r * r0i) + (h01r * r1i - h01i * r1r));
    }
  }
  double s = 0.0;
  for (int i = 0; i < 12; i++) {
    const double wr = PHICH_W[seq][i % 4][0], wi = PHICH_W[seq][i % 4][1], sg = cs[i] ? -1.0 : 1.0;
    const double yr = wr * x[2 * i] + wi * x[2 * i + 1], yi = wr * x[2 * i + 1] - wi * x[2 * i];   /* conj(w) x */
    s += sg * (yr + yi) / sqrt(2.0);
  }
  return (float)(-s);
}

int or_tx_phich(const or_ctrl_t *q, uint32_t group, uint32_t seq, int ack, const float *h_re_im, float *iq) {
  const or_cell_t *c = &q->cell;
  const uint32_t W = 12 * c->nof_prb, P = c->nof_ports;
  const size_t plane = (size_t)OR_NSYMB * W;
  uint32_t re[12];
  if (or_phich_res(q, group, re) || seq > 7) return -1;
  uint8_t cs[12];
  or_gold(or_phich_cinit(c->id, q->sf), cs, 12);
  double d[24];
  const double s2 = 1.0 / sqrt(2.0), zb = ack ? -s2 : s2;   /* bit = HI, BPSK (1 - 2b)(1 + j)/sqrt2 */
  for (int i = 0; i < 12; i++) {
    const double wr = PHICH_W[seq][i % 4][0], wi = PHICH_W[seq][i % 4][1], sg = cs[i] ? -1.0 : 1.0;
    d[2 * i] = sg * (wr * zb - wi * zb);        /* w * z, z = zb (1 + j) */
    d[2 * i + 1] = sg * (wr * zb + wi * zb);
  }
  double *grid = (double *)calloc((size_t)2 * P * plane, sizeof(double));
  for (int j = 0; j < 12; j += (P == 2 ? 2 : 1)) {
    if (P == 1) { grid[2 * re[j]] = d[2 * j]; grid[2 * re[j] + 1] = d[2 * j + 1]; }
    else sfbc_put(grid, plane, re[j], re[j + 1], d[2 * j], d[2 * j + 1], d[2 * j + 2], d[2 * j + 3]);
  }
  add_ctrl_grid(c, 1, grid, h_re_im, iq);
  free(grid);
  return 0;
}
