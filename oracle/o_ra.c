/*
 * o_ra.c -- DL resource allocation and DCI -> grant (TEST INFRASTRUCTURE ONLY, see oracle.h).
 *
 * Restates what srsLTE's srslte_dci_msg_to_dl_grant does for srsUE (phch_worker.cc:297, the grant of
 * the DCI found by srslte_ue_dl_find_dl_dci_type at :293), written from the specification:
 *   36.212 5.3.3.1.2 / 5.3.3.1.3 / 5.3.3.1.4  field layouts of DCI formats 1, 1A and 1C
 *   36.213 7.1.6.1 / 7.1.6.2 / 7.1.6.3         resource allocation types 0, 1 and 2 (RIV)
 *   36.211 6.2.3.2                             distributed VRB -> PRB mapping (gap, interleaver, slot hop)
 *   36.213 7.1.7                               MCS / TBS, format 1A N_PRB^1A and the 1C TBS table
 *
 * The formulations here are deliberately the literal ones of the specification text (the interleaver
 * as a written-row / read-column matrix with null cells, type-1 subsets as lists of RBGs), so that the
 * product's closed-form versions (srsue_amd/csrc/ue_dl.cpp) are checked against something different.
 * The PRB mask output uses the two-slot encoding of or_pdsch_re_list: bit 0 = PRB used in slot 0,
 * bit 1 = PRB used in slot 1.
 */
#include <string.h>

#include "oracle.h"

static uint32_t ra_ceil_log2(uint32_t x) { uint32_t n = 0; while ((1u << n) < x) n++; return n; }
static uint32_t ra_get(const uint8_t *b, uint32_t *pos, uint32_t n) {
  uint32_t v = 0;
  for (uint32_t i = 0; i < n; i++) v = (v << 1) | (b[(*pos)++] & 1u);
  return v;
}

/* 36.213 Table 7.1.6.1-1: RBG size P */
uint32_t or_rbg_size(uint32_t nof_prb) {
  if (nof_prb <= 10) return 1;
  if (nof_prb <= 26) return 2;
  if (nof_prb <= 63) return 3;
  return 4;
}

/* 36.211 Table 6.2.3.2-1: N_gap,1 and N_gap,2 (0 = not defined) */
uint32_t or_ngap(uint32_t nof_prb, int gap2) {
  if (gap2) {
    if (nof_prb < 50) return 0;
    return nof_prb <= 63 ? 9 : 16;
  }
  if (nof_prb <= 10) return (nof_prb + 1) / 2;
  if (nof_prb == 11) return 4;
  if (nof_prb <= 19) return 8;
  if (nof_prb <= 26) return 12;
  if (nof_prb <= 44) return 18;
  if (nof_prb <= 63) return 27;
  if (nof_prb <= 79) return 32;
  return 48;
}

/* N_VRB^DL of the distributed mapping (36.211 6.2.3.2) */
uint32_t or_nvrb_dist(uint32_t nof_prb, int gap2) {
  const uint32_t g = or_ngap(nof_prb, gap2);
  if (!gap2) return 2 * (g < nof_prb - g ? g : nof_prb - g);
  return g ? (nof_prb / (2 * g)) * 2 * g : 0;
}

/* 36.211 6.2.3.2, literal form: the VRBs of one interleaver unit of N~ VRBs are written row by row into a
 * 4-column matrix of N_row = ceil(N~ / 4P) P rows whose last N_null/2 rows of the 2nd and 4th column hold
 * null cells, and read out column by column (skipping nulls) as the slot-0 PRB order; slot 1 is shifted
 * by N~/2 inside the unit; finally the upper half of a unit is moved by the gap. */
int or_vrb_to_prb(uint32_t nof_prb, int gap2, uint32_t n_vrb, uint32_t slot) {
  const uint32_t P = or_rbg_size(nof_prb), Ngap = or_ngap(nof_prb, gap2);
  const uint32_t Nt = gap2 ? 2 * Ngap : or_nvrb_dist(nof_prb, 0), Nvrb = or_nvrb_dist(nof_prb, gap2);
  if (!Nt || n_vrb >= Nvrb) return -1;
  const uint32_t Nrow = ((Nt + 4 * P - 1) / (4 * P)) * P, Nnull = 4 * Nrow - Nt;
  int cell[4 * 4 * 28];        /* [row][col]: VRB index of the unit or -1 (null); N_row <= 4 * 28 */
  if (Nrow > 4 * 28) return -1;
  uint32_t v = 0;
  for (uint32_t r = 0; r < Nrow; r++)
    for (uint32_t c = 0; c < 4; c++) {
      const int is_null = (c == 1 || c == 3) && r >= Nrow - Nnull / 2;
      cell[r * 4 + c] = is_null ? -1 : (int)v++;
    }
  if (v != Nt) return -1;
  const uint32_t unit = n_vrb / Nt, nt = n_vrb % Nt;
  uint32_t pos = 0, found = 0, p0 = 0;
  for (uint32_t c = 0; c < 4 && !found; c++)
    for (uint32_t r = 0; r < Nrow; r++) {
      const int x = cell[r * 4 + c];
      if (x < 0) continue;
      if ((uint32_t)x == nt) { p0 = pos; found = 1; break; }
      pos++;
    }
  if (!found) return -1;
  uint32_t pt = slot ? (p0 + Nt / 2) % Nt : p0;
  pt += Nt * unit;
  return (int)(pt < Nt / 2 ? pt : pt + Ngap - Nt / 2);
}

/* 36.213 7.1.6.3: RIV -> (start, length) over an N-wide index space; -1 if out of range */
static int ra_riv_decode(uint32_t riv, uint32_t N, uint32_t *start, uint32_t *L) {
  /* search the (start, L) whose RIV equals riv (the definition read forwards) */
  for (uint32_t l = 1; l <= N; l++)
    for (uint32_t s = 0; s + l <= N; s++) {
      const uint32_t r = (l - 1 <= N / 2) ? N * (l - 1) + s : N * (N - l + 1) + (N - 1 - s);
      if (r == riv) { *start = s; *L = l; return 0; }
    }
  return -1;
}

/* 36.212 5.3.3.1.4: format 1C size.  36.213 7.1.6.3: N_step 2 (N < 50) / 4, N'_VRB = floor(N_VRB,gap1 / N_step) */
static uint32_t ra_1c_rba_bits(uint32_t nof_prb) {
  const uint32_t step = nof_prb < 50 ? 2 : 4, Np = or_nvrb_dist(nof_prb, 0) / step;
  return ra_ceil_log2(Np * (Np + 1) / 2);
}
uint32_t or_dci1c_size(uint32_t nof_prb) { return (nof_prb >= 50 ? 1 : 0) + ra_1c_rba_bits(nof_prb) + 5; }

/* 36.213 Table 7.1.7.2.3-1 (format 1C transport block sizes, I_TBS 0..31) */
static const uint16_t tbs_1c[32] = {40,  56,  72,  120, 136, 144, 176, 208, 224, 256, 280,
                                    296, 328, 336, 392, 488, 552, 600, 632, 696, 776, 840,
                                    904, 1000, 1064, 1128, 1224, 1288, 1384, 1480, 1608, 1736};

static int is_common_rnti(uint16_t rnti) { return rnti < 0x003D || rnti > 0xFFF3; }   /* RA 1..60, P, SI */

static void ra_mark_vrbs_distributed(or_dl_grant_t *g, uint32_t nof_prb, int gap2, uint32_t start, uint32_t L) {
  for (uint32_t n = start; n < start + L; n++)
    for (uint32_t s = 0; s < 2; s++) {
      const int p = or_vrb_to_prb(nof_prb, gap2, n, s);
      if (p >= 0 && (uint32_t)p < nof_prb) g->prb[p] |= (uint8_t)(1u << s);
    }
}

int or_dl_dci_to_grant(const uint8_t *bits, uint32_t nbits, uint16_t rnti, uint32_t nof_prb, or_dl_grant_t *g) {
  memset(g, 0, sizeof(*g));
  const uint32_t N = nof_prb, n1a = or_dci_size(OR_DCI_1A, N), n1 = or_dci_size(OR_DCI_1, N);
  const uint32_t n1c = or_dci1c_size(N);
  const int common = is_common_rnti(rnti);
  uint32_t pos = 0;
  if (nbits == n1a && bits[0] == 1) {
    /* 36.212 5.3.3.1.3 */
    const uint32_t rba = ra_ceil_log2(N * (N + 1) / 2);
    g->format = OR_DCI_1A;
    pos = 1;
    g->distributed = ra_get(bits, &pos, 1);
    uint32_t riv_bits = rba, gap_from_rba = 0;
    if (g->distributed && N >= 50 && !common) { gap_from_rba = 1; riv_bits = rba - 1; }
    if (gap_from_rba) g->gap2 = ra_get(bits, &pos, 1);
    const uint32_t riv = ra_get(bits, &pos, riv_bits);
    uint32_t start, L;
    if (ra_riv_decode(riv, N, &start, &L)) return -1;
    g->mcs = ra_get(bits, &pos, 5);
    g->harq = ra_get(bits, &pos, 3);
    const uint32_t ndi = ra_get(bits, &pos, 1);
    g->rv = ra_get(bits, &pos, 2);
    g->tpc = ra_get(bits, &pos, 2);
    if (common) {
      if (g->distributed && N >= 50) g->gap2 = ndi;     /* the NDI bit carries the gap */
    } else {
      g->ndi = ndi;
    }
    g->alloc_type = 2;
    if (!g->distributed) {
      for (uint32_t p = start; p < start + L; p++) g->prb[p] = 3;
    } else {
      if (start + L > or_nvrb_dist(N, (int)g->gap2)) return -1;
      ra_mark_vrbs_distributed(g, N, (int)g->gap2, start, L);
    }
    g->nof_prb = L;
    if (common) {
      g->Qm = 2;
      g->i_tbs = g->mcs;
      g->n_prb_tbs = (g->tpc & 1u) ? 3 : 2;       /* N_PRB^1A from the TPC LSB */
    } else {
      if (or_mcs(g->mcs, &g->Qm, &g->i_tbs)) return -1;
      g->n_prb_tbs = L;
    }
    if (g->i_tbs > 26) return -1;
  } else if (nbits == n1c && common) {
    /* 36.212 5.3.3.1.4 */
    const uint32_t step = N < 50 ? 2 : 4, Np = or_nvrb_dist(N, 0) / step;
    g->format = OR_DCI_1C;
    g->distributed = 1;
    if (N >= 50) g->gap2 = ra_get(bits, &pos, 1);
    const uint32_t riv = ra_get(bits, &pos, ra_1c_rba_bits(N));
    uint32_t s, l;
    if (ra_riv_decode(riv, Np, &s, &l)) return -1;
    const uint32_t start = s * step, L = l * step;
    if (start + L > or_nvrb_dist(N, (int)g->gap2)) return -1;
    g->mcs = ra_get(bits, &pos, 5);
    g->alloc_type = 2;
    ra_mark_vrbs_distributed(g, N, (int)g->gap2, start, L);
    g->nof_prb = L;
    g->Qm = 2;
    g->i_tbs = g->mcs;
    g->n_prb_tbs = 0;
    g->tbs = tbs_1c[g->mcs];
    return 0;
  } else if (nbits == n1) {
    /* 36.212 5.3.3.1.2 */
    const uint32_t P = or_rbg_size(N), nrbg = (N + P - 1) / P;
    g->format = OR_DCI_1;
    g->alloc_type = (N > 10) ? ra_get(bits, &pos, 1) : 0;
    if (g->alloc_type == 0) {
      for (uint32_t r = 0; r < nrbg; r++)
        if (ra_get(bits, &pos, 1))
          for (uint32_t p = r * P; p < r * P + P && p < N; p++) g->prb[p] = 3;
    } else {
      /* 36.213 7.1.6.2: subset p (ceil(log2 P) bits), shift (1 bit), bitmap over the subset's VRBs */
      const uint32_t pb = ra_ceil_log2(P), nt1 = nrbg - pb - 1;
      const uint32_t sub = ra_get(bits, &pos, pb), shift = ra_get(bits, &pos, 1);
      if (sub >= P) return -1;
      uint32_t list[OR_NRB_MAX], nl = 0;            /* the subset's PRBs in ascending order */
      for (uint32_t r = sub; r < nrbg; r += P)
        for (uint32_t p = r * P; p < r * P + P && p < N; p++) list[nl++] = p;
      const uint32_t delta = shift ? (nl > nt1 ? nl - nt1 : 0) : 0;
      for (uint32_t i = 0; i < nt1; i++)
        if (ra_get(bits, &pos, 1)) {
          if (i + delta >= nl) return -1;
          g->prb[list[i + delta]] = 3;
        }
    }
    for (uint32_t p = 0; p < N; p++) g->nof_prb += g->prb[p] ? 1 : 0;
    g->mcs = ra_get(bits, &pos, 5);
    g->harq = ra_get(bits, &pos, 3);
    g->ndi = ra_get(bits, &pos, 1);
    g->rv = ra_get(bits, &pos, 2);
    g->tpc = ra_get(bits, &pos, 2);
    if (!g->nof_prb || or_mcs(g->mcs, &g->Qm, &g->i_tbs)) return -1;
    g->n_prb_tbs = g->nof_prb;
  } else {
    return -1;
  }
  g->tbs = or_tbs(g->i_tbs, g->n_prb_tbs);   /* -1 for columns the oracle does not carry */
  return 0;
}
