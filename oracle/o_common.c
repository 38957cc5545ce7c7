/*
 * o_common.c -- spec tables and index helpers for the oracle (TEST INFRASTRUCTURE ONLY).
 *
 * Restates the srsLTE-1.0 helpers behind srslte_ue_dl_cfg_grant / srslte_ra_tbs_from_idx
 * (called at /root/reference/ue/src/phy/phch_worker.cc:337 and ue/src/phy/phy.cc:118) from
 * 3GPP TS 36.211 / 36.212 / 36.213.  srsLTE is not in the container: see oracle.h header.
 */
#include "oracle.h"
#include <math.h>
#include <string.h>

int or_symbol_sz(uint32_t nof_prb) {
  if (nof_prb <= 6) return 128;
  if (nof_prb <= 15) return 256;
  if (nof_prb <= 25) return 512;
  if (nof_prb <= 50) return 1024;
  if (nof_prb <= 75) return 1536;
  if (nof_prb <= 110) return 2048;
  return -1;
}

/* 36.211 Table 6.12-1, normal CP, scaled from the 30.72 Msps values */
int or_cp_len(uint32_t N, uint32_t l_in_slot) { return (int)((l_in_slot == 0 ? 160u : 144u) * N / 2048u); }

int or_sf_len(uint32_t nof_prb) { return 15 * or_symbol_sz(nof_prb); }

/* 36.211 7.2: length-31 Gold sequence, Nc = 1600 */
void or_gold(uint32_t c_init, uint8_t *c, uint32_t len) {
  const uint32_t Nc = 1600;
  /* run the two LFSRs bit by bit keeping 31-bit windows: bit i of s = x(n+i) */
  uint32_t s1 = 1, s2 = c_init & 0x7fffffffu;
  for (uint32_t n = 0; n < Nc + len; n++) {
    if (n >= Nc) c[n - Nc] = (uint8_t)((s1 ^ s2) & 1u);
    uint32_t nb1 = ((s1 >> 3) ^ s1) & 1u;                            /* x1(n+31)=x1(n+3)+x1(n) */
    uint32_t nb2 = ((s2 >> 3) ^ (s2 >> 2) ^ (s2 >> 1) ^ s2) & 1u;    /* x2(n+31)=x2(n+3)+x2(n+2)+x2(n+1)+x2(n) */
    s1 = (s1 >> 1) | (nb1 << 30);
    s2 = (s2 >> 1) | (nb2 << 30);
  }
}

/* bit-serial CRC, zero initial register, MSB first (36.212 5.1.1) */
uint32_t or_crc(const uint8_t *bits, uint32_t len, uint32_t poly, int order) {
  uint32_t mask = (order == 32) ? 0xffffffffu : ((1u << order) - 1u);
  uint32_t crc = 0;
  for (uint32_t i = 0; i < len; i++) {
    uint32_t fb = ((crc >> (order - 1)) & 1u) ^ (bits[i] & 1u);
    crc = (crc << 1) & mask;
    if (fb) crc ^= poly & mask;
  }
  return crc;
}
uint32_t or_crc24a(const uint8_t *b, uint32_t n) { return or_crc(b, n, 0x864CFBu, 24); }
uint32_t or_crc24b(const uint8_t *b, uint32_t n) { return or_crc(b, n, 0x800063u, 24); }
uint32_t or_crc16(const uint8_t *b, uint32_t n) { return or_crc(b, n, 0x11021u, 16); }

/* 36.212 Table 5.1.3-3: turbo interleaver parameters (K, f1, f2), 188 entries */
static const uint16_t qpp_tab[188][3] = {
  {40,3,10},{48,7,12},{56,19,42},{64,7,16},{72,7,18},{80,11,20},{88,5,22},{96,11,24},
  {104,7,26},{112,41,84},{120,103,90},{128,15,32},{136,9,34},{144,17,108},{152,9,38},{160,21,120},
  {168,101,84},{176,21,44},{184,57,46},{192,23,48},{200,13,50},{208,27,52},{216,11,36},{224,27,56},
  {232,85,58},{240,29,60},{248,33,62},{256,15,32},{264,17,198},{272,33,68},{280,103,210},{288,19,36},
  {296,19,74},{304,37,76},{312,19,78},{320,21,120},{328,21,82},{336,115,84},{344,193,86},{352,21,44},
  {360,133,90},{368,81,46},{376,45,94},{384,23,48},{392,243,98},{400,151,40},{408,155,102},{416,25,52},
  {424,51,106},{432,47,72},{440,91,110},{448,29,168},{456,29,114},{464,247,58},{472,29,118},{480,89,180},
  {488,91,122},{496,157,62},{504,55,84},{512,31,64},{528,17,66},{544,35,68},{560,227,420},{576,65,96},
  {592,19,74},{608,37,76},{624,41,234},{640,39,80},{656,185,82},{672,43,252},{688,21,86},{704,155,44},
  {720,79,120},{736,139,92},{752,23,94},{768,217,48},{784,25,98},{800,17,80},{816,127,102},{832,25,52},
  {848,239,106},{864,17,48},{880,137,110},{896,215,112},{912,29,114},{928,15,58},{944,147,118},{960,29,60},
  {976,59,122},{992,65,124},{1008,55,84},{1024,31,64},{1056,17,66},{1088,171,204},{1120,67,140},{1152,35,72},
  {1184,19,74},{1216,39,76},{1248,19,78},{1280,199,240},{1312,21,82},{1344,211,252},{1376,21,86},{1408,43,88},
  {1440,149,60},{1472,45,92},{1504,49,846},{1536,71,48},{1568,13,28},{1600,17,80},{1632,25,102},{1664,183,104},
  {1696,55,954},{1728,127,96},{1760,27,110},{1792,29,112},{1824,29,114},{1856,57,116},{1888,45,354},{1920,31,120},
  {1952,59,610},{1984,185,124},{2016,113,420},{2048,31,64},{2112,17,66},{2176,171,136},{2240,209,420},{2304,253,216},
  {2368,367,444},{2432,265,456},{2496,181,468},{2560,39,80},{2624,27,164},{2688,127,504},{2752,143,172},{2816,43,88},
  {2880,29,300},{2944,45,92},{3008,157,188},{3072,47,96},{3136,13,28},{3200,111,240},{3264,443,204},{3328,51,104},
  {3392,51,212},{3456,451,192},{3520,257,220},{3584,57,336},{3648,313,228},{3712,271,232},{3776,179,236},{3840,331,120},
  {3904,363,244},{3968,375,248},{4032,127,168},{4096,31,64},{4160,33,130},{4224,43,264},{4288,33,134},{4352,477,408},
  {4416,35,138},{4480,233,280},{4544,357,142},{4608,337,480},{4672,37,146},{4736,71,444},{4800,71,120},{4864,37,152},
  {4928,39,462},{4992,127,234},{5056,39,158},{5120,39,80},{5184,31,96},{5248,113,902},{5312,41,166},{5376,251,336},
  {5440,43,170},{5504,21,86},{5568,43,174},{5632,45,176},{5696,45,178},{5760,161,120},{5824,89,182},{5888,323,184},
  {5952,47,186},{6016,23,94},{6080,47,190},{6144,263,480}};

int or_cb_size_idx(uint32_t K) {
  for (int i = 0; i < 188; i++) if (qpp_tab[i][0] == K) return i;
  return -1;
}
uint32_t or_cb_size(uint32_t idx) { return idx < 188 ? qpp_tab[idx][0] : 0; }

int or_qpp_f(uint32_t K, uint32_t *f1, uint32_t *f2) {
  int i = or_cb_size_idx(K);
  if (i < 0) return -1;
  *f1 = qpp_tab[i][1]; *f2 = qpp_tab[i][2];
  return 0;
}

/* 36.212 5.1.3.2.3: Pi(i) = (f1*i + f2*i^2) mod K */
int or_qpp(uint32_t K, uint32_t *pi) {
  uint32_t f1, f2;
  if (or_qpp_f(K, &f1, &f2)) return -1;
  for (uint64_t i = 0; i < K; i++) pi[i] = (uint32_t)((f1 * i + (uint64_t)f2 * i % K * i) % K);
  return 0;
}

/* 36.212 5.1.2 code block segmentation */
int or_cbsegm(uint32_t tbs, or_cbsegm_t *s) {
  const uint32_t Z = 6144;
  uint32_t B = tbs + 24, Bp, C;
  memset(s, 0, sizeof(*s));
  if (B <= Z) { C = 1; Bp = B; }
  else { C = (B + (Z - 24) - 1) / (Z - 24); Bp = B + 24 * C; }
  /* K+ = min K with C*K >= B' */
  int ip = -1;
  for (int i = 0; i < 188; i++) if (C * qpp_tab[i][0] >= Bp) { ip = i; break; }
  if (ip < 0) return -1;
  uint32_t Kp = qpp_tab[ip][0], Km = 0, Cm = 0, Cp;
  if (C == 1) { Cp = 1; Km = 0; Cm = 0; }
  else {
    Km = ip > 0 ? qpp_tab[ip - 1][0] : 0;
    uint32_t dK = Kp - Km;
    Cm = (C * Kp - Bp) / dK;
    Cp = C - Cm;
  }
  s->C = C; s->Cp = Cp; s->Cm = Cm; s->Kp = Kp; s->Km = Km; s->B = B;
  s->F = Cp * Kp + Cm * Km - Bp;
  return 0;
}

/* 36.213 Table 7.1.7.1-1 (PDSCH MCS, 64QAM UE): Qm and I_TBS */
int or_mcs(uint32_t mcs, uint32_t *qm, uint32_t *i_tbs) {
  if (mcs <= 9) { *qm = 2; *i_tbs = mcs; }
  else if (mcs <= 16) { *qm = 4; *i_tbs = mcs - 1; }
  else if (mcs <= 28) { *qm = 6; *i_tbs = mcs - 2; }
  else return -1;
  return 0;
}

/* 36.213 Table 7.1.7.2.1-1, spot columns only (N_PRB = 6, 25, 50, 100); other columns are not
 * needed by the tests (the TBS on the hot path arrives in the grant, phch_worker.cc:355). */
static const int tbs6[27] = {152,208,256,328,408,504,600,712,808,936,1032,1192,1352,1544,1736,1800,
  1928,2152,2344,2600,2792,2984,3240,3496,3624,3752,4392};
static const int tbs25[27] = {680,904,1096,1416,1800,2216,2600,3112,3496,4008,4392,4968,5736,6456,7224,
  7736,7992,9144,9912,10680,11448,12576,13536,14112,15264,15840,18336};
static const int tbs50[27] = {1384,1800,2216,2856,3624,4392,5160,6200,6968,7992,8760,9912,11448,12960,
  14112,15264,16416,18336,19848,21384,22920,25456,27376,28336,30576,31704,36696};
static const int tbs100[27] = {2792,3624,4584,5736,7224,8760,10296,12216,14112,15840,17568,19848,22920,
  25456,28336,30576,32856,36696,39232,43816,46888,51024,55056,57336,61664,63776,75376};
int or_tbs(uint32_t i_tbs, uint32_t nof_prb) {
  if (i_tbs > 26) return -1;
  switch (nof_prb) {
    case 6: return tbs6[i_tbs];
    case 25: return tbs25[i_tbs];
    case 50: return tbs50[i_tbs];
    case 100: return tbs100[i_tbs];
    default: return -1;
  }
}

/* 36.211 6.10.1.1: CRS r_{l,ns}(m), m = 0 .. 2*110-1 (complex, interleaved) */
void or_crs_seq(uint32_t id, uint32_t ns, uint32_t l, float *re_im) {
  uint32_t c_init = 1024u * (7u * (ns + 1u) + l + 1u) * (2u * id + 1u) + 2u * id + 1u;
  uint8_t c[4 * OR_NRB_MAX];
  or_gold(c_init, c, 4 * OR_NRB_MAX);
  const double a = 1.0 / sqrt(2.0);
  for (int m = 0; m < 2 * OR_NRB_MAX; m++) {
    re_im[2 * m] = (float)(a * (1 - 2 * (int)c[2 * m]));
    re_im[2 * m + 1] = (float)(a * (1 - 2 * (int)c[2 * m + 1]));
  }
}

int or_ctrl_symbols(const or_cell_t *c, uint32_t cfi) { return (int)cfi + (c->nof_prb <= 10 ? 1 : 0); }

/* Resource-element membership of the PDSCH (36.211 6.3.5 / 6.4 / 6.6 / 6.10 / 6.11, FDD, normal CP).
 * CRS REs of every configured port, PBCH (sf0, slot1 l=0..3) and PSS/SSS (sf0/5, slot0 l=5,6)
 * over the central 72 subcarriers are excluded. */
int or_is_pdsch_re(const or_cell_t *c, uint32_t cfi, uint32_t sf, uint32_t l, uint32_t k) {
  if ((int)l < or_ctrl_symbols(c, cfi)) return 0;
  uint32_t lp = l % 7, vs = c->id % 6;
  if (lp == 0 || lp == 4) {
    if (c->nof_ports == 1) {
      uint32_t off = ((lp == 0 ? 0u : 3u) + vs) % 6u;
      if (k % 6 == off) return 0;
    } else {
      if (k % 3 == vs % 3) return 0;
    }
  }
  uint32_t center = 6 * c->nof_prb;
  if (k + 36 >= center && k < center + 36) {
    if (sf == 0 && l >= 7 && l <= 10) return 0;
    if ((sf == 0 || sf == 5) && (l == 5 || l == 6)) return 0;
  }
  return 1;
}

int or_pdsch_re_list(const or_cell_t *c, uint32_t cfi, uint32_t sf, const uint8_t *prb_mask,
                     uint32_t *re_idx) {
  int n = 0, two_slot = 0;
  uint32_t W = 12 * c->nof_prb;
  for (uint32_t p = 0; p < c->nof_prb; p++) two_slot |= prb_mask[p] >= 2;
  for (uint32_t l = 0; l < OR_NSYMB; l++)
    for (uint32_t p = 0; p < c->nof_prb; p++) {
      if (two_slot ? !((prb_mask[p] >> (l / 7)) & 1u) : !prb_mask[p]) continue;
      for (uint32_t k = 12 * p; k < 12 * p + 12; k++)
        if (or_is_pdsch_re(c, cfi, sf, l, k)) re_idx[n++] = l * W + k;
    }
  return n;
}

/* 36.212 5.1.4.1.2: rate-matching output length E_r of code block r */
int or_rm_E(uint32_t G, uint32_t C, uint32_t Qm, uint32_t NL, uint32_t r) {
  uint32_t Gp = G / (NL * Qm);
  uint32_t gamma = Gp % C;
  if (r <= C - gamma - 1) return (int)(NL * Qm * (Gp / C));
  return (int)(NL * Qm * ((Gp + C - 1) / C));
}
