// tables.cpp -- host-side spec tables and index maps used by the batch planner (see tables.h).
// 3GPP TS 36.211 / 36.212 / 36.213 Rel-8; the srsLTE entry points they back are cited in
// include/srslte/srslte.h.
#include "tables.h"
#include "tbs_table.h"

#include <math.h>

#include <algorithm>
#include <string.h>

#include "dl_common.h"

namespace mi {

// 36.212 Table 5.1.3-3 (K, f1, f2)
static const uint16_t QPP[188][3] = {
    {40, 3, 10},      {48, 7, 12},      {56, 19, 42},     {64, 7, 16},      {72, 7, 18},      {80, 11, 20},
    {88, 5, 22},      {96, 11, 24},     {104, 7, 26},     {112, 41, 84},    {120, 103, 90},   {128, 15, 32},
    {136, 9, 34},     {144, 17, 108},   {152, 9, 38},     {160, 21, 120},   {168, 101, 84},   {176, 21, 44},
    {184, 57, 46},    {192, 23, 48},    {200, 13, 50},    {208, 27, 52},    {216, 11, 36},    {224, 27, 56},
    {232, 85, 58},    {240, 29, 60},    {248, 33, 62},    {256, 15, 32},    {264, 17, 198},   {272, 33, 68},
    {280, 103, 210},  {288, 19, 36},    {296, 19, 74},    {304, 37, 76},    {312, 19, 78},    {320, 21, 120},
    {328, 21, 82},    {336, 115, 84},   {344, 193, 86},   {352, 21, 44},    {360, 133, 90},   {368, 81, 46},
    {376, 45, 94},    {384, 23, 48},    {392, 243, 98},   {400, 151, 40},   {408, 155, 102},  {416, 25, 52},
    {424, 51, 106},   {432, 47, 72},    {440, 91, 110},   {448, 29, 168},   {456, 29, 114},   {464, 247, 58},
    {472, 29, 118},   {480, 89, 180},   {488, 91, 122},   {496, 157, 62},   {504, 55, 84},    {512, 31, 64},
    {528, 17, 66},    {544, 35, 68},    {560, 227, 420},  {576, 65, 96},    {592, 19, 74},    {608, 37, 76},
    {624, 41, 234},   {640, 39, 80},    {656, 185, 82},   {672, 43, 252},   {688, 21, 86},    {704, 155, 44},
    {720, 79, 120},   {736, 139, 92},   {752, 23, 94},    {768, 217, 48},   {784, 25, 98},    {800, 17, 80},
    {816, 127, 102},  {832, 25, 52},    {848, 239, 106},  {864, 17, 48},    {880, 137, 110},  {896, 215, 112},
    {912, 29, 114},   {928, 15, 58},    {944, 147, 118},  {960, 29, 60},    {976, 59, 122},   {992, 65, 124},
    {1008, 55, 84},   {1024, 31, 64},   {1056, 17, 66},   {1088, 171, 204}, {1120, 67, 140},  {1152, 35, 72},
    {1184, 19, 74},   {1216, 39, 76},   {1248, 19, 78},   {1280, 199, 240}, {1312, 21, 82},   {1344, 211, 252},
    {1376, 21, 86},   {1408, 43, 88},   {1440, 149, 60},  {1472, 45, 92},   {1504, 49, 846},  {1536, 71, 48},
    {1568, 13, 28},   {1600, 17, 80},   {1632, 25, 102},  {1664, 183, 104}, {1696, 55, 954},  {1728, 127, 96},
    {1760, 27, 110},  {1792, 29, 112},  {1824, 29, 114},  {1856, 57, 116},  {1888, 45, 354},  {1920, 31, 120},
    {1952, 59, 610},  {1984, 185, 124}, {2016, 113, 420}, {2048, 31, 64},   {2112, 17, 66},   {2176, 171, 136},
    {2240, 209, 420}, {2304, 253, 216}, {2368, 367, 444}, {2432, 265, 456}, {2496, 181, 468}, {2560, 39, 80},
    {2624, 27, 164},  {2688, 127, 504}, {2752, 143, 172}, {2816, 43, 88},   {2880, 29, 300},  {2944, 45, 92},
    {3008, 157, 188}, {3072, 47, 96},   {3136, 13, 28},   {3200, 111, 240}, {3264, 443, 204}, {3328, 51, 104},
    {3392, 51, 212},  {3456, 451, 192}, {3520, 257, 220}, {3584, 57, 336},  {3648, 313, 228}, {3712, 271, 232},
    {3776, 179, 236}, {3840, 331, 120}, {3904, 363, 244}, {3968, 375, 248}, {4032, 127, 168}, {4096, 31, 64},
    {4160, 33, 130},  {4224, 43, 264},  {4288, 33, 134},  {4352, 477, 408}, {4416, 35, 138},  {4480, 233, 280},
    {4544, 357, 142}, {4608, 337, 480}, {4672, 37, 146},  {4736, 71, 444},  {4800, 71, 120},  {4864, 37, 152},
    {4928, 39, 462},  {4992, 127, 234}, {5056, 39, 158},  {5120, 39, 80},   {5184, 31, 96},   {5248, 113, 902},
    {5312, 41, 166},  {5376, 251, 336}, {5440, 43, 170},  {5504, 21, 86},   {5568, 43, 174},  {5632, 45, 176},
    {5696, 45, 178},  {5760, 161, 120}, {5824, 89, 182},  {5888, 323, 184}, {5952, 47, 186},  {6016, 23, 94},
    {6080, 47, 190},  {6144, 263, 480}};

static int qpp_index(uint32_t K) {
  int lo = 0, hi = 187;
  while (lo <= hi) {
    int m = (lo + hi) / 2;
    if (QPP[m][0] == K) return m;
    if (QPP[m][0] < K) lo = m + 1; else hi = m - 1;
  }
  return -1;
}

int qpp_params(uint32_t K, uint32_t* f1, uint32_t* f2) {
  int i = qpp_index(K);
  if (i < 0) return -1;
  *f1 = QPP[i][1];
  *f2 = QPP[i][2];
  return 0;
}
bool cb_size_valid(uint32_t K) { return qpp_index(K) >= 0; }

void qpp_table(uint32_t K, std::vector<uint32_t>& pi) {
  uint32_t f1 = 0, f2 = 0;
  qpp_params(K, &f1, &f2);
  pi.resize(K);
  // incremental form: Pi(i+1) = Pi(i) + g(i), g(i+1) = g(i) + 2 f2 (mod K)
  uint64_t p = 0, g = (f1 + f2) % K;
  for (uint32_t i = 0; i < K; i++) {
    pi[i] = (uint32_t)p;
    p = (p + g) % K;
    g = (g + 2ull * f2) % K;
  }
}

void crc_bit_table(uint32_t K, uint32_t poly, std::vector<uint32_t>& t) {
  t.resize(K);
  uint32_t c = poly;   // message "1": register = g mod x^24
  for (int i = (int)K - 1; i >= 0; i--) {
    t[i] = c;
    const uint32_t fb = (c >> 23) & 1u;   // append one zero bit
    c = ((c << 1) & 0xFFFFFFu) ^ (fb ? poly : 0u);
  }
}

int cbsegm(uint32_t tbs, CbSegm* s) {
  const uint32_t Z = 6144;
  memset(s, 0, sizeof(*s));
  uint32_t B = tbs + 24, C, Bp;
  if (B <= Z) { C = 1; Bp = B; }
  else { C = (B + Z - 24 - 1) / (Z - 24); Bp = B + 24 * C; }
  int ip = -1;
  for (int i = 0; i < 188; i++)
    if (C * QPP[i][0] >= Bp) { ip = i; break; }
  if (ip < 0) return -1;
  s->C = C; s->B = B; s->Kp = QPP[ip][0];
  if (C == 1) { s->Cp = 1; s->Km = 0; s->Cm = 0; }
  else {
    s->Km = ip > 0 ? QPP[ip - 1][0] : 0;
    s->Cm = (C * s->Kp - Bp) / (s->Kp - s->Km);
    s->Cp = C - s->Cm;
  }
  s->F = s->Cp * s->Kp + s->Cm * s->Km - Bp;
  return 0;
}

int mcs_to_itbs(uint32_t mcs, uint32_t* qm) {
  if (mcs <= 9) { *qm = 2; return (int)mcs; }
  if (mcs <= 16) { *qm = 4; return (int)mcs - 1; }
  if (mcs <= 28) { *qm = 6; return (int)mcs - 2; }
  return -1;
}

// 36.213 Table 7.1.7.2.1-1 (tbs_table.h): every I_TBS 0..26 and N_PRB 1..110
int tbs_from_idx(uint32_t i_tbs, uint32_t nof_prb) {
  if (i_tbs > 26 || nof_prb < 1 || nof_prb > 110) return -1;
  return (int)TBS_TABLE[i_tbs][nof_prb - 1];
}

uint32_t rm_E(uint32_t G, uint32_t C, uint32_t Qm, uint32_t NL, uint32_t r) {
  const uint32_t Gp = G / (NL * Qm), gamma = Gp % C;
  return r <= C - gamma - 1 ? NL * Qm * (Gp / C) : NL * Qm * ((Gp + C - 1) / C);
}

uint32_t ncb_of(uint32_t K) { return 3 * 32 * ((K + 4 + 31) / 32); }

uint32_t k0_of(uint32_t K, uint32_t rv) {
  const uint32_t R = (K + 4 + 31) / 32, Ncb = ncb_of(K);
  return R * (2 * ((Ncb + 8 * R - 1) / (8 * R)) * rv + 2);
}

// position in the circular buffer w of d-stream element (i, k): 36.212 5.1.4.1.1 inverted
void cb_pos_table(uint32_t K, std::vector<uint32_t>& pos) {
  const uint32_t D = K + 4, R = (D + 31) / 32, KP = 32 * R, ND = KP - D;
  pos.resize(3 * D);
  for (uint32_t k = 0; k < D; k++) {
    const uint32_t j = k + ND;                                  // y index of d_k
    const uint32_t kk01 = subblock_perm(j % 32) * R + j / 32;   // v index (streams 0 and 1)
    const uint32_t t = (j + KP - 1) % KP;                       // stream 2: y index = pi(kk) => t = P(c)+32r
    const uint32_t kk2 = subblock_perm(t % 32) * R + t / 32;
    pos[3 * k] = kk01;
    pos[3 * k + 1] = KP + 2 * kk01;
    pos[3 * k + 2] = KP + 2 * kk2 + 1;
  }
}

void cb_rank_table(uint32_t K, uint32_t F, std::vector<int32_t>& rank, uint32_t* Nv) {
  const uint32_t D = K + 4, R = (D + 31) / 32, KP = 32 * R, ND = KP - D, Ncb = 3 * KP;
  std::vector<uint8_t> null(Ncb, 0);
  for (uint32_t kk = 0; kk < KP; kk++) {
    const uint32_t c = subblock_perm(kk / R), r = kk % R;
    const uint32_t j01 = c + 32 * r, j2 = (c + 32 * r + 1) % KP;
    const bool n01 = j01 < ND || (j01 - ND) < F;   // dummy bit, or filler (d0 / d1 only)
    null[kk] = n01;
    null[KP + 2 * kk] = n01;
    null[KP + 2 * kk + 1] = j2 < ND;
  }
  rank.resize(Ncb);
  int32_t cnt = 0;
  for (uint32_t p = 0; p < Ncb; p++) {
    rank[p] = null[p] ? -1 : cnt;
    if (!null[p]) cnt++;
  }
  *Nv = (uint32_t)cnt;
}

void gold_bits(uint32_t c_init, uint32_t nbits, uint8_t* bits) {
  uint32_t x1 = 1, x2 = c_init & 0x7fffffffu;
  for (uint32_t n = 0; n < 1600 + nbits; n++) {
    if (n >= 1600) bits[n - 1600] = (uint8_t)((x1 ^ x2) & 1u);
    const uint32_t f1 = ((x1 >> 3) ^ x1) & 1u, f2 = ((x2 >> 3) ^ (x2 >> 2) ^ (x2 >> 1) ^ x2) & 1u;
    x1 = (x1 >> 1) | (f1 << 30);
    x2 = (x2 >> 1) | (f2 << 30);
  }
}

void gold_words(uint32_t c_init, uint32_t nbits, uint32_t* words) {
  std::vector<uint8_t> b(nbits + 32, 0);
  gold_bits(c_init, nbits, b.data());
  for (uint32_t w = 0; w < (nbits + 31) / 32; w++) {
    uint32_t v = 0;
    for (int i = 0; i < 32; i++) v |= (uint32_t)b[32 * w + i] << i;
    words[w] = v;
  }
}

void crs_seq(uint32_t id, uint32_t ns, uint32_t l, float* re_im) {
  const uint32_t c_init = 1024u * (7u * (ns + 1u) + l + 1u) * (2u * id + 1u) + 2u * id + 1u;
  uint8_t c[4 * NRB_MAX];
  gold_bits(c_init, 4 * NRB_MAX, c);
  const float a = 0.70710678118654752440f;
  for (int m = 0; m < 2 * NRB_MAX; m++) {
    re_im[2 * m] = a * (float)(1 - 2 * (int)c[2 * m]);
    re_im[2 * m + 1] = a * (float)(1 - 2 * (int)c[2 * m + 1]);
  }
}

int ctrl_symbols(uint32_t nof_prb, uint32_t cfi) { return (int)cfi + (nof_prb <= 10 ? 1 : 0); }

bool is_pdsch_re(uint32_t id, uint32_t nof_prb, uint32_t nof_ports, uint32_t cfi, uint32_t sf, uint32_t l, uint32_t k) {
  if ((int)l < ctrl_symbols(nof_prb, cfi)) return false;
  const uint32_t lp = l % 7, vs = id % 6;
  if (lp == 0 || lp == 4) {
    if (nof_ports == 1) {
      if (k % 6 == ((lp == 0 ? 0u : 3u) + vs) % 6) return false;
    } else if (k % 3 == vs % 3) {
      return false;
    }
  }
  const uint32_t center = 6 * nof_prb;
  if (k + 36 >= center && k < center + 36) {
    if (sf == 0 && l >= 7 && l <= 10) return false;                 // PBCH
    if ((sf == 0 || sf == 5) && (l == 5 || l == 6)) return false;   // SSS, PSS
  }
  return true;
}

uint32_t pdsch_re_list(uint32_t id, uint32_t nof_prb, uint32_t nof_ports, uint32_t cfi, uint32_t sf,
                       const uint8_t* prb_mask, std::vector<uint32_t>& re) {
  re.clear();
  const uint32_t W = 12 * nof_prb;
  uint8_t any_slot_bits = 0;
  for (uint32_t p = 0; p < nof_prb; p++) any_slot_bits |= prb_mask[p] & ~1u;
  // per-slot use of each PRB: bit 0 / bit 1 (distributed VRB), or "both" for 0/1 masks
  uint8_t use[2][110];
  for (uint32_t p = 0; p < nof_prb; p++) {
    use[0][p] = any_slot_bits ? (prb_mask[p] & 1u) : (prb_mask[p] != 0);
    use[1][p] = any_slot_bits ? ((prb_mask[p] >> 1) & 1u) : (prb_mask[p] != 0);
  }
  for (uint32_t l = 0; l < (uint32_t)NSYMB; l++)
    for (uint32_t p = 0; p < nof_prb; p++) {
      if (!use[l / 7][p]) continue;
      for (uint32_t k = 12 * p; k < 12 * p + 12; k++)
        if (is_pdsch_re(id, nof_prb, nof_ports, cfi, sf, l, k)) re.push_back(l * W + k);
    }
  return (uint32_t)re.size();
}

void pcfich_k(uint32_t id, uint32_t nof_prb, uint32_t* k16) {
  const uint32_t W = 12 * nof_prb, kbar = 6 * (id % (2 * nof_prb)), vs3 = (id % 6) % 3;
  int n = 0;
  for (uint32_t i = 0; i < 4; i++) {
    const uint32_t kreg = (kbar + (i * nof_prb / 2) * 6) % W;
    for (uint32_t k = kreg; k < kreg + 6; k++)
      if (k % 3 != vs3) k16[n++] = k;
  }
}

uint32_t pcfich_cinit(uint32_t id, uint32_t sf) { return (sf + 1) * (2 * id + 1) * 512 + id; }

void cfi_codeword(uint32_t cfi, uint8_t* b) {
  static const uint8_t pat[3][3] = {{0, 1, 1}, {1, 0, 1}, {1, 1, 0}};
  for (int i = 0; i < 32; i++) b[i] = (cfi >= 1 && cfi <= 3) ? pat[cfi - 1][i % 3] : 0;
}

// ---- DL control ---------------------------------------------------------------------------------
static const uint8_t P_CONV[32] = {1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
                                   0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30};

uint32_t phich_ngroups(uint32_t nof_prb, uint32_t ng) {
  static const uint32_t num[4] = {1, 3, 6, 12};   // Ng = num / 6; N_group = ceil(Ng N_RB / 8)
  return (num[ng & 3] * nof_prb + 47) / 48;
}

uint32_t pdcch_regs(uint32_t id, uint32_t nof_prb, uint32_t ng, uint32_t cfi, std::vector<uint32_t>* re4) {
  const uint32_t W = 12 * nof_prb, L = (uint32_t)ctrl_symbols(nof_prb, cfi), n0 = 2 * nof_prb;
  std::vector<uint8_t> used0(n0, 0);
  const uint32_t kbar = 6 * (id % (2 * nof_prb));
  for (uint32_t i = 0; i < 4; i++) used0[((kbar + (i * nof_prb / 2) * 6) % W) / 6] = 1;   // PCFICH
  std::vector<uint32_t> free0;
  for (uint32_t r = 0; r < n0; r++) if (!used0[r]) free0.push_back(r);
  const uint32_t nf = (uint32_t)free0.size(), ngr = phich_ngroups(nof_prb, ng);
  for (uint32_t m = 0; m < ngr; m++)                                                      // PHICH
    for (uint32_t i = 0; i < 3; i++) used0[free0[(id + m + (i * nf) / 3) % nf]] = 2;
  if (re4) re4->clear();
  const uint32_t vs3 = (id % 6) % 3;
  uint32_t n = 0;
  for (uint32_t k = 0; k < W; k++)
    for (uint32_t l = 0; l < L; l++) {
      const bool start = l == 0 ? (k % 6 == 0) : (k % 4 == 0);
      if (!start || (l == 0 && used0[k / 6])) continue;
      if (re4) {
        if (l == 0) {
          for (uint32_t kk = k; kk < k + 6; kk++) if (kk % 3 != vs3) re4->push_back(kk);
        } else {
          for (uint32_t i = 0; i < 4; i++) re4->push_back(l * W + k + i);
        }
      }
      n++;
    }
  return n;
}

void phich_calc(uint32_t nof_prb, uint32_t ng, uint32_t I_lowest, uint32_t n_dmrs, uint32_t* group, uint32_t* seq) {
  const uint32_t N = phich_ngroups(nof_prb, ng);
  *group = (I_lowest + n_dmrs) % N;
  *seq = (I_lowest / N + n_dmrs) % 8;
}

// REG n_i = (N_ID + m + floor(i n0' / 3)) mod n0' of the symbol-0 REGs not used by the PCFICH
// (36.211 6.9.3, normal duration), its 4 non-CRS REs each
int phich_res(uint32_t id, uint32_t nof_prb, uint32_t ng, uint32_t group, uint32_t* re12) {
  if (group >= phich_ngroups(nof_prb, ng)) return -1;
  const uint32_t W = 12 * nof_prb, n0 = 2 * nof_prb, vs3 = (id % 6) % 3;
  std::vector<uint8_t> used0(n0, 0);
  const uint32_t kbar = 6 * (id % (2 * nof_prb));
  for (uint32_t i = 0; i < 4; i++) used0[((kbar + (i * nof_prb / 2) * 6) % W) / 6] = 1;
  std::vector<uint32_t> free0;
  for (uint32_t r = 0; r < n0; r++) if (!used0[r]) free0.push_back(r);
  const uint32_t nf = (uint32_t)free0.size();
  uint32_t n = 0;
  for (uint32_t i = 0; i < 3; i++) {
    const uint32_t k0 = 6 * free0[(id + group + (i * nf) / 3) % nf];
    for (uint32_t k = k0; k < k0 + 6; k++) if (k % 3 != vs3) re12[n++] = k;
  }
  return 0;
}

void pdcch_quad_perm(uint32_t M, uint32_t id, std::vector<uint32_t>& log_of_reg) {
  const uint32_t R = (M + 31) / 32, ND = 32 * R - M;
  std::vector<uint32_t> w;
  w.reserve(M);
  for (uint32_t col = 0; col < 32; col++)
    for (uint32_t r = 0; r < R; r++) {
      const uint32_t y = r * 32 + P_CONV[col];
      if (y >= ND) w.push_back(y - ND);
    }
  log_of_reg.resize(M);
  for (uint32_t i = 0; i < M; i++) log_of_reg[i] = w[(i + id) % M];
}

uint32_t ceil_log2(uint32_t x) {
  uint32_t n = 0;
  while ((1u << n) < x) n++;
  return n;
}
static bool dci_ambiguous(uint32_t n) {
  return n == 12 || n == 14 || n == 16 || n == 20 || n == 24 || n == 26 || n == 32 || n == 40 || n == 44 || n == 56;
}
uint32_t dci_size(int format, uint32_t nof_prb) {
  const uint32_t rba = ceil_log2(nof_prb * (nof_prb + 1) / 2);
  uint32_t n01a = 15 + rba;   // 1A = 15 + RBA >= format 0 = 14 + RBA (FDD)
  if (dci_ambiguous(n01a)) n01a++;
  if (format == DCI_1C) return (nof_prb >= 50 ? 1 : 0) + dci1c_rba_bits(nof_prb) + 5;   // 36.212 5.3.3.1.4
  if (format != DCI_1) return n01a;
  const uint32_t P = nof_prb <= 10 ? 1 : nof_prb <= 26 ? 2 : nof_prb <= 63 ? 3 : 4;
  uint32_t s1 = (nof_prb > 10 ? 1 : 0) + (nof_prb + P - 1) / P + 13;
  // 36.212 5.3.3.1.2: pad until neither the 0/1A size nor one of Table 5.3.3.1.2-1
  while (s1 == n01a || dci_ambiguous(s1)) s1++;
  return s1;
}

uint32_t rbg_size(uint32_t nof_prb) { return nof_prb <= 10 ? 1 : nof_prb <= 26 ? 2 : nof_prb <= 63 ? 3 : 4; }

uint32_t n_gap(uint32_t nof_prb, bool gap2) {
  if (gap2) return nof_prb < 50 ? 0 : nof_prb < 64 ? 9 : 16;
  static const struct { uint32_t max_prb, gap; } T[] = {{11, 4}, {19, 8}, {26, 12}, {44, 18}, {63, 27}, {79, 32}, {110, 48}};
  if (nof_prb <= 10) return (nof_prb + 1) / 2;
  for (const auto& t : T)
    if (nof_prb <= t.max_prb) return t.gap;
  return 0;
}

uint32_t n_vrb_dist(uint32_t nof_prb, bool gap2) {
  const uint32_t g = n_gap(nof_prb, gap2);
  if (!g) return 0;
  return gap2 ? (nof_prb / (2 * g)) * (2 * g) : 2 * std::min(g, nof_prb - g);
}

// 36.211 6.2.3.2 closed form: n~'_PRB from n~''_PRB (2 N_row (n~ mod 2) + n~/2) or n~'''_PRB
// (N_row (n~ mod 4) + n~/4) with the null-cell corrections, odd slot shifted by N~/2, gap applied
int vrb_to_prb(uint32_t nof_prb, bool gap2, uint32_t n_vrb, uint32_t slot) {
  const uint32_t gap = n_gap(nof_prb, gap2), Nt = gap2 ? 2 * gap : n_vrb_dist(nof_prb, false);
  if (!Nt || n_vrb >= n_vrb_dist(nof_prb, gap2)) return -1;
  const uint32_t P = rbg_size(nof_prb), Nrow = (Nt + 4 * P - 1) / (4 * P) * P, Nnull = 4 * Nrow - Nt;
  const uint32_t nt = n_vrb % Nt, base = Nt * (n_vrb / Nt);
  const uint32_t p2 = 2 * Nrow * (nt & 1u) + nt / 2 + base, p3 = Nrow * (nt & 3u) + nt / 4 + base;
  uint32_t pp;
  if (Nnull && nt >= Nt - Nnull) pp = (nt & 1u) ? p2 - Nrow : p2 - Nrow + Nnull / 2;
  else if (Nnull && (nt & 3u) >= 2) pp = p3 - Nnull / 2;
  else pp = p3;
  const uint32_t pt = slot ? (pp + Nt / 2) % Nt + base : pp;
  return (int)(pt < Nt / 2 ? pt : pt + gap - Nt / 2);
}

uint32_t dci1c_rba_bits(uint32_t nof_prb) {
  const uint32_t np = n_vrb_dist(nof_prb, false) / (nof_prb < 50 ? 2u : 4u);
  return ceil_log2(np * (np + 1) / 2);
}

int tbs_1c(uint32_t i_tbs) {
  static const int T[32] = {40,  56,  72,  120, 136, 144, 176, 208,  224,  256,  280,  296,  328,  336,  392,  488,
                            552, 600, 632, 696, 776, 840, 904, 1000, 1064, 1128, 1224, 1288, 1384, 1480, 1608, 1736};
  return i_tbs < 32 ? T[i_tbs] : -1;
}

void conv_rank_table(uint32_t D, std::vector<uint32_t>& rank) {
  const uint32_t R = (D + 31) / 32, KP = 32 * R, ND = KP - D;
  rank.assign(3 * D, 0);
  uint32_t cnt = 0;
  for (uint32_t i = 0; i < 3; i++)
    for (uint32_t col = 0; col < 32; col++)
      for (uint32_t r = 0; r < R; r++) {
        const uint32_t y = r * 32 + P_CONV[col];
        if (y >= ND) rank[i * D + (y - ND)] = cnt++;
      }
}

int search_space(uint32_t n_cce, uint32_t sf, uint16_t rnti, bool common, uint32_t* Ls, uint32_t* ncce) {
  static const uint32_t LU[4] = {1, 2, 4, 8}, MU[4] = {6, 6, 2, 2}, LC[2] = {4, 8}, MC[2] = {4, 2};
  uint32_t Y = 0;
  if (!common) {
    Y = rnti;
    for (uint32_t k = 0; k <= sf; k++) Y = (39827u * Y) % 65537u;
  }
  int n = 0;
  for (int li = 0; li < (common ? 2 : 4); li++) {
    const uint32_t L = common ? LC[li] : LU[li], M = common ? MC[li] : MU[li], nl = n_cce / L;
    if (!nl) continue;
    for (uint32_t m = 0; m < M; m++) {
      Ls[n] = L;
      ncce[n] = L * ((Y + m) % nl);
      n++;
    }
  }
  return n;
}

}  // namespace mi
