// srslte_util.cpp -- the small srsLTE 1.0 host helpers srsUE's PHY worker and MAC call around the DL path
// (reference ue/src/phy/phch_worker.cc:314-315,449,470,495,507-523,531-532,654; ue/src/mac/dl_harq.cc:195).
// Reporting instants follow 36.213 (CQI Table 7.2.2-1A, SR Table 10.1.5-1, UE SRS Table 8.2-1) and
// 36.211 Table 5.5.3.3-1 (cell SRS subframes, FDD); the CQI packing follows 36.212 5.2.3.3.
#include <string.h>

#include "srslte/srslte.h"

extern "C" {

int srslte_verbose = SRSLTE_VERBOSE_NONE;

void get_time_interval(struct timeval* tdata) {
  tdata[0].tv_sec = tdata[2].tv_sec - tdata[1].tv_sec;
  tdata[0].tv_usec = tdata[2].tv_usec - tdata[1].tv_usec;
  if (tdata[0].tv_usec < 0) {
    tdata[0].tv_sec--;
    tdata[0].tv_usec += 1000000;
  }
}

int srslte_tti_interval(uint32_t tti1, uint32_t tti2) {
  return tti1 >= tti2 ? (int)(tti1 - tti2) : (int)(10240 - tti2 + tti1);
}

static bool periodic(uint32_t tti, uint32_t period, uint32_t offset) {
  return ((tti + 10240 - offset % 10240) % 10240) % period == 0;
}

// 36.213 Table 7.2.2-1A (FDD): N_pd and N_OFFSET,CQI of I_CQI/PMI; reported where
// (10 n_f + floor(n_s / 2) - N_offset) mod N_pd = 0
bool srslte_cqi_send(uint32_t I, uint32_t tti) {
  static const uint32_t lim[] = {1, 6, 16, 36, 76, 156, 316}, per[] = {2, 5, 10, 20, 40, 80, 160};
  static const uint32_t base[] = {0, 2, 7, 17, 37, 77, 157};
  for (int i = 0; i < 7; i++)
    if (I <= lim[i]) return periodic(tti, per[i], I - base[i]);
  if (I >= 318 && I <= 349) return periodic(tti, 32, I - 318);
  if (I >= 350 && I <= 413) return periodic(tti, 64, I - 350);
  if (I >= 414 && I <= 541) return periodic(tti, 128, I - 414);
  return false;   // 317, 542..1023: reserved
}

// 36.213 Table 10.1.5-1: SR periodicity / subframe offset of I_SR
bool srslte_ue_ul_sr_send_tti(uint32_t I, uint32_t tti) {
  if (I < 5) return periodic(tti, 5, I);
  if (I < 15) return periodic(tti, 10, I - 5);
  if (I < 35) return periodic(tti, 20, I - 15);
  if (I < 75) return periodic(tti, 40, I - 35);
  if (I < 155) return periodic(tti, 80, I - 75);
  if (I < 157) return periodic(tti, 2, I - 155);
  if (I == 157) return true;
  return false;
}

// 36.211 Table 5.5.3.3-1 (FDD): cell-specific SRS subframes; 1 = SRS subframe, 0 = not, -1 = reserved
int srslte_refsignal_srs_send_cs(uint32_t cfg, uint32_t sf_idx) {
  static const uint32_t T[15] = {1, 2, 2, 5, 5, 5, 5, 5, 5, 10, 10, 10, 10, 10, 10};
  static const uint16_t D[15] = {0x1, 0x1, 0x2, 0x1, 0x2, 0x4, 0x8, 0x3, 0xc, 0x1, 0x2, 0x4, 0x8,
                                 0x15f /* 0,1,2,3,4,6,8 */, 0x17f /* 0..6,8 */};
  if (cfg > 14 || sf_idx > 9) return -1;
  return (D[cfg] >> (sf_idx % T[cfg])) & 1u;
}

// 36.213 Table 8.2-1 (FDD): UE-specific SRS periodicity T_SRS and offset of I_SRS
int srslte_refsignal_srs_send_ue(uint32_t I, uint32_t tti) {
  static const uint32_t lim[] = {1, 6, 16, 36, 76, 156, 316, 636}, per[] = {2, 5, 10, 20, 40, 80, 160, 320};
  static const uint32_t base[] = {0, 2, 7, 17, 37, 77, 157, 317};
  for (int i = 0; i < 8; i++)
    if (I <= lim[i]) return periodic(tti, per[i], I - base[i]) ? 1 : 0;
  return -1;
}

// wideband CQI from the reference-signal SNR (dB): the SNR thresholds of CQI 1..15 srsLTE 1.0 used for
// its periodic reports (SURVEY.md [X]: recollection, srsLTE is not in the container)
uint8_t srslte_cqi_from_snr(float snr) {
  static const float thr[15] = {1.95f, 4.0f, 6.0f, 8.0f, 10.0f, 11.95f, 14.05f, 16.0f,
                                17.9f, 19.9f, 21.5f, 23.45f, 25.0f, 27.3f, 29.0f};
  for (int c = 14; c >= 0; c--)
    if (snr >= thr[c]) return (uint8_t)(c + 1);
  return 0;
}

// 36.212 5.2.3.3.1: wideband CQI = 4 bits; UE-selected subband CQI = 4 bits + the subband label (L = 1
// bit here, srsLTE 1.0's packing [X]); bits MSB first, one per byte; returns the bit count
int srslte_cqi_value_pack(srslte_cqi_value_t* v, uint8_t buff[SRSLTE_CQI_MAX_BITS]) {
  if (!v || !buff) return SRSLTE_ERROR;
  const uint32_t cqi = v->type == SRSLTE_CQI_TYPE_WIDEBAND ? v->wideband.wideband_cqi : v->subband.subband_cqi;
  for (int i = 0; i < 4; i++) buff[i] = (uint8_t)((cqi >> (3 - i)) & 1u);
  if (v->type == SRSLTE_CQI_TYPE_WIDEBAND) return 4;
  buff[4] = (uint8_t)(v->subband.subband_label & 1u);
  return 5;
}

uint32_t srslte_vec_max_fi(float* x, uint32_t len) {
  uint32_t k = 0;
  for (uint32_t i = 1; i < len; i++)
    if (x[i] > x[k]) k = i;
  return k;
}

void srslte_vec_fprint_hex(FILE* f, uint8_t* x, uint32_t len) {
  fprintf(f, "[");
  for (uint32_t i = 0; i + 8 <= len; i += 8) {
    uint32_t b = 0;
    for (uint32_t j = 0; j < 8; j++) b = (b << 1) | (x[i + j] & 1u);
    fprintf(f, "%02x ", b);
  }
  fprintf(f, "];\n");
}

void srslte_ra_pusch_fprint(FILE* f, srslte_ra_ul_dci_t* q, uint32_t nof_prb) {
  if (!f || !q) return;
  fprintf(f, " - Resource Allocation Type 2 (nof_prb=%u): start %u, len %u, hop %u\n", nof_prb, q->type2_start,
          q->type2_len, q->freq_hop_fl);
  fprintf(f, " - MCS %u, RV %u, NDI %d, TPC %u, n_dmrs %u, CQI request %d\n", q->mcs_idx, q->rv_idx, (int)q->ndi,
          q->tpc_pusch, q->n_dmrs, (int)q->cqi_request);
}

}  // extern "C"

/* ---- bit utilities (srslte/utils/bit.h): one bit per byte, MSB first -------------------------------- */
extern "C" {

uint32_t srslte_bit_pack(uint8_t** bits, int nof_bits) {
  uint32_t v = 0;
  for (int i = 0; i < nof_bits; i++) v = (v << 1) | ((*bits)[i] & 1u);
  *bits += nof_bits;
  return v;
}

void srslte_bit_unpack(uint32_t value, uint8_t** bits, int nof_bits) {
  for (int i = 0; i < nof_bits; i++) (*bits)[i] = (uint8_t)((value >> (nof_bits - 1 - i)) & 1u);
  *bits += nof_bits;
}

// a trailing partial byte is left-aligned (its low bits zero)
void srslte_bit_pack_vector(uint8_t* unpacked, uint8_t* packed, int nof_bits) {
  for (int i = 0; i < nof_bits / 8; i++) packed[i] = (uint8_t)srslte_bit_pack(&unpacked, 8);
  if (nof_bits % 8) packed[nof_bits / 8] = (uint8_t)(srslte_bit_pack(&unpacked, nof_bits % 8) << (8 - nof_bits % 8));
}

void srslte_bit_unpack_vector(uint8_t* packed, uint8_t* unpacked, int nof_bits) {
  for (int i = 0; i < nof_bits / 8; i++) srslte_bit_unpack(packed[i], &unpacked, 8);
  if (nof_bits % 8) srslte_bit_unpack((uint32_t)packed[nof_bits / 8] >> (8 - nof_bits % 8), &unpacked, nof_bits % 8);
}

/* ---- helpers around the PHY outside the worker (srslte/srslte.h "host utilities") --------------------- */
float srslte_agc_get_gain(srslte_agc_t* q) { return q ? q->gain : 1.0f; }

// 36.331 MasterInformationBlock: dl-Bandwidth (3), phich-Duration (1), phich-Resource (2), the 8 MSBs of
// the SFN (the 2 LSBs come from the PBCH's 40 ms phase: sfn_offset, phch_recv.cc:255), 10 spare bits
void srslte_pbch_mib_unpack(uint8_t* msg, srslte_cell_t* cell, uint32_t* sfn) {
  static const uint32_t bw_prb[6] = {6, 15, 25, 50, 75, 100};
  const uint32_t bw = srslte_bit_pack(&msg, 3);
  if (cell) {
    cell->bw_idx = bw;
    cell->nof_prb = bw < 6 ? bw_prb[bw] : 0;
    cell->phich_length = srslte_bit_pack(&msg, 1) ? SRSLTE_PHICH_EXT : SRSLTE_PHICH_NORM;
    cell->phich_resources = (srslte_phich_resources_t)srslte_bit_pack(&msg, 2);
  } else {
    msg += 3;
  }
  const uint32_t s = srslte_bit_pack(&msg, 8);
  if (sfn) *sfn = s << 2;
}

void srslte_pbch_mib_pack(srslte_cell_t* cell, uint32_t sfn, uint8_t* msg) {
  static const uint32_t bw_prb[6] = {6, 15, 25, 50, 75, 100};
  uint32_t bw = 0;
  for (uint32_t i = 0; i < 6; i++)
    if (bw_prb[i] == cell->nof_prb) bw = i;
  memset(msg, 0, SRSLTE_BCH_PAYLOAD_LEN);
  srslte_bit_unpack(bw, &msg, 3);
  srslte_bit_unpack(cell->phich_length == SRSLTE_PHICH_EXT ? 1u : 0u, &msg, 1);
  srslte_bit_unpack((uint32_t)cell->phich_resources, &msg, 2);
  srslte_bit_unpack((sfn >> 2) & 0xFFu, &msg, 8);
}

char* srslte_cp_string(srslte_cp_t cp) {
  return const_cast<char*>(cp == SRSLTE_CP_NORM ? "Normal  " : "Extended");
}

void srslte_cell_fprint(FILE* stream, srslte_cell_t* cell, uint32_t sfn) {
  static const char* res[4] = {"1/6", "1/2", "1", "2"};
  fprintf(stream, " - Cell ID:         %u\n", cell->id);
  fprintf(stream, " - Nof ports:       %u\n", cell->nof_ports);
  fprintf(stream, " - CP:              %s\n", srslte_cp_string(cell->cp));
  fprintf(stream, " - PRB:             %u\n", cell->nof_prb);
  fprintf(stream, " - PHICH Length:    %s\n", cell->phich_length == SRSLTE_PHICH_EXT ? "Extended" : "Normal");
  fprintf(stream, " - PHICH Resources: %s\n", res[(uint32_t)cell->phich_resources & 3u]);
  fprintf(stream, " - SFN:             %u\n", sfn);
}

// 36.213 4.2.3: a RAR's 11-bit T_A sets N_TA = 16 T_A; a MAC CE's 6-bit T_A adjusts N_TA by 16 (T_A - 31)
uint32_t srslte_N_ta_new_rar(uint32_t ta) { return ta * 16; }
uint32_t srslte_N_ta_new(uint32_t N_ta_old, uint32_t ta) {
  const int n = (int)N_ta_old + ((int)ta - 31) * 16;
  return n < 0 ? 0u : (uint32_t)n;
}

// 36.213 6.2: hopping flag (1), fixed-size RB assignment (10), truncated MCS (4), TPC for PUSCH (3),
// UL delay (1), CSI request (1)
void srslte_dci_rar_grant_unpack(srslte_dci_rar_grant_t* rar, uint8_t grant[SRSLTE_RAR_GRANT_LEN]) {
  uint8_t* g = grant;
  rar->hopping_flag = srslte_bit_pack(&g, 1) != 0;
  rar->rba = srslte_bit_pack(&g, 10);
  rar->trunc_mcs = srslte_bit_pack(&g, 4);
  rar->tpc_pusch = srslte_bit_pack(&g, 3);
  rar->ul_delay = srslte_bit_pack(&g, 1) != 0;
  rar->cqi_request = srslte_bit_pack(&g, 1) != 0;
}

float srslte_vec_avg_power_cf(cf_t* x, uint32_t len) {
  if (!len) return 0.0f;
  const float* f = reinterpret_cast<const float*>(x);
  double acc = 0.0;
  for (uint32_t i = 0; i < 2 * len; i++) acc += (double)f[i] * f[i];
  return (float)(acc / len);
}

void srslte_vec_sc_prod_cfc(cf_t* x, float h, cf_t* z, uint32_t len) {
  const float* a = reinterpret_cast<const float*>(x);
  float* b = reinterpret_cast<float*>(z);
  for (uint32_t i = 0; i < 2 * len; i++) b[i] = a[i] * h;
}

}  // extern "C"
