/*
 * srslte/srslte.h -- srsLTE-1.0-compatible DOWNLINK subset, backed by MI355X (gfx950) kernels.
 *
 * srsUE (/root/reference) compiles against "srslte/srslte.h" (e.g. ue/hdr/phy/phch_worker.h:31)
 * and requires srsLTE >= 1.0.0 (ue/hdr/srslte_version_check.h:30-41, checked at ue/src/ue.cc:39-49).
 * This header declares the types and entry points srsUE's PHY worker calls on its DL data path
 * (SURVEY.md 8b).  Each function cites the call site it replaces.  Field names that srsUE
 * reads directly (ue_dl.sf_symbols, ue_dl.ce, ue_dl.pdsch, ue_dl.pdsch.dl_sch, ue_dl.pdsch_cfg.grant,
 * ue_dl.chest, ue_dl.pdcch, ue_dl.last_n_cce, ue_dl.last_location) are kept.
 *
 * Beyond the DL data path the header also carries the SURVEY.md 8f rows built on the GPU: DL control
 * (PDCCH/DCI, PHICH), the sync tracking subset and the UL PUSCH encoder.  Cell search / MIB, PUCCH,
 * SRS, PRACH, power control and the radio still come from srsLTE itself.
 *
 * Conventions: 0 = SRSLTE_SUCCESS, -1 = SRSLTE_ERROR; srslte_pdsch_decode_rnti returns 0 iff
 * the TB CRC passes; payload bits are packed MSB first.
 */
#ifndef SRSLTE_MI355X_H
#define SRSLTE_MI355X_H
#include <stdbool.h>
#include <stdint.h>
#include <stddef.h>
#include <time.h>
#include <math.h>
#include <stdio.h>

#include "srslte/common/timestamp.h"
#include "srslte/utils/debug.h"
#include "srslte/utils/bit.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SRSLTE_API __attribute__((visibility("default")))

#define SRSLTE_VERSION_MAJOR 1
#define SRSLTE_VERSION_MINOR 0
#define SRSLTE_VERSION_PATCH 0
#define SRSLTE_VERSION_STRING "1.0.0-mi355x"
#define SRSLTE_VERSION_ENCODE(major, minor, patch) (((major) * 10000) + ((minor) * 100) + (patch))
#define SRSLTE_VERSION SRSLTE_VERSION_ENCODE(SRSLTE_VERSION_MAJOR, SRSLTE_VERSION_MINOR, SRSLTE_VERSION_PATCH)
#define SRSLTE_VERSION_CHECK(major, minor, patch) (SRSLTE_VERSION >= SRSLTE_VERSION_ENCODE(major, minor, patch))

#define SRSLTE_SUCCESS 0
#define SRSLTE_ERROR -1
#define SRSLTE_ERROR_INVALID_INPUTS -2

#define SRSLTE_MAX_PORTS 4
#define SRSLTE_MAX_LAYERS 4
#define SRSLTE_MAX_PRB 110
#define SRSLTE_NRE 12
#define SRSLTE_CP_NORM_NSYMB 7
#define SRSLTE_NSUBFRAMES_X_FRAME 10
#define SRSLTE_PDSCH_MAX_TDEC_ITERS 4   /* ue.conf.example:83 documents the default 4 */

typedef _Complex float cf_t;

typedef enum { SRSLTE_CP_NORM = 0, SRSLTE_CP_EXT } srslte_cp_t;
typedef enum { SRSLTE_PHICH_NORM = 0, SRSLTE_PHICH_EXT } srslte_phich_length_t;
typedef enum { SRSLTE_PHICH_R_1_6 = 0, SRSLTE_PHICH_R_1_2, SRSLTE_PHICH_R_1, SRSLTE_PHICH_R_2 } srslte_phich_resources_t;
typedef enum { SRSLTE_MOD_BPSK = 0, SRSLTE_MOD_QPSK, SRSLTE_MOD_16QAM, SRSLTE_MOD_64QAM, SRSLTE_MOD_LAST } srslte_mod_t;
typedef enum { SRSLTE_RNTI_USER = 0, SRSLTE_RNTI_SI, SRSLTE_RNTI_RAR, SRSLTE_RNTI_TEMP, SRSLTE_RNTI_SPS,
               SRSLTE_RNTI_PCH, SRSLTE_RNTI_NOF_TYPES } srslte_rnti_type_t;
typedef enum { SRSLTE_MIMO_TYPE_SINGLE_ANTENNA = 0, SRSLTE_MIMO_TYPE_TX_DIVERSITY,
               SRSLTE_MIMO_TYPE_SPATIAL_MULTIPLEX } srslte_mimo_type_t;

/* srslte_cell_t, held by value by srsUE (phch_worker.h:101) */
typedef struct SRSLTE_API {
  uint32_t nof_prb;
  uint32_t nof_ports;
  uint32_t bw_idx;
  uint32_t id;
  srslte_cp_t cp;
  srslte_phich_length_t phich_length;
  srslte_phich_resources_t phich_resources;
} srslte_cell_t;

typedef struct SRSLTE_API {
  srslte_mod_t mod;
  int tbs;
  uint32_t idx;
} srslte_ra_mcs_t;

/* DL grant (srslte_dci_msg_to_dl_grant output, phch_worker.cc:297; read at :355-364) */
typedef struct SRSLTE_API {
  bool prb_idx[2][SRSLTE_MAX_PRB];
  uint32_t nof_prb;
  uint32_t Qm;
  srslte_ra_mcs_t mcs;
} srslte_ra_dl_grant_t;

typedef struct SRSLTE_API {
  uint32_t nof_re;
  uint32_t nof_symb;
  uint32_t nof_bits;
  uint32_t lstart;
} srslte_ra_nbits_t;

typedef struct SRSLTE_API {
  uint32_t F, C, K1, K2, C1, C2, tbs;
} srslte_cbsegm_t;

typedef struct SRSLTE_API {
  srslte_cbsegm_t cb_segm;
  srslte_ra_dl_grant_t grant;
  srslte_ra_nbits_t nbits;
  uint32_t rv;
  uint32_t sf_idx;
  srslte_mimo_type_t mimo_type;
  uint32_t nof_layers;
} srslte_pdsch_cfg_t;

/* HARQ softbuffer: embedded by value in srsUE's dl_harq_process (dl_harq.h:88); the soft bits
 * live in HBM (group-interleaved layout, see srsue_amd/csrc/rm_body.h), dev is opaque. */
typedef struct SRSLTE_API {
  uint32_t max_cb;
  float **buffer_f;       /* kept for layout compatibility; NULL (soft bits are device resident) */
  void *dev;              /* device arena: 2 groups x [N_cb][64] floats (K- and K+ code blocks) */
  uint64_t dev_bytes;
  uint32_t reset_pending; /* reset / reset_tbs since the last decode: the decode clears the arena first, on its own
                             stream (a reset has no stream of its own to order it with the decoding instance's) */
} srslte_softbuffer_rx_t;

typedef struct SRSLTE_API {
  uint32_t max_iterations;
  uint32_t nof_iterations;          /* srslte_pdsch_last_noi (phch_worker.cc:360,848) */
  float average_nof_iterations;
} srslte_sch_t;

struct mi_ue_dl_ctx;

typedef struct SRSLTE_API {
  srslte_cell_t cell;
  srslte_sch_t dl_sch;              /* srslte_sch_set_max_noi(&ue_dl.pdsch.dl_sch, n) (phch_worker.cc:88) */
  uint16_t rnti;
  bool rnti_is_set;
  struct mi_ue_dl_ctx *ctx;
} srslte_pdsch_t;

typedef struct SRSLTE_API {
  srslte_cell_t cell;
  float rsrp, rssi, rsrq, noise_estimate, snr;
} srslte_chest_dl_t;

typedef struct SRSLTE_API {
  uint32_t L;
  uint32_t ncce;
} srslte_dci_location_t;

/* PDCCH (srslte_pdcch_extract_llr, phch_worker.cc:260): soft bits and blind search on the GPU
 * (srsue_amd/csrc/ctrl.hip); ctx = the owning srslte_ue_dl_t's device context */
typedef struct SRSLTE_API {
  srslte_cell_t cell;
  uint32_t nof_cce;
  struct mi_ue_dl_ctx *ctx;
} srslte_pdcch_t;

#define SRSLTE_DCI_MAX_BITS 64
typedef enum { SRSLTE_DCI_FORMAT0 = 0, SRSLTE_DCI_FORMAT1, SRSLTE_DCI_FORMAT1A, SRSLTE_DCI_FORMAT1C,
               SRSLTE_DCI_FORMAT_ERROR } srslte_dci_format_t;
typedef enum { SRSLTE_RA_ALLOC_TYPE0 = 0, SRSLTE_RA_ALLOC_TYPE1, SRSLTE_RA_ALLOC_TYPE2 } srslte_ra_type_t;
/* DCI message (srslte_ue_dl_find_dl_dci_type output, phch_worker.cc:293; srsUE reads nof_bits, data) */
typedef struct SRSLTE_API {
  uint8_t data[SRSLTE_DCI_MAX_BITS];
  uint32_t nof_bits;
  srslte_dci_format_t format;
} srslte_dci_msg_t;
/* unpacked DL DCI (srslte_dci_msg_to_dl_grant, phch_worker.cc:297; srsUE reads ndi, harq_process,
 * rv_idx at :304-308) */
typedef struct SRSLTE_API {
  srslte_ra_type_t alloc_type;
  uint32_t type2_start, type2_len;   /* RIV-decoded localized allocation (format 1A) */
  uint32_t type0_alloc;              /* RBG bitmap (format 1), RBG 0 = MSB of the field */
  uint32_t mcs_idx;
  uint32_t harq_process;
  bool ndi;
  uint32_t rv_idx;
  uint32_t tpc_pucch;
  srslte_dci_format_t dci_format;
  /* appended (srsUE does not read them): type-1 subset / shift / VRB bitmap (format 1, 36.213 7.1.6.2),
   * type-2 distributed VRB flag and gap (formats 1A / 1C, 36.211 6.2.3.2: 0 = N_gap,1, 1 = N_gap,2) */
  uint32_t type1_subset, type1_shift, type1_bitmap;
  bool type2_distributed;
  uint32_t type2_gap;
} srslte_ra_dl_dci_t;

/* srslte_ue_dl_t, owned by value per phch_worker (phch_worker.h:111) */
typedef struct SRSLTE_API {
  srslte_pdcch_t pdcch;
  srslte_pdsch_t pdsch;
  srslte_chest_dl_t chest;
  srslte_pdsch_cfg_t pdsch_cfg;
  srslte_cell_t cell;
  cf_t *sf_symbols;                 /* host mirror of the OFDM grid (read by srslte_pdcch_extract_llr, :260) */
  cf_t *ce[SRSLTE_MAX_PORTS];       /* host mirror of the channel estimates */
  uint32_t cfi;
  uint16_t current_rnti;
  uint32_t last_n_cce;
  srslte_dci_location_t last_location;
  uint64_t pkt_errors, pkts_total;
  struct mi_ue_dl_ctx *ctx;         /* MI355X device context: HIP stream + HBM workspace */
} srslte_ue_dl_t;

/* ---- version (ue.cc:39-49) ----------------------------------------------------------------- */
SRSLTE_API int srslte_get_version_major(void);
SRSLTE_API int srslte_get_version_minor(void);
SRSLTE_API int srslte_get_version_patch(void);
SRSLTE_API char *srslte_get_version(void);
SRSLTE_API int srslte_check_version(int major, int minor, int patch);

/* ---- UE DL (phch_worker.cc:74,104,127,254,337) ------------------------------------------------ */
SRSLTE_API int srslte_ue_dl_init(srslte_ue_dl_t *q, srslte_cell_t cell);
SRSLTE_API void srslte_ue_dl_free(srslte_ue_dl_t *q);
SRSLTE_API void srslte_ue_dl_set_rnti(srslte_ue_dl_t *q, uint16_t rnti);
SRSLTE_API int srslte_ue_dl_decode_fft_estimate(srslte_ue_dl_t *q, cf_t *input, uint32_t sf_idx, uint32_t *cfi);
SRSLTE_API int srslte_ue_dl_cfg_grant(srslte_ue_dl_t *q, srslte_ra_dl_grant_t *grant, uint32_t cfi, uint32_t sf_idx,
                                      uint32_t rvidx);

/* ---- PDCCH / DCI (phch_worker.cc:260, 293, 297, 314, 426) --------------------------------------
 * Blind search order (srsLTE's dci_blind_search, one format over all candidates at a time): C-RNTI:
 * UE-specific space L = 1, 2, 4, 8 with format 1A then format 1, then the common space L = 4, 8 with
 * format 1A; SI/RA/P-RNTI: the common space only, format 1A then format 1C.  find_* return 1 when found.
 * dci_msg_to_dl_grant (36.212 5.3.3.1, 36.213 7.1.6 / 7.1.7, 36.211 6.2.3.2): format 1 with resource
 * allocation type 0 (RBG bitmap) or type 1 (RBG subset, shift, VRB bitmap); format 1A localized or
 * distributed VRB (N_gap,1 / N_gap,2; with SI/RA/P-RNTI the NDI bit is the gap and the TPC LSB selects
 * N_PRB^1A = 2 / 3 with QPSK and I_TBS = I_MCS); format 1C (distributed, N_step, Table 7.1.7.2.3-1).
 * Distributed allocations set different PRBs in grant->prb_idx[0] (slot 0) and prb_idx[1] (slot 1);
 * the PDSCH RE gather honours both. */
SRSLTE_API int srslte_pdcch_extract_llr(srslte_pdcch_t *q, cf_t *sf_symbols, cf_t *ce[SRSLTE_MAX_PORTS],
                                        float noise_estimate, uint32_t nsubframe, uint32_t cfi);
SRSLTE_API int srslte_ue_dl_find_dl_dci(srslte_ue_dl_t *q, srslte_dci_msg_t *dci_msg, uint32_t cfi, uint32_t sf_idx,
                                        uint16_t rnti);
SRSLTE_API int srslte_ue_dl_find_dl_dci_type(srslte_ue_dl_t *q, srslte_dci_msg_t *dci_msg, uint32_t cfi,
                                             uint32_t sf_idx, uint16_t rnti, srslte_rnti_type_t rnti_type);
SRSLTE_API int srslte_ue_dl_find_ul_dci(srslte_ue_dl_t *q, srslte_dci_msg_t *dci_msg, uint32_t cfi, uint32_t sf_idx,
                                        uint16_t rnti);
SRSLTE_API uint32_t srslte_ue_dl_get_ncce(srslte_ue_dl_t *q);
/* PHICH (phch_worker.cc:381): HARQ indicator of the UL grant with lowest PRB index n_prb_lowest and
 * DMRS cyclic shift n_dmrs (36.213 9.1.2, FDD) in the subframe decode_fft_estimate processed; true =
 * ACK (maximum-likelihood decision on the despread soft value, GPU phich_kernel). */
SRSLTE_API bool srslte_ue_dl_decode_phich(srslte_ue_dl_t *q, uint32_t sf_idx, uint32_t n_prb_lowest, uint32_t n_dmrs);
SRSLTE_API int srslte_dci_msg_to_dl_grant(srslte_dci_msg_t *msg, uint16_t msg_rnti, uint32_t nof_prb,
                                          srslte_ra_dl_dci_t *dl_dci, srslte_ra_dl_grant_t *grant);
SRSLTE_API char *srslte_ra_dl_dci_string(srslte_ra_dl_dci_t *dci);

/* ---- PDSCH (phch_worker.cc:347-348, :360, :848; :88) ------------------------------------------ */
SRSLTE_API int srslte_pdsch_decode_rnti(srslte_pdsch_t *q, srslte_pdsch_cfg_t *cfg, srslte_softbuffer_rx_t *softbuffer,
                                        cf_t *sf_symbols, cf_t *ce[SRSLTE_MAX_PORTS], float noise_estimate,
                                        uint16_t rnti, uint8_t *data);
SRSLTE_API uint32_t srslte_pdsch_last_noi(srslte_pdsch_t *q);
SRSLTE_API void srslte_sch_set_max_noi(srslte_sch_t *q, uint32_t max_iterations);

/* ---- softbuffer (dl_harq.cc:169,174,232; ue_itf_test_sib1.cc:121,136) -------------------------- */
SRSLTE_API int srslte_softbuffer_rx_init(srslte_softbuffer_rx_t *q, uint32_t nof_prb);
SRSLTE_API void srslte_softbuffer_rx_free(srslte_softbuffer_rx_t *q);
SRSLTE_API void srslte_softbuffer_rx_reset(srslte_softbuffer_rx_t *q);
SRSLTE_API void srslte_softbuffer_rx_reset_tbs(srslte_softbuffer_rx_t *q, uint32_t tbs);

/* ---- channel-estimation metrics (phch_worker.cc:359,512,519,799,821-823,842,847) --------------- */
SRSLTE_API float srslte_chest_dl_get_snr(srslte_chest_dl_t *q);
SRSLTE_API float srslte_chest_dl_get_rssi(srslte_chest_dl_t *q);
SRSLTE_API float srslte_chest_dl_get_rsrp(srslte_chest_dl_t *q);
SRSLTE_API float srslte_chest_dl_get_rsrq(srslte_chest_dl_t *q);
SRSLTE_API float srslte_chest_dl_get_noise_estimate(srslte_chest_dl_t *q);

/* ---- resource allocation helpers (phy.cc:118) ------------------------------------------------ */
SRSLTE_API int srslte_ra_tbs_from_idx(uint32_t tbs_idx, uint32_t n_prb);
SRSLTE_API int srslte_ra_tbs_idx_from_mcs(uint32_t mcs);
SRSLTE_API srslte_mod_t srslte_ra_mod_from_mcs(uint32_t mcs);
SRSLTE_API uint32_t srslte_mod_bits_x_symbol(srslte_mod_t mod);
SRSLTE_API int srslte_cbsegm(srslte_cbsegm_t *s, uint32_t tbs);

/* ---- misc (phch_worker.cc:69) ----------------------------------------------------------------- */
#define SRSLTE_SF_LEN_PRB(nof_prb) (15 * srslte_symbol_sz(nof_prb))
SRSLTE_API int srslte_symbol_sz(uint32_t nof_prb);
SRSLTE_API void *srslte_vec_malloc(uint32_t size);   /* 256-B aligned, free()-compatible (phch_worker.cc:102) */
SRSLTE_API void srslte_vec_free(void *ptr);

/* ---- UL PUSCH (phch_worker.cc:79-84, 105, 128, 213, 545-590, 748) -------------
 * srslte_ue_ul on the GPU (srsue_amd/csrc/ul.hip, ue_ul.cpp): cfg_grant plans the transmission,
 * pusch_encode_rnti_softbuffer copies the payload to HBM, runs TB CRC -> turbo encoder -> rate matching
 * -> channel interleaver -> scrambling -> modulation -> transform precoding + DMRS -> SC-FDMA and copies
 * the subframe (SRSLTE_SF_LEN_PRB samples) to output_signal.  The UCI in uci_data is multiplexed into the
 * PUSCH (36.212 5.2.2.6-5.2.2.8, beta_offsets from set_cfg's uci_cfg): HARQ-ACK (1 or 2 bits), periodic
 * CQI (uci_cqi / uci_cqi_len, up to 64 bits: the (32, O) block code up to 11 bits, CRC8 + tail-biting
 * convolutional code above) and RI (uci_ri / uci_ri_len, 1 or 2 bits).  Limits: PUSCH hopping type 1 only (36.213 8.4.1: DCI format 0 hopping
 * bits through srslte_dci_msg_to_ul_grant's n_rb_ho, intra- or inter-subframe mode from set_cfg's hopping
 * configuration; type 2 returns SRSLTE_ERROR), L_prb >= 3; PUCCH, SRS and UL
 * power control stay in srsLTE.  set_cfg uses the DMRS and hopping configurations, the others are
 * accepted.  set_normalization(true) scales by nof_prb / (15 sqrt(L_prb)) (srsLTE's factor as recorded
 * in DESIGN.md, unverified: srsLTE is not in the container); set_cfo(cfo) shifts the output by cfo
 * subcarrier spacings when set_cfo_enable(true). */
#define SRSLTE_CQI_MAX_BITS 64
typedef struct SRSLTE_API {
  uint32_t n_prb[2];                /* first PRB of slots 0 / 1 (read at phch_worker.cc:580) */
  uint32_t n_prb_tilde[2];          /* (read at :223) */
  uint32_t L_prb;
  uint32_t freq_hopping;
  uint32_t nof_re, nof_symb;
  srslte_ra_mcs_t mcs;
  uint32_t Qm;
  uint32_t ncs_dmrs;                /* DCI format 0 cyclic-shift field (read at :223) */
} srslte_ra_ul_grant_t;
typedef struct SRSLTE_API {
  srslte_ra_type_t alloc_type;
  uint32_t type2_start, type2_len;  /* RIV-decoded allocation */
  uint32_t mcs_idx, rv_idx, n_dmrs, freq_hop_fl, tpc_pusch;
  bool ndi, cqi_request;
} srslte_ra_ul_dci_t;
typedef struct SRSLTE_API {           /* random-access response grant, 36.213 6.2 (phch_worker.cc:412) */
  bool hopping_flag;
  uint32_t rba;
  uint32_t trunc_mcs;
  uint32_t tpc_pusch;
  bool ul_delay;
  bool cqi_request;
} srslte_dci_rar_grant_t;
typedef struct SRSLTE_API {           /* phch_worker.cc:681-685 */
  bool group_hopping_en;
  bool sequence_hopping_en;
  uint32_t cyclic_shift;
  uint32_t delta_ss;
} srslte_refsignal_dmrs_pusch_cfg_t;
typedef struct SRSLTE_API {           /* phch_worker.cc:688-693 */
  enum { SRSLTE_PUSCH_HOP_MODE_INTER_SF = 1, SRSLTE_PUSCH_HOP_MODE_INTRA_SF = 0 } hop_mode;
  uint32_t hopping_offset;
  uint32_t n_sb;
} srslte_pusch_hopping_cfg_t;
typedef struct SRSLTE_API {           /* accepted by set_cfg, used by srsLTE's SRS (out of scope) */
  bool configured;
  uint32_t subframe_config, bw_cfg, I_srs, B, b_hop, n_rrc, k_tc, n_srs;
} srslte_refsignal_srs_cfg_t;
typedef struct SRSLTE_API {           /* accepted by set_cfg (PUCCH: out of scope) */
  uint32_t delta_pucch_shift, N_cs, n_rb_2;
  bool srs_configured;
  uint32_t srs_cs_subf_cfg;
  bool srs_simul_ack;
} srslte_pucch_cfg_t;
typedef struct SRSLTE_API {
  uint32_t n_pucch_1[4];
  uint32_t N_pucch_1, n_pucch_2, n_pucch_sr;
} srslte_pucch_sched_t;
typedef struct SRSLTE_API { uint32_t I_offset_cqi, I_offset_ri, I_offset_ack; } srslte_uci_cfg_t;
typedef struct SRSLTE_API {           /* accepted by set_cfg (UL power control: out of scope) */
  float p0_nominal_pusch, alpha, p0_nominal_pucch, delta_f_pucch[5], delta_preamble_msg3, p0_ue_pusch;
  bool delta_mcs_based, acc_enabled;
  float p0_ue_pucch, p_srs_offset;
} srslte_ue_ul_powerctrl_t;
typedef struct SRSLTE_API {           /* phch_worker.h:118, filled at :481-523 */
  uint8_t uci_cqi[SRSLTE_CQI_MAX_BITS];
  uint32_t uci_cqi_len;
  uint8_t uci_ri;
  uint32_t uci_ri_len;
  uint8_t uci_ack;
  uint32_t uci_ack_len;
  bool ri_periodic_report;
  bool scheduling_request;
} srslte_uci_data_t;
/* HARQ tx softbuffer: embedded by value in srsUE's ul_harq_process (ul_harq.h:97) */
typedef struct SRSLTE_API {
  uint32_t max_cb;
  uint8_t **buffer_b;     /* kept for layout compatibility; NULL */
  void *dev;              /* device copy of the last new-data TB (a retransmission re-encodes it) */
  uint32_t tbs;           /* bits of that TB, 0 = none */
} srslte_softbuffer_tx_t;
typedef struct SRSLTE_API {
  srslte_cbsegm_t cb_segm;
  srslte_ra_ul_grant_t grant;
  uint32_t rv;
  uint32_t sf_idx;
  uint32_t tti;
  uint32_t current_tx_nb;
} srslte_pusch_cfg_t;
struct mi_ue_ul_ctx;
typedef struct SRSLTE_API {         /* PUCCH state srsUE reads (phch_worker.cc:628); PUCCH itself is out of scope */
  bool shortened;
} srslte_pucch_t;
typedef struct SRSLTE_API {         /* owned by value per phch_worker (phch_worker.h:116) */
  srslte_cell_t cell;
  srslte_pusch_cfg_t pusch_cfg;     /* ue_ul.pusch_cfg.grant.n_prb_tilde (phch_worker.cc:223) */
  srslte_refsignal_dmrs_pusch_cfg_t dmrs_cfg;
  srslte_pusch_hopping_cfg_t hopping_cfg;
  srslte_uci_cfg_t uci_cfg;         /* beta_offset indices of UCI on PUSCH (set_cfg) */
  uint16_t current_rnti;
  bool normalize_en;
  bool cfo_en;
  float current_cfo;
  uint32_t last_pucch_format;
  srslte_pucch_t pucch;
  struct mi_ue_ul_ctx *ctx;         /* MI355X device context: HIP stream + HBM workspace */
} srslte_ue_ul_t;

SRSLTE_API int srslte_ue_ul_init(srslte_ue_ul_t *q, srslte_cell_t cell);
SRSLTE_API void srslte_ue_ul_free(srslte_ue_ul_t *q);
SRSLTE_API void srslte_ue_ul_set_rnti(srslte_ue_ul_t *q, uint16_t rnti);
SRSLTE_API void srslte_ue_ul_set_normalization(srslte_ue_ul_t *q, bool enabled);
SRSLTE_API void srslte_ue_ul_set_cfo_enable(srslte_ue_ul_t *q, bool enabled);
SRSLTE_API void srslte_ue_ul_set_cfo(srslte_ue_ul_t *q, float cur_cfo);
SRSLTE_API void srslte_ue_ul_set_cfg(srslte_ue_ul_t *q, srslte_refsignal_dmrs_pusch_cfg_t *dmrs_cfg,
                                     srslte_refsignal_srs_cfg_t *srs_cfg, srslte_pucch_cfg_t *pucch_cfg,
                                     srslte_pucch_sched_t *pucch_sched, srslte_uci_cfg_t *uci_cfg,
                                     srslte_pusch_hopping_cfg_t *hopping_cfg, srslte_ue_ul_powerctrl_t *power_ctrl);
SRSLTE_API int srslte_ue_ul_cfg_grant(srslte_ue_ul_t *q, srslte_ra_ul_grant_t *grant, uint32_t tti, uint32_t rvidx,
                                      uint32_t current_tx_nb);
SRSLTE_API int srslte_ue_ul_pusch_encode_rnti_softbuffer(srslte_ue_ul_t *q, uint8_t *data, srslte_uci_data_t uci_data,
                                                         srslte_softbuffer_tx_t *softbuffer, uint16_t rnti,
                                                         cf_t *output_signal);
SRSLTE_API int srslte_softbuffer_tx_init(srslte_softbuffer_tx_t *q, uint32_t nof_prb);
SRSLTE_API void srslte_softbuffer_tx_reset(srslte_softbuffer_tx_t *q);
SRSLTE_API void srslte_softbuffer_tx_free(srslte_softbuffer_tx_t *q);
/* DCI format 0 (36.212 5.3.3.1.1) / RAR grant (36.213 6.2) -> UL grant: MCS per 36.213 Table 8.6.1-1
 * (29-31: retransmission, rv 1-3, TBS of the last grant not known here: error); TBS from the full
 * 36.213 Table 7.1.7.2.1-1. */
SRSLTE_API int srslte_dci_msg_to_ul_grant(srslte_dci_msg_t *msg, uint32_t nof_prb, uint32_t n_rb_ho,
                                          srslte_ra_ul_dci_t *ul_dci, srslte_ra_ul_grant_t *grant, uint32_t harq_pid);
SRSLTE_API int srslte_dci_rar_to_ul_grant(srslte_dci_rar_grant_t *rar, uint32_t nof_prb, uint32_t n_rb_ho,
                                          srslte_ra_ul_dci_t *ul_dci, srslte_ra_ul_grant_t *grant);

/* ---- sync front end (phch_recv.cc:108-120, 231-240, 321-335) ----------------
 * srslte_ue_sync in tracking mode on the GPU (srsue_amd/csrc/sync.hip, ue_sync.cpp): the first
 * zerocopy() calls search a half frame for the cell's PSS (its N_ID_2 = cell.id % 3), check the SSS
 * (N_ID_1, subframe 0 or 5) and align the stream to a subframe boundary (return 0); afterwards every
 * call reads one subframe through the receive callback, re-times and re-estimates the CFO on the PSS
 * of subframes 0 and 5 (an exponential average, srslte_sync_set_em_alpha), corrects the CFO on the GPU
 * into input_buffer and returns 1.  get_cfo / set_cfo: Hz; get_sfo: mean timing drift in samples/s.
 * Cell search (srslte_ue_cellsearch_*), MIB decoding (srslte_ue_mib_*) and AGC stay in srsLTE;
 * start_agc() returns an error, set_agc_period() is accepted. */
typedef struct SRSLTE_API { float threshold; float em_alpha; } srslte_sync_t;
typedef struct SRSLTE_API { float gain; } srslte_agc_t;
typedef struct mi_ue_sync_ctx mi_ue_sync_ctx;
typedef struct SRSLTE_API {
  srslte_cell_t cell;
  srslte_sync_t strack;
  srslte_agc_t agc;
  cf_t *input_buffer;       /* the last delivered subframe (get_buffer) */
  mi_ue_sync_ctx *ctx;
} srslte_ue_sync_t;
SRSLTE_API int srslte_ue_sync_init(srslte_ue_sync_t *q, srslte_cell_t cell,
                                   int(recv_callback)(void *, void *, uint32_t, srslte_timestamp_t *),
                                   void *stream_handler);
SRSLTE_API void srslte_ue_sync_free(srslte_ue_sync_t *q);
SRSLTE_API int srslte_ue_sync_zerocopy(srslte_ue_sync_t *q, cf_t *input_buffer);
SRSLTE_API int srslte_ue_sync_get_buffer(srslte_ue_sync_t *q, cf_t **sf_symbols);
SRSLTE_API uint32_t srslte_ue_sync_get_sfidx(srslte_ue_sync_t *q);
SRSLTE_API float srslte_ue_sync_get_cfo(srslte_ue_sync_t *q);
SRSLTE_API float srslte_ue_sync_get_sfo(srslte_ue_sync_t *q);
SRSLTE_API void srslte_ue_sync_set_cfo(srslte_ue_sync_t *q, float cfo);
SRSLTE_API void srslte_ue_sync_decode_sss_on_track(srslte_ue_sync_t *q, bool enabled);
SRSLTE_API void srslte_ue_sync_get_last_timestamp(srslte_ue_sync_t *q, srslte_timestamp_t *timestamp);
SRSLTE_API void srslte_ue_sync_set_agc_period(srslte_ue_sync_t *q, uint32_t period);
SRSLTE_API int srslte_ue_sync_start_agc(srslte_ue_sync_t *q, double(set_gain_callback)(void *, double),
                                        float init_gain_value);
SRSLTE_API void srslte_sync_set_threshold(srslte_sync_t *q, float threshold);
SRSLTE_API void srslte_sync_set_em_alpha(srslte_sync_t *q, float alpha);
SRSLTE_API int srslte_sampling_freq_hz(uint32_t nof_prb);

/* ---- MAC <-> PHY grant container (reference ue/hdr/common/mac_interface.h:59,73,83) -------------- */
typedef union SRSLTE_API {
  srslte_ra_ul_grant_t ul;
  srslte_ra_dl_grant_t dl;
} srslte_phy_grant_t;
#define SRSLTE_RAR_GRANT_LEN 20   /* 36.213 6.2: RAR UL grant bits (phy_interface.h:174) */

/* ---- periodic CQI reporting (phch_worker.h:128, phch_worker.cc:495-523): 36.213 7.2.2 reporting
 * instances (Table 7.2.2-1A), wideband / UE-selected subband CQI values packed for PUCCH format 2 or
 * PUSCH (36.212 5.2.3.3 / 5.2.2.6.4: 4-bit wideband CQI, 4-bit subband CQI + L-bit label) -------------- */
typedef struct SRSLTE_API {
  bool configured;
  uint32_t pmi_idx;
  bool simul_cqi_ack;
  bool format_is_subband;
  uint32_t subband_size;
} srslte_cqi_periodic_cfg_t;
typedef struct SRSLTE_API { uint8_t wideband_cqi; } srslte_cqi_format2_wideband_t;
typedef struct SRSLTE_API { uint8_t subband_cqi; uint8_t subband_label; } srslte_cqi_format2_subband_t;
typedef enum { SRSLTE_CQI_TYPE_WIDEBAND = 0, SRSLTE_CQI_TYPE_SUBBAND } srslte_cqi_type_t;
typedef struct SRSLTE_API {
  union {
    srslte_cqi_format2_wideband_t wideband;
    srslte_cqi_format2_subband_t subband;
  };
  srslte_cqi_type_t type;
} srslte_cqi_value_t;
SRSLTE_API int srslte_cqi_value_pack(srslte_cqi_value_t *value, uint8_t buff[SRSLTE_CQI_MAX_BITS]);
SRSLTE_API bool srslte_cqi_send(uint32_t I_cqi_pmi, uint32_t tti);
SRSLTE_API uint8_t srslte_cqi_from_snr(float snr);

/* ---- small helpers srsUE calls (phch_worker.cc:449,495,531-532,654; dl_harq.cc:195) ---------------- */
#define SRSLTE_VEC_EMA(data, average, coeff) ((coeff) * (data) + (1 - (coeff)) * (average))
SRSLTE_API uint32_t srslte_vec_max_fi(float *x, uint32_t len);
SRSLTE_API void srslte_vec_fprint_hex(FILE *stream, uint8_t *x, uint32_t len);
SRSLTE_API int srslte_tti_interval(uint32_t tti1, uint32_t tti2);
SRSLTE_API bool srslte_ue_ul_sr_send_tti(uint32_t I_sr, uint32_t current_tti);
SRSLTE_API int srslte_refsignal_srs_send_cs(uint32_t subframe_config, uint32_t sf_idx);
SRSLTE_API int srslte_refsignal_srs_send_ue(uint32_t I_srs, uint32_t tti);
SRSLTE_API void srslte_ra_pusch_fprint(FILE *f, srslte_ra_ul_dci_t *q, uint32_t nof_prb);

/* ---- OUT OF SCOPE (SURVEY.md 8 / DESIGN.md 9): PUCCH, SRS, UL power control and PRACH are not on the
 * DL decode path.  They are declared so srsUE compiles against this header unchanged; this library does
 * not implement them: an integration links srsLTE's own modules rebuilt against this header, or stubs
 * (INTEGRATION.md). -------- */
SRSLTE_API void srslte_ue_ul_pregen_signals(srslte_ue_ul_t *q);
SRSLTE_API int srslte_ue_ul_pucch_encode(srslte_ue_ul_t *q, srslte_uci_data_t uci_data, uint32_t pdcch_n_cce,
                                         uint32_t tti, cf_t *output_signal);
SRSLTE_API int srslte_ue_ul_srs_encode(srslte_ue_ul_t *q, uint32_t tti, cf_t *output_signal);
SRSLTE_API float srslte_ue_ul_pusch_power(srslte_ue_ul_t *q, float PL, float p0_preamble);
SRSLTE_API float srslte_ue_ul_pucch_power(srslte_ue_ul_t *q, float PL, uint32_t format, uint32_t n_cqi,
                                          uint32_t n_harq);
SRSLTE_API float srslte_ue_ul_srs_power(srslte_ue_ul_t *q, float PL);
typedef struct SRSLTE_API { uint32_t N_seq, N_cp; void *impl; } srslte_prach_t;   /* prach.h:64 (srsLTE) */
typedef struct SRSLTE_API { uint32_t nsamples; void *impl; } srslte_cfo_t;         /* prach.h:68 (srsLTE) */
/* PRACH preamble generation and its CFO pre-correction (reference ue/src/phy/prach.cc:56-57,77-98,130,152) */
SRSLTE_API int srslte_prach_init(srslte_prach_t *p, uint32_t N_ifft_ul, uint32_t preamble_format,
                                 uint32_t root_seq_index, bool high_speed_flag, uint32_t zero_corr_zone_config);
SRSLTE_API int srslte_prach_free(srslte_prach_t *p);
SRSLTE_API uint32_t srslte_prach_get_preamble_format(uint32_t config_idx);
SRSLTE_API int srslte_prach_gen(srslte_prach_t *p, uint32_t seq_index, uint32_t freq_offset, cf_t *signal);
SRSLTE_API bool srslte_prach_send_tti(uint32_t config_idx, uint32_t current_tti, int allowed_subframe);
SRSLTE_API int srslte_cfo_init(srslte_cfo_t *h, uint32_t nsamples);
SRSLTE_API void srslte_cfo_free(srslte_cfo_t *h);
SRSLTE_API void srslte_cfo_correct(srslte_cfo_t *h, cf_t *input, cf_t *output, float freq);

/* Cell search and MIB decoding (reference ue/src/phy/phch_recv.cc:98,137-220,246-253; types held by value
 * at ue/hdr/phy/phch_recv.h:77 and by the cell-search locals).  The types carry the members srsUE touches
 * (cs.ue_sync.agc, ue_mib_sync.ue_sync.agc, ue_mib.pbch). */
#define SRSLTE_BCH_PAYLOAD_LEN 24            /* MIB bits, 36.331 MasterInformationBlock */
#define SRSLTE_UE_MIB_FOUND 1
#define SRSLTE_UE_MIB_NOTFOUND 0
typedef struct SRSLTE_API { uint32_t frame_idx; void *impl; } srslte_pbch_t;
typedef struct SRSLTE_API { srslte_cell_t cell; srslte_pbch_t pbch; void *impl; } srslte_ue_mib_t;
typedef struct SRSLTE_API { srslte_ue_mib_t ue_mib; srslte_ue_sync_t ue_sync; void *impl; } srslte_ue_mib_sync_t;
typedef struct SRSLTE_API {
  uint32_t cell_id;
  srslte_cp_t cp;
  float peak;
  float mode;
  float psr;
  float cfo;
} srslte_ue_cellsearch_result_t;
typedef struct SRSLTE_API {
  srslte_ue_sync_t ue_sync;
  uint32_t max_frames;
  uint32_t nof_valid_frames;
  void *impl;
} srslte_ue_cellsearch_t;
SRSLTE_API int srslte_ue_mib_init(srslte_ue_mib_t *q, srslte_cell_t cell);
SRSLTE_API void srslte_ue_mib_free(srslte_ue_mib_t *q);
SRSLTE_API int srslte_ue_mib_decode(srslte_ue_mib_t *q, cf_t *input, uint8_t bch_payload[SRSLTE_BCH_PAYLOAD_LEN],
                                    uint32_t *nof_tx_ports, uint32_t *sfn_offset);
SRSLTE_API void srslte_pbch_decode_reset(srslte_pbch_t *q);
SRSLTE_API int srslte_ue_mib_sync_init(srslte_ue_mib_sync_t *q, uint32_t cell_id, srslte_cp_t cp,
                                       int(recv_callback)(void *, void *, uint32_t, srslte_timestamp_t *),
                                       void *stream_handler);
SRSLTE_API void srslte_ue_mib_sync_free(srslte_ue_mib_sync_t *q);
SRSLTE_API int srslte_ue_mib_sync_decode(srslte_ue_mib_sync_t *q, uint32_t max_frames_timeout,
                                         uint8_t bch_payload[SRSLTE_BCH_PAYLOAD_LEN], uint32_t *nof_tx_ports,
                                         uint32_t *sfn_offset);
SRSLTE_API int srslte_ue_cellsearch_init(srslte_ue_cellsearch_t *q,
                                         int(recv_callback)(void *, void *, uint32_t, srslte_timestamp_t *),
                                         void *stream_handler);
SRSLTE_API void srslte_ue_cellsearch_free(srslte_ue_cellsearch_t *q);
SRSLTE_API void srslte_ue_cellsearch_set_nof_frames_to_scan(srslte_ue_cellsearch_t *q, uint32_t nof_frames);
SRSLTE_API void srslte_ue_cellsearch_set_threshold(srslte_ue_cellsearch_t *q, float threshold);
SRSLTE_API int srslte_ue_cellsearch_scan_N_id_2(srslte_ue_cellsearch_t *q, uint32_t N_id_2,
                                                srslte_ue_cellsearch_result_t *found_cell);
SRSLTE_API int srslte_ue_cellsearch_scan(srslte_ue_cellsearch_t *q, srslte_ue_cellsearch_result_t found_cells[3],
                                         uint32_t *max_N_id_2);

/* ---- host utilities srsUE calls outside the worker, implemented here (srslte_util.cpp) ---------------
 * AGC gain (phch_recv.cc:174,211), MIB unpacking (36.331: dl-Bandwidth 3 bits, phich-Config 1 + 2 bits,
 * systemFrameNumber 8 MSBs; phch_recv.cc:216,253), cell / CP printing (:192,218), timing advance (36.213
 * 4.2.3: N_TA = 16 T_A from a RAR, N_TA += 16 (T_A - 31) from a MAC CE; phy.cc:125-132), the RAR grant's
 * 20 bits (36.213 6.2; phch_common.cc:122), PRACH power / scaling helpers (prach.cc:157-168) */
#define SRSLTE_LTE_TS (1.0f / (15000.0f * 2048.0f))   /* basic time unit T_s, 36.211 4 */
#define SRSLTE_PC_MAX 23                              /* dBm, power class 3 */
#define SRSLTE_MIN(a, b) ((a) < (b) ? (a) : (b))
#define SRSLTE_MAX(a, b) ((a) > (b) ? (a) : (b))
#define SRSLTE_SIRNTI 0xFFFF
#define SRSLTE_PRNTI 0xFFFE
SRSLTE_API float srslte_agc_get_gain(srslte_agc_t *q);
SRSLTE_API void srslte_pbch_mib_unpack(uint8_t *msg, srslte_cell_t *cell, uint32_t *sfn);
SRSLTE_API void srslte_pbch_mib_pack(srslte_cell_t *cell, uint32_t sfn, uint8_t *msg);
SRSLTE_API char *srslte_cp_string(srslte_cp_t cp);
SRSLTE_API void srslte_cell_fprint(FILE *stream, srslte_cell_t *cell, uint32_t sfn);
SRSLTE_API uint32_t srslte_N_ta_new_rar(uint32_t ta);
SRSLTE_API uint32_t srslte_N_ta_new(uint32_t N_ta_old, uint32_t ta);
SRSLTE_API void srslte_dci_rar_grant_unpack(srslte_dci_rar_grant_t *rar, uint8_t grant[SRSLTE_RAR_GRANT_LEN]);
SRSLTE_API float srslte_vec_avg_power_cf(cf_t *x, uint32_t len);
SRSLTE_API void srslte_vec_sc_prod_cfc(cf_t *x, float h, cf_t *z, uint32_t len);

#ifdef __cplusplus
}
#endif
#endif
