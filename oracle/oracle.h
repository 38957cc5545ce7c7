/*
 * oracle.h -- CPU restatement of the LTE DL PDSCH receive chain (TEST INFRASTRUCTURE ONLY).
 *
 * This directory is the parity oracle for the MI355X-native PHY in srsue_amd/.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as the checker
 * (or the CPU baseline that is timed beside the GPU).  The product path never links it.
 *
 * What it restates: the srsLTE-1.0 functions srsUE calls on its DL hot path
 * (reference: /root/reference/ue/src/phy/phch_worker.cc:74,254,337,347-348; dl_harq.cc:174,232).
 * srsLTE itself is NOT in the container, so the arithmetic below is
 * written from 3GPP TS 36.211/36.212/36.213 plus the srsLTE conventions recorded in SURVEY.md
 * section 8a ([X] tags: LLR>0 => bit 1, MMSE sigma^2 passed in (0.01 from phch_worker.cc:340),
 * triplet-interleaved turbo input, CRC early stop, N_cb = K_w, MSB-first payload).
 *
 * PARITY STATUS: "parity unpinned" against srsLTE's own arithmetic (no reference test or golden
 * vector exists for this path).  The oracle is pinned instead by 3GPP known-answer
 * tests (CRC, Gold, QPP permutations, TBS spot values, 36.212 tail layout) and by transmit-chain
 * ground truth: decoded TB bits must equal the transmitted ones whenever CRC passes.
 */
#ifndef LTE_ORACLE_H
#define LTE_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_NRB_MAX        110
#define OR_MAX_PORTS      2
#define OR_NSYMB          14           /* normal CP, symbols per subframe */
#define OR_TCOD_MAX_K     6144
#define OR_FILLER_LLR     (-10000.0f)  /* known-zero filler bit, systematic/parity1 (36.212 5.1.2) */

/* ---- cell / grant ---------------------------------------------------------------------- */
typedef struct {
  uint32_t id;        /* N_ID^cell 0..503 */
  uint32_t nof_prb;   /* 6,15,25,50,75,100 */
  uint32_t nof_ports; /* 1 or 2 */
} or_cell_t;

typedef struct {
  uint32_t C, Cp, Cm, Kp, Km, F, B;   /* 36.212 5.1.2 */
} or_cbsegm_t;

/* ---- tables & small helpers (o_common.c) ------------------------------------------------ */
int      or_symbol_sz(uint32_t nof_prb);                  /* FFT size N */
int      or_cp_len(uint32_t N, uint32_t l_in_slot);       /* 160/144 scaled by N/2048 */
void     or_gold(uint32_t c_init, uint8_t *c, uint32_t len);
uint32_t or_crc(const uint8_t *bits, uint32_t len, uint32_t poly, int order);
uint32_t or_crc24a(const uint8_t *bits, uint32_t len);
uint32_t or_crc24b(const uint8_t *bits, uint32_t len);
uint32_t or_crc16(const uint8_t *bits, uint32_t len);
int      or_cb_size_idx(uint32_t K);                      /* index in the 188-entry table or -1 */
uint32_t or_cb_size(uint32_t idx);
int      or_qpp(uint32_t K, uint32_t *pi);                /* pi[i] = (f1 i + f2 i^2) mod K */
int      or_qpp_f(uint32_t K, uint32_t *f1, uint32_t *f2);
int      or_cbsegm(uint32_t tbs, or_cbsegm_t *s);
int      or_tbs(uint32_t i_tbs, uint32_t nof_prb);        /* -1 if unknown */
int      or_mcs(uint32_t mcs, uint32_t *qm, uint32_t *i_tbs);
void     or_crs_seq(uint32_t id, uint32_t ns, uint32_t l, float *re_im /* 2*220 */);
int      or_ctrl_symbols(const or_cell_t *c, uint32_t cfi);
int      or_is_pdsch_re(const or_cell_t *c, uint32_t cfi, uint32_t sf, uint32_t l, uint32_t k);
/* RE list of the PDSCH in mapping order (36.211 6.3.5): index l*12*nof_prb + k; returns count.
 * prb_mask: if any entry is >= 2, bit s of entry p = PRB p is used in slot s (distributed VRB); else
 * a non-zero entry = PRB used in both slots. */
int      or_pdsch_re_list(const or_cell_t *c, uint32_t cfi, uint32_t sf, const uint8_t *prb_mask,
                          uint32_t *re_idx);
int      or_rm_E(uint32_t G, uint32_t C, uint32_t Qm, uint32_t NL, uint32_t r);

/* ---- FFT (o_fft.c), double precision, N = 2^a 3^b ------------------------------------- */
void     or_dft(const double *in /*2N*/, double *out /*2N*/, int N, int inverse);

/* ---- FEC (o_fec.c) ---------------------------------------------------------------------- */
/* Turbo encoder, 36.212 5.1.3.2.  in[K] bits (filler positions may hold 0), out = 3(K+4) bits
 * triplet-interleaved d0_k,d1_k,d2_k; filler d0/d1 positions marked 2 (NULL). */
int      or_tcod(const uint8_t *in, uint32_t K, uint32_t F, uint8_t *d);
/* Rate matching (TX), 36.212 5.1.4.1. d: 3(K+4) with 2=NULL. e: E bits */
int      or_rm_tx(const uint8_t *d, uint32_t K, uint32_t E, uint32_t rv, uint8_t *e);
/* Rate dematching + HARQ combine (RX): sb[N_cb] softbuffer row (w domain, combined by +=),
 * new_tb != 0 overwrites (== srsLTE reset_tbs to RX_NULL followed by first write).
 * out: decoder input 3(K+4) floats, triplet order; filler d0/d1 -> OR_FILLER_LLR. */
int      or_rm_rx(const float *e, uint32_t E, uint32_t K, uint32_t F, uint32_t rv, int new_tb,
                  float *sb, float *out);
uint32_t or_ncb(uint32_t K);
/* max-log-MAP turbo decoder (float), see o_fec.c header for the exact operation order */
typedef struct {
  uint32_t K;
  uint32_t pi[OR_TCOD_MAX_K], pinv[OR_TCOD_MAX_K];
  float w[OR_TCOD_MAX_K], llr1[OR_TCOD_MAX_K], llr2[OR_TCOD_MAX_K];
  float xs[OR_TCOD_MAX_K + 3], xp[OR_TCOD_MAX_K + 3];
  float beta[(OR_TCOD_MAX_K + 4) * 8];
} or_tdec_t;
int      or_tdec_reset(or_tdec_t *h, uint32_t K);
void     or_tdec_iteration(or_tdec_t *h, const float *in);
void     or_tdec_decision(const or_tdec_t *h, uint8_t *bits);
/* decode one codeblock: returns iterations used; *crc_ok set. crc_type 0 = 24B, 1 = 24A */
int      or_decode_cb(or_tdec_t *h, const float *in, uint32_t K, uint32_t max_its, int early_stop,
                      int crc_type, uint8_t *bits, int *crc_ok);
/* int16 ("SSE") max-log-MAP: exact-integer restatement of srsLTE's SSE decoder design, see the
 * o_fec.c section header for the quantisation and clamps.  Same call contract as the float one. */
#define OR_I16_SCALE 32.0f
#define OR_I16_CI    511
#define OR_I16_CX    1535
#define OR_I16_CW    1023
typedef struct {
  uint32_t K;
  uint32_t pi[OR_TCOD_MAX_K], pinv[OR_TCOD_MAX_K];
  int32_t  w[OR_TCOD_MAX_K], llr1[OR_TCOD_MAX_K], llr2[OR_TCOD_MAX_K];
  int32_t  xs[OR_TCOD_MAX_K + 3], xp[OR_TCOD_MAX_K + 3];
  int32_t  q[3 * OR_TCOD_MAX_K + 12];
  int32_t  beta[(OR_TCOD_MAX_K + 4) * 8];
} or_tdec16_t;
int32_t  or_q16(float x);
int      or_tdec16_reset(or_tdec16_t *h, uint32_t K);
void     or_tdec16_iteration(or_tdec16_t *h, const float *in);
void     or_tdec16_decision(const or_tdec16_t *h, uint8_t *bits);
int      or_decode_cb16(or_tdec16_t *h, const float *in, uint32_t K, uint32_t max_its, int early_stop,
                        int crc_type, uint8_t *bits, int *crc_ok);
/* decoder used by or_dlsch_decode / or_decode_subframe (test infrastructure switch) */
#define OR_TDEC_GEN 0
#define OR_TDEC_I16 1
#define OR_TDEC_SIMD 2   /* the SSE4.1 implementation of the int16 decoder (o_simd.c) */
#define OR_TDEC_AVX2 3   /* the AVX2 implementation, two code blocks per __m256i (o_avx2.c; or_avx2_available()) */
void     or_set_tdec_mode(int mode);
int      or_get_tdec_mode(void);
/* SSE4.1 int16 decoder (CPU baseline), bit-identical to or_decode_cb16.  state: or_simd_tdec_size()
 * bytes (any alignment).  Batch: n code blocks of equal K, input i at in + i*stride floats. */
/* AVX2 int16 decoder, two equal-K code blocks per call (lane 0 = A, lane 1 = B; inB NULL = A alone), each
 * bit-identical to or_decode_cb16 (o_avx2.c).  Requires or_avx2_available(). */
int      or_avx2_available(void);
size_t   or_avx2_tdec_size(void);
void     or_avx2_tdec_init(void *state);
int      or_avx2_decode_pair(void *state, const float *inA, const float *inB, uint32_t K, uint32_t max_its,
                             int early_stop, int crc_type, uint8_t *bitsA, uint8_t *bitsB, int *okA, int *okB,
                             int *itsA, int *itsB);
int      or_avx2_decode_batch(const float *in, uint32_t stride, uint32_t n, uint32_t K, uint32_t max_its,
                              int early_stop, int crc_type, uint8_t *bits, uint32_t *its, uint8_t *ok,
                              uint32_t nthreads);
size_t   or_simd_tdec_size(void);
void     or_simd_tdec_init(void *state);
int      or_simd_decode_cb(void *state, const float *in, uint32_t K, uint32_t max_its, int early_stop,
                           int crc_type, uint8_t *bits, int *crc_ok);
int      or_simd_decode_batch(const float *in, uint32_t stride, uint32_t n, uint32_t K, uint32_t max_its,
                              int early_stop, int crc_type, uint8_t *bits, uint32_t *its, uint8_t *ok,
                              uint32_t nthreads);

/* ---- DL control channels (o_ctrl.c): PHICH/PCFICH REG allocation, PDCCH, DCI ---- */
#define OR_DCI_MAX_BITS 64
enum { OR_DCI_0 = 0, OR_DCI_1 = 1, OR_DCI_1A = 2, OR_DCI_1C = 3 };
typedef struct {
  or_cell_t cell;
  uint32_t  ng;        /* PHICH resources Ng: 0 = 1/6, 1 = 1/2, 2 = 1, 3 = 2 (srslte_phich_resources_t) */
  uint32_t  cfi, sf;   /* PHICH duration normal, normal CP */
} or_ctrl_t;
typedef struct { uint32_t rb_start, L_crb, mcs, harq, ndi, rv, tpc; } or_dci1a_t;
typedef struct { uint32_t format, nbits, L, ncce; uint8_t bits[OR_DCI_MAX_BITS]; } or_dci_found_t;
uint32_t or_phich_ngroups(uint32_t nof_prb, uint32_t ng);
/* PDCCH REGs (not PCFICH/PHICH) in 36.211 6.8.5 mapping order, 4 RE indices (l*W + k) each;
 * returns N_REG, *n_cce = N_REG / 9.  re4 may be NULL (count only). */
int      or_pdcch_regs(const or_ctrl_t *q, uint32_t *re4, uint32_t *n_cce);
void     or_pdcch_quad_perm(uint32_t M, uint32_t cell_id, uint32_t *log_of_reg);
/* PDCCH soft bits [8 N_REG] in logical (CCE) order, descrambled; srslte_pdcch_extract_llr */
int      or_pdcch_llr(const or_ctrl_t *q, const float *grid, const float *ce, float noise, float *llr,
                      uint32_t *n_cce);
void     or_conv_encode_tb(const uint8_t *c, uint32_t D, uint8_t *d /* d0 | d1 | d2 */);
int      or_conv_rm_tx(const uint8_t *d, uint32_t D, uint32_t E, uint8_t *e);
void     or_conv_rm_rx(const float *e, uint32_t E, uint32_t D, float *d);
void     or_viterbi_tb(const float *d, uint32_t D, uint8_t *c);
uint32_t or_dci_size(uint32_t format, uint32_t nof_prb);
uint32_t or_riv(uint32_t nof_prb, uint32_t rb_start, uint32_t L);
int      or_dci1a_pack(uint32_t nof_prb, const or_dci1a_t *g, uint8_t *bits);
int      or_dci1a_unpack(uint32_t nof_prb, const uint8_t *bits, uint32_t nbits, or_dci1a_t *g);
int      or_dci_encode(const uint8_t *a, uint32_t A, uint16_t rnti, uint32_t L, uint8_t *e /* 72 L */);
int      or_dci_decode(const float *e, uint32_t L, uint32_t A, uint16_t rnti, uint8_t *a);   /* 1 = CRC ok */
int      or_search_space(uint32_t n_cce, uint32_t sf, uint16_t rnti, int common, uint32_t *L, uint32_t *ncce);
int      or_find_dci(const float *llr, uint32_t n_cce, uint32_t nof_prb, uint32_t sf, uint16_t rnti, int ul,
                     or_dci_found_t *out);
/* mode 0 = DL C-RNTI, 1 = UL (format 0), 2 = DL SI/RA/P-RNTI (common space, formats 1A then 1C) */
int      or_find_dci_mode(const float *llr, uint32_t n_cce, uint32_t nof_prb, uint32_t sf, uint16_t rnti, int mode,
                          or_dci_found_t *out);
/* ---- DL resource allocation / DCI -> grant (o_ra.c; srslte_dci_msg_to_dl_grant, phch_worker.cc:297) ---- */
typedef struct {
  uint8_t  prb[OR_NRB_MAX];   /* bit 0: PRB used in slot 0, bit 1: in slot 1 (or_pdsch_re_list encoding) */
  uint32_t format, alloc_type, distributed, gap2;
  uint32_t nof_prb;           /* PRBs (VRBs) per slot */
  uint32_t mcs, harq, ndi, rv, tpc, Qm, i_tbs, n_prb_tbs;
  int      tbs;               /* -1: TBS column not carried by the oracle (n_prb_tbs / i_tbs still valid) */
} or_dl_grant_t;
uint32_t or_rbg_size(uint32_t nof_prb);
uint32_t or_ngap(uint32_t nof_prb, int gap2);
uint32_t or_nvrb_dist(uint32_t nof_prb, int gap2);
int      or_vrb_to_prb(uint32_t nof_prb, int gap2, uint32_t n_vrb, uint32_t slot);
uint32_t or_dci1c_size(uint32_t nof_prb);
int      or_dl_dci_to_grant(const uint8_t *bits, uint32_t nbits, uint16_t rnti, uint32_t nof_prb, or_dl_grant_t *g);
/* PHICH (o_ctrl.c): resource of an UL grant, its 12 REs, soft HI (> 0 favours ACK), transmitter */
void     or_phich_calc(uint32_t nof_prb, uint32_t ng, uint32_t I_lowest, uint32_t n_dmrs, uint32_t *group,
                       uint32_t *seq);
uint32_t or_phich_cinit(uint32_t cell_id, uint32_t sf);
int      or_phich_res(const or_ctrl_t *q, uint32_t group, uint32_t *re12);
float    or_phich_soft(const or_ctrl_t *q, const float *grid, const float *ce, uint32_t group, uint32_t seq);
int      or_tx_phich(const or_ctrl_t *q, uint32_t group, uint32_t seq, int ack, const float *h_re_im, float *iq);
int      or_tx_pdcch(const or_ctrl_t *q, uint16_t rnti, uint32_t L, uint32_t ncce, const uint8_t *a, uint32_t A,
                     const float *h_re_im, float *iq);

/* ---- PHY TX (o_tx.c): synthetic subframe generator (ground truth) ----------------------- */
typedef struct {
  or_cell_t cell;
  uint32_t  sf_idx, cfi, mcs, rv, rnti, tm;  /* tm: 1 = single port, 2 = SFBC (nof_ports = 2) */
  uint32_t  tbs, qm;                          /* 0 => from the MCS / TBS tables */
  uint8_t   prb_mask[OR_NRB_MAX];
  float     snr_db;                           /* per-RE SNR; >= 200 => noiseless */
  float     h_re[OR_MAX_PORTS], h_im[OR_MAX_PORTS]; /* flat per-port channel */
  uint64_t  noise_seed;
  uint32_t  nl_td;                            /* N_L used in rate matching for TM2 (spec: 2) */
} or_tx_cfg_t;
/* Builds IQ for one subframe (samples: 2*SF_LEN floats).  tb: TBS/8 bytes (MSB-first).
 * Also returns the coded/scrambled bits count G and writes iq. Returns 0 ok. */
int      or_tx_subframe(const or_tx_cfg_t *cfg, const uint8_t *tb, float *iq, uint32_t *G_out);
int      or_sf_len(uint32_t nof_prb);

/* ---- PHY RX (o_rx.c) ------------------------------------------------------------------- */
/* OFDM RX: iq -> grid[14][12 nof_prb] complex (interleaved float) */
int      or_ofdm_rx(const or_cell_t *c, const float *iq, float *grid);
/* channel estimation: ce[p][14][12 nof_prb]; metrics[5] = {rsrp, rssi, rsrq, noise, snr} */
int      or_chest(const or_cell_t *c, uint32_t sf, const float *grid, float *ce, float *metrics);
/* PDSCH soft bits: equalise+demap+descramble; llr[G] */
int      or_pdsch_llr(const or_cell_t *c, uint32_t cfi, uint32_t sf, const uint8_t *prb_mask,
                      uint32_t Qm, uint32_t rnti, uint32_t tm, float noise, const float *grid,
                      const float *ce, float *llr, uint32_t *G_out, float *symbols_out);
/* PCFICH -> cfi (1..3), 0 on failure */
int      or_pcfich(const or_cell_t *c, uint32_t sf, const float *grid, const float *ce);
/* Full TB decode from LLRs: rm_rx per CB (+softbuffer) -> tdec -> TB CRC -> payload.
 * sb: C rows of or_ncb(K) floats (row stride sb_stride). Returns 0 if TB CRC ok. */
int      or_dlsch_decode(const float *llr, uint32_t G, uint32_t tbs, uint32_t Qm, uint32_t NL,
                         uint32_t rv, int new_tb, float *sb, uint32_t sb_stride, uint32_t max_its,
                         uint8_t *payload, uint32_t *noi_out, uint32_t *cb_crc_ok_out);
/* same, plus each code block's iteration count (cb_its_out[C], may be NULL) */
/* PUSCH hopping type 2 (36.211 5.3.4): each VRB's PRB in slot ns (prb[L]); returns the lowest or -1 */
int      or_pusch_hop_type2(uint32_t nof_prb, uint32_t n_ho, uint32_t n_sb, int intra, uint32_t cell_id,
                            uint32_t n_vrb, uint32_t L, uint32_t ns, uint32_t current_tx_nb, uint32_t *prb);
int      or_dlsch_decode_cbits(const float *llr, uint32_t G, uint32_t tbs, uint32_t Qm, uint32_t NL,
                               uint32_t rv, int new_tb, float *sb, uint32_t sb_stride, uint32_t max_its,
                               uint8_t *payload, uint32_t *noi_out, uint32_t *cb_crc_ok_out, uint32_t *cb_its_out);
/* End-to-end subframe decode (what srslte_ue_dl_decode_fft_estimate + srslte_pdsch_decode_rnti
 * do back to back).  Returns 0 if CRC ok. */
int      or_decode_subframe(const or_cell_t *c, uint32_t sf, uint32_t cfi, const uint8_t *prb_mask,
                            uint32_t tbs, uint32_t Qm, uint32_t rv, uint32_t rnti, uint32_t tm, uint32_t nl_td,
                            const float *iq, float *sb, uint32_t sb_stride, int new_tb,
                            uint32_t max_its, uint8_t *payload, uint32_t *noi_out);

/* ---- sync front end (o_sync.c) ------------------------------------------- */
typedef struct { uint32_t nid2, lag; float rho, cfo; } or_pss_res_t;
void     or_pss_seq(uint32_t nid2, float *d /* 62 complex */);
void     or_sss_m(uint32_t nid1, uint32_t *m0, uint32_t *m1);
void     or_sss_seq(uint32_t nid1, uint32_t nid2, uint32_t sf5, float *d /* 62 real */);
void     or_pss_time(uint32_t nid2, uint32_t nof_prb, float *x /* 2N: PSS symbol useful part */);
uint32_t or_sync_sym_off(uint32_t N, uint32_t l);
int      or_tx_sync(uint32_t cell_id, uint32_t nof_prb, uint32_t sf_idx, float amp, float *iq);
int      or_pss_find(const float *x, uint32_t nof_prb, uint32_t nid2_mask, uint32_t nlag, or_pss_res_t *r);
void     or_cfo_correct(const float *x, uint32_t n, float cfo, uint32_t N, float *y);
int      or_sss_detect(const float *sf_iq, uint32_t nof_prb, uint32_t nid2, uint32_t *nid1, uint32_t *sf5,
                       float *score);

/* ---- UL PUSCH transmit chain (o_ul.c) ------------------------------------- */
typedef struct {
  uint32_t cell_id, nof_prb, sf_idx, rnti;
  uint32_t n_prb, L_prb, tbs, Qm, rv;                 /* allocation (no hopping), TB, modulation, rv */
  uint32_t group_hopping, sequence_hopping, delta_ss;  /* DMRS cell configuration */
  uint32_t cyclic_shift, n_dmrs2;                      /* RRC cyclicShift, DCI 0 cyclic-shift field (0..7) */
  uint32_t ack_len, ack, I_offset_ack;                 /* HARQ-ACK on PUSCH: 0..2 bits (bit 0 = o0), beta index */
  uint32_t hop, n_prb1;                                /* hop = 1: slot 1 starts at PRB n_prb1 (36.213 8.4) */
  uint32_t cqi_len, I_offset_cqi;                      /* CQI on PUSCH (36.212 5.2.2.6.4): 0..64 bits, beta index */
  uint8_t  cqi[64];                                    /* o_0 .. o_{O-1}, one bit per byte */
  uint32_t ri_len, ri, I_offset_ri;                    /* RI on PUSCH (5.2.2.6): 0..2 bits (bit 0 = o0), beta index */
} or_ul_cfg_t;
double   or_pam_level(const uint8_t *b, uint32_t Qm);
uint32_t or_pusch_G(const or_ul_cfg_t *c);                /* all coded bits: 12 M Qm (normal CP, no SRS) */
/* UL-SCH data + CQI: the multiplexed sequence g (36.212 5.2.2.7) = Q_CQI CQI bits then the G data bits
 * (G = 12 M Qm - Q_CQI - Q_RI); returns its length H = Q_CQI + G, -1 on error */
int      or_ulsch_encode(const or_ul_cfg_t *c, const uint8_t *tb, uint8_t *g);
/* channel interleaver (5.2.2.8) with RI / HARQ-ACK insertion, scrambling, modulation: g -> 12 M symbols */
int      or_pusch_mod(const or_ul_cfg_t *c, const uint8_t *g, float *x /* 12 M complex, symbol-major */);
void     or_dft_m(const float *in, uint32_t M, float *out, int inverse);
int      or_dmrs_params(const or_ul_cfg_t *c, uint32_t ns, uint32_t *u, uint32_t *v, uint32_t *ncs);
int      or_dmrs_pusch(const or_ul_cfg_t *c, uint32_t ns, float *r);
int      or_pusch_grid(const or_ul_cfg_t *c, const uint8_t *tb, float *grid /* 14 x 12 N_RB complex */);
int      or_scfdma_tx(uint32_t nof_prb, const float *grid, float *iq);
int      or_pusch_encode(const or_ul_cfg_t *c, const uint8_t *tb, float *iq);
/* HARQ-ACK on PUSCH (36.212 5.2.2.6): number of coded modulation symbols Q'_ACK, and the encoded
 * block (codes 0 / 1 = bit, 2 = placeholder x, 3 = placeholder y), returns its length in bits */
uint32_t or_ack_qprime(const or_ul_cfg_t *c);
uint32_t or_ack_block(const or_ul_cfg_t *c, uint8_t *blk /* <= 18 */);
/* RI / CQI on PUSCH (36.212 5.2.2.6, beta_offset 36.213 Tables 8.6.3-2 / -3): Q'_RI, Q'_CQI (symbols; 0 if
 * absent, (uint32_t)-1 for an invalid configuration), the RI block (as or_ack_block) and the Q_CQI CQI coded
 * bits (O <= 11: the (32, O) block code of Table 5.2.2.6.4-1 repeated; O > 11: CRC8, tail-biting
 * convolutional code, rate matching 5.1.4.2) */
uint32_t or_ri_qprime(const or_ul_cfg_t *c);
uint32_t or_cqi_qprime(const or_ul_cfg_t *c);
uint32_t or_ri_block(const or_ul_cfg_t *c, uint8_t *blk /* <= 18 */);
int      or_cqi_encode(const or_ul_cfg_t *c, uint8_t *q);
uint32_t or_cqi_rm32(const uint8_t *o, uint32_t O);    /* the 32 RM code bits b_0..b_31, b_0 = MSB of the result */

#ifdef __cplusplus
}
#endif
#endif
