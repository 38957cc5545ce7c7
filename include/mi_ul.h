/*
 * mi_ul.h -- batched C ABI of the MI355X UL PUSCH transmit path.
 *
 * The per-TTI srsLTE entry points srsUE calls (srslte_ue_ul_cfg_grant + srslte_ue_ul_pusch_encode_
 * rnti_softbuffer, /root/reference/ue/src/phy/phch_worker.cc:551-560) are in srslte/srslte.h; this is
 * the throughput form: N PUSCH transmissions planned once, encoded per call on the caller's stream
 * from device-resident TB payloads into device-resident SC-FDMA IQ.
 *
 * Chain (gfx950 kernels, srsue_amd/csrc/ul.hip): TB CRC24A -> segmentation + CRC24B -> turbo encoder
 * (36.212 5.1.3.2, chunk-parallel recursive encoders) -> rate matching (5.1.4.1, full circular buffer)
 * -> channel interleaver (5.2.2.8, no UCI) -> scrambling (36.211 5.3.1) -> modulation (7.1) ->
 * transform precoding (5.3.3, mixed-radix DFT of M = 12 L_prb) -> mapping (5.3.4, per-slot PRBs) +
 * DMRS (5.5.2.1; L_prb 1, 2: the tabulated base sequences of 5.5.1.2) -> SC-FDMA (5.6: N-point transform, half-subcarrier shift, CP).
 * Uplink control information is multiplexed as 36.212 5.2.2.6-5.2.2.8 prescribe: CQI (O <= 11 bits: the
 * (32, O) block code; O > 11: CRC8 + tail-biting convolutional code) ahead of the data in the multiplexed
 * sequence, RI (1 or 2 bits) in the interleaver columns next to the HARQ-ACK ones (rate matching of the
 * data around both), HARQ-ACK (1 or 2 bits) puncturing the data next to the DMRS.
 * Normalisation: unit average power per used subcarrier (1/sqrt(M) DFT, 1/sqrt(N) IDFT).
 */
#ifndef MI_UL_H
#define MI_UL_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint32_t cell_id, nof_prb, sf_idx, rnti;
  uint32_t n_prb, L_prb, tbs, Qm, rv;                 /* allocation (no hopping), TB bits, 2/4/6, rv 0..3 */
  uint32_t group_hopping, sequence_hopping, delta_ss;  /* DMRS cell configuration (srslte_refsignal_dmrs_pusch_cfg_t) */
  uint32_t cyclic_shift, n_dmrs2;                      /* RRC cyclicShift, DCI format 0 cyclic-shift field (0..7) */
  uint32_t ack_len, ack, I_offset_ack;                 /* HARQ-ACK on PUSCH (36.212 5.2.2.6): 0, 1 or 2 bits
                                                          (bit 0 = first), beta_offset index (36.213 8.6.3-1) */
  uint32_t hop, n_prb1;                                /* hop = 1: slot 1 starts at PRB n_prb1 (frequency hopping,
                                                          36.213 8.4 -- the per-TTI API computes it from the DCI) */
  uint32_t cqi_len, I_offset_cqi;                      /* CQI on PUSCH (36.212 5.2.2.6.4): 0..64 bits, beta_offset
                                                          index 2..15 (36.213 Table 8.6.3-3) */
  uint8_t  cqi[64];                                    /* CQI bits o_0 .. o_{O-1}, one per byte (srslte_uci_data_t) */
  uint32_t ri_len, ri, I_offset_ri;                    /* RI on PUSCH: 0..2 bits (bit 0 = o0), index 0..12 (8.6.3-2) */
} mi_ul_cfg_t;

enum { MI_UL_STAGE_CRC = 0, MI_UL_STAGE_ENCODE, MI_UL_STAGE_MOD, MI_UL_NSTAGES };
#define MI_UL_FLAG_PROFILE 1u

typedef struct mi_ul_batch mi_ul_batch_t;

mi_ul_batch_t *mi_ul_batch_create(const mi_ul_cfg_t *cfgs, uint32_t n, uint32_t flags);
void   mi_ul_batch_destroy(mi_ul_batch_t *b);
/* payload layout: TB i (tbs/8 bytes, MSB first) at byte offset mi_ul_batch_payload_offset(b, i) */
size_t mi_ul_batch_payload_offset(const mi_ul_batch_t *b, uint32_t i);
size_t mi_ul_batch_payload_bytes(const mi_ul_batch_t *b);
/* output layout: subframe i (15 N cf32 samples) at cf32 offset mi_ul_batch_iq_offset(b, i) */
size_t mi_ul_batch_iq_offset(const mi_ul_batch_t *b, uint32_t i);
size_t mi_ul_batch_iq_samples(const mi_ul_batch_t *b);
uint32_t mi_ul_batch_n_codeblocks(const mi_ul_batch_t *b);
/* enqueue the chain on `stream` (hipStream_t, NULL = default): d_payload -> d_iq (both device) */
int    mi_ul_batch_run(mi_ul_batch_t *b, const void *d_payload, void *d_iq, void *stream);
/* parity hooks: the coded symbols of transmission i after the last run in channel-interleaver input order
 * (36.212 5.2.2.7 g: Q'_CQI CQI symbols, then the rate-matched data), Qm bits per byte, first bit = MSB;
 * 12 M bytes are written, of which the last Q'_RI (the RI cells) are zero */
int    mi_ul_batch_symbols(mi_ul_batch_t *b, uint32_t i, uint8_t *host);
int    mi_ul_batch_stage_ms(mi_ul_batch_t *b, float *ms /* MI_UL_NSTAGES */, uint32_t *nruns);
void   mi_ul_batch_profile_reset(mi_ul_batch_t *b);
/* algorithmic HBM bytes per run: payload read + IQ write (SURVEY.md 8d convention) */
double mi_ul_batch_algo_bytes(const mi_ul_batch_t *b);

/* PUSCH frequency hopping type 2 (subband hopping, 36.211 5.3.4; selected by the DCI format 0 / RAR hopping
 * bits, 36.213 8.4 Table 8.4-1): the first PRB of the allocation n_vrb .. n_vrb + L - 1 in slot ns (0..19) of
 * the frame, given the cell's pusch-HoppingOffset n_ho, hopping subbands n_sb (>= 1), the hopping mode
 * (intra = intra- and inter-subframe, else inter-subframe) and CURRENT_TX_NB.  Every VRB is mapped by
 *   n~_PRB = (n~_VRB + f_hop(i) N_sb^RB + ((N_sb^RB - 1) - 2 (n~_VRB mod N_sb^RB)) f_m(i)) mod (N_sb^RB N_sb),
 * n~_VRB = n_VRB - N~_HO / 2 and n_PRB = n~_PRB + N~_HO / 2 (N_sb > 1; N~_HO = n_ho rounded up to even,
 * N_sb^RB = floor((N_RB - N~_HO - N_RB mod 2) / N_sb)), N_sb^RB = N_RB and no offset for N_sb = 1; f_hop and
 * f_m from the Gold sequence c(k) with c_init = N_ID^cell restarted each frame, i = ns (intra) or ns / 2.
 * Returns the lowest PRB of the mapped set, or -1 if the set is not L contiguous PRBs inside the band. */
int mi_ul_hop_type2(uint32_t nof_prb, uint32_t n_ho, uint32_t n_sb, int intra, uint32_t cell_id, uint32_t n_vrb,
                    uint32_t L, uint32_t ns, uint32_t current_tx_nb);

#ifdef __cplusplus
}
#endif
#endif
