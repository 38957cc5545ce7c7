/*
 * ue_ul_harness.c -- drives the srsLTE-1.0-compatible UL PUSCH API (include/srslte/srslte.h) the way
 * srsUE's phch_worker does (/root/reference/ue/src/phy/phch_worker.cc):
 *   init_cell: srslte_ue_ul_init (:79), srslte_ue_ul_set_normalization (:83), _set_cfo_enable (:84),
 *              srslte_ue_ul_set_rnti (:128), srslte_ue_ul_set_cfg (:748)
 *   MAC:       srslte_softbuffer_tx_init (ul_harq.cc:198)
 *   per TTI:   srslte_ue_ul_set_cfo (:213), srslte_dci_msg_to_ul_grant (:429, DCI mode), or for a random-access
 *              response grant srslte_dci_rar_grant_unpack (phch_common.cc:122) + srslte_dci_rar_to_ul_grant (:412),
 *              srslte_ue_ul_cfg_grant(&ue_ul, grant, tti + 4, rv, tx_nb) (:551),
 *              srslte_ue_ul_pusch_encode_rnti_softbuffer(.., payload, uci_data, softbuffer, rnti, signal) (:555)
 * Input file : int32 hdr[8] = {cell_id, nof_prb, ntx, group_hopping, sequence_hopping, delta_ss, cyclic_shift,
 *              flags (1 = normalisation, 2 = CFO, bits 8-11 = I_offset_ack, bits 12-19 = pusch-HoppingOffset,
 *              bit 20 = intra-subframe hopping, bits 21-24 = I_offset_cqi, bits 25-28 = I_offset_ri,
 *              bits 29-30 = pusch-HoppingSubbands N_sb - 1)} + float cfo;
 *              per transmission int32
 *              p[12] = {tti, rnti, rv | CURRENT_TX_NB << 8, use_dci (0 direct, 1 DCI format 0, 2 RAR grant: the first
 *              20 of the 64 bit bytes), n_prb, L_prb, tbs, Qm, ncs_dmrs, pass_data, ack_len,
 *              ack} + int32 dci_nof_bits + 64 DCI bit bytes + int32 u[3] = {cqi, ri_len, ri} + 64 CQI bit bytes +
 *              tbs/8 payload bytes.  cqi > 0: a wideband CQI report of value cqi - 1 packed with
 *              srslte_cqi_value_pack as srsUE does (phch_worker.cc:517-521); cqi < 0: -cqi raw CQI bits from the
 *              64 bytes; 0: no CQI.  Payload bytes (pass_data = 0: the payload pointer is NULL -- a retransmission from the
 *              softbuffer).
 * Output file: per transmission int32 r[7] = {ret, n_prb slot 0, L_prb, tbs, Qm, ncs_dmrs, n_prb slot 1} + SF_LEN
 *              cf32 samples (the slot PRBs as cfg_grant set them in ue_ul.pusch_cfg.grant).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "srslte/srslte.h"

int main(int argc, char **argv) {
  if (argc != 3) { fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]); return 2; }
  FILE *fi = fopen(argv[1], "rb"), *fo = fopen(argv[2], "wb");
  if (!fi || !fo) return 2;
  int32_t hdr[8];
  float cfo;
  if (fread(hdr, 4, 8, fi) != 8 || fread(&cfo, 4, 1, fi) != 1) return 2;
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.id = (uint32_t)hdr[0];
  cell.nof_prb = (uint32_t)hdr[1];
  cell.nof_ports = 1;
  cell.cp = SRSLTE_CP_NORM;
  srslte_ue_ul_t ue_ul;
  if (srslte_ue_ul_init(&ue_ul, cell)) { fprintf(stderr, "ue_ul_init\n"); return 3; }
  srslte_ue_ul_set_normalization(&ue_ul, (hdr[7] & 1) != 0);
  srslte_ue_ul_set_cfo_enable(&ue_ul, (hdr[7] & 2) != 0);
  srslte_refsignal_dmrs_pusch_cfg_t dmrs_cfg;
  srslte_pusch_hopping_cfg_t pusch_hopping;
  srslte_refsignal_srs_cfg_t srs_cfg;
  srslte_pucch_cfg_t pucch_cfg;
  srslte_pucch_sched_t pucch_sched;
  srslte_uci_cfg_t uci_cfg;
  srslte_ue_ul_powerctrl_t power_ctrl;
  memset(&dmrs_cfg, 0, sizeof(dmrs_cfg)); memset(&pusch_hopping, 0, sizeof(pusch_hopping));
  memset(&srs_cfg, 0, sizeof(srs_cfg)); memset(&pucch_cfg, 0, sizeof(pucch_cfg));
  memset(&pucch_sched, 0, sizeof(pucch_sched)); memset(&uci_cfg, 0, sizeof(uci_cfg));
  memset(&power_ctrl, 0, sizeof(power_ctrl));
  uci_cfg.I_offset_ack = (uint32_t)(hdr[7] >> 8) & 15u;
  uci_cfg.I_offset_cqi = (uint32_t)(hdr[7] >> 21) & 15u;
  uci_cfg.I_offset_ri = (uint32_t)(hdr[7] >> 25) & 15u;
  dmrs_cfg.group_hopping_en = hdr[3] != 0;
  dmrs_cfg.sequence_hopping_en = hdr[4] != 0;
  dmrs_cfg.delta_ss = (uint32_t)hdr[5];
  dmrs_cfg.cyclic_shift = (uint32_t)hdr[6];
  pusch_hopping.hop_mode = (hdr[7] >> 20) & 1 ? SRSLTE_PUSCH_HOP_MODE_INTRA_SF : SRSLTE_PUSCH_HOP_MODE_INTER_SF;
  pusch_hopping.hopping_offset = (uint32_t)(hdr[7] >> 12) & 255u;
  pusch_hopping.n_sb = 1u + ((uint32_t)(hdr[7] >> 29) & 3u);
  srslte_ue_ul_set_cfg(&ue_ul, &dmrs_cfg, &srs_cfg, &pucch_cfg, &pucch_sched, &uci_cfg, &pusch_hopping, &power_ctrl);
  srslte_softbuffer_tx_t softbuffer;
  if (srslte_softbuffer_tx_init(&softbuffer, 100)) { fprintf(stderr, "softbuffer_tx\n"); return 3; }
  const uint32_t sflen = SRSLTE_SF_LEN_PRB(cell.nof_prb);
  cf_t *signal = (cf_t *)srslte_vec_malloc(sflen * sizeof(cf_t));
  uint8_t *payload = (uint8_t *)malloc(12288);
  for (int i = 0; i < hdr[2]; i++) {
    int32_t p[12], nbits;
    srslte_dci_msg_t dci_msg;
    memset(&dci_msg, 0, sizeof(dci_msg));
    int32_t u[3];
    uint8_t cqi_bits[64];
    if (fread(p, 4, 12, fi) != 12 || fread(&nbits, 4, 1, fi) != 1 || fread(dci_msg.data, 1, 64, fi) != 64) return 4;
    if (fread(u, 4, 3, fi) != 3 || fread(cqi_bits, 1, 64, fi) != 64) return 4;
    if (fread(payload, 1, (size_t)p[6] / 8, fi) != (size_t)p[6] / 8) return 4;
    dci_msg.nof_bits = (uint32_t)nbits;
    srslte_ue_ul_set_rnti(&ue_ul, (uint16_t)p[1]);
    srslte_ue_ul_set_cfo(&ue_ul, cfo);
    srslte_ra_ul_grant_t grant;
    memset(&grant, 0, sizeof(grant));
    int ret = 0;
    if (p[3] == 2) {   /* Msg3: the MAC's RAR grant bits, unpacked by phch_common then converted by the worker */
      srslte_dci_rar_grant_t rar;
      srslte_ra_ul_dci_t dci_unpacked;
      srslte_dci_rar_grant_unpack(&rar, dci_msg.data);
      ret = srslte_dci_rar_to_ul_grant(&rar, cell.nof_prb, pusch_hopping.hopping_offset, &dci_unpacked, &grant);
    } else if (p[3]) {
      srslte_ra_ul_dci_t dci_unpacked;
      ret = srslte_dci_msg_to_ul_grant(&dci_msg, cell.nof_prb, pusch_hopping.hopping_offset, &dci_unpacked, &grant,
                                       (uint32_t)p[0]);
    } else {
      grant.n_prb[0] = grant.n_prb[1] = (uint32_t)p[4];
      grant.L_prb = (uint32_t)p[5];
      grant.mcs.tbs = p[6];
      grant.Qm = (uint32_t)p[7];
      grant.ncs_dmrs = (uint32_t)p[8];
    }
    if (!ret)
      ret = srslte_ue_ul_cfg_grant(&ue_ul, &grant, (uint32_t)p[0], (uint32_t)p[2] & 255u, (uint32_t)p[2] >> 8) ? -2 : 0;
    srslte_uci_data_t uci_data;
    memset(&uci_data, 0, sizeof(uci_data));
    uci_data.uci_ack_len = (uint32_t)p[10];   /* phch_worker.cc:486-487 */
    uci_data.uci_ack = (uint8_t)p[11];
    if (u[0] > 0) {   /* periodic wideband CQI, phch_worker.cc:517-521 */
      srslte_cqi_value_t cqi_report;
      memset(&cqi_report, 0, sizeof(cqi_report));
      cqi_report.type = SRSLTE_CQI_TYPE_WIDEBAND;
      cqi_report.wideband.wideband_cqi = (uint8_t)(u[0] - 1);
      uci_data.uci_cqi_len = (uint32_t)srslte_cqi_value_pack(&cqi_report, uci_data.uci_cqi);
    } else if (u[0] < 0) {
      uci_data.uci_cqi_len = (uint32_t)(-u[0]);
      memcpy(uci_data.uci_cqi, cqi_bits, uci_data.uci_cqi_len);
    }
    uci_data.uci_ri_len = (uint32_t)u[1];
    uci_data.uci_ri = (uint8_t)u[2];
    memset(signal, 0, sflen * sizeof(cf_t));
    if (!ret)
      ret = srslte_ue_ul_pusch_encode_rnti_softbuffer(&ue_ul, p[9] ? payload : NULL, uci_data, &softbuffer,
                                                      (uint16_t)p[1], signal) ? -3 : 0;
    const srslte_ra_ul_grant_t* gs = ret ? &grant : &ue_ul.pusch_cfg.grant;
    int32_t r[7] = {ret, (int32_t)gs->n_prb[0], (int32_t)grant.L_prb, grant.mcs.tbs, (int32_t)grant.Qm,
                    (int32_t)grant.ncs_dmrs, (int32_t)gs->n_prb[1]};
    fwrite(r, 4, 7, fo);
    fwrite(signal, 8, sflen, fo);
  }
  srslte_softbuffer_tx_free(&softbuffer);
  srslte_ue_ul_free(&ue_ul);
  free(payload);
  srslte_vec_free(signal);
  fclose(fi);
  fclose(fo);
  return 0;
}
