/*
 * ue_dl_harness.c -- drives the srsLTE-1.0-compatible DL API (include/srslte/srslte.h) the way
 * srsUE's phch_worker does per TTI (/root/reference/ue/src/phy/phch_worker.cc):
 *   init_cell: srslte_ue_dl_init (:74), srslte_sch_set_max_noi (:88), srslte_ue_dl_set_rnti (:127)
 *   MAC:       srslte_softbuffer_rx_init (dl_harq.cc:174), _reset_tbs on a new TB (dl_harq.cc:232)
 *   per TTI:   srslte_ue_dl_decode_fft_estimate (:254), srslte_ue_dl_cfg_grant (:337),
 *              srslte_pdsch_decode_rnti(.., ue_dl.sf_symbols, ue_dl.ce, 0.01, ..) (:347-348),
 *              srslte_pdsch_last_noi (:360), srslte_chest_dl_get_* (:799-848)
 *   PDCCH mode (hdr[5] = 1): srslte_pdcch_extract_llr (:260), srslte_ue_dl_find_dl_dci_type (:293),
 *              srslte_dci_msg_to_dl_grant (:297), srslte_ue_dl_get_ncce (:314); the PDSCH grant and
 *              rv come from the decoded DCI (p[2], p[3] unused)
 *   PHICH (hdr[6] = 1): srslte_ue_dl_decode_phich(&ue_dl, sf, I_lowest, n_dmrs) (:381) after the PDSCH,
 *              with I_lowest = hdr[7] & 0xffff, n_dmrs = hdr[7] >> 16
 * Input file : int32 hdr[8] = {cell_id, nof_prb, nof_ports, nsf, phich_ng, pdcch_mode, phich, query}; per subframe
 *              int32 p[8] = {sf_idx, tbs, Qm, rv, reset_tbs, rnti, max_its, pass_own_buffers} +
 *              2*SF_LEN floats.  p[5] = rnti | rnti_type << 16 (srslte_rnti_type_t of the PDCCH search:
 *              SRSLTE_RNTI_USER searches the C-RNTI spaces, SI/RAR/PCH the common space with 1A and 1C).
 * Output file: per subframe int32 r[8] = {ret, cfi, noi, dci_found, ncce, grant_tbs, harq, rv} +
 *              float m[5] + int32 phich (1 ACK, 0 NACK, -1 not asked) + tbs/8 payload bytes.
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
  if (fread(hdr, 4, 8, fi) != 8) return 2;
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.id = (uint32_t)hdr[0]; cell.nof_prb = (uint32_t)hdr[1]; cell.nof_ports = (uint32_t)hdr[2];
  cell.cp = SRSLTE_CP_NORM;
  cell.phich_length = SRSLTE_PHICH_NORM;
  cell.phich_resources = (srslte_phich_resources_t)hdr[4];
  const int pdcch_mode = hdr[5];
  if (!srslte_check_version(1, 0, 0)) { fprintf(stderr, "version\n"); return 3; }
  srslte_ue_dl_t ue_dl;
  if (srslte_ue_dl_init(&ue_dl, cell)) { fprintf(stderr, "ue_dl_init\n"); return 3; }
  srslte_softbuffer_rx_t sb;
  if (srslte_softbuffer_rx_init(&sb, 100)) { fprintf(stderr, "softbuffer\n"); return 3; }
  const uint32_t sflen = SRSLTE_SF_LEN_PRB(cell.nof_prb);
  cf_t *buf = (cf_t *)srslte_vec_malloc(2 * sflen * sizeof(cf_t));
  uint8_t *payload = (uint8_t *)malloc(19200);
  for (int s = 0; s < hdr[3]; s++) {
    int32_t p[8];
    if (fread(p, 4, 8, fi) != 8 || fread(buf, 8, sflen, fi) != sflen) return 4;
    if (p[6] > 0) srslte_sch_set_max_noi(&ue_dl.pdsch.dl_sch, (uint32_t)p[6]);
    const uint16_t rnti = (uint16_t)(p[5] & 0xffff);
    const srslte_rnti_type_t rtype = (srslte_rnti_type_t)(p[5] >> 16);
    if (rtype == SRSLTE_RNTI_USER) srslte_ue_dl_set_rnti(&ue_dl, rnti);
    if (p[4]) srslte_softbuffer_rx_reset_tbs(&sb, (uint32_t)p[1]);
    int32_t r[8] = {0};
    float m[5] = {0};
    uint32_t cfi = 0;
    int ret = srslte_ue_dl_decode_fft_estimate(&ue_dl, buf, (uint32_t)p[0], &cfi);
    if (ret < 0) ret = -9;
    srslte_ra_dl_grant_t grant;
    memset(&grant, 0, sizeof(grant));
    uint32_t rv = (uint32_t)p[3];
    if (ret >= 0 && pdcch_mode) {
      srslte_dci_msg_t msg;
      srslte_ra_dl_dci_t dci;
      if (srslte_pdcch_extract_llr(&ue_dl.pdcch, ue_dl.sf_symbols, ue_dl.ce, 0, (uint32_t)p[0], cfi)) {
        ret = -11;
      } else if ((r[3] = srslte_ue_dl_find_dl_dci_type(&ue_dl, &msg, cfi, (uint32_t)p[0], rnti, rtype)) != 1) {
        ret = -12;
      } else if (srslte_dci_msg_to_dl_grant(&msg, rnti, cell.nof_prb, &dci, &grant)) {
        ret = -13;
      } else {
        r[4] = (int32_t)srslte_ue_dl_get_ncce(&ue_dl);
        r[5] = grant.mcs.tbs;
        r[6] = (int32_t)dci.harq_process;
        r[7] = (int32_t)dci.rv_idx;
        rv = dci.rv_idx;
      }
    } else if (ret >= 0) {
      for (uint32_t q = 0; q < cell.nof_prb; q++) grant.prb_idx[0][q] = grant.prb_idx[1][q] = true;
      grant.nof_prb = cell.nof_prb;
      grant.Qm = (uint32_t)p[2];
      grant.mcs.mod = p[2] == 2 ? SRSLTE_MOD_QPSK : p[2] == 4 ? SRSLTE_MOD_16QAM : SRSLTE_MOD_64QAM;
      grant.mcs.tbs = p[1];
    }
    if (ret >= 0) {
      if (srslte_ue_dl_cfg_grant(&ue_dl, &grant, cfi, (uint32_t)p[0], rv)) {
        ret = -10;
      } else if (ue_dl.pdsch_cfg.grant.mcs.mod > 0 && ue_dl.pdsch_cfg.grant.mcs.tbs >= 0) {
        cf_t *grid = ue_dl.sf_symbols;
        cf_t *ce[SRSLTE_MAX_PORTS] = {ue_dl.ce[0], ue_dl.ce[1], ue_dl.ce[2], ue_dl.ce[3]};
        cf_t *copy = NULL, *ce_copy[SRSLTE_MAX_PORTS] = {0};
        if (!p[7]) {   /* caller-owned copies: exercises the upload path */
          size_t n = 14 * 12 * cell.nof_prb;
          copy = (cf_t *)malloc(n * sizeof(cf_t));
          memcpy(copy, grid, n * sizeof(cf_t));
          grid = copy;
          for (uint32_t q = 0; q < cell.nof_ports; q++) {
            ce_copy[q] = (cf_t *)malloc(n * sizeof(cf_t));
            memcpy(ce_copy[q], ue_dl.ce[q], n * sizeof(cf_t));
            ce[q] = ce_copy[q];
          }
        }
        ret = srslte_pdsch_decode_rnti(&ue_dl.pdsch, &ue_dl.pdsch_cfg, &sb, grid, ce, 0.01f, rnti, payload);
        free(copy);
        for (uint32_t q = 0; q < SRSLTE_MAX_PORTS; q++) free(ce_copy[q]);
      }
    }
    r[0] = ret; r[1] = (int32_t)cfi; r[2] = (int32_t)srslte_pdsch_last_noi(&ue_dl.pdsch);
    if (!pdcch_mode) r[3] = r[4] = r[5] = r[6] = r[7] = 0;
    m[0] = srslte_chest_dl_get_rsrp(&ue_dl.chest); m[1] = srslte_chest_dl_get_rssi(&ue_dl.chest);
    m[2] = srslte_chest_dl_get_rsrq(&ue_dl.chest); m[3] = srslte_chest_dl_get_noise_estimate(&ue_dl.chest);
    m[4] = srslte_chest_dl_get_snr(&ue_dl.chest);
    int32_t ph = -1;
    if (hdr[6]) ph = srslte_ue_dl_decode_phich(&ue_dl, (uint32_t)p[0], (uint32_t)hdr[7] & 0xffffu, (uint32_t)hdr[7] >> 16);
    fwrite(r, 4, 8, fo);
    fwrite(m, 4, 5, fo);
    fwrite(&ph, 4, 1, fo);
    fwrite(payload, 1, (size_t)p[1] / 8, fo);
  }
  srslte_softbuffer_rx_free(&sb);
  srslte_ue_dl_free(&ue_dl);
  free(buf);
  free(payload);
  fclose(fi);
  fclose(fo);
  return 0;
}
