/*
 * tti_latency.c -- per-TTI latency of the srsLTE-compatible API as srsUE's phch_worker drives it
 * (/root/reference/ue/src/phy/phch_worker.cc): per DL subframe srslte_ue_dl_decode_fft_estimate (:254),
 * srslte_ue_dl_cfg_grant (:337), srslte_pdsch_decode_rnti (:347) from the worker's host IQ buffer
 * (H2D, kernels, mirrors and payload D2H all included), and per UL subframe srslte_ue_ul_cfg_grant +
 * srslte_ue_ul_pusch_encode_rnti_softbuffer (:551-555) into the worker's host signal buffer.
 * srsUE must finish the DL decode (and encode the ACK-carrying UL) within ~3 ms of the subframe's
 * arrival (UL at TTI + 4, phch_recv.cc:332-337) with 1-4 workers.
 * Usage: tti_latency <nof_prb> <ntti>   ->  one JSON line on stdout.
 */
#define _POSIX_C_SOURCE 199309L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mi_dl.h"
#include "srslte/srslte.h"

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}
static int cmp(const void *a, const void *b) {
  const double x = *(const double *)a, y = *(const double *)b;
  return x < y ? -1 : x > y;
}
static void stats(const char *name, double *v, int n, int last) {
  qsort(v, (size_t)n, sizeof(double), cmp);
  double s = 0;
  for (int i = 0; i < n; i++) s += v[i];
  printf("\"%s\": {\"mean_us\": %.1f, \"p50_us\": %.1f, \"p99_us\": %.1f, \"max_us\": %.1f}%s", name, s / n, v[n / 2],
         v[(int)(0.99 * (n - 1))], v[n - 1], last ? "" : ", ");
}

int main(int argc, char **argv) {
  const uint32_t nof_prb = argc > 1 ? (uint32_t)atoi(argv[1]) : 100;
  const int ntti = argc > 2 ? atoi(argv[2]) : 200;
  const uint32_t tbs_dl = 75376, tbs_ul = 43816;   /* DL MCS 28 (100 PRB), UL 16QAM MCS 20 */
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.id = 1; cell.nof_prb = nof_prb; cell.nof_ports = 1; cell.cp = SRSLTE_CP_NORM;
  srslte_ue_dl_t ue_dl;
  srslte_ue_ul_t ue_ul;
  srslte_softbuffer_rx_t sbr;
  srslte_softbuffer_tx_t sbt;
  if (srslte_ue_dl_init(&ue_dl, cell) || srslte_ue_ul_init(&ue_ul, cell) || srslte_softbuffer_rx_init(&sbr, 100) ||
      srslte_softbuffer_tx_init(&sbt, 100)) { fprintf(stderr, "init\n"); return 3; }
  srslte_ue_dl_set_rnti(&ue_dl, 0x46);
  srslte_ue_ul_set_rnti(&ue_ul, 0x46);
  const uint32_t sflen = SRSLTE_SF_LEN_PRB(nof_prb);
  /* 10 subframes of synthetic IQ (the product's transmitter), one per sf_idx, decoded in TTI order */
  cf_t *iq[10];
  uint8_t *tb = (uint8_t *)malloc(tbs_dl / 8), *pay = (uint8_t *)malloc(tbs_dl / 8), *ul_tb = (uint8_t *)malloc(tbs_ul / 8);
  for (uint32_t i = 0; i < tbs_dl / 8; i++) tb[i] = (uint8_t)(i * 131 + 7);
  for (uint32_t i = 0; i < tbs_ul / 8; i++) ul_tb[i] = (uint8_t)(i * 29 + 3);
  for (int s = 0; s < 10; s++) {
    mi_dl_sf_cfg_t c;
    memset(&c, 0, sizeof(c));
    c.cell_id = 1; c.nof_prb = nof_prb; c.nof_ports = 1; c.sf_idx = (uint32_t)s; c.cfi = 1; c.tm = 1; c.rnti = 0x46;
    c.tbs = (s == 0 || s == 5) ? 61664 : tbs_dl; c.Qm = 6; c.new_tb = 1;
    for (uint32_t q = 0; q < nof_prb; q++) c.prb_mask[q] = 1;
    iq[s] = (cf_t *)srslte_vec_malloc(sflen * sizeof(cf_t));
    if (mi_tx_subframe(&c, tb, NULL, 30.0f, 0xA5A5 + s, (float *)iq[s])) { fprintf(stderr, "tx\n"); return 3; }
  }
  cf_t *signal = (cf_t *)srslte_vec_malloc(sflen * sizeof(cf_t));
  double *fft = malloc(sizeof(double) * ntti), *dec = malloc(sizeof(double) * ntti), *tot = malloc(sizeof(double) * ntti),
         *ul = malloc(sizeof(double) * ntti);
  int ok = 0, n = 0;
  for (int it = -20; it < ntti; it++) {   /* 20 warm-up TTIs */
    const uint32_t sf = (uint32_t)((it + 20) % 10);
    if (sf == 0 || sf == 5) continue;     /* data subframes only (TBS of the headline config) */
    uint32_t cfi = 0;
    srslte_ra_dl_grant_t g;
    memset(&g, 0, sizeof(g));
    for (uint32_t q = 0; q < nof_prb; q++) g.prb_idx[0][q] = g.prb_idx[1][q] = true;
    g.nof_prb = nof_prb; g.Qm = 6; g.mcs.mod = SRSLTE_MOD_64QAM; g.mcs.tbs = (int)tbs_dl;
    const double t0 = now_us();
    if (srslte_ue_dl_decode_fft_estimate(&ue_dl, iq[sf], sf, &cfi) < 0) { fprintf(stderr, "fft\n"); return 4; }
    const double t1 = now_us();
    srslte_softbuffer_rx_reset_tbs(&sbr, tbs_dl);
    if (srslte_ue_dl_cfg_grant(&ue_dl, &g, cfi, sf, 0)) { fprintf(stderr, "grant\n"); return 4; }
    const int r = srslte_pdsch_decode_rnti(&ue_dl.pdsch, &ue_dl.pdsch_cfg, &sbr, ue_dl.sf_symbols, ue_dl.ce, 0.01f, 0x46, pay);
    const double t2 = now_us();
    srslte_ra_ul_grant_t ug;
    memset(&ug, 0, sizeof(ug));
    ug.L_prb = nof_prb; ug.Qm = 4; ug.mcs.tbs = (int)tbs_ul; ug.mcs.mod = SRSLTE_MOD_16QAM;
    srslte_uci_data_t uci;
    memset(&uci, 0, sizeof(uci));
    if (srslte_ue_ul_cfg_grant(&ue_ul, &ug, (sf + 4) % 10, 0, 0) ||
        srslte_ue_ul_pusch_encode_rnti_softbuffer(&ue_ul, ul_tb, uci, &sbt, 0x46, signal)) { fprintf(stderr, "ul\n"); return 4; }
    const double t3 = now_us();
    if (it >= 0 && n < ntti) {
      fft[n] = t1 - t0; dec[n] = t2 - t1; tot[n] = t2 - t0; ul[n] = t3 - t2;
      ok += r == 0 && !memcmp(pay, tb, tbs_dl / 8);
      n++;
    }
  }
  printf("{\"workload\": \"per-TTI srsLTE API, %u PRB: DL TM1 MCS 28 (TBS %u) decode_fft_estimate + cfg_grant + "
         "pdsch_decode_rnti from host IQ; UL 16QAM MCS 20 (TBS %u) cfg_grant + pusch_encode to host\", "
         "\"ttis\": %d, \"crc_ok_and_payload_match\": %d, ", nof_prb, tbs_dl, tbs_ul, n, ok);
  stats("decode_fft_estimate", fft, n, 0);
  stats("pdsch_decode_rnti", dec, n, 0);
  stats("dl_total", tot, n, 0);
  stats("ul_pusch_encode", ul, n, 1);
  printf("}\n");
  srslte_ue_dl_free(&ue_dl);
  srslte_ue_ul_free(&ue_ul);
  return 0;
}
