/*
 * tti_latency.c -- per-TTI latency of the srsLTE-compatible API as srsUE's phch_worker drives it
 * (/root/reference/ue/src/phy/phch_worker.cc): per DL subframe srslte_ue_dl_decode_fft_estimate (:254),
 * srslte_ue_dl_cfg_grant (:337), srslte_pdsch_decode_rnti (:347) from the worker's host IQ buffer
 * (H2D, kernels, mirrors and payload D2H all included), and per UL subframe srslte_ue_ul_cfg_grant +
 * srslte_ue_ul_pusch_encode_rnti_softbuffer (:551-555) into the worker's host signal buffer.
 * srsUE must finish the DL decode (and encode the ACK-carrying UL) within ~3 ms of the subframe's
 * arrival (UL at TTI + 4, phch_recv.cc:332-337) with 1-4 workers (phy.h:118-119).
 * With <workers> > 1, that many threads each own their instances (srslte_ue_dl_t, srslte_ue_ul_t, softbuffers, as
 * each phch_worker does) and run their TTIs at the same time, released together; the statistics pool every
 * worker's TTIs (what one TTI costs while the other workers decode theirs).
 * Usage: tti_latency <nof_prb> <ntti per worker> [workers]  ->  one JSON line on stdout.
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
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

static const uint32_t TBS_DL = 75376, TBS_UL = 43816;   /* DL MCS 28 (100 PRB), UL 16QAM MCS 20 */

typedef struct {
  uint32_t nof_prb;
  int ntti;
  cf_t **iq;                 /* [10] shared read-only subframes */
  const uint8_t *tb, *ul_tb;
  pthread_barrier_t *bar;
  double *fft, *dec, *tot, *ul;   /* [ntti] this worker's latencies */
  int ok, n, err;
} job_t;

/* one phch_worker: its own instances, srsUE's per-TTI call sequence over its TTIs */
static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.id = 1; cell.nof_prb = j->nof_prb; cell.nof_ports = 1; cell.cp = SRSLTE_CP_NORM;
  srslte_ue_dl_t ue_dl;
  srslte_ue_ul_t ue_ul;
  srslte_softbuffer_rx_t sbr;
  srslte_softbuffer_tx_t sbt;
  if (srslte_ue_dl_init(&ue_dl, cell) || srslte_ue_ul_init(&ue_ul, cell) || srslte_softbuffer_rx_init(&sbr, 100) ||
      srslte_softbuffer_tx_init(&sbt, 100)) { j->err = 3; if (j->bar) pthread_barrier_wait(j->bar); return NULL; }
  srslte_ue_dl_set_rnti(&ue_dl, 0x46);
  srslte_ue_ul_set_rnti(&ue_ul, 0x46);
  const uint32_t sflen = SRSLTE_SF_LEN_PRB(j->nof_prb);
  cf_t *signal = (cf_t *)srslte_vec_malloc(sflen * sizeof(cf_t));
  uint8_t *pay = (uint8_t *)malloc(TBS_DL / 8);
  if (j->bar) pthread_barrier_wait(j->bar);
  for (int it = -20; it < 2 * j->ntti && j->n < j->ntti; it++) {   /* 20 warm-up TTIs */
    const uint32_t sf = (uint32_t)((it + 20) % 10);
    if (sf == 0 || sf == 5) continue;     /* data subframes only (TBS of the headline config) */
    uint32_t cfi = 0;
    srslte_ra_dl_grant_t g;
    memset(&g, 0, sizeof(g));
    for (uint32_t q = 0; q < j->nof_prb; q++) g.prb_idx[0][q] = g.prb_idx[1][q] = true;
    g.nof_prb = j->nof_prb; g.Qm = 6; g.mcs.mod = SRSLTE_MOD_64QAM; g.mcs.tbs = (int)TBS_DL;
    const double t0 = now_us();
    if (srslte_ue_dl_decode_fft_estimate(&ue_dl, j->iq[sf], sf, &cfi) < 0) { j->err = 4; break; }
    const double t1 = now_us();
    srslte_softbuffer_rx_reset_tbs(&sbr, TBS_DL);
    if (srslte_ue_dl_cfg_grant(&ue_dl, &g, cfi, sf, 0)) { j->err = 5; break; }
    const int r = srslte_pdsch_decode_rnti(&ue_dl.pdsch, &ue_dl.pdsch_cfg, &sbr, ue_dl.sf_symbols, ue_dl.ce, 0.01f, 0x46, pay);
    const double t2 = now_us();
    srslte_ra_ul_grant_t ug;
    memset(&ug, 0, sizeof(ug));
    ug.L_prb = j->nof_prb; ug.Qm = 4; ug.mcs.tbs = (int)TBS_UL; ug.mcs.mod = SRSLTE_MOD_16QAM;
    srslte_uci_data_t uci;
    memset(&uci, 0, sizeof(uci));
    if (srslte_ue_ul_cfg_grant(&ue_ul, &ug, (sf + 4) % 10, 0, 0) ||
        srslte_ue_ul_pusch_encode_rnti_softbuffer(&ue_ul, (uint8_t *)j->ul_tb, uci, &sbt, 0x46, signal)) { j->err = 6; break; }
    const double t3 = now_us();
    if (it >= 0) {
      j->fft[j->n] = t1 - t0; j->dec[j->n] = t2 - t1; j->tot[j->n] = t2 - t0; j->ul[j->n] = t3 - t2;
      j->ok += r == 0 && !memcmp(pay, j->tb, TBS_DL / 8);
      j->n++;
    }
  }
  free(pay);
  free(signal);
  srslte_softbuffer_rx_free(&sbr);
  srslte_softbuffer_tx_free(&sbt);
  srslte_ue_dl_free(&ue_dl);
  srslte_ue_ul_free(&ue_ul);
  return NULL;
}

int main(int argc, char **argv) {
  const uint32_t nof_prb = argc > 1 ? (uint32_t)atoi(argv[1]) : 100;
  const int ntti = argc > 2 ? atoi(argv[2]) : 200;
  const int nw = argc > 3 ? atoi(argv[3]) : 1;
  if (ntti < 1 || nw < 1 || nw > 16) return 2;
  const uint32_t sflen = SRSLTE_SF_LEN_PRB(nof_prb);
  /* 10 subframes of synthetic IQ (the product's transmitter), one per sf_idx, decoded in TTI order */
  cf_t *iq[10];
  uint8_t *tb = (uint8_t *)malloc(TBS_DL / 8), *ul_tb = (uint8_t *)malloc(TBS_UL / 8);
  for (uint32_t i = 0; i < TBS_DL / 8; i++) tb[i] = (uint8_t)(i * 131 + 7);
  for (uint32_t i = 0; i < TBS_UL / 8; i++) ul_tb[i] = (uint8_t)(i * 29 + 3);
  for (int s = 0; s < 10; s++) {
    mi_dl_sf_cfg_t c;
    memset(&c, 0, sizeof(c));
    c.cell_id = 1; c.nof_prb = nof_prb; c.nof_ports = 1; c.sf_idx = (uint32_t)s; c.cfi = 1; c.tm = 1; c.rnti = 0x46;
    c.tbs = (s == 0 || s == 5) ? 61664 : TBS_DL; c.Qm = 6; c.new_tb = 1;
    for (uint32_t q = 0; q < nof_prb; q++) c.prb_mask[q] = 1;
    iq[s] = (cf_t *)srslte_vec_malloc(sflen * sizeof(cf_t));
    if (mi_tx_subframe(&c, tb, NULL, 30.0f, 0xA5A5 + s, (float *)iq[s])) { fprintf(stderr, "tx\n"); return 3; }
  }
  job_t *jobs = calloc((size_t)nw, sizeof(job_t));
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)nw);
  pthread_t th[16];
  for (int w = 0; w < nw; w++) {
    job_t *j = &jobs[w];
    j->nof_prb = nof_prb; j->ntti = ntti; j->iq = iq; j->tb = tb; j->ul_tb = ul_tb; j->bar = nw > 1 ? &bar : NULL;
    j->fft = malloc(sizeof(double) * ntti); j->dec = malloc(sizeof(double) * ntti);
    j->tot = malloc(sizeof(double) * ntti); j->ul = malloc(sizeof(double) * ntti);
  }
  const double t0 = now_us();
  for (int w = 0; w < nw; w++) pthread_create(&th[w], NULL, worker, &jobs[w]);
  for (int w = 0; w < nw; w++) pthread_join(th[w], NULL);
  const double wall = now_us() - t0;
  const int N = nw * ntti;
  double *fft = malloc(sizeof(double) * N), *dec = malloc(sizeof(double) * N), *tot = malloc(sizeof(double) * N),
         *ul = malloc(sizeof(double) * N);
  int ok = 0, n = 0, err = 0;
  for (int w = 0; w < nw; w++) {
    const job_t *j = &jobs[w];
    if (j->err) { fprintf(stderr, "worker %d: error %d\n", w, j->err); err = j->err; }
    for (int i = 0; i < j->n; i++) {
      fft[n] = j->fft[i]; dec[n] = j->dec[i]; tot[n] = j->tot[i]; ul[n] = j->ul[i];
      n++;
    }
    ok += j->ok;
  }
  if (err || !n) return 4;
  printf("{\"workload\": \"per-TTI srsLTE API, %u PRB: DL TM1 MCS 28 (TBS %u) decode_fft_estimate + cfg_grant + "
         "pdsch_decode_rnti from host IQ; UL 16QAM MCS 20 (TBS %u) cfg_grant + pusch_encode to host\", "
         "\"workers\": %d, \"ttis\": %d, \"crc_ok_and_payload_match\": %d, \"wall_us\": %.1f, ", nof_prb, TBS_DL, TBS_UL,
         nw, n, ok, wall);
  stats("decode_fft_estimate", fft, n, 0);
  stats("pdsch_decode_rnti", dec, n, 0);
  stats("dl_total", tot, n, 0);
  stats("ul_pusch_encode", ul, n, 1);
  printf("}\n");
  return 0;
}
