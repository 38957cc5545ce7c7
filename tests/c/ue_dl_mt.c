/*
 * ue_dl_mt.c -- concurrent per-TTI instances, as srsUE runs them: 1-4 phch_worker threads, each with its own
 * srslte_ue_dl_t and softbuffer (/root/reference/ue/hdr/phy/phy.h:118-119, phch_worker.cc:69-74), each
 * decoding its own TTIs through srslte_ue_dl_decode_fft_estimate (:254) -> srslte_ue_dl_cfg_grant (:337) ->
 * srslte_pdsch_decode_rnti (:347), all at the same time.
 *
 * Every thread's TTIs are first decoded sequentially by one instance (the reference results), then by
 * <nthreads> instances in <nthreads> threads released together; per TTI the return value, CFI, iteration
 * count and payload must be identical, and every CRC-OK payload must equal the transmitted TB.  Half of the
 * TTIs are in the turbo waterfall (some iterate to the cap and fail), so early stop and iteration counts
 * are exercised under concurrency too.
 * Usage: ue_dl_mt <nthreads> <ttis per thread>  ->  one JSON line; exit 0 iff everything matched.
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mi_dl.h"
#include "srslte/srslte.h"

#define NPRB 100
#define TBS 75376
#define TBS05 61664   /* sf 0 / 5: PBCH / sync symbols leave fewer REs; MCS 28 shrinks the TBS */

typedef struct {
  int ret, noi;
  uint32_t cfi;
  uint8_t pay[TBS / 8];
} res_t;

typedef struct {
  int t, n;
  cf_t **iq;        /* [n] subframes */
  uint8_t **tb;     /* [n] transmitted TBs */
  res_t *out;       /* [n] */
  pthread_barrier_t *bar;
  double us;
  int err;
} job_t;

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static uint16_t rnti_of(int t) { return (uint16_t)(0x46 + 17 * t); }
static uint32_t tbs_of(uint32_t sf) { return (sf == 0 || sf == 5) ? TBS05 : TBS; }

/* one worker: its own instance and softbuffer, the srsUE per-TTI call sequence over its TTIs */
static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  srslte_cell_t cell;
  memset(&cell, 0, sizeof(cell));
  cell.id = 1; cell.nof_prb = NPRB; cell.nof_ports = 1; cell.cp = SRSLTE_CP_NORM;
  srslte_ue_dl_t ue_dl;
  srslte_softbuffer_rx_t sb;
  if (srslte_ue_dl_init(&ue_dl, cell) || srslte_softbuffer_rx_init(&sb, NPRB)) { j->err = 1; return NULL; }
  srslte_ue_dl_set_rnti(&ue_dl, rnti_of(j->t));
  if (j->bar) pthread_barrier_wait(j->bar);
  const double t0 = now_us();
  for (int i = 0; i < j->n; i++) {
    const uint32_t sf = (uint32_t)(i % 10);
    res_t *r = &j->out[i];
    memset(r, 0, sizeof(*r));
    if (srslte_ue_dl_decode_fft_estimate(&ue_dl, j->iq[i], sf, &r->cfi) < 0) { j->err = 2; break; }
    srslte_ra_dl_grant_t g;
    memset(&g, 0, sizeof(g));
    for (uint32_t q = 0; q < NPRB; q++) g.prb_idx[0][q] = g.prb_idx[1][q] = true;
    g.nof_prb = NPRB; g.Qm = 6; g.mcs.mod = SRSLTE_MOD_64QAM; g.mcs.tbs = (int)tbs_of(sf);
    srslte_softbuffer_rx_reset_tbs(&sb, tbs_of(sf));
    if (srslte_ue_dl_cfg_grant(&ue_dl, &g, r->cfi, sf, 0)) { j->err = 3; break; }
    r->ret = srslte_pdsch_decode_rnti(&ue_dl.pdsch, &ue_dl.pdsch_cfg, &sb, ue_dl.sf_symbols, ue_dl.ce, 0.01f,
                                      rnti_of(j->t), r->pay);
    r->noi = (int)srslte_pdsch_last_noi(&ue_dl.pdsch);
  }
  j->us = now_us() - t0;
  srslte_softbuffer_rx_free(&sb);
  srslte_ue_dl_free(&ue_dl);
  return NULL;
}

int main(int argc, char **argv) {
  const int nt = argc > 1 ? atoi(argv[1]) : 4;
  const int n = argc > 2 ? atoi(argv[2]) : 20;
  if (nt < 1 || nt > 16 || n < 1) return 2;
  const uint32_t sflen = SRSLTE_SF_LEN_PRB(NPRB);
  job_t *jobs = calloc((size_t)nt, sizeof(job_t));
  res_t **seq = calloc((size_t)nt, sizeof(res_t *));
  for (int t = 0; t < nt; t++) {
    job_t *j = &jobs[t];
    j->t = t; j->n = n;
    j->iq = calloc((size_t)n, sizeof(cf_t *));
    j->tb = calloc((size_t)n, sizeof(uint8_t *));
    j->out = calloc((size_t)n, sizeof(res_t));
    seq[t] = calloc((size_t)n, sizeof(res_t));
    for (int i = 0; i < n; i++) {
      const uint32_t sf = (uint32_t)(i % 10);
      mi_dl_sf_cfg_t c;
      memset(&c, 0, sizeof(c));
      c.cell_id = 1; c.nof_prb = NPRB; c.nof_ports = 1; c.sf_idx = sf; c.cfi = 1 + (uint32_t)((t + i) % 3); c.tm = 1;
      c.rnti = rnti_of(t); c.tbs = tbs_of(sf); c.Qm = 6; c.new_tb = 1;
      for (uint32_t q = 0; q < NPRB; q++) c.prb_mask[q] = 1;
      j->tb[i] = malloc(TBS / 8);
      for (uint32_t b = 0; b < TBS / 8; b++) j->tb[i][b] = (uint8_t)((b * 131u + 7u * (uint32_t)i + 29u * (uint32_t)t) ^ (b >> 5));
      j->iq[i] = (cf_t *)srslte_vec_malloc(sflen * sizeof(cf_t));
      /* odd TTIs in the waterfall (iterating, some failing), even ones clean */
      const float snr = (i & 1) ? 19.5f : 30.0f;
      if (mi_tx_subframe(&c, j->tb[i], NULL, snr, 0x5EED00ull + 1000ull * (uint64_t)t + (uint64_t)i, (float *)j->iq[i])) {
        fprintf(stderr, "tx\n");
        return 3;
      }
    }
  }
  /* sequential reference: thread t's TTIs through one instance, one thread after the other */
  const double ts = now_us();
  for (int t = 0; t < nt; t++) {
    job_t s = jobs[t];
    s.out = seq[t];
    s.bar = NULL;
    worker(&s);
    if (s.err) { fprintf(stderr, "sequential worker %d: error %d\n", t, s.err); return 4; }
  }
  const double seq_wall = now_us() - ts;
  /* concurrent: nt instances in nt threads, released together */
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)nt);
  pthread_t th[16];
  const double t0 = now_us();
  for (int t = 0; t < nt; t++) {
    jobs[t].bar = &bar;
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < nt; t++) pthread_join(th[t], NULL);
  const double wall = now_us() - t0;
  int mism = 0, errs = 0, crc_ok = 0, bad_payload = 0, iterating = 0, failed = 0;
  for (int t = 0; t < nt; t++) {
    errs += jobs[t].err != 0;
    for (int i = 0; i < n; i++) {
      const res_t *a = &jobs[t].out[i], *b = &seq[t][i];
      const uint32_t nb = tbs_of((uint32_t)(i % 10)) / 8;
      if (a->ret != b->ret || a->noi != b->noi || a->cfi != b->cfi || memcmp(a->pay, b->pay, nb)) mism++;
      if (a->ret == 0) {
        crc_ok++;
        bad_payload += memcmp(a->pay, jobs[t].tb[i], nb) != 0;
      } else {
        failed++;
      }
      iterating += a->noi > 1;
    }
  }
  printf("{\"threads\": %d, \"ttis_per_thread\": %d, \"errors\": %d, \"mismatches_vs_sequential\": %d, "
         "\"crc_ok\": %d, \"crc_failed\": %d, \"iterating_ttis\": %d, \"crc_ok_payload_mismatches\": %d, "
         "\"wall_us\": %.1f, \"us_per_tti_per_thread\": %.1f, \"sequential_us_per_tti\": %.1f, "
         "\"concurrent_ttis_per_s\": %.1f}\n",
         nt, n, errs, mism, crc_ok, failed, iterating, bad_payload, wall, wall / n, seq_wall / (nt * n),
         nt * n / (wall * 1e-6));
  return (errs || mism || bad_payload) ? 1 : 0;
}
