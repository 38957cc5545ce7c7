/*
 * o_sync.c -- sync front end: PSS / SSS (36.211 6.11), their transmission, PSS timing + N_ID_2
 * search, PSS-based CFO estimation, SSS detection and CFO correction (TEST INFRASTRUCTURE ONLY).
 * what srsUE reaches through srslte_ue_sync_zerocopy (phch_recv.cc:321) and
 * srslte_ue_sync_get_cfo / _get_sfidx (:322-329, :241).  srsLTE is not in the container: parity
 * against it is unpinned; the ground truth is the transmitter below (a PSS / SSS put on the air at a
 * known timing offset and CFO must be found there).
 *
 * Detection contract (the GPU kernels in srsue_amd/csrc/sync.hip reproduce it in fp32):
 *   template   p[n] = (1/sqrt N) sum_{m<62} d_u(m) e^{+j 2 pi b(m) n / N}, b(m) = FFT bin of
 *              subcarrier m - 31 + 6 N_RB (DC skipped), n < N (useful part of the PSS symbol)
 *   metric     for each lag t: y(t) = sum_n x[t + n] conj(p[n]);  rho(t) = |y|^2 / (E_x(t) E_p),
 *              E_x(t) = sum_n |x[t + n]|^2; the peak is the largest rho over (N_ID_2, t) (first on ties,
 *              N_ID_2 ascending, then t ascending)
 *   CFO        at the peak: y1 = sum_{n < N/2}, y2 = sum_{n >= N/2}; cfo = arg(conj(y1) y2) / pi in
 *              subcarrier spacings (|cfo| < 1)
 *   SSS        after CFO correction: Y(m) = DFT of the SSS symbol at the 62 bins, H(m) = DFT of the PSS
 *              symbol / d_u(m); score(N_ID_1, half) = Re sum_m conj(H(m)) Y(m) d(m); the largest wins
 *   correction y[n] = x[n] e^{-j 2 pi cfo n / N}, phase restarting at every subframe start
 */
#include "oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

static const uint32_t PSS_ROOT[3] = {25, 29, 34};

void or_pss_seq(uint32_t nid2, float *d) {
  const double u = PSS_ROOT[nid2 % 3];
  for (int n = 0; n < 62; n++) {
    const double ph = n < 31 ? -M_PI * u * n * (n + 1) / 63.0 : -M_PI * u * (n + 1) * (n + 2) / 63.0;
    d[2 * n] = (float)cos(ph);
    d[2 * n + 1] = (float)sin(ph);
  }
}

/* m-sequences of 36.211 6.11.2.1: x(i+5) = sum of taps mod 2, x(0..3) = 0, x(4) = 1 */
static void mseq(int t1, int t2, int t3, int t4, int *s) {
  int x[31] = {0, 0, 0, 0, 1};
  for (int i = 0; i < 26; i++) {
    int v = x[i];
    if (t1) v ^= x[i + 1];
    if (t2) v ^= x[i + 2];
    if (t3) v ^= x[i + 3];
    if (t4) v ^= x[i + 4];
    x[i + 5] = v;
  }
  for (int i = 0; i < 31; i++) s[i] = 1 - 2 * x[i];
}

void or_sss_m(uint32_t nid1, uint32_t *m0, uint32_t *m1) {
  const uint32_t qp = nid1 / 30, q = (nid1 + qp * (qp + 1) / 2) / 30, mp = nid1 + q * (q + 1) / 2;
  *m0 = mp % 31;
  *m1 = (*m0 + mp / 31 + 1) % 31;
}

void or_sss_seq(uint32_t nid1, uint32_t nid2, uint32_t sf5, float *d /* 62 real: d(0..61) */) {
  int st[31], ct[31], zt[31];
  mseq(0, 1, 0, 0, st);   /* x(i+5) = x(i+2) + x(i) */
  mseq(0, 0, 1, 0, ct);   /* x(i+5) = x(i+3) + x(i) */
  mseq(1, 1, 0, 1, zt);   /* x(i+5) = x(i+4) + x(i+2) + x(i+1) + x(i) */
  uint32_t m0, m1;
  or_sss_m(nid1, &m0, &m1);
  for (int n = 0; n < 31; n++) {
    const int s0 = st[(n + m0) % 31], s1 = st[(n + m1) % 31];
    const int c0 = ct[(n + nid2) % 31], c1 = ct[(n + nid2 + 3) % 31];
    const int z0 = zt[(n + (m0 % 8)) % 31], z1 = zt[(n + (m1 % 8)) % 31];
    d[2 * n] = (float)(sf5 ? s1 * c0 : s0 * c0);
    d[2 * n + 1] = (float)(sf5 ? s0 * c1 * z1 : s1 * c1 * z0);
  }
}

static uint32_t sync_bin(uint32_t m, uint32_t nof_prb, uint32_t N) {
  const uint32_t W = 12 * nof_prb, k = m - 31 + W / 2;
  return k < W / 2 ? N - W / 2 + k : k - W / 2 + 1;
}

void or_pss_time(uint32_t nid2, uint32_t nof_prb, float *x) {
  const uint32_t N = (uint32_t)or_symbol_sz(nof_prb);
  float d[124];
  or_pss_seq(nid2, d);
  double *X = (double *)calloc(2 * N, sizeof(double)), *t = (double *)malloc(sizeof(double) * 2 * N);
  for (uint32_t m = 0; m < 62; m++) {
    const uint32_t b = sync_bin(m, nof_prb, N);
    X[2 * b] = d[2 * m]; X[2 * b + 1] = d[2 * m + 1];
  }
  or_dft(X, t, (int)N, 1);
  const double nrm = 1.0 / sqrt((double)N);
  for (uint32_t n = 0; n < 2 * N; n++) x[n] = (float)(t[n] * nrm);
  free(X); free(t);
}

/* sample offset of the useful part of symbol l of the subframe */
static uint32_t sym_off(uint32_t N, uint32_t l) {
  uint32_t off = (l / 7) * (15 * N / 2);
  for (uint32_t q = 0; q < l % 7; q++) off += (uint32_t)or_cp_len(N, q) + N;
  return off + (uint32_t)or_cp_len(N, l % 7);
}
uint32_t or_sync_sym_off(uint32_t N, uint32_t l) { return sym_off(N, l); }

int or_tx_sync(uint32_t cell_id, uint32_t nof_prb, uint32_t sf_idx, float amp, float *iq) {
  if (sf_idx != 0 && sf_idx != 5) return 0;
  const uint32_t N = (uint32_t)or_symbol_sz(nof_prb);
  float d[124];
  double *X = (double *)malloc(sizeof(double) * 2 * N), *t = (double *)malloc(sizeof(double) * 2 * N);
  const double nrm = amp / sqrt((double)N);
  for (int sym = 0; sym < 2; sym++) {      /* l = 5: SSS, l = 6: PSS (last symbol of slot 0) */
    if (sym == 0) {
      float r[62];                                              /* real SSS d(0..61) */
      or_sss_seq(cell_id / 3, cell_id % 3, sf_idx == 5, r);
      for (int m = 0; m < 62; m++) { d[2 * m] = r[m]; d[2 * m + 1] = 0.0f; }
    } else {
      or_pss_seq(cell_id % 3, d);
    }
    memset(X, 0, sizeof(double) * 2 * N);
    for (uint32_t m = 0; m < 62; m++) {
      const uint32_t b = sync_bin(m, nof_prb, N);
      X[2 * b] = d[2 * m]; X[2 * b + 1] = d[2 * m + 1];
    }
    or_dft(X, t, (int)N, 1);
    const uint32_t l = 5 + (uint32_t)sym, cp = (uint32_t)or_cp_len(N, l), s0 = sym_off(N, l) - cp;
    for (uint32_t n = 0; n < N + cp; n++) {
      const uint32_t src = (n + N - cp) % N;
      iq[2 * (s0 + n)] += (float)(t[2 * src] * nrm);
      iq[2 * (s0 + n) + 1] += (float)(t[2 * src + 1] * nrm);
    }
  }
  free(X); free(t);
  return 1;
}

int or_pss_find(const float *x, uint32_t nof_prb, uint32_t nid2_mask, uint32_t nlag, or_pss_res_t *r) {
  const uint32_t N = (uint32_t)or_symbol_sz(nof_prb);
  float *p = (float *)malloc(sizeof(float) * 2 * N);
  double best = -1.0;
  memset(r, 0, sizeof(*r));
  for (uint32_t u = 0; u < 3; u++) {
    if (!((nid2_mask >> u) & 1u)) continue;
    or_pss_time(u, nof_prb, p);
    double ep = 0;
    for (uint32_t n = 0; n < N; n++) ep += (double)p[2 * n] * p[2 * n] + (double)p[2 * n + 1] * p[2 * n + 1];
    for (uint32_t t = 0; t < nlag; t++) {
      double y1r = 0, y1i = 0, y2r = 0, y2i = 0, ex = 0;
      for (uint32_t n = 0; n < N; n++) {
        const double ar = x[2 * (t + n)], ai = x[2 * (t + n) + 1], br = p[2 * n], bi = p[2 * n + 1];
        const double cr = ar * br + ai * bi, ci = ai * br - ar * bi;   /* x conj(p) */
        if (n < N / 2) { y1r += cr; y1i += ci; } else { y2r += cr; y2i += ci; }
        ex += ar * ar + ai * ai;
      }
      const double yr = y1r + y2r, yi = y1i + y2i;
      const double rho = ex > 0 ? (yr * yr + yi * yi) / (ex * ep) : 0.0;
      if (rho > best) {
        best = rho;
        r->nid2 = u; r->lag = t; r->rho = (float)rho;
        r->cfo = (float)(atan2(y1r * y2i - y1i * y2r, y1r * y2r + y1i * y2i) / M_PI);
      }
    }
  }
  free(p);
  return best >= 0 ? 0 : -1;
}

void or_cfo_correct(const float *x, uint32_t n, float cfo, uint32_t N, float *y) {
  for (uint32_t i = 0; i < n; i++) {
    const double ph = -2.0 * M_PI * (double)cfo * (double)i / (double)N;
    const double c = cos(ph), s = sin(ph), a = x[2 * i], b = x[2 * i + 1];
    y[2 * i] = (float)(a * c - b * s);
    y[2 * i + 1] = (float)(a * s + b * c);
  }
}

/* 62-bin DFT of one symbol's useful part (N samples) */
static void bins62(const float *sym, uint32_t nof_prb, uint32_t N, double *Y) {
  for (uint32_t m = 0; m < 62; m++) {
    const uint32_t b = sync_bin(m, nof_prb, N);
    double re = 0, im = 0;
    for (uint32_t n = 0; n < N; n++) {
      const double ph = -2.0 * M_PI * (double)((uint64_t)b * n % N) / (double)N, c = cos(ph), s = sin(ph);
      re += sym[2 * n] * c - sym[2 * n + 1] * s;
      im += sym[2 * n] * s + sym[2 * n + 1] * c;
    }
    Y[2 * m] = re; Y[2 * m + 1] = im;
  }
}

int or_sss_detect(const float *sf_iq, uint32_t nof_prb, uint32_t nid2, uint32_t *nid1, uint32_t *sf5, float *score) {
  const uint32_t N = (uint32_t)or_symbol_sz(nof_prb);
  double Y[124], P[124];
  bins62(sf_iq + 2 * sym_off(N, 5), nof_prb, N, Y);
  bins62(sf_iq + 2 * sym_off(N, 6), nof_prb, N, P);
  float dp[124], ds[62];
  or_pss_seq(nid2, dp);
  double H[124];
  for (int m = 0; m < 62; m++) {   /* H = P / d_pss = P conj(d_pss) (|d_pss| = 1) */
    H[2 * m] = P[2 * m] * dp[2 * m] + P[2 * m + 1] * dp[2 * m + 1];
    H[2 * m + 1] = P[2 * m + 1] * dp[2 * m] - P[2 * m] * dp[2 * m + 1];
  }
  double best = -1e300;
  for (uint32_t h = 0; h < 336; h++) {
    or_sss_seq(h >> 1, nid2, h & 1, ds);
    double s = 0;
    for (int m = 0; m < 62; m++) s += (H[2 * m] * Y[2 * m] + H[2 * m + 1] * Y[2 * m + 1]) * ds[m];   /* Re conj(H) Y d */
    if (s > best) { best = s; *nid1 = h >> 1; *sf5 = h & 1; }
  }
  if (score) *score = (float)best;
  return 0;
}
