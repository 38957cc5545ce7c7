/*
 * o_fft.c -- double-precision DFT for the oracle (TEST INFRASTRUCTURE ONLY).
 * Restates the FFTW plan srsLTE's srslte_ofdm_rx_sf uses: sizes
 * N = 2^a (128..2048) and 1536 = 3 * 512.  Forward: X[b] = sum_n x[n] e^{-j 2 pi b n / N}
 * (unnormalised); inverse: x[n] = sum_b X[b] e^{+j 2 pi b n / N} (unnormalised).
 */
#include "oracle.h"
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* Twiddles of every radix-2 stage (len = 2 .. 2048), both signs, computed once with exactly the expression
 * the butterfly loop used to evaluate per call -- cos / sin(sgn 2 pi k / len) -- so the transform is
 * bit-identical to the per-call form, about 4x faster (the CPU baseline runs this chain).  Entry (len, k)
 * at index len / 2 - 1 + k. */
#define TW_NMAX 2048
static double tw_re[2][TW_NMAX], tw_im[2][TW_NMAX];
static pthread_once_t tw_once = PTHREAD_ONCE_INIT;
static void tw_init(void) {
  for (int inv = 0; inv < 2; inv++) {
    const double sgn = inv ? 1.0 : -1.0;
    for (int len = 2; len <= TW_NMAX; len <<= 1)
      for (int k = 0; k < len / 2; k++) {
        double ang = sgn * 2.0 * M_PI * k / len;
        tw_re[inv][len / 2 - 1 + k] = cos(ang);
        tw_im[inv][len / 2 - 1 + k] = sin(ang);
      }
  }
}

static void fft_pow2(double *a, int N, int inverse) {
  /* iterative radix-2, bit reversal */
  for (int i = 1, j = 0; i < N; i++) {
    int bit = N >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) {
      double tr = a[2 * i], ti = a[2 * i + 1];
      a[2 * i] = a[2 * j]; a[2 * i + 1] = a[2 * j + 1];
      a[2 * j] = tr; a[2 * j + 1] = ti;
    }
  }
  pthread_once(&tw_once, tw_init);
  const double *twr = tw_re[inverse ? 1 : 0], *twi = tw_im[inverse ? 1 : 0];
  for (int len = 2; len <= N; len <<= 1) {
    int h = len >> 1;
    for (int k = 0; k < h; k++) {
      const double wr = twr[h - 1 + k], wi = twi[h - 1 + k];
      for (int i = k; i < N; i += len) {
        double *u = a + 2 * i, *v = a + 2 * (i + h);
        double vr = v[0] * wr - v[1] * wi, vi = v[0] * wi + v[1] * wr;
        v[0] = u[0] - vr; v[1] = u[1] - vi;
        u[0] += vr; u[1] += vi;
      }
    }
  }
}

void or_dft(const double *in, double *out, int N, int inverse) {
  if (N > TW_NMAX) abort();   /* LTE: N <= 2048 */
  if ((N & (N - 1)) == 0) {
    memcpy(out, in, sizeof(double) * 2 * N);
    fft_pow2(out, N, inverse);
    return;
  }
  /* N = 3 M, M power of two: X[k + M t] = sum_{j<3} W_N^{j(k+Mt)} Y_j[k] */
  int M = N / 3;
  double *y = (double *)malloc(sizeof(double) * 2 * N);
  for (int j = 0; j < 3; j++) {
    for (int q = 0; q < M; q++) {
      y[2 * (j * M + q)] = in[2 * (3 * q + j)];
      y[2 * (j * M + q) + 1] = in[2 * (3 * q + j) + 1];
    }
    fft_pow2(y + 2 * j * M, M, inverse);
  }
  const double sgn = inverse ? 1.0 : -1.0;
  for (int k = 0; k < N; k++) {
    double sr = 0, si = 0;
    int kk = k % M;
    for (int j = 0; j < 3; j++) {
      double ang = sgn * 2.0 * M_PI * (double)((long)j * k % N) / N;
      double wr = cos(ang), wi = sin(ang);
      double yr = y[2 * (j * M + kk)], yi = y[2 * (j * M + kk) + 1];
      sr += yr * wr - yi * wi;
      si += yr * wi + yi * wr;
    }
    out[2 * k] = sr; out[2 * k + 1] = si;
  }
  free(y);
}
