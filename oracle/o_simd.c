/*
 * o_simd.c -- SSE4.1 int16 max-log-MAP turbo decoder (TEST / BENCH INFRASTRUCTURE ONLY: it is the
 * CPU baseline bench.py times and a second, independently written check of or_decode_cb16).
 *
 * Mirrors the design of srsLTE's SSE decoder (srslte_tdec_sse, selected when CMake finds SSE4.1:
 * reference CMakeLists.txt:58-68 adds -DLV_HAVE_SSE): the eight int16
 * state metrics of one trellis step live in one __m128i, the state permutations of the RSC
 * trellis are pshufb shuffles, branch metrics are broadcast + mask, additions saturate.  The
 * arithmetic contract is or_decode_cb16's (o_fec.c "int16" section): inside its bounds no int16
 * operation saturates on a reachable metric, so the results are bit-identical to the int32
 * restatement; unreachable states start at -32768 and can never win a max.
 *
 * One code block per call; callers parallelise over code blocks / subframes with threads
 * (or_simd_decode_batch here, a thread pool over or_decode_subframe in bench.py).
 */
#include "oracle.h"
#include <smmintrin.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

void or_trellis(int s, int u, int *next, int *z);

/* Decoder state of one thread.  The QPP table of the last K stays valid across calls (K_tab), so a TB's code
 * blocks (and a batch of equal-K blocks) build it once; the three input streams are de-interleaved once per
 * code block (qs / qp1 / qp2) instead of per iteration. */
struct or_simd_tdec {
  uint32_t K, K_tab;
  uint32_t pi[OR_TCOD_MAX_K];
  int16_t  w[OR_TCOD_MAX_K], llr1[OR_TCOD_MAX_K], llr2[OR_TCOD_MAX_K];
  int16_t  xs[OR_TCOD_MAX_K + 3], xp[OR_TCOD_MAX_K + 3], xp2[OR_TCOD_MAX_K + 3];
  int16_t  qs[OR_TCOD_MAX_K + 8];
  int16_t  q[3 * OR_TCOD_MAX_K + 12];
  uint8_t  bytes[OR_TCOD_MAX_K / 8 + 1];
  __m128i  beta[OR_TCOD_MAX_K + 4];
};

/* byte-wise CRC24A / CRC24B tables (register of a message byte; the bit-serial or_crc24a/b of o_common.c
 * over the same bits gives the same remainder) */
static uint32_t CRC_A8[256], CRC_B8[256];
static void __attribute__((constructor)) crc_tables_init(void) {
  for (uint32_t b = 0; b < 256; b++) {
    uint32_t ra = b << 16, rb = b << 16;
    for (int i = 0; i < 8; i++) {
      ra = (ra & 0x800000u) ? ((ra << 1) ^ 0x864CFBu) : (ra << 1);
      rb = (rb & 0x800000u) ? ((rb << 1) ^ 0x800063u) : (rb << 1);
    }
    CRC_A8[b] = ra & 0xFFFFFFu;
    CRC_B8[b] = rb & 0xFFFFFFu;
  }
}
static uint32_t crc24_bytes(const uint8_t *p, uint32_t n, const uint32_t *T) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < n; i++) r = ((r << 8) & 0xFFFFFFu) ^ T[((r >> 16) ^ p[i]) & 0xFFu];
  return r;
}

/* shuffle controls and masks derived from the trellis (see o_fec.c header) */
static __m128i SN0, SN1, MP0, MP1, SA, SB, MA, MB, BC0;
static void __attribute__((constructor)) simd_init(void) {
  uint8_t sn0[16], sn1[16], sa[16], sb[16], bc0[16];
  int16_t mp0[8], mp1[8], ma[8], mb[8];
  int cnt[8] = {0}, ps[8][2], pu[8][2];
  for (int s = 0; s < 8; s++)
    for (int u = 0; u < 2; u++) {
      int n, z;
      or_trellis(s, u, &n, &z);
      uint8_t *sn = u ? sn1 : sn0;
      sn[2 * s] = (uint8_t)(2 * n); sn[2 * s + 1] = (uint8_t)(2 * n + 1);
      (u ? mp1 : mp0)[s] = z ? -1 : 0;
      ps[n][cnt[n]] = s; pu[n][cnt[n]] = u; cnt[n]++;
    }
  for (int s = 0; s < 8; s++) {
    sa[2 * s] = (uint8_t)(2 * ps[s][0]); sa[2 * s + 1] = (uint8_t)(2 * ps[s][0] + 1);
    sb[2 * s] = (uint8_t)(2 * ps[s][1]); sb[2 * s + 1] = (uint8_t)(2 * ps[s][1] + 1);
    ma[s] = pu[s][0] ? -1 : 0; mb[s] = pu[s][1] ? -1 : 0;
    bc0[2 * s] = 0; bc0[2 * s + 1] = 1;
  }
  SN0 = _mm_loadu_si128((const __m128i *)sn0); SN1 = _mm_loadu_si128((const __m128i *)sn1);
  SA = _mm_loadu_si128((const __m128i *)sa);   SB = _mm_loadu_si128((const __m128i *)sb);
  BC0 = _mm_loadu_si128((const __m128i *)bc0);
  MP0 = _mm_loadu_si128((const __m128i *)mp0); MP1 = _mm_loadu_si128((const __m128i *)mp1);
  MA = _mm_loadu_si128((const __m128i *)ma);   MB = _mm_loadu_si128((const __m128i *)mb);
}

/* signed horizontal max of 8 int16 via phminposuw on 0x7fff - x */
static inline int32_t hmax16(__m128i x) {
  const __m128i K7 = _mm_set1_epi16(0x7fff);
  return 0x7fff - (int32_t)(uint16_t)_mm_cvtsi128_si32(_mm_minpos_epu16(_mm_sub_epi16(K7, x)));
}

static void map_sse(const int16_t *xs, const int16_t *xp, int16_t *out, uint32_t K, __m128i *beta) {
  const __m128i NEGV = _mm_set1_epi16(-32768);
  beta[K + 3] = _mm_insert_epi16(NEGV, 0, 0);
  for (int k = (int)K + 2; k >= 1; k--) {
    __m128i vxs = _mm_set1_epi16(xs[k]), vxp = _mm_set1_epi16(xp[k]);
    __m128i g0 = _mm_and_si128(vxp, MP0), g1 = _mm_adds_epi16(vxs, _mm_and_si128(vxp, MP1));
    __m128i bn = beta[k + 1];
    __m128i m = _mm_max_epi16(_mm_adds_epi16(_mm_shuffle_epi8(bn, SN0), g0),
                              _mm_adds_epi16(_mm_shuffle_epi8(bn, SN1), g1));
    beta[k] = _mm_subs_epi16(m, _mm_shuffle_epi8(m, BC0));
  }
  __m128i a = _mm_insert_epi16(NEGV, 0, 0);
  for (uint32_t k = 0; k < K; k++) {
    __m128i vxs = _mm_set1_epi16(xs[k]), vxp = _mm_set1_epi16(xp[k]);
    __m128i g0 = _mm_and_si128(vxp, MP0), g1 = _mm_adds_epi16(vxs, _mm_and_si128(vxp, MP1));
    __m128i bn = beta[k + 1];
    __m128i c0 = _mm_adds_epi16(a, g0), c1 = _mm_adds_epi16(a, g1);
    int32_t m0 = hmax16(_mm_adds_epi16(c0, _mm_shuffle_epi8(bn, SN0)));
    int32_t m1 = hmax16(_mm_adds_epi16(c1, _mm_shuffle_epi8(bn, SN1)));
    out[k] = (int16_t)(m1 - m0);
    __m128i A = _mm_blendv_epi8(_mm_shuffle_epi8(c0, SA), _mm_shuffle_epi8(c1, SA), MA);
    __m128i B = _mm_blendv_epi8(_mm_shuffle_epi8(c0, SB), _mm_shuffle_epi8(c1, SB), MB);
    __m128i m = _mm_max_epi16(A, B);
    a = _mm_subs_epi16(m, _mm_shuffle_epi8(m, BC0));
  }
}

static inline int16_t clamp16(int32_t x, int32_t c) { return (int16_t)(x < -c ? -c : (x > c ? c : x)); }

/* q(x) = clamp(rint(32 x), +-511) for n floats (cvtps rounds to nearest-even like rintf) */
static void quantize(const float *in, int16_t *q, uint32_t n) {
  const __m128 S = _mm_set1_ps(OR_I16_SCALE), LO = _mm_set1_ps(-(float)OR_I16_CI), HI = _mm_set1_ps((float)OR_I16_CI);
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8) {
    __m128 a = _mm_min_ps(_mm_max_ps(_mm_mul_ps(_mm_loadu_ps(in + i), S), LO), HI);
    __m128 b = _mm_min_ps(_mm_max_ps(_mm_mul_ps(_mm_loadu_ps(in + i + 4), S), LO), HI);
    _mm_storeu_si128((__m128i *)(q + i), _mm_packs_epi32(_mm_cvtps_epi32(a), _mm_cvtps_epi32(b)));
  }
  for (; i < n; i++) q[i] = (int16_t)or_q16(in[i]);
}

size_t or_simd_tdec_size(void) { return sizeof(struct or_simd_tdec) + 64; }
/* a fresh state (the QPP-table cache starts empty) */
void or_simd_tdec_init(void *state) {
  struct or_simd_tdec *h = (struct or_simd_tdec *)(((uintptr_t)state + 63) & ~(uintptr_t)63);
  h->K_tab = 0;
}

int or_simd_decode_cb(void *state, const float *in, uint32_t K, uint32_t max_its, int early_stop, int crc_type,
                      uint8_t *bits, int *crc_ok) {
  struct or_simd_tdec *h = (struct or_simd_tdec *)(((uintptr_t)state + 63) & ~(uintptr_t)63);
  if (K > OR_TCOD_MAX_K || K % 8) return -1;
  if (h->K_tab != K) {
    if (or_qpp(K, h->pi)) return -1;
    h->K_tab = K;
  }
  h->K = K;
  memset(h->w, 0, sizeof(int16_t) * K);
  quantize(in, h->q, 3 * K + 12);
  const int16_t *q = h->q;
  /* de-interleave once: systematic, parity 1 (DEC1's xp) and parity 2 (DEC2's xp), tails included */
  for (uint32_t k = 0; k < K; k++) { h->qs[k] = q[3 * k]; h->xp[k] = q[3 * k + 1]; h->xp2[k] = q[3 * k + 2]; }
  for (uint32_t j = 0; j < 3; j++) {
    h->xp[K + j] = q[3 * K + 2 * j + 1];
    h->xp2[K + j] = q[3 * K + 7 + 2 * j];
  }
  const uint32_t *T = crc_type ? CRC_A8 : CRC_B8;
  uint32_t its = 0;
  int ok = 0;
  do {
    /* DEC1 systematic + extrinsic, 8 at a time (wrapping add as the scalar int16 cast; no overflow in bounds) */
    for (uint32_t k = 0; k < K; k += 8)
      _mm_storeu_si128((__m128i *)(h->xs + k), _mm_add_epi16(_mm_loadu_si128((const __m128i *)(h->qs + k)),
                                                            _mm_loadu_si128((const __m128i *)(h->w + k))));
    for (uint32_t j = 0; j < 3; j++) h->xs[K + j] = q[3 * K + 2 * j];
    map_sse(h->xs, h->xp, h->llr1, K, h->beta);
    for (uint32_t k = 0; k < K; k++) {
      const uint32_t p = h->pi[k];
      h->xs[k] = clamp16((int32_t)h->llr1[p] - h->w[p], OR_I16_CX);
    }
    for (uint32_t j = 0; j < 3; j++) h->xs[K + j] = q[3 * K + 6 + 2 * j];
    map_sse(h->xs, h->xp2, h->llr2, K, h->beta);
    /* extrinsic update and decisions in natural order in one pass */
    for (uint32_t k = 0; k < K; k++) {
      const uint32_t p = h->pi[k];
      h->w[p] = clamp16((int32_t)h->llr2[k] - h->xs[k], OR_I16_CW);
      bits[p] = h->llr2[k] > 0 ? 1 : 0;
    }
    its++;
    for (uint32_t i = 0; i < K / 8; i++) {
      const uint8_t *b = bits + 8 * i;
      h->bytes[i] = (uint8_t)(b[0] << 7 | b[1] << 6 | b[2] << 5 | b[3] << 4 | b[4] << 3 | b[5] << 2 | b[6] << 1 | b[7]);
    }
    ok = crc24_bytes(h->bytes, K / 8, T) == 0;
    if (early_stop && ok) break;
  } while (its < max_its);
  *crc_ok = ok;
  return (int)its;
}

/* ---- batch of equal-K code blocks over nthreads (config 1's CPU baseline) ---------------- */
typedef struct {
  const float *in; uint32_t stride, K, max_its, crc_type; int early_stop;
  uint8_t *bits; uint32_t *its; uint8_t *ok;
  uint32_t n, next; pthread_mutex_t mu;
} batch_job_t;

static void *batch_worker(void *arg) {
  batch_job_t *j = (batch_job_t *)arg;
  void *st = malloc(or_simd_tdec_size());
  or_simd_tdec_init(st);
  for (;;) {
    pthread_mutex_lock(&j->mu);
    uint32_t i = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (i >= j->n) break;
    int ok;
    j->its[i] = (uint32_t)or_simd_decode_cb(st, j->in + (size_t)i * j->stride, j->K, j->max_its, j->early_stop,
                                            (int)j->crc_type, j->bits + (size_t)i * j->K, &ok);
    j->ok[i] = (uint8_t)ok;
  }
  free(st);
  return NULL;
}

int or_simd_decode_batch(const float *in, uint32_t stride, uint32_t n, uint32_t K, uint32_t max_its, int early_stop,
                         int crc_type, uint8_t *bits, uint32_t *its, uint8_t *ok, uint32_t nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  batch_job_t j = {in, stride, K, max_its, (uint32_t)crc_type, early_stop, bits, its, ok, n, 0,
                   PTHREAD_MUTEX_INITIALIZER};
  pthread_t th[256];
  for (uint32_t t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &j);
  for (uint32_t t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  return 0;
}
