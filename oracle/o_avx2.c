/*
 * o_avx2.c -- AVX2 int16 max-log-MAP turbo decoder, TWO code blocks per __m256i (TEST / BENCH INFRASTRUCTURE
 * ONLY: the CPU baseline bench.py times when the host has AVX2; SURVEY.md 7 step 1 asks for an "SSE4.1/AVX2"
 * decoder in srsLTE's SSE design).
 *
 * The SSE4.1 decoder (o_simd.c) keeps the eight int16 state metrics of ONE code block in a __m128i.  Here the two
 * 128-bit lanes of a __m256i carry two code blocks of equal K (lane 0 = block A, lane 1 = block B): every
 * AVX2 shuffle (vpshufb), blend, add and max works within a 128-bit lane, so the trellis permutations, branch
 * metrics and normalisations of o_simd.c apply to both blocks at once with the same per-lane constants.  The
 * scalar parts (interleaving, extrinsic update, decisions, CRC) run per block.  The arithmetic is o_simd.c's
 * operation for operation -- saturating int16 adds (never saturating on a reachable metric inside or_decode_cb16's
 * bounds), exact horizontal maxima, wrapping int16 LLR differences -- so each block's decisions, iteration count
 * and CRC verdict equal or_decode_cb16's (tests/test_oracle.py test_avx2_*).  Per-block early stop: the pair
 * iterates while either block is undecided; a block that stopped keeps the outputs of its last iteration.
 *
 * The functions carry __attribute__((target("avx2"))) (the library is built for SSE4.1 hosts); callers check
 * or_avx2_available() first.
 */
#include "oracle.h"
#include <immintrin.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

void or_trellis(int s, int u, int *next, int *z);

#define AVX2 __attribute__((target("avx2")))

int or_avx2_available(void) {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx2") ? 1 : 0;
}

/* state of one thread: both blocks' streams interleaved as int16 pairs (element 2k = block A, 2k + 1 = block B) */
struct or_avx2_tdec {
  uint32_t K_tab;
  uint32_t pi[OR_TCOD_MAX_K];
  int16_t q[2][3 * OR_TCOD_MAX_K + 12];
  int16_t qs[2 * (OR_TCOD_MAX_K + 8)], xs[2 * (OR_TCOD_MAX_K + 8)], xp1[2 * (OR_TCOD_MAX_K + 8)],
      xp2[2 * (OR_TCOD_MAX_K + 8)], w[2 * (OR_TCOD_MAX_K + 8)], llr1[2 * (OR_TCOD_MAX_K + 8)],
      llr2[2 * (OR_TCOD_MAX_K + 8)];
  uint8_t bits[2][OR_TCOD_MAX_K];
  uint8_t bytes[OR_TCOD_MAX_K / 8 + 1];
  __m256i beta[OR_TCOD_MAX_K + 4];
};

static uint32_t A8[256], B8[256];
/* the trellis constants of o_simd.c, as 128-bit patterns (broadcast to both lanes at use) */
static uint8_t SN0b[16], SN1b[16], SAb[16], SBb[16], BC0b[16], BCPb[32], SWb[16];
static int16_t MP0h[8], MP1h[8], MAh[8], MBh[8];
static void __attribute__((constructor)) avx2_init(void) {
  for (uint32_t b = 0; b < 256; b++) {
    uint32_t ra = b << 16, rb = b << 16;
    for (int i = 0; i < 8; i++) {
      ra = (ra & 0x800000u) ? ((ra << 1) ^ 0x864CFBu) : (ra << 1);
      rb = (rb & 0x800000u) ? ((rb << 1) ^ 0x800063u) : (rb << 1);
    }
    A8[b] = ra & 0xFFFFFFu;
    B8[b] = rb & 0xFFFFFFu;
  }
  int cnt[8] = {0}, ps[8][2], pu[8][2];
  for (int s = 0; s < 8; s++)
    for (int u = 0; u < 2; u++) {
      int n, z;
      or_trellis(s, u, &n, &z);
      uint8_t *sn = u ? SN1b : SN0b;
      sn[2 * s] = (uint8_t)(2 * n); sn[2 * s + 1] = (uint8_t)(2 * n + 1);
      (u ? MP1h : MP0h)[s] = z ? -1 : 0;
      ps[n][cnt[n]] = s; pu[n][cnt[n]] = u; cnt[n]++;
    }
  for (int s = 0; s < 8; s++) {
    SAb[2 * s] = (uint8_t)(2 * ps[s][0]); SAb[2 * s + 1] = (uint8_t)(2 * ps[s][0] + 1);
    SBb[2 * s] = (uint8_t)(2 * ps[s][1]); SBb[2 * s + 1] = (uint8_t)(2 * ps[s][1] + 1);
    MAh[s] = pu[s][0] ? -1 : 0; MBh[s] = pu[s][1] ? -1 : 0;
    BC0b[2 * s] = 0; BC0b[2 * s + 1] = 1;
    /* pair broadcast: lane 0 takes int16 0 (block A) of the dword, lane 1 int16 1 (block B) */
    BCPb[2 * s] = 0; BCPb[2 * s + 1] = 1; BCPb[16 + 2 * s] = 2; BCPb[16 + 2 * s + 1] = 3;
    /* swap adjacent int16 */
    SWb[2 * s] = (uint8_t)(2 * (s ^ 1)); SWb[2 * s + 1] = (uint8_t)(2 * (s ^ 1) + 1);
  }
}

AVX2 static inline __m256i b128(const void *p) { return _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)p)); }

typedef struct { __m256i SN0, SN1, SA, SB, BC0, BCP, SW, MP0, MP1, MA, MB, INIT; } consts_t;
AVX2 static consts_t load_consts(void) {
  consts_t c;
  c.SN0 = b128(SN0b); c.SN1 = b128(SN1b); c.SA = b128(SAb); c.SB = b128(SBb); c.BC0 = b128(BC0b);
  c.BCP = _mm256_loadu_si256((const __m256i *)BCPb); c.SW = b128(SWb);
  c.MP0 = b128(MP0h); c.MP1 = b128(MP1h); c.MA = b128(MAh); c.MB = b128(MBh);
  c.INIT = _mm256_broadcastsi128_si256(_mm_insert_epi16(_mm_set1_epi16(-32768), 0, 0));
  return c;
}

/* the pair (A, B) of int16 at element pair k broadcast: lane 0 = 8 x A, lane 1 = 8 x B */
AVX2 static inline __m256i bpair(const int16_t *v, uint32_t k, __m256i BCP) {
  int32_t d;
  memcpy(&d, v + 2 * k, 4);
  return _mm256_shuffle_epi8(_mm256_set1_epi32(d), BCP);
}

/* one constituent decoder for both blocks (o_simd.c map_sse per lane) */
AVX2 static void map_avx2(const consts_t *c, const int16_t *xs, const int16_t *xp, int16_t *out, uint32_t K,
                          __m256i *beta) {
  beta[K + 3] = c->INIT;
  for (int k = (int)K + 2; k >= 1; k--) {
    const __m256i vxs = bpair(xs, (uint32_t)k, c->BCP), vxp = bpair(xp, (uint32_t)k, c->BCP);
    const __m256i g0 = _mm256_and_si256(vxp, c->MP0), g1 = _mm256_adds_epi16(vxs, _mm256_and_si256(vxp, c->MP1));
    const __m256i bn = beta[k + 1];
    const __m256i m = _mm256_max_epi16(_mm256_adds_epi16(_mm256_shuffle_epi8(bn, c->SN0), g0),
                                       _mm256_adds_epi16(_mm256_shuffle_epi8(bn, c->SN1), g1));
    beta[k] = _mm256_subs_epi16(m, _mm256_shuffle_epi8(m, c->BC0));
  }
  __m256i a = c->INIT;
  for (uint32_t k = 0; k < K; k++) {
    const __m256i vxs = bpair(xs, k, c->BCP), vxp = bpair(xp, k, c->BCP);
    const __m256i g0 = _mm256_and_si256(vxp, c->MP0), g1 = _mm256_adds_epi16(vxs, _mm256_and_si256(vxp, c->MP1));
    const __m256i bn = beta[k + 1];
    const __m256i c0 = _mm256_adds_epi16(a, g0), c1 = _mm256_adds_epi16(a, g1);
    const __m256i x0 = _mm256_adds_epi16(c0, _mm256_shuffle_epi8(bn, c->SN0));
    const __m256i x1 = _mm256_adds_epi16(c1, _mm256_shuffle_epi8(bn, c->SN1));
    /* exact maxima over the 8 states of x0 and of x1, per lane: int16 0 = max x0, int16 4 = max x1 */
    __m256i t = _mm256_max_epi16(_mm256_unpacklo_epi64(x0, x1), _mm256_unpackhi_epi64(x0, x1));
    t = _mm256_max_epi16(t, _mm256_shuffle_epi32(t, _MM_SHUFFLE(2, 3, 0, 1)));
    t = _mm256_max_epi16(t, _mm256_shuffle_epi8(t, c->SW));
    /* m1 - m0 as a wrapping int16 difference (o_simd.c: (int16_t)(m1 - m0)) */
    const __m256i d = _mm256_sub_epi16(_mm256_srli_si256(t, 8), t);
    out[2 * k] = (int16_t)_mm256_extract_epi16(d, 0);
    out[2 * k + 1] = (int16_t)_mm256_extract_epi16(d, 8);
    const __m256i A = _mm256_blendv_epi8(_mm256_shuffle_epi8(c0, c->SA), _mm256_shuffle_epi8(c1, c->SA), c->MA);
    const __m256i B = _mm256_blendv_epi8(_mm256_shuffle_epi8(c0, c->SB), _mm256_shuffle_epi8(c1, c->SB), c->MB);
    const __m256i m = _mm256_max_epi16(A, B);
    a = _mm256_subs_epi16(m, _mm256_shuffle_epi8(m, c->BC0));
  }
}

static inline int16_t clamp16(int32_t x, int32_t c) { return (int16_t)(x < -c ? -c : (x > c ? c : x)); }
/* q(x) = clamp(rint(32 x), +-511): cvtps rounds to nearest-even like rintf (o_simd.c quantize) */
AVX2 static void quantize(const float *in, int16_t *q, uint32_t n) {
  const __m256 S = _mm256_set1_ps(OR_I16_SCALE), LO = _mm256_set1_ps(-(float)OR_I16_CI),
               HI = _mm256_set1_ps((float)OR_I16_CI);
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8) {
    const __m256 a = _mm256_min_ps(_mm256_max_ps(_mm256_mul_ps(_mm256_loadu_ps(in + i), S), LO), HI);
    const __m256i v = _mm256_cvtps_epi32(a);
    _mm_storeu_si128((__m128i *)(q + i), _mm_packs_epi32(_mm256_castsi256_si128(v), _mm256_extracti128_si256(v, 1)));
  }
  for (; i < n; i++) q[i] = (int16_t)or_q16(in[i]);
}
static uint32_t crc24_bytes(const uint8_t *p, uint32_t n, const uint32_t *T) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < n; i++) r = ((r << 8) & 0xFFFFFFu) ^ T[((r >> 16) ^ p[i]) & 0xFFu];
  return r;
}

size_t or_avx2_tdec_size(void) { return sizeof(struct or_avx2_tdec) + 64; }
void or_avx2_tdec_init(void *state) {
  struct or_avx2_tdec *h = (struct or_avx2_tdec *)(((uintptr_t)state + 63) & ~(uintptr_t)63);
  h->K_tab = 0;
}

/* Decodes blocks A (inA) and B (inB) of size K together (inB == NULL: A alone, the second lane decodes a copy of A
 * whose outputs are dropped).  Per block: decisions (1 byte per bit), CRC verdict, iterations used. */
AVX2 int or_avx2_decode_pair(void *state, const float *inA, const float *inB, uint32_t K, uint32_t max_its,
                             int early_stop, int crc_type, uint8_t *bitsA, uint8_t *bitsB, int *okA, int *okB,
                             int *itsA, int *itsB) {
  struct or_avx2_tdec *h = (struct or_avx2_tdec *)(((uintptr_t)state + 63) & ~(uintptr_t)63);
  if (K > OR_TCOD_MAX_K || K % 8) return -1;
  if (h->K_tab != K) {
    if (or_qpp(K, h->pi)) return -1;
    h->K_tab = K;
  }
  const consts_t c = load_consts();
  const int two = inB != NULL;
  quantize(inA, h->q[0], 3 * K + 12);
  if (two) quantize(inB, h->q[1], 3 * K + 12);
  else memcpy(h->q[1], h->q[0], sizeof(int16_t) * (3 * K + 12));
  for (int b = 0; b < 2; b++) {
    const int16_t *q = h->q[b];
    for (uint32_t k = 0; k < K; k++) {
      h->qs[2 * k + b] = q[3 * k]; h->xp1[2 * k + b] = q[3 * k + 1]; h->xp2[2 * k + b] = q[3 * k + 2];
      h->w[2 * k + b] = 0;
    }
    for (uint32_t j = 0; j < 3; j++) {
      h->xp1[2 * (K + j) + b] = q[3 * K + 2 * j + 1];
      h->xp2[2 * (K + j) + b] = q[3 * K + 7 + 2 * j];
    }
  }
  const uint32_t *T = crc_type ? A8 : B8;
  uint8_t *out_bits[2] = {bitsA, bitsB};
  int ok[2] = {0, 0}, its[2] = {0, 0}, active = two ? 3 : 1;
  for (int it = 1; it <= (int)max_its && active; it++) {
    /* DEC1 systematic + extrinsic (wrapping int16 add, as o_simd.c) */
    for (uint32_t k = 0; k < 2 * K; k += 16)
      _mm256_storeu_si256((__m256i *)(h->xs + k), _mm256_add_epi16(_mm256_loadu_si256((const __m256i *)(h->qs + k)),
                                                                   _mm256_loadu_si256((const __m256i *)(h->w + k))));
    for (int b = 0; b < 2; b++)
      for (uint32_t j = 0; j < 3; j++) h->xs[2 * (K + j) + b] = h->q[b][3 * K + 2 * j];
    map_avx2(&c, h->xs, h->xp1, h->llr1, K, h->beta);
    for (uint32_t k = 0; k < K; k++) {
      const uint32_t p = h->pi[k];
      h->xs[2 * k] = clamp16((int32_t)h->llr1[2 * p] - h->w[2 * p], OR_I16_CX);
      h->xs[2 * k + 1] = clamp16((int32_t)h->llr1[2 * p + 1] - h->w[2 * p + 1], OR_I16_CX);
    }
    for (int b = 0; b < 2; b++)
      for (uint32_t j = 0; j < 3; j++) h->xs[2 * (K + j) + b] = h->q[b][3 * K + 6 + 2 * j];
    map_avx2(&c, h->xs, h->xp2, h->llr2, K, h->beta);
    for (uint32_t k = 0; k < K; k++) {
      const uint32_t p = h->pi[k];
      h->w[2 * p] = clamp16((int32_t)h->llr2[2 * k] - h->xs[2 * k], OR_I16_CW);
      h->w[2 * p + 1] = clamp16((int32_t)h->llr2[2 * k + 1] - h->xs[2 * k + 1], OR_I16_CW);
      h->bits[0][p] = h->llr2[2 * k] > 0 ? 1 : 0;
      h->bits[1][p] = h->llr2[2 * k + 1] > 0 ? 1 : 0;
    }
    for (int b = 0; b < 2; b++) {
      if (!((active >> b) & 1)) continue;
      const uint8_t *bb = h->bits[b];
      for (uint32_t i = 0; i < K / 8; i++) {
        const uint8_t *x = bb + 8 * i;
        h->bytes[i] = (uint8_t)(x[0] << 7 | x[1] << 6 | x[2] << 5 | x[3] << 4 | x[4] << 3 | x[5] << 2 | x[6] << 1 | x[7]);
      }
      ok[b] = crc24_bytes(h->bytes, K / 8, T) == 0;
      its[b] = it;
      memcpy(out_bits[b], bb, K);
      if ((early_stop && ok[b]) || it == (int)max_its) active &= ~(1 << b);
    }
  }
  *okA = ok[0]; *itsA = its[0];
  if (two) { *okB = ok[1]; *itsB = its[1]; }
  return 0;
}

/* ---- batch of equal-K code blocks over nthreads (config 1's CPU baseline), pairs per work item ------------- */
typedef struct {
  const float *in; uint32_t stride, K, max_its, crc_type; int early_stop;
  uint8_t *bits; uint32_t *its; uint8_t *ok;
  uint32_t n, next; pthread_mutex_t mu;
} batch_job_t;

static void *batch_worker(void *arg) {
  batch_job_t *j = (batch_job_t *)arg;
  void *st = malloc(or_avx2_tdec_size());
  or_avx2_tdec_init(st);
  for (;;) {
    pthread_mutex_lock(&j->mu);
    uint32_t i = j->next;
    j->next += 2;
    pthread_mutex_unlock(&j->mu);
    if (i >= j->n) break;
    const int two = i + 1 < j->n;
    int okA, okB = 0, itsA, itsB = 0;
    or_avx2_decode_pair(st, j->in + (size_t)i * j->stride, two ? j->in + (size_t)(i + 1) * j->stride : NULL, j->K,
                        j->max_its, j->early_stop, (int)j->crc_type, j->bits + (size_t)i * j->K,
                        two ? j->bits + (size_t)(i + 1) * j->K : NULL, &okA, &okB, &itsA, &itsB);
    j->its[i] = (uint32_t)itsA; j->ok[i] = (uint8_t)okA;
    if (two) { j->its[i + 1] = (uint32_t)itsB; j->ok[i + 1] = (uint8_t)okB; }
  }
  free(st);
  return NULL;
}

int or_avx2_decode_batch(const float *in, uint32_t stride, uint32_t n, uint32_t K, uint32_t max_its, int early_stop,
                         int crc_type, uint8_t *bits, uint32_t *its, uint8_t *ok, uint32_t nthreads) {
  if (!or_avx2_available()) return -1;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  batch_job_t j = {in, stride, K, max_its, (uint32_t)crc_type, early_stop, bits, its, ok, n, 0,
                   PTHREAD_MUTEX_INITIALIZER};
  pthread_t th[256];
  for (uint32_t t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &j);
  for (uint32_t t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  return 0;
}
