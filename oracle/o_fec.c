/*
 * o_fec.c -- turbo code, rate (de)matching and the max-log-MAP decoder (TEST INFRASTRUCTURE ONLY).
 *
 * Restates srsLTE 1.0 srslte_tcod / srslte_rm_turbo_tx / srslte_rm_turbo_rx / srslte_tdec_gen
 * (called through srslte_pdsch_decode_rnti at /root/reference/ue/src/phy/phch_worker.cc:347 and
 * capped by srslte_sch_set_max_noi at phch_worker.cc:88) from 36.212 5.1.3 / 5.1.4.1.
 *
 * Decoder contract (the GPU kernel srsue_amd/csrc/tdec.hip reproduces it operation by
 * operation, so decisions AND extrinsics are bit-identical in fp32):
 *   trellis  state s = 4 s1 + 2 s2 + s3, a = u^s2^s3, z = a^s1^s3, next = 4a + (s>>1)
 *   branch   g(u,z) = u*Lu + z*Lp  with g00 = 0, g01 = Lp, g10 = Lu, g11 = Lu + Lp
 *   beta     beta_{K+3} = [0,-inf..]; k = K+2..1: m_s = max(beta_{k+1}(n(s,0)) + g(0,z(s,0)),
 *                                                       beta_{k+1}(n(s,1)) + g(1,z(s,1)));
 *            beta_k(s) = m_s - m_0            (tail steps use the regular trellis)
 *   alpha    alpha_0 = [0,-inf..]; c(s,u) = alpha_k(s) + g(u,z(s,u));
 *            llr_k = max_s (c(s,1) + beta_{k+1}(n(s,1))) - max_s (c(s,0) + beta_{k+1}(n(s,0)))
 *            alpha_{k+1}(s') = m_{s'} - m_0, m_{s'} = max of the two c into s'
 *   iteration (srsLTE-gen schedule):
 *            DEC1 xs = Ls + w, xp = Lp1 -> llr1;  DEC2 xs = llr1[pi] - w[pi], xp = Lp2 -> llr2;
 *            w[i] = w[i] + (llr2[pi^-1(i)] - llr1[i]);  decision bit_i = llr2[pi^-1(i)] > 0
 *   LLR sign: > 0 means bit 1.  Tail layout (36.212 5.1.3.2.2): 3K..3K+11 =
 *            x_K z_K x_K+1 z_K+1 x_K+2 z_K+2 x'_K z'_K x'_K+1 z'_K+1 x'_K+2 z'_K+2.
 */
#include "oracle.h"
#include <math.h>
#include <string.h>
#include <stdlib.h>

static const uint8_t P_COL[32] = {0,16,8,24,4,20,12,28,2,18,10,26,6,22,14,30,
                                  1,17,9,25,5,21,13,29,3,19,11,27,7,23,15,31};

void or_trellis(int s, int u, int *next, int *z) {
  int s1 = (s >> 2) & 1, s2 = (s >> 1) & 1, s3 = s & 1;
  int a = u ^ s2 ^ s3;
  *z = a ^ s1 ^ s3;
  *next = (a << 2) | (s >> 1);
}

int or_tcod(const uint8_t *in, uint32_t K, uint32_t F, uint8_t *d) {
  static uint32_t pi[OR_TCOD_MAX_K];
  if (or_qpp(K, pi)) return -1;
  int s = 0, n, z;
  uint8_t tail[12];
  for (uint32_t k = 0; k < K; k++) {
    int u = (k < F) ? 0 : (in[k] & 1);
    or_trellis(s, u, &n, &z);
    d[3 * k] = (uint8_t)u; d[3 * k + 1] = (uint8_t)z; s = n;
  }
  for (int j = 0; j < 3; j++) {
    int s1 = (s >> 2) & 1, s2 = (s >> 1) & 1, s3 = s & 1;
    tail[2 * j] = (uint8_t)(s2 ^ s3); tail[2 * j + 1] = (uint8_t)(s1 ^ s3);
    s >>= 1;
  }
  s = 0;
  for (uint32_t k = 0; k < K; k++) {
    uint32_t src = pi[k];
    int u = (src < F) ? 0 : (in[src] & 1);
    or_trellis(s, u, &n, &z);
    d[3 * k + 2] = (uint8_t)z; s = n;
  }
  for (int j = 0; j < 3; j++) {
    int s1 = (s >> 2) & 1, s2 = (s >> 1) & 1, s3 = s & 1;
    tail[6 + 2 * j] = (uint8_t)(s2 ^ s3); tail[6 + 2 * j + 1] = (uint8_t)(s1 ^ s3);
    s >>= 1;
  }
  memcpy(d + 3 * K, tail, 12);
  for (uint32_t k = 0; k < F; k++) { d[3 * k] = 2; d[3 * k + 1] = 2; }
  return 0;
}

/* circular-buffer position -> triplet index of d (or -1 for <NULL>), 36.212 5.1.4.1.1/2 */
static uint32_t build_wmap(uint32_t K, uint32_t F, int32_t *wmap, uint32_t *R_out) {
  uint32_t D = K + 4, R = (D + 31) / 32, KP = 32 * R, ND = KP - D;
  for (uint32_t kk = 0; kk < KP; kk++) {
    uint32_t col = P_COL[kk / R], row = kk % R;
    uint32_t j01 = col + 32 * row, j2 = (col + 32 * row + 1) % KP;
    int32_t s0 = -1, s1 = -1, s2 = -1;
    if (j01 >= ND) { uint32_t k = j01 - ND; if (k >= F) { s0 = (int32_t)(3 * k); s1 = (int32_t)(3 * k + 1); } }
    if (j2 >= ND) { uint32_t k = j2 - ND; s2 = (int32_t)(3 * k + 2); }
    wmap[kk] = s0; wmap[KP + 2 * kk] = s1; wmap[KP + 2 * kk + 1] = s2;
  }
  *R_out = R;
  return 3 * KP;
}

uint32_t or_ncb(uint32_t K) { return 3 * 32 * ((K + 4 + 31) / 32); }

static uint32_t k0_of(uint32_t R, uint32_t Ncb, uint32_t rv) {
  return R * (2 * ((Ncb + 8 * R - 1) / (8 * R)) * rv + 2);
}

int or_rm_tx(const uint8_t *d, uint32_t K, uint32_t E, uint32_t rv, uint8_t *e) {
  /* F is encoded in d as NULL(2) marks; recover it */
  uint32_t F = 0;
  while (F < K && d[3 * F] == 2) F++;
  int32_t *wmap = (int32_t *)malloc(sizeof(int32_t) * or_ncb(K));
  uint32_t R, Ncb = build_wmap(K, F, wmap, &R), k0 = k0_of(R, Ncb, rv);
  for (uint32_t k = 0, j = 0; k < E; j++) {
    int32_t src = wmap[(k0 + j) % Ncb];
    if (src >= 0) e[k++] = d[src];
  }
  free(wmap);
  return 0;
}

int or_rm_rx(const float *e, uint32_t E, uint32_t K, uint32_t F, uint32_t rv, int new_tb, float *sb,
             float *out) {
  int32_t *wmap = (int32_t *)malloc(sizeof(int32_t) * or_ncb(K));
  uint32_t R, Ncb = build_wmap(K, F, wmap, &R), k0 = k0_of(R, Ncb, rv);
  if (new_tb) for (uint32_t p = 0; p < Ncb; p++) sb[p] = 0.0f;   /* == srsLTE reset_tbs (RX_NULL) */
  for (uint32_t k = 0, j = 0; k < E; j++) {
    uint32_t p = (k0 + j) % Ncb;
    if (wmap[p] >= 0) { sb[p] = sb[p] + e[k]; k++; }
  }
  for (uint32_t p = 0; p < Ncb; p++) if (wmap[p] >= 0) out[wmap[p]] = sb[p];
  for (uint32_t k = 0; k < F; k++) { out[3 * k] = OR_FILLER_LLR; out[3 * k + 1] = OR_FILLER_LLR; }
  free(wmap);
  return 0;
}

/* ------------------------------- max-log-MAP ------------------------------------------- */
static int NEXT[8][2], PAR[8][2], PREV_S[8][2], PREV_U[8][2];
static int tables_ready = 0;
static void __attribute__((constructor)) init_tables(void) {
  if (tables_ready) return;
  int cnt[8] = {0};
  for (int s = 0; s < 8; s++)
    for (int u = 0; u < 2; u++) {
      int n, z;
      or_trellis(s, u, &n, &z);
      NEXT[s][u] = n; PAR[s][u] = z;
      PREV_S[n][cnt[n]] = s; PREV_U[n][cnt[n]] = u; cnt[n]++;
    }
  tables_ready = 1;
}

static void map_dec(const float *xs, const float *xp, float *out, uint32_t K, float *beta) {
  const float NINF = -INFINITY;
  for (int s = 0; s < 8; s++) beta[(K + 3) * 8 + s] = s ? NINF : 0.0f;
  for (int k = (int)K + 2; k >= 1; k--) {
    float g[2][2];
    g[0][0] = 0.0f; g[0][1] = xp[k]; g[1][0] = xs[k]; g[1][1] = xs[k] + xp[k];
    const float *bn = beta + (k + 1) * 8;
    float m[8];
    for (int s = 0; s < 8; s++) {
      float b0 = bn[NEXT[s][0]] + g[0][PAR[s][0]];
      float b1 = bn[NEXT[s][1]] + g[1][PAR[s][1]];
      m[s] = fmaxf(b0, b1);
    }
    for (int s = 0; s < 8; s++) beta[k * 8 + s] = m[s] - m[0];
  }
  float alpha[8];
  for (int s = 0; s < 8; s++) alpha[s] = s ? NINF : 0.0f;
  for (uint32_t k = 0; k < K; k++) {
    float g[2][2];
    g[0][0] = 0.0f; g[0][1] = xp[k]; g[1][0] = xs[k]; g[1][1] = xs[k] + xp[k];
    const float *bn = beta + (k + 1) * 8;
    float c[8][2], m0 = NINF, m1 = NINF;
    for (int s = 0; s < 8; s++)
      for (int u = 0; u < 2; u++) {
        c[s][u] = alpha[s] + g[u][PAR[s][u]];
        float t = c[s][u] + bn[NEXT[s][u]];
        if (u) m1 = fmaxf(m1, t); else m0 = fmaxf(m0, t);
      }
    out[k] = m1 - m0;
    float a[8];
    for (int s = 0; s < 8; s++)
      a[s] = fmaxf(c[PREV_S[s][0]][PREV_U[s][0]], c[PREV_S[s][1]][PREV_U[s][1]]);
    for (int s = 0; s < 8; s++) alpha[s] = a[s] - a[0];
  }
}

int or_tdec_reset(or_tdec_t *h, uint32_t K) {
  init_tables();
  if (K > OR_TCOD_MAX_K || or_qpp(K, h->pi)) return -1;
  h->K = K;
  for (uint32_t i = 0; i < K; i++) h->pinv[h->pi[i]] = i;
  memset(h->w, 0, sizeof(float) * K);
  return 0;
}

void or_tdec_iteration(or_tdec_t *h, const float *in) {
  uint32_t K = h->K;
  for (uint32_t k = 0; k < K; k++) { h->xs[k] = in[3 * k] + h->w[k]; h->xp[k] = in[3 * k + 1]; }
  for (uint32_t j = 0; j < 3; j++) { h->xs[K + j] = in[3 * K + 2 * j]; h->xp[K + j] = in[3 * K + 2 * j + 1]; }
  map_dec(h->xs, h->xp, h->llr1, K, h->beta);
  for (uint32_t k = 0; k < K; k++) { h->xs[k] = h->llr1[h->pi[k]] - h->w[h->pi[k]]; h->xp[k] = in[3 * k + 2]; }
  for (uint32_t j = 0; j < 3; j++) { h->xs[K + j] = in[3 * K + 6 + 2 * j]; h->xp[K + j] = in[3 * K + 7 + 2 * j]; }
  map_dec(h->xs, h->xp, h->llr2, K, h->beta);
  for (uint32_t i = 0; i < K; i++) h->w[i] = h->w[i] + (h->llr2[h->pinv[i]] - h->llr1[i]);
}

void or_tdec_decision(const or_tdec_t *h, uint8_t *bits) {
  for (uint32_t i = 0; i < h->K; i++) bits[i] = h->llr2[h->pinv[i]] > 0.0f ? 1 : 0;
}

int or_decode_cb(or_tdec_t *h, const float *in, uint32_t K, uint32_t max_its, int early_stop,
                 int crc_type, uint8_t *bits, int *crc_ok) {
  if (or_tdec_reset(h, K)) return -1;
  uint32_t its = 0;
  int ok = 0;
  do {
    or_tdec_iteration(h, in);
    its++;
    or_tdec_decision(h, bits);
    ok = ((crc_type ? or_crc24a(bits, K) : or_crc24b(bits, K)) == 0);
    if (early_stop && ok) break;
  } while (its < max_its);
  *crc_ok = ok;
  return (int)its;
}

/* ------------------------- int16 ("SSE") max-log-MAP ----------------------------------------
 * Restates the design of srsLTE's SSE turbo decoder (srslte_tdec_sse, built when CMake finds
 * SSE4.1: reference CMakeLists.txt:58-68 -> -DLV_HAVE_SSE; SURVEY.md 8a a5.6: 8 int16 state
 * metrics per __m128i, float LLRs converted to int16 on entry).  The srsLTE source is not in the
 * container, so the fixed-point constants are this build's, chosen so that NO int16 operation
 * can overflow: every value below is an exact integer and the three implementations (this int32
 * code, the SSE4.1 CPU baseline in oracle/o_simd.c with saturating int16 ops, and the GPU kernel
 * computing on integer-valued fp32) produce identical extrinsics, decisions and iteration counts.
 *   input    q(x) = clamp(rint(32 x), +-511)                 (filler -10000 -> -511)
 *   DEC1     xs1 = q(Ls) + w                 (|w| <= 1023, so |xs1| <= 1534: no clamp), xp = q(Lp1)
 *   DEC2     xs2 = clamp(llr1[pi] - w[pi], +-1535),  xp = q(Lp2); tails use q() directly
 *   extr.    w[pi(k)] = clamp(llr2_k - xs2_k, +-1023)   (DEC2's extrinsic; equals the gen
 *            schedule's w + llr2 - llr1 whenever no clamp engages)
 *   decision bit_i = llr2[pi^-1(i)] > 0
 *   trellis  exactly the float recursion above (normalised to state 0; -inf = any value below
 *            -2^15, it can never win a max).  Bounds: R = 1535 + 511 = 2046 bounds the spread of
 *            one step's branch metrics, any state reaches any other in 3 steps, so normalised
 *            alpha/beta lie in +-3R = +-6138, pre-normalisation candidates in +-4R and LLRs in
 *            +-13R = +-26598; llr1 - w and llr2 - xs2 stay inside +-28133: all inside int16.
 */
static int32_t clampi(int32_t x, int32_t c) { return x < -c ? -c : (x > c ? c : x); }

int32_t or_q16(float x) {
  float y = rintf(x * OR_I16_SCALE);
  y = fminf(fmaxf(y, (float)-OR_I16_CI), (float)OR_I16_CI);
  return (int32_t)y;
}

#define NEG16 (-(1 << 28))
static void map_dec16(const int32_t *xs, const int32_t *xp, int32_t *out, uint32_t K, int32_t *beta) {
  for (int s = 0; s < 8; s++) beta[(K + 3) * 8 + s] = s ? NEG16 : 0;
  for (int k = (int)K + 2; k >= 1; k--) {
    int32_t g[2][2] = {{0, xp[k]}, {xs[k], xs[k] + xp[k]}};
    const int32_t *bn = beta + (k + 1) * 8;
    int32_t m[8];
    for (int s = 0; s < 8; s++) {
      int32_t b0 = bn[NEXT[s][0]] + g[0][PAR[s][0]], b1 = bn[NEXT[s][1]] + g[1][PAR[s][1]];
      m[s] = b0 > b1 ? b0 : b1;
    }
    for (int s = 0; s < 8; s++) beta[k * 8 + s] = m[s] - m[0];
  }
  int32_t alpha[8];
  for (int s = 0; s < 8; s++) alpha[s] = s ? NEG16 : 0;
  for (uint32_t k = 0; k < K; k++) {
    int32_t g[2][2] = {{0, xp[k]}, {xs[k], xs[k] + xp[k]}};
    const int32_t *bn = beta + (k + 1) * 8;
    int32_t c[8][2], m0 = INT32_MIN, m1 = INT32_MIN;
    for (int s = 0; s < 8; s++)
      for (int u = 0; u < 2; u++) {
        c[s][u] = alpha[s] + g[u][PAR[s][u]];
        int32_t t = c[s][u] + bn[NEXT[s][u]];
        if (u) { if (t > m1) m1 = t; } else { if (t > m0) m0 = t; }
      }
    out[k] = m1 - m0;
    int32_t a[8];
    for (int s = 0; s < 8; s++) {
      int32_t x0 = c[PREV_S[s][0]][PREV_U[s][0]], x1 = c[PREV_S[s][1]][PREV_U[s][1]];
      a[s] = x0 > x1 ? x0 : x1;
    }
    for (int s = 0; s < 8; s++) alpha[s] = a[s] - a[0];
  }
}

int or_tdec16_reset(or_tdec16_t *h, uint32_t K) {
  init_tables();
  if (K > OR_TCOD_MAX_K || or_qpp(K, h->pi)) return -1;
  h->K = K;
  for (uint32_t i = 0; i < K; i++) h->pinv[h->pi[i]] = i;
  memset(h->w, 0, sizeof(int32_t) * K);
  return 0;
}

void or_tdec16_iteration(or_tdec16_t *h, const float *in) {
  uint32_t K = h->K;
  for (uint32_t k = 0; k < 3 * K + 12; k++) h->q[k] = or_q16(in[k]);
  const int32_t *q = h->q;
  for (uint32_t k = 0; k < K; k++) { h->xs[k] = q[3 * k] + h->w[k]; h->xp[k] = q[3 * k + 1]; }
  for (uint32_t j = 0; j < 3; j++) { h->xs[K + j] = q[3 * K + 2 * j]; h->xp[K + j] = q[3 * K + 2 * j + 1]; }
  map_dec16(h->xs, h->xp, h->llr1, K, h->beta);
  for (uint32_t k = 0; k < K; k++) {
    h->xs[k] = clampi(h->llr1[h->pi[k]] - h->w[h->pi[k]], OR_I16_CX);
    h->xp[k] = q[3 * k + 2];
  }
  for (uint32_t j = 0; j < 3; j++) { h->xs[K + j] = q[3 * K + 6 + 2 * j]; h->xp[K + j] = q[3 * K + 7 + 2 * j]; }
  map_dec16(h->xs, h->xp, h->llr2, K, h->beta);
  for (uint32_t k = 0; k < K; k++) h->w[h->pi[k]] = clampi(h->llr2[k] - h->xs[k], OR_I16_CW);
}

void or_tdec16_decision(const or_tdec16_t *h, uint8_t *bits) {
  for (uint32_t i = 0; i < h->K; i++) bits[i] = h->llr2[h->pinv[i]] > 0 ? 1 : 0;
}

int or_decode_cb16(or_tdec16_t *h, const float *in, uint32_t K, uint32_t max_its, int early_stop,
                   int crc_type, uint8_t *bits, int *crc_ok) {
  if (or_tdec16_reset(h, K)) return -1;
  uint32_t its = 0;
  int ok = 0;
  do {
    or_tdec16_iteration(h, in);
    its++;
    or_tdec16_decision(h, bits);
    ok = ((crc_type ? or_crc24a(bits, K) : or_crc24b(bits, K)) == 0);
    if (early_stop && ok) break;
  } while (its < max_its);
  *crc_ok = ok;
  return (int)its;
}

static int g_tdec_mode = OR_TDEC_GEN;
void or_set_tdec_mode(int mode) { g_tdec_mode = mode; }
int or_get_tdec_mode(void) { return g_tdec_mode; }
