// ul.hip -- UL PUSCH transmit chain on gfx950: what srsUE reaches through
// srslte_ue_ul_pusch_encode_rnti_softbuffer (/root/reference/ue/src/phy/phch_worker.cc:555-560).
//
//   ul_tbcrc_kernel   one workgroup per transport block: CRC24A of the payload bytes, chunk-parallel
//                     byte-table CRCs combined by GF(2) shifts (CRC(A||B) = CRC(A) x^|B| + CRC(B));
//   ul_encode_kernel  one workgroup per code block: code-block bits in LDS (filler, TB bits, TB CRC,
//                     CB CRC24B), both recursive constituent encoders chunk-parallel (the encoder is
//                     linear over GF(2): every chunk first runs from state 0, a scan of the 3-bit end
//                     states gives each chunk its true start state, then each chunk re-runs and emits
//                     its parity), trellis termination, rate matching through the per-(K, F) selection
//                     table, Qm coded bits packed per output symbol;
//   pusch_mod_kernel  one workgroup per (transmission, slot): channel interleaver read (36.212
//                     5.2.2.8), scrambling, modulation, M-point transform precoding and the DMRS
//                     sequence, mapping, N-point SC-FDMA transform with the half-subcarrier shift and
//                     the cyclic prefix -- mixed-radix Stockham transforms in LDS, twiddles staged once
//                     per workgroup.
#include "kernels.h"
#include "tb_body.h"
#include "ul_common.h"

namespace mi {

// 36.211 Tables 5.5.1.2-1 / 5.5.1.2-2: phi(n) of the base sequences r_u(n) = exp(j phi(n) pi / 4) for M_sc = 12
// and 24 (L_prb = 1, 2), sequence-group number u = 0..29.  Transcribed from the specification; the CPU suite
// checks every row's low-PAPR design property (tests/test_oracle_ul.py), the oracle holds its own copy.
__constant__ int8_t UL_PHI12[30][12] = {
    {-1,  1,  3, -3,  3,  3,  1,  1,  3,  1, -3,  3},
    { 1,  1,  3,  3,  3, -1,  1, -3, -3,  1, -3,  3},
    { 1,  1, -3, -3, -3, -1, -3, -3,  1, -3,  1, -1},
    {-1,  1,  1,  1,  1, -1, -3, -3,  1, -3,  3, -1},
    {-1,  3,  1, -1,  1, -1, -3, -1,  1, -1,  1,  3},
    { 1, -3,  3, -1, -1,  1,  1, -1, -1,  3, -3,  1},
    {-1,  3, -3, -3, -3,  3,  1, -1,  3,  3, -3,  1},
    {-3, -1, -1, -1,  1, -3,  3, -1,  1, -3,  3,  1},
    { 1, -3,  3,  1, -1, -1, -1,  1,  1,  3, -1,  1},
    { 1, -3, -1,  3,  3, -1, -3,  1,  1,  1,  1,  1},
    {-1,  3, -1,  1,  1, -3, -3, -1, -3, -3,  3, -1},
    { 3,  1, -1, -1,  3,  3, -3,  1,  3,  1,  3,  3},
    { 1, -3,  1,  1, -3,  1,  1,  1, -3, -3, -3,  1},
    { 3,  3, -3,  3, -3,  1,  1,  3, -1, -3,  3,  3},
    {-3,  1, -1, -3, -1,  3,  1,  3,  3,  3, -1,  1},
    { 3, -1,  1, -3, -1, -1,  1,  1,  3,  1, -1, -3},
    { 1,  3,  1, -1,  1,  3,  3,  3, -1, -1,  3, -1},
    {-3,  1,  1,  3, -3,  3, -3, -3,  3,  1,  3, -1},
    {-3,  3,  1,  1, -3,  1, -3, -3, -1, -1,  1, -3},
    {-1,  3,  1,  3,  1, -1, -1,  3, -3, -1, -3, -1},
    {-1, -3,  1,  1,  1,  1,  3,  1, -1,  1, -3, -1},
    {-1,  3, -1,  1, -3, -3, -3, -3, -3,  1, -1, -3},
    { 1,  1, -3, -3, -3, -3, -1,  3, -3,  1, -3,  3},
    { 1,  1, -1, -3, -1, -3,  1, -1,  1,  3, -1,  1},
    { 1,  1,  3,  1,  3,  3, -1,  1, -1, -3, -3,  1},
    { 1, -3,  3,  3,  1,  3,  3,  1, -3, -1, -1,  3},
    { 1,  3, -3, -3,  3, -3,  1, -1, -1,  3, -1, -3},
    {-3, -1, -3, -1, -3,  3,  1, -1,  1,  3, -3, -3},
    {-1,  3, -3,  3, -1,  3,  3, -3,  3,  3, -1, -1},
    { 3, -3, -3, -1, -1, -3, -1,  3, -3,  3,  1, -1}};
__constant__ int8_t UL_PHI24[30][24] = {
    {-1,  3,  1, -3,  3, -1,  1,  3, -3,  3,  1,  3, -3,  3,  1,  1, -1,  1,  3, -3,  3, -3, -1, -3},
    {-3,  3, -3, -3, -3,  1, -3, -3,  3, -1,  1,  1,  1,  3,  1, -1,  3, -3, -3,  1,  3,  1,  1, -3},
    { 3, -1,  3,  3,  1,  1, -3,  3,  3,  3,  3,  1, -1,  3, -1,  1,  1, -1, -3, -1, -1,  1,  3,  3},
    {-1, -3,  1,  1,  3, -3,  1,  1, -3, -1, -1,  1,  3,  1,  3,  1, -1,  3,  1,  1, -3, -1, -3, -1},
    {-1, -1, -1, -3, -3, -1,  1,  1,  3,  3, -1,  3, -1,  1, -1, -3,  1, -1, -3, -3,  1, -3, -1, -1},
    {-3,  1,  1,  3, -1,  1,  3,  1, -3,  1, -3,  1,  1, -1, -1,  3, -1, -3,  3, -3, -3, -3,  1,  1},
    { 1,  1, -1, -1,  3, -3, -3,  3, -3,  1, -1, -1,  1, -1,  1,  1, -1, -3, -1,  1, -1,  3, -1, -3},
    {-3,  3,  3, -1, -1, -3, -1,  3,  1,  3,  1,  3,  1,  1, -1,  3,  1, -1,  1,  3, -3, -1, -1,  1},
    {-3,  1,  3, -3,  1, -1, -3,  3, -3,  3, -1, -1, -1, -1,  1, -3, -3, -3,  1, -3, -3, -3,  1, -3},
    { 1,  1, -3,  3,  3, -1, -3, -1,  3, -3,  3,  3,  3, -1,  1,  1, -3,  1, -1,  1,  1, -3,  1,  1},
    {-1,  1, -3, -3,  3, -1,  3, -1, -1, -3, -3, -3, -1, -3, -3,  1, -1,  1,  3,  3, -1,  1, -1,  3},
    { 1,  3,  3, -3, -3,  1,  3,  1, -1, -3, -3, -3,  3,  3, -3,  3,  3, -1, -3,  3, -1,  1, -3,  1},
    { 1,  3,  3,  1,  1,  1, -1, -1,  1, -3,  3, -1,  1,  1, -3,  3,  3, -1, -3,  3, -3, -1, -3, -1},
    { 3, -1, -1, -1, -1, -3, -1,  3,  3,  1, -1,  1,  3,  3,  3, -1,  1,  1, -3,  1,  3, -1, -3,  3},
    {-3, -3,  3,  1,  3,  1, -3,  3,  1,  3,  1,  1,  3,  3, -1, -1, -3,  1, -3, -1,  3,  1,  1,  3},
    {-1, -1,  1, -3,  1,  3, -3,  1, -1, -3, -1,  3,  1,  3,  1, -1, -3, -3, -1, -1, -3, -3, -3, -1},
    {-1, -3,  3, -1, -1, -1, -1,  1,  1, -3,  3,  1,  3,  3,  1, -1,  1, -3,  1, -3,  1,  1, -3, -1},
    { 1,  3, -1,  3,  3, -1, -3,  1, -1, -3,  3,  3,  3, -1,  1,  1,  3, -1, -3, -1,  3, -1, -1, -1},
    { 1,  1,  1,  1,  1, -1,  3, -1, -3,  1,  1,  3, -3,  1, -3, -1,  1,  1, -3, -3,  3,  1,  1, -3},
    { 1,  3,  3,  1, -1, -3,  3, -1,  3,  3,  3, -3,  1, -1,  1, -1, -3, -1,  1,  3, -1,  3, -3, -3},
    {-1, -3,  3, -3, -3, -3, -1, -1, -3, -1, -3,  3,  1,  3, -3, -1,  3, -1,  1, -1,  3, -3,  1, -1},
    {-3, -3,  1,  1, -1,  1, -1,  1, -1,  3,  1, -3, -1,  1, -1,  1, -1, -1,  3,  3, -3, -1,  1, -3},
    {-3, -1, -3,  3,  1, -1, -3, -1, -3, -3,  3, -3,  3, -3, -1,  1,  3,  1, -3,  1,  3,  3, -1, -3},
    {-1, -1, -1, -1,  3,  3,  3,  1,  3,  3, -3,  1,  3, -1,  3, -1,  3,  3, -3,  3,  1, -1,  3,  3},
    { 1, -1,  3,  3, -1, -3,  3, -3, -1, -1,  3, -1,  3, -1, -1,  1,  1,  1,  1, -1, -1, -3, -1,  3},
    { 1, -1,  1, -1,  3, -1,  3,  1,  1, -1, -1, -3,  1,  1, -3,  1,  3, -3,  1,  1, -3, -3, -1, -1},
    {-3, -1,  1,  3,  1,  1, -3, -1, -1, -3,  3, -3,  3,  1, -3,  3, -3,  1, -1,  1, -3,  1,  1,  1},
    {-1, -3,  3,  3,  1,  1,  3, -1, -3, -1, -1, -1,  3,  1, -3, -3, -1,  3, -3, -1, -3, -1, -3, -1},
    {-1, -3, -1, -1,  1, -3, -1, -1,  1, -1, -3,  1,  1, -3,  1, -3, -3,  3,  1,  1, -1,  3, -1, -1},
    { 1,  1, -1, -1, -3, -1,  3, -1,  3, -1,  1,  3,  1, -1,  3,  1,  3, -3, -3,  1, -1, -1,  1,  3}};

namespace {

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ float2 mul_nj(float2 a) { return make_float2(a.y, -a.x); }   // * (-j)

// forward radix-R butterflies (exp(-2 pi i / R))
__device__ __forceinline__ void bf2(float2* v) { const float2 a = v[0]; v[0] = cadd(a, v[1]); v[1] = csub(a, v[1]); }
__device__ __forceinline__ void bf3(float2* v) {
  const float s = 0.86602540378443864676f;
  const float2 a = v[0], t = cadd(v[1], v[2]), u = csub(v[1], v[2]);
  const float2 m = make_float2(a.x - 0.5f * t.x, a.y - 0.5f * t.y);
  v[0] = cadd(a, t);
  v[1] = make_float2(m.x + s * u.y, m.y - s * u.x);
  v[2] = make_float2(m.x - s * u.y, m.y + s * u.x);
}
__device__ __forceinline__ void bf4(float2* v) {
  const float2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]), t2 = cadd(v[1], v[3]), t3 = csub(v[1], v[3]);
  v[0] = cadd(t0, t2);
  v[2] = csub(t0, t2);
  v[1] = make_float2(t1.x + t3.y, t1.y - t3.x);
  v[3] = make_float2(t1.x - t3.y, t1.y + t3.x);
}
__device__ __forceinline__ void bf5(float2* v) {
  const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
  const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
  const float2 a = v[0], b1 = cadd(v[1], v[4]), b2 = cadd(v[2], v[3]), d1 = csub(v[1], v[4]), d2 = csub(v[2], v[3]);
  const float2 p1 = make_float2(a.x + c1 * b1.x + c2 * b2.x, a.y + c1 * b1.y + c2 * b2.y);
  const float2 p2 = make_float2(a.x + c2 * b1.x + c1 * b2.x, a.y + c2 * b1.y + c1 * b2.y);
  const float2 q1 = mul_nj(make_float2(s1 * d1.x + s2 * d2.x, s1 * d1.y + s2 * d2.y));
  const float2 q2 = mul_nj(make_float2(s2 * d1.x - s1 * d2.x, s2 * d1.y - s1 * d2.y));
  v[0] = cadd(a, cadd(b1, b2));
  v[1] = cadd(p1, q1);
  v[4] = csub(p1, q1);
  v[2] = cadd(p2, q2);
  v[3] = csub(p2, q2);
}

__device__ __forceinline__ void bf8(float2* v) {
  float2 e[4] = {v[0], v[2], v[4], v[6]}, o[4] = {v[1], v[3], v[5], v[7]};
  bf4(e);
  bf4(o);
  const float r = 0.70710678118654752440f;
  o[1] = make_float2((o[1].x + o[1].y) * r, (o[1].y - o[1].x) * r);      // * (1 - j) / sqrt 2
  o[2] = mul_nj(o[2]);                                                     // * -j
  o[3] = make_float2((o[3].y - o[3].x) * r, (-o[3].x - o[3].y) * r);     // * (-1 - j) / sqrt 2
#pragma unroll
  for (int i = 0; i < 4; i++) {
    v[i] = cadd(e[i], o[i]);
    v[i + 4] = csub(e[i], o[i]);
  }
}

template <int R>
__device__ __forceinline__ void bf(float2 (&v)[R]) {
  if constexpr (R == 2) bf2(v);
  else if constexpr (R == 3) bf3(v);
  else if constexpr (R == 4) bf4(v);
  else if constexpr (R == 5) bf5(v);
  else bf8(v);
}

// One Stockham stage (decimation in time) of an n-point forward DFT in LDS, radix R, Ns points done so
// far: butterfly j (< n / R) reads x[j + r n/R], twiddles by W_{Ns R}^{(j mod Ns) r} (tw[t] =
// exp(-2 pi i t / n)), writes y[(j / Ns) Ns R + j mod Ns + r Ns].  All threads of the block take part.
template <int R>
__device__ __forceinline__ void fft_stage(float2* buf, uint32_t n, uint32_t Ns, const float2* tw) {
  constexpr int PER = (UL_NMAX / R + UL_THREADS - 1) / UL_THREADS;
  const uint32_t nb = n / R, tws = n / (Ns * R);
  float2 v[PER][R];
#pragma unroll
  for (int p = 0; p < PER; p++) {
    const uint32_t j = threadIdx.x + p * UL_THREADS;
    if (j < nb) {
#pragma unroll
      for (int r = 0; r < R; r++) v[p][r] = buf[j + r * nb];
    }
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < PER; p++) {
    const uint32_t j = threadIdx.x + p * UL_THREADS;
    if (j < nb) {
      const uint32_t k = j % Ns;
#pragma unroll
      for (int r = 1; r < R; r++) v[p][r] = cmul(v[p][r], tw[k * r * tws]);   // k r tws < n
      bf<R>(v[p]);
      const uint32_t base = (j / Ns) * Ns * R + k;
#pragma unroll
      for (int r = 0; r < R; r++) buf[base + r * Ns] = v[p][r];
    }
  }
  __syncthreads();
}

// In-place forward DFT of n <= 2048 points over the radix list `plan` (4 bits per stage)
__device__ __forceinline__ void fft_lds(float2* buf, uint32_t n, uint32_t plan, const float2* tw) {
  uint32_t Ns = 1;
  for (int st = 0; st < 8; st++) {
    const uint32_t R = (plan >> (4 * st)) & 15u;
    if (!R) break;
    switch (R) {
      case 2: fft_stage<2>(buf, n, Ns, tw); break;
      case 3: fft_stage<3>(buf, n, Ns, tw); break;
      case 4: fft_stage<4>(buf, n, Ns, tw); break;
      case 5: fft_stage<5>(buf, n, Ns, tw); break;
      default: fft_stage<8>(buf, n, Ns, tw); break;
    }
    Ns *= R;
  }
}

template <int P>
__device__ __forceinline__ uint32_t block_xor_u32(uint32_t v, uint32_t* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v ^= (uint32_t)__shfl_xor((int)v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < P / 64; i++) r ^= red[i];
  __syncthreads();
  return r;
}

// this thread's term of the CRC register over bytes src[0..n): its contiguous chunk through the byte
// table, shifted by the bytes after it
__device__ __forceinline__ uint32_t crc_chunk_term(const uint8_t* src, uint32_t n, const uint32_t* tab, uint32_t poly) {
  const uint32_t per = (n + UL_THREADS - 1) / UL_THREADS, s = threadIdx.x * per;
  if (s >= n) return 0;
  const uint32_t e = s + per < n ? s + per : n;
  uint32_t r = 0;
  for (uint32_t j = s; j < e; j++) r = ((r << 8) & 0xFFFFFFu) ^ tab[((r >> 16) ^ src[j]) & 0xFFu];
  return r ? gf24_mulmod(r, gf24_xpow8(n - e, poly), poly) : 0u;
}

// 36.212 5.1.3.2.1 constituent encoder (s = 4 s1 + 2 s2 + s3): feedback a = u ^ s2 ^ s3,
// parity z = a ^ s1 ^ s3, next state (a, s1, s2)
__device__ __forceinline__ uint32_t rsc_next(uint32_t s, uint32_t u) { return (((u ^ (s >> 1) ^ s) & 1u) << 2) | (s >> 1); }
__device__ __forceinline__ uint32_t rsc_par(uint32_t s, uint32_t u) { return (u ^ (s >> 1) ^ s ^ (s >> 2) ^ s) & 1u; }

}  // namespace

__global__ __launch_bounds__(UL_THREADS) void ul_tbcrc_kernel(const uint8_t* __restrict__ pay,
                                                              const MiUlTx* __restrict__ txs,
                                                              uint32_t* __restrict__ tbcrc) {
  __shared__ uint32_t tab[256];
  __shared__ uint32_t red[UL_THREADS / 64];
  const MiUlTx t = txs[blockIdx.x];
  tab[threadIdx.x] = crc24_byte_entry(threadIdx.x, CRC24A_POLY);
  __syncthreads();
  const uint32_t c = block_xor_u32<UL_THREADS>(crc_chunk_term(pay + t.pay_off, t.tbs / 8, tab, CRC24A_POLY), red);
  if (threadIdx.x == 0) tbcrc[blockIdx.x] = c;
}

__global__ __launch_bounds__(UL_THREADS) void ul_encode_kernel(const uint8_t* __restrict__ pay,
                                                               const uint32_t* __restrict__ tbcrc,
                                                               const MiUlTx* __restrict__ txs,
                                                               const MiUlCb* __restrict__ cbs,
                                                               const uint32_t* __restrict__ kdata,
                                                               uint8_t* __restrict__ syms) {
  __shared__ uint8_t cbit[KMAX];                 // code-block bits c_k
  __shared__ uint8_t d[3 * (KMAX + 4)];          // d-stream bits, triplet order t = 3k + i (2 = <NULL>)
  __shared__ uint8_t src[KMAX / 8];              // the code block's (TB || CRC24A) bytes
  __shared__ uint32_t tab[256];
  __shared__ uint32_t red[UL_THREADS / 64];
  __shared__ uint8_t zend[UL_THREADS], sstart[UL_THREADS];
  const MiUlCb b = cbs[blockIdx.x];
  const MiUlTx tx = txs[b.tx];
  const uint32_t t = threadIdx.x, K = b.K, F = b.F, L = b.C > 1 ? 24 : 0, nTB = tx.tbs / 8;
  tab[t] = crc24_byte_entry(t, CRC24B_POLY);
  const uint32_t tc = tbcrc[b.tx];
  for (uint32_t j = t; j < b.nbytes; j += UL_THREADS) {
    const uint32_t g = b.byte0 + j;
    src[j] = g < nTB ? pay[tx.pay_off + g] : (uint8_t)(tc >> (8 * (2 - (g - nTB))));
  }
  __syncthreads();
  for (uint32_t k = t; k < K - L; k += UL_THREADS)
    cbit[k] = k < F ? 0 : (src[(k - F) >> 3] >> (7 - ((k - F) & 7))) & 1u;
  if (L) {   // CB CRC24B over the code block's bytes (the leading filler zero bytes leave the register 0)
    const uint32_t cb = block_xor_u32<UL_THREADS>(crc_chunk_term(src, b.nbytes, tab, CRC24B_POLY), red);
    if (t < 24) cbit[K - 24 + t] = (cb >> (23 - t)) & 1u;
  }
  __syncthreads();
  // ---- turbo encoder: threads 0..127 the first constituent encoder (natural order), 128..255 the
  // second (QPP order); chunk c of CH steps per thread
  constexpr uint32_t HALF = UL_THREADS / 2;
  const bool enc2 = t >= HALF;
  const uint32_t c = t % HALF, CH = (K + HALF - 1) / HALF, k0 = c * CH, k1 = k0 + CH < K ? k0 + CH : K;
  const uint32_t* pi = kdata + b.pi_off;
  auto in_bit = [&](uint32_t k) -> uint32_t { return enc2 ? cbit[pi[k]] : cbit[k]; };
  uint32_t s = 0;
  for (uint32_t k = k0; k < k1; k++) s = rsc_next(s, in_bit(k));
  zend[t] = (uint8_t)s;
  __syncthreads();
  if (c == 0) {
    // A^CH as a packed table (3 bits per state): the zero-input state map over one full chunk
    uint32_t jump = 0;
    for (uint32_t s0 = 0; s0 < 8; s0++) {
      uint32_t x = s0;
      for (uint32_t i = 0; i < CH % 7; i++) x = rsc_next(x, 0);   // the zero-input map has order 7
      jump |= x << (3 * s0);
    }
    uint32_t v = 0;
    const uint32_t base = enc2 ? HALF : 0;
    for (uint32_t i = 0; i < HALF; i++) {
      sstart[base + i] = (uint8_t)v;
      v = ((jump >> (3 * v)) & 7u) ^ zend[base + i];   // end state of chunk i = A^CH start ^ zero-start end
    }
  }
  __syncthreads();
  s = sstart[t];
  for (uint32_t k = k0; k < k1; k++) {
    const uint32_t u = in_bit(k);
    if (!enc2) {
      d[3 * k] = (uint8_t)u;
      d[3 * k + 1] = (uint8_t)rsc_par(s, u);
    } else {
      d[3 * k + 2] = (uint8_t)rsc_par(s, u);
    }
    s = rsc_next(s, u);
  }
  if (k0 < K && k1 == K) {   // the last chunk terminates its trellis (36.212 5.1.3.2.2): 3 steps
    for (uint32_t j = 0; j < 3; j++) {
      const uint32_t s1 = (s >> 2) & 1u, s2 = (s >> 1) & 1u, s3 = s & 1u;
      d[3 * K + (enc2 ? 6 : 0) + 2 * j] = (uint8_t)(s2 ^ s3);
      d[3 * K + (enc2 ? 6 : 0) + 2 * j + 1] = (uint8_t)(s1 ^ s3);
      s >>= 1;
    }
  }
  __syncthreads();
  for (uint32_t k = t; k < F; k += UL_THREADS) { d[3 * k] = 2; d[3 * k + 1] = 2; }
  __syncthreads();
  // ---- rate matching (bit selection from k0(rv) over the non-null positions) + symbol packing
  const uint32_t* sel = kdata + b.sel_off;
  const uint32_t nsym = b.E / tx.Qm;
  uint8_t* out = syms + tx.sym_off + b.sym0;
  for (uint32_t q = t; q < nsym; q += UL_THREADS) {
    uint32_t v = 0, n = (b.r0 + q * tx.Qm) % b.Nv;
    for (uint32_t i = 0; i < tx.Qm; i++) {
      v = (v << 1) | d[sel[n]];
      n = n + 1 == b.Nv ? 0 : n + 1;
    }
    out[q] = (uint8_t)v;
  }
}

__global__ __launch_bounds__(UL_THREADS) void pusch_mod_kernel(const uint8_t* __restrict__ syms,
                                                               const uint32_t* __restrict__ scr,
                                                               const MiUlTx* __restrict__ txs,
                                                               const float2* __restrict__ twg,
                                                               float2* __restrict__ iq, uint32_t per) {
  __shared__ float2 buf[UL_NMAX];
  __shared__ float2 twn[UL_NMAX];
  __shared__ float2 twm[UL_MMAX];
  const MiUlTx x = txs[blockIdx.x];
  // symbols l0 .. l0 + per - 1 of the subframe (per = 7: one workgroup per slot, twiddles staged once
  // for 7 symbols -- batches; per = 1: one workgroup per symbol -- the per-TTI latency path)
  const uint32_t l0 = blockIdx.y * per, slot = l0 / 7, t = threadIdx.x, N = x.N, M = x.M, Qm = x.Qm;
  const uint32_t dq = slot ? x.q[1] : x.q[0], dncs = slot ? x.ncs[1] : x.ncs[0];   // no dynamic struct index
  for (uint32_t i = t; i < N; i += UL_THREADS) twn[i] = twg[x.twn_off + i];
  for (uint32_t i = t; i < M; i += UL_THREADS) twm[i] = twg[x.twm_off + i];
  const float sM = rsqrtf((float)M), gN = rsqrtf((float)N) * x.scale;
  constexpr int PM = (UL_MMAX + UL_THREADS - 1) / UL_THREADS;
  // allocation's first subcarrier relative to W/2 (slot 1 may hop: 36.213 8.4)
  const int off = (int)(12 * (slot ? x.n_prb1 : x.n_prb)) - (int)(x.W / 2);
  uint32_t pos = (uint32_t)(symbol_offset((int)N, (int)l0) - cp_len((int)N, (int)(l0 % 7)));   // first sample of l0
  __syncthreads();
  for (uint32_t ls = l0 % 7; ls < l0 % 7 + per; ls++) {
    const uint32_t l = 7 * slot + ls, cp = cp_len((int)N, (int)ls);
    if (ls == 3) {
      // DMRS 36.211 5.5.2.1: r(n) = exp(j alpha n) x_q(n mod N_ZC), x_q(m) = exp(-j pi q m (m+1) / N_ZC); for
      // M_sc = 12 / 24 (nzc == 0, dq = the group u) the tabulated base sequence exp(j phi_u(n) pi / 4) (5.5.1.2)
      for (uint32_t n = t; n < M; n += UL_THREADS) {
        const uint32_t cs = (dncs * n) % 12;
        float ph;
        if (x.nzc) {
          const uint32_t m = n % x.nzc;
          const uint32_t a = (uint32_t)(((uint64_t)dq * m * (m + 1)) % (2ull * x.nzc));
          ph = -(float)a / (float)x.nzc + (float)cs / 6.0f;
        } else {
          ph = (float)(M == 12 ? UL_PHI12[dq][n] : UL_PHI24[dq][n]) * 0.25f + (float)cs / 6.0f;
        }
        float sv, cv;
        sincospif(ph, &sv, &cv);
        buf[n] = make_float2(cv, sv);
      }
      __syncthreads();
    } else {
      const uint32_t ld = l - (l > 3 ? 1 : 0) - (l > 10 ? 1 : 0);   // data symbol 0..11
      for (uint32_t m = t; m < M; m += UL_THREADS) {
        // channel interleaver (36.212 5.2.2.8): matrix row m, column ld.  RI symbol i sits in row M - 1 - i / 4
        // of column {1, 10, 7, 4}[i % 4], HARQ-ACK symbol i in row M - 1 - i / 4 of column {2, 9, 8, 3}[i % 4]
        // (ColumnSets {1, 4, 7, 10} / {2, 3, 8, 9} walked with j = (j + 3) mod 4); the multiplexed sequence g
        // (CQI then data) fills the other cells row by row, skipping the RI cells; HARQ-ACK overwrites g.
        const uint32_t i0 = (ld * M + m) * Qm;
        const int ta = x.q_ack ? (ld == 2 ? 0 : ld == 9 ? 1 : ld == 8 ? 2 : ld == 3 ? 3 : -1) : -1;
        const int tr = x.q_ri ? (ld == 1 ? 0 : ld == 10 ? 1 : ld == 7 ? 2 : ld == 4 ? 3 : -1) : -1;
        const uint32_t ia = 4 * (M - 1 - m) + (uint32_t)ta, ir = 4 * (M - 1 - m) + (uint32_t)tr;
        const bool is_ack = ta >= 0 && ia < x.q_ack, is_ri = tr >= 0 && ir < x.q_ri;
        uint32_t bits = 0;
        if (is_ack || is_ri) {
          // 36.211 5.3.1 placeholders: x -> 1, y -> the previous scrambled bit
          const uint32_t nb = is_ack ? x.ack_nblk : x.ri_nblk, ks = nb == 1 ? 0u : (is_ack ? ia : ir) % 3;
          const uint32_t w0 = is_ack ? x.ack_sym[0] : x.ri_sym[0], w1 = is_ack ? x.ack_sym[1] : x.ri_sym[1];
          const uint32_t w2 = is_ack ? x.ack_sym[2] : x.ri_sym[2];
          const uint32_t cw = ks == 0 ? w0 : ks == 1 ? w1 : w2;   // selects, no dynamic index into x
          uint32_t prev = 0;
          for (uint32_t b = 0; b < Qm; b++) {
            const uint32_t i = i0 + b, code = (cw >> (2 * b)) & 3u;
            const uint32_t bit = code == 2 ? 1u : code == 3 ? prev : ((code ^ (scr[x.scr_off + (i >> 5)] >> (i & 31))) & 1u);
            bits = (bits << 1) | bit;
            prev = bit;
          }
        } else {
          // g index of cell (m, ld): cells of the rows above less their RI cells, plus the free cells left of
          // ld in row m (RI cells of rows >= r: min(Q'_RI, 4 (M - r)); row m's fill {1, 10, 7, 4} in order)
          uint32_t k = 12 * m + ld;
          if (x.q_ri) {
            const uint32_t below = min(x.q_ri, 4 * (M - 1 - m)), from = min(x.q_ri, 4 * (M - m)), nrow = from - below;
            const uint32_t left = (nrow > 0 && ld > 1) + (nrow > 3 && ld > 4) + (nrow > 2 && ld > 7) + (nrow > 1 && ld > 10);
            k -= (x.q_ri - from) + left;
          }
          const uint32_t v = syms[x.sym_off + k];
          for (uint32_t b = 0; b < Qm; b++) {
            const uint32_t i = i0 + b;
            bits = (bits << 1) | (((v >> (Qm - 1 - b)) ^ (scr[x.scr_off + (i >> 5)] >> (i & 31))) & 1u);
          }
        }
        // 36.211 7.1: bits b0 b1 .. (b0 = MSB); I from b0, b2, b4 and Q from b1, b3, b5
        const uint32_t b0 = (bits >> (Qm - 1)) & 1u, b1 = (bits >> (Qm - 2)) & 1u;
        float re, im;
        if (Qm == 2) {
          re = (1.0f - 2.0f * b0) * 0.70710678118654752f;
          im = (1.0f - 2.0f * b1) * 0.70710678118654752f;
        } else if (Qm == 4) {
          const uint32_t b2 = (bits >> 1) & 1u, b3 = bits & 1u;
          re = (1.0f - 2.0f * b0) * (1.0f + 2.0f * b2) * 0.31622776601683794f;
          im = (1.0f - 2.0f * b1) * (1.0f + 2.0f * b3) * 0.31622776601683794f;
        } else {
          const uint32_t b2 = (bits >> 3) & 1u, b3 = (bits >> 2) & 1u, b4 = (bits >> 1) & 1u, b5 = bits & 1u;
          re = (1.0f - 2.0f * b0) * (4.0f - (1.0f - 2.0f * b2) * (2.0f - (1.0f - 2.0f * b4))) * 0.15430334996209191f;
          im = (1.0f - 2.0f * b1) * (4.0f - (1.0f - 2.0f * b3) * (2.0f - (1.0f - 2.0f * b5))) * 0.15430334996209191f;
        }
        buf[m] = make_float2(re, im);
      }
      __syncthreads();
      fft_lds(buf, M, x.fact, twm);   // transform precoding (5.3.3), scaled below
    }
    // mapping (5.3.4) into the N-point transform input, conjugated: IDFT(X) = conj(DFT(conj(X)))
    float2 z[PM];
    const float zs = ls == 3 ? 1.0f : sM;
#pragma unroll
    for (int p = 0; p < PM; p++) {
      const uint32_t k = t + p * UL_THREADS;
      if (k < M) z[p] = buf[k];
    }
    __syncthreads();
    for (uint32_t i = t; i < N; i += UL_THREADS) buf[i] = make_float2(0.0f, 0.0f);
    __syncthreads();
#pragma unroll
    for (int p = 0; p < PM; p++) {
      const uint32_t k = t + p * UL_THREADS;
      if (k < M) buf[(uint32_t)((int)k + off + (int)N) % N] = make_float2(z[p].x * zs, -z[p].y * zs);
    }
    __syncthreads();
    fft_lds(buf, N, x.fact_n, twn);
    // SC-FDMA 5.6: s(n) = conj(buf[n mod N]) exp(j pi n / N) / sqrt(N), n = -cp .. N-1
    float2* dst = iq + x.iq_off + pos;
    for (uint32_t i = t; i < N + cp; i += UL_THREADS) {
      const int n = (int)i - (int)cp;
      const float2 y = buf[(uint32_t)(n + (int)N) % N];
      // half-subcarrier shift, plus the frequency offset srslte_ue_ul_set_cfo asks for (cfo subcarriers
      // over the subframe's sample index), in units of pi
      const float ph = ((float)n + 2.0f * x.cfo * (float)(pos + i)) / (float)N;
      float sv, cv;
      sincospif(ph, &sv, &cv);
      dst[i] = make_float2((y.x * cv + y.y * sv) * gN, (y.x * sv - y.y * cv) * gN);
    }
    __syncthreads();
    pos += N + cp;
  }
}

void launch_ul(const uint8_t* pay, uint32_t* tbcrc, const MiUlTx* txs, uint32_t n_tx, const MiUlCb* cbs, uint32_t n_cb,
               const uint32_t* kdata, const uint32_t* scr, const float2* tw, uint8_t* syms, float2* iq, int stage,
               hipStream_t st) {
  if (!n_tx) return;
  if (stage == 0) hipLaunchKernelGGL(ul_tbcrc_kernel, dim3(n_tx), dim3(UL_THREADS), 0, st, pay, txs, tbcrc);
  if (stage == 1) hipLaunchKernelGGL(ul_encode_kernel, dim3(n_cb), dim3(UL_THREADS), 0, st, pay, tbcrc, txs, cbs, kdata, syms);
  if (stage == 2) {
    const uint32_t per = n_tx >= 64 ? 7 : 1;   // small batches: a workgroup per symbol (latency)
    hipLaunchKernelGGL(pusch_mod_kernel, dim3(n_tx, 14 / per), dim3(UL_THREADS), 0, st, syms, scr, txs, tw, iq, per);
  }
}

}  // namespace mi
