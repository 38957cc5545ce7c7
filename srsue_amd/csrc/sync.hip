// sync.hip -- sync front end on the GPU: what srsUE reaches through
// srslte_ue_sync_zerocopy (/root/reference/ue/src/phy/phch_recv.cc:321) and _get_cfo / _get_sfidx
// (:241, :326).  Detection contract: oracle/o_sync.c (reproduced here in fp32).
//
// MI355X layout:
//   * pss_search_kernel: one workgroup per search window; the three time-domain PSS templates of the
//     bandwidth are staged in LDS (3 x N complex); 1, 2 or 4 threads share a lag (a tracking window of
//     63 lags keeps 252 threads busy) and stream their segment once for all candidates in the job's
//     mask, keeping the two half-window sums per candidate for the CFO estimate; partial sums combine
//     by lane shuffles and the (rho, N_ID_2, lag) maximum is reduced in LDS with the oracle's tie order;
//   * sss_detect_kernel: one workgroup per subframe: the SSS and PSS symbols are CFO-corrected into LDS
//     with an N-entry twiddle table, 124 threads take their 62-bin DFTs, 168 x 2 hypotheses are scored
//     coherently against the PSS-derived channel, argmax in LDS;
//   * cfo_correct_kernel: streaming y[n] = x[n] exp(-j 2 pi cfo n / N) per subframe (HBM-bound: one read
//     and one write of each sample; sincospi keeps the phase exact to float rounding of its argument).
#include "kernels.h"
#include "sync.h"

namespace mi {

constexpr int PSS_T = 256;

// TPL threads share a lag (consecutive lanes, each a contiguous N / TPL segment, combined by shuffles);
// only the candidates in the job's mask are correlated
template <int TPL>
__global__ __launch_bounds__(PSS_T) void pss_search_kernel(const float2* __restrict__ iq, const float2* __restrict__ tmpl,
                                                          const MiPssJob* __restrict__ jobs, MiPssRes* __restrict__ res,
                                                          uint32_t N) {
  extern __shared__ float2 p[];   // [3][N] templates
  __shared__ float s_rho[PSS_T];
  __shared__ uint32_t s_key[PSS_T];
  __shared__ float s_cfo[PSS_T];
  const MiPssJob jb = jobs[blockIdx.x];
  const uint32_t tid = threadIdx.x, part = tid % TPL, slot = tid / TPL;
  const bool on[3] = {(jb.mask & 1u) != 0, (jb.mask & 2u) != 0, (jb.mask & 4u) != 0};
  for (uint32_t i = tid; i < 3 * N; i += PSS_T) p[i] = tmpl[i];
  __syncthreads();
  float ep[3];
#pragma unroll
  for (int u = 0; u < 3; u++) {
    float e = 0.f;
    if (on[u])
      for (uint32_t n = 0; n < N; n++) e += p[u * N + n].x * p[u * N + n].x + p[u * N + n].y * p[u * N + n].y;
    ep[u] = e;   // every thread computes the same sums in the same order
  }
  float best = -1.f, bcfo = 0.f;
  uint32_t bkey = 0xFFFFFFFFu;   // (u << 20) | lag of this thread's best
  const float2* x = iq + jb.off;
  const uint32_t seg = N / TPL, n0 = part * seg;
  for (uint32_t t0 = 0; t0 < jb.nlag; t0 += PSS_T / TPL) {   // uniform trip count: shuffles stay convergent
    const uint32_t t = t0 + slot;
    const bool live = t < jb.nlag;
    float y1r[3] = {0.f, 0.f, 0.f}, y1i[3] = {0.f, 0.f, 0.f}, y2r[3] = {0.f, 0.f, 0.f}, y2i[3] = {0.f, 0.f, 0.f};
    float ex = 0.f;
    if (live) {
      for (uint32_t n = n0; n < n0 + seg; n++) {
        const float2 a = x[t + n];
        ex += a.x * a.x + a.y * a.y;
        const bool h2 = n >= N / 2;
#pragma unroll
        for (int u = 0; u < 3; u++) {
          if (!on[u]) continue;
          const float2 b = p[u * N + n];
          const float cr = a.x * b.x + a.y * b.y, ci = a.y * b.x - a.x * b.y;   // x conj(p)
          if (h2) { y2r[u] += cr; y2i[u] += ci; } else { y1r[u] += cr; y1i[u] += ci; }
        }
      }
    }
#pragma unroll
    for (int o = 1; o < TPL; o <<= 1) {
      ex += __shfl_xor(ex, o, 64);
#pragma unroll
      for (int u = 0; u < 3; u++) {
        y1r[u] += __shfl_xor(y1r[u], o, 64); y1i[u] += __shfl_xor(y1i[u], o, 64);
        y2r[u] += __shfl_xor(y2r[u], o, 64); y2i[u] += __shfl_xor(y2i[u], o, 64);
      }
    }
    if (!live || part != 0) continue;
#pragma unroll
    for (int u = 0; u < 3; u++) {
      if (!on[u]) continue;
      const float yr = y1r[u] + y2r[u], yi = y1i[u] + y2i[u];
      const float rho = ex > 0.f ? (yr * yr + yi * yi) / (ex * ep[u]) : 0.f;
      const uint32_t key = ((uint32_t)u << 20) | t;
      if (rho > best || (rho == best && key < bkey)) {
        best = rho;
        bkey = key;
        bcfo = atan2f(y1r[u] * y2i[u] - y1i[u] * y2r[u], y1r[u] * y2r[u] + y1i[u] * y2i[u]) * 0.318309886183790672f;
      }
    }
  }
  s_rho[tid] = best; s_key[tid] = bkey; s_cfo[tid] = bcfo;
  __syncthreads();
  for (uint32_t s = PSS_T / 2; s > 0; s >>= 1) {
    if (tid < s) {
      const float r2 = s_rho[tid + s];
      const uint32_t k2 = s_key[tid + s];
      if (r2 > s_rho[tid] || (r2 == s_rho[tid] && k2 < s_key[tid])) {
        s_rho[tid] = r2; s_key[tid] = k2; s_cfo[tid] = s_cfo[tid + s];
      }
    }
    __syncthreads();
  }
  if (tid == 0) res[blockIdx.x] = MiPssRes{s_key[0] >> 20, s_key[0] & 0xFFFFFu, s_rho[0], s_cfo[0]};
}

// m-sequences of 36.211 6.11.2.1 (s~, c~, z~ as +-1)
__constant__ int8_t SSS_S[31] = {1, 1, 1, 1, -1, 1, 1, -1, 1, -1, -1, 1, 1, -1, -1, -1, -1, -1, 1, 1, 1, -1, -1, 1, -1, -1, -1, 1, -1, 1, -1};
__constant__ int8_t SSS_C[31] = {1, 1, 1, 1, -1, 1, -1, 1, -1, -1, -1, 1, -1, -1, 1, 1, 1, -1, -1, -1, -1, -1, 1, 1, -1, -1, 1, -1, 1, 1, -1};
__constant__ int8_t SSS_Z[31] = {1, 1, 1, 1, -1, -1, -1, 1, 1, -1, -1, 1, -1, -1, -1, -1, -1, 1, -1, 1, 1, 1, -1, 1, 1, -1, 1, -1, 1, -1, -1};

__device__ inline float sss_d(uint32_t nid1, uint32_t nid2, uint32_t sf5, uint32_t n) {
  const uint32_t qp = nid1 / 30, q = (nid1 + qp * (qp + 1) / 2) / 30, mp = nid1 + q * (q + 1) / 2;
  const uint32_t m0 = mp % 31, m1 = (m0 + mp / 31 + 1) % 31, k = n >> 1;
  if ((n & 1) == 0) {
    const int s = SSS_S[(k + (sf5 ? m1 : m0)) % 31], c = SSS_C[(k + nid2) % 31];
    return (float)(s * c);
  }
  const int s = SSS_S[(k + (sf5 ? m0 : m1)) % 31], c = SSS_C[(k + nid2 + 3) % 31];
  const int z = SSS_Z[(k + ((sf5 ? m1 : m0) % 8)) % 31];
  return (float)(s * c * z);
}

__device__ inline uint32_t sync_bin_d(uint32_t m, uint32_t nof_prb, uint32_t N) {
  const uint32_t W = 12 * nof_prb, k = m - 31 + W / 2;
  return k < W / 2 ? N - W / 2 + k : k - W / 2 + 1;
}

__device__ inline float2 pss_d(uint32_t nid2, uint32_t n) {
  const uint32_t u = nid2 == 0 ? 25 : nid2 == 1 ? 29 : 34;
  const uint32_t e = n < 31 ? (u * n * (n + 1)) % 126 : (u * (n + 1) * (n + 2)) % 126;   // phase -pi e / 63
  float s, c;
  sincospif(-(float)e / 63.0f, &s, &c);
  return make_float2(c, s);
}

__global__ __launch_bounds__(256) void sss_detect_kernel(const float2* __restrict__ iq, const MiSssJob* __restrict__ jobs,
                                                        MiSssRes* __restrict__ res, uint32_t N, uint32_t nof_prb,
                                                        uint32_t l5, uint32_t l6) {
  extern __shared__ float2 sm[];   // [2][N] CFO-corrected SSS / PSS symbols, then [N] twiddles
  float2* tw = sm + 2 * N;
  __shared__ float2 Y[62], H[62];
  __shared__ float s_sc[256];
  __shared__ uint32_t s_h[256];
  const MiSssJob jb = jobs[blockIdx.x];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < 2 * N; i += 256) {
    const uint32_t n = i % N, s0 = (i < N ? l5 : l6);
    const float2 a = iq[jb.off + s0 + n];
    float cs, cc;
    sincospif(-2.0f * jb.cfo * (float)(s0 + n) / (float)N, &cs, &cc);   // CFO removal, subframe phase
    sm[i] = make_float2(a.x * cc - a.y * cs, a.x * cs + a.y * cc);
  }
  for (uint32_t n = tid; n < N; n += 256) {
    float ws, wc;
    sincospif(-2.0f * (float)n / (float)N, &ws, &wc);
    tw[n] = make_float2(wc, ws);
  }
  __syncthreads();
  if (tid < 124) {   // 62-bin DFT of the SSS (sym 0) and PSS (sym 1) symbols
    const uint32_t m = tid % 62, sym = tid / 62, b = sync_bin_d(m, nof_prb, N);
    const float2* x = sm + sym * N;
    float re = 0.f, im = 0.f;
    uint32_t k = 0;
    for (uint32_t n = 0; n < N; n++) {
      const float2 w = tw[k], a = x[n];
      re += a.x * w.x - a.y * w.y;
      im += a.x * w.y + a.y * w.x;
      k += b;
      if (k >= N) k -= N;
    }
    if (sym) {
      const float2 d = pss_d(jb.nid2, m);
      H[m] = make_float2(re * d.x + im * d.y, im * d.x - re * d.y);   // P conj(d)
    } else {
      Y[m] = make_float2(re, im);
    }
  }
  __syncthreads();
  float best = -3.0e38f;
  uint32_t bh = 0xFFFFFFFFu;
  for (uint32_t h = tid; h < 336; h += 256) {
    float sc = 0.f;
    for (uint32_t m = 0; m < 62; m++) sc += (H[m].x * Y[m].x + H[m].y * Y[m].y) * sss_d(h >> 1, jb.nid2, h & 1, m);
    if (sc > best) { best = sc; bh = h; }
  }
  s_sc[tid] = best; s_h[tid] = bh;
  __syncthreads();
  for (uint32_t st = 128; st > 0; st >>= 1) {
    if (tid < st && (s_sc[tid + st] > s_sc[tid] || (s_sc[tid + st] == s_sc[tid] && s_h[tid + st] < s_h[tid]))) {
      s_sc[tid] = s_sc[tid + st];
      s_h[tid] = s_h[tid + st];
    }
    __syncthreads();
  }
  if (tid == 0) res[blockIdx.x] = MiSssRes{s_h[0] >> 1, s_h[0] & 1u, s_sc[0], 0.f};
}

__global__ __launch_bounds__(256) void cfo_correct_kernel(const float2* __restrict__ src, float2* __restrict__ dst,
                                                         const MiCfoJob* __restrict__ jobs, uint32_t len, uint32_t N) {
  const MiCfoJob jb = jobs[blockIdx.y];
  const float k = -2.0f * jb.cfo / (float)N;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < len; i += gridDim.x * 256) {
    const float2 a = src[jb.src + i];
    float s, c;
    sincospif(k * (float)i, &s, &c);
    dst[jb.dst + i] = make_float2(a.x * c - a.y * s, a.x * s + a.y * c);
  }
}

void launch_pss_search(const float2* iq, const float2* tmpl, const MiPssJob* jobs, MiPssRes* res, uint32_t n, uint32_t N,
                       uint32_t max_nlag, hipStream_t st) {
  if (!n) return;
  // threads per lag from the (host-known) largest window: 64 lags or fewer -> 4, 128 or fewer -> 2
  const size_t lds = 3 * N * sizeof(float2);
  if (max_nlag <= PSS_T / 4)
    hipLaunchKernelGGL(pss_search_kernel<4>, dim3(n), dim3(PSS_T), lds, st, iq, tmpl, jobs, res, N);
  else if (max_nlag <= PSS_T / 2)
    hipLaunchKernelGGL(pss_search_kernel<2>, dim3(n), dim3(PSS_T), lds, st, iq, tmpl, jobs, res, N);
  else
    hipLaunchKernelGGL(pss_search_kernel<1>, dim3(n), dim3(PSS_T), lds, st, iq, tmpl, jobs, res, N);
}
void launch_sss_detect(const float2* iq, const MiSssJob* jobs, MiSssRes* res, uint32_t n, uint32_t N, uint32_t nof_prb,
                       uint32_t l5, uint32_t l6, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(sss_detect_kernel, dim3(n), dim3(256), 3 * N * sizeof(float2), st, iq, jobs, res, N, nof_prb,
                     l5, l6);
}
void launch_cfo_correct(const float2* src, float2* dst, const MiCfoJob* jobs, uint32_t n, uint32_t len, uint32_t N,
                        hipStream_t st) {
  if (!n || !len) return;
  const uint32_t gx = std::min<uint32_t>((len + 255) / 256, 32);
  hipLaunchKernelGGL(cfo_correct_kernel, dim3(gx, n), dim3(256), 0, st, src, dst, jobs, len, N);
}

}  // namespace mi
