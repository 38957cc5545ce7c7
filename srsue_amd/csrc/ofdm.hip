// ofdm.hip -- OFDM demodulation (replaces srslte_ofdm_rx_sf inside srslte_ue_dl_decode_fft_estimate,
// /root/reference/ue/src/phy/phch_worker.cc:254).
//
// One 256-thread workgroup per subframe runs the 14 symbol FFTs back to back: the first Stockham
// stage reads the IQ straight from HBM with consecutive lanes on consecutive samples (coalesced),
// the remaining radix-8/4/3 stages exchange through one LDS buffer, and the twiddles
// exp(-2 pi i t / N) (a half-wave table, tw_at) are staged into LDS once per workgroup and reused by all
// 14 symbols.  The
// last pass writes the 12 N_RB used subcarriers (DC skipped) row-major [symbol][subcarrier].
// Unnormalised forward DFT (oracle/o_rx.c convention).
#include "kernels.h"

namespace mi {

__device__ __forceinline__ float2 c_add(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 c_sub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 c_mul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 c_mul_nj(float2 a) { return make_float2(a.y, -a.x); }   // * (-j)

__device__ __forceinline__ void dft2(float2& a, float2& b) { float2 t = a; a = c_add(t, b); b = c_sub(t, b); }

__device__ __forceinline__ void dft4(float2& a, float2& b, float2& c, float2& d) {
  float2 t0 = c_add(a, c), t1 = c_sub(a, c), t2 = c_add(b, d), t3 = c_sub(b, d);
  a = c_add(t0, t2);
  c = c_sub(t0, t2);
  b = make_float2(t1.x + t3.y, t1.y - t3.x);   // t1 - j t3
  d = make_float2(t1.x - t3.y, t1.y + t3.x);   // t1 + j t3
}

template <int R> __device__ __forceinline__ void dft(float2 (&v)[R]);

template <> __device__ __forceinline__ void dft<2>(float2 (&v)[2]) { dft2(v[0], v[1]); }
template <> __device__ __forceinline__ void dft<4>(float2 (&v)[4]) { dft4(v[0], v[1], v[2], v[3]); }
template <> __device__ __forceinline__ void dft<3>(float2 (&v)[3]) {
  const float s = 0.86602540378443864676f;
  float2 a = v[0], t = c_add(v[1], v[2]), u = c_sub(v[1], v[2]);
  float2 m = make_float2(a.x - 0.5f * t.x, a.y - 0.5f * t.y);
  v[0] = c_add(a, t);
  v[1] = make_float2(m.x + s * u.y, m.y - s * u.x);
  v[2] = make_float2(m.x - s * u.y, m.y + s * u.x);
}
template <> __device__ __forceinline__ void dft<8>(float2 (&v)[8]) {
  float2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
  float2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
  dft4(e0, e1, e2, e3);
  dft4(o0, o1, o2, o3);
  const float r = 0.70710678118654752440f;
  o1 = make_float2((o1.x + o1.y) * r, (o1.y - o1.x) * r);     // * (1-j)/sqrt2
  o2 = c_mul_nj(o2);                                          // * -j
  o3 = make_float2((o3.y - o3.x) * r, (-o3.x - o3.y) * r);    // * (-1-j)/sqrt2
  v[0] = c_add(e0, o0); v[4] = c_sub(e0, o0);
  v[1] = c_add(e1, o1); v[5] = c_sub(e1, o1);
  v[2] = c_add(e2, o2); v[6] = c_sub(e2, o2);
  v[3] = c_add(e3, o3); v[7] = c_sub(e3, o3);
}

// Padded LDS layout of the first stage's output: float2 index a -> a + a / 32 (one pad slot per 32).  Thread j
// writes 8 j + r (r < 8), which with ds_write_b64's 16-lane groups and 32 banks is an 8-way conflict; the pad
// spreads it (LDS write cycles per 2048-point FFT 1,536 -> 768, the minimum being 512; the second stage's reads
// stay conflict-free; bank model of MI355X_MICROARCH.md 'LDS').  Only this one buffer hand-off is padded, and
// both sides keep immediate offsets: 8 j + r -> (8 j + j / 4) + r, and j + r NB -> (j + j / 32) + r (NB + NB / 32)
// since every NB here is a multiple of 32 -- no address registers are added (an XOR swizzle, 640 cycles,
// needed one per access and spilled).
constexpr int OFDM_PAD_SH = 5;
__device__ __forceinline__ int lpad(int a) { return a + (a >> OFDM_PAD_SH); }

// One Stockham stage (decimation in time): butterfly j reads x[j + r N/R], twiddles by
// W_{Ns R}^{(j mod Ns) r}, writes y[(j / Ns) Ns R + j mod Ns + r Ns].
// IQ sample i of a symbol: fc32, or UHD sc16 (fc32 = sc16 / 32768, exact in fp32) -- MI_DL_FLAG_IQ_SC16
__device__ __forceinline__ float2 load_iq(const float2* __restrict__ p, int i) { return p[i]; }
__device__ __forceinline__ float2 load_iq(const short2* __restrict__ p, int i) {
  const short2 v = p[i];
  return make_float2((float)v.x * (1.0f / 32768.0f), (float)v.y * (1.0f / 32768.0f));
}

// twiddle W_N^t from the half-wave table tw2[t mod N/2] (t < N): W_N^(t0 + N/2) = -W_N^t0.  The LDS holds N/2
// entries instead of N: for N = 2048 the workgroup needs 24 KB instead of 32 KB of LDS (6 instead of 5
// workgroups per CU) and stages 8 KB of twiddles instead of 16.
template <int N>
__device__ __forceinline__ float2 tw_at(const float2* tw2, int t) {
  constexpr int H = N / 2;
  const bool hi = t >= H;
  const float2 w = tw2[hi ? t - H : t];
  return hi ? make_float2(-w.x, -w.y) : w;
}

template <int N, int R, bool FIRST, typename IQ, bool PAD_IN = false>   // PAD_IN: the input was written padded
__device__ __forceinline__ void fft_stage(float2* buf, const IQ* __restrict__ gsrc, const float2* tw, int Ns) {
  constexpr int NB = N / R;
  constexpr int PER = (NB + 255) / 256;
  const int tid = threadIdx.x;
  float2 v[PER][R];
#pragma unroll
  for (int p = 0; p < PER; p++) {
    const int j = tid + p * 256;
    if (j < NB) {
#pragma unroll
      for (int r = 0; r < R; r++) {
        if constexpr (FIRST) {
          v[p][r] = load_iq(gsrc, j + r * NB);
        } else if constexpr (PAD_IN) {
          static_assert(NB % (1 << OFDM_PAD_SH) == 0, "padded hand-off: NB a multiple of 32");
          v[p][r] = buf[lpad(j) + r * lpad(NB)];
        } else {
          v[p][r] = buf[j + r * NB];
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < PER; p++) {
    const int j = tid + p * 256;
    if (j < NB) {
      const int k = j % Ns;
      if (!FIRST) {
        const int step = k * (N / (Ns * R));
#pragma unroll
        for (int r = 1; r < R; r++) v[p][r] = c_mul(v[p][r], tw_at<N>(tw, step * r));
      }
      dft<R>(v[p]);
      const int base = (j / Ns) * Ns * R + k;
#pragma unroll
      for (int r = 0; r < R; r++) buf[base + r * Ns] = v[p][r];
    }
  }
  __syncthreads();
}

// The first stage (radix 8 for every size) reads the symbol's IQ straight from HBM.  Its loads are split
// off (FirstIn / first_load) so the subframe loop can issue the NEXT symbol's loads before the current
// symbol's LDS stages run: the HBM latency of every symbol but the first hides behind a symbol of work.
template <int N>
struct FirstIn {
  static constexpr int NB = N / 8, PER = (NB + 255) / 256;
  float2 v[PER][8];
};
template <int N, typename IQ>
__device__ __forceinline__ void first_load(const IQ* __restrict__ src, FirstIn<N>& f) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int p = 0; p < FirstIn<N>::PER; p++) {
    const int j = tid + p * 256;
    if (j < FirstIn<N>::NB) {
#pragma unroll
      for (int r = 0; r < 8; r++) f.v[p][r] = load_iq(src, j + r * FirstIn<N>::NB);
    }
  }
}
// fft_stage<N, 8, true> on loaded values (Ns = 1: no twiddles); the caller synchronised buf's readers
template <int N>
__device__ __forceinline__ void first_stage(float2* buf, FirstIn<N>& f) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int p = 0; p < FirstIn<N>::PER; p++) {
    const int j = tid + p * 256;
    if (j < FirstIn<N>::NB) {
      dft<8>(f.v[p]);
      const int L = lpad(j * 8);   // lpad(8 j + r) = lpad(8 j) + r for r < 8
#pragma unroll
      for (int r = 0; r < 8; r++) buf[L + r] = f.v[p][r];
    }
  }
  __syncthreads();
}
// the stages after the first
template <int N, typename IQ>
__device__ __forceinline__ void fft_rest(float2* buf, const float2* tw) {
  if constexpr (N == 2048) {
    fft_stage<N, 8, false, IQ, true>(buf, nullptr, tw, 8); fft_stage<N, 8, false, IQ>(buf, nullptr, tw, 64);
    fft_stage<N, 4, false, IQ>(buf, nullptr, tw, 512);
  } else if constexpr (N == 1536) {
    fft_stage<N, 8, false, IQ, true>(buf, nullptr, tw, 8); fft_stage<N, 8, false, IQ>(buf, nullptr, tw, 64);
    fft_stage<N, 3, false, IQ>(buf, nullptr, tw, 512);
  } else if constexpr (N == 1024) {
    fft_stage<N, 8, false, IQ, true>(buf, nullptr, tw, 8); fft_stage<N, 4, false, IQ>(buf, nullptr, tw, 64);
    fft_stage<N, 4, false, IQ>(buf, nullptr, tw, 256);
  } else if constexpr (N == 512) {
    fft_stage<N, 8, false, IQ, true>(buf, nullptr, tw, 8); fft_stage<N, 8, false, IQ>(buf, nullptr, tw, 64);
  } else if constexpr (N == 256) {
    fft_stage<N, 8, false, IQ, true>(buf, nullptr, tw, 8); fft_stage<N, 4, false, IQ>(buf, nullptr, tw, 64);
  } else {
    static_assert(N == 128, "unsupported FFT size");
    fft_stage<N, 4, false, IQ, true>(buf, nullptr, tw, 8); fft_stage<N, 4, false, IQ>(buf, nullptr, tw, 32);
  }
}

// symbols [blockIdx.y * per, (blockIdx.y + 1) * per) of a subframe: per = 14 (one workgroup per
// subframe, twiddles staged once for 14 FFTs -- batches) or 1 (a workgroup per symbol -- small batches,
// the per-TTI latency path)
// 6 waves per SIMD: the VGPR budget (<= 80) that matches the 6 workgroups per CU the LDS now allows
constexpr int OFDM_WAVES = 6;
template <int N, typename IQ>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OFDM_WAVES))) void ofdm_rx_kernel(const IQ* __restrict__ iq, float2* __restrict__ grid,
                                                      const MiSfDesc* __restrict__ sfs,
                                                      const uint32_t* __restrict__ list,
                                                      const float2* __restrict__ twg, uint32_t W, int per) {
  __shared__ float2 buf[N + (N >> OFDM_PAD_SH)];
  __shared__ float2 tw[N / 2];   // half-wave table (tw_at)
  const MiSfDesc d = sfs[list[blockIdx.x]];
  for (int t = threadIdx.x; t < N / 2; t += 256) tw[t] = twg[t];
  __syncthreads();
  const IQ* src_sf = iq + d.iq_off;
  float2* dst = grid + d.grid_off;
  const int l0 = (int)blockIdx.y * per;
  FirstIn<N> cur, nxt;
  first_load<N, IQ>(src_sf + symbol_offset(N, l0), nxt);
  for (int l = l0; l < l0 + per; l++) {
    cur = nxt;
    if (l + 1 < l0 + per) first_load<N, IQ>(src_sf + symbol_offset(N, l + 1), nxt);   // in flight meanwhile
    first_stage<N>(buf, cur);
    fft_rest<N, IQ>(buf, tw);
    for (int k = threadIdx.x; k < (int)W; k += 256) dst[l * W + k] = buf[sc_bin(k, (int)W, N)];
    __syncthreads();
  }
}

template <typename IQ>
static void launch_ofdm_rx_t(int N, const IQ* iq, float2* grid, const MiSfDesc* sfs, const uint32_t* list, uint32_t n,
                             const float2* tw, uint32_t W, hipStream_t st) {
  const int per = n >= 256 ? NSYMB : 1;   // small batches: a workgroup per symbol (latency)
  dim3 g(n, NSYMB / per), b(256);
  switch (N) {
    case 2048: hipLaunchKernelGGL((ofdm_rx_kernel<2048, IQ>), g, b, 0, st, iq, grid, sfs, list, tw, W, per); break;
    case 1536: hipLaunchKernelGGL((ofdm_rx_kernel<1536, IQ>), g, b, 0, st, iq, grid, sfs, list, tw, W, per); break;
    case 1024: hipLaunchKernelGGL((ofdm_rx_kernel<1024, IQ>), g, b, 0, st, iq, grid, sfs, list, tw, W, per); break;
    case 512: hipLaunchKernelGGL((ofdm_rx_kernel<512, IQ>), g, b, 0, st, iq, grid, sfs, list, tw, W, per); break;
    case 256: hipLaunchKernelGGL((ofdm_rx_kernel<256, IQ>), g, b, 0, st, iq, grid, sfs, list, tw, W, per); break;
    case 128: hipLaunchKernelGGL((ofdm_rx_kernel<128, IQ>), g, b, 0, st, iq, grid, sfs, list, tw, W, per); break;
    default: break;
  }
}

void launch_ofdm_rx(int N, const void* iq, bool sc16, float2* grid, const MiSfDesc* sfs, const uint32_t* list,
                    uint32_t n, const float2* tw, uint32_t W, hipStream_t st) {
  if (n == 0) return;
  if (sc16) launch_ofdm_rx_t(N, static_cast<const short2*>(iq), grid, sfs, list, n, tw, W, st);
  else launch_ofdm_rx_t(N, static_cast<const float2*>(iq), grid, sfs, list, n, tw, W, st);
}

}  // namespace mi
