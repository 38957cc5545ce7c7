// chest.hip -- downlink CRS channel estimation (replaces srslte_chest_dl_estimate inside
// srslte_ue_dl_decode_fft_estimate, /root/reference/ue/src/phy/phch_worker.cc:254, and backs the
// srslte_chest_dl_get_{rsrp,rssi,rsrq,noise_estimate,snr} getters read at :359, :799-848).
//
// One 256-thread workgroup per subframe.  Per port: LS estimate on the 4 pilot symbols
// (p = y conj(r), CRS r from a per-cell device table), 3-tap smoothing [0.1 0.8 0.1] with edge
// taps renormalised; then each thread owns subcarriers k: linear interpolation in frequency of the
// 4 pilot symbols at k (registers), linear interpolation / extrapolation in time straight to HBM
// (coalesced rows of ce[port][l][k]).  LDS holds only the pilot rows (14 KB): 8 workgroups per CU.
// Metrics are reduced in the workgroup (wave shuffles + LDS) and written once per subframe.
#include "kernels.h"

namespace mi {

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); i++) s += red[i];
  return s;
}

__global__ __launch_bounds__(256) void chest_kernel(const float2* __restrict__ grid, float2* __restrict__ ce,
                                                   const MiSfDesc* __restrict__ sfs,
                                                   const MiCellDesc* __restrict__ cells,
                                                   const float2* __restrict__ crs, float* __restrict__ metrics,
                                                   uint32_t compact) {
  constexpr int PL[4] = {0, 4, 7, 11};
  constexpr float W1 = 0.1f, W0 = 0.8f;
  __shared__ float2 hp[4][2 * NRB_MAX];
  __shared__ float2 hs[4][2 * NRB_MAX];
  __shared__ float red[4];
  const MiSfDesc d = sfs[blockIdx.x];
  const MiCellDesc c = cells[d.cell];
  const int W = (int)c.W, NP = 2 * (int)c.nof_prb;
  const float2* g = grid + d.grid_off;
  float rsrp = 0.f, noise = 0.f, rssi = 0.f;
  // every loop runs over (uniform row, thread-strided column): no integer division by runtime sizes
  const int tid = (int)threadIdx.x;
  for (int p = 0; p < (int)c.nof_ports; p++) {
    int offs[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int lp = PL[i] % 7;
      const int v = (p == 0) ? (lp == 0 ? 0 : 3) : (lp == 0 ? 3 : 0);
      offs[i] = (v + (int)(c.id % 6)) % 6;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int l = PL[i], lp = l % 7;
      const float2* rr = crs + c.crs_off + ((2 * d.sf_idx + l / 7) * 2 + (lp == 4)) * (2 * NRB_MAX) + NRB_MAX - c.nof_prb;
      for (int m = tid; m < NP; m += 256) {
        const float2 y = g[l * W + 6 * m + offs[i]];
        const float2 r = rr[m];
        const float2 h = make_float2(y.x * r.x + y.y * r.y, y.y * r.x - y.x * r.y);
        hp[i][m] = h;
        if (p == 0) rsrp += h.x * h.x + h.y * h.y;
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; i++) {
      for (int m = tid; m < NP; m += 256) {
        float2 s;
        if (m == 0) {
          s = make_float2((W0 * hp[i][0].x + W1 * hp[i][1].x) / (W0 + W1), (W0 * hp[i][0].y + W1 * hp[i][1].y) / (W0 + W1));
        } else if (m == NP - 1) {
          s = make_float2((W1 * hp[i][m - 1].x + W0 * hp[i][m].x) / (W0 + W1), (W1 * hp[i][m - 1].y + W0 * hp[i][m].y) / (W0 + W1));
        } else {
          s = make_float2(W1 * hp[i][m - 1].x + W0 * hp[i][m].x + W1 * hp[i][m + 1].x,
                          W1 * hp[i][m - 1].y + W0 * hp[i][m].y + W1 * hp[i][m + 1].y);
        }
        hs[i][m] = s;
        const float dx = hp[i][m].x - s.x, dy = hp[i][m].y - s.y;
        noise += dx * dx + dy * dy;
      }
    }
    __syncthreads();
    // frequency interpolation of the 4 pilot symbols at subcarrier k (kept in registers), then the
    // time interpolation / extrapolation of all 14 symbols at k: coalesced rows of ce[port][l][k]
    // compact (MI_DL_FLAG_CE_COMPACT): the 4 frequency-interpolated pilot rows [port][4][W] only
    float2* cp = ce + d.ce_off + (size_t)p * (compact ? 4 : NSYMB) * W;
    for (int k = tid; k < W; k += 256) {
      float2 hk[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int off = offs[i];
        int m = (k - off) / 6;
        if (k < off) m = 0;
        if (m > NP - 2) m = NP - 2;
        const float frac = (float)(k - (6 * m + off)) / 6.0f;
        const float2 a = hs[i][m], b = hs[i][m + 1];
        hk[i] = make_float2(a.x + frac * (b.x - a.x), a.y + frac * (b.y - a.y));
      }
      if (compact) {
#pragma unroll
        for (int i = 0; i < 4; i++) cp[i * W + k] = hk[i];
        continue;
      }
#pragma unroll
      for (int l = 0; l < NSYMB; l++) cp[l * W + k] = ce_time_interp(hk[ce_ia(l)], hk[ce_ia(l) + 1], CE_TT[l]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; i++)
    for (int k = tid; k < W; k += 256) {
      const float2 y = g[PL[i] * W + k];
      rssi += y.x * y.x + y.y * y.y;
    }
  rsrp = block_sum(rsrp, red);
  noise = block_sum(noise, red);
  rssi = block_sum(rssi, red);
  if (threadIdx.x == 0) {
    const float rs = rsrp / (float)(4 * NP), no = noise / (float)(4 * NP * c.nof_ports), ri = rssi / 4.0f;
    float* m = metrics + (size_t)blockIdx.x * 5;
    m[0] = rs; m[1] = ri; m[2] = ri > 0.f ? (float)c.nof_prb * rs / ri : 0.f;
    m[3] = no; m[4] = no > 0.f ? rs / no : 0.f;
  }
}

void launch_chest(const float2* grid, float2* ce, const MiSfDesc* sfs, const MiCellDesc* cells, const float2* crs,
                  float* metrics, uint32_t n_sf, hipStream_t st, bool compact) {
  if (!n_sf) return;
  hipLaunchKernelGGL(chest_kernel, dim3(n_sf), dim3(256), 0, st, grid, ce, sfs, cells, crs, metrics,
                     (uint32_t)compact);
}

}  // namespace mi
