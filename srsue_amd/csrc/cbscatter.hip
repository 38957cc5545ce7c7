// cbscatter.hip -- raw code-block input for the turbo decoder (srslte_tdec_iteration's input
// contract, BASELINE configs[0] = srsLTE turbodecoder_test): decoder inputs d[cb][3(K+4)] in
// triplet order are written into the group-interleaved layout [N_cb][64] the turbo kernel reads,
// through the same per-K position table (LDS transpose: coalesced reads of each code block's row,
// 256-B coalesced row writes); every row is materialised in the sparse-row map.
#include "kernels.h"

namespace mi {

constexpr int SC_T = 64;   // decoder-input elements per workgroup

__global__ __launch_bounds__(256) void cb_scatter_kernel(const float* __restrict__ d, float* __restrict__ sb,
                                                        const MiGroupDesc* __restrict__ groups,
                                                        const MiKTab* __restrict__ ktabs,
                                                        const uint32_t* __restrict__ kdata, uint32_t n_cb) {
  __shared__ float tile[LANES][SC_T + 1];
  const MiGroupDesc g = groups[blockIdx.y];
  const uint32_t T = 3 * (g.K + 4), t0 = blockIdx.x * SC_T;
  if (t0 >= T) return;
  const uint32_t tid = threadIdx.x, q = tid & 63, w = tid >> 6;
  for (uint32_t l = w; l < (uint32_t)LANES; l += 4) {
    const uint32_t cb = g.lane0 + l;
    tile[l][q] = (cb < n_cb && t0 + q < T) ? d[(size_t)cb * T + t0 + q] : 0.0f;
  }
  __syncthreads();
  float* sbg = sb + g.sb_off;
  for (uint32_t i = w; i < (uint32_t)SC_T; i += 4) {
    const uint32_t t = t0 + i;
    if (t < T) sbg[(size_t)t * LANES + q] = tile[q][i];   // rows in decoder-input order (dl_common.h)
  }
  if (blockIdx.x == 0) {   // every row written: the whole map materialised, plus the zero row
    uint8_t* map = reinterpret_cast<uint8_t*>(sbg + sb_map_off(g.Ncb));
    for (uint32_t p = tid; p < g.Ncb; p += 256) map[p] = 1;
    if (tid < LANES) sbg[(size_t)g.Ncb * LANES + tid] = 0.0f;
  }
}

void launch_cb_scatter(const float* d, float* sb, const MiGroupDesc* groups, const MiKTab* ktabs,
                       const uint32_t* kdata, uint32_t n_groups, uint32_t K, uint32_t n_cb, hipStream_t st) {
  if (!n_groups) return;
  dim3 g((3 * (K + 4) + SC_T - 1) / SC_T, n_groups);
  hipLaunchKernelGGL(cb_scatter_kernel, g, dim3(256), 0, st, d, sb, groups, ktabs, kdata, n_cb);
}

}  // namespace mi
