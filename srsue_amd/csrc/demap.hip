// demap.hip -- PDSCH RE gather + equalisation + max-log soft demapping + descrambling.
//
// Replaces, inside srslte_pdsch_decode_rnti (/root/reference/ue/src/phy/phch_worker.cc:347-348,
// noise_estimate = 0.01 from :340): srslte_pdsch_get (RE gather), srslte_predecoding_single /
// srslte_predecoding_diversity + layerdemap (TM1 / TM2 SFBC), srslte_demod_soft_demodulate
// (max-log, sigma^2 = 0.5, LLR > 0 => bit 1) and srslte_scrambling_f (c(i) = 1 flips the sign).
//
// One lane per RE (TM1) or per SFBC RE pair (TM2).  The RE list (36.211 6.3.5 mapping order) is
// a per-configuration device table, so grid/ce reads walk consecutive subcarriers and every lane
// writes its Qm LLRs contiguously (float2 stores): the LLR stream leaves fully coalesced.
#include "demap_body.h"
#include "kernels.h"

namespace mi {

template <int QM>
__device__ __forceinline__ void demap_store(float2 x, const uint32_t* __restrict__ scr, uint32_t bit0,
                                            float* __restrict__ out) {
  float l[QM];
  demap_dim<QM>(x.x, l);
  demap_dim<QM>(x.y, l + 1);
#pragma unroll
  for (int b = 0; b < QM; b++) {
    const uint32_t i = bit0 + b;
    if ((scr[i >> 5] >> (i & 31)) & 1u) l[b] = -l[b];
  }
  float2* o = reinterpret_cast<float2*>(out + bit0);
#pragma unroll
  for (int b = 0; b < QM; b += 2) o[b / 2] = make_float2(l[b], l[b + 1]);
}

template <int QM>
__device__ __forceinline__ void demap_unit(const MiPdschDesc& pd, uint32_t u, const float2* __restrict__ g,
                                           const float2* __restrict__ c0, const float2* __restrict__ c1,
                                           const uint32_t* __restrict__ re, const uint32_t* __restrict__ scr,
                                           float* __restrict__ e, float noise) {
  if (pd.tm != 2) {
    const uint32_t r = re[u];
    demap_store<QM>(eq_single(g[r], c0[r], noise), scr, u * QM, e);
  } else {
    const uint32_t ra = re[2 * u], rb = re[2 * u + 1];
    float2 x0, x1;
    eq_sfbc(g[ra], g[rb], c0[ra], c0[rb], c1[ra], c1[rb], &x0, &x1);
    demap_store<QM>(x0, scr, 2 * u * QM, e);
    demap_store<QM>(x1, scr, (2 * u + 1) * QM, e);
  }
}

__global__ __launch_bounds__(256) void demap_kernel(const float2* __restrict__ grid, const float2* __restrict__ ce,
                                                   float* __restrict__ e, const MiSfDesc* __restrict__ sfs,
                                                   const MiPdschDesc* __restrict__ pds,
                                                   const MiCellDesc* __restrict__ cells,
                                                   const uint32_t* __restrict__ re_tab,
                                                   const uint32_t* __restrict__ scr_tab, float noise) {
  const MiSfDesc d = sfs[blockIdx.y];
  const MiPdschDesc pd = pds[d.pdsch];
  const uint32_t units = pd.tm == 2 ? pd.nre / 2 : pd.nre;
  const uint32_t u = blockIdx.x * 256 + threadIdx.x;
  if (u >= units) return;
  const MiCellDesc c = cells[d.cell];
  const float2* g = grid + d.grid_off;
  const float2* c0 = ce + d.ce_off;
  const float2* c1 = c0 + (size_t)NSYMB * c.W;
  const uint32_t* re = re_tab + pd.re_off;
  const uint32_t* scr = scr_tab + pd.scr_off;
  float* out = e + d.e_off;
  switch (pd.Qm) {
    case 2: demap_unit<2>(pd, u, g, c0, c1, re, scr, out, noise); break;
    case 4: demap_unit<4>(pd, u, g, c0, c1, re, scr, out, noise); break;
    default: demap_unit<6>(pd, u, g, c0, c1, re, scr, out, noise); break;
  }
}

void launch_demap(const float2* grid, const float2* ce, float* e, const MiSfDesc* sfs, const MiPdschDesc* pd,
                  const MiCellDesc* cells, const uint32_t* re_tab, const uint32_t* scr, uint32_t n_sf,
                  uint32_t max_units, float noise, hipStream_t st) {
  if (!n_sf || !max_units) return;
  dim3 g((max_units + 255) / 256, n_sf);
  hipLaunchKernelGGL(demap_kernel, g, dim3(256), 0, st, grid, ce, e, sfs, pd, cells, re_tab, scr, noise);
}

}  // namespace mi
