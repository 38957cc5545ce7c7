// rm.hip -- rate de-matching + HARQ combine into the group-interleaved softbuffer [Ncb][64 lanes].
//
// Semantics: rm_body.h (bit-identical to the serial srslte_rm_turbo_rx loop).  MI355X layout: one
// 256-thread workgroup owns RM_CHUNK circular-buffer positions of one 64-code-block group.  The
// positions of a chunk receive a contiguous run of each code block's LLRs (the non-null ranks of
// the chunk, modulo N_v), so the workgroup first stages, per lane, that run of e into an LDS tile
// with coalesced loads (consecutive threads on consecutive LLRs of one code block), then every
// wavefront combines one position for all 64 lanes: softbuffer rows are read and written as 256-B
// coalesced rows and the LLRs come from LDS (row stride RM_CHUNK + 1 floats: conflict-free column
// reads).  No integer division in the loops: ranks are rebased with one conditional add.
// Repetition beyond N_v (E > N_v, low code rates) adds the further copies from HBM in order.
#include "kernels.h"
#include "rm_body.h"

namespace mi {

__global__ __launch_bounds__(256) void rm_combine_kernel(const float* __restrict__ e, float* __restrict__ sb,
                                                        const MiGroupDesc* __restrict__ groups,
                                                        const MiLaneDesc* __restrict__ lanes,
                                                        const uint32_t* __restrict__ kdata) {
  __shared__ float tile[LANES][RM_CHUNK + 1];
  __shared__ uint32_t s_j0[LANES], s_nr[LANES], s_nv[LANES], s_E[LANES];
  __shared__ uint64_t s_eoff[LANES];
  const MiGroupDesc g = groups[blockIdx.y];
  const uint32_t pa = blockIdx.x * RM_CHUNK;
  if (pa >= g.Ncb) return;
  const uint32_t tid = threadIdx.x;
  if (tid < LANES) {
    const MiLaneDesc ld = lanes[g.lane0 + tid];
    uint32_t j0 = 0, nr = 0;
    if (ld.valid) {
      const uint32_t* ch = kdata + ld.rank_off + g.Ncb;
      const uint32_t ra = ch[pa / RM_CHUNK];
      nr = ch[pa / RM_CHUNK + 1] - ra;
      j0 = ra >= ld.r0 ? ra - ld.r0 : ra + ld.Nv - ld.r0;   // LLR index of the chunk's first rank
    }
    s_j0[tid] = j0; s_nr[tid] = nr; s_nv[tid] = ld.Nv; s_E[tid] = ld.E; s_eoff[tid] = ld.e_off;
  }
  __syncthreads();
  // stage: tile[l][t] = e_l[(j0 + t) mod Nv] (0 beyond E), t < nr; 64 threads per code-block row
  for (uint32_t l = tid >> 6; l < (uint32_t)LANES; l += 4) {
    const uint32_t nr = s_nr[l], nv = s_nv[l], E = s_E[l];
    const float* el = e + s_eoff[l];
    uint32_t j = s_j0[l] + (tid & 63);
    if (j >= nv) j -= nv;
    for (uint32_t t = tid & 63; t < nr; t += 64) {
      tile[l][t] = j < E ? el[j] : 0.0f;
      j += 64;
      if (j >= nv) j -= nv;
    }
  }
  __syncthreads();
  const int lane = (int)(tid & 63), wave = (int)(tid >> 6);
  const MiLaneDesc ld = lanes[g.lane0 + lane];
  if (!ld.valid) return;
  const int32_t* rank = reinterpret_cast<const int32_t*>(kdata + ld.rank_off);
  float* sbg = sb + g.sb_off;
  const uint32_t* ch = kdata + ld.rank_off + g.Ncb;
  const uint32_t ra = ch[pa / RM_CHUNK];
  const uint32_t j0 = s_j0[lane], nv = ld.Nv, E = ld.E;
  const bool rep = E > nv;
  for (uint32_t i = (uint32_t)wave; i < (uint32_t)RM_CHUNK; i += 4) {
    const uint32_t p = pa + i;
    if (p >= g.Ncb) break;
    const int32_t rk = rank[p];
    float v = ld.new_tb ? 0.0f : sbg[(size_t)p * LANES + lane];
    if (rk >= 0) {
      const uint32_t t = (uint32_t)rk - ra;
      uint32_t j = j0 + t;
      if (j >= nv) j -= nv;
      if (j < E) v = v + tile[lane][t];
      if (rep)
        for (j += nv; j < E; j += nv) v = v + e[ld.e_off + j];
    }
    sbg[(size_t)p * LANES + lane] = v;
  }
}

void launch_rm_combine(const float* e, float* sb, const MiGroupDesc* groups, const MiLaneDesc* lanes,
                       const MiKTab* /*ktabs*/, const uint32_t* ktab_data, uint32_t n_groups, uint32_t max_ncb,
                       hipStream_t st) {
  if (!n_groups) return;
  dim3 g((max_ncb + RM_CHUNK - 1) / RM_CHUNK, n_groups);
  hipLaunchKernelGGL(rm_combine_kernel, g, dim3(256), 0, st, e, sb, groups, lanes, ktab_data);
}

}  // namespace mi
