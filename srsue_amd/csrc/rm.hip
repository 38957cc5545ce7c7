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
//
// Sparse rows (dl_common.h sb_group_floats): a row is written only when some lane receives an LLR
// there or a combining lane keeps a materialised history; each wavefront owns 32 consecutive rows,
// whose map bytes it reads and rewrites with one 32-byte access (the bits live in a scalar register
// in between).  A chunk that receives nothing and holds nothing exits after its first barrier.
// Punctured positions of a first transmission (60 % of the circular buffer at MCS 28) thus cost no
// HBM traffic, here or in the decoder.
#include "kernels.h"
#include "rm_body.h"

#ifndef MI_RM_NT
#define MI_RM_NT 0   // non-temporal softbuffer stores (A/B switch)
#endif
#ifndef MI_RM_DENSE
#define MI_RM_DENSE 0   // A/B switch: write and materialise every row (the pre-sparse behaviour)
#endif

namespace mi {

__global__ __launch_bounds__(256) void rm_combine_kernel(const float* __restrict__ e, float* __restrict__ sb,
                                                        const MiGroupDesc* __restrict__ groups,
                                                        const MiLaneDesc* __restrict__ lanes,
                                                        const uint32_t* __restrict__ kdata) {
  __shared__ float tile[LANES][RM_CHUNK + 1];
  __shared__ uint32_t s_j0[LANES], s_nr[LANES], s_nv[LANES], s_E[LANES];
  __shared__ uint64_t s_eoff[LANES];
  __shared__ uint32_t s_comb, s_new;
  const MiGroupDesc g = groups[blockIdx.y];
  const uint32_t pa = blockIdx.x * RM_CHUNK;
  if (pa >= g.Ncb) return;
  const uint32_t tid = threadIdx.x;
  float* sbg = sb + g.sb_off;
  uint8_t* map = reinterpret_cast<uint8_t*>(sbg + sb_map_off(g.Ncb)) + pa;   // map rounded up to 256 B
  int busy = 0;
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
    // does any LLR of this lane land in the chunk (LLR indices j0 .. j0+nr-1 mod Nv against [0, E))?
    busy = nr > 0 && (ld.E >= ld.Nv || j0 < ld.E || j0 + nr > ld.Nv);
    const uint64_t comb = __ballot(ld.valid && !ld.new_tb), fresh = __ballot(ld.valid && ld.new_tb);
    if (tid == 0) { s_comb = comb != 0; s_new = fresh != 0; }
    if (blockIdx.x == 0) sbg[(size_t)g.Ncb * LANES + tid] = 0.0f;   // the group's zero row
  }
  if (tid < RM_CHUNK / 4) busy |= reinterpret_cast<const uint32_t*>(map)[tid] != 0;
  // nothing received and nothing materialised: the chunk stays all-zero, no HBM traffic
  if (!__syncthreads_or(busy)) return;
  // stage: tile[l][t] = e_l[(j0 + t) mod Nv] (0 beyond E), t < nr; a wavefront per code-block row,
  // all of a wavefront's loads issued before its LDS writes
  constexpr int ROWS = LANES / 4, PER = RM_CHUNK / 64;
  {
    float v[ROWS][PER];
    const uint32_t w = tid >> 6, q = tid & 63;
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
      const uint32_t l = w + 4 * r;
      const uint32_t nr = s_nr[l], nv = s_nv[l], E = s_E[l];
      const float* el = e + s_eoff[l];
#pragma unroll
      for (int c = 0; c < PER; c++) {
        const uint32_t t = q + 64 * c;
        uint32_t j = s_j0[l] + t;
        if (j >= nv) j -= nv;
        v[r][c] = (t < nr && j < E) ? el[j] : 0.0f;
      }
    }
#pragma unroll
    for (int r = 0; r < ROWS; r++)
#pragma unroll
      for (int c = 0; c < PER; c++) tile[w + 4 * r][q + 64 * c] = v[r][c];
  }
  __syncthreads();
  // combine: wavefront w owns the NP consecutive positions pw .. pw+NP-1, one row (64 lanes) each
  constexpr int NP = RM_CHUNK / 4;
  const int lane = (int)(tid & 63), wave = (int)(tid >> 6);
  const uint32_t pw = pa + NP * (uint32_t)wave, np = g.Ncb > pw ? min(g.Ncb - pw, (uint32_t)NP) : 0u;
  const MiLaneDesc ld = lanes[g.lane0 + lane];
  const int32_t* rank = reinterpret_cast<const int32_t*>(kdata + ld.rank_off);
  const uint32_t* ch = kdata + ld.rank_off + g.Ncb;
  const uint32_t ra = ld.valid ? ch[pa / RM_CHUNK] : 0;
  const uint32_t j0 = s_j0[lane], nv = ld.Nv, E = ld.E;
  const bool rep = E > nv, comb = s_comb, fresh = s_new;
  // materialised-before bits of the wave's rows (wave-uniform)
  const uint32_t was_m = (uint32_t)__ballot(lane < NP && (uint32_t)lane < np && map[NP * wave + lane] != 0);
  int32_t rk[NP];
  float old[NP];
#pragma unroll
  for (int i = 0; i < NP; i++) {
    const uint32_t p = pw + i;
    rk[i] = (ld.valid && (uint32_t)i < np) ? rank[p] : -2;
    old[i] = (((was_m >> i) & 1u) && ld.valid && !ld.new_tb) ? sbg[(size_t)p * LANES + lane] : 0.0f;
  }
  uint32_t mat_m = 0;
#pragma unroll
  for (int i = 0; i < NP; i++) {
    if ((uint32_t)i >= np) continue;   // uniform: only the group's last wavefront has np < NP
    const uint32_t p = pw + i;
    float v = old[i];
    bool c = false;
    if (rk[i] >= 0) {
      const uint32_t t = (uint32_t)rk[i] - ra;
      uint32_t j = j0 + t;
      if (j >= nv) j -= nv;
      if (j < E) { v = v + tile[lane][t]; c = true; }
      if (rep)
        for (j += nv; j < E; j += nv) v = v + e[ld.e_off + j];
    }
    const bool any = __ballot(c) != 0, was = (was_m >> i) & 1u;
    const bool mat = MI_RM_DENSE || any || (was && comb);   // row holds data after this launch
    if (mat && (MI_RM_DENSE || any || !was || fresh) && ld.valid) {
#if MI_RM_NT
      __builtin_nontemporal_store(v, &sbg[(size_t)p * LANES + lane]);
#else
      sbg[(size_t)p * LANES + lane] = v;
#endif
    }
    mat_m |= (uint32_t)mat << i;
  }
  if ((uint32_t)lane < np) map[NP * wave + lane] = (uint8_t)((mat_m >> lane) & 1u);
}

void launch_rm_combine(const float* e, float* sb, const MiGroupDesc* groups, const MiLaneDesc* lanes,
                       const MiKTab* /*ktabs*/, const uint32_t* ktab_data, uint32_t n_groups, uint32_t max_ncb,
                       hipStream_t st) {
  if (!n_groups) return;
  dim3 g((max_ncb + RM_CHUNK - 1) / RM_CHUNK, n_groups);
  hipLaunchKernelGGL(rm_combine_kernel, g, dim3(256), 0, st, e, sb, groups, lanes, ktab_data);
}

}  // namespace mi
