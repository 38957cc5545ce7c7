// rm.hip -- rate de-matching + HARQ combine into the group-interleaved softbuffer [Ncb][64 lanes].
// See rm_body.h.  Each wavefront owns a run of circular-buffer positions for the 64 code blocks of
// a group, so softbuffer reads and writes are 256-B coalesced rows; each lane streams its own
// code block's LLRs in order (cache-line reuse across consecutive positions).
#include "kernels.h"
#include "rm_body.h"

namespace mi {

constexpr int RM_PPW = 32;   // positions per wavefront

__global__ __launch_bounds__(256) void rm_combine_kernel(const float* __restrict__ e, float* __restrict__ sb,
                                                        const MiGroupDesc* __restrict__ groups,
                                                        const MiLaneDesc* __restrict__ lanes,
                                                        const uint32_t* __restrict__ kdata) {
  const MiGroupDesc g = groups[blockIdx.y];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const MiLaneDesc ld = lanes[g.lane0 + lane];
  if (!ld.valid) return;
  const int32_t* rank = reinterpret_cast<const int32_t*>(kdata + ld.rank_off);
  float* sbg = sb + g.sb_off;
  const uint32_t p0 = (blockIdx.x * 4 + wave) * RM_PPW;
  for (int i = 0; i < RM_PPW; i++) {
    const uint32_t p = p0 + i;
    if (p >= g.Ncb) break;
    rm_combine_one(ld, rank, e, sbg, p, lane);
  }
}

void launch_rm_combine(const float* e, float* sb, const MiGroupDesc* groups, const MiLaneDesc* lanes,
                       const MiKTab* /*ktabs*/, const uint32_t* ktab_data, uint32_t n_groups, uint32_t max_ncb,
                       hipStream_t st) {
  if (!n_groups) return;
  dim3 g((max_ncb + 4 * RM_PPW - 1) / (4 * RM_PPW), n_groups);
  hipLaunchKernelGGL(rm_combine_kernel, g, dim3(256), 0, st, e, sb, groups, lanes, ktab_data);
}

}  // namespace mi
