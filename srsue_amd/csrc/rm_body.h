// rm_body.h -- rate de-matching + HARQ soft combining for one (circular-buffer position, lane).
//
// Replaces srslte_rm_turbo_rx (36.212 5.1.4.1) called per code block inside
// srslte_pdsch_decode_rnti (/root/reference/ue/src/phy/phch_worker.cc:347), with the softbuffer
// semantics of srslte_softbuffer_rx_reset_tbs (dl_harq.cc:232): a new TB overwrites, a
// retransmission adds.  Inverting the bit selection per position makes it a gather (no atomics):
// position p of the circular buffer receives e[j0], e[j0 + Nv], ... with
// j0 = (rank(p) - rank(k0) + Nv) mod Nv, summed in increasing j -- the same order as the serial
// reference loop, so the combined value is bit-identical.
#pragma once
#include "dl_common.h"
#ifndef MI_HD
#define MI_HD __host__ __device__
#endif

namespace mi {

MI_HD inline void rm_combine_one(const MiLaneDesc& ld, const int32_t* rank, const float* e, float* sbg, uint32_t p,
                                 int lane) {
  const int32_t rk = rank[p];
  float v = ld.new_tb ? 0.0f : sbg[(size_t)p * LANES + lane];
  if (rk >= 0) {
    uint32_t j = ((uint32_t)rk + ld.Nv - ld.r0) % ld.Nv;
    const float* el = e + ld.e_off;
    for (; j < ld.E; j += ld.Nv) v = v + el[j];
  }
  sbg[(size_t)p * LANES + lane] = v;
}

}  // namespace mi
