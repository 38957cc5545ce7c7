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

// value of position p for one lane: `old` (a combining lane's materialised history, else 0) plus the
// LLRs received there; *got = at least one LLR lands on p
MI_HD inline float rm_value(const MiLaneDesc& ld, const int32_t* rank, const float* e, float old, uint32_t p, bool* got) {
  const int32_t rk = rank[p];
  float v = old;
  *got = false;
  if (rk >= 0) {
    uint32_t j = ((uint32_t)rk + ld.Nv - ld.r0) % ld.Nv;
    const float* el = e + ld.e_off;
    for (; j < ld.E; j += ld.Nv) { v = v + el[j]; *got = true; }
  }
  return v;
}

// row p of a group (all lanes) with the sparse-row rule of rm_combine_kernel: the row is materialised
// after the launch iff some lane receives an LLR there, or it was materialised and a lane combines; every
// written value also goes to the row's int16 mirror
MI_HD inline void rm_combine_row(const MiLaneDesc* lds, const uint32_t* kdata, const float* e, float* sbg, uint32_t Ncb,
                                 uint32_t p, const uint32_t* ipos) {
  uint8_t* map = reinterpret_cast<uint8_t*>(sbg + sb_map_off(Ncb));
  const size_t row = ipos[p];   // rows in decoder-input order (dl_common.h)
  bool comb = false, any = false;
  for (int l = 0; l < LANES; l++) comb |= lds[l].valid && !lds[l].new_tb;
  const bool was = map[p] != 0;
  float v[LANES];
  for (int l = 0; l < LANES; l++) {
    const MiLaneDesc& ld = lds[l];
    v[l] = 0.0f;
    if (!ld.valid) continue;
    bool got;
    const float old = (was && !ld.new_tb) ? sbg[row * LANES + l] : 0.0f;
    v[l] = rm_value(ld, reinterpret_cast<const int32_t*>(kdata + ld.rank_off), e, old, p, &got);
    any |= got;
  }
  const bool mat = any || (was && comb);
  if (mat)
    for (int l = 0; l < LANES; l++)
      if (lds[l].valid) {
        sbg[row * LANES + l] = v[l];
      }
  map[p] = mat ? 1 : 0;
}

}  // namespace mi
