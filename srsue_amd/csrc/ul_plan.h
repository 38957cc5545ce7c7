// ul_plan.h -- host planner of the UL PUSCH transmit path (no HIP dependency): segmentation, rate
// matching splits and selection tables, scrambling words, DMRS parameters, DFT radix plans and
// twiddle tables for a batch of transmissions.
#pragma once
#include <array>
#include <map>
#include <vector>

#include "mi_ul.h"
#include "tables.h"
#include "ul_common.h"

namespace mi {

// 36.211 5.5.2.1 / 5.5.1: DMRS root q, Zadoff-Chu length and cyclic shift of slot ns (0..19)
int ul_dmrs_params(const mi_ul_cfg_t& c, uint32_t ns, uint32_t* q, uint32_t* nzc, uint32_t* ncs);
// radix list (8, 4, 2, 3, 5; 4 bits per stage) of an n-point transform, 0 if n has another factor
uint32_t ul_radix_plan(uint32_t n);
// CQI channel coding on PUSCH (36.212 5.2.2.6.4): the Q coded bits of the O-bit report o (O <= 11: the
// (32, O) block code repeated; O > 11: CRC8, tail-biting convolutional code, 5.1.4.2 rate matching)
void ul_cqi_code(const uint8_t* o, uint32_t O, uint32_t Q, std::vector<uint8_t>& q);

struct UlPlan {
  std::vector<MiUlTx> txs;
  std::vector<MiUlCb> cbs;
  std::vector<uint32_t> kdata;      // QPP and selection tables
  std::vector<uint32_t> scr;        // scrambling words
  std::vector<float> tw;            // float2 twiddle tables
  std::vector<uint32_t> tb_cb0;     // first code block of each transmission (n + 1 entries)
  std::vector<uint8_t> cqi_syms;    // CQI coded symbols of every transmission (Qm bits per byte, MSB first)
  std::vector<uint32_t> cqi_off;    // per transmission: offset of its Q'_CQI symbols in cqi_syms
  size_t payload_bytes = 0, sym_bytes = 0, iq_samples = 0;
  double algo_bytes = 0;

  std::map<uint32_t, uint32_t> pi_off, tw_off;
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> sel_off;   // (K, F) -> kdata offset of this build
  // per-key tables kept across builds (the per-TTI path re-plans every grant)
  struct SelTab { std::vector<uint32_t> sel; uint32_t r0[4]; };
  std::map<std::pair<uint32_t, uint32_t>, SelTab> sel_cache;
  std::map<uint32_t, std::vector<uint32_t>> pi_cache;
  std::map<uint32_t, std::vector<float>> tw_cache;   // DFT length -> interleaved cos / sin twiddles
  // scrambling words by (c_init, bits): srsUE's RNTI and cell are fixed, so a worker sees a handful of
  // keys (10 subframes x the grant sizes); bounded, cleared when it grows past SCR_CACHE_MAX
  std::map<std::pair<uint32_t, uint32_t>, std::vector<uint32_t>> scr_cache;
  static constexpr size_t SCR_CACHE_MAX = 256;
  int build(const mi_ul_cfg_t* cfgs, uint32_t n);
};

}  // namespace mi
