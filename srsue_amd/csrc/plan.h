// plan.h -- host planner of the DL PDSCH receive chain (no HIP runtime dependency, so the
// test-only emulation build can link it too).
#pragma once
#include <map>
#include <string>
#include <cstring>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "dl_common.h"
#include "mi_dl.h"
#include "tables.h"

namespace mi {

void set_error(const std::string& s);
const char* last_error();

// Everything a build produces (what the kernels' tables and launch sizes come from).  Kept apart from the
// planner's lookup caches so that a built plan can be parked and re-activated by a swap (Engine::plan_memo).
struct PlanData {
  std::vector<MiCellDesc> cells;
  std::vector<float> crs;                 // float2 pairs
  std::vector<MiPdschDesc> pds;
  std::vector<uint32_t> re_tab, scr_tab;
  std::vector<MiSfDesc> sfs;
  std::vector<MiLaneDesc> lanes;
  std::vector<MiLaneSrc> lane_src;        // per lane (same index): the fused demap's inputs
  uint32_t unit_kind = 0;                 // Qm + 8 (TM2) shared by every valid lane, 0 = mixed
  // rate de-matching work list: (group << 9 | chunk) of the chunks where some lane receives LLRs (chunk 0
  // of every group included: it writes the group's zero row), then the other chunks (rm_busy items first)
  std::vector<uint32_t> rm_items;
  uint32_t rm_busy = 0;
  uint32_t rm_dbusy = 0;                  // the leading busy items that belong to direct groups (rm_direct)
  // per busy item, its folded record (rm.hip): lane0, Ncb | chunk << 16, softbuffer float offset / 64, the
  // K table's ipos offset (rows in decoder-input order, dl_common.h)
  std::vector<uint32_t> rm_recs;
  // direct groups (rm.hip, Plan::build): every valid lane a new TB with the same rank table, the same k0 rank
  // and E <= N_v -- each received position gets exactly one LLR.  Their busy chunks are in rm_items (record
  // flag: rank-driven stores), their idle chunks are not: rm_direct_map_kernel rewrites their whole row map
  // from these records (MiRmDirect, 8 u32 each)
  std::vector<uint32_t> rm_direct;
  bool rm_rep = false;                    // some code block repeats LLRs (E > N_v): no compact estimates
  std::vector<MiGroupDesc> groups;
  // pairs of equal-K groups for the packed two-code-blocks-per-lane turbo decoder (tdec_p2_body.h):
  // [2p] = group A, [2p + 1] = group B or 0xFFFFFFFF; a pair's decoder scratch spans both groups' regions
  // (consecutive), an unpaired group is followed by one group's worth of padding
  std::vector<uint32_t> pairs;
  std::vector<MiKTab> ktabs;
  std::vector<uint32_t> kdata;
  std::vector<MiTbDesc> tbs;
  std::vector<uint32_t> cb_list;
  std::vector<std::pair<int, std::vector<uint32_t>>> fft_lists;   // FFT size -> subframe indices
  std::vector<uint32_t> fft_list_flat;
  std::vector<size_t> fft_list_off;
  std::vector<uint32_t> fft_W;
  size_t iq_samples = 0, grid_elems = 0, ce_elems = 0, e_floats = 0, sb_floats = 0, scratch_floats = 0;
  size_t dec_bytes = 0, payload_bytes = 0;
  uint32_t max_units = 0, max_ncb = 0, n_cb = 0;
  bool has_pdsch = true;
  // algorithmic byte counts
  double bytes_compulsory = 0;
  double stage_bytes[MI_DL_NSTAGES] = {0};
  uint32_t cb_K = 0, cb_n = 0;
};

// A PDSCH RE list depends on the cell, CFI, subframe and PRB mask only (not on RNTI, Qm or the transmission
// mode): one list per distinct key per build (and across builds: re_cache), shared by every descriptor that uses it
struct ReKey {
  uint32_t cell_id, nof_prb, nof_ports, cfi, sf;
  uint8_t mask[(NRB_MAX + 3) & ~3];   // whole words: no padding bytes
  bool operator==(const ReKey& o) const { return !memcmp(this, &o, sizeof(ReKey)); }
  bool operator<(const ReKey& o) const { return memcmp(this, &o, sizeof(ReKey)) < 0; }
};
struct ReKeyHash {
  size_t operator()(const ReKey& k) const {
    uint64_t h = 1469598103934665603ull;
    const uint64_t* w = reinterpret_cast<const uint64_t*>(&k);
    for (size_t i = 0; i < sizeof(ReKey) / 8; i++) h = (h ^ w[i]) * 1099511628211ull;
    const uint8_t* b = reinterpret_cast<const uint8_t*>(&k);
    for (size_t i = sizeof(ReKey) / 8 * 8; i < sizeof(ReKey); i++) h = (h ^ b[i]) * 1099511628211ull;
    return (size_t)(h ^ (h >> 29));
  }
};
static_assert(sizeof(ReKey) == 20 + ((NRB_MAX + 3) & ~3), "ReKey must be padding-free (memcmp / hash over its bytes)");

struct Plan : PlanData {
  // A/B switches, set once at engine creation (Engine::Engine: MI_RM_DIRECT, MI_RM_XCDQ): direct rate de-matching
  // groups, and the rate de-matching work list dealt to 8 XCD queues (plan.cpp xcd_order)
  bool rm_direct_on = true, xcd_queues = true;
  void build_pairs();
  // cached per-key tables (kept across rebuilds)
  std::map<std::tuple<uint32_t, uint32_t, uint32_t>, std::vector<float>> crs_cache;
  std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, std::vector<uint32_t>> scr_cache;
  std::map<uint32_t, std::vector<std::vector<uint32_t>>> kpos_cache;   // K -> {pos, pi, crcA, crcB}
  void add_ktab(uint32_t K);   // appends K's tables to kdata and a MiKTab to ktabs
  std::map<std::pair<uint32_t, uint32_t>, std::pair<std::vector<int32_t>, uint32_t>> rank_cache;
  // PDSCH RE lists per (cell, CFI, sf, PRB mask) (plan.cpp ReKey): [0] = count, then the grid indices
  std::unordered_map<ReKey, std::vector<uint32_t>, ReKeyHash> re_cache;

  // has_pdsch = false plans only OFDM + channel estimation (per-TTI front half)
  int build(const mi_dl_sf_cfg_t* cfgs, uint32_t n, bool has_pdsch);
  // raw code-block mode (srslte_tdec_* contract): n_cb blocks of size K, no PHY front end
  int build_codeblocks(uint32_t K, uint32_t n_cb, bool crc24a);
};

}  // namespace mi
