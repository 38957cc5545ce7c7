// kernels.h -- host launchers of the gfx950 kernels of the DL PDSCH path.
#pragma once
#include <hip/hip_runtime.h>
#include "dl_common.h"
#include "kernels_consts.h"

namespace mi {

// OFDM RX (srslte_ofdm_rx_sf): one workgroup per subframe, 14 FFTs of size N
void launch_ofdm_rx(int N, const void* iq, bool sc16, float2* grid, const MiSfDesc* sfs, const uint32_t* list,
                    uint32_t n, const float2* tw, uint32_t W, hipStream_t st);
// channel estimation (srslte_chest_dl_estimate): one workgroup per subframe, all ports
void launch_chest(const float2* grid, float2* ce, const MiSfDesc* sfs, const MiCellDesc* cells,
                  const float2* crs, float* metrics, uint32_t n_sf, hipStream_t st,
                  bool compact = false /* MI_DL_FLAG_CE_COMPACT: only the 4 pilot rows per port */);
// equalise + soft demap + descramble (srslte_predecoding_* / demod_soft / scrambling_f)
void launch_demap(const float2* grid, const float2* ce, float* e, const MiSfDesc* sfs,
                  const MiPdschDesc* pd, const MiCellDesc* cells, const uint32_t* re_tab,
                  const uint32_t* scr, uint32_t n_sf, uint32_t max_units, float noise, hipStream_t st);
// rate de-matching + HARQ combining into the group-interleaved softbuffer (srslte_rm_turbo_rx)
void launch_rm_combine(const float* e, float* sb, const MiGroupDesc* groups, const MiLaneDesc* lanes,
                       const MiKTab* ktabs, const uint32_t* ktab_data, uint32_t n_groups,
                       uint32_t max_ncb, const uint32_t* items, const uint4* recs /* Plan::rm_recs */, uint32_t n_busy,
                       uint32_t n_dbusy /* Plan::rm_dbusy */,
                       uint32_t n_items, hipStream_t st);
// demap fused into rate de-matching: LLRs computed from grid + ce inside the rm staging (no LLR stream)
void launch_rm_fused(const float2* grid, const float2* ce, const MiLaneSrc* lane_src, const uint32_t* re_tab,
                     const uint32_t* scr_tab, float noise, float* sb, const MiGroupDesc* groups, const MiLaneDesc* lanes,
                     const MiKTab* ktabs, const uint32_t* ktab_data, uint32_t n_groups, uint32_t max_ncb,
                     uint32_t unit_kind /* Qm + 8 TM2 common to all lanes, 0 = mixed */,
                     const uint32_t* items /* Plan::rm_items, NULL = every chunk */,
                     const uint4* recs /* Plan::rm_recs: the busy items' folded records */, uint32_t n_busy,
                     uint32_t n_dbusy /* Plan::rm_dbusy: the leading direct-group items */, uint32_t n_items,
                     bool compact_ce, hipStream_t st);
// row maps and zero rows of Plan::rm_direct's groups (rm.hip rm_direct_map_kernel), before the combine launch
void launch_rm_direct_maps(float* sb, const uint32_t* ktab_data, const MiRmDirect* dgs, uint32_t ndg, hipStream_t st);
// turbo decoder (srslte_tdec_*): one wavefront per group of 64 code blocks
// window masks of the sparse softbuffer rows (which decoder inputs have a materialised row)
void launch_rowmask(const float* sb, uint32_t* wm, const MiGroupDesc* groups, const MiKTab* ktabs,
                    const uint32_t* kdata, uint32_t n_groups, uint32_t* zero, hipStream_t st);
void launch_tdec(const float* sb, const uint32_t* wm, float* scratch, uint8_t* dec, uint8_t* cb_bytes, uint32_t* cb_its,
                 uint32_t* cb_crc, uint32_t* cb_tbp, const MiGroupDesc* groups, const MiLaneDesc* lanes,
                 const MiKTab* ktabs, const uint32_t* ktab_data, uint32_t n_groups, uint32_t max_its,
                 uint32_t early_stop, bool q16, int crossed /* 0 one wavefront per group, 1 crossed, 2 crossed recompute */, hipStream_t st);
// packed int16 decoder, two code blocks per lane: one workgroup (crossed wavefronts F and B) per group pair
// (Plan::pairs)
void launch_tdec_p2(const float* sb, const uint32_t* wm, float* scratch, uint8_t* dec, uint8_t* cb_bytes,
                    uint32_t* cb_its, uint32_t* cb_crc, uint32_t* cb_tbp, const MiGroupDesc* groups,
                    const MiLaneDesc* lanes, const MiKTab* ktabs, const uint32_t* ktab_data, const uint32_t* pairs,
                    uint32_t n_pairs, uint32_t max_its, uint32_t early_stop,
                    uint8_t* payload /* PDSCH batches: payload bytes written in place; nullptr = cb_bytes rows */,
                    bool no_w /* DEC2 stores no extrinsic rows (a one-iteration first launch, tdec_p2_body.h) */,
                    hipStream_t st);
// waterfall compaction after iteration 0 of launch_tdec_p2 (one K, early stop; tdec_p2_body.h P2ContSrc):
// gather the CRC-failing code blocks into dense continuation pairs (cscr: max_pairs x pair_u32 words, cdec:
// max_pairs x K x 64 bytes, cont: 1 + lanes words) and decode iterations 1 .. max_its - 1 there
bool launch_tdec_cont(const float* sb, const uint32_t* wm, float* scratch, size_t scr_pair_u32, uint8_t* dec,
                      uint8_t* cb_bytes, uint32_t* cb_its, uint32_t* cb_crc, uint32_t* cb_tbp, const MiGroupDesc* groups,
                      const MiLaneDesc* lanes, const uint32_t* ktab_data, const MiKTab& kt, uint32_t n_groups, uint32_t* cont,
                      uint32_t* cscr, uint8_t* cdec, uint32_t max_pairs, size_t pair_u32, uint32_t K, uint32_t max_its,
                      uint32_t gather_wgs, uint8_t* payload,
                      bool w_stored /* the first launch stored w rows: gather them (no DEC2 re-run) */,
                      bool rounds /* one iteration per launch, the failing code blocks re-compacted between them;
                                     cont holds 3 n_groups * 64 + 2 words, scratch / dec are reused as pair buffers */,
                      uint32_t* h_count /* page-locked [CONT_HIST]: the code blocks each round decodes (round 1:
                                           those continuing after iteration 0) */,
                      uint32_t seg /* 0, or the rounds after the first segmented over 4 / 8 wavefronts per pair
                                      (tdec_kernel_p2s) */,
                      bool cont_zeroed /* cont[0] already reset on st (launch_rowmask's zero) */, hipStream_t st);
constexpr uint32_t CONT_HIST = 8;   // rounds whose counts are recorded (h_count)
// latency form of the int16 turbo decoder: one workgroup of `threads` (64/128/256) per code block
// (lane descriptor), exact trellis segments (tdec_win_body.h); max_k sizes the dynamic LDS
void launch_tdec_win(const float* sb, uint8_t* cb_bytes, uint32_t* cb_its, uint32_t* cb_crc, uint32_t* cb_tbp,
                     const MiGroupDesc* groups, const MiLaneDesc* lanes, const MiKTab* ktabs, const uint32_t* kdata,
                     uint32_t n_lanes, uint32_t max_k, uint32_t max_its, uint32_t early_stop, uint32_t threads,
                     hipStream_t st);
// raw code-block decoder input [cb][3(K+4)] -> group-interleaved softbuffer layout
void launch_cb_scatter(const float* d, float* sb, const MiGroupDesc* groups, const MiKTab* ktabs,
                       const uint32_t* kdata, uint32_t n_groups, uint32_t K, uint32_t n_cb, hipStream_t st);
// TB assembly + CRC24A + payload packing
void launch_tb(const uint8_t* cb_bytes, uint8_t* payload, uint32_t* tb_crc_ok, uint32_t* tb_its,
               const uint32_t* cb_its, const uint32_t* cb_tbp, const MiTbDesc* tbs, uint32_t n_tb,
               const uint32_t* cb_list, const uint32_t* kdata, bool copy /* false: payload already written */,
               hipStream_t st);

}  // namespace mi
