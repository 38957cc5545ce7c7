// ctrl.h -- DL control channels: descriptors, launchers and the host engine
// that plans PCFICH / PDCCH / DCI blind search over the grid and channel estimates of an Engine.
#pragma once
#include <vector>

#include "engine.h"

namespace mi {

constexpr uint32_t DCI_MAX_BITS = 64;

struct MiCtrlSf {            // one per subframe
  uint64_t grid_off, ce_off; // float2 offsets (port p of ce at ce_off + p * plane)
  uint32_t plane;            // 14 * 12 N_RB
  uint32_t ports;
  uint32_t M;                // PDCCH REGs (not PCFICH / PHICH)
  uint32_t n_cce;
  uint32_t reg_off;          // cdata offset: re[4 M] (grid indices), then logical quadruplet [M]
  uint32_t scr_off;          // cdata offset: scrambling words (8 M bits)
  uint32_t pcfich_off;       // cdata offset: 16 PCFICH REs + 1 scrambling word
  uint32_t llr_off;          // float offset of this subframe's PDCCH soft bits [8 M]
  uint32_t phich_off;        // cdata offset: PHICH query: 12 REs, scrambling word (12 bits), sequence
};

struct MiDciJob {            // one (candidate, DCI size) of one subframe
  uint32_t sf, llr_off, L, ncce, A, D, rank_off, rnti;
};
struct MiDciRes { uint32_t found; uint32_t bits[2]; };   // bits MSB first

void launch_pcfich(const float2* grid, const float2* ce, const MiCtrlSf* sfs, const uint32_t* cdata, uint32_t* cfi,
                   uint32_t n_sf, hipStream_t st);
void launch_pdcch_llr(const float2* grid, const float2* ce, const MiCtrlSf* sfs, const uint32_t* cdata, float* llr,
                      uint32_t n_sf, uint32_t max_regs, float noise, hipStream_t st);
void launch_dci_search(const float* llr, const MiDciJob* jobs, const uint32_t* cdata, MiDciRes* res, uint32_t n_jobs,
                       hipStream_t st);
void launch_phich(const float2* grid, const float2* ce, const MiCtrlSf* sfs, const uint32_t* cdata, float* soft,
                  uint32_t n_sf, hipStream_t st);

struct DciFound { uint32_t found, format, nbits, L, ncce; uint8_t bits[DCI_MAX_BITS]; };

// the tables one build produces (a parked copy can be swapped back in: the per-TTI API's memo, ue_dl.cpp)
struct CtrlTables {
  std::vector<MiCtrlSf> sfs;
  std::vector<uint32_t> cdata;
  std::vector<MiDciJob> jobs;
  std::vector<uint8_t> job_fmt;      // per job: bit 2 = common space; bits 0-1: 0 = 0/1A size, DCI_1, DCI_1C
  std::vector<uint32_t> job_begin;   // per subframe: jobs [job_begin[s], job_begin[s+1]) in search order
  std::vector<uint32_t> nof_prb;     // per subframe
  DevBuf d_sfs, d_cdata, d_jobs;
  size_t llr_floats = 0;
  uint32_t max_regs = 0;
  void swap_tables(CtrlTables& o) {
    sfs.swap(o.sfs); cdata.swap(o.cdata); jobs.swap(o.jobs); job_fmt.swap(o.job_fmt); job_begin.swap(o.job_begin);
    nof_prb.swap(o.nof_prb); d_sfs.swap(o.d_sfs); d_cdata.swap(o.d_cdata); d_jobs.swap(o.d_jobs);
    std::swap(llr_floats, o.llr_floats); std::swap(max_regs, o.max_regs);
  }
};

struct CtrlEngine : CtrlTables {
  DevBuf d_llr, d_res, d_cfi, d_phich;
  std::vector<MiDciRes> res;         // host copy after download
  // plan over the subframes of P (cells, grid / ce layout) with per-subframe CFI and RNTI; phich: per
  // subframe the PHICH query I_lowest | n_dmrs << 16 (36.213 9.1.2), empty = (0, 0)
  int build(const Plan& P, const std::vector<uint32_t>& cfi, uint32_t phich_ng, const std::vector<uint16_t>& rnti,
            const std::vector<uint32_t>& phich = {});
  int upload(hipStream_t st);
  // stages: 1 = PCFICH, 2 = PDCCH soft bits, 4 = blind search, 8 = PHICH
  int run(const float2* grid, const float2* ce, uint32_t mask, float noise, hipStream_t st);
  int download(hipStream_t st);
  // first match in search order: DL = format 1A (flag 1) or 1; UL = format 0 (flag 0)
  DciFound select(uint32_t sf, bool ul, bool common_only) const;
};

}  // namespace mi
