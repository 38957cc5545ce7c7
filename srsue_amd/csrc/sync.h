// sync.h -- sync front end: PSS timing / N_ID_2 search, PSS CFO estimate, SSS
// detection, CFO correction on the GPU; the host engine behind mi_sync_* and srslte_ue_sync_*.
#pragma once
#include <vector>

#include "engine.h"

namespace mi {

struct MiPssJob { uint64_t off; uint32_t nlag, mask; };       // window at iq[off], lags 0..nlag-1
struct MiPssRes { uint32_t nid2, lag; float rho, cfo; };
struct MiSssJob { uint64_t off; uint32_t nid2; float cfo; };  // subframe start at iq[off]
struct MiSssRes { uint32_t nid1, sf5; float score, pad; };
struct MiCfoJob { uint64_t src, dst; float cfo; uint32_t pad; };

void launch_pss_search(const float2* iq, const float2* tmpl, const MiPssJob* jobs, MiPssRes* res, uint32_t n, uint32_t N,
                       uint32_t max_nlag, hipStream_t st);
void launch_sss_detect(const float2* iq, const MiSssJob* jobs, MiSssRes* res, uint32_t n, uint32_t N, uint32_t nof_prb,
                       uint32_t l5, uint32_t l6, hipStream_t st);
void launch_cfo_correct(const float2* src, float2* dst, const MiCfoJob* jobs, uint32_t n, uint32_t len, uint32_t N,
                        hipStream_t st);

// PSS / SSS sequences and the time-domain PSS templates of one bandwidth (tables.cpp restatement)
void pss_seq(uint32_t nid2, float2* d62);
void sss_seq(uint32_t nid1, uint32_t nid2, uint32_t sf5, float* d62);
uint32_t sync_bin(uint32_t m, uint32_t nof_prb, uint32_t N);

struct SyncEngine {
  uint32_t nof_prb = 0, N = 0;
  DevBuf d_tmpl, d_pjobs, d_pres, d_sjobs, d_sres, d_cjobs;
  std::vector<MiPssRes> pres;
  std::vector<MiSssRes> sres;
  int init(uint32_t nof_prb);
  int pss(const float2* iq, const std::vector<MiPssJob>& jobs, hipStream_t st);   // results -> pres (synchronous)
  int sss(const float2* iq, const std::vector<MiSssJob>& jobs, hipStream_t st);   // results -> sres (synchronous)
  int correct(const float2* src, float2* dst, const std::vector<MiCfoJob>& jobs, uint32_t len, hipStream_t st);
};

}  // namespace mi
