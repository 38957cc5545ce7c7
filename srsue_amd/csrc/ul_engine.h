// ul_engine.h -- device workspace + launch sequence of one UL PUSCH plan (shared by the batched ABI,
// ul_batch.cpp, and the per-TTI srslte_ue_ul_t, ue_ul.cpp).
#pragma once
#include <vector>

#include "engine.h"
#include "ul_plan.h"

namespace mi {
void launch_ul(const uint8_t* pay, uint32_t* tbcrc, const MiUlTx* txs, uint32_t n_tx, const MiUlCb* cbs, uint32_t n_cb,
               const uint32_t* kdata, const uint32_t* scr, const float2* tw, uint8_t* syms, float2* iq, int stage,
               hipStream_t st);

// device workspace of one UL plan (shared by the batch ABI and the per-TTI srslte_ue_ul_t)
struct UlEngine {
  UlPlan plan;
  DevBuf d_txs, d_cbs, d_kdata, d_scr, d_tw, d_tbcrc, d_syms;
  bool profile = false;
  std::vector<std::vector<hipEvent_t>> ev_sets;
  size_t ev_used = 0;

  ~UlEngine() {
    for (auto& s : ev_sets)
      for (auto& e : s) (void)hipEventDestroy(e);
  }
  template <class T>
  static bool up(DevBuf& b, const std::vector<T>& v, hipStream_t st) {
    if (!b.ensure(sizeof(T) * (v.empty() ? 1 : v.size()))) return false;
    return v.empty() || hip_ok(hipMemcpyAsync(b.p, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, st), "ul upload");
  }
  // host copies of the static tables last uploaded: the per-TTI path re-plans every grant, and the
  // QPP / selection tables and twiddles only change with the code-block sizes and bandwidth
  std::vector<uint32_t> up_kdata;
  std::vector<float> up_tw;
  int upload(hipStream_t st) {
    const UlPlan& P = plan;
    bool ok = up(d_txs, P.txs, st) && up(d_cbs, P.cbs, st) && up(d_scr, P.scr, st) &&
              d_tbcrc.ensure(P.txs.size() * 4) && d_syms.ensure(P.sym_bytes);
    // CQI symbols head each transmission's multiplexed sequence (the encoder writes the data after them)
    for (size_t i = 0; ok && i < P.txs.size(); i++)
      if (P.txs[i].q_cqi)
        ok = hip_ok(hipMemcpyAsync(d_syms.as<uint8_t>() + P.txs[i].sym_off, P.cqi_syms.data() + P.cqi_off[i],
                                   P.txs[i].q_cqi, hipMemcpyHostToDevice, st), "cqi upload");
    if (ok && P.kdata != up_kdata) {
      ok = up(d_kdata, P.kdata, st);
      up_kdata = P.kdata;
    }
    if (ok && P.tw != up_tw) {
      ok = up(d_tw, P.tw, st);
      up_tw = P.tw;
    }
    return ok ? 0 : -1;
  }
  int run(const void* d_pay, void* d_iq, hipStream_t st) {
    const UlPlan& P = plan;
    hipEvent_t* ev = nullptr;
    if (profile) {
      if (ev_used == ev_sets.size()) {
        std::vector<hipEvent_t> s(MI_UL_NSTAGES + 1);
        for (auto& e : s)
          if (!hip_ok(hipEventCreate(&e), "event")) return -1;
        ev_sets.push_back(s);
      }
      ev = ev_sets[ev_used++].data();
    }
    for (int stage = 0; stage < MI_UL_NSTAGES; stage++) {
      if (ev) (void)hipEventRecord(ev[stage], st);
      launch_ul(static_cast<const uint8_t*>(d_pay), d_tbcrc.as<uint32_t>(), d_txs.as<MiUlTx>(), (uint32_t)P.txs.size(),
                d_cbs.as<MiUlCb>(), (uint32_t)P.cbs.size(), d_kdata.as<uint32_t>(), d_scr.as<uint32_t>(),
                d_tw.as<float2>(), d_syms.as<uint8_t>(), static_cast<float2*>(d_iq), stage, st);
    }
    if (ev) (void)hipEventRecord(ev[MI_UL_NSTAGES], st);
    return hip_ok(hipGetLastError(), "ul launch") ? 0 : -1;
  }
  int stage_ms(float* ms, uint32_t* nruns) {
    if (!ev_used) { set_error("no profiled run (MI_UL_FLAG_PROFILE)"); return -1; }
    for (int i = 0; i < MI_UL_NSTAGES; i++) ms[i] = 0.f;
    for (size_t r = 0; r < ev_used; r++) {
      hipEvent_t* ev = ev_sets[r].data();
      if (!hip_ok(hipEventSynchronize(ev[MI_UL_NSTAGES]), "event sync")) return -1;
      for (int i = 0; i < MI_UL_NSTAGES; i++) {
        float t = 0.f;
        if (!hip_ok(hipEventElapsedTime(&t, ev[i], ev[i + 1]), "elapsed")) return -1;
        ms[i] += t / (float)ev_used;
      }
    }
    if (nruns) *nruns = (uint32_t)ev_used;
    return 0;
  }
};

}  // namespace mi
