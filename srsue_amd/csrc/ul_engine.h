// ul_engine.h -- device workspace + launch sequence of one UL PUSCH plan (shared by the batched ABI,
// ul_batch.cpp, and the per-TTI srslte_ue_ul_t, ue_ul.cpp).
#pragma once
#include <string.h>

#include <algorithm>
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
    if (stage_done) {
      (void)hipEventSynchronize(stage_done);
      (void)hipEventDestroy(stage_done);
    }
    if (h_stage) (void)hipHostFree(h_stage);
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
  // packed upload (the per-TTI path): the per-grant tables (transmissions, code blocks, scrambling words)
  // packed into one page-locked buffer and copied with a single DMA into one device arena
  DevBuf d_tables;
  void* h_stage = nullptr;
  size_t h_stage_bytes = 0;
  hipEvent_t stage_done = nullptr;
  bool packed = false;
  bool up_packed(hipStream_t st) {
    const UlPlan& P = plan;
    const size_t b0 = P.txs.size() * sizeof(MiUlTx), b1 = P.cbs.size() * sizeof(MiUlCb), b2 = P.scr.size() * 4;
    auto span = [](size_t b) { return (std::max<size_t>(b, 1) + 255) & ~(size_t)255; };
    const size_t o1 = span(b0), o2 = o1 + span(b1), total = o2 + span(b2);
    if (stage_done && !hip_ok(hipEventSynchronize(stage_done), "ul stage wait")) return false;
    if (total > h_stage_bytes) {
      if (h_stage) (void)hipHostFree(h_stage);
      h_stage = nullptr;
      h_stage_bytes = 0;
      if (!hip_ok(hipHostMalloc(&h_stage, total, hipHostMallocDefault), "ul stage")) return false;
      h_stage_bytes = total;
    }
    if (total > d_tables.bytes) {
      d_txs.release(); d_cbs.release(); d_scr.release();
      if (!d_tables.ensure(total)) return false;
    }
    char* h = static_cast<char*>(h_stage);
    if (b0) memcpy(h, P.txs.data(), b0);
    if (b1) memcpy(h + o1, P.cbs.data(), b1);
    if (b2) memcpy(h + o2, P.scr.data(), b2);
    char* d = static_cast<char*>(d_tables.p);
    d_txs.set_view(d, std::max<size_t>(b0, 1));
    d_cbs.set_view(d + o1, std::max<size_t>(b1, 1));
    d_scr.set_view(d + o2, std::max<size_t>(b2, 1));
    if (!stage_done && !hip_ok(hipEventCreateWithFlags(&stage_done, hipEventDisableTiming), "event")) return false;
    return hip_ok(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, st), "ul upload") &&
           hip_ok(hipEventRecord(stage_done, st), "event");
  }
  int upload(hipStream_t st) {
    const UlPlan& P = plan;
    bool ok = (packed ? up_packed(st) : (up(d_txs, P.txs, st) && up(d_cbs, P.cbs, st) && up(d_scr, P.scr, st))) &&
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
