// ul_batch.cpp -- C ABI of the batched UL PUSCH transmitter (include/mi_ul.h): plan once, upload the
// tables, enqueue the three kernels of ul.hip per run.
#include <string.h>

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
  int upload(hipStream_t st) {
    const UlPlan& P = plan;
    const bool ok = up(d_txs, P.txs, st) && up(d_cbs, P.cbs, st) && up(d_kdata, P.kdata, st) && up(d_scr, P.scr, st) &&
                    up(d_tw, P.tw, st) && d_tbcrc.ensure(P.txs.size() * 4) && d_syms.ensure(P.sym_bytes);
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

struct mi_ul_batch {
  mi::UlEngine eng;
};

extern "C" {

mi_ul_batch_t* mi_ul_batch_create(const mi_ul_cfg_t* cfgs, uint32_t n, uint32_t flags) {
  if (!cfgs || !n) { mi::set_error("empty UL batch"); return nullptr; }
  auto* b = new mi_ul_batch();
  b->eng.profile = (flags & MI_UL_FLAG_PROFILE) != 0;
  if (b->eng.plan.build(cfgs, n) || b->eng.upload(nullptr) || !mi::hip_ok(hipStreamSynchronize(nullptr), "ul upload sync")) {
    delete b;
    return nullptr;
  }
  return b;
}
void mi_ul_batch_destroy(mi_ul_batch_t* b) { delete b; }
size_t mi_ul_batch_payload_offset(const mi_ul_batch_t* b, uint32_t i) {
  return i < b->eng.plan.txs.size() ? b->eng.plan.txs[i].pay_off : 0;
}
size_t mi_ul_batch_payload_bytes(const mi_ul_batch_t* b) { return b->eng.plan.payload_bytes; }
size_t mi_ul_batch_iq_offset(const mi_ul_batch_t* b, uint32_t i) {
  return i < b->eng.plan.txs.size() ? b->eng.plan.txs[i].iq_off : 0;
}
size_t mi_ul_batch_iq_samples(const mi_ul_batch_t* b) { return b->eng.plan.iq_samples; }
uint32_t mi_ul_batch_n_codeblocks(const mi_ul_batch_t* b) { return (uint32_t)b->eng.plan.cbs.size(); }
int mi_ul_batch_run(mi_ul_batch_t* b, const void* d_payload, void* d_iq, void* stream) {
  if (!d_payload || !d_iq) { mi::set_error("null device buffer"); return -1; }
  return b->eng.run(d_payload, d_iq, reinterpret_cast<hipStream_t>(stream));
}
int mi_ul_batch_symbols(mi_ul_batch_t* b, uint32_t i, uint8_t* host) {
  if (i >= b->eng.plan.txs.size()) { mi::set_error("transmission index"); return -1; }
  const MiUlTx& t = b->eng.plan.txs[i];
  if (!mi::hip_ok(hipDeviceSynchronize(), "sync")) return -1;
  return mi::hip_ok(hipMemcpy(host, b->eng.d_syms.as<uint8_t>() + t.sym_off, 12 * (size_t)t.M, hipMemcpyDeviceToHost),
                    "symbols D2H") ? 0 : -1;
}
int mi_ul_batch_stage_ms(mi_ul_batch_t* b, float* ms, uint32_t* nruns) { return b->eng.stage_ms(ms, nruns); }
void mi_ul_batch_profile_reset(mi_ul_batch_t* b) { b->eng.ev_used = 0; }
double mi_ul_batch_algo_bytes(const mi_ul_batch_t* b) { return b->eng.plan.algo_bytes; }

}  // extern "C"
