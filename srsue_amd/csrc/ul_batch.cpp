// ul_batch.cpp -- C ABI of the batched UL PUSCH transmitter (include/mi_ul.h): plan once, upload the
// tables, enqueue the three kernels of ul.hip per run.
#include <string.h>

#include <vector>

#include "ul_engine.h"


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
  const size_t h = 12 * (size_t)t.M - t.q_ri;   // the multiplexed sequence g; the RI cells follow as zeros
  memset(host + h, 0, t.q_ri);
  return mi::hip_ok(hipMemcpy(host, b->eng.d_syms.as<uint8_t>() + t.sym_off, h, hipMemcpyDeviceToHost),
                    "symbols D2H") ? 0 : -1;
}
int mi_ul_batch_stage_ms(mi_ul_batch_t* b, float* ms, uint32_t* nruns) { return b->eng.stage_ms(ms, nruns); }
void mi_ul_batch_profile_reset(mi_ul_batch_t* b) { b->eng.ev_used = 0; }
double mi_ul_batch_algo_bytes(const mi_ul_batch_t* b) { return b->eng.plan.algo_bytes; }

}  // extern "C"
