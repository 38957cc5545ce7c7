// batch.cpp -- C ABI of the batched receiver (include/mi_dl.h).
#include <string.h>

#include "engine.h"
#include "kernels.h"

namespace mi { const char* last_error(); }

#include "batch_impl.h"

extern "C" {

mi_dl_batch_t* mi_dl_batch_create(const mi_dl_sf_cfg_t* cfgs, uint32_t n_sf, uint32_t max_its, uint32_t flags) {
  if (!cfgs || !n_sf) { mi::set_error("empty batch"); return nullptr; }
  auto* b = new mi_dl_batch();
  b->cfgs.assign(cfgs, cfgs + n_sf);
  b->eng.max_its = max_its ? max_its : 4;
  b->eng.flags = flags;
  if (!mi::hip_ok(hipGetDevice(&b->eng.device), "device") || b->eng.plan.build(cfgs, n_sf, true) || b->eng.upload(nullptr, true) ||
      !mi::hip_ok(hipStreamSynchronize(nullptr), "upload sync")) {
    delete b;
    return nullptr;
  }
  return b;
}

void mi_dl_batch_destroy(mi_dl_batch_t* b) { delete b; }

size_t mi_dl_batch_iq_offset(const mi_dl_batch_t* b, uint32_t sf) {
  return sf < b->eng.plan.sfs.size() ? b->eng.plan.sfs[sf].iq_off : 0;
}
size_t mi_dl_batch_iq_samples(const mi_dl_batch_t* b) { return b->eng.plan.iq_samples; }
size_t mi_dl_batch_payload_offset(const mi_dl_batch_t* b, uint32_t sf) {
  return sf < b->eng.plan.tbs.size() ? b->eng.plan.tbs[sf].pay_off : 0;
}

static mi::DevBuf* buf_of(mi_dl_batch_t* b, int which, size_t* bytes) {
  const mi::Plan& P = b->eng.plan;
  const size_t nsf = P.sfs.size();
  switch (which) {
    case MI_DL_BUF_GRID: *bytes = P.grid_elems * 8; return &b->eng.d_grid;
    case MI_DL_BUF_CE: *bytes = P.ce_elems * 8; return &b->eng.d_ce;
    case MI_DL_BUF_LLR: *bytes = P.e_floats * 4; return b->eng.ensure_llr() ? &b->eng.d_e : nullptr;
    case MI_DL_BUF_PAYLOAD: *bytes = P.payload_bytes; return &b->eng.d_payload;
    case MI_DL_BUF_TB_CRC: *bytes = nsf * 4; return &b->eng.d_tbok;
    case MI_DL_BUF_TB_ITS: *bytes = nsf * 4; return &b->eng.d_tbits;
    case MI_DL_BUF_METRICS: *bytes = nsf * 5 * 4; return &b->eng.d_metrics;
    case MI_DL_BUF_CB_ITS: *bytes = P.lanes.size() * 4; return &b->eng.d_cbits;
    case MI_DL_BUF_CB_CRC: *bytes = P.lanes.size() * 4; return &b->eng.d_cbcrc;
    case MI_DL_BUF_SOFTBUFFER: *bytes = P.sb_floats * 4; return &b->eng.d_sb;
  }
  *bytes = 0;
  return nullptr;
}

size_t mi_dl_batch_bytes(const mi_dl_batch_t* b, int which) {
  size_t n = 0;
  buf_of(const_cast<mi_dl_batch_t*>(b), which, &n);
  return n;
}

size_t mi_dl_batch_offset(const mi_dl_batch_t* b, int which, uint32_t sf) {
  const mi::Plan& P = b->eng.plan;
  if (sf >= P.sfs.size()) return 0;
  switch (which) {
    case MI_DL_BUF_GRID: return P.sfs[sf].grid_off;
    case MI_DL_BUF_CE: return P.sfs[sf].ce_off;
    case MI_DL_BUF_LLR: return P.sfs[sf].e_off;
    case MI_DL_BUF_PAYLOAD: return P.tbs[sf].pay_off;
    default: return sf;
  }
}

int mi_dl_batch_run(mi_dl_batch_t* b, const void* d_iq, void* stream) {
  if (!b || !d_iq) { mi::set_error("null argument"); return -1; }
  return b->eng.run(d_iq, reinterpret_cast<hipStream_t>(stream), 0xFFFFFFFFu, nullptr);
}

int mi_dl_batch_run_stages(mi_dl_batch_t* b, const void* d_iq, void* stream, uint32_t mask) {
  if (!b) { mi::set_error("null argument"); return -1; }
  if ((mask & 1u) && !d_iq) { mi::set_error("OFDM stage needs IQ"); return -1; }
  return b->eng.run(d_iq, reinterpret_cast<hipStream_t>(stream), mask, nullptr);
}

int mi_dl_batch_run_split(mi_dl_batch_t* b, const void* d_iq, void* front_stream, void* back_stream) {
  if (!b || !d_iq) { mi::set_error("null argument"); return -1; }
  if (front_stream == back_stream) return mi_dl_batch_run(b, d_iq, front_stream);
  const hipStream_t back = reinterpret_cast<hipStream_t>(back_stream);
  return b->eng.run(d_iq, reinterpret_cast<hipStream_t>(front_stream), 0xFFFFFFFFu, nullptr, &back);
}

int mi_dl_batch_upload(mi_dl_batch_t* b, int which, const void* host, size_t bytes) {
  size_t n = 0;
  mi::DevBuf* d = buf_of(b, which, &n);
  if (!d || bytes > n) { mi::set_error("bad buffer or size"); return -1; }
  if (!mi::hip_ok(hipStreamSynchronize(b->eng.last_stream), "sync")) return -1;
  return mi::hip_ok(hipMemcpy(d->p, host, bytes, hipMemcpyHostToDevice), "upload") ? 0 : -1;
}

int mi_dl_batch_download(mi_dl_batch_t* b, int which, void* host, size_t bytes) {
  size_t n = 0;
  mi::DevBuf* d = buf_of(b, which, &n);
  if (!d || bytes > n) { mi::set_error("bad buffer or size"); return -1; }
  if (!mi::hip_ok(hipStreamSynchronize(b->eng.last_stream), "sync")) return -1;
  return mi::hip_ok(hipMemcpy(host, d->p, bytes, hipMemcpyDeviceToHost), "download") ? 0 : -1;
}

void* mi_dl_batch_device_ptr(mi_dl_batch_t* b, int which) {
  size_t n = 0;
  mi::DevBuf* d = buf_of(b, which, &n);
  return d ? d->p : nullptr;
}

int mi_dl_batch_stage_ms(mi_dl_batch_t* b, float* ms, uint32_t* nruns) { return b->eng.stage_ms(ms, nruns); }
void mi_dl_batch_profile_reset(mi_dl_batch_t* b) { b->eng.profile_reset(); }

double mi_dl_batch_algo_bytes(const mi_dl_batch_t* b, int which_stage) {
  if (which_stage < 0) return b->eng.plan.bytes_compulsory;
  if (which_stage >= MI_DL_NSTAGES) return 0;
  return b->eng.plan.stage_bytes[which_stage];
}

uint32_t mi_dl_batch_n_codeblocks(const mi_dl_batch_t* b) { return b->eng.plan.n_cb; }
static int turbo_sched(const mi::Engine& e) {
  if (e.use_win()) return 1;
  const int x = e.tdec_crossed();
  return x == 3 ? 4 : x == 2 ? 3 : x ? 2 : 0;
}
int mi_dl_batch_turbo_win(const mi_dl_batch_t* b) { return turbo_sched(b->eng); }
int mi_dl_batch_turbo_compact(const mi_dl_batch_t* b) { return b->eng.tdec_compact() ? 1 : 0; }
uint32_t mi_dl_batch_n_groups(const mi_dl_batch_t* b) { return (uint32_t)b->eng.plan.groups.size(); }
uint32_t mi_dl_batch_rm_direct_groups(const mi_dl_batch_t* b) { return (uint32_t)(b->eng.plan.rm_direct.size() / 8); }

/* ---- streaming re-planning (include/mi_dl.h) ------------------------------------------------ */
struct mi_dl_plan {
  mi::Plan plan;
  std::vector<mi_dl_sf_cfg_t> cfgs;
  bool built = false;
};

mi_dl_plan_t* mi_dl_plan_create(void) { return new mi_dl_plan(); }
void mi_dl_plan_destroy(mi_dl_plan_t* p) { delete p; }

size_t mi_dl_batch_device_bytes(mi_dl_batch_t* b) {
  return b ? b->eng.work_bytes(true, b->eng.d_e.bytes != 0) + b->eng.d_tables.bytes + b->eng.d_tw.bytes : 0;
}

size_t mi_dl_plan_device_bytes(const mi_dl_plan_t* p, uint32_t max_its, uint32_t flags) {
  if (!p || !p->built) { mi::set_error("mi_dl_plan_device_bytes: no built plan"); return 0; }
  mi::Engine e;   // host only: the sizes of the buffers a batch of this plan would allocate
  static_cast<mi::PlanData&>(e.plan) = p->plan;
  e.max_its = max_its ? max_its : 4;
  e.flags = flags;
  return e.work_bytes(true, (flags & MI_DL_FLAG_KEEP_LLR) != 0);
}

int mi_dl_plan_build(mi_dl_plan_t* p, const mi_dl_sf_cfg_t* cfgs, uint32_t n_sf) {
  if (!p || !cfgs || !n_sf) { mi::set_error("empty batch"); return -1; }
  p->built = false;
  if (p->plan.build(cfgs, n_sf, true)) return -1;
  p->cfgs.assign(cfgs, cfgs + n_sf);
  p->built = true;
  return 0;
}

int mi_dl_batch_replan(mi_dl_batch_t* b, mi_dl_plan_t* p, void* stream) {
  if (!b || !p || !p->built) { mi::set_error("mi_dl_batch_replan: no built plan"); return -1; }
  const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // the table upload rewrites what a pending split run's back end reads
  if (!b->eng.order_after_split(st)) return -1;
  // the active plan data and the built one trade places (the planner's caches stay with each object)
  std::swap(static_cast<mi::PlanData&>(b->eng.plan), static_cast<mi::PlanData&>(p->plan));
  std::swap(b->cfgs, p->cfgs);
  p->built = false;
  b->eng.last_stream = st;
  // HARQ continuity per group (include/mi_dl.h): p->plan now holds the old plan
  const mi::PlanData &nw = b->eng.plan, &old = p->plan;
  auto same_group = [&](size_t g) {
    if (g >= old.groups.size()) return false;
    const MiGroupDesc &x = nw.groups[g], &y = old.groups[g];
    if (x.K != y.K || x.Ncb != y.Ncb || x.lane0 != y.lane0 || x.sb_off != y.sb_off) return false;
    for (uint32_t l = x.lane0; l < x.lane0 + mi::LANES; l++) {
      const bool a = l < nw.lanes.size(), c = l < old.lanes.size();
      if (a != c) return false;
      if (!a) continue;
      const MiLaneDesc &u = nw.lanes[l], &v = old.lanes[l];
      if (u.valid != v.valid || (u.valid && (u.tb != v.tb || u.F != v.F))) return false;
    }
    return true;
  };
  // the regions to clear: groups with a retransmission lane whose layout changed (contiguous regions merged)
  std::vector<std::pair<size_t, size_t>> clear;
  for (size_t g = 0; g < nw.groups.size(); g++) {
    const MiGroupDesc& x = nw.groups[g];
    bool combines = false;
    for (uint32_t l = x.lane0; l < x.lane0 + mi::LANES && l < nw.lanes.size(); l++)
      combines |= nw.lanes[l].valid && !nw.lanes[l].new_tb;
    if (!combines || same_group(g)) continue;
    const size_t off = x.sb_off, n = mi::sb_group_floats(x.Ncb);
    if (!clear.empty() && clear.back().first + clear.back().second == off) clear.back().second += n;
    else clear.emplace_back(off, n);
  }
  const size_t had = b->eng.d_sb.bytes;
  if (b->eng.upload(st, true)) return -1;
  // (a first softbuffer was zeroed by upload; a grown one keeps its contents and zeroes only its new tail)
  if (!had) return 0;
  for (const auto& c : clear)
    if (!mi::hip_ok(hipMemsetAsync(b->eng.d_sb.as<float>() + c.first, 0, c.second * sizeof(float), st),
                    "replan softbuffer reset"))
      return -1;
  return 0;
}

int mi_dl_batch_set_tdec_history(mi_dl_batch_t* b, int mode) {
  if (!b || mode < -1 || mode > 1) { mi::set_error("mi_dl_batch_set_tdec_history: mode is -1, 0 or 1"); return -1; }
  b->eng.cont_mode = mode;
  return 0;
}
void mi_dl_batch_reset_history(mi_dl_batch_t* b) {
  if (b) b->eng.reset_history();
}

/* ---- raw code-block decoding (srslte_tdec_* contract) ---------------------------------------- */
struct mi_tdec_batch {
  mi::Engine eng;
};

mi_tdec_batch_t* mi_tdec_create(uint32_t K, uint32_t n_cb, uint32_t max_its, int early_stop, int crc24a,
                                uint32_t flags) {
  auto* b = new mi_tdec_batch();
  b->eng.max_its = max_its ? max_its : 8;
  b->eng.early_stop = early_stop ? 1 : 0;
  b->eng.flags = flags;
  if (b->eng.plan.build_codeblocks(K, n_cb, crc24a != 0) || b->eng.upload(nullptr, true) ||
      !mi::hip_ok(hipStreamSynchronize(nullptr), "upload sync")) {
    delete b;
    return nullptr;
  }
  return b;
}
void mi_tdec_destroy(mi_tdec_batch_t* b) { delete b; }
int mi_tdec_run(mi_tdec_batch_t* b, const float* d_in, void* stream) {
  if (!b || !d_in) { mi::set_error("null argument"); return -1; }
  return b->eng.run_codeblocks(d_in, reinterpret_cast<hipStream_t>(stream));
}
int mi_tdec_download(mi_tdec_batch_t* b, uint8_t* bits, uint32_t* its, uint32_t* crc_ok) {
  const mi::Plan& P = b->eng.plan;
  if (!mi::hip_ok(hipStreamSynchronize(b->eng.last_stream), "sync")) return -1;
  std::vector<uint32_t> li(P.lanes.size()), lc(P.lanes.size());
  std::vector<uint8_t> rows((size_t)P.lanes.size() * mi::CB_BYTES_STRIDE);
  bool ok = mi::hip_ok(hipMemcpy(rows.data(), b->eng.d_cbbytes.p, rows.size(), hipMemcpyDeviceToHost), "D2H") &&
            mi::hip_ok(hipMemcpy(li.data(), b->eng.d_cbits.p, li.size() * 4, hipMemcpyDeviceToHost), "D2H") &&
            mi::hip_ok(hipMemcpy(lc.data(), b->eng.d_cbcrc.p, lc.size() * 4, hipMemcpyDeviceToHost), "D2H");
  if (!ok) return -1;
  for (uint32_t c = 0; c < P.cb_n; c++) {   // lanes are in code-block order
    if (bits) memcpy(bits + (size_t)c * (P.cb_K / 8), &rows[(size_t)c * mi::CB_BYTES_STRIDE], P.cb_K / 8);
    if (its) its[c] = li[c];
    if (crc_ok) crc_ok[c] = lc[c];
  }
  return 0;
}
int mi_tdec_stage_ms(mi_tdec_batch_t* b, float* ms, uint32_t* nruns) { return b->eng.stage_ms(ms, nruns); }
void mi_tdec_profile_reset(mi_tdec_batch_t* b) { b->eng.profile_reset(); }
double mi_tdec_algo_bytes(const mi_tdec_batch_t* b) { return b->eng.plan.stage_bytes[MI_DL_STAGE_TDEC]; }
int mi_tdec_turbo_win(const mi_tdec_batch_t* b) { return turbo_sched(b->eng); }

// ---- host-IQ pipeline (double buffering) ---------------------------------------
}  // extern "C"

struct mi_dl_pipe {
  mi_dl_batch_t* slot[2] = {nullptr, nullptr};
  mi::DevBuf iq[2];
  hipStream_t copy = nullptr, comp = nullptr;
  hipEvent_t copied[2] = {nullptr, nullptr}, decoded[2] = {nullptr, nullptr};
  bool busy[2] = {false, false};
  int next = 0;
  size_t iq_bytes = 0;
  ~mi_dl_pipe() {
    if (comp) (void)hipStreamSynchronize(comp);
    if (copy) (void)hipStreamSynchronize(copy);
    for (int s = 0; s < 2; s++) {
      if (copied[s]) (void)hipEventDestroy(copied[s]);
      if (decoded[s]) (void)hipEventDestroy(decoded[s]);
      delete slot[s];
    }
    if (copy) (void)hipStreamDestroy(copy);
    if (comp) (void)hipStreamDestroy(comp);
  }
};

extern "C" {

mi_dl_pipe_t* mi_dl_pipe_create(const mi_dl_sf_cfg_t* cfgs, uint32_t n_sf, uint32_t max_its, uint32_t flags) {
  auto* p = new mi_dl_pipe();
  bool ok = mi::hip_ok(hipStreamCreateWithFlags(&p->copy, hipStreamNonBlocking), "stream") &&
            mi::hip_ok(hipStreamCreateWithFlags(&p->comp, hipStreamNonBlocking), "stream");
  for (int s = 0; ok && s < 2; s++) {
    p->slot[s] = mi_dl_batch_create(cfgs, n_sf, max_its, flags);
    ok = p->slot[s] != nullptr;
    if (ok) {
      p->iq_bytes = mi_dl_batch_iq_samples(p->slot[s]) * ((flags & MI_DL_FLAG_IQ_SC16) ? 4 : 8);
      ok = p->iq[s].ensure(p->iq_bytes) &&
           mi::hip_ok(hipEventCreateWithFlags(&p->copied[s], hipEventDisableTiming), "event") &&
           mi::hip_ok(hipEventCreateWithFlags(&p->decoded[s], hipEventDisableTiming), "event");
    }
  }
  if (!ok) { delete p; return nullptr; }
  return p;
}

void mi_dl_pipe_destroy(mi_dl_pipe_t* p) { delete p; }

int mi_dl_pipe_submit(mi_dl_pipe_t* p, const void* host_iq) {
  if (!p || !host_iq) { mi::set_error("null argument"); return -1; }
  const int s = p->next;
  // the slot's previous decode must have consumed its device IQ before the copy overwrites it
  bool ok = (!p->busy[s] || mi::hip_ok(hipStreamWaitEvent(p->copy, p->decoded[s], 0), "wait")) &&
            mi::hip_ok(hipMemcpyAsync(p->iq[s].p, host_iq, p->iq_bytes, hipMemcpyHostToDevice, p->copy), "H2D") &&
            mi::hip_ok(hipEventRecord(p->copied[s], p->copy), "record") &&
            mi::hip_ok(hipStreamWaitEvent(p->comp, p->copied[s], 0), "wait") &&
            p->slot[s]->eng.run(p->iq[s].p, p->comp, 0xFFFFFFFFu, nullptr) == 0 &&
            mi::hip_ok(hipEventRecord(p->decoded[s], p->comp), "record");
  if (!ok) return -1;
  p->busy[s] = true;
  p->next ^= 1;
  return s;
}

int mi_dl_pipe_wait(mi_dl_pipe_t* p, int slot) {
  if (!p || slot < 0 || slot > 1) { mi::set_error("bad slot"); return -1; }
  if (!p->busy[slot]) return 0;
  return mi::hip_ok(hipEventSynchronize(p->decoded[slot]), "event sync") ? 0 : -1;
}

mi_dl_batch_t* mi_dl_pipe_batch(mi_dl_pipe_t* p, int slot) {
  return (p && slot >= 0 && slot < 2) ? p->slot[slot] : nullptr;
}

void* mi_host_alloc(size_t bytes) {
  void* h = nullptr;
  return mi::hip_ok(hipHostMalloc(&h, bytes, hipHostMallocDefault), "hipHostMalloc") ? h : nullptr;
}
void mi_host_free(void* h) {
  if (h) (void)hipHostFree(h);
}

int mi_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
int mi_set_device(int dev) { return mi::hip_ok(hipSetDevice(dev), "hipSetDevice") ? 0 : -1; }

int mi_stream_create_cu_share(uint32_t first, uint32_t count, void** stream) {
  if (!stream || !count || first >= 8 || first + count > 8) {
    mi::set_error("mi_stream_create_cu_share: eighths [first, first + count) must lie in [0, 8)");
    return -1;
  }
  hipStream_t s = nullptr;
  if (count == 8) {
    if (!mi::hip_ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "stream")) return -1;
  } else {
    int dev = 0, n_cu = 0;
    if (!mi::hip_ok(hipGetDevice(&dev), "device") ||
        !mi::hip_ok(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev), "CU count"))
      return -1;
    // CU i is in the share when i mod 8 lies in [first, first + count): every eighth CU index, so that the share
    // spans the device's XCDs and shader engines evenly
    std::vector<uint32_t> mask(((size_t)n_cu + 31) / 32, 0u);
    for (int i = 0; i < n_cu; i++)
      if ((uint32_t)(i % 8) - first < count) mask[i / 32] |= 1u << (i % 32);
    if (!mi::hip_ok(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()), "CU-masked stream"))
      return -1;
  }
  *stream = s;
  return 0;
}
int mi_stream_destroy(void* stream) {
  return mi::hip_ok(hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)), "stream destroy") ? 0 : -1;
}
const char* mi_last_error(void) { return mi::last_error(); }

}  // extern "C"
