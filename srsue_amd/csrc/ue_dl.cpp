// ue_dl.cpp -- the srsLTE-1.0 DL entry points srsUE's phch_worker calls, backed by the MI355X
// engine (include/srslte/srslte.h documents each call site in /root/reference).
//
// Per srslte_ue_dl_t instance (one per phch_worker thread, phch_worker.h:111): one HIP stream,
// one Engine (HBM workspace for one subframe), host mirrors of the grid and channel estimates
// (srsUE reads them on the host for PDCCH, phch_worker.cc:260).  Re-entrant per instance, no
// global mutable state besides the cached read-only spec tables inside each Engine.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <memory>
#include <tuple>
#include <vector>

#include "../../include/srslte/srslte.h"
#include "ctrl.h"
#include "engine.h"
#include "tables.h"

struct mi_ue_dl_ctx {
  mi::Engine eng;
  hipStream_t st = nullptr;
  mi::DevBuf d_iq;
  // page-locked staging: the subframe's IQ (srsUE's buffer is pageable; a pageable H2D costs ~70 us
  // through HIP's own staging), the small per-call results and the payload
  cf_t* h_iq = nullptr;
  struct Small { float met[5]; uint32_t cfi, tb_ok, its; float phich; };
  Small* h_small = nullptr;
  uint8_t* h_pay = nullptr;
  static constexpr size_t MAX_TB_BYTES = 16384;   // > 75,376 bits, the largest single-layer TBS
  mi_dl_sf_cfg_t cfg{};    // current subframe configuration
  uint32_t cfi = 1, sf_idx = 0;
  bool fft_done = false;
  cf_t* host_grid = nullptr;
  cf_t* host_ce[SRSLTE_MAX_PORTS] = {};
  mi::CtrlEngine ctrl;     // PCFICH / PDCCH / DCI blind search over eng's grid and ce (ctrl.hip)
  // control-plan memo: (sf_idx, cfi, rnti, PHICH query) -> parked tables (ctrl_plan); -1 = none active
  struct CtrlMemo {
    std::tuple<uint32_t, uint32_t, uint32_t, uint32_t> key;
    mi::CtrlTables t;
    uint64_t used = 0;
  };
  std::vector<std::unique_ptr<CtrlMemo>> ctrl_memo;
  int ctrl_active = -1;
  uint64_t ctrl_clock = 0;
  uint32_t phich_ng = 0;
  bool llr_done = false;
  // per-phase host-clock breakdown of the per-TTI calls (MI_UE_DL_PROF=1: the stream is synchronised at
  // every mark so GPU work is attributed to its phase; printed to stderr by srslte_ue_dl_free)
  struct Prof {
    bool on = getenv("MI_UE_DL_PROF") != nullptr;
    double acc[12] = {}, last = 0;
    uint64_t n[12] = {};
    static double now() {
      timespec t;
      clock_gettime(CLOCK_MONOTONIC, &t);
      return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
    }
    void start() { if (on) last = now(); }
    void mark(int i, hipStream_t st) {
      if (!on) return;
      (void)hipStreamSynchronize(st);
      const double t = now();
      acc[i] += t - last; n[i]++; last = t;
    }
  } prof;
  ~mi_ue_dl_ctx() {
    if (st) (void)hipStreamSynchronize(st);
    for (void* p : {(void*)h_iq, (void*)h_small, (void*)h_pay})
      if (p) (void)hipHostFree(p);
    if (st) (void)hipStreamDestroy(st);
  }
};

namespace {

// plan the control stage for the instance's single subframe.  srsUE asks for the same few plans every
// frame (per subframe index: PCFICH, PDCCH soft bits, the blind search of each RNTI, PHICH), so built
// plans are memoised: a repeat swaps its parked tables (device copies included) back in.
bool ctrl_plan(mi_ue_dl_ctx* c, uint32_t cfi, uint16_t rnti, uint32_t phich_q = 0) {
  const auto key = std::make_tuple(c->sf_idx, cfi, (uint32_t)rnti, phich_q);
  if (c->ctrl_active >= 0) {
    if (c->ctrl_memo[(size_t)c->ctrl_active]->key == key) return true;
    c->ctrl.swap_tables(c->ctrl_memo[(size_t)c->ctrl_active]->t);   // park
    c->ctrl_active = -1;
  }
  int hit = -1;
  for (size_t i = 0; i < c->ctrl_memo.size(); i++)
    if (c->ctrl_memo[i]->key == key) { hit = (int)i; break; }
  if (hit < 0) {
    if (c->ctrl.build(c->eng.plan, std::vector<uint32_t>{cfi}, c->phich_ng, std::vector<uint16_t>{rnti},
                      std::vector<uint32_t>{phich_q}) != 0 ||
        c->ctrl.upload(c->st) != 0)
      return false;
    if (c->ctrl_memo.size() >= 64) {   // least recently used entry out (upload synchronised the stream)
      size_t lru = 0;
      for (size_t i = 1; i < c->ctrl_memo.size(); i++)
        if (c->ctrl_memo[i]->used < c->ctrl_memo[lru]->used) lru = i;
      c->ctrl_memo.erase(c->ctrl_memo.begin() + (ptrdiff_t)lru);
    }
    c->ctrl_memo.push_back(std::make_unique<mi_ue_dl_ctx::CtrlMemo>());
    hit = (int)c->ctrl_memo.size() - 1;
    c->ctrl_memo.back()->key = key;
    c->ctrl.swap_tables(c->ctrl_memo.back()->t);   // park the fresh build, re-activated below
  }
  c->ctrl.swap_tables(c->ctrl_memo[(size_t)hit]->t);
  c->ctrl_active = hit;
  c->ctrl_memo[(size_t)hit]->used = ++c->ctrl_clock;
  return true;
}

// grid / ce on the device: the copies decode_fft_estimate left are reused when the caller passes this
// instance's own host mirrors (srsUE passes ue_dl.sf_symbols / ue_dl.ce); other buffers are uploaded
bool device_grid(mi_ue_dl_ctx* c, const srslte_cell_t& cell, cf_t* sf_symbols, cf_t* const* ce) {
  const size_t n = (size_t)mi::NSYMB * 12 * cell.nof_prb;
  bool own = c->fft_done && sf_symbols == c->host_grid;
  for (uint32_t p = 0; p < cell.nof_ports; p++) own = own && ce[p] == c->host_ce[p];
  if (own) return true;
  bool ok = mi::hip_ok(hipMemcpyAsync(c->eng.d_grid.p, sf_symbols, n * 8, hipMemcpyHostToDevice, c->st), "H2D grid");
  for (uint32_t p = 0; p < cell.nof_ports && ok; p++)
    ok = mi::hip_ok(hipMemcpyAsync(c->eng.d_ce.as<float2>() + p * n, ce[p], n * 8, hipMemcpyHostToDevice, c->st),
                    "H2D ce");
  return ok;
}

// error return after work was enqueued on the instance stream: the next call rewrites the page-locked
// staging (h_iq, h_small, h_pay) assuming the previous call's copies ended at its stream sync, so an
// early return drains the stream first
int fail_sync(mi_ue_dl_ctx* c) {
  (void)hipStreamSynchronize(c->st);
  return SRSLTE_ERROR;
}

uint32_t mod_bits(srslte_mod_t m) {
  switch (m) {
    case SRSLTE_MOD_BPSK: return 1;
    case SRSLTE_MOD_QPSK: return 2;
    case SRSLTE_MOD_16QAM: return 4;
    case SRSLTE_MOD_64QAM: return 6;
    default: return 0;
  }
}

}  // namespace

extern "C" {

/* ---- version ------------------------------------------------------------------------------ */
int srslte_get_version_major(void) { return SRSLTE_VERSION_MAJOR; }
int srslte_get_version_minor(void) { return SRSLTE_VERSION_MINOR; }
int srslte_get_version_patch(void) { return SRSLTE_VERSION_PATCH; }
char* srslte_get_version(void) { return const_cast<char*>(SRSLTE_VERSION_STRING); }
int srslte_check_version(int major, int minor, int patch) {
  return SRSLTE_VERSION >= SRSLTE_VERSION_ENCODE(major, minor, patch);
}

/* ---- misc --------------------------------------------------------------------------------- */
int srslte_symbol_sz(uint32_t nof_prb) { return mi::symbol_sz(nof_prb); }
void* srslte_vec_malloc(uint32_t size) {
  void* p = nullptr;
  if (posix_memalign(&p, 256, size ? size : 1)) return nullptr;
  return p;
}
void srslte_vec_free(void* ptr) { free(ptr); }

int srslte_ra_tbs_idx_from_mcs(uint32_t mcs) {
  uint32_t qm;
  return mi::mcs_to_itbs(mcs, &qm);
}
srslte_mod_t srslte_ra_mod_from_mcs(uint32_t mcs) {
  uint32_t qm = 0;
  if (mi::mcs_to_itbs(mcs, &qm) < 0) return SRSLTE_MOD_LAST;
  return qm == 2 ? SRSLTE_MOD_QPSK : qm == 4 ? SRSLTE_MOD_16QAM : SRSLTE_MOD_64QAM;
}
int srslte_ra_tbs_from_idx(uint32_t tbs_idx, uint32_t n_prb) { return mi::tbs_from_idx(tbs_idx, n_prb); }
uint32_t srslte_mod_bits_x_symbol(srslte_mod_t mod) { return mod_bits(mod); }
int srslte_cbsegm(srslte_cbsegm_t* s, uint32_t tbs) {
  mi::CbSegm g;
  if (!s || mi::cbsegm(tbs, &g)) return SRSLTE_ERROR;
  s->F = g.F; s->C = g.C; s->K1 = g.Kp; s->K2 = g.Km; s->C1 = g.Cp; s->C2 = g.Cm; s->tbs = tbs;
  return SRSLTE_SUCCESS;
}

/* ---- softbuffer --------------------------------------------------------------------------- */
int srslte_softbuffer_rx_init(srslte_softbuffer_rx_t* q, uint32_t nof_prb) {
  if (!q) return SRSLTE_ERROR_INVALID_INPUTS;
  memset(q, 0, sizeof(*q));
  // max code blocks of the largest single-layer TBS at nof_prb (13 at 100 PRB)
  q->max_cb = (nof_prb * 12 * 14 * 6 + 6119) / 6120 + 1;
  q->dev_bytes = (uint64_t)2 * mi::sb_group_floats(mi::NCB_MAX) * sizeof(float);
  if (hipMalloc(&q->dev, q->dev_bytes) != hipSuccess) { q->dev = nullptr; return SRSLTE_ERROR; }
  srslte_softbuffer_rx_reset(q);
  return SRSLTE_SUCCESS;
}
void srslte_softbuffer_rx_free(srslte_softbuffer_rx_t* q) {
  if (q && q->dev) (void)hipFree(q->dev);
  if (q) memset(q, 0, sizeof(*q));
}
void srslte_softbuffer_rx_reset(srslte_softbuffer_rx_t* q) {
  // == RX_NULL everywhere from the next decode on.  The clear itself runs on the decoding instance's stream, ordered
  // before that decode (srslte_pdsch_decode_rnti): a memset here would run on the null stream, which the instances'
  // non-blocking streams do not wait for -- beside other workers' decodes it could still be clearing while the next
  // decode combined into the arena
  if (q) q->reset_pending = 1;
}
void srslte_softbuffer_rx_reset_tbs(srslte_softbuffer_rx_t* q, uint32_t /*tbs*/) {
  // srsLTE resets the rows of the TB's code blocks; the arena only ever holds one TB
  srslte_softbuffer_rx_reset(q);
}

/* ---- UE DL --------------------------------------------------------------------------------- */
int srslte_ue_dl_init(srslte_ue_dl_t* q, srslte_cell_t cell) {
  if (!q || mi::symbol_sz(cell.nof_prb) < 0 || cell.nof_ports < 1 || cell.nof_ports > 2 || cell.cp != SRSLTE_CP_NORM)
    return SRSLTE_ERROR_INVALID_INPUTS;
  memset(q, 0, sizeof(*q));
  q->cell = cell;
  q->pdsch.cell = cell;
  q->chest.cell = cell;
  q->pdcch.cell = cell;
  q->pdsch.dl_sch.max_iterations = SRSLTE_PDSCH_MAX_TDEC_ITERS;
  auto* ctx = new mi_ue_dl_ctx();
  if (hipStreamCreateWithFlags(&ctx->st, hipStreamNonBlocking) != hipSuccess) { delete ctx; return SRSLTE_ERROR; }
  const size_t W = 12 * cell.nof_prb, n = (size_t)mi::NSYMB * W;
  // host mirrors of the grid / estimates (srsUE reads them, phch_worker.cc:260): page-locked, so their
  // per-TTI D2H copies are direct DMA (this library allocates and frees them)
  auto host_alloc = [](size_t bytes) -> cf_t* {
    void* p = nullptr;
    return hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess ? (cf_t*)p : nullptr;
  };
  q->sf_symbols = host_alloc(n * sizeof(cf_t));
  for (uint32_t p = 0; p < cell.nof_ports; p++) q->ce[p] = host_alloc(n * sizeof(cf_t));
  if (!q->sf_symbols || !q->ce[0] || (cell.nof_ports == 2 && !q->ce[1])) { delete ctx; return SRSLTE_ERROR; }
  const size_t sfl = (size_t)mi::sf_len(mi::symbol_sz(cell.nof_prb));
  if (!ctx->d_iq.ensure(sfl * 8)) { delete ctx; return SRSLTE_ERROR; }
  ctx->h_iq = host_alloc(sfl * sizeof(cf_t));
  ctx->h_small = reinterpret_cast<mi_ue_dl_ctx::Small*>(host_alloc(sizeof(mi_ue_dl_ctx::Small)));
  ctx->h_pay = reinterpret_cast<uint8_t*>(host_alloc(mi_ue_dl_ctx::MAX_TB_BYTES));
  if (!ctx->h_iq || !ctx->h_small || !ctx->h_pay) { delete ctx; return SRSLTE_ERROR; }
  ctx->cfg.cell_id = cell.id;
  ctx->cfg.nof_prb = cell.nof_prb;
  ctx->cfg.nof_ports = cell.nof_ports;
  ctx->cfg.tm = cell.nof_ports == 2 ? 2 : 1;
  ctx->cfg.nl_td = 2;
  ctx->host_grid = q->sf_symbols;
  for (int p = 0; p < SRSLTE_MAX_PORTS; p++) ctx->host_ce[p] = q->ce[p];
  ctx->phich_ng = (uint32_t)cell.phich_resources;
  q->ctx = ctx;
  q->pdsch.ctx = ctx;
  q->pdcch.ctx = ctx;
  return SRSLTE_SUCCESS;
}

void srslte_ue_dl_free(srslte_ue_dl_t* q) {
  if (!q) return;
  if (q->ctx) {
    const auto& pf = q->ctx->prof;
    if (pf.on) {
      static const char* names[11] = {"fft.h2d_iq", "fft.plan_upload", "fft.ofdm_chest", "fft.ctrl_plan", "fft.pcfich",
                                      "fft.d2h_sync", "pdsch.plan_upload", "-", "pdsch.grid", "pdsch.kernels",
                                      "pdsch.d2h_sync"};
      fprintf(stderr, "{\"ue_dl_prof_us\": {");
      for (int i = 0; i < 11; i++)
        fprintf(stderr, "\"%s\": %.1f%s", names[i], pf.n[i] ? pf.acc[i] / (double)pf.n[i] : 0.0, i < 10 ? ", " : "");
      fprintf(stderr, "}}\n");
    }
    delete q->ctx;
  }
  if (q->sf_symbols) (void)hipHostFree(q->sf_symbols);
  for (int p = 0; p < SRSLTE_MAX_PORTS; p++)
    if (q->ce[p]) (void)hipHostFree(q->ce[p]);
  memset(q, 0, sizeof(*q));
}

void srslte_ue_dl_set_rnti(srslte_ue_dl_t* q, uint16_t rnti) {
  if (!q) return;
  q->current_rnti = rnti;
  q->pdsch.rnti = rnti;
  q->pdsch.rnti_is_set = true;
}

int srslte_ue_dl_decode_fft_estimate(srslte_ue_dl_t* q, cf_t* input, uint32_t sf_idx, uint32_t* cfi) {
  if (!q || !q->ctx || !input || sf_idx > 9) return SRSLTE_ERROR_INVALID_INPUTS;
  mi_ue_dl_ctx* c = q->ctx;
  c->cfg.sf_idx = sf_idx;
  c->sf_idx = sf_idx;
  const size_t W = 12 * q->cell.nof_prb, n = (size_t)mi::NSYMB * W;
  const size_t sfl = (size_t)mi::sf_len(mi::symbol_sz(q->cell.nof_prb));
  c->prof.start();
  memcpy(c->h_iq, input, sfl * 8);   // the previous call's DMA out of h_iq ended with its stream sync
  if (!mi::hip_ok(hipMemcpyAsync(c->d_iq.p, c->h_iq, sfl * 8, hipMemcpyHostToDevice, c->st), "H2D iq"))
    return fail_sync(c);
  c->prof.mark(0, c->st);
  if (c->eng.plan_memo(&c->cfg, 1, false, c->st)) return fail_sync(c);
  c->prof.mark(1, c->st);
  if (c->eng.run(c->d_iq.p, c->st, (1u << MI_DL_STAGE_OFDM) | (1u << MI_DL_STAGE_CHEST), nullptr)) return fail_sync(c);
  c->prof.mark(2, c->st);
  // PCFICH -> CFI on the GPU (the control plan's PCFICH tables do not depend on the CFI)
  if (!ctrl_plan(c, 1, q->current_rnti)) return fail_sync(c);
  c->prof.mark(3, c->st);
  if (c->ctrl.run(c->eng.d_grid.as<float2>(), c->eng.d_ce.as<float2>(), 1u, 0.0f, c->st)) return fail_sync(c);
  c->prof.mark(4, c->st);
  mi_ue_dl_ctx::Small* hs = c->h_small;
  bool ok = mi::hip_ok(hipMemcpyAsync(q->sf_symbols, c->eng.d_grid.p, n * 8, hipMemcpyDeviceToHost, c->st), "D2H");
  for (uint32_t p = 0; p < q->cell.nof_ports && ok; p++)
    ok = mi::hip_ok(hipMemcpyAsync(q->ce[p], c->eng.d_ce.as<float2>() + p * n, n * 8, hipMemcpyDeviceToHost, c->st), "D2H");
  ok = ok && mi::hip_ok(hipMemcpyAsync(hs->met, c->eng.d_metrics.p, sizeof(hs->met), hipMemcpyDeviceToHost, c->st), "D2H") &&
       mi::hip_ok(hipMemcpyAsync(&hs->cfi, c->ctrl.d_cfi.p, 4, hipMemcpyDeviceToHost, c->st), "D2H") &&
       mi::hip_ok(hipStreamSynchronize(c->st), "sync");
  const float* met = hs->met;
  const uint32_t cf = hs->cfi;
  if (!ok) return fail_sync(c);
  c->prof.mark(5, c->st);
  q->chest.rsrp = met[0]; q->chest.rssi = met[1]; q->chest.rsrq = met[2];
  q->chest.noise_estimate = met[3]; q->chest.snr = met[4];
  if (cf < 1 || cf > 3) return SRSLTE_ERROR;
  c->llr_done = false;
  q->cfi = cf;
  c->cfi = cf;
  c->fft_done = true;
  if (cfi) *cfi = cf;
  return SRSLTE_SUCCESS;
}

// grant PRBs per slot -> the two-slot mask encoding of mi_dl_sf_cfg_t (bit s: used in slot s)
static void slot_mask(const srslte_ra_dl_grant_t* g, uint8_t* mask) {
  for (int p = 0; p < SRSLTE_MAX_PRB; p++) mask[p] = (uint8_t)((g->prb_idx[0][p] ? 1u : 0u) | (g->prb_idx[1][p] ? 2u : 0u));
}

int srslte_ue_dl_cfg_grant(srslte_ue_dl_t* q, srslte_ra_dl_grant_t* grant, uint32_t cfi, uint32_t sf_idx,
                           uint32_t rvidx) {
  if (!q || !grant || cfi < 1 || cfi > 3 || sf_idx > 9 || rvidx > 3) return SRSLTE_ERROR_INVALID_INPUTS;
  srslte_pdsch_cfg_t* pc = &q->pdsch_cfg;
  memcpy(&pc->grant, grant, sizeof(*grant));
  if (!pc->grant.Qm) pc->grant.Qm = mod_bits(grant->mcs.mod);
  pc->rv = rvidx;
  pc->sf_idx = sf_idx;
  pc->mimo_type = q->cell.nof_ports == 2 ? SRSLTE_MIMO_TYPE_TX_DIVERSITY : SRSLTE_MIMO_TYPE_SINGLE_ANTENNA;
  pc->nof_layers = q->cell.nof_ports;
  uint8_t mask[SRSLTE_MAX_PRB];
  slot_mask(grant, mask);
  std::vector<uint32_t> re;
  pc->nbits.nof_re = mi::pdsch_re_list(q->cell.id, q->cell.nof_prb, q->cell.nof_ports, cfi, sf_idx, mask, re);
  pc->nbits.nof_bits = pc->nbits.nof_re * pc->grant.Qm;
  pc->nbits.lstart = (uint32_t)mi::ctrl_symbols(q->cell.nof_prb, cfi);
  pc->nbits.nof_symb = 2 * SRSLTE_CP_NORM_NSYMB - pc->nbits.lstart;
  if (grant->mcs.tbs > 0 && srslte_cbsegm(&pc->cb_segm, (uint32_t)grant->mcs.tbs)) return SRSLTE_ERROR;
  q->cfi = cfi;
  if (q->ctx) q->ctx->cfi = cfi;
  return SRSLTE_SUCCESS;
}

/* ---- PDSCH --------------------------------------------------------------------------------- */
int srslte_pdsch_decode_rnti(srslte_pdsch_t* q, srslte_pdsch_cfg_t* cfg, srslte_softbuffer_rx_t* softbuffer,
                             cf_t* sf_symbols, cf_t* ce[SRSLTE_MAX_PORTS], float noise_estimate, uint16_t rnti,
                             uint8_t* data) {
  if (!q || !q->ctx || !cfg || !softbuffer || !softbuffer->dev || !sf_symbols || !ce || !data)
    return SRSLTE_ERROR_INVALID_INPUTS;
  mi_ue_dl_ctx* c = q->ctx;
  const srslte_cell_t& cell = q->cell;
  if (cfg->grant.mcs.tbs <= 0 || cfg->grant.mcs.tbs % 8) return SRSLTE_ERROR_INVALID_INPUTS;
  mi_dl_sf_cfg_t s = c->cfg;
  s.sf_idx = cfg->sf_idx;
  s.cfi = c->cfi;
  s.rnti = rnti;
  s.rv = cfg->rv;
  s.tbs = (uint32_t)cfg->grant.mcs.tbs;
  s.Qm = cfg->grant.Qm ? cfg->grant.Qm : mod_bits(cfg->grant.mcs.mod);
  s.new_tb = 0;   // the MAC resets the softbuffer for a new TB (srslte_softbuffer_rx_reset_tbs)
  slot_mask(&cfg->grant, s.prb_mask);
  c->eng.noise = noise_estimate;
  c->eng.max_its = q->dl_sch.max_iterations ? q->dl_sch.max_iterations : SRSLTE_PDSCH_MAX_TDEC_ITERS;
  c->prof.start();
  if (c->eng.plan_memo(&s, 1, true, c->st)) return fail_sync(c);
  c->prof.mark(6, c->st);
  if (c->eng.plan.sb_floats * sizeof(float) > softbuffer->dev_bytes) return fail_sync(c);
  bool ok = device_grid(c, cell, sf_symbols, ce);
  if (!ok) return fail_sync(c);
  if (softbuffer->reset_pending) {   // srslte_softbuffer_rx_reset since the last decode: RX_NULL, ordered on this stream
    if (!mi::hip_ok(hipMemsetAsync(softbuffer->dev, 0, softbuffer->dev_bytes, c->st), "softbuffer reset"))
      return fail_sync(c);
    softbuffer->reset_pending = 0;
  }
  c->prof.mark(8, c->st);
  const uint32_t stages = (1u << MI_DL_STAGE_DEMAP) | (1u << MI_DL_STAGE_RM) | (1u << MI_DL_STAGE_TDEC) |
                          (1u << MI_DL_STAGE_TB);
  if (c->eng.run(nullptr, c->st, stages, reinterpret_cast<float*>(softbuffer->dev))) return fail_sync(c);
  c->prof.mark(9, c->st);
  if (s.tbs / 8 > mi_ue_dl_ctx::MAX_TB_BYTES) return fail_sync(c);
  mi_ue_dl_ctx::Small* hs = c->h_small;
  ok = mi::hip_ok(hipMemcpyAsync(c->h_pay, c->eng.d_payload.p, s.tbs / 8, hipMemcpyDeviceToHost, c->st), "D2H") &&
       mi::hip_ok(hipMemcpyAsync(&hs->tb_ok, c->eng.d_tbok.p, 4, hipMemcpyDeviceToHost, c->st), "D2H") &&
       mi::hip_ok(hipMemcpyAsync(&hs->its, c->eng.d_tbits.p, 4, hipMemcpyDeviceToHost, c->st), "D2H") &&
       mi::hip_ok(hipStreamSynchronize(c->st), "sync");
  if (!ok) return fail_sync(c);
  memcpy(data, c->h_pay, s.tbs / 8);
  const uint32_t tb_ok = hs->tb_ok, its = hs->its;
  c->prof.mark(10, c->st);
  q->dl_sch.nof_iterations = its;
  q->dl_sch.average_nof_iterations = 0.8f * q->dl_sch.average_nof_iterations + 0.2f * (float)its;
  return tb_ok ? SRSLTE_SUCCESS : SRSLTE_ERROR;
}

uint32_t srslte_pdsch_last_noi(srslte_pdsch_t* q) { return q ? q->dl_sch.nof_iterations : 0; }
void srslte_sch_set_max_noi(srslte_sch_t* q, uint32_t max_iterations) {
  if (q && max_iterations > 0) q->max_iterations = max_iterations;
}

/* ---- PDCCH / DCI --------------------------------------------------------------------------- */
int srslte_pdcch_extract_llr(srslte_pdcch_t* q, cf_t* sf_symbols, cf_t* ce[SRSLTE_MAX_PORTS], float noise_estimate,
                             uint32_t nsubframe, uint32_t cfi) {
  if (!q || !q->ctx || !sf_symbols || !ce || cfi < 1 || cfi > 3 || nsubframe > 9) return SRSLTE_ERROR_INVALID_INPUTS;
  mi_ue_dl_ctx* c = q->ctx;
  if (c->sf_idx != nsubframe || !c->fft_done) return SRSLTE_ERROR_INVALID_INPUTS;
  if (!device_grid(c, q->cell, sf_symbols, ce) || !ctrl_plan(c, cfi, 0) ||
      c->ctrl.run(c->eng.d_grid.as<float2>(), c->eng.d_ce.as<float2>(), 2u, noise_estimate, c->st))
    return SRSLTE_ERROR;
  c->cfi = cfi;
  c->llr_done = true;
  q->nof_cce = c->ctrl.sfs[0].n_cce;
  return SRSLTE_SUCCESS;
}

static int find_dci(srslte_ue_dl_t* q, srslte_dci_msg_t* msg, uint32_t cfi, uint32_t sf_idx, uint16_t rnti, bool ul,
                    bool common_only) {
  if (!q || !q->ctx || !msg || cfi < 1 || cfi > 3 || sf_idx > 9) return SRSLTE_ERROR_INVALID_INPUTS;
  mi_ue_dl_ctx* c = q->ctx;
  if (!c->llr_done || c->cfi != cfi || c->sf_idx != sf_idx) return SRSLTE_ERROR_INVALID_INPUTS;
  if (!ctrl_plan(c, cfi, rnti) || c->ctrl.run(nullptr, nullptr, 4u, 0.0f, c->st) || c->ctrl.download(c->st))
    return SRSLTE_ERROR;
  const mi::DciFound f = c->ctrl.select(0, ul, common_only);
  if (!f.found) return 0;
  memset(msg, 0, sizeof(*msg));
  memcpy(msg->data, f.bits, f.nbits);
  msg->nof_bits = f.nbits;
  msg->format = f.format == mi::DCI_0    ? SRSLTE_DCI_FORMAT0
                : f.format == mi::DCI_1  ? SRSLTE_DCI_FORMAT1
                : f.format == mi::DCI_1C ? SRSLTE_DCI_FORMAT1C
                                         : SRSLTE_DCI_FORMAT1A;
  q->last_location.L = f.L;
  q->last_location.ncce = f.ncce;
  q->last_n_cce = f.ncce;
  return 1;
}

int srslte_ue_dl_find_dl_dci_type(srslte_ue_dl_t* q, srslte_dci_msg_t* msg, uint32_t cfi, uint32_t sf_idx,
                                  uint16_t rnti, srslte_rnti_type_t type) {
  const bool common = type == SRSLTE_RNTI_SI || type == SRSLTE_RNTI_RAR || type == SRSLTE_RNTI_PCH;
  return find_dci(q, msg, cfi, sf_idx, rnti, false, common);
}
int srslte_ue_dl_find_dl_dci(srslte_ue_dl_t* q, srslte_dci_msg_t* msg, uint32_t cfi, uint32_t sf_idx, uint16_t rnti) {
  return find_dci(q, msg, cfi, sf_idx, rnti, false, false);
}
int srslte_ue_dl_find_ul_dci(srslte_ue_dl_t* q, srslte_dci_msg_t* msg, uint32_t cfi, uint32_t sf_idx, uint16_t rnti) {
  return find_dci(q, msg, cfi, sf_idx, rnti, true, false);
}
uint32_t srslte_ue_dl_get_ncce(srslte_ue_dl_t* q) { return q ? q->last_n_cce : 0; }

bool srslte_ue_dl_decode_phich(srslte_ue_dl_t* q, uint32_t sf_idx, uint32_t n_prb_lowest, uint32_t n_dmrs) {
  if (!q || !q->ctx || !q->ctx->fft_done || sf_idx != q->ctx->sf_idx || n_prb_lowest > 0xFFFFu || n_dmrs > 7)
    return false;
  mi_ue_dl_ctx* c = q->ctx;
  // the grid / ce of the last decode_fft_estimate are still in HBM (device_grid keeps them)
  if (!ctrl_plan(c, c->cfi ? c->cfi : 1, q->current_rnti, n_prb_lowest | (n_dmrs << 16)) ||
      c->ctrl.run(c->eng.d_grid.as<float2>(), c->eng.d_ce.as<float2>(), 8u, 0.0f, c->st) ||
      !mi::hip_ok(hipMemcpyAsync(&c->h_small->phich, c->ctrl.d_phich.p, 4, hipMemcpyDeviceToHost, c->st), "D2H") ||
      !mi::hip_ok(hipStreamSynchronize(c->st), "sync"))
    return false;
  const float soft = c->h_small->phich;
  // the rebuilt plan has the same CFI: the PDCCH soft bits stay valid for find_ul_dci (:426)
  return soft > 0.0f;
}

static uint32_t take_bits(const uint8_t* b, uint32_t* pos, uint32_t n) {
  uint32_t v = 0;
  for (uint32_t i = 0; i < n; i++) v = (v << 1) | b[(*pos)++];
  return v;
}

// 36.213 7.1.6.3: RIV over an N-wide space -> (start, L)
static bool riv_decode(uint32_t riv, uint32_t N, uint32_t* start, uint32_t* L) {
  if (!N) return false;
  const uint32_t a = riv / N, b = riv % N;
  if (a + b < N) { *L = a + 1; *start = b; }
  else { *L = N - a + 1; *start = N - 1 - b; }
  return *L >= 1 && *start + *L <= N && riv < N * (N + 1) / 2;
}

static void set_prb(srslte_ra_dl_grant_t* g, uint32_t slot, int p) {
  if (p >= 0 && p < SRSLTE_MAX_PRB) g->prb_idx[slot][p] = true;
}

int srslte_dci_msg_to_dl_grant(srslte_dci_msg_t* msg, uint16_t msg_rnti, uint32_t nof_prb, srslte_ra_dl_dci_t* dci,
                               srslte_ra_dl_grant_t* grant) {
  if (!msg || !dci || !grant || mi::symbol_sz(nof_prb) < 0) return SRSLTE_ERROR_INVALID_INPUTS;
  memset(dci, 0, sizeof(*dci));
  memset(grant, 0, sizeof(*grant));
  const uint32_t N = nof_prb, n1a = mi::dci_size(mi::DCI_1A, N), n1 = mi::dci_size(mi::DCI_1, N);
  const uint32_t n1c = mi::dci_size(mi::DCI_1C, N);
  // SI-RNTI, P-RNTI and RA-RNTI (1..60) scramble common-control DCIs (36.321 7.1)
  const bool common = msg_rnti < 0x003D || msg_rnti > 0xFFF3;
  uint32_t pos = 0, itbs_1a_common = 0, nprb_tbs = 0;
  if (msg->nof_bits == n1a && msg->data[0] == 1) {
    // format 1A (36.212 5.3.3.1.3): flag, L/D VRB flag, RBA, MCS, HARQ, NDI, RV, TPC
    const uint32_t rba = mi::ceil_log2(N * (N + 1) / 2);
    pos = 1;
    const bool dist = take_bits(msg->data, &pos, 1) != 0;
    // distributed, N_RB >= 50, C-RNTI: the RBA's MSB selects the gap (N_gap,1 / N_gap,2)
    const bool gap_in_rba = dist && N >= 50 && !common;
    const uint32_t gap_rba = gap_in_rba ? take_bits(msg->data, &pos, 1) : 0;
    const uint32_t riv = take_bits(msg->data, &pos, gap_in_rba ? rba - 1 : rba);
    uint32_t start, L;
    if (!riv_decode(riv, N, &start, &L)) return SRSLTE_ERROR;
    dci->mcs_idx = take_bits(msg->data, &pos, 5);
    dci->harq_process = take_bits(msg->data, &pos, 3);
    const uint32_t ndi = take_bits(msg->data, &pos, 1);
    dci->rv_idx = take_bits(msg->data, &pos, 2);
    dci->tpc_pucch = take_bits(msg->data, &pos, 2);
    // SI/RA/P-RNTI: the NDI bit carries the gap of a distributed allocation (N_RB >= 50), the TPC LSB the
    // TBS column N_PRB^1A (36.213 7.1.7.2.1: 2 or 3 PRBs), modulation QPSK with I_TBS = I_MCS
    dci->ndi = !common && ndi;
    dci->type2_gap = gap_in_rba ? gap_rba : (common && dist && N >= 50) ? ndi : 0;
    dci->alloc_type = SRSLTE_RA_ALLOC_TYPE2;
    dci->type2_start = start;
    dci->type2_len = L;
    dci->type2_distributed = dist;
    dci->dci_format = SRSLTE_DCI_FORMAT1A;
    if (!dist) {
      for (uint32_t p = start; p < start + L; p++) grant->prb_idx[0][p] = grant->prb_idx[1][p] = true;
    } else {
      if (start + L > mi::n_vrb_dist(N, dci->type2_gap != 0)) return SRSLTE_ERROR;
      for (uint32_t n = start; n < start + L; n++)
        for (uint32_t s = 0; s < 2; s++) set_prb(grant, s, mi::vrb_to_prb(N, dci->type2_gap != 0, n, s));
    }
    grant->nof_prb = L;
    if (common) {
      itbs_1a_common = 1;
      nprb_tbs = (dci->tpc_pucch & 1u) ? 3 : 2;
    } else {
      nprb_tbs = L;
    }
  } else if (msg->nof_bits == n1c && common) {
    // format 1C (36.212 5.3.3.1.4): [gap if N_RB >= 50], RBA over N'_VRB = N_VRB,gap1 / N_step, I_TBS
    const uint32_t step = N < 50 ? 2 : 4, np = mi::n_vrb_dist(N, false) / step;
    dci->type2_gap = N >= 50 ? take_bits(msg->data, &pos, 1) : 0;
    const uint32_t riv = take_bits(msg->data, &pos, mi::dci1c_rba_bits(N));
    uint32_t s1, l1;
    if (!riv_decode(riv, np, &s1, &l1)) return SRSLTE_ERROR;
    const uint32_t start = s1 * step, L = l1 * step;
    if (start + L > mi::n_vrb_dist(N, dci->type2_gap != 0)) return SRSLTE_ERROR;
    dci->mcs_idx = take_bits(msg->data, &pos, 5);
    dci->alloc_type = SRSLTE_RA_ALLOC_TYPE2;
    dci->type2_start = start;
    dci->type2_len = L;
    dci->type2_distributed = true;
    dci->dci_format = SRSLTE_DCI_FORMAT1C;
    for (uint32_t n = start; n < start + L; n++)
      for (uint32_t s = 0; s < 2; s++) set_prb(grant, s, mi::vrb_to_prb(N, dci->type2_gap != 0, n, s));
    grant->nof_prb = L;
    grant->Qm = 2;
    grant->mcs.idx = dci->mcs_idx;
    grant->mcs.tbs = mi::tbs_1c(dci->mcs_idx);
    grant->mcs.mod = SRSLTE_MOD_QPSK;
    return SRSLTE_SUCCESS;
  } else if (msg->nof_bits == n1) {
    // format 1 (36.212 5.3.3.1.2): [RA header if N_RB > 10], type 0 / type 1 field, MCS, HARQ, NDI, RV, TPC
    const uint32_t P = mi::rbg_size(N), nrbg = (N + P - 1) / P;
    const bool type1 = N > 10 && take_bits(msg->data, &pos, 1);
    dci->dci_format = SRSLTE_DCI_FORMAT1;
    if (!type1) {
      dci->alloc_type = SRSLTE_RA_ALLOC_TYPE0;
      for (uint32_t g = 0; g < nrbg; g++) {
        const uint32_t bit = take_bits(msg->data, &pos, 1);
        dci->type0_alloc = (dci->type0_alloc << 1) | bit;
        for (uint32_t p = g * P; bit && p < (g + 1) * P && p < N; p++) grant->prb_idx[0][p] = grant->prb_idx[1][p] = true;
      }
    } else {
      // type 1 (36.213 7.1.6.2): subset p, shift, bitmap over N_RB^TYPE1 VRBs of the subset
      dci->alloc_type = SRSLTE_RA_ALLOC_TYPE1;
      const uint32_t pb = mi::ceil_log2(P), nt1 = nrbg - pb - 1;
      dci->type1_subset = take_bits(msg->data, &pos, pb);
      dci->type1_shift = take_bits(msg->data, &pos, 1);
      dci->type1_bitmap = take_bits(msg->data, &pos, nt1);
      const uint32_t sp = dci->type1_subset;
      if (sp >= P) return SRSLTE_ERROR;
      // VRBs in subset p: full RBG rows below the last RBG's subset, the partial last one, none above
      const uint32_t last = (N - 1) / P % P, rows = (N - 1) / (P * P);
      const uint32_t n_sub = sp < last ? rows * P + P : sp == last ? rows * P + (N - 1) % P + 1 : rows * P;
      const uint32_t delta = dci->type1_shift ? (n_sub > nt1 ? n_sub - nt1 : 0) : 0;
      for (uint32_t i = 0; i < nt1; i++) {
        if (!((dci->type1_bitmap >> (nt1 - 1 - i)) & 1u)) continue;
        const uint32_t j = i + delta, p = (j / P) * P * P + sp * P + j % P;
        if (j >= n_sub || p >= N) return SRSLTE_ERROR;
        grant->prb_idx[0][p] = grant->prb_idx[1][p] = true;
      }
    }
    for (uint32_t p = 0; p < N; p++) grant->nof_prb += grant->prb_idx[0][p] ? 1 : 0;
    if (!grant->nof_prb) return SRSLTE_ERROR;
    nprb_tbs = grant->nof_prb;
  } else {
    return SRSLTE_ERROR;
  }
  if (dci->dci_format == SRSLTE_DCI_FORMAT1) {
    dci->mcs_idx = take_bits(msg->data, &pos, 5);
    dci->harq_process = take_bits(msg->data, &pos, 3);
    dci->ndi = take_bits(msg->data, &pos, 1) != 0;
    dci->rv_idx = take_bits(msg->data, &pos, 2);
    dci->tpc_pucch = take_bits(msg->data, &pos, 2);
  }
  uint32_t qm = 2;
  const int itbs = itbs_1a_common ? (dci->mcs_idx <= 26 ? (int)dci->mcs_idx : -1) : mi::mcs_to_itbs(dci->mcs_idx, &qm);
  const int tbs = itbs < 0 ? -1 : mi::tbs_from_idx((uint32_t)itbs, nprb_tbs);
  if (tbs <= 0) return SRSLTE_ERROR;
  grant->Qm = qm;
  grant->mcs.idx = dci->mcs_idx;
  grant->mcs.tbs = tbs;
  grant->mcs.mod = qm == 2 ? SRSLTE_MOD_QPSK : qm == 4 ? SRSLTE_MOD_16QAM : SRSLTE_MOD_64QAM;
  return SRSLTE_SUCCESS;
}

char* srslte_ra_dl_dci_string(srslte_ra_dl_dci_t* dci) {
  static thread_local char buf[96];
  if (!dci) return buf;
  const char* fmt = dci->dci_format == SRSLTE_DCI_FORMAT1 ? "1" : dci->dci_format == SRSLTE_DCI_FORMAT1C ? "1C" : "1A";
  snprintf(buf, sizeof(buf), "format=%s, mcs=%u, harq=%u, ndi=%d, rv=%u", fmt, dci->mcs_idx, dci->harq_process,
           (int)dci->ndi, dci->rv_idx);
  return buf;
}

/* ---- chest metrics ------------------------------------------------------------------------- */
float srslte_chest_dl_get_snr(srslte_chest_dl_t* q) { return q ? q->snr : 0.f; }
float srslte_chest_dl_get_rssi(srslte_chest_dl_t* q) { return q ? q->rssi : 0.f; }
float srslte_chest_dl_get_rsrp(srslte_chest_dl_t* q) { return q ? q->rsrp : 0.f; }
float srslte_chest_dl_get_rsrq(srslte_chest_dl_t* q) { return q ? q->rsrq : 0.f; }
float srslte_chest_dl_get_noise_estimate(srslte_chest_dl_t* q) { return q ? q->noise_estimate : 0.f; }

}  // extern "C"
