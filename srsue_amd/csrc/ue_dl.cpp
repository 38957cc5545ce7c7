// ue_dl.cpp -- the srsLTE-1.0 DL entry points srsUE's phch_worker calls, backed by the MI355X
// engine (include/srslte/srslte.h documents each call site in /root/reference).
//
// Per srslte_ue_dl_t instance (one per phch_worker thread, phch_worker.h:111): one HIP stream,
// one Engine (HBM workspace for one subframe), host mirrors of the grid and channel estimates
// (srsUE reads them on the host for PDCCH, phch_worker.cc:260).  Re-entrant per instance, no
// global mutable state besides the cached read-only spec tables inside each Engine.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/srslte/srslte.h"
#include "engine.h"

struct mi_ue_dl_ctx {
  mi::Engine eng;
  hipStream_t st = nullptr;
  mi::DevBuf d_iq;
  mi_dl_sf_cfg_t cfg{};    // current subframe configuration
  uint32_t cfi = 1, sf_idx = 0;
  bool fft_done = false;
  cf_t* host_grid = nullptr;
  cf_t* host_ce[SRSLTE_MAX_PORTS] = {};
};

namespace {

void pcfich_host(const srslte_cell_t& cell, uint32_t sf, const cf_t* grid, cf_t* const* ce, uint32_t* cfi_out) {
  uint32_t kk[16];
  mi::pcfich_k(cell.id, cell.nof_prb, kk);
  const float* g = reinterpret_cast<const float*>(grid);
  const float* h0 = reinterpret_cast<const float*>(ce[0]);
  const float* h1 = cell.nof_ports == 2 ? reinterpret_cast<const float*>(ce[1]) : nullptr;
  float xr[16], xi[16];
  for (int i = 0; i < 16; i += (h1 ? 2 : 1)) {
    if (!h1) {
      const float yr = g[2 * kk[i]], yi = g[2 * kk[i] + 1], hr = h0[2 * kk[i]], hi = h0[2 * kk[i] + 1];
      const float den = hr * hr + hi * hi + 1e-9f;
      xr[i] = (yr * hr + yi * hi) / den;
      xi[i] = (yi * hr - yr * hi) / den;
    } else {
      const uint32_t a = kk[i], b = kk[i + 1];
      const float r0r = g[2 * a], r0i = g[2 * a + 1], r1r = g[2 * b], r1i = g[2 * b + 1];
      const float h00r = h0[2 * a], h00i = h0[2 * a + 1], h01r = h0[2 * b], h01i = h0[2 * b + 1];
      const float h10r = h1[2 * a], h10i = h1[2 * a + 1], h11r = h1[2 * b], h11i = h1[2 * b + 1];
      float hh = h00r * h00r + h00i * h00i + h11r * h11r + h11i * h11i;
      if (hh <= 0) hh = 1e-9f;
      const float s = 1.41421356f / hh;
      xr[i] = s * ((h00r * r0r + h00i * r0i) + (h11r * r1r + h11i * r1i));
      xi[i] = s * ((h00r * r0i - h00i * r0r) + (h11i * r1r - h11r * r1i));
      xr[i + 1] = s * (-(h10r * r0r + h10i * r0i) + (h01r * r1r + h01i * r1i));
      xi[i + 1] = s * (-(h10i * r0r - h10r * r0i) + (h01r * r1i - h01i * r1r));
    }
  }
  uint8_t sc[32];
  mi::gold_bits(mi::pcfich_cinit(cell.id, sf), 32, sc);
  float llr[32];
  for (int i = 0; i < 16; i++) {   // QPSK max-log LLR (> 0 => bit 1), descrambled
    llr[2 * i] = -xr[i] * (sc[2 * i] ? -1.f : 1.f);
    llr[2 * i + 1] = -xi[i] * (sc[2 * i + 1] ? -1.f : 1.f);
  }
  float best = -1e30f;
  uint32_t bc = 0;
  for (uint32_t c = 1; c <= 3; c++) {
    uint8_t cw[32];
    mi::cfi_codeword(c, cw);
    float s = 0;
    for (int i = 0; i < 32; i++) s += cw[i] ? llr[i] : -llr[i];
    if (s > best) { best = s; bc = c; }
  }
  *cfi_out = bc;
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
  q->dev_bytes = (uint64_t)2 * mi::NCB_MAX * mi::LANES * sizeof(float);
  if (hipMalloc(&q->dev, q->dev_bytes) != hipSuccess) { q->dev = nullptr; return SRSLTE_ERROR; }
  srslte_softbuffer_rx_reset(q);
  return SRSLTE_SUCCESS;
}
void srslte_softbuffer_rx_free(srslte_softbuffer_rx_t* q) {
  if (q && q->dev) (void)hipFree(q->dev);
  if (q) memset(q, 0, sizeof(*q));
}
void srslte_softbuffer_rx_reset(srslte_softbuffer_rx_t* q) {
  if (q && q->dev) (void)hipMemset(q->dev, 0, q->dev_bytes);   // == RX_NULL everywhere
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
  q->sf_symbols = (cf_t*)srslte_vec_malloc((uint32_t)(n * sizeof(cf_t)));
  for (uint32_t p = 0; p < cell.nof_ports; p++) q->ce[p] = (cf_t*)srslte_vec_malloc((uint32_t)(n * sizeof(cf_t)));
  if (!ctx->d_iq.ensure((size_t)mi::sf_len(mi::symbol_sz(cell.nof_prb)) * 8)) { delete ctx; return SRSLTE_ERROR; }
  ctx->cfg.cell_id = cell.id;
  ctx->cfg.nof_prb = cell.nof_prb;
  ctx->cfg.nof_ports = cell.nof_ports;
  ctx->cfg.tm = cell.nof_ports == 2 ? 2 : 1;
  ctx->cfg.nl_td = 2;
  ctx->host_grid = q->sf_symbols;
  for (int p = 0; p < SRSLTE_MAX_PORTS; p++) ctx->host_ce[p] = q->ce[p];
  q->ctx = ctx;
  q->pdsch.ctx = ctx;
  return SRSLTE_SUCCESS;
}

void srslte_ue_dl_free(srslte_ue_dl_t* q) {
  if (!q) return;
  if (q->ctx) {
    if (q->ctx->st) (void)hipStreamDestroy(q->ctx->st);
    delete q->ctx;
  }
  free(q->sf_symbols);
  for (int p = 0; p < SRSLTE_MAX_PORTS; p++) free(q->ce[p]);
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
  if (!mi::hip_ok(hipMemcpyAsync(c->d_iq.p, input, sfl * 8, hipMemcpyHostToDevice, c->st), "H2D iq"))
    return SRSLTE_ERROR;
  if (c->eng.plan.build(&c->cfg, 1, false) || c->eng.upload(c->st, false)) return SRSLTE_ERROR;
  if (c->eng.run(c->d_iq.p, c->st, (1u << MI_DL_STAGE_OFDM) | (1u << MI_DL_STAGE_CHEST), nullptr)) return SRSLTE_ERROR;
  float met[5];
  bool ok = mi::hip_ok(hipMemcpyAsync(q->sf_symbols, c->eng.d_grid.p, n * 8, hipMemcpyDeviceToHost, c->st), "D2H");
  for (uint32_t p = 0; p < q->cell.nof_ports && ok; p++)
    ok = mi::hip_ok(hipMemcpyAsync(q->ce[p], c->eng.d_ce.as<float2>() + p * n, n * 8, hipMemcpyDeviceToHost, c->st), "D2H");
  ok = ok && mi::hip_ok(hipMemcpyAsync(met, c->eng.d_metrics.p, sizeof(met), hipMemcpyDeviceToHost, c->st), "D2H") &&
       mi::hip_ok(hipStreamSynchronize(c->st), "sync");
  if (!ok) return SRSLTE_ERROR;
  q->chest.rsrp = met[0]; q->chest.rssi = met[1]; q->chest.rsrq = met[2];
  q->chest.noise_estimate = met[3]; q->chest.snr = met[4];
  uint32_t cf = 0;
  pcfich_host(q->cell, sf_idx, q->sf_symbols, q->ce, &cf);
  if (cf < 1 || cf > 3) return SRSLTE_ERROR;
  q->cfi = cf;
  c->cfi = cf;
  c->fft_done = true;
  if (cfi) *cfi = cf;
  return SRSLTE_SUCCESS;
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
  for (int p = 0; p < SRSLTE_MAX_PRB; p++) mask[p] = grant->prb_idx[0][p] ? 1 : 0;
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
  for (int p = 0; p < SRSLTE_MAX_PRB; p++) s.prb_mask[p] = cfg->grant.prb_idx[0][p] ? 1 : 0;
  c->eng.noise = noise_estimate;
  c->eng.max_its = q->dl_sch.max_iterations ? q->dl_sch.max_iterations : SRSLTE_PDSCH_MAX_TDEC_ITERS;
  if (c->eng.plan.build(&s, 1, true) || c->eng.upload(c->st, false)) return SRSLTE_ERROR;
  if (c->eng.plan.sb_floats * sizeof(float) > softbuffer->dev_bytes) return SRSLTE_ERROR;
  // grid / ce: the device copies left by decode_fft_estimate are reused when the caller passes this
  // instance's own host mirrors (srsUE passes ue_dl.sf_symbols / ue_dl.ce, phch_worker.cc:347-348);
  // any other buffers are uploaded.
  const size_t W = 12 * cell.nof_prb, n = (size_t)mi::NSYMB * W;
  bool own = c->fft_done && sf_symbols == c->host_grid;
  for (uint32_t p = 0; p < cell.nof_ports; p++) own = own && ce[p] == c->host_ce[p];
  bool ok = true;
  if (!own) {
    ok = mi::hip_ok(hipMemcpyAsync(c->eng.d_grid.p, sf_symbols, n * 8, hipMemcpyHostToDevice, c->st), "H2D grid");
    for (uint32_t p = 0; p < cell.nof_ports && ok; p++)
      ok = mi::hip_ok(hipMemcpyAsync(c->eng.d_ce.as<float2>() + p * n, ce[p], n * 8, hipMemcpyHostToDevice, c->st),
                      "H2D ce");
  }
  if (!ok) return SRSLTE_ERROR;
  const uint32_t stages = (1u << MI_DL_STAGE_DEMAP) | (1u << MI_DL_STAGE_RM) | (1u << MI_DL_STAGE_TDEC) |
                          (1u << MI_DL_STAGE_TB);
  if (c->eng.run(nullptr, c->st, stages, reinterpret_cast<float*>(softbuffer->dev))) return SRSLTE_ERROR;
  uint32_t tb_ok = 0, its = 0;
  ok = mi::hip_ok(hipMemcpyAsync(data, c->eng.d_payload.p, s.tbs / 8, hipMemcpyDeviceToHost, c->st), "D2H") &&
       mi::hip_ok(hipMemcpyAsync(&tb_ok, c->eng.d_tbok.p, 4, hipMemcpyDeviceToHost, c->st), "D2H") &&
       mi::hip_ok(hipMemcpyAsync(&its, c->eng.d_tbits.p, 4, hipMemcpyDeviceToHost, c->st), "D2H") &&
       mi::hip_ok(hipStreamSynchronize(c->st), "sync");
  if (!ok) return SRSLTE_ERROR;
  q->dl_sch.nof_iterations = its;
  q->dl_sch.average_nof_iterations = 0.8f * q->dl_sch.average_nof_iterations + 0.2f * (float)its;
  return tb_ok ? SRSLTE_SUCCESS : SRSLTE_ERROR;
}

uint32_t srslte_pdsch_last_noi(srslte_pdsch_t* q) { return q ? q->dl_sch.nof_iterations : 0; }
void srslte_sch_set_max_noi(srslte_sch_t* q, uint32_t max_iterations) {
  if (q && max_iterations > 0) q->max_iterations = max_iterations;
}

/* ---- chest metrics ------------------------------------------------------------------------- */
float srslte_chest_dl_get_snr(srslte_chest_dl_t* q) { return q ? q->snr : 0.f; }
float srslte_chest_dl_get_rssi(srslte_chest_dl_t* q) { return q ? q->rssi : 0.f; }
float srslte_chest_dl_get_rsrp(srslte_chest_dl_t* q) { return q ? q->rsrp : 0.f; }
float srslte_chest_dl_get_rsrq(srslte_chest_dl_t* q) { return q ? q->rsrq : 0.f; }
float srslte_chest_dl_get_noise_estimate(srslte_chest_dl_t* q) { return q ? q->noise_estimate : 0.f; }

}  // extern "C"
