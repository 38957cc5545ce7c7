// ue_sync.cpp -- the srslte_ue_sync tracking subset srsUE's sync thread calls (include/srslte/srslte.h;
// /root/reference/ue/src/phy/phch_recv.cc:108-120 init, :236 get_buffer, :321 zerocopy, :326-327
// get_sfo / get_cfo, :330 get_last_timestamp) on the GPU sync front end (sync.h / sync.hip).
//
// Host state machine over the receive callback's sample stream:
//   FIND  : read one half frame + one symbol, search every lag for the cell's PSS (N_ID_2 = id % 3) in
//           parallel chunks, check the SSS (N_ID_1, subframe 0 / 5) at the found boundary, initialise
//           the CFO from the PSS, align to that subframe (returns 0);
//   TRACK : per call one subframe (H2D); on subframes 0 / 5 the PSS is searched +-31 samples around
//           its expected position: the timing error re-times the NEXT subframe boundary and the CFO
//           estimate enters an exponential average (em_alpha); the CFO is removed on the GPU into the
//           caller's buffer (D2H), the subframe index advances (returns 1).
#include <math.h>
#include <string.h>

#include <vector>

#include "srslte/srslte.h"
#include "sync.h"

struct mi_ue_sync_ctx {
  mi::SyncEngine eng;
  hipStream_t st = nullptr;
  int (*recv)(void*, void*, uint32_t, srslte_timestamp_t*) = nullptr;
  void* handler = nullptr;
  uint32_t N = 0, sf_len = 0, sym6 = 0;    // sym6: PSS useful part within a subframe
  double srate = 0;
  std::vector<float2> ring;                // received samples [base, base + ring.size())
  uint64_t base = 0, pos = 0;              // pos: stream index of the next subframe boundary
  srslte_timestamp_t ring_ts{};            // timestamp of sample `base`
  bool tracking = false, sss_on_track = false, cfo_set = false, have_sf = false;
  uint32_t sf_idx = 0;
  float cfo = 0.f;                         // subcarrier spacings
  double sfo = 0.0;                        // samples / s
  srslte_timestamp_t last_ts{};
  mi::DevBuf d_win, d_out;
};

namespace {

constexpr uint32_t TRACK_M = 31;           // tracking window: +-31 samples around the expected PSS (63 lags)
constexpr float FIND_MIN_RHO = 0.01f;

void ts_add(srslte_timestamp_t* t, double secs) {
  double f = t->frac_secs + secs;
  const double w = floor(f);
  t->full_secs += (time_t)w;
  t->frac_secs = f - w;
}

// make the ring hold the stream up to (excluding) index `upto`
bool fill(mi_ue_sync_ctx* c, uint64_t upto) {
  const uint64_t have = c->base + c->ring.size();
  if (upto <= have) return true;
  const uint32_t n = (uint32_t)(upto - have);
  std::vector<float2> tmp(n);
  srslte_timestamp_t ts{};
  const int r = c->recv(c->handler, tmp.data(), n, &ts);
  if (r < (int)n) { mi::set_error("ue_sync: receive callback"); return false; }
  if (c->ring.empty()) {
    c->ring_ts = ts;
    c->base = have;
  }
  c->ring.insert(c->ring.end(), tmp.begin(), tmp.end());
  return true;
}

void drop(mi_ue_sync_ctx* c, uint64_t before) {
  if (before <= c->base) return;
  const uint64_t k = std::min<uint64_t>(before - c->base, c->ring.size());
  c->ring.erase(c->ring.begin(), c->ring.begin() + (ptrdiff_t)k);
  ts_add(&c->ring_ts, (double)k / c->srate);
  c->base += k;
}

bool upload(mi_ue_sync_ctx* c, uint64_t from, uint32_t n) {
  return c->d_win.ensure((size_t)n * sizeof(float2)) &&
         mi::hip_ok(hipMemcpyAsync(c->d_win.p, c->ring.data() + (from - c->base), (size_t)n * sizeof(float2),
                                   hipMemcpyHostToDevice, c->st),
                    "H2D");
}

int find(srslte_ue_sync_t* q) {
  mi_ue_sync_ctx* c = q->ctx;
  const uint32_t half = 5 * c->sf_len, nid2 = q->cell.id % 3;
  if (!fill(c, c->pos + half + c->N) || !upload(c, c->pos, half + c->N)) return -1;
  std::vector<mi::MiPssJob> jobs;
  constexpr uint32_t CH = 2048;
  for (uint32_t o = 0; o < half; o += CH) jobs.push_back(mi::MiPssJob{o, std::min(CH, half - o), 1u << nid2});
  if (c->eng.pss(c->d_win.as<float2>(), jobs, c->st)) return -1;
  uint32_t bi = 0;
  for (uint32_t i = 1; i < jobs.size(); i++)
    if (c->eng.pres[i].rho > c->eng.pres[bi].rho) bi = i;
  const mi::MiPssRes r = c->eng.pres[bi];
  if (!(r.rho > std::max(q->strack.threshold, FIND_MIN_RHO))) {   // nothing convincing: next half frame
    drop(c, c->pos + half);
    c->pos += half;
    return 0;
  }
  uint64_t s = c->pos + jobs[bi].off + r.lag;   // stream index of the PSS useful part
  s = s >= c->sym6 + c->pos ? s - c->sym6 : s - c->sym6 + half;   // boundary of the PSS's subframe
  if (!fill(c, s + c->sf_len) || !upload(c, s, c->sf_len)) return -1;
  const float cfo = c->cfo_set ? c->cfo : r.cfo;
  if (c->eng.sss(c->d_win.as<float2>(), {mi::MiSssJob{0, nid2, r.cfo}}, c->st)) return -1;
  if (c->eng.sres[0].nid1 != q->cell.id / 3) {   // another cell's PSS: keep searching
    drop(c, c->pos + half);
    c->pos += half;
    return 0;
  }
  c->cfo = c->cfo_set ? cfo : r.cfo;
  c->cfo_set = true;
  c->sf_idx = c->eng.sres[0].sf5 ? 5 : 0;
  drop(c, s);
  c->pos = s;
  c->tracking = true;
  return 0;
}

int track(srslte_ue_sync_t* q, cf_t* out) {
  mi_ue_sync_ctx* c = q->ctx;
  if (!fill(c, c->pos + c->sf_len) || !upload(c, c->pos, c->sf_len)) return -1;
  int32_t delta = 0;
  if (c->sf_idx == 0 || c->sf_idx == 5) {
    const uint32_t nid2 = q->cell.id % 3;
    if (c->eng.pss(c->d_win.as<float2>(), {mi::MiPssJob{c->sym6 - TRACK_M, 2 * TRACK_M + 1, 1u << nid2}}, c->st))
      return -1;
    const mi::MiPssRes r = c->eng.pres[0];
    delta = (int32_t)r.lag - (int32_t)TRACK_M;
    const float a = q->strack.em_alpha > 0.f ? q->strack.em_alpha : 0.1f;
    c->cfo = (1.f - a) * c->cfo + a * r.cfo;
    c->sfo = 0.9 * c->sfo + 0.1 * (double)delta / 5e-3;
    if (c->sss_on_track) {
      if (c->eng.sss(c->d_win.as<float2>(), {mi::MiSssJob{0, nid2, c->cfo}}, c->st)) return -1;
      c->sf_idx = c->eng.sres[0].sf5 ? 5 : 0;
    }
  }
  if (!c->d_out.ensure((size_t)c->sf_len * sizeof(float2)) ||
      c->eng.correct(c->d_win.as<float2>(), c->d_out.as<float2>(), {mi::MiCfoJob{0, 0, c->cfo, 0}}, c->sf_len, c->st) ||
      !mi::hip_ok(hipMemcpyAsync(out, c->d_out.p, (size_t)c->sf_len * sizeof(float2), hipMemcpyDeviceToHost, c->st),
                  "D2H") ||
      !mi::hip_ok(hipStreamSynchronize(c->st), "sync"))
    return -1;
  c->last_ts = c->ring_ts;
  ts_add(&c->last_ts, (double)(c->pos - c->base) / c->srate);
  c->pos += (uint64_t)((int64_t)c->sf_len + delta);   // the timing error re-times the next boundary
  drop(c, std::min<uint64_t>(c->pos, c->base + c->ring.size()));
  q->input_buffer = out;
  c->have_sf = true;
  c->sf_idx = (c->sf_idx + 1) % 10;
  return 1;
}

}  // namespace

extern "C" {

int srslte_ue_sync_init(srslte_ue_sync_t* q, srslte_cell_t cell,
                        int(recv_callback)(void*, void*, uint32_t, srslte_timestamp_t*), void* stream_handler) {
  if (!q || !recv_callback || mi::symbol_sz(cell.nof_prb) < 0 || cell.id > 503 || cell.cp != SRSLTE_CP_NORM)
    return SRSLTE_ERROR_INVALID_INPUTS;
  memset(q, 0, sizeof(*q));
  auto* c = new mi_ue_sync_ctx();
  if (c->eng.init(cell.nof_prb) || !mi::hip_ok(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking), "stream")) {
    delete c;
    return SRSLTE_ERROR;
  }
  c->recv = recv_callback;
  c->handler = stream_handler;
  c->N = c->eng.N;
  c->sf_len = 15 * c->N;
  c->sym6 = (uint32_t)mi::symbol_offset((int)c->N, 6);
  c->srate = 15000.0 * c->N;
  q->cell = cell;
  q->strack.em_alpha = 0.1f;
  q->ctx = c;
  return SRSLTE_SUCCESS;
}

void srslte_ue_sync_free(srslte_ue_sync_t* q) {
  if (!q) return;
  if (q->ctx) {
    if (q->ctx->st) (void)hipStreamDestroy(q->ctx->st);
    delete q->ctx;
  }
  memset(q, 0, sizeof(*q));
}

int srslte_ue_sync_zerocopy(srslte_ue_sync_t* q, cf_t* input_buffer) {
  if (!q || !q->ctx || !input_buffer) return SRSLTE_ERROR_INVALID_INPUTS;
  const int r = q->ctx->tracking ? track(q, input_buffer) : find(q);
  return r < 0 ? SRSLTE_ERROR : r;
}

int srslte_ue_sync_get_buffer(srslte_ue_sync_t* q, cf_t** sf_symbols) {
  if (!q || !q->ctx || !sf_symbols) return SRSLTE_ERROR_INVALID_INPUTS;
  static thread_local std::vector<cf_t> buf;   // srsLTE returns its internal buffer
  buf.resize(q->ctx->sf_len);
  const int r = srslte_ue_sync_zerocopy(q, buf.data());
  *sf_symbols = buf.data();
  return r;
}

uint32_t srslte_ue_sync_get_sfidx(srslte_ue_sync_t* q) {
  // the index of the subframe the last zerocopy() delivered
  return (q && q->ctx) ? (q->ctx->sf_idx + 9) % 10 : 0;
}
float srslte_ue_sync_get_cfo(srslte_ue_sync_t* q) { return (q && q->ctx) ? 15000.f * q->ctx->cfo : 0.f; }
float srslte_ue_sync_get_sfo(srslte_ue_sync_t* q) { return (q && q->ctx) ? (float)q->ctx->sfo : 0.f; }
void srslte_ue_sync_set_cfo(srslte_ue_sync_t* q, float cfo) {
  if (!q || !q->ctx) return;
  q->ctx->cfo = cfo / 15000.f;
  q->ctx->cfo_set = true;
}
void srslte_ue_sync_decode_sss_on_track(srslte_ue_sync_t* q, bool enabled) {
  if (q && q->ctx) q->ctx->sss_on_track = enabled;
}
void srslte_ue_sync_get_last_timestamp(srslte_ue_sync_t* q, srslte_timestamp_t* t) {
  if (q && q->ctx && t) *t = q->ctx->last_ts;
}
void srslte_ue_sync_set_agc_period(srslte_ue_sync_t*, uint32_t) {}
int srslte_ue_sync_start_agc(srslte_ue_sync_t*, double(set_gain_callback)(void*, double), float) {
  (void)set_gain_callback;
  mi::set_error("AGC is not implemented (the gain stays as configured)");
  return SRSLTE_ERROR;
}
void srslte_sync_set_threshold(srslte_sync_t* q, float threshold) {
  if (q) q->threshold = threshold;
}
void srslte_sync_set_em_alpha(srslte_sync_t* q, float alpha) {
  if (q) q->em_alpha = alpha;
}
int srslte_sampling_freq_hz(uint32_t nof_prb) {
  const int n = mi::symbol_sz(nof_prb);
  return n < 0 ? -1 : 15000 * n;
}
void srslte_timestamp_copy(srslte_timestamp_t* dest, srslte_timestamp_t* src) {
  if (dest && src) *dest = *src;
}
int srslte_timestamp_add(srslte_timestamp_t* t, time_t full_secs, double frac_secs) {
  if (!t) return SRSLTE_ERROR_INVALID_INPUTS;
  t->full_secs += full_secs;
  ts_add(t, frac_secs);
  return SRSLTE_SUCCESS;
}

}  // extern "C"
