// ue_ul.cpp -- the srsLTE-1.0 UL PUSCH entry points srsUE's phch_worker calls (include/srslte/srslte.h
// documents each call site in /root/reference), backed by the GPU transmitter of ul.hip.
//
// Per srslte_ue_ul_t instance (one per phch_worker thread, phch_worker.h:116): one HIP stream, one
// UlEngine planned for the current grant (cfg_grant), a device payload buffer and a device subframe.
// A retransmission (rv > 0) re-encodes the TB kept in the HARQ softbuffer: the circular buffer is a
// deterministic function of the TB, so this equals srsLTE's reuse of its stored coded bits.
#include <time.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/srslte/srslte.h"
#include "tables.h"
#include "ul_engine.h"
#include "../../include/mi_ul.h"

struct mi_ue_ul_ctx {
  mi::UlEngine eng;
  hipStream_t st = nullptr;
  mi::DevBuf d_pay, d_iq;
  // page-locked staging of the TB (H2D) and of the subframe's IQ (D2H): srsUE's buffers are pageable
  uint8_t* h_pay = nullptr;
  cf_t* h_iq = nullptr;
  mi_ul_cfg_t cfg{};
  bool planned = false;
  // per-phase host-clock breakdown of pusch_encode (MI_UE_UL_PROF=1: the stream is synchronised at every
  // mark so GPU work is attributed to its phase; printed to stderr when the instance is freed):
  // 0 payload H2D, 1 plan, 2 table upload, 3 kernels, 4 IQ D2H + copy out
  struct Prof {
    bool on = getenv("MI_UE_UL_PROF") != nullptr;
    double acc[5] = {}, last = 0;
    uint64_t n[5] = {};
    static double now() {
      timespec t;
      clock_gettime(CLOCK_MONOTONIC, &t);
      return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
    }
    void start() { if (on) last = now(); }
    void mark(int i, hipStream_t s) {
      if (!on) return;
      (void)hipStreamSynchronize(s);
      const double t = now();
      acc[i] += t - last; n[i]++; last = t;
    }
  } prof;
  ~mi_ue_ul_ctx() {
    if (prof.on) {
      static const char* name[5] = {"payload_h2d", "plan", "upload", "kernels", "iq_d2h"};
      fprintf(stderr, "{\"ue_ul_prof_us\": {");
      for (int i = 0; i < 5; i++)
        fprintf(stderr, "%s\"%s\": %.1f", i ? ", " : "", name[i], prof.n[i] ? prof.acc[i] / prof.n[i] : 0.0);
      fprintf(stderr, "}}\n");
    }
    // the stream is owned here (as in ue_dl.cpp): synchronised, the staging freed, then destroyed
    if (st) (void)hipStreamSynchronize(st);
    if (h_pay) (void)hipHostFree(h_pay);
    if (h_iq) (void)hipHostFree(h_iq);
    if (st) (void)hipStreamDestroy(st);
  }
};

namespace {
constexpr uint32_t TX_MAX_BYTES = 12 * 1024;   // > the largest Rel-8 UL TB (75,376 bits)

uint32_t take_bits(const uint8_t* b, uint32_t* pos, uint32_t n) {
  uint32_t v = 0;
  for (uint32_t i = 0; i < n; i++) v = (v << 1) | b[(*pos)++];
  return v;
}

// 36.213 Table 8.6.1-1: I_MCS -> (Q_m, I_TBS); 29-31 are retransmissions (rv 1-3)
int ul_mcs(uint32_t mcs, uint32_t* qm, uint32_t* itbs) {
  if (mcs <= 10) { *qm = 2; *itbs = mcs; return 0; }
  if (mcs <= 20) { *qm = 4; *itbs = mcs - 1; return 0; }
  if (mcs <= 28) { *qm = 6; *itbs = mcs - 2; return 0; }
  return -1;
}

// 36.213 8.4: N~_HO = N_HO rounded up to even (pusch-HoppingOffset)
uint32_t ul_nho_tilde(uint32_t n_rb_ho) { return n_rb_ho + (n_rb_ho & 1u); }

// fill the grant of a contiguous allocation (type 2 RIV, 36.213 8.1.1 / 36.212 5.3.3.1.1)
int grant_from_riv(uint32_t riv, uint32_t nof_prb, uint32_t mcs, uint32_t n_dmrs, srslte_ra_ul_dci_t* dci,
                   srslte_ra_ul_grant_t* g) {
  const uint32_t a = riv / nof_prb, b = riv % nof_prb;
  uint32_t L, start;
  if (a + b < nof_prb) { L = a + 1; start = b; }
  else { L = nof_prb - a + 1; start = nof_prb - 1 - b; }
  if (start + L > nof_prb) return SRSLTE_ERROR;
  // the DFT-spread size M = 12 L must factor as 2^a 3^b 5^c (36.211 5.3.3)
  uint32_t r = L;
  for (uint32_t f : {2u, 3u, 5u}) while (r % f == 0) r /= f;
  if (r != 1) { mi::set_error("L_prb must be 2^a 3^b 5^c (36.211 5.3.3)"); return SRSLTE_ERROR; }
  uint32_t qm = 0, itbs = 0;
  if (ul_mcs(mcs, &qm, &itbs)) return SRSLTE_ERROR;
  const int tbs = mi::tbs_from_idx(itbs, L);
  if (tbs <= 0) return SRSLTE_ERROR;
  dci->alloc_type = SRSLTE_RA_ALLOC_TYPE2;
  dci->type2_start = start;
  dci->type2_len = L;
  dci->mcs_idx = mcs;
  dci->n_dmrs = n_dmrs;
  memset(g, 0, sizeof(*g));
  g->n_prb[0] = g->n_prb[1] = start;
  g->n_prb_tilde[0] = g->n_prb_tilde[1] = start;
  g->L_prb = L;
  g->nof_symb = 12;
  g->nof_re = 12 * 12 * L;
  g->Qm = qm;
  g->mcs.idx = mcs;
  g->mcs.tbs = tbs;
  g->mcs.mod = qm == 2 ? SRSLTE_MOD_QPSK : qm == 4 ? SRSLTE_MOD_16QAM : SRSLTE_MOD_64QAM;
  g->ncs_dmrs = n_dmrs;
  return SRSLTE_SUCCESS;
}

// hopping bits of a format-0 / RAR grant (36.213 8.4, Tables 8.4-1 / 8.4-2): type 1 offsets the slot-1 (or
// odd-transmission) allocation in the PUSCH hopping band of N_RB^PUSCH PRBs; the all-ones pattern ('1' for
// N_UL_hop = 1, '11' for 2) selects type 2 (subband hopping, resolved per slot by srslte_ue_ul_cfg_grant)
int apply_hopping_bits(uint32_t nof_prb, uint32_t n_rb_ho, uint32_t nh, uint32_t hbits, srslte_ra_ul_grant_t* grant) {
  if (hbits == (nh == 1 ? 1u : 3u)) {
    grant->freq_hopping = 2;
    return SRSLTE_SUCCESS;
  }
  const uint32_t N = nof_prb - ul_nho_tilde(n_rb_ho) - (nof_prb & 1u), s1 = grant->n_prb_tilde[0];
  if (N == 0 || N > nof_prb || s1 + grant->L_prb > N) return SRSLTE_ERROR;
  const uint32_t d = nh == 1 ? N / 2 : hbits == 0 ? N / 4 : hbits == 1 ? N - N / 4 : N / 2;
  const uint32_t s2 = (s1 + d) % N;
  if (s2 + grant->L_prb > N) return SRSLTE_ERROR;
  grant->freq_hopping = 1;
  grant->n_prb_tilde[1] = s2;
  return SRSLTE_SUCCESS;
}

uint32_t rba_bits(uint32_t nof_prb) {
  uint32_t b = 0;
  while ((1u << b) < nof_prb * (nof_prb + 1) / 2) b++;
  return b;
}
}  // namespace

extern "C" {

int srslte_ue_ul_init(srslte_ue_ul_t* q, srslte_cell_t cell) {
  if (!q || mi::symbol_sz(cell.nof_prb) < 0) return SRSLTE_ERROR_INVALID_INPUTS;
  memset(q, 0, sizeof(*q));
  q->cell = cell;
  auto* c = new mi_ue_ul_ctx();
  c->eng.packed = true;
  const size_t iq_bytes = (size_t)15 * mi::symbol_sz(cell.nof_prb) * 8;
  if (!mi::hip_ok(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking), "stream") || !c->d_pay.ensure(TX_MAX_BYTES) ||
      !c->d_iq.ensure(iq_bytes) ||
      !mi::hip_ok(hipHostMalloc(reinterpret_cast<void**>(&c->h_pay), TX_MAX_BYTES, hipHostMallocDefault), "pinned") ||
      !mi::hip_ok(hipHostMalloc(reinterpret_cast<void**>(&c->h_iq), iq_bytes, hipHostMallocDefault), "pinned")) {
    delete c;   // the destructor destroys the stream
    return SRSLTE_ERROR;
  }
  q->ctx = c;
  return SRSLTE_SUCCESS;
}

void srslte_ue_ul_free(srslte_ue_ul_t* q) {
  if (!q || !q->ctx) return;
  delete q->ctx;   // synchronises and destroys the instance's stream
  q->ctx = nullptr;
}

void srslte_ue_ul_set_rnti(srslte_ue_ul_t* q, uint16_t rnti) {
  if (q) q->current_rnti = rnti;
}
void srslte_ue_ul_set_normalization(srslte_ue_ul_t* q, bool enabled) {
  if (q) q->normalize_en = enabled;
}
void srslte_ue_ul_set_cfo_enable(srslte_ue_ul_t* q, bool enabled) {
  if (q) q->cfo_en = enabled;
}
void srslte_ue_ul_set_cfo(srslte_ue_ul_t* q, float cur_cfo) {
  if (q) q->current_cfo = cur_cfo;
}

void srslte_ue_ul_set_cfg(srslte_ue_ul_t* q, srslte_refsignal_dmrs_pusch_cfg_t* dmrs_cfg, srslte_refsignal_srs_cfg_t*,
                          srslte_pucch_cfg_t*, srslte_pucch_sched_t*, srslte_uci_cfg_t* uci_cfg,
                          srslte_pusch_hopping_cfg_t* hopping_cfg, srslte_ue_ul_powerctrl_t*) {
  if (!q) return;
  if (dmrs_cfg) q->dmrs_cfg = *dmrs_cfg;
  if (hopping_cfg) q->hopping_cfg = *hopping_cfg;
  if (uci_cfg) q->uci_cfg = *uci_cfg;
}

int srslte_ue_ul_cfg_grant(srslte_ue_ul_t* q, srslte_ra_ul_grant_t* grant, uint32_t tti, uint32_t rvidx,
                           uint32_t current_tx_nb) {
  if (!q || !q->ctx || !grant) return SRSLTE_ERROR_INVALID_INPUTS;
  if (grant->freq_hopping > 2) return SRSLTE_ERROR_INVALID_INPUTS;
  mi::CbSegm sg;
  if (grant->mcs.tbs <= 0 || mi::cbsegm((uint32_t)grant->mcs.tbs, &sg)) return SRSLTE_ERROR;
  q->pusch_cfg.grant = *grant;
  q->pusch_cfg.rv = rvidx;
  q->pusch_cfg.tti = tti;
  q->pusch_cfg.sf_idx = tti % 10;
  q->pusch_cfg.current_tx_nb = current_tx_nb;
  q->pusch_cfg.cb_segm.tbs = (uint32_t)grant->mcs.tbs;
  q->pusch_cfg.cb_segm.C = sg.C;
  q->pusch_cfg.cb_segm.F = sg.F;
  q->pusch_cfg.cb_segm.K1 = sg.Kp;
  q->pusch_cfg.cb_segm.K2 = sg.Km;
  q->pusch_cfg.cb_segm.C1 = sg.Cp;
  q->pusch_cfg.cb_segm.C2 = sg.Cm;
  mi_ul_cfg_t& c = q->ctx->cfg;
  c.cell_id = q->cell.id;
  c.nof_prb = q->cell.nof_prb;
  c.sf_idx = tti % 10;
  c.n_prb = grant->n_prb[0];
  c.hop = 0;
  c.n_prb1 = 0;
  if (grant->freq_hopping == 1) {
    // 36.213 8.4.1, type 1: n_PRB = n~_PRB + N~_HO / 2; slot 1 hops (intra-subframe mode), or the whole
    // subframe takes the hopped position when CURRENT_TX_NB is odd (inter-subframe mode)
    const uint32_t ho = ul_nho_tilde(q->hopping_cfg.hopping_offset) / 2;
    const uint32_t a = grant->n_prb_tilde[0] + ho, b = grant->n_prb_tilde[1] + ho;
    const bool intra = q->hopping_cfg.hop_mode == srslte_pusch_hopping_cfg_t::SRSLTE_PUSCH_HOP_MODE_INTRA_SF;
    const uint32_t s0 = intra ? a : (current_tx_nb & 1u) ? b : a, s1 = intra ? b : s0;
    if (s0 + grant->L_prb > q->cell.nof_prb || s1 + grant->L_prb > q->cell.nof_prb) return SRSLTE_ERROR;
    c.n_prb = s0;
    c.hop = s1 != s0;
    c.n_prb1 = s1;
    q->pusch_cfg.grant.n_prb[0] = s0;
    q->pusch_cfg.grant.n_prb[1] = s1;
  } else if (grant->freq_hopping == 2) {
    // type 2 (subband hopping, 36.211 5.3.4): both slots of subframe tti % 10 through the cell's hopping
    // pattern from the grant's first VRB (mi_ul_hop_type2)
    const bool intra = q->hopping_cfg.hop_mode == srslte_pusch_hopping_cfg_t::SRSLTE_PUSCH_HOP_MODE_INTRA_SF;
    int p[2];
    for (uint32_t sl = 0; sl < 2; sl++) {
      p[sl] = mi_ul_hop_type2(q->cell.nof_prb, q->hopping_cfg.hopping_offset, q->hopping_cfg.n_sb ? q->hopping_cfg.n_sb : 1,
                              intra, q->cell.id, grant->n_prb_tilde[0], grant->L_prb, 2 * (tti % 10) + sl, current_tx_nb);
      if (p[sl] < 0) { mi::set_error("type-2 hopping maps the allocation outside the band"); return SRSLTE_ERROR; }
    }
    c.n_prb = (uint32_t)p[0];
    c.hop = p[1] != p[0];
    c.n_prb1 = (uint32_t)p[1];
    q->pusch_cfg.grant.n_prb[0] = (uint32_t)p[0];
    q->pusch_cfg.grant.n_prb[1] = (uint32_t)p[1];
  }
  c.L_prb = grant->L_prb;
  c.tbs = (uint32_t)grant->mcs.tbs;
  c.Qm = grant->Qm;
  c.rv = rvidx;
  c.group_hopping = q->dmrs_cfg.group_hopping_en;
  c.sequence_hopping = q->dmrs_cfg.sequence_hopping_en;
  c.delta_ss = q->dmrs_cfg.delta_ss;
  c.cyclic_shift = q->dmrs_cfg.cyclic_shift;
  c.n_dmrs2 = grant->ncs_dmrs;
  q->ctx->planned = false;   // the scrambling sequence needs the RNTI: planned at encode time
  return SRSLTE_SUCCESS;
}

int srslte_ue_ul_pusch_encode_rnti_softbuffer(srslte_ue_ul_t* q, uint8_t* data, srslte_uci_data_t uci,
                                              srslte_softbuffer_tx_t* sb, uint16_t rnti, cf_t* output_signal) {
  if (!q || !q->ctx || !output_signal) return SRSLTE_ERROR_INVALID_INPUTS;
  mi_ue_ul_ctx* c = q->ctx;
  if (uci.uci_cqi_len > SRSLTE_CQI_MAX_BITS || uci.uci_ri_len > 2 || uci.uci_ack_len > 2) {
    mi::set_error("UCI on PUSCH: up to 64 CQI bits, 2 RI bits, 2 HARQ-ACK bits");
    return SRSLTE_ERROR;
  }
  c->cfg.rnti = rnti;
  c->cfg.ack_len = uci.uci_ack_len;   // HARQ-ACK on PUSCH (srsUE: 1 bit, phch_worker.cc:486-487)
  c->cfg.ack = uci.uci_ack & 3u;
  c->cfg.I_offset_ack = q->uci_cfg.I_offset_ack;
  // periodic CQI (srsUE packs it at phch_worker.cc:507-523 before this call, :555) and RI, 36.212 5.2.2.6
  c->cfg.cqi_len = uci.uci_cqi_len;
  memcpy(c->cfg.cqi, uci.uci_cqi, uci.uci_cqi_len);
  c->cfg.I_offset_cqi = q->uci_cfg.I_offset_cqi;
  c->cfg.ri_len = uci.uci_ri_len;
  c->cfg.ri = uci.uci_ri & 3u;
  c->cfg.I_offset_ri = q->uci_cfg.I_offset_ri;
  const uint32_t nbytes = c->cfg.tbs / 8;
  if (nbytes > TX_MAX_BYTES) return SRSLTE_ERROR;
  // the TB: new data from `data`; a retransmission without data re-encodes the softbuffer's copy
  const void* src = nullptr;
  c->prof.start();
  if (data) {
    memcpy(c->h_pay, data, nbytes);   // the previous call's DMA out of h_pay ended with its stream sync
    if (!mi::hip_ok(hipMemcpyAsync(c->d_pay.p, c->h_pay, nbytes, hipMemcpyHostToDevice, c->st), "H2D payload"))
      return SRSLTE_ERROR;
    if (sb && sb->dev && c->cfg.rv == 0) {
      if (!mi::hip_ok(hipMemcpyAsync(sb->dev, c->d_pay.p, nbytes, hipMemcpyDeviceToDevice, c->st), "softbuffer"))
        return SRSLTE_ERROR;
      sb->tbs = c->cfg.tbs;
    }
    src = c->d_pay.p;
  } else if (sb && sb->dev && sb->tbs == c->cfg.tbs) {
    src = sb->dev;
  } else {
    mi::set_error("no data and no stored TB of this size in the softbuffer");
    return SRSLTE_ERROR;
  }
  c->prof.mark(0, c->st);
  mi::UlPlan& P = c->eng.plan;
  if (P.build(&c->cfg, 1)) return SRSLTE_ERROR;
  if (q->normalize_en) P.txs[0].scale = (float)q->cell.nof_prb / 15.0f / sqrtf((float)c->cfg.L_prb);
  if (q->cfo_en) P.txs[0].cfo = q->current_cfo;
  c->prof.mark(1, c->st);
  const size_t n = (size_t)15 * mi::symbol_sz(q->cell.nof_prb);
  if (c->eng.upload(c->st)) return SRSLTE_ERROR;
  c->prof.mark(2, c->st);
  if (c->eng.run(src, c->d_iq.p, c->st)) return SRSLTE_ERROR;
  c->prof.mark(3, c->st);
  if (!mi::hip_ok(hipMemcpyAsync(c->h_iq, c->d_iq.p, n * 8, hipMemcpyDeviceToHost, c->st), "D2H IQ") ||
      !mi::hip_ok(hipStreamSynchronize(c->st), "ul sync"))
    return SRSLTE_ERROR;
  memcpy(output_signal, c->h_iq, n * 8);
  c->prof.mark(4, c->st);
  return SRSLTE_SUCCESS;
}

int srslte_softbuffer_tx_init(srslte_softbuffer_tx_t* q, uint32_t nof_prb) {
  if (!q || mi::symbol_sz(nof_prb) < 0) return SRSLTE_ERROR_INVALID_INPUTS;
  memset(q, 0, sizeof(*q));
  mi::CbSegm sg;
  q->max_cb = mi::cbsegm(75376, &sg) ? 1 : sg.C;
  if (!mi::hip_ok(hipMalloc(&q->dev, TX_MAX_BYTES), "softbuffer_tx")) { q->dev = nullptr; return SRSLTE_ERROR; }
  return SRSLTE_SUCCESS;
}
void srslte_softbuffer_tx_reset(srslte_softbuffer_tx_t* q) {
  if (q) q->tbs = 0;
}
void srslte_softbuffer_tx_free(srslte_softbuffer_tx_t* q) {
  if (!q) return;
  if (q->dev) (void)hipFree(q->dev);
  memset(q, 0, sizeof(*q));
}

int srslte_dci_msg_to_ul_grant(srslte_dci_msg_t* msg, uint32_t nof_prb, uint32_t n_rb_ho, srslte_ra_ul_dci_t* dci,
                               srslte_ra_ul_grant_t* grant, uint32_t /*tti*/) {
  if (!msg || !dci || !grant || mi::symbol_sz(nof_prb) < 0) return SRSLTE_ERROR_INVALID_INPUTS;
  memset(dci, 0, sizeof(*dci));
  if (msg->nof_bits != mi::dci_size(mi::DCI_0, nof_prb) || msg->data[0] != 0) return SRSLTE_ERROR;
  // 36.212 5.3.3.1.1: flag, hopping flag, RIV, MCS/RV, NDI, TPC, cyclic shift DM RS, CQI request
  uint32_t pos = 1;
  dci->freq_hop_fl = take_bits(msg->data, &pos, 1);
  // with hopping the resource-allocation field's N_UL_hop MSBs are the hopping bits (36.213 8.4,
  // Table 8.4-1), the rest is the RIV
  const uint32_t nh = dci->freq_hop_fl ? (nof_prb < 50 ? 1u : 2u) : 0u;
  const uint32_t hbits = take_bits(msg->data, &pos, nh);
  const uint32_t riv = take_bits(msg->data, &pos, rba_bits(nof_prb) - nh);
  const uint32_t mcs = take_bits(msg->data, &pos, 5);
  dci->ndi = take_bits(msg->data, &pos, 1) != 0;
  dci->tpc_pusch = take_bits(msg->data, &pos, 2);
  const uint32_t ncs = take_bits(msg->data, &pos, 3);
  dci->cqi_request = take_bits(msg->data, &pos, 1) != 0;
  dci->rv_idx = mcs > 28 ? mcs - 28 : 0;
  if (grant_from_riv(riv, nof_prb, mcs, ncs, dci, grant)) return SRSLTE_ERROR;
  if (dci->freq_hop_fl) return apply_hopping_bits(nof_prb, n_rb_ho, nh, hbits, grant);
  return SRSLTE_SUCCESS;
}

int srslte_dci_rar_to_ul_grant(srslte_dci_rar_grant_t* rar, uint32_t nof_prb, uint32_t n_rb_ho,
                               srslte_ra_ul_dci_t* dci, srslte_ra_ul_grant_t* grant) {
  if (!rar || !dci || !grant || mi::symbol_sz(nof_prb) < 0) return SRSLTE_ERROR_INVALID_INPUTS;
  memset(dci, 0, sizeof(*dci));
  // 36.213 6.2: the 10-bit fixed-size resource block assignment becomes format 0's b-bit field: its b LSBs
  // (N_RB <= 44), or (N_RB > 44) b - 10 zero bits inserted after the N_UL_hop hopping bits (none without
  // hopping: zero-extended).  The field's N_UL_hop MSBs are the hopping bits, the rest the RIV; the truncated
  // MCS is I_MCS 0..15
  const uint32_t b = rba_bits(nof_prb);
  const uint32_t nh = rar->hopping_flag ? (nof_prb < 50 ? 1u : 2u) : 0u;
  uint32_t field;
  if (nof_prb <= 44) {
    field = rar->rba & ((1u << b) - 1u);
  } else {
    const uint32_t hb = (rar->rba >> (10 - nh)) & ((1u << nh) - 1u), rest = rar->rba & ((1u << (10 - nh)) - 1u);
    field = (hb << (b - nh)) | rest;
  }
  const uint32_t hbits = nh ? field >> (b - nh) : 0u, riv = field & ((1u << (b - nh)) - 1u);
  dci->freq_hop_fl = rar->hopping_flag;
  dci->tpc_pusch = rar->tpc_pusch;
  dci->cqi_request = rar->cqi_request;
  dci->ndi = true;
  if (grant_from_riv(riv, nof_prb, rar->trunc_mcs & 15u, 0, dci, grant)) return SRSLTE_ERROR;
  return nh ? apply_hopping_bits(nof_prb, n_rb_ho, nh, hbits, grant) : SRSLTE_SUCCESS;
}

}  // extern "C"
