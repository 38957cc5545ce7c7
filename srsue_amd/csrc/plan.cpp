// plan.cpp -- batch planner (see engine.cpp header): RE lists, scrambling words, CRS tables,
// code-block segmentation, rate-matching splits and 64-lane grouping of equal-K code blocks.
#include "plan.h"
#ifdef MI_PLAN_PROF
#include <chrono>
#include <cstdio>
#endif
#include "tb_body.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <set>
#include <tuple>
#include <unordered_map>

namespace mi {

static thread_local std::string g_err;
void set_error(const std::string& s) { g_err = s; }
const char* last_error() { return g_err.c_str(); }

static size_t align4(size_t x) { return (x + 3) & ~(size_t)3; }

void Plan::add_ktab(uint32_t K) {
  auto& kp = kpos_cache[K];
  if (kp.empty()) {
    kp.resize(5);
    cb_pos_table(K, kp[0]);
    qpp_table(K, kp[1]);
    crc_bit_table(K, 0x864CFBu, kp[2]);
    crc_bit_table(K, 0x800063u, kp[3]);
    kp[4].assign(ncb_of(K), 0xFFFFFFFFu);   // inverse of pos (tdec_win_body.h win_load)
    for (uint32_t i = 0; i < (uint32_t)kp[0].size(); i++) kp[4][kp[0][i]] = i;
  }
  MiKTab t{K, ncb_of(K), 0, 0, 0, 0, 0};
  uint32_t* offs[5] = {&t.pos_off, &t.pi_off, &t.crca_off, &t.crcb_off, &t.ipos_off};
  for (int q = 0; q < 5; q++) {
    while (kdata.size() % 4) kdata.push_back(0u);   // 16-B aligned tables (tdec_body.h pos_window)
    *offs[q] = (uint32_t)kdata.size();
    kdata.insert(kdata.end(), kp[q].begin(), kp[q].end());
  }
  ktabs.push_back(t);
}

#ifdef MI_PLAN_PROF
#define PLAN_T(name) do { auto _n = std::chrono::steady_clock::now(); fprintf(stderr, " %s %.2f", name, std::chrono::duration<double, std::milli>(_n - _pt).count()); _pt = _n; } while (0)
#else
#define PLAN_T(name) ((void)0)
#endif
int Plan::build(const mi_dl_sf_cfg_t* cfgs, uint32_t n, bool with_pdsch) {
#ifdef MI_PLAN_PROF
  auto _pt = std::chrono::steady_clock::now();
  fprintf(stderr, "\n");
#endif
  has_pdsch = with_pdsch;
  cb_K = cb_n = 0;
  cells.clear(); crs.clear(); pds.clear(); re_tab.clear(); scr_tab.clear(); sfs.clear(); lanes.clear();
  groups.clear(); ktabs.clear(); kdata.clear(); tbs.clear(); cb_list.clear(); fft_lists.clear(); rm_items.clear(); rm_recs.clear();
  pairs.clear();
  rm_direct.clear();
  rm_busy = rm_dbusy = 0;
  rm_rep = false;
  fft_list_flat.clear(); fft_list_off.clear(); fft_W.clear();
  iq_samples = grid_elems = ce_elems = e_floats = sb_floats = scratch_floats = dec_bytes = payload_bytes = 0;
  max_units = max_ncb = n_cb = 0;
  bytes_compulsory = 0;
  for (double& b : stage_bytes) b = 0;
  sfs.reserve(n);
  tbs.reserve(n);

  std::map<std::tuple<uint32_t, uint32_t, uint32_t>, uint32_t> cell_idx;
  std::unordered_map<ReKey, uint32_t, ReKeyHash> re_idx;        // -> offset in re_tab (this build)
  std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, uint32_t> scr_idx;   // (cell, rnti, sf, G) -> scr_tab
  std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>, uint32_t> pd_idx;
  std::map<int, std::vector<uint32_t>> fft_map;
  std::vector<uint32_t> re;

  // code blocks: per TB the index of its first one (cb_first), per code block its K, E and LLR offset
  std::vector<CbSegm> segs(n);
  std::vector<uint32_t> cb_first(n + 1, 0), cb_E;
  std::vector<uint64_t> cb_eoff;
  cb_E.reserve((size_t)n * 4);
  cb_eoff.reserve((size_t)n * 4);
  uint32_t last_tbs = 0;
  CbSegm last_sg{};
  ReKey rk{}, last_rk{};
  uint32_t last_re = 0xFFFFFFFFu;

  for (uint32_t s = 0; s < n; s++) {
    const mi_dl_sf_cfg_t& c = cfgs[s];
    const int N = symbol_sz(c.nof_prb);
    if (N < 0 || c.nof_prb == 0 || c.nof_ports < 1 || c.nof_ports > 2 || c.sf_idx > 9) {
      set_error("invalid cell configuration");
      return -1;
    }
    const uint32_t W = 12 * c.nof_prb;
    auto ck = std::make_tuple(c.cell_id, c.nof_prb, c.nof_ports);
    uint32_t ci;
    auto it = cell_idx.find(ck);
    if (it == cell_idx.end()) {
      ci = (uint32_t)cells.size();
      cell_idx[ck] = ci;
      MiCellDesc cd{c.cell_id, c.nof_prb, c.nof_ports, (uint32_t)N, W, (uint32_t)(crs.size() / 2)};
      cells.push_back(cd);
      auto& tab = crs_cache[ck];
      if (tab.empty()) {
        tab.resize(20 * 2 * 2 * NRB_MAX * 2);
        for (uint32_t ns = 0; ns < 20; ns++)
          for (uint32_t li = 0; li < 2; li++) crs_seq(c.cell_id, ns, li ? 4 : 0, &tab[((ns * 2 + li) * 2 * NRB_MAX) * 2]);
      }
      crs.insert(crs.end(), tab.begin(), tab.end());
    } else {
      ci = it->second;
    }
    MiSfDesc sd{};
    sd.iq_off = iq_samples;
    sd.grid_off = grid_elems;
    sd.ce_off = ce_elems;
    sd.cell = ci;
    sd.sf_idx = c.sf_idx;
    sd.tb = s;
    iq_samples += (size_t)sf_len(N);
    grid_elems += (size_t)NSYMB * W;
    ce_elems += (size_t)NSYMB * W * c.nof_ports;
    fft_map[N].push_back(s);
    stage_bytes[MI_DL_STAGE_OFDM] += (double)sf_len(N) * 8 + (double)NSYMB * W * 8;
    stage_bytes[MI_DL_STAGE_CHEST] += (double)NSYMB * W * 8 * c.nof_ports + 4.0 * W * 8;
    bytes_compulsory += (double)sf_len(N) * 8;

    if (with_pdsch) {
      if (c.tm == 2 && c.nof_ports != 2) { set_error("TM2 needs 2 ports"); return -1; }
      if (c.Qm != 2 && c.Qm != 4 && c.Qm != 6) { set_error("Qm must be 2, 4 or 6"); return -1; }
      if (c.tbs == 0 || c.tbs % 8) { set_error("TBS must be a positive multiple of 8"); return -1; }
      // the RE list of (cell, cfi, sf, mask): consecutive subframes usually repeat the previous key
      rk.cell_id = c.cell_id; rk.nof_prb = c.nof_prb; rk.nof_ports = c.nof_ports; rk.cfi = c.cfi; rk.sf = c.sf_idx;
      memset(rk.mask, 0, sizeof(rk.mask));
      for (uint32_t p = 0; p < c.nof_prb; p++) rk.mask[p] = c.prb_mask[p];
      uint32_t re_off;
      if (last_re != 0xFFFFFFFFu && rk == last_rk) {
        re_off = last_re;
      } else {
        auto ri = re_idx.find(rk);
        if (ri == re_idx.end()) {
          auto& cached = re_cache[rk];
          if (cached.empty()) {
            pdsch_re_list(c.cell_id, c.nof_prb, c.nof_ports, c.cfi, c.sf_idx, c.prb_mask, re);
            cached.reserve(re.size() + 1);
            cached.push_back((uint32_t)re.size());   // [0] = count (an empty list stays distinguishable)
            cached.insert(cached.end(), re.begin(), re.end());
          }
          ri = re_idx.emplace(rk, (uint32_t)re_tab.size()).first;
          re_tab.insert(re_tab.end(), cached.begin(), cached.end());   // count, then the list
        }
        re_off = last_re = ri->second;
        last_rk = rk;
      }
      const uint32_t nre = re_tab[re_off];
      if (c.tm == 2 && (nre & 1)) { set_error("odd RE count for SFBC"); return -1; }
      const uint32_t G = nre * c.Qm;
      const auto sk = std::make_tuple(c.cell_id, c.rnti, c.sf_idx, G);
      auto si = scr_idx.find(sk);
      if (si == scr_idx.end()) {
        auto& words = scr_cache[sk];
        if (words.empty()) {
          words.resize((G + 31) / 32 + 1);
          gold_words((c.rnti << 14) | (c.sf_idx << 9) | c.cell_id, G, words.data());
        }
        si = scr_idx.emplace(sk, (uint32_t)scr_tab.size()).first;
        scr_tab.insert(scr_tab.end(), words.begin(), words.end());
      }
      const auto pk = std::make_tuple(ci, c.sf_idx, re_off, si->second, c.Qm, c.tm);
      auto pit = pd_idx.find(pk);
      uint32_t pi_;
      if (pit == pd_idx.end()) {
        pi_ = (uint32_t)pds.size();
        pd_idx.emplace(pk, pi_);
        pds.push_back(MiPdschDesc{ci, c.sf_idx, nre, c.Qm, c.tm, G, re_off + 1, si->second});
      } else {
        pi_ = pit->second;
      }
      const MiPdschDesc& pd = pds[pi_];
      sd.pdsch = pi_;
      sd.e_off = e_floats;
      e_floats += align4(pd.G);
      const uint32_t units = pd.tm == 2 ? pd.nre / 2 : pd.nre;
      max_units = std::max(max_units, units);
      // ---- transport block (segmentation depends on the TBS only)
      if (c.tbs != last_tbs) {
        if (cbsegm(c.tbs, &last_sg)) { set_error("segmentation failed"); return -1; }
        last_tbs = c.tbs;
      }
      const CbSegm& sg = last_sg;
      segs[s] = sg;
      MiTbDesc tb{};
      tb.tbs = c.tbs; tb.C = sg.C; tb.Kp = sg.Kp; tb.Km = sg.Km; tb.Cm = sg.Cm; tb.F = sg.F;
      tb.pay_off = (uint32_t)payload_bytes;
      payload_bytes += c.tbs / 8;
      tbs.push_back(tb);
      const uint32_t NL = c.tm == 2 ? (c.nl_td ? c.nl_td : 2) : 1;
      uint64_t eo = sd.e_off;
      cb_first[s] = (uint32_t)cb_E.size();
      for (uint32_t r = 0; r < sg.C; r++) {
        const uint32_t E = rm_E(pd.G, sg.C, c.Qm, NL, r);
        cb_E.push_back(E);
        cb_eoff.push_back(eo);
        eo += E;
      }
      stage_bytes[MI_DL_STAGE_DEMAP] += (double)pd.nre * 8 * (1 + c.nof_ports) + (double)pd.G * 4;
      bytes_compulsory += (double)c.tbs / 8;
    }
    sfs.push_back(sd);
  }
  cb_first[n] = (uint32_t)cb_E.size();
  PLAN_T("sf");
  for (auto& kv : fft_map) {
    fft_lists.push_back(kv);
    fft_list_off.push_back(fft_list_flat.size());
    fft_list_flat.insert(fft_list_flat.end(), kv.second.begin(), kv.second.end());
    fft_W.push_back(12 * cfgs[kv.second[0]].nof_prb);
  }
  if (!with_pdsch) return 0;

  PLAN_T("fft");
  // ---- group code blocks of equal K into 64-lane wavefront groups: a stable counting sort by K (TB order,
  // then r, within each K)
  struct CbRef { uint32_t K, tb, r; };
  const uint32_t ncbs = cb_first[n];
  std::vector<CbRef> cbs(ncbs);
  {
    std::map<uint32_t, uint32_t> kcount;
    for (uint32_t s = 0; s < n; s++) {
      const CbSegm& sg = segs[s];
      if (sg.Cm) kcount[sg.Km] += sg.Cm;
      kcount[sg.Kp] += sg.C - sg.Cm;
    }
    std::map<uint32_t, uint32_t> kpos;
    uint32_t acc = 0;
    for (auto& kv : kcount) { kpos[kv.first] = acc; acc += kv.second; }
    uint32_t lastK = 0, *slot = nullptr;
    for (uint32_t s = 0; s < n; s++) {
      const CbSegm& sg = segs[s];
      for (uint32_t r = 0; r < sg.C; r++) {
        const uint32_t K = r < sg.Cm ? sg.Km : sg.Kp;
        if (K != lastK || !slot) { slot = &kpos[K]; lastK = K; }
        cbs[(*slot)++] = CbRef{K, s, r};
      }
    }
  }
  PLAN_T("sort");
  // per (K, F, rv): the rank table, N_v and the rank of k0 (r0), computed once
  struct LaneRm { const std::vector<int32_t>* rk; uint32_t Nv, r0; };
  std::unordered_map<uint64_t, LaneRm> lrm;
  auto lane_rm = [&](uint32_t K, uint32_t F, uint32_t rv) -> const LaneRm& {
    const uint64_t key = (uint64_t)K | ((uint64_t)F << 16) | ((uint64_t)rv << 32);
    auto it = lrm.find(key);
    if (it != lrm.end()) return it->second;
    auto& rkc = rank_cache[{K, F}];
    if (rkc.first.empty()) cb_rank_table(K, F, rkc.first, &rkc.second);
    const uint32_t k0 = k0_of(K, rv), Ncb = ncb_of(K);
    uint32_t r0 = 0;
    for (uint32_t p = 0; p < k0 && p < Ncb; p++) r0 += rkc.first[p] >= 0 ? 1 : 0;
    return lrm.emplace(key, LaneRm{&rkc.first, rkc.second, r0 % rkc.second}).first->second;
  };
  lanes.reserve((ncbs / LANES + 256) * LANES);
  std::map<uint32_t, uint32_t> ktab_idx;
  for (size_t i = 0; i < cbs.size();) {
    const uint32_t K = cbs[i].K;
    size_t j = i;
    while (j < cbs.size() && cbs[j].K == K) j++;
    uint32_t kt;
    auto kit = ktab_idx.find(K);
    if (kit == ktab_idx.end()) {
      kt = (uint32_t)ktabs.size();
      ktab_idx[K] = kt;
      add_ktab(K);
    } else {
      kt = kit->second;
    }
    const uint32_t Ncb = ncb_of(K);
    max_ncb = std::max(max_ncb, Ncb);
    const size_t gsz = sb_group_floats(Ncb), ssz = (size_t)LANES * (2 * K + 8 * (K / TDEC_CK_MIN + 1));
    for (size_t g0 = i; g0 < j; g0 += LANES) {
      MiGroupDesc g{};
      g.K = K; g.Ncb = Ncb; g.ktab = kt;
      g.lane0 = (uint32_t)lanes.size();
      g.sb_off = sb_floats;
      g.scratch_off = scratch_floats;
      g.dec_off = dec_bytes;
      sb_floats += gsz;
      scratch_floats += ssz;
      dec_bytes += (size_t)K * LANES;
      groups.push_back(g);
      for (size_t q = 0; q < (size_t)LANES; q++) {
        MiLaneDesc ld{};
        if (g0 + q < j) {
          const CbRef& cr = cbs[g0 + q];
          const mi_dl_sf_cfg_t& c = cfgs[cr.tb];
          const CbSegm& sg = segs[cr.tb];
          const uint32_t F = cr.r == 0 ? sg.F : 0;
          const uint32_t cbi = cb_first[cr.tb] + cr.r;
          ld.e_off = cb_eoff[cbi];
          ld.E = cb_E[cbi];
          const LaneRm& lr = lane_rm(K, F, c.rv);
          ld.Nv = lr.Nv;
          ld.r0 = lr.r0;
          ld.F = F;
          ld.new_tb = c.new_tb ? 1 : 0;
          ld.crc24a = sg.C == 1 ? 1 : 0;
          ld.tb = cr.tb;
          ld.valid = 1;
          {
            // payload run of CB r (tb_kernel's closed form): bytes s(r) .. s(r + 1) - 1 of the TB, clipped at
            // TBS / 8 (the last code block also carries the TB CRC)
            const MiTbDesc& tb = tbs[cr.tb];
            const uint32_t r = cr.r, nm = r < tb.Cm ? r : tb.Cm;
            ld.pay_st = tb.pay_off + nm * (tb.Km / 8) + (r - nm) * (tb.Kp / 8) - (r ? tb.F / 8 : 0) -
                        (tb.C > 1 ? 3 * r : 0);
            ld.tbcrc = (sg.C == 1 || cr.r + 1 == sg.C) ? 1 : 0;
          }
          // rank table offset: one copy per (K, F) in kdata
          ld.rank_off = 0xFFFFFFFFu;
          lanes.push_back(ld);
          stage_bytes[MI_DL_STAGE_RM] += (double)ld.E * 4 + (double)Ncb * 4 * (ld.new_tb ? 1 : 2);
          stage_bytes[MI_DL_STAGE_TDEC] += (double)(3 * K + 12) * 4 + (double)K / 8;
          bytes_compulsory += (double)Ncb * 4 * (ld.new_tb ? 1 : 2);
          n_cb++;
        } else {
          lanes.push_back(ld);
        }
      }
    }
    if (((j - i + LANES - 1) / LANES) & 1)   // odd group count: padding for the unpaired group's pair scratch
      scratch_floats += ssz;
    i = j;
  }
  PLAN_T("lanes");
  build_pairs();
  // fused demap sources of every lane
  lane_src.assign(lanes.size(), MiLaneSrc{0, 0, 0, 0, 0, 2, 0, 0, 0});
  for (size_t li = 0; li < lanes.size(); li++) {
    const MiLaneDesc& ld = lanes[li];
    if (!ld.valid) continue;
    const MiSfDesc& sd = sfs[ld.tb];
    const MiPdschDesc& pd = pds[sd.pdsch];
    // pad: floor(2^32 / W) + 1, so that __umulhi(re, pad) = re / W exactly for every RE index (< 2^32 / W)
    const uint32_t W = cells[sd.cell].W;
    lane_src[li] = MiLaneSrc{sd.grid_off, sd.ce_off, (uint32_t)NSYMB * W, pd.re_off, pd.scr_off, pd.Qm,
                             pd.tm == 2 ? 1u : 0u, (uint32_t)(ld.e_off - sd.e_off),
                             (uint32_t)(0x100000000ull / W + 1)};
    rm_rep |= ld.E > ld.Nv;
  }
  unit_kind = 0;
  bool mixed = false;
  for (size_t li = 0; li < lanes.size(); li++) {
    if (!lanes[li].valid) continue;
    const uint32_t k = lane_src[li].qm + 8 * lane_src[li].tm2;
    if (!unit_kind) unit_kind = k;
    else if (k != unit_kind) mixed = true;
  }
  if (mixed) unit_kind = 0;
  PLAN_T("lanesrc");
  // rank tables into kdata, patch lane offsets
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> rank_off;
  {
    std::pair<uint32_t, uint32_t> lastk{0xFFFFFFFFu, 0};
    uint32_t lasto = 0;
    for (size_t gi = 0; gi < groups.size(); gi++) {
      for (uint32_t q = 0; q < (uint32_t)LANES; q++) {
        MiLaneDesc& ld = lanes[groups[gi].lane0 + q];
        if (!ld.valid) continue;
        const auto key = std::make_pair(groups[gi].K, ld.F);
        if (key == lastk) { ld.rank_off = lasto; continue; }
        auto ro = rank_off.find(key);
        if (ro == rank_off.end()) {
          const auto& rk = rank_cache[key].first;
          uint32_t off = (uint32_t)kdata.size();
          for (int32_t v : rk) kdata.push_back((uint32_t)v);
          // chunk table: non-null positions before c * RM_CHUNK, c = 0 .. ceil(Ncb / RM_CHUNK)
          const uint32_t nch = (uint32_t)((rk.size() + RM_CHUNK - 1) / RM_CHUNK);
          uint32_t cnt = 0;
          for (uint32_t c = 0, p = 0; c <= nch; c++) {
            const uint32_t end = std::min<uint32_t>(c * RM_CHUNK, (uint32_t)rk.size());
            for (; p < end; p++) cnt += rk[p] >= 0 ? 1 : 0;
            kdata.push_back(cnt);
          }
          ro = rank_off.emplace(key, off).first;
        }
        ld.rank_off = lasto = ro->second;
        lastk = key;
      }
    }
  }
  PLAN_T("rank");
  // direct groups (rm.hip): every valid lane new, one rank table, one k0 rank, one unit kind, whole units, E <= N_v;
  // their rank -> row tables (row = ipos[p], decoder-input order) into kdata.  rm_direct_on = false (MI_RM_DIRECT=0 at
  // engine creation) sends every group through the general combine (A/B and parity tests).
  std::vector<uint8_t> direct(groups.size(), 0);
  std::vector<uint32_t> direct_rrow(groups.size(), 0);
  {
    const bool off = !rm_direct_on;
    std::map<std::pair<uint32_t, uint32_t>, uint32_t> rrow_off;
    for (size_t gi = 0; gi < groups.size() && !off; gi++) {
      const MiGroupDesc& g = groups[gi];
      const MiLaneDesc* L = &lanes[g.lane0];
      int f = -1;
      bool ok = true;
      uint32_t emax = 0, kind = 0;
      for (uint32_t q = 0; q < (uint32_t)LANES && ok; q++) {
        if (!L[q].valid) continue;
        const uint32_t k = lane_src[g.lane0 + q].qm + 8 * lane_src[g.lane0 + q].tm2;
        if (f < 0) { f = (int)q; kind = k; }
        const uint32_t U = (k & 7u) * (k >> 3 ? 2u : 1u);   // LLRs per demap unit: whole units per code block
        ok = L[q].new_tb && L[q].E <= L[q].Nv && L[q].rank_off == L[f].rank_off && L[q].r0 == L[f].r0 &&
             L[q].Nv == L[f].Nv && k == kind && L[q].E % U == 0 && lane_src[g.lane0 + q].eb % U == 0;
        emax = std::max(emax, L[q].E);
      }
      if (!ok || f < 0) continue;
      const MiLaneDesc& l0 = L[f];
      const auto key = std::make_pair(g.K, l0.F);
      auto ro = rrow_off.find(key);
      if (ro == rrow_off.end()) {
        const auto& rk = rank_cache[key].first;
        std::vector<uint32_t> rrow(l0.Nv, 0u);
        for (uint32_t p = 0; p < (uint32_t)rk.size(); p++)
          if (rk[p] >= 0) rrow[(uint32_t)rk[p]] = kdata[ktabs[g.ktab].ipos_off + p];
        ro = rrow_off.emplace(key, (uint32_t)kdata.size()).first;
        kdata.insert(kdata.end(), rrow.begin(), rrow.end());
      }
      direct[gi] = 1;
      direct_rrow[gi] = ro->second;
      rm_direct.insert(rm_direct.end(), {g.lane0, g.Ncb, (uint32_t)(g.sb_off / LANES), ro->second, l0.r0, l0.Nv,
                                         emax | (kind << 24), l0.rank_off});
    }
  }
  PLAN_T("direct");
  // rate de-matching chunks with received LLRs (rm.hip): the kernel's per-lane test
  // (nr > 0 && (E >= Nv || j0 < E || j0 + nr > Nv)), i.e. chunk c's rank run [ch[c], ch[c + 1]) meets the lane's
  // circular window of ranks [r0, r0 + E) mod N_v -- found per distinct lane parameters by binary search over the
  // monotone chunk table, marked in a difference array
  {
    std::vector<uint32_t> idle, gbusy;
    std::vector<int32_t> diff;
    std::vector<std::array<uint32_t, 4>> seen;
    rm_items.clear();
    rm_items.reserve((size_t)groups.size() * 80);
    for (size_t gi = 0; gi < groups.size(); gi++) {
      const uint32_t Ncb = groups[gi].Ncb, nch = (Ncb + RM_CHUNK - 1) / RM_CHUNK;
      diff.assign(nch + 1, 0);
      diff[0] += 1;   // chunk 0 always (it writes the group's zero row)
      diff[1] -= 1;
      seen.clear();
      for (uint32_t q = 0; q < (uint32_t)LANES; q++) {
        const MiLaneDesc& ld = lanes[groups[gi].lane0 + q];
        if (!ld.valid) continue;
        const std::array<uint32_t, 4> sk{ld.rank_off, ld.r0, ld.Nv, ld.E};
        if (std::find(seen.begin(), seen.end(), sk) != seen.end()) continue;
        seen.push_back(sk);
        const uint32_t* ch = &kdata[(size_t)ld.rank_off + Ncb];   // ch[0..nch], monotone
        // chunks whose rank run meets [a, b): ch[c + 1] > a and ch[c] < b (and nr > 0)
        auto mark = [&](uint32_t a, uint32_t b) {
          if (a >= b) return;
          const uint32_t c0 = (uint32_t)(std::upper_bound(ch + 1, ch + nch + 1, a) - (ch + 1));
          const uint32_t c1 = (uint32_t)(std::lower_bound(ch, ch + nch, b) - ch);   // first chunk with ch[c] >= b
          if (c0 < c1) { diff[c0] += 1; diff[c1] -= 1; }
        };
        if (ld.E >= ld.Nv) {
          mark(0, ld.Nv);
        } else if (ld.r0 + ld.E <= ld.Nv) {
          mark(ld.r0, ld.r0 + ld.E);
        } else {
          mark(ld.r0, ld.Nv);
          mark(0, ld.r0 + ld.E - ld.Nv);
        }
      }
      int32_t acc = 0;
      for (uint32_t c = 0; c < nch; c++) {
        acc += diff[c];
        if (acc > 0) (direct[gi] ? rm_items : gbusy).push_back(((uint32_t)gi << 9) | c);
        else if (!direct[gi]) idle.push_back(((uint32_t)gi << 9) | c);   // direct groups: the map kernel
      }
    }
    // XCD queues (round 4): workgroup b of a launch runs on XCD b mod 8 (dispatch deals blocks round-robin over
    // the 8 XCDs; speed only, never correctness).  The chunks of one group read the same subframes' grid and
    // channel-estimate lines -- each chunk a few REs per code block, so every line is shared by neighbouring
    // chunks and the compact estimates' pilot rows by all of them -- but dealt in launch order they land on all
    // eight XCDs and every XCD's L2 fetches the group's lines again (TCC_EA0_RDREQ: 6.8 GB per 12,500 subframes
    // against ~2 GB of distinct bytes).  So whole groups go to one queue (the least-loaded one, in group order),
    // each queue keeps its groups' chunks in order, and launch position 8 i + q takes queue q's item i; the
    // shorter queues are padded with empty items (chunk 511: the kernel returns at its first test).
    auto xcd_order = [](std::vector<uint32_t>& its) {
      if (its.empty()) return;
      std::vector<std::vector<uint32_t>> q(8);
      std::vector<size_t> load(8, 0);
      for (size_t a = 0; a < its.size();) {
        size_t b = a;
        while (b < its.size() && (its[b] >> 9) == (its[a] >> 9)) b++;   // one group's chunks
        const size_t k = (size_t)(std::min_element(load.begin(), load.end()) - load.begin());
        q[k].insert(q[k].end(), its.begin() + a, its.begin() + b);
        load[k] += b - a;
        a = b;
      }
      const size_t len = *std::max_element(load.begin(), load.end());
      its.assign(8 * len, 0u);
      for (size_t i = 0; i < len; i++)
        for (size_t k = 0; k < 8; k++) its[8 * i + k] = i < q[k].size() ? q[k][i] : ((q[k].empty() ? 0u : q[k][0] >> 9) << 9) | 511u;
    };
    if (xcd_queues) {   // A/B: false = launch order
      xcd_order(rm_items);
      xcd_order(gbusy);
    }
    rm_dbusy = (uint32_t)rm_items.size();   // direct groups' chunks first (their own launch, rm.hip)
    rm_items.insert(rm_items.end(), gbusy.begin(), gbusy.end());
    rm_busy = (uint32_t)rm_items.size();
    rm_recs.resize((size_t)rm_busy * 4);
    for (uint32_t k = 0; k < rm_busy; k++) {
      const uint32_t it = rm_items[k];
      const MiGroupDesc& g = groups[it >> 9];
      // the softbuffer offset in units of 64 floats (every group region is a multiple: sb_group_floats)
      // Ncb < 2^15 (<= 18,444): bit 15 flags a direct group, whose last field is its rank -> row table
      const bool dr = direct[it >> 9];
      uint32_t* rec = &rm_recs[(size_t)k * 4];
      rec[0] = g.lane0;
      rec[1] = g.Ncb | (dr ? 1u << 15 : 0u) | ((it & 511u) << 16);
      rec[2] = (uint32_t)(g.sb_off / LANES);
      rec[3] = dr ? direct_rrow[it >> 9] : ktabs[g.ktab].ipos_off;
    }
    rm_items.insert(rm_items.end(), idle.begin(), idle.end());
  }
  PLAN_T("busy");
  // TB -> lane lists (counting sort by TB; lanes of a TB in group order = CB order within each K run, K- blocks
  // (r < Cm) first: 36.212 5.1.2)
  {
    std::vector<uint32_t> cnt(n + 1, 0);
    for (const MiLaneDesc& ld : lanes)
      if (ld.valid) cnt[ld.tb + 1]++;
    for (uint32_t s = 0; s < n; s++) cnt[s + 1] += cnt[s];
    cb_list.assign(cnt[n], 0);
    for (uint32_t s = 0; s < n; s++) tbs[s].cb_list = cnt[s];
    for (size_t gi = 0; gi < groups.size(); gi++)
      for (uint32_t q = 0; q < (uint32_t)LANES; q++) {
        const MiLaneDesc& ld = lanes[groups[gi].lane0 + q];
        if (ld.valid) cb_list[cnt[ld.tb]++] = groups[gi].lane0 + q;
      }
  }
  PLAN_T("tblist");
  // TB-CRC multipliers per segmentation: CB r's partial CRC register is shifted over the payload bytes
  // that follow it (tb_body.h tb_crc_term), precomputed once per distinct TB shape (= per TBS)
  std::unordered_map<uint32_t, uint32_t> mul_off;
  for (uint32_t s = 0; s < n; s++) {
    MiTbDesc& t = tbs[s];
    auto it = mul_off.find(t.tbs);
    if (it == mul_off.end()) {
      const uint32_t off = (uint32_t)kdata.size();
      for (uint32_t r = 0; r < t.C; r++) {
        uint32_t after = 0;
        for (uint32_t j = r + 1; j < t.C; j++) after += tb_cb_nbytes(t, j);
        kdata.push_back(gf24_xpow8(after, CRC24A_POLY));
      }
      it = mul_off.emplace(t.tbs, off).first;
    }
    t.crc_mul = it->second;
  }
  PLAN_T("mul");
  return 0;
}

void Plan::build_pairs() {
  pairs.clear();
  for (size_t g = 0; g < groups.size();) {
    const bool two = g + 1 < groups.size() && groups[g + 1].K == groups[g].K;
    pairs.push_back((uint32_t)g);
    pairs.push_back(two ? (uint32_t)(g + 1) : 0xFFFFFFFFu);
    g += two ? 2 : 1;
  }
}

int Plan::build_codeblocks(uint32_t K, uint32_t ncb_req, bool crc24a) {
  if (!cb_size_valid(K) || ncb_req == 0) { set_error("invalid code block size"); return -1; }
  cells.clear(); crs.clear(); pds.clear(); re_tab.clear(); scr_tab.clear(); sfs.clear(); lanes.clear();
  groups.clear(); ktabs.clear(); kdata.clear(); tbs.clear(); cb_list.clear(); fft_lists.clear(); rm_items.clear(); rm_recs.clear();
  pairs.clear();
  rm_direct.clear();
  rm_busy = rm_dbusy = 0;
  fft_list_flat.clear(); fft_list_off.clear(); fft_W.clear();
  iq_samples = grid_elems = ce_elems = e_floats = sb_floats = scratch_floats = dec_bytes = payload_bytes = 0;
  max_units = max_ncb = n_cb = 0;
  bytes_compulsory = 0;
  for (double& b : stage_bytes) b = 0;

  has_pdsch = false;
  cb_K = K;
  cb_n = ncb_req;
  add_ktab(K);
  const uint32_t Ncb = ncb_of(K);
  max_ncb = Ncb;
  for (uint32_t g0 = 0; g0 < ncb_req; g0 += LANES) {
    MiGroupDesc g{};
    g.K = K; g.Ncb = Ncb; g.ktab = 0;
    g.lane0 = (uint32_t)lanes.size();
    g.sb_off = sb_floats;
    g.scratch_off = scratch_floats;
    g.dec_off = dec_bytes;
    sb_floats += sb_group_floats(Ncb);
    scratch_floats += (size_t)LANES * (2 * K + 8 * (K / TDEC_CK_MIN + 1));
    dec_bytes += (size_t)K * LANES;
    groups.push_back(g);
    for (uint32_t q = 0; q < (uint32_t)LANES; q++) {
      MiLaneDesc ld{};
      if (g0 + q < ncb_req) {
        ld.valid = 1; ld.crc24a = crc24a ? 1 : 0; ld.tb = g0 + q; ld.F = 0;
      }
      lanes.push_back(ld);
    }
  }
  if (groups.size() & 1) scratch_floats += (size_t)LANES * (2 * K + 8 * (K / TDEC_CK_MIN + 1));   // pair padding
  build_pairs();
  n_cb = ncb_req;
  stage_bytes[MI_DL_STAGE_RM] = (double)ncb_req * (3 * K + 12) * 4 * 2;        // scatter: read + write
  stage_bytes[MI_DL_STAGE_TDEC] = (double)ncb_req * ((3 * K + 12) * 4 + K / 8);  // SURVEY 8d per CB
  bytes_compulsory = stage_bytes[MI_DL_STAGE_TDEC];
  return 0;
}

}  // namespace mi
