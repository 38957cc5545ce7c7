// ctrl.cpp -- host planner of the DL control stage (ctrl.h) and the mi_dl_ctrl_* C ABI.
#include "ctrl.h"

#include <string.h>

#include <map>
#include <tuple>

#include "kernels.h"
#include "tables.h"

namespace mi {

int CtrlEngine::build(const Plan& P, const std::vector<uint32_t>& cfi, uint32_t phich_ng,
                      const std::vector<uint16_t>& rnti, const std::vector<uint32_t>& phich) {
  const size_t n = P.sfs.size();
  if (cfi.size() != n || rnti.size() != n || (!phich.empty() && phich.size() != n)) {
    set_error("ctrl: per-subframe cfi / rnti / phich");
    return -1;
  }
  std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, uint32_t> phich_cache;
  sfs.clear(); cdata.clear(); jobs.clear(); job_fmt.clear(); job_begin.clear(); nof_prb.clear();
  llr_floats = 0; max_regs = 0;
  std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, std::pair<uint32_t, uint32_t>> reg_cache;  // -> (off, M)
  std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, uint32_t> scr_cache, pcf_cache;
  std::map<uint32_t, uint32_t> rank_cache;   // D -> cdata offset
  for (size_t s = 0; s < n; s++) {
    const MiSfDesc& sd = P.sfs[s];
    const MiCellDesc& c = P.cells[sd.cell];
    if (cfi[s] < 1 || cfi[s] > 3) { set_error("ctrl: cfi"); return -1; }
    MiCtrlSf d{};
    d.grid_off = sd.grid_off;
    d.ce_off = sd.ce_off;
    d.plane = NSYMB * c.W;
    d.ports = c.nof_ports;
    auto rk = std::make_tuple(c.id, c.nof_prb, phich_ng, cfi[s]);
    auto it = reg_cache.find(rk);
    if (it == reg_cache.end()) {
      std::vector<uint32_t> re4, lg;
      const uint32_t M = pdcch_regs(c.id, c.nof_prb, phich_ng, cfi[s], &re4);
      pdcch_quad_perm(M, c.id, lg);
      const uint32_t off = (uint32_t)cdata.size();
      cdata.insert(cdata.end(), re4.begin(), re4.end());
      cdata.insert(cdata.end(), lg.begin(), lg.end());
      it = reg_cache.emplace(rk, std::make_pair(off, M)).first;
    }
    d.reg_off = it->second.first;
    d.M = it->second.second;
    d.n_cce = d.M / 9;
    auto sk = std::make_tuple(c.id, sd.sf_idx, d.M, 0u);
    auto si = scr_cache.find(sk);
    if (si == scr_cache.end()) {
      std::vector<uint32_t> w((8 * d.M + 31) / 32);
      gold_words(sd.sf_idx * 512 + c.id, 8 * d.M, w.data());    // 36.211 6.8.2
      si = scr_cache.emplace(sk, (uint32_t)cdata.size()).first;
      cdata.insert(cdata.end(), w.begin(), w.end());
    }
    d.scr_off = si->second;
    auto pk = std::make_tuple(c.id, c.nof_prb, sd.sf_idx, 0u);
    auto pi = pcf_cache.find(pk);
    if (pi == pcf_cache.end()) {
      uint32_t k16[16], w = 0;
      pcfich_k(c.id, c.nof_prb, k16);
      gold_words(pcfich_cinit(c.id, sd.sf_idx), 32, &w);
      pi = pcf_cache.emplace(pk, (uint32_t)cdata.size()).first;
      cdata.insert(cdata.end(), k16, k16 + 16);
      cdata.push_back(w);
    }
    d.pcfich_off = pi->second;
    {   // PHICH query of this subframe
      uint32_t grp, seq;
      const uint32_t qv = phich.empty() ? 0u : phich[s];
      phich_calc(c.nof_prb, phich_ng, qv & 0xFFFFu, qv >> 16, &grp, &seq);
      auto hk = std::make_tuple(c.id, (c.nof_prb << 8) | (phich_ng << 4) | seq, sd.sf_idx, grp);
      auto hi = phich_cache.find(hk);
      if (hi == phich_cache.end()) {
        uint32_t re12[12], w = 0;
        if (phich_res(c.id, c.nof_prb, phich_ng, grp, re12)) { set_error("ctrl: phich group"); return -1; }
        gold_words(phich_cinit(c.id, sd.sf_idx), 12, &w);
        hi = phich_cache.emplace(hk, (uint32_t)cdata.size()).first;
        cdata.insert(cdata.end(), re12, re12 + 12);
        cdata.push_back(w);
        cdata.push_back(seq);
      }
      d.phich_off = hi->second;
    }
    d.llr_off = (uint32_t)llr_floats;
    llr_floats += (size_t)8 * d.M;
    max_regs = std::max(max_regs, d.M);
    sfs.push_back(d);
    nof_prb.push_back(c.nof_prb);
    // jobs in srsLTE's search order (dci_blind_search: one size over all candidates of a space): UE-specific
    // space with the 1A/0 size then format 1, common space with the 1A/0 size then format 1C (1C is only
    // selected for SI/RA/P-RNTI searches)
    job_begin.push_back((uint32_t)jobs.size());
    const uint32_t sizes[2][2] = {{dci_size(DCI_1A, c.nof_prb), dci_size(DCI_1, c.nof_prb)},
                                  {dci_size(DCI_1A, c.nof_prb), dci_size(DCI_1C, c.nof_prb)}};
    for (int common = 0; common < 2; common++) {
      uint32_t Ls[16], nc[16];
      const int nk = search_space(d.n_cce, sd.sf_idx, rnti[s], common != 0, Ls, nc);
      for (int f = 0; f < 2; f++)
        for (int k = 0; k < nk; k++) {
          const uint32_t A = sizes[common][f], D = A + 16;
          auto ri = rank_cache.find(D);
          if (ri == rank_cache.end()) {
            std::vector<uint32_t> rank;
            conv_rank_table(D, rank);
            ri = rank_cache.emplace(D, (uint32_t)cdata.size()).first;
            cdata.insert(cdata.end(), rank.begin(), rank.end());
          }
          jobs.push_back(MiDciJob{(uint32_t)s, d.llr_off, Ls[k], nc[k], A, D, ri->second, rnti[s]});
          job_fmt.push_back((uint8_t)((common << 2) | (f == 0 ? 0 : common ? DCI_1C : DCI_1)));
        }
    }
  }
  job_begin.push_back((uint32_t)jobs.size());
  return 0;
}

int CtrlEngine::upload(hipStream_t st) {
  auto up = [&](DevBuf& b, const void* h, size_t bytes) {
    return b.ensure(bytes) && (bytes == 0 || hip_ok(hipMemcpyAsync(b.p, h, bytes, hipMemcpyHostToDevice, st), "H2D"));
  };
  const bool ok = up(d_sfs, sfs.data(), sfs.size() * sizeof(MiCtrlSf)) &&
                  up(d_cdata, cdata.data(), cdata.size() * 4) && up(d_jobs, jobs.data(), jobs.size() * sizeof(MiDciJob)) &&
                  d_llr.ensure(llr_floats * 4) && d_res.ensure(jobs.size() * sizeof(MiDciRes)) &&
                  d_cfi.ensure(sfs.size() * 4) && d_phich.ensure(sfs.size() * 4) &&
                  hip_ok(hipStreamSynchronize(st), "ctrl upload");
  return ok ? 0 : -1;
}

int CtrlEngine::run(const float2* grid, const float2* ce, uint32_t mask, float noise, hipStream_t st) {
  const uint32_t n = (uint32_t)sfs.size();
  if (mask & 1u) launch_pcfich(grid, ce, d_sfs.as<MiCtrlSf>(), d_cdata.as<uint32_t>(), d_cfi.as<uint32_t>(), n, st);
  if (mask & 2u)
    launch_pdcch_llr(grid, ce, d_sfs.as<MiCtrlSf>(), d_cdata.as<uint32_t>(), d_llr.as<float>(), n, max_regs, noise, st);
  if (mask & 4u)
    launch_dci_search(d_llr.as<float>(), d_jobs.as<MiDciJob>(), d_cdata.as<uint32_t>(), d_res.as<MiDciRes>(),
                      (uint32_t)jobs.size(), st);
  if (mask & 8u) launch_phich(grid, ce, d_sfs.as<MiCtrlSf>(), d_cdata.as<uint32_t>(), d_phich.as<float>(), n, st);
  return hip_ok(hipGetLastError(), "ctrl launch") ? 0 : -1;
}

int CtrlEngine::download(hipStream_t st) {
  res.resize(jobs.size());
  return hip_ok(hipMemcpyAsync(res.data(), d_res.p, res.size() * sizeof(MiDciRes), hipMemcpyDeviceToHost, st), "D2H") &&
                 hip_ok(hipStreamSynchronize(st), "sync")
             ? 0
             : -1;
}

DciFound CtrlEngine::select(uint32_t s, bool ul, bool common_only) const {
  DciFound out{};
  for (uint32_t j = job_begin[s]; j < job_begin[s + 1]; j++) {
    const MiDciJob& jb = jobs[j];
    const MiDciRes& r = res[j];
    if (!r.found) continue;
    const bool common = (job_fmt[j] >> 2) != 0;
    int fmt = job_fmt[j] & 3;
    if (fmt == 0) fmt = ((r.bits[0] >> 31) & 1u) ? DCI_1A : DCI_0;   // the 0/1A flag
    if (ul ? fmt != DCI_0 : fmt == DCI_0) continue;
    if (common_only ? !common : fmt == DCI_1C) continue;            // 1C: SI/RA/P-RNTI only
    out.found = 1;
    out.format = (uint32_t)fmt;
    out.nbits = jb.A;
    out.L = jb.L;
    out.ncce = jb.ncce;
    for (uint32_t i = 0; i < jb.A; i++) out.bits[i] = (uint8_t)((r.bits[i >> 5] >> (31 - (i & 31))) & 1u);
    return out;
  }
  return out;
}

}  // namespace mi

// ---- C ABI (include/mi_dl.h) -----------------------------------------------------------------
#include "batch_impl.h"

struct mi_dl_ctrl {
  mi::CtrlEngine ce;
  mi_dl_batch_t* b = nullptr;
  hipStream_t last = nullptr;
  bool have_res = false, have_phich = false;
  uint32_t phich_ng = 0;
  std::vector<uint32_t> cfi;
  std::vector<float> phich;
};

extern "C" {

mi_dl_ctrl_t* mi_dl_ctrl_create(mi_dl_batch_t* b, uint32_t phich_ng) {
  if (!b) { mi::set_error("null batch"); return nullptr; }
  auto* c = new mi_dl_ctrl();
  c->b = b;
  c->phich_ng = phich_ng;
  std::vector<uint32_t> cfi;
  std::vector<uint16_t> rnti;
  for (const mi_dl_sf_cfg_t& s : b->cfgs) { cfi.push_back(s.cfi); rnti.push_back((uint16_t)s.rnti); }
  if (c->ce.build(b->eng.plan, cfi, phich_ng, rnti) || c->ce.upload(nullptr)) { delete c; return nullptr; }
  return c;
}

void mi_dl_ctrl_destroy(mi_dl_ctrl_t* c) { delete c; }

int mi_dl_ctrl_run_stages(mi_dl_ctrl_t* c, uint32_t mask, void* stream) {
  if (!c) { mi::set_error("null argument"); return -1; }
  c->last = reinterpret_cast<hipStream_t>(stream);
  c->have_res = false;
  c->have_phich = false;
  return c->ce.run(c->b->eng.d_grid.as<float2>(), c->b->eng.d_ce.as<float2>(), mask, 0.0f, c->last);
}
int mi_dl_ctrl_run(mi_dl_ctrl_t* c, void* stream) { return mi_dl_ctrl_run_stages(c, 15u, stream); }

int mi_dl_ctrl_set_phich(mi_dl_ctrl_t* c, const uint32_t* i_lowest, const uint32_t* n_dmrs) {
  if (!c || !i_lowest || !n_dmrs) { mi::set_error("null argument"); return -1; }
  std::vector<uint32_t> cfi, q;
  std::vector<uint16_t> rnti;
  for (size_t s = 0; s < c->b->cfgs.size(); s++) {
    cfi.push_back(c->b->cfgs[s].cfi);
    rnti.push_back((uint16_t)c->b->cfgs[s].rnti);
    if (i_lowest[s] > 0xFFFFu || n_dmrs[s] > 7) { mi::set_error("phich query"); return -1; }
    q.push_back(i_lowest[s] | (n_dmrs[s] << 16));
  }
  if (c->last && !mi::hip_ok(hipStreamSynchronize(c->last), "sync")) return -1;
  return (c->ce.build(c->b->eng.plan, cfi, c->phich_ng, rnti, q) || c->ce.upload(nullptr)) ? -1 : 0;
}

int mi_dl_ctrl_phich(mi_dl_ctrl_t* c, uint32_t sf, float* soft) {
  if (!c || sf >= c->ce.sfs.size()) { mi::set_error("bad subframe"); return -1; }
  if (!c->have_phich) {
    c->phich.resize(c->ce.sfs.size());
    if (!mi::hip_ok(hipStreamSynchronize(c->last), "sync") ||
        !mi::hip_ok(hipMemcpy(c->phich.data(), c->ce.d_phich.p, c->phich.size() * 4, hipMemcpyDeviceToHost), "D2H"))
      return -1;
    c->have_phich = true;
  }
  if (soft) *soft = c->phich[sf];
  return c->phich[sf] > 0.0f ? 1 : 0;
}

int mi_dl_ctrl_result(mi_dl_ctrl_t* c, uint32_t sf, int ul, uint32_t* cfi, uint32_t* format, uint32_t* L,
                      uint32_t* ncce, uint8_t* bits, uint32_t* nbits) {
  if (!c || sf >= c->ce.sfs.size()) { mi::set_error("bad subframe"); return -1; }
  if (!c->have_res) {
    c->cfi.resize(c->ce.sfs.size());
    if (c->ce.download(c->last) ||
        !mi::hip_ok(hipMemcpy(c->cfi.data(), c->ce.d_cfi.p, c->cfi.size() * 4, hipMemcpyDeviceToHost), "D2H"))
      return -1;
    c->have_res = true;
  }
  if (cfi) *cfi = c->cfi[sf];
  const mi::DciFound f = c->ce.select(sf, ul == 1, ul == 2);
  if (!f.found) return 0;
  if (format) *format = f.format;
  if (L) *L = f.L;
  if (ncce) *ncce = f.ncce;
  if (nbits) *nbits = f.nbits;
  if (bits) memcpy(bits, f.bits, f.nbits);
  return 1;
}

size_t mi_dl_ctrl_llr_floats(const mi_dl_ctrl_t* c) { return c ? c->ce.llr_floats : 0; }
size_t mi_dl_ctrl_llr_offset(const mi_dl_ctrl_t* c, uint32_t sf) {
  return (c && sf < c->ce.sfs.size()) ? c->ce.sfs[sf].llr_off : 0;
}
uint32_t mi_dl_ctrl_n_cce(const mi_dl_ctrl_t* c, uint32_t sf) {
  return (c && sf < c->ce.sfs.size()) ? c->ce.sfs[sf].n_cce : 0;
}
int mi_dl_ctrl_llr(mi_dl_ctrl_t* c, float* host, size_t n, int upload) {
  if (!c || n > c->ce.llr_floats) { mi::set_error("llr size"); return -1; }
  const bool ok = upload ? mi::hip_ok(hipMemcpy(c->ce.d_llr.p, host, n * 4, hipMemcpyHostToDevice), "H2D")
                         : (mi::hip_ok(hipStreamSynchronize(c->last), "sync") &&
                            mi::hip_ok(hipMemcpy(host, c->ce.d_llr.p, n * 4, hipMemcpyDeviceToHost), "D2H"));
  return ok ? 0 : -1;
}

}  // extern "C"
