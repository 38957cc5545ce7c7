// plan_dump.cpp -- planner equivalence check (tools/plan_check.sh): builds seeded batch configurations with
// mi::Plan and prints a canonical digest of everything the kernels read, with table offsets resolved to the
// table CONTENTS (so a planner that lays its tables out differently but feeds the kernels the same values
// prints the same digest), and the build time.  Host only (g++ -DMI_EMU, like the emulation library).
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "plan.h"

using namespace mi;

static uint64_t H = 1469598103934665603ull;
static void mix(const void* p, size_t n) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  for (size_t i = 0; i < n; i++) { H ^= b[i]; H *= 1099511628211ull; }
}
template <class T> static void mixv(const T& v) { mix(&v, sizeof(v)); }

static uint64_t rng_s = 1;
static uint32_t rnd(uint32_t n) { rng_s = rng_s * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)((rng_s >> 33) % n); }

static const uint32_t SFC[8] = {1, 2, 3, 4, 6, 7, 8, 9};
static const uint32_t TBS100[27] = {2792, 3624, 4584, 5736, 7224, 8760, 10296, 12216, 14112, 15840, 17568, 19848, 22920,
                                    25456, 28336, 30576, 32856, 36696, 39232, 43816, 46888, 51024, 55056, 57336, 61664,
                                    63776, 75376};
static mi_dl_sf_cfg_t base(uint32_t prb) {
  mi_dl_sf_cfg_t c{};
  c.cell_id = 1; c.nof_prb = prb; c.nof_ports = 1; c.cfi = 1; c.tm = 1; c.nl_td = 2; c.rnti = 0x46; c.rv = 0;
  c.tbs = 75376; c.Qm = 6; c.new_tb = 1;
  for (uint32_t p = 0; p < prb; p++) c.prb_mask[p] = 1;
  return c;
}

static std::vector<mi_dl_sf_cfg_t> scenario(int k, uint32_t n) {
  std::vector<mi_dl_sf_cfg_t> v;
  rng_s = 1234 + k;
  uint32_t rnti[64];
  for (int i = 0; i < 64; i++) rnti[i] = 0x3D + rnd(0xFF00);
  for (uint32_t i = 0; i < n; i++) {
    mi_dl_sf_cfg_t c = base(100);
    c.sf_idx = SFC[i % 8];
    if (k == 1 || k == 3) {   // varied grants: RNTI, MCS 20..28, rv {0,0,0,2}; k == 3: HARQ mix
      const uint32_t mcs = 20 + rnd(9);
      c.Qm = 6; c.tbs = TBS100[mcs - 2];
      c.rnti = rnti[rnd(64)];
      c.rv = rnd(4) == 3 ? 2 : 0;
      if (k == 3) { c.new_tb = rnd(3) != 0; c.rv = rnd(4); }
    } else if (k == 2) {      // mixed cells, partial allocations, TM2
      static const uint32_t P[4] = {6, 25, 50, 100};
      const uint32_t prb = P[i % 4];
      c = base(prb);
      c.sf_idx = SFC[i % 8];
      c.cell_id = 1 + i % 4;
      c.cfi = prb > 10 ? 1 + rnd(3) : 2;
      const uint32_t L = 1 + rnd(prb), st = rnd(prb - L + 1);
      for (uint32_t p = 0; p < prb; p++) c.prb_mask[p] = (p >= st && p < st + L) ? 1 : 0;
      if (rnd(4) == 0) { c.nof_ports = 2; c.tm = 2; }
      const uint32_t G = 12 * L * 9 * 2;
      c.Qm = 2 + 2 * rnd(3);
      c.tbs = 8 * (1 + rnd(G * c.Qm / 16 / 8 + 1));
      if (c.tbs < 16) c.tbs = 16;
      c.rnti = rnti[rnd(64)];
    }
    v.push_back(c);
  }
  return v;
}

static void digest(const Plan& P) {
  H = 1469598103934665603ull;
  for (const auto& c : P.cells) mixv(c);
  mix(P.crs.data(), P.crs.size() * 4);
  for (const auto& s : P.sfs) {
    MiSfDesc t = s;
    t.pdsch = 0;
    mixv(t);
    if (!P.has_pdsch) continue;
    const MiPdschDesc& d = P.pds[s.pdsch];
    mixv(d.cell); mixv(d.sf_idx); mixv(d.nre); mixv(d.Qm); mixv(d.tm); mixv(d.G);
    mix(&P.re_tab[d.re_off], (size_t)d.nre * 4);
    mix(&P.scr_tab[d.scr_off], (size_t)((d.G + 31) / 32 + 1) * 4);
  }
  for (size_t i = 0; i < P.lanes.size(); i++) {
    mixv(P.lanes[i]);
    MiLaneSrc t = P.lane_src[i];
    t.re = t.scr = 0;   // resolved through the subframe's descriptor above
    mixv(t);
  }
  mixv(P.unit_kind);
  mix(P.rm_items.data(), P.rm_items.size() * 4);
  mixv(P.rm_busy); mixv(P.rm_dbusy);
  mix(P.rm_recs.data(), P.rm_recs.size() * 4);
  mix(P.rm_direct.data(), P.rm_direct.size() * 4);
  mixv(P.rm_rep);
  for (const auto& g : P.groups) mixv(g);
  mix(P.pairs.data(), P.pairs.size() * 4);
  for (const auto& t : P.ktabs) mixv(t);
  mix(P.kdata.data(), P.kdata.size() * 4);
  for (const auto& t : P.tbs) mixv(t);
  mix(P.cb_list.data(), P.cb_list.size() * 4);
  mix(P.fft_list_flat.data(), P.fft_list_flat.size() * 4);
  for (size_t x : P.fft_list_off) mixv(x);
  mix(P.fft_W.data(), P.fft_W.size() * 4);
  size_t sz[] = {P.iq_samples, P.grid_elems, P.ce_elems, P.e_floats, P.sb_floats, P.scratch_floats, P.dec_bytes,
                 P.payload_bytes};
  mix(sz, sizeof(sz));
  uint32_t u[] = {P.max_units, P.max_ncb, P.n_cb};
  mix(u, sizeof(u));
  mixv(P.bytes_compulsory);
  mix(P.stage_bytes, sizeof(P.stage_bytes));
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 12500;
  Plan P;
  // MI_RM_XCDQ=0: the work list in launch order (the engine reads this at creation, engine.cpp Engine::Engine)
  if (const char* e = getenv("MI_RM_XCDQ")) P.xcd_queues = atoi(e) != 0;
  for (int k = 0; k < 4; k++) {
    const auto cfgs = scenario(k, n);
    double best = 1e30;
    for (int rep = 0; rep < 3; rep++) {
      const auto t0 = std::chrono::steady_clock::now();
      if (P.build(cfgs.data(), (uint32_t)cfgs.size(), true)) { printf("scenario %d: build failed: %s\n", k, last_error()); return 1; }
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      best = ms < best ? ms : best;
      if (rep == 0) printf("scenario %d cold %.1f ms ", k, ms);
    }
    digest(P);
    printf("warm %.1f ms  digest %016llx  (pds %zu re_tab %zu scr_tab %zu)\n", best, (unsigned long long)H,
           P.pds.size(), P.re_tab.size(), P.scr_tab.size());
  }
  return 0;
}
