// emu.cpp -- TEST-ONLY host emulation of the per-lane kernel bodies (rm_body.h, tdec_body.h,
// tb_body.h) driven by the real planner.  Built into libsrsue_amd_emu.so with g++ -DMI_EMU; it is
// never linked into the product library.  Lanes of those kernels never communicate, so running
// each lane's code to completion in turn reproduces the GPU result operation for operation; the
// CPU test suite uses it to check planner + rate de-matching + turbo + TB assembly bit-exactly
// against the oracle without a GPU.
#include <algorithm>
#include <string.h>

#include <vector>

#include "kernels_consts.h"
#include "plan.h"
#include "rm_body.h"
#include "tb_body.h"
#include "tdec_body.h"
#include "tdec_p2_body.h"
#include "tdec_win_body.h"

static int g_q16 = 0;   // turbo arithmetic of the emulated decoder (MI_DL_FLAG_TDEC_I16)
extern "C" void emu_set_tdec_i16(int on) { g_q16 = on; }

static uint32_t crc8[256], crc8b[256];   // CRC24A / CRC24B byte tables

// crossed-schedule lane decoder (two wavefronts per group, tdec_body.h tdec_lane_x): 0 = off, 1 = register
// form, 2 = recompute form, 3 = two code blocks per lane (int16 only, tdec_p2_body.h)
static int g_x = 0;
extern "C" void emu_set_tdec_x(int on) { g_x = on; }
// packed decoder: waterfall compaction after iteration 0 (tdec_p2_body.h P2ContSrc; tdec.hip tdec_cont_*),
// continuation pairs filled in REVERSE lane order (the GPU's order depends on atomics: results may not)
static int g_compact = 0;
static uint64_t g_cont_cbs = 0;
extern "C" void emu_set_tdec_compact(int on) { g_compact = on; g_cont_cbs = 0; }
static int g_store_w = 0;   // compaction: the first launch stores its w rows, the continuation gathers them
extern "C" void emu_set_tdec_store_w(int on) { g_store_w = on; }
static int g_seg = 0;      // compaction rounds after the first: segmented, g_seg wavefronts per pair (tdec_kernel_p2s)
extern "C" void emu_set_tdec_seg(int s) { g_seg = s; }
static int g_rounds = 0;    // compaction: one iteration per round, the failing code blocks re-compacted between rounds
static uint64_t g_round_cbs = 0;
extern "C" void emu_set_tdec_rounds(int on) { g_rounds = on; g_round_cbs = 0; }
extern "C" uint64_t emu_round_codeblocks() { return g_round_cbs; }
extern "C" uint64_t emu_cont_codeblocks() { return g_cont_cbs; }
template <bool Q16>
static mi::TdecLaneResult emu_lane_x(const mi::TdecArgs& a, int lane) {
  mi::TdecExecHost ex;
  mi::TdecLaneResult r = g_x == 2 ? mi::tdec_lane_x<Q16, true>(a, lane, ex) : mi::tdec_lane_x<Q16, false>(a, lane, ex);
  r.tb_part = mi::tdec_pack(a, lane);
  return r;
}

// latency-form (segment-parallel) int16 decoder: threads per code block, 0 = off (tdec_win_body.h).
// Each phase of the GPU kernel (between two barriers) runs every segment in turn: within a phase a
// segment only reads what earlier phases wrote, so this reproduces the kernel exactly.
static uint32_t g_win = 0;
static uint64_t g_win_rounds = 0, g_win_halves = 0;
extern "C" void emu_set_tdec_win(uint32_t threads) { g_win = threads; g_win_rounds = g_win_halves = 0; }
extern "C" void emu_win_stats(uint64_t* rounds, uint64_t* halves) { *rounds = g_win_rounds; *halves = g_win_halves; }

template <bool DEC2>
static void emu_win_half(const mi::WinCb& c) {
  g_win_halves++;
  for (uint32_t j = 0; j < c.nseg; j++) mi::win_bwd_first<DEC2>(c, j);
  std::vector<float> v(8 * c.nseg);
  for (;;) {
    for (uint32_t j = 0; j + 1 < c.nseg; j++) mi::ck_get(c.bend + (j + 1) * 8, *reinterpret_cast<float(*)[8]>(&v[8 * j]));
    bool any = false;
    for (uint32_t j = 0; j + 1 < c.nseg; j++) any |= mi::win_bwd_fix<DEC2>(c, j, *reinterpret_cast<float(*)[8]>(&v[8 * j]));
    g_win_rounds++;
    if (!any) break;
  }
  for (uint32_t j = 0; j < c.nseg; j++) mi::win_fwd_first<DEC2>(c, j);
  for (;;) {
    for (uint32_t j = 1; j < c.nseg; j++) mi::ck_get(c.aend + (j - 1) * 8, *reinterpret_cast<float(*)[8]>(&v[8 * j]));
    bool any = false;
    for (uint32_t j = 1; j < c.nseg; j++) any |= mi::win_fwd_fix<DEC2>(c, j, *reinterpret_cast<float(*)[8]>(&v[8 * j]));
    g_win_rounds++;
    if (!any) break;
  }
}

// one code block (lane `lane` of group g) through the latency-form decoder, as tdec_win_kernel does
static mi::TdecLaneResult emu_win_cb(const MiGroupDesc& g, const MiKTab& kt, const MiLaneDesc& ld, const float* sbg,
                                     const uint32_t* kdata, uint32_t lane, uint32_t max_its, uint8_t* row) {
  const uint32_t K = g.K, P = g_win;
  mi::WinCb c;
  c.K = K;
  mi::win_geometry(K, P, c.S, c.nseg);
  std::vector<int16_t> q(3 * K + 12), d(K), w(K), bck((K / 4 + 1) * 8), ack((K / 4 + 1) * 8), bend(P * 8), aend(P * 8);
  std::vector<uint16_t> pi(K);
  std::vector<uint8_t> dec(K), pk(K / 8);
  c.q = q.data(); c.pi = pi.data(); c.d = d.data(); c.w = w.data(); c.dec = dec.data();
  c.bck = bck.data(); c.ack = ack.data(); c.bend = bend.data(); c.aend = aend.data();
  std::vector<uint8_t> lmap((g.Ncb + 15) / 16 * 16);
  c.lmap = lmap.data();
  for (uint32_t t = 0; t < P; t++) mi::win_load_map(c, t, P, sbg, g.Ncb);
  for (uint32_t t = 0; t < P; t++)
    mi::win_load(c, t, P, sbg, kdata + kt.pos_off, kdata + kt.pi_off, lane, ld.F);
  const uint32_t* tab = kdata + (ld.crc24a ? kt.crca_off : kt.crcb_off);
  mi::TdecLaneResult r{0, 0, 0};
  for (uint32_t it = 0; it < max_its; it++) {
    emu_win_half<false>(c);
    emu_win_half<true>(c);
    uint32_t x = 0;
    for (uint32_t t = 0; t < P; t++) x ^= mi::win_crc_part(c, t, P, tab);
    r.its = it + 1;
    r.crc_ok = x == 0;
    if (r.crc_ok) break;
  }
  for (uint32_t t = 0; t < P; t++) mi::win_pack(c, t, P, pk.data());
  memcpy(row, pk.data(), K / 8);
  const uint32_t b0 = ld.F / 8, b1 = K / 8 - (ld.crc24a ? 0 : 3);
  for (uint32_t t = 0; t < P; t++) r.tb_part ^= mi::win_tb_term(c, t, P, pk.data(), b0, b1, crc8);
  return r;
}

// the packed decoder writes each code block's payload run in place (tdec.hip p2_out)
static void emu_p2_out(mi::TdecArgsP2& a, int h, uint8_t* payload, const MiLaneDesc& ld) {
  a.out_bytes = payload;
  a.cb_off[h] = ld.pay_st;
  a.crc24a[h] = ld.crc24a | (ld.tbcrc << 1);
  a.to_payload = 1;
}

extern "C" int emu_decode_llr(const mi_dl_sf_cfg_t* cfgs, uint32_t n, const float* llr_concat, uint32_t max_its,
                              uint8_t* payload, uint32_t* tb_ok, uint32_t* tb_its, uint32_t* cb_its) {
  for (uint32_t b = 0; b < 256; b++) {
    crc8[b] = mi::crc24_byte_entry(b, mi::CRC24A_POLY);
    crc8b[b] = mi::crc24_byte_entry(b, mi::CRC24B_POLY);
  }
  mi::Plan P;
  if (P.build(cfgs, n, true)) return -1;
  std::vector<float> e(P.e_floats, 0.f), sb(P.sb_floats, 0.f), scr(P.scratch_floats, 0.f);
  std::vector<uint8_t> dec(P.dec_bytes, 0), cbb(P.lanes.size() * mi::CB_BYTES_STRIDE, 0);
  std::vector<uint32_t> cits(P.lanes.size(), 0), ccrc(P.lanes.size(), 0), ctbp(P.lanes.size(), 0);
  size_t src = 0;
  for (uint32_t s = 0; s < n; s++) {
    const uint32_t G = P.pds[P.sfs[s].pdsch].G;
    memcpy(&e[P.sfs[s].e_off], llr_concat + src, G * sizeof(float));
    src += G;
  }
  if (g_x == 3 && g_q16) {
    // two code blocks per lane (tdec_p2_body.h): rate de-matching of every group, then the group pairs
    std::vector<std::vector<uint32_t>> wms(P.groups.size());
    for (size_t gi = 0; gi < P.groups.size(); gi++) {
      const MiGroupDesc& g = P.groups[gi];
      float* sbg = &sb[g.sb_off];
      uint8_t* map = reinterpret_cast<uint8_t*>(sbg + mi::sb_map_off(g.Ncb));
      for (uint32_t p = 0; p < g.Ncb; p++) mi::rm_combine_row(&P.lanes[g.lane0], P.kdata.data(), e.data(), sbg, g.Ncb, p,
                                                              &P.kdata[P.ktabs[g.ktab].ipos_off]);
      const MiKTab& kt = P.ktabs[g.ktab];
      wms[gi].resize(g.K / mi::BETA_W + 1);
      for (uint32_t w = 0; w < wms[gi].size(); w++) wms[gi][w] = mi::tdec_window_mask(map, &P.kdata[kt.pos_off], w);
    }
    std::vector<uint32_t> stash((size_t)mi::P2_STASH_ROWS * mi::LANES);
    for (size_t pp = 0; pp < P.pairs.size(); pp += 2) {
      const uint32_t ga = P.pairs[pp], gbi = P.pairs[pp + 1];
      const bool paired = gbi != 0xFFFFFFFFu;
      const uint32_t gb = paired ? gbi : ga;
      const MiGroupDesc &gA = P.groups[ga], &gB = P.groups[gb];
      const MiKTab& kt = P.ktabs[gA.ktab];
      for (int lane = 0; lane < mi::LANES; lane++) {
        const uint32_t li[2] = {gA.lane0 + lane, gB.lane0 + lane};
        const MiLaneDesc &l0 = P.lanes[li[0]], &l1 = P.lanes[li[1]];
        mi::TdecArgsP2 a;
        a.live = (l0.valid ? 1u : 0u) | (paired && l1.valid ? 2u : 0u);
        if (!a.live) continue;
        a.sb[0] = &sb[gA.sb_off]; a.sb[1] = &sb[gB.sb_off];
        a.stash = stash.data();   // the LDS stash of the 16-step spans (one lane at a time here)
        a.wm[0] = wms[ga].data(); a.wm[1] = wms[gb].data();
        a.zrow[0] = gA.Ncb; a.zrow[1] = gB.Ncb;
        a.scr = reinterpret_cast<uint32_t*>(&scr[gA.scratch_off]);
        a.q = a.scr + (size_t)(4 * gA.K + 8) * mi::LANES;
        a.pos = &P.kdata[kt.pos_off]; a.pi = &P.kdata[kt.pi_off];
        a.crc8 = crc8;
        a.crc8b = crc8b;
        a.dec = &dec[gA.dec_off];
        for (int h = 0; h < 2; h++) emu_p2_out(a, h, payload, P.lanes[li[(a.live >> h) & 1u ? h : 0]]);
        a.K = gA.K;
        a.F[0] = l0.F; a.F[1] = paired ? l1.F : l0.F;

        a.max_its = g_compact && max_its > 1 ? 1 : max_its; a.early_stop = 1;
        a.cont_w = 0;
        a.no_w = a.max_its == 1 && !g_store_w;   // tdec.hip launch_tdec_p2
        mi::TdecP2ExecHost ex;
        // the spacing of tdec.hip tdec_kernel_p2x: 16-step spans
        const mi::TdecP2Result r = a.max_its == 1  ? mi::tdec_p2_lane<false, mi::P2_CKS, true>(a, lane, ex)
                                   : !a.early_stop ? mi::tdec_p2_lane<false, mi::P2_CKS, false, 0u>(a, lane, ex)
                                                   : mi::tdec_p2_lane<false, mi::P2_CKS>(a, lane, ex);
        for (int h = 0; h < 2; h++) {
          if (!((a.live >> h) & 1u)) continue;
          cits[li[h]] = r.its[h];
          ccrc[li[h]] = r.crc_ok[h];
          ctbp[li[h]] = r.tb_part[h];
        }
      }
    }
    if (g_compact && max_its > 1) {
      // each group's pair (its first group) and half
      std::vector<uint32_t> pa(P.groups.size()), ph(P.groups.size());
      for (size_t pp = 0; pp < P.pairs.size(); pp += 2)
        for (int h = 0; h < 2; h++)
          if (P.pairs[pp + h] != 0xFFFFFFFFu) { pa[P.pairs[pp + h]] = P.pairs[pp]; ph[P.pairs[pp + h]] = h; }
      std::vector<uint32_t> ks;
      for (const MiGroupDesc& g : P.groups)
        if (std::find(ks.begin(), ks.end(), g.K) == ks.end()) ks.push_back(g.K);
      for (uint32_t K : ks) {
        std::vector<uint32_t> cont;   // continuing code blocks of this K, reverse lane order
        for (size_t gi = P.groups.size(); gi-- > 0;)
          if (P.groups[gi].K == K)
            for (int l = mi::LANES - 1; l >= 0; l--) {
              const uint32_t li = P.groups[gi].lane0 + l;
              if (P.lanes[li].valid && !ccrc[li]) cont.push_back(li);
            }
        g_cont_cbs += cont.size();
        const uint32_t gi0 = [&] { uint32_t g = 0; while (P.groups[g].K != K) g++; return g; }();
        const MiKTab& kt = P.ktabs[P.groups[gi0].ktab];
        const uint32_t* pos = &P.kdata[kt.pos_off];
        const size_t PU = (size_t)(7 * K + 20) * mi::LANES;   // tdec.hip: a dense continuation pair
        const size_t np1 = (cont.size() + 2 * mi::LANES - 1) / (2 * mi::LANES);
        std::vector<std::vector<uint32_t>> bufs(np1, std::vector<uint32_t>(PU, 0u));
        // round 1's gather (tdec_cont_gather_kernel): q rows from the softbuffer, w or x2 rows from the source pairs
        for (size_t p = 0; p < np1; p++)
          for (int lane = 0; lane < mi::LANES; lane++) {
            uint32_t live = 0;
            mi::P2ContSrc src[2] = {};
            for (int h = 0; h < 2; h++) {
              const size_t d = p * 2 * mi::LANES + (size_t)h * mi::LANES + lane;
              if (d >= cont.size()) continue;
              const uint32_t li = cont[d];
              live |= 1u << h;
              const uint32_t g = li / mi::LANES;
              src[h] = {&sb[P.groups[g].sb_off], wms[g].data(),
                        reinterpret_cast<const uint32_t*>(&scr[P.groups[pa[g]].scratch_off]), li % mi::LANES, ph[g]};
            }
            if (!live) continue;
            uint32_t* cscr = bufs[p].data();
            uint32_t* cq = &cscr[(size_t)(4 * K + 8) * mi::LANES];
            for (uint32_t w = 0; w < mi::p2_cont_qwins(K); w++) {
              uint32_t q[3 * mi::BETA_W];
              mi::p2_cont_qwin(src, live, pos, w, q);
              for (int i = 0; i < 3 * mi::BETA_W; i++) cq[(size_t)(3 * mi::BETA_W * w + i) * mi::LANES + lane] = q[i];
            }
            for (uint32_t k = 0; k < K; k++) {
              if (g_store_w) cscr[(size_t)k * mi::LANES + lane] = mi::p2_cont_wrow(src, live, k);
              else cscr[(size_t)(K + k) * mi::LANES + lane] = mi::p2_cont_xrow(src, live, K, k);
            }
          }
        // iterations it0 .. it_end - 1 of every dense pair (tdec_kernel_p2c)
        std::vector<uint32_t> segv((size_t)4 * 64 * mi::P2_CKW * mi::LANES);   // the segmented form's boundary vectors
        auto run_pairs = [&](std::vector<std::vector<uint32_t>>& pb, const std::vector<uint32_t>& list, uint32_t it0,
                             uint32_t it_end) {
          for (size_t p = 0; p < pb.size(); p++) {
            std::vector<uint8_t> cdec((size_t)K * mi::LANES, 0);
            for (int lane = 0; lane < mi::LANES; lane++) {
              uint32_t li[2] = {0, 0};
              mi::TdecArgsP2 a{};
              for (int h = 0; h < 2; h++) {
                const size_t d = p * 2 * mi::LANES + (size_t)h * mi::LANES + lane;
                if (d < list.size()) { li[h] = list[d]; a.live |= 1u << h; }
              }
              if (!a.live) continue;
              if (!(a.live & 2u)) li[1] = li[0];
              a.scr = pb[p].data();
              a.q = a.scr + (size_t)(4 * K + 8) * mi::LANES;
              a.pos = pos; a.pi = &P.kdata[kt.pi_off];
              a.crc8 = crc8; a.crc8b = crc8b;
              a.dec = cdec.data();
              for (int h = 0; h < 2; h++) {
                emu_p2_out(a, h, payload, P.lanes[li[h]]);
                a.F[h] = P.lanes[li[h]].F;
              }
              a.K = K; a.max_its = max_its; a.early_stop = 1;
              a.cont_w = it0 > 1 || g_store_w;
              a.it0 = it0; a.it_end = it_end;
              mi::TdecP2ExecHost ex;
              mi::TdecP2Result r{};
              if (g_seg && it0 > 1) {
                // tdec.hip tdec_kernel_p2s: the segments of one lane in turn, fix-up rounds until nothing changes
                const size_t vw = (size_t)g_seg * mi::P2_CKW * mi::LANES;
                mi::P2SegVecs V{&segv[0], &segv[vw], &segv[2 * vw], &segv[3 * vw]};
                mi::p2s_half_host<false>(a, lane, (uint32_t)g_seg, V);
                mi::p2s_half_host<true>(a, lane, (uint32_t)g_seg, V);
                uint32_t tbp[2] = {0u, 0u};
                const uint32_t ok = mi::tdec_p2_check(a, lane, a.live, tbp);
                for (int h = 0; h < 2; h++) r.its[h] = it0 + 1, r.crc_ok[h] = (ok >> h) & 1u, r.tb_part[h] = tbp[h];
              } else {
                // tdec.hip launch_tdec_cont: 4-step checkpoints in the rounds after the first
                r = it0 > 1 ? mi::tdec_p2_lane<true, mi::P2C_CKS_LATE>(a, lane, ex)
                            : mi::tdec_p2_lane<true, mi::P2C_CKS>(a, lane, ex);
              }
              for (int h = 0; h < 2; h++) {
                if (!((a.live >> h) & 1u)) continue;
                cits[li[h]] = r.its[h];
                ccrc[li[h]] = r.crc_ok[h];
                ctbp[li[h]] = r.tb_part[h];
              }
            }
          }
        };
        if (!g_rounds) {
          run_pairs(bufs, cont, 1, max_its);
          continue;
        }
        // re-compaction rounds (tdec.hip launch_tdec_cont): one iteration each, the code blocks still failing
        // gathered -- here in reverse slot order, so again with new partners -- into fewer dense pairs
        run_pairs(bufs, cont, 1, 2);
        for (uint32_t it = 2; it < max_its; it++) {
          std::vector<uint32_t> next, srcs;
          for (size_t d = cont.size(); d-- > 0;)
            if (!ccrc[cont[d]]) { next.push_back(cont[d]); srcs.push_back((uint32_t)d); }
          g_round_cbs += next.size();
          const size_t np = (next.size() + 2 * mi::LANES - 1) / (2 * mi::LANES);
          std::vector<std::vector<uint32_t>> nb(np, std::vector<uint32_t>(PU, 0u));
          for (size_t p = 0; p < np; p++)   // tdec_cont_gather2_kernel
            for (int lane = 0; lane < mi::LANES; lane++) {
              uint32_t live = 0;
              mi::P2ContSrc src[2] = {};
              for (int h = 0; h < 2; h++) {
                const size_t d = p * 2 * mi::LANES + (size_t)h * mi::LANES + lane;
                if (d >= next.size()) continue;
                const uint32_t e = srcs[d];
                live |= 1u << h;
                src[h].scr = bufs[e / (2 * mi::LANES)].data();
                src[h].ls = e % mi::LANES;
                src[h].hs = (e / mi::LANES) & 1u;
              }
              if (!live) continue;
              for (uint32_t r = 0; r < K; r++) nb[p][(size_t)r * mi::LANES + lane] = mi::p2_cont_drow(src, live, r);
              for (uint32_t r = 0; r < 3 * (K + 4); r++) {
                const size_t row = (size_t)(4 * K + 8) + r;
                nb[p][row * mi::LANES + lane] = mi::p2_cont_drow(src, live, row);
              }
            }
          run_pairs(nb, next, it, it + 1);
          cont.swap(next);
          bufs.swap(nb);
        }
      }
    }
  }
  for (const MiGroupDesc& g : P.groups) {
    if (g_x == 3 && g_q16) break;
    float* sbg = &sb[g.sb_off];
    uint8_t* map = reinterpret_cast<uint8_t*>(sbg + mi::sb_map_off(g.Ncb));
    for (uint32_t p = 0; p < g.Ncb; p++) mi::rm_combine_row(&P.lanes[g.lane0], P.kdata.data(), e.data(), sbg, g.Ncb, p,
                                                              &P.kdata[P.ktabs[g.ktab].ipos_off]);
    const MiKTab& kt = P.ktabs[g.ktab];
    std::vector<uint32_t> wm(g.K / mi::BETA_W + 1);
    for (uint32_t w = 0; w < wm.size(); w++) wm[w] = mi::tdec_window_mask(map, &P.kdata[kt.pos_off], w);
    int16_t* q16 = reinterpret_cast<int16_t*>(&scr[g.scratch_off]) + mi::q16_elem_off(g.K);
    for (int lane = 0; lane < mi::LANES; lane++) {
      const uint32_t li = g.lane0 + lane;
      const MiLaneDesc& ld = P.lanes[li];
      if (!ld.valid) continue;
      mi::TdecArgs a;
      a.sb = sbg;
      a.wm = wm.data();
      a.zrow = g.Ncb;
      a.q16 = q16;
      a.pos = &P.kdata[kt.pos_off];
      a.pi = &P.kdata[kt.pi_off];
      a.crc_a = &P.kdata[kt.crca_off];
      a.crc_b = &P.kdata[kt.crcb_off];
      a.crc8 = crc8;
      a.scr = &scr[g.scratch_off];
      a.dec = &dec[g.dec_off];
      a.cb_bytes = &cbb[(size_t)li * mi::CB_BYTES_STRIDE];
      a.K = g.K; a.F = ld.F; a.max_its = max_its; a.early_stop = 1; a.crc24a = ld.crc24a;
      mi::TdecLaneResult r = g_win && g_q16 ? emu_win_cb(g, kt, ld, sbg, P.kdata.data(), lane, max_its, a.cb_bytes)
                           : g_x ? (g_q16 ? emu_lane_x<true>(a, lane) : emu_lane_x<false>(a, lane))
                           : g_q16 ? mi::tdec_lane<true>(a, lane) : mi::tdec_lane<false>(a, lane);
      cits[li] = r.its;
      ccrc[li] = r.crc_ok;
      ctbp[li] = r.tb_part;
    }
  }
  for (uint32_t t = 0; t < n; t++) {
    const MiTbDesc& tb = P.tbs[t];
    const uint32_t* lanes = &P.cb_list[tb.cb_list];
    std::vector<uint8_t> buf;
    for (uint32_t r = 0; r < tb.C; r++) {
      const uint8_t* src = &cbb[(size_t)lanes[r] * mi::CB_BYTES_STRIDE + (r == 0 ? tb.F / 8 : 0)];
      buf.insert(buf.end(), src, src + mi::tb_cb_nbytes(tb, r));
    }
    if (!(g_x == 3 && g_q16)) memcpy(payload + tb.pay_off, buf.data(), tb.tbs / 8);   // p2: written in place
    // TB CRC from the decoder's per-code-block partial registers (tb_kernel's formulation)
    uint32_t crc = 0;
    for (uint32_t r = 0; r < tb.C; r++) crc ^= mi::tb_crc_term(tb, r, ctbp[lanes[r]]);
    tb_ok[t] = crc == 0;
    uint32_t its = 0;
    for (uint32_t r = 0; r < tb.C; r++) its = cits[lanes[r]] > its ? cits[lanes[r]] : its;
    tb_its[t] = its;
  }
  if (cb_its) memcpy(cb_its, cits.data(), cits.size() * 4);
  return 0;
}

extern "C" size_t emu_payload_offset(const mi_dl_sf_cfg_t* cfgs, uint32_t n, uint32_t sf) {
  mi::Plan P;
  if (P.build(cfgs, n, true)) return 0;
  return P.tbs[sf].pay_off;
}

// The packed decoder's trellis start (tdec_p2_body.h header, p2.h tadd_a): the LLRs of steps 0..2 taken from the start
// state with the saturating alpha adds and no masking of the unreachable states, against the float recursion with -inf
// (the oracle's semantics, oracle/o_fec.c), at adversarial magnitudes -- inputs drawn at the quantiser's clamps half of
// the time and beta vectors from backward recursions over such inputs (the running beta of phase 2: 0..3 unnormalised
// steps after a window normalisation).  ninf: the start value of the unreachable alpha states (the product's is
// Metric<P2>::ninf_alpha(), -32768; a weaker one must fail, which shows the draws reach the margin).  Returns the number
// of (trial, step, half) LLRs -- of llr_step and of alpha_step -- that differ.
extern "C" uint64_t emu_p2_start_llr_check(uint64_t seed, uint32_t trials, int ninf) {
  uint64_t st = seed | 1u, bad = 0;
  auto rnd = [&]() {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(st >> 33);
  };
  auto pick = [&](int lim) {
    const uint32_t r = rnd();
    if (r & 1u) return (r & 2u) ? lim : -lim;
    return (int)(rnd() % (uint32_t)(2 * lim + 1)) - lim;
  };
  const int XS = 1535, XP = (int)mi::I16_CI;   // DEC2's systematic clamp (DEC1: 511 + 1023), the parity quantiser
  for (uint32_t t = 0; t < trials; t++) {
    float bf[2][8], xsf[2][3], xpf[2][3];
    for (int h = 0; h < 2; h++) {
      for (int s = 0; s < 8; s++) bf[h][s] = 0.f;
      const int n = 4 + 4 * (int)(rnd() % 4), extra = (int)(rnd() % 4);
      for (int i = 0; i < n + extra; i++) {
        float nb[8];
        mi::beta_step<false>(bf[h], (float)pick(XS), (float)pick(XP), nb);
        for (int s = 0; s < 8; s++) bf[h][s] = nb[s];
        if (i < n && (i & 3) == 3) mi::norm8<true>(bf[h]);
      }
      for (int k = 0; k < 3; k++) {
        xsf[h][k] = (float)pick(XS);
        xpf[h][k] = (float)pick(XP);
      }
    }
    mi::P2 bp[8], ap[8];
    float af[2][8];
    for (int s = 0; s < 8; s++) {
      bp[s] = mi::p2_make((int)bf[0][s], (int)bf[1][s]);
      ap[s] = s ? mi::p2_make(ninf, ninf) : mi::Metric<mi::P2>::zero();
      for (int h = 0; h < 2; h++) af[h][s] = s ? -INFINITY : 0.f;
    }
    for (int k = 0; k < 3; k++) {
      const mi::P2 xs = mi::p2_make((int)xsf[0][k], (int)xsf[1][k]), xp = mi::p2_make((int)xpf[0][k], (int)xpf[1][k]);
      const mi::P2 lp = mi::llr_step(ap, bp, xs, xp);
      mi::P2 ap2[8];
      for (int s = 0; s < 8; s++) ap2[s] = ap[s];
      const mi::P2 lp2 = mi::alpha_step<false>(ap2, bp, xs, xp);
      for (int h = 0; h < 2; h++) {
        float a2[8];
        for (int s = 0; s < 8; s++) a2[s] = af[h][s];
        const float lf = mi::alpha_step<false>(a2, bf[h], xsf[h][k], xpf[h][k]);
        const int lo = h ? mi::p2_hi(lp) : mi::p2_lo(lp), lo2 = h ? mi::p2_hi(lp2) : mi::p2_lo(lp2);
        bad += (float)lo != lf;
        bad += (float)lo2 != lf;
      }
      // both recursions one step on (the next step's alpha), the reachable states checked on the way
      mi::alpha_fwd<false>(ap, xs, xp);
      for (int h = 0; h < 2; h++) {
        mi::alpha_fwd<false>(af[h], xsf[h][k], xpf[h][k]);
        for (int s = 0; s < 8; s++)
          if (af[h][s] != -INFINITY) bad += (float)(h ? mi::p2_hi(ap[s]) : mi::p2_lo(ap[s])) != af[h][s];
      }
      // and the beta of the next (lower) step from this one's inputs, as phase 2 walks backwards -- kept as drawn: any
      // vector of bounded spread stands for beta_{k+1}
    }
  }
  return bad;
}
