// engine.cpp -- batch planner, HBM workspace and kernel launch sequence (see engine.h).
//
// Planning happens once per batch (or once per TTI with cached tables for the per-TTI srsLTE
// API): resource-element lists, scrambling words, CRS tables, code-block segmentation, rate
// matching splits and the grouping of code blocks into 64-lane wavefront groups of equal K.
// run() only enqueues kernels on the caller's stream, so it can be captured in a HIP graph.
#include "engine.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>

#include "kernels.h"

namespace mi {

bool hip_ok(hipError_t e, const char* what) {
  if (e == hipSuccess) return true;
  set_error(std::string(what) + ": " + hipGetErrorString(e));
  return false;
}

bool DevBuf::ensure(size_t n) {
  if (n <= bytes && p && !view) return true;
  release();
  size_t a = (n + 255) & ~(size_t)255;
  if (a == 0) a = 256;
  if (!hip_ok(hipMalloc(&p, a), "hipMalloc")) { p = nullptr; bytes = 0; return false; }
  bytes = a;
  return true;
}
void DevBuf::release() {
  if (p && !view) (void)hipFree(p);
  p = nullptr;
  bytes = 0;
  view = false;
}

namespace {
int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
}  // namespace

Engine::Engine() {
  opts.tdec_x = env_int("MI_TDEC_X", -1);
  opts.compact = env_int("MI_TDEC_COMPACT", -1);
  opts.store_w = env_int("MI_TDEC_STORE_W", -1);
  opts.rounds = env_int("MI_TDEC_ROUNDS", -1);
  opts.seg = env_int("MI_TDEC_SEG", -1);
  if (opts.seg != -1 && opts.seg != 0 && opts.seg != 4 && opts.seg != 8) {
    // an A/B run must measure the schedule it asked for: an unsupported value is reported and ignored
    fprintf(stderr, "srsue_amd: MI_TDEC_SEG=%d is not 0 (off), 4 or 8: ignored (automatic)\n", opts.seg);
    opts.seg = -1;
  }
  opts.win_threads = (uint32_t)std::max(0, env_int("MI_TDEC_WIN_THREADS", 0));
  plan.rm_direct_on = env_int("MI_RM_DIRECT", 1) != 0;
  plan.xcd_queues = env_int("MI_RM_XCDQ", 1) != 0;
  // the SIMD count the turbo schedule is chosen by, once per engine (on the device current at creation)
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  simds = 4u * (uint32_t)cus;
}

Engine::~Engine() {
  if (cont_ev) {
    (void)hipEventSynchronize(cont_ev);
    (void)hipEventDestroy(cont_ev);
  }
  for (int k = 0; k < NSTAGE; k++) {
    if (stage_done[k]) {
      (void)hipEventSynchronize(stage_done[k]);
      (void)hipEventDestroy(stage_done[k]);
    }
    if (h_stage[k]) (void)hipHostFree(h_stage[k]);
  }
  if (h_cont) (void)hipHostFree(h_cont);
  for (auto& set : ev_sets)
    for (auto& e : set) (void)hipEventDestroy(e);
  if (back_ev) {
    (void)hipEventSynchronize(back_ev);
    (void)hipEventDestroy(back_ev);
  }
  if (split_ev) (void)hipEventDestroy(split_ev);
}

template <class T>
static bool up(DevBuf& b, const std::vector<T>& v, hipStream_t st) {
  if (!b.ensure(sizeof(T) * std::max<size_t>(v.size(), 1))) return false;
  if (v.empty()) return true;
  return hip_ok(hipMemcpyAsync(b.p, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, st), "upload");
}

namespace {
struct Tab { DevBuf* dst; const void* src; size_t bytes; };
size_t tab_span(size_t bytes) { return (std::max<size_t>(bytes, 1) + 255) & ~(size_t)255; }
}  // namespace

// the descriptor tables of the current plan, in arena order
#define MI_ENGINE_TABS(P)                                                                                           \
  auto tab = [](DevBuf& d, const auto& v) { return Tab{&d, v.data(), v.size() * sizeof(v[0])}; };                   \
  const Tab tabs[] = {tab(d_cells, P.cells), tab(d_crs, P.crs), tab(d_pds, P.pds), tab(d_re, P.re_tab),              \
                      tab(d_scr, P.scr_tab), tab(d_sfs, P.sfs), tab(d_lanes, P.lanes), tab(d_lanesrc, P.lane_src),   \
                      tab(d_groups, P.groups), tab(d_ktabs, P.ktabs), tab(d_kdata, P.kdata), tab(d_tbs, P.tbs),      \
                      tab(d_cblist, P.cb_list), tab(d_fftlist, P.fft_list_flat), tab(d_rmitems, P.rm_items),         \
                      tab(d_rmrecs, P.rm_recs), tab(d_pairs, P.pairs), tab(d_rmdir, P.rm_direct)}

int Engine::stage_tables(DevBuf& arena, std::vector<size_t>& offs, hipStream_t st) {
  const Plan& P = plan;
  MI_ENGINE_TABS(P);
  size_t total = 0;
  for (const Tab& t : tabs) total += tab_span(t.bytes);
  // this staging buffer's previous DMA must be done before it is rewritten
  const int k = stage_next;
  stage_next = (stage_next + 1) % NSTAGE;
  if (stage_done[k] && !hip_ok(hipEventSynchronize(stage_done[k]), "stage wait")) return -1;
  if (total > h_stage_bytes[k]) {
    if (h_stage[k]) (void)hipHostFree(h_stage[k]);
    h_stage[k] = nullptr;
    h_stage_bytes[k] = 0;
    if (!hip_ok(hipHostMalloc(&h_stage[k], total, hipHostMallocDefault), "hipHostMalloc tables")) return -1;
    h_stage_bytes[k] = total;
  }
  if (total > arena.bytes || arena.view) {
    if (&arena == &d_tables)
      for (const Tab& t : tabs) t.dst->release();   // views into the old arena
    if (!arena.ensure(total)) return -1;
  }
  offs.clear();
  size_t off = 0;
  for (const Tab& t : tabs) {
    if (t.bytes) memcpy(static_cast<char*>(h_stage[k]) + off, t.src, t.bytes);
    offs.push_back(off);
    off += tab_span(t.bytes);
  }
  if (!stage_done[k] && !hip_ok(hipEventCreateWithFlags(&stage_done[k], hipEventDisableTiming), "event")) return -1;
  return hip_ok(hipMemcpyAsync(arena.p, h_stage[k], total, hipMemcpyHostToDevice, st), "upload tables") &&
                 hip_ok(hipEventRecord(stage_done[k], st), "event")
             ? 0
             : -1;
}

void Engine::bind_tables(const DevBuf& arena, const std::vector<size_t>& offs) {
  const Plan& P = plan;
  MI_ENGINE_TABS(P);
  for (size_t i = 0; i < sizeof(tabs) / sizeof(tabs[0]); i++)
    tabs[i].dst->set_view(static_cast<char*>(arena.p) + offs[i], std::max<size_t>(tabs[i].bytes, 1));
}

int Engine::ensure_work(hipStream_t st, bool alloc_sb) {
  const Plan& P = plan;
  // twiddles per FFT size (double precision on the host)
  bool need_tw = false;
  for (auto& fl : P.fft_lists) need_tw |= !tw_off.count(fl.first);
  if (need_tw) {
    std::vector<float> tw;
    tw_off.clear();
    for (int N : {128, 256, 512, 1024, 1536, 2048}) {
      tw_off[N] = tw.size() / 2;
      for (int t = 0; t < N; t++) {
        tw.push_back((float)cos(-2.0 * M_PI * t / N));
        tw.push_back((float)sin(-2.0 * M_PI * t / N));
      }
    }
    if (!up(d_tw, tw, st) || !hip_ok(hipStreamSynchronize(st), "twiddles")) return -1;
  }
  bool ok = true;
  for (const auto& w : work_set()) ok = ok && w.first->ensure(w.second);
  if (ok && (P.has_pdsch || P.cb_n) && alloc_sb) {
    // the softbuffer arena grows keeping its contents: a re-plan decides per group what is cleared (batch.cpp
    // mi_dl_batch_replan), so the groups whose layout is unchanged keep combining across the reallocation
    const size_t before = d_sb.bytes;
    if (before && P.sb_floats * 4 > before && !d_sb.view) {
      DevBuf grown;
      ok = grown.ensure(P.sb_floats * 4) &&
           hip_ok(hipMemcpyAsync(grown.p, d_sb.p, before, hipMemcpyDeviceToDevice, st), "sb keep") &&
           hip_ok(hipMemsetAsync(grown.as<char>() + before, 0, grown.bytes - before, st), "memset sb tail") &&
           hip_ok(hipStreamSynchronize(st), "sb keep");   // the old arena is freed below
      if (ok) d_sb.swap(grown);
    } else {
      ok = d_sb.ensure(P.sb_floats * 4);
      if (ok && d_sb.bytes != before) ok = hip_ok(hipMemsetAsync(d_sb.p, 0, d_sb.bytes, st), "memset sb");
    }
  }
  return ok ? 0 : -1;
}

// the work buffers of the current plan and their sizes (ensure_work allocates them; work_bytes counts them).  The
// LLR stream (d_e, 360 KB per 20 MHz MCS-28 subframe) is not among them: the default fused demap never writes it, so
// it is allocated on first use (ensure_llr): 4.5 GB less per 12,500-subframe workspace
std::vector<std::pair<DevBuf*, size_t>> Engine::work_set() {
  const Plan& P = plan;
  const size_t nsf = std::max<size_t>(P.sfs.size(), 1);
  std::vector<std::pair<DevBuf*, size_t>> w{{&d_grid, P.grid_elems * 8}, {&d_ce, P.ce_elems * 8}, {&d_metrics, nsf * 5 * 4}};
  if (P.has_pdsch || P.cb_n) {
    w.insert(w.end(), {{&d_wm, P.groups.size() * WM_STRIDE * 4}, {&d_scratch, P.scratch_floats * 4},
                       {&d_dec, P.dec_bytes}, {&d_cbbytes, (size_t)P.lanes.size() * CB_BYTES_STRIDE},
                       {&d_cbits, P.lanes.size() * 4}, {&d_cbcrc, P.lanes.size() * 4}, {&d_cbtbp, P.lanes.size() * 4},
                       {&d_payload, P.payload_bytes}, {&d_tbok, nsf * 4}, {&d_tbits, nsf * 4}});
    if (tdec_compact()) {
      const uint32_t np = cont_max_pairs();
      w.insert(w.end(), {{&d_cont, (3 * P.lanes.size() + 2) * 4}, {&d_cscr, (size_t)np * cont_pair_u32() * 4},
                         {&d_cdec, (size_t)np * P.groups[0].K * LANES}});
    }
  }
  return w;
}

bool Engine::ensure_llr() { return d_e.ensure(plan.e_floats * 4); }

size_t Engine::work_bytes(bool with_sb, bool with_llr) {
  auto al = [](size_t n) { return std::max<size_t>((n + 255) & ~(size_t)255, 256); };   // DevBuf::ensure
  size_t t = 0;
  for (const auto& w : work_set()) t += al(w.second);
  if (plan.has_pdsch || plan.cb_n) {
    if (with_sb) t += al(plan.sb_floats * 4);
    if (with_llr) t += al(plan.e_floats * 4);
  }
  return t;
}

int Engine::upload(hipStream_t st, bool alloc_sb) {
  // a plain plan.build() over an active memo entry overwrote that entry's (swapped-in) plan: drop the entry
  if (memo_active >= 0) {
    if (hipStreamSynchronize(st) != hipSuccess) {
      set_error("upload: an earlier launch on the stream failed");
      return -1;
    }
    memo.erase(memo.begin() + memo_active);
    memo_active = -1;
  }
  std::vector<size_t> offs;
  if (stage_tables(d_tables, offs, st)) return -1;
  bind_tables(d_tables, offs);
  if (ensure_work(st, alloc_sb)) return -1;
  // per-lane outputs: padding lanes (a group's unused lanes) are never written by a decoder, so they read 0 in
  // every batch plan, a re-planned workspace included (the kernels overwrite every valid lane's entry each run)
  if (plan.lanes.size() && (plan.has_pdsch || plan.cb_n))
    return hip_ok(hipMemsetAsync(d_cbits.p, 0, plan.lanes.size() * 4, st), "memset cb its") &&
                   hip_ok(hipMemsetAsync(d_cbcrc.p, 0, plan.lanes.size() * 4, st), "memset cb crc")
               ? 0
               : -1;
  return 0;
}

int Engine::plan_memo(const mi_dl_sf_cfg_t* cfgs, uint32_t n, bool with_pdsch, hipStream_t st) {
  std::string key(reinterpret_cast<const char*>(cfgs), sizeof(mi_dl_sf_cfg_t) * n);
  key.push_back(with_pdsch ? 'P' : 'F');
  // park the active entry's plan back in its slot
  if (memo_active >= 0) std::swap(static_cast<PlanData&>(plan), memo[(size_t)memo_active]->plan);
  memo_active = -1;
  int hit = -1;
  for (size_t i = 0; i < memo.size(); i++)
    if (memo[i]->key == key) { hit = (int)i; break; }
  if (hit < 0) {
    if (plan.build(cfgs, n, with_pdsch)) return -1;
    if (memo.size() >= MEMO_MAX) {   // evict the least recently used entry
      size_t lru = 0;
      for (size_t i = 1; i < memo.size(); i++)
        if (memo[i]->used < memo[lru]->used) lru = i;
      // its arena may still be read by this stream's kernels
      if (hipStreamSynchronize(st) != hipSuccess) {
        set_error("plan memo: an earlier launch on the stream failed");
        return -1;
      }
      memo.erase(memo.begin() + (ptrdiff_t)lru);
    }
    memo.push_back(std::make_unique<PlanMemo>());
    hit = (int)memo.size() - 1;
    PlanMemo& e = *memo[(size_t)hit];
    e.key = key;
    if (stage_tables(e.arena, e.offs, st)) { memo.pop_back(); return -1; }
    std::swap(static_cast<PlanData&>(plan), e.plan);   // park, then activate below
  }
  PlanMemo& e = *memo[(size_t)hit];
  std::swap(static_cast<PlanData&>(plan), e.plan);
  memo_active = hit;
  e.used = ++memo_clock;
  bind_tables(e.arena, e.offs);
  return ensure_work(st, false);
}

int Engine::run(const void* d_iq, hipStream_t st, uint32_t mask, float* sb_override, const hipStream_t* back) {
  const Plan& P = plan;
  // after a split run, any run of this batch (split or not, on any stream) waits for that run's back end: it rewrites
  // what the back end reads
  if (!order_after_split(st)) return -1;
  if (back && ((!split_ev && !hip_ok(hipEventCreateWithFlags(&split_ev, hipEventDisableTiming), "event")) ||
               (!back_ev && !hip_ok(hipEventCreateWithFlags(&back_ev, hipEventDisableTiming), "event"))))
    return -1;
  last_stream = back ? *back : st;
  // the stream the next launches go to: st, then (split run) the back-end stream from the hand-off on
  hipStream_t cur = st;
  const bool prof = flags & MI_DL_FLAG_PROFILE;
  hipEvent_t* ev = nullptr;
  if (prof) {
    if (ev_used == ev_sets.size()) {
      std::vector<hipEvent_t> set(MI_DL_NSTAGES + 1);
      for (auto& e : set)
        if (!hip_ok(hipEventCreate(&e), "event")) return -1;
      ev_sets.push_back(set);
    }
    ev = ev_sets[ev_used++].data();
  }
  bool ok = true;
  auto mark = [&](int i) {
    if (prof) ok = hip_ok(hipEventRecord(ev[i], cur), "event") && ok;
  };
  // split run: the back-end stream waits for the front end, and the launches from here on go to it
  auto handoff = [&]() {
    if (!back) return;
    ok = hip_ok(hipEventRecord(split_ev, st), "record") && hip_ok(hipStreamWaitEvent(*back, split_ev, 0), "wait") && ok;
    cur = *back;
  };
  const uint32_t nsf = (uint32_t)P.sfs.size();
  // compact channel estimates (MI_DL_FLAG_CE_COMPACT): only when this run both writes and consumes them
  // (channel estimation and the fused demap in one run), nothing else reads the full estimates, and no
  // code block repeats LLRs (the single-LLR repetition path reads full estimates)
  const uint32_t full = (1u << MI_DL_STAGE_CHEST) | (1u << MI_DL_STAGE_DEMAP) | (1u << MI_DL_STAGE_RM);
  const bool compact = (flags & MI_DL_FLAG_CE_COMPACT) && !(flags & MI_DL_FLAG_KEEP_LLR) && P.has_pdsch &&
                       (mask & full) == full && !P.rm_rep;
  // the demap stage (alone or fused into rate de-matching) reads the estimates; without a chest stage in
  // this run they must be full ones
  if (P.has_pdsch && ce_compact && !(mask & (1u << MI_DL_STAGE_CHEST)) && (mask & (1u << MI_DL_STAGE_DEMAP))) {
    set_error("the channel estimates are in compact form (MI_DL_FLAG_CE_COMPACT): re-run with the CHEST stage");
    return -1;
  }
  mark(0);
  if (mask & (1u << MI_DL_STAGE_OFDM)) {
    for (size_t i = 0; i < P.fft_lists.size(); i++) {
      const int N = P.fft_lists[i].first;
      launch_ofdm_rx(N, d_iq, (flags & MI_DL_FLAG_IQ_SC16) != 0, d_grid.as<float2>(), d_sfs.as<MiSfDesc>(),
                     d_fftlist.as<uint32_t>() + P.fft_list_off[i], (uint32_t)P.fft_lists[i].second.size(),
                     d_tw.as<float2>() + tw_off[N], P.fft_W[i], st);
    }
  }
  mark(1);
  if (mask & (1u << MI_DL_STAGE_CHEST))
    launch_chest(d_grid.as<float2>(), d_ce.as<float2>(), d_sfs.as<MiSfDesc>(), d_cells.as<MiCellDesc>(),
                 d_crs.as<float2>(), d_metrics.as<float>(), nsf, st, compact);
  if (mask & (1u << MI_DL_STAGE_CHEST)) ce_compact = compact;
  mark(2);
  if (P.has_pdsch) {
    float* sb = sb_override ? sb_override : d_sb.as<float>();
    // fused demap -> rate de-matching unless the caller keeps the LLR stream (or supplies it)
    const bool fuse = (mask & (1u << MI_DL_STAGE_DEMAP)) && (mask & (1u << MI_DL_STAGE_RM)) &&
                      !(flags & MI_DL_FLAG_KEEP_LLR);
    if (!fuse && (mask & ((1u << MI_DL_STAGE_DEMAP) | (1u << MI_DL_STAGE_RM))) && !ensure_llr()) return -1;
    if ((mask & (1u << MI_DL_STAGE_DEMAP)) && !fuse)
      launch_demap(d_grid.as<float2>(), d_ce.as<float2>(), d_e.as<float>(), d_sfs.as<MiSfDesc>(),
                   d_pds.as<MiPdschDesc>(), d_cells.as<MiCellDesc>(), d_re.as<uint32_t>(), d_scr.as<uint32_t>(), nsf,
                   P.max_units, noise, st);
    mark(3);
    // the direct groups' row maps (Plan::rm_direct) before the combine kernel stages their chunks -- only in a
    // run that rate de-matches (a run without RM must leave the softbuffer, maps included, untouched)
    if (mask & (1u << MI_DL_STAGE_RM))
      launch_rm_direct_maps(sb, d_kdata.as<uint32_t>(), reinterpret_cast<const MiRmDirect*>(d_rmdir.as<uint32_t>()),
                          (uint32_t)(P.rm_direct.size() / 8), st);
    if (fuse)
      launch_rm_fused(d_grid.as<float2>(), d_ce.as<float2>(), d_lanesrc.as<MiLaneSrc>(), d_re.as<uint32_t>(),
                      d_scr.as<uint32_t>(), noise, sb, d_groups.as<MiGroupDesc>(), d_lanes.as<MiLaneDesc>(),
                      d_ktabs.as<MiKTab>(), d_kdata.as<uint32_t>(), (uint32_t)P.groups.size(), P.max_ncb, P.unit_kind,
                      rm_items(),
                      rm_recs(), P.rm_busy, P.rm_dbusy, (uint32_t)P.rm_items.size(), compact, st);
    else if (mask & (1u << MI_DL_STAGE_RM))
      launch_rm_combine(d_e.as<float>(), sb, d_groups.as<MiGroupDesc>(), d_lanes.as<MiLaneDesc>(),
                        d_ktabs.as<MiKTab>(), d_kdata.as<uint32_t>(), (uint32_t)P.groups.size(), P.max_ncb,
                        rm_items(), rm_recs(), P.rm_busy, P.rm_dbusy, (uint32_t)P.rm_items.size(), st);
    mark(4);
    handoff();
    if (mask & (1u << MI_DL_STAGE_TDEC)) ok = launch_turbo(sb, cur) && ok;
    mark(5);
    if (mask & (1u << MI_DL_STAGE_TB))
      launch_tb(d_cbbytes.as<uint8_t>(), d_payload.as<uint8_t>(), d_tbok.as<uint32_t>(), d_tbits.as<uint32_t>(),
                d_cbits.as<uint32_t>(), d_cbtbp.as<uint32_t>(), d_tbs.as<MiTbDesc>(), (uint32_t)P.tbs.size(),
                d_cblist.as<uint32_t>(), d_kdata.as<uint32_t>(), !tb_copied, cur);
    mark(6);
  } else {
    for (int i = 3; i <= 4; i++) mark(i);
    handoff();
    for (int i = 5; i <= 6; i++) mark(i);
  }
  if (back) {
    back_pending = hip_ok(hipEventRecord(back_ev, cur), "record");
    ok = back_pending && ok;
  }
  return hip_ok(hipGetLastError(), "launch") && ok ? 0 : -1;
}

int Engine::run_codeblocks(const float* d_in, hipStream_t st) {
  const Plan& P = plan;
  last_stream = st;
  const bool prof = flags & MI_DL_FLAG_PROFILE;
  hipEvent_t* ev = nullptr;
  if (prof) {
    if (ev_used == ev_sets.size()) {
      std::vector<hipEvent_t> set(MI_DL_NSTAGES + 1);
      for (auto& e : set)
        if (!hip_ok(hipEventCreate(&e), "event")) return -1;
      ev_sets.push_back(set);
    }
    ev = ev_sets[ev_used++].data();
  }
  bool ok = true;
  auto mark = [&](int i) {
    if (prof) ok = hip_ok(hipEventRecord(ev[i], st), "event") && ok;
  };
  for (int i = 0; i <= MI_DL_STAGE_RM; i++) mark(i);
  launch_cb_scatter(d_in, d_sb.as<float>(), d_groups.as<MiGroupDesc>(), d_ktabs.as<MiKTab>(), d_kdata.as<uint32_t>(),
                    (uint32_t)P.groups.size(), P.cb_K, P.cb_n, st);
  mark(MI_DL_STAGE_TDEC);
  ok = launch_turbo(d_sb.as<float>(), st) && ok;
  mark(MI_DL_STAGE_TB);
  mark(MI_DL_NSTAGES);
  return hip_ok(hipGetLastError(), "launch") && ok ? 0 : -1;
}

bool Engine::use_win() const {
  if (!q16()) return false;   // the float decoder is not shift-invariant: lane-per-code-block only
  if (flags & MI_DL_FLAG_TDEC_WIN) return true;
  if (flags & MI_DL_FLAG_TDEC_LANE) return false;
  return plan.n_cb <= MI_TDEC_WIN_AUTO_CBS;
}

// lane-per-code-block decoder in the crossed schedule (two wavefronts per group, tdec_body.h)
// Lane form schedule.  Crossed (two wavefronts per group, tdec_body.h) by default: the decode time is
// each wavefront's serial chain (profiles/r1/sfsweep).  Its register form holds 4 waves per SIMD; when
// the batch's 2 G wavefronts do not fit at 4 but fit at 5 per SIMD (the headline: 2,540 groups), the
// recompute form (92 VGPRs) keeps them all resident in one round (-6 % at the headline; at lower
// occupancy its extra VALU makes it slower than the register form).  MI_DL_FLAG_TDEC_LANE alone = one
// wavefront per group; MI_DL_FLAG_TDEC_X = crossed; Opts::tdec_x (MI_TDEC_X at creation, A/B) forces a form.
int Engine::tdec_crossed() const {
  const uint64_t waves = 2ull * plan.groups.size();
  const int form = (q16() && waves > 4ull * simds && waves <= 5ull * simds) ? 2 : 1;
  if (opts.tdec_x >= 0) return opts.tdec_x;   // A/B
  if (flags & MI_DL_FLAG_TDEC_P2) return q16() ? 3 : 1;
  if (flags & MI_DL_FLAG_TDEC_XR) return q16() ? 2 : 1;
  if (flags & MI_DL_FLAG_TDEC_X) return form;
  if (flags & MI_DL_FLAG_TDEC_LANE) return 0;
  if (!q16()) return waves < 4ull * simds ? 1 : 0;   // float decoder: crossed below 2 groups per SIMD (measured)
  // packed int16, two code blocks per lane: half the VALU per code block but half the wavefronts, so it
  // pays once its wavefronts (2 per group pair) still cover every SIMD -- the headline (2.5 per SIMD:
  // 7.68 vs 7.95 ms) and configs[0] (1 per SIMD, 8 iterations: 35.2 vs 36.6 ms); below that the per-wave
  // chain dominates (configs[2], 0.2 per SIMD: 8.5 vs 6.1 ms; profiles/r2/ab_p2)
  if (2ull * (plan.pairs.size() / 2) >= simds) return 3;
  return form;
}

bool Engine::tdec_compact() const {
  const Plan& P = plan;
  if (P.groups.empty() || use_win() || !q16() || tdec_crossed() != 3 || !early_stop || max_its < 2) return false;
  if (opts.compact == 0) return false;   // A/B
  for (size_t g = 0; g < P.groups.size(); g++)
    if (P.groups[g].K != P.groups[0].K || P.groups[g].lane0 != g * LANES) return false;
  return true;
}
size_t Engine::cont_pair_u32() const {
  const uint32_t K = plan.groups.empty() ? 0 : plan.groups[0].K;
  return ((size_t)(7 * K + 20) * LANES + 63) & ~(size_t)63;   // w, llr1, checkpoints, q rows (tdec_p2_body.h)
}
uint32_t Engine::cont_max_pairs() const { return (uint32_t)((plan.lanes.size() + 2 * LANES - 1) / (2 * LANES)); }

// turbo stage: the latency form (one workgroup per code block) or the lane-per-code-block wavefronts
bool Engine::launch_turbo(float* sb, hipStream_t st) {
  const Plan& P = plan;
  tb_copied = false;
  if (use_win()) {
    uint32_t kmax = 0;
    for (const MiGroupDesc& g : P.groups) kmax = std::max(kmax, g.K);
    // threads per code block: segments of >= ~16 trellis steps (fewer fix-up rounds), at most 256
    uint32_t th = win_threads ? win_threads : opts.win_threads;
    if (!th) th = kmax >= 4096 ? 256 : kmax >= 1024 ? 128 : 64;
    launch_tdec_win(sb, d_cbbytes.as<uint8_t>(), d_cbits.as<uint32_t>(), d_cbcrc.as<uint32_t>(), d_cbtbp.as<uint32_t>(),
                    d_groups.as<MiGroupDesc>(), d_lanes.as<MiLaneDesc>(), d_ktabs.as<MiKTab>(), d_kdata.as<uint32_t>(),
                    (uint32_t)P.lanes.size(), kmax, max_its, early_stop, th, st);
    return true;
  }
  const bool p2 = tdec_crossed() == 3 && q16();
  // compaction needs its buffers (ensure_work sized them for this plan and max_its); without them the
  // packed decoder runs every iteration itself -- the same results either way
  const bool cont = p2 && tdec_compact() && d_cscr.bytes >= (size_t)cont_max_pairs() * cont_pair_u32() * 4 &&
                    d_cont.bytes >= (3 * P.lanes.size() + 2) * 4 &&
                    d_cdec.bytes >= (size_t)cont_max_pairs() * P.groups[0].K * LANES;
  // (the row masks' kernel also resets the continuation's count: no memset launch between the decoder and its assign)
  launch_rowmask(sb, d_wm.as<uint32_t>(), d_groups.as<MiGroupDesc>(), d_ktabs.as<MiKTab>(), d_kdata.as<uint32_t>(),
                 (uint32_t)P.groups.size(), cont ? d_cont.as<uint32_t>() : nullptr, st);
  if (p2) {
    // PDSCH batches: the decoder writes the payload bytes in place (tb_kernel then only combines the CRCs)
    const bool direct = P.has_pdsch && !P.cb_n;
    tb_copied = direct;
    // The one-iteration first launch stores no extrinsic rows w when few code blocks continue (the continuation
    // re-forms them by re-running iteration 0's DEC2 from gathered x2 rows: 12 KB per code block less for all, about
    // half an iteration more for the continuing ones); when the previous run of this workspace continued more than
    // 2 % of its code blocks (the waterfall), it stores them and the continuation gathers them instead.  Both are
    // exact: only the schedule depends on the history.  Opts::store_w forces (A/B).
    bool store_w = false;
    if (cont) {
      if (!h_cont) {
        static_assert(sizeof(cont_last) / sizeof(cont_last[0]) == CONT_HIST, "one count per recorded round");
        if (!hip_ok(hipHostMalloc(reinterpret_cast<void**>(&h_cont), 4 * CONT_HIST, hipHostMallocDefault), "pinned") ||
            !hip_ok(hipEventCreateWithFlags(&cont_ev, hipEventDisableTiming), "event"))
          return false;
        memset(h_cont, 0, 4 * CONT_HIST);
      }
      // the previous run's count, once its copy has landed (an event query, no wait); until then the last one read
      if (cont_pending && hipEventQuery(cont_ev) == hipSuccess) {
        memcpy(cont_last, h_cont, sizeof(cont_last));
        cont_pending = false;
      }
      store_w = opts.store_w >= 0  ? opts.store_w != 0
                : cont_mode >= 0     ? cont_mode != 0
                                     : (uint64_t)cont_last[0] * 50 > P.lanes.size();
    }
    launch_tdec_p2(sb, d_wm.as<uint32_t>(), d_scratch.as<float>(), d_dec.as<uint8_t>(), d_cbbytes.as<uint8_t>(),
                   d_cbits.as<uint32_t>(), d_cbcrc.as<uint32_t>(), d_cbtbp.as<uint32_t>(), d_groups.as<MiGroupDesc>(),
                   d_lanes.as<MiLaneDesc>(), d_ktabs.as<MiKTab>(), d_kdata.as<uint32_t>(), d_pairs.as<uint32_t>(),
                   (uint32_t)(P.pairs.size() / 2), cont ? 1u : max_its, early_stop, direct ? d_payload.as<uint8_t>() : nullptr,
                   cont && !store_w, st);
    if (cont) {
      // the code blocks still failing after iteration 0, compacted into dense pairs for iterations 1 ..
      // many continuing code blocks (the same history): one iteration per launch, re-compacting the code blocks that
      // still fail between them, so a pair no longer runs until its slowest of 128 code blocks stops (21.5 dB:
      // 379 + 84 + 19 pair-iterations instead of 3 x 379).  Opts::rounds forces (A/B).
      const bool rounds = opts.rounds >= 0 ? opts.rounds != 0 : store_w;
      const size_t ssz = (size_t)LANES * (2 * P.groups[0].K + 8 * (P.groups[0].K / TDEC_CK_MIN + 1));   // plan.cpp
      if (!launch_tdec_cont(sb, d_wm.as<uint32_t>(), d_scratch.as<float>(), 2 * ssz, d_dec.as<uint8_t>(),
                       d_cbbytes.as<uint8_t>(), d_cbits.as<uint32_t>(),
                       d_cbcrc.as<uint32_t>(), d_cbtbp.as<uint32_t>(), d_groups.as<MiGroupDesc>(),
                       d_lanes.as<MiLaneDesc>(), d_kdata.as<uint32_t>(), P.ktabs[P.groups[0].ktab],
                       (uint32_t)P.groups.size(), d_cont.as<uint32_t>(), d_cscr.as<uint32_t>(), d_cdec.as<uint8_t>(),
                       cont_max_pairs(), cont_pair_u32(), P.groups[0].K, max_its,
                       // the gather is grid-stride: when the history continued nothing, a small grid (its 2048
                       // early-exiting workgroups otherwise wait ~1 ms for CU slots behind the other streams' decoders)
                       (cont_mode >= 0 ? cont_mode != 0 : cont_last[0] || cont_last[1]) ? 2048u : 64u,
                       direct ? d_payload.as<uint8_t>() : nullptr, store_w, rounds, cont_pending ? nullptr : h_cont,
                       opts.seg == 4 || opts.seg == 8 ? (uint32_t)opts.seg
                       : opts.seg < 0 && (flags & MI_DL_FLAG_TDEC_SEG) ? 8u : 0u, true, st))
        return false;
      // the copy of the count (skipped while an earlier one is still unread) is complete when cont_ev is
      if (!cont_pending) {
        if (!hip_ok(hipEventRecord(cont_ev, st), "event")) return false;
        cont_pending = true;
      }
    }
    return true;
  }
  launch_tdec(sb, d_wm.as<uint32_t>(), d_scratch.as<float>(), d_dec.as<uint8_t>(), d_cbbytes.as<uint8_t>(),
              d_cbits.as<uint32_t>(), d_cbcrc.as<uint32_t>(), d_cbtbp.as<uint32_t>(), d_groups.as<MiGroupDesc>(),
              d_lanes.as<MiLaneDesc>(), d_ktabs.as<MiKTab>(), d_kdata.as<uint32_t>(), (uint32_t)P.groups.size(),
              max_its, early_stop, q16(), tdec_crossed(), st);
  return true;
}

void Engine::reset_history() {
  if (cont_pending && cont_ev) (void)hipEventSynchronize(cont_ev);
  cont_pending = false;
  memset(cont_last, 0, sizeof(cont_last));
  if (h_cont) memset(h_cont, 0, 4 * CONT_HIST);
}

int Engine::stage_ms(float* ms, uint32_t* nruns) {
  if (!ev_used) { set_error("no profiled run (MI_DL_FLAG_PROFILE)"); return -1; }
  for (int i = 0; i < MI_DL_NSTAGES; i++) ms[i] = 0.f;
  for (size_t r = 0; r < ev_used; r++) {
    hipEvent_t* ev = ev_sets[r].data();
    if (!hip_ok(hipEventSynchronize(ev[MI_DL_NSTAGES]), "event sync")) return -1;
    for (int i = 0; i < MI_DL_NSTAGES; i++) {
      float t = 0.f;
      if (!hip_ok(hipEventElapsedTime(&t, ev[i], ev[i + 1]), "elapsed")) return -1;
      ms[i] += t / (float)ev_used;
    }
  }
  if (nruns) *nruns = (uint32_t)ev_used;
  return 0;
}

}  // namespace mi
