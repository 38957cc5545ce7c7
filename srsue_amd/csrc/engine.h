// engine.h -- batch planner + device workspace + launch sequence of the DL PDSCH receive chain.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "plan.h"

namespace mi {

bool hip_ok(hipError_t e, const char* what);

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  bool view = false;       // points into another allocation (the packed table arena): never freed here
  bool ensure(size_t n);   // grow-only
  void release();
  void set_view(void* ptr, size_t n) { release(); p = ptr; bytes = n; view = true; }
  void swap(DevBuf& o) { std::swap(p, o.p); std::swap(bytes, o.bytes); std::swap(view, o.view); }
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

// Device workspace + launcher.  One per batch or per srslte_ue_dl_t instance.
struct Engine {
  Plan plan;
  uint32_t max_its = 4, early_stop = 1, flags = 0;
  // Schedule overrides for A/B runs and equivalence tests, read from the environment ONCE, when the engine (a batch
  // or a per-TTI instance) is created -- never on the run path.  Every choice they force is exact: results are
  // identical either way.  -1 / 0 = automatic.
  //   MI_TDEC_X        turbo form (0 lane, 1 crossed, 2 crossed recompute, 3 packed pairs)
  //   MI_TDEC_COMPACT  0 = no waterfall compaction;  MI_TDEC_STORE_W / MI_TDEC_ROUNDS  0 / 1 = force
  //   MI_TDEC_WIN_THREADS  latency form: threads per code block;  MI_RM_DIRECT=0 / MI_RM_XCDQ=0 (Plan)
  //   MI_TDEC_SEG=4/8  the waterfall's late rounds segmented over 4 / 8 wavefronts per pair (tdec_kernel_p2s)
  //                    instead of the crossed form; 0 = explicitly off (overrides MI_DL_FLAG_TDEC_SEG); any other
  //                    value is reported on stderr and ignored
  struct Opts {
    int tdec_x = -1, compact = -1, store_w = -1, rounds = -1, seg = -1;
    uint32_t win_threads = 0;
  } opts;
  Engine();
  uint32_t simds = 1024;   // SIMDs of the device (4 per CU), read once at construction: no shared mutable state
  bool q16() const { return (flags & MI_DL_FLAG_TDEC_GEN) == 0; }   // int16 turbo arithmetic (default)
  uint32_t win_threads = 0;   // latency-form turbo: threads per code block (0 = by K)
  bool use_win() const;       // latency-form (segment-parallel) turbo decoder for this plan
  // lane form: 0 one wavefront per group, 1 crossed, 2 crossed (recompute form), 3 crossed with two code
  // blocks per lane (packed int16, tdec_p2_body.h)
  int tdec_crossed() const;
  // waterfall compaction of the packed decoder after iteration 0 (tdec.hip launch_tdec_cont): schedule 3,
  // early stop, max_its > 1, one K (pairs are groups 2j, 2j + 1); MI_TDEC_COMPACT=0 (env, A/B) disables
  bool tdec_compact() const;
  size_t cont_pair_u32() const;   // continuation pair scratch, u32 words
  uint32_t cont_max_pairs() const;
  bool launch_turbo(float* sb, hipStream_t st);   // false: a HIP call failed (mi_last_error)
  bool tb_copied = false;
  // the last turbo stage wrote the payload bytes itself (packed decoder, PDSCH batch)
  // waterfall compaction: the number of continuing code blocks of an earlier run (page-locked, copied back after every
  // compacted run) steers whether the first launch stores its extrinsic rows.  It is read only once cont_ev (recorded
  // after the copy) has completed -- never while the copy may be in flight -- and otherwise the last value read
  // (cont_last) is used: only the schedule depends on it, both forms are exact
  // h_cont[r]: the code blocks continuation round r + 1 decoded (CONT_HIST words); cont_last: the last counts read
  uint32_t* h_cont = nullptr;
  hipEvent_t cont_ev = nullptr;
  bool cont_pending = false;
  uint32_t cont_last[8] = {};
  // the schedule's source (mi_dl_batch_set_tdec_history): -1 = the history above, 0 / 1 = fixed (few continue /
  // waterfall)
  int cont_mode = -1;
  // forget the recorded counts (a pending copy is waited for, so it cannot land in cont_last later)
  void reset_history();
  float noise = 0.01f;   // MMSE regulariser (srsUE passes 0.01: phch_worker.cc:340)
  // descriptor tables
  DevBuf d_cells, d_crs, d_pds, d_re, d_scr, d_sfs, d_lanes, d_lanesrc, d_groups, d_ktabs, d_kdata, d_tbs, d_cblist,
      d_fftlist, d_tw, d_pairs;
  // data buffers
  DevBuf d_grid, d_ce, d_metrics, d_e, d_sb, d_wm, d_scratch, d_dec, d_cbbytes, d_cbits, d_cbcrc, d_cbtbp, d_payload, d_tbok,
      d_tbits, d_cont, d_cscr, d_cdec;
  std::map<int, size_t> tw_off;   // FFT size -> float2 offset in d_tw
  // the plan's descriptor tables, packed 256-B aligned into one page-locked host buffer and copied to
  // one device arena with a single DMA per upload (the per-TTI API re-plans every call)
  DevBuf d_tables;
  DevBuf d_rmitems, d_rmrecs;   // Plan::rm_items, Plan::rm_recs (views into d_tables)
  DevBuf d_rmdir;               // Plan::rm_direct
  const uint32_t* rm_items() const { return plan.rm_items.empty() ? nullptr : d_rmitems.as<uint32_t>(); }
  const uint4* rm_recs() const { return plan.rm_recs.empty() ? nullptr : d_rmrecs.as<uint4>(); }
  // two page-locked staging buffers used in turn, each with the event of its last DMA (waited for before it is
  // rewritten): a re-plan does not wait for the previous one's table upload, which another stream may still have
  // queued behind its kernels (the main thread blocked 7-26 ms per pipelined re-plan)
  static constexpr int NSTAGE = 2;
  void* h_stage[NSTAGE] = {nullptr, nullptr};
  size_t h_stage_bytes[NSTAGE] = {0, 0};
  hipEvent_t stage_done[NSTAGE] = {nullptr, nullptr};
  int stage_next = 0;
  // Per-TTI plan memo (the srsLTE per-TTI API re-plans every call; srsUE cycles through the same few
  // configurations -- one per subframe index and stage): a configuration planned before is re-activated
  // by swapping its parked plan in and pointing the table views at its own device arena, instead of
  // rebuilding and re-uploading the tables.  Entries hold the plan data, the arena and the table offsets.
  struct PlanMemo {
    std::string key;
    PlanData plan;
    DevBuf arena;
    std::vector<size_t> offs;
    uint64_t used = 0;
  };
  std::vector<std::unique_ptr<PlanMemo>> memo;
  int memo_active = -1;
  uint64_t memo_clock = 0;
  static constexpr size_t MEMO_MAX = 32;
  // build + upload of the plan of cfgs unless memoised (alloc_sb = false: the per-TTI API's external
  // softbuffer); 0 on success
  int plan_memo(const mi_dl_sf_cfg_t* cfgs, uint32_t n, bool with_pdsch, hipStream_t st);
  hipStream_t last_stream = nullptr;
  // layout the last channel-estimation stage wrote: true = compact (4 pilot rows per port).  A run that
  // reads the estimates without re-estimating them is rejected while they are compact
  bool ce_compact = false;
  // profiling: one event set per run since the last reset (MI_DL_FLAG_PROFILE)
  std::vector<std::vector<hipEvent_t>> ev_sets;
  size_t ev_used = 0;
  int device = 0;

  ~Engine();
  int upload(hipStream_t st, bool alloc_sb);
  // upload() in parts: the descriptor tables packed into `arena` with one DMA (offsets per table), the
  // table views pointed into an arena, and the work buffers / twiddles sized for the current plan
  int stage_tables(DevBuf& arena, std::vector<size_t>& offs, hipStream_t st);
  void bind_tables(const DevBuf& arena, const std::vector<size_t>& offs);
  int ensure_work(hipStream_t st, bool alloc_sb);
  std::vector<std::pair<DevBuf*, size_t>> work_set();   // the plan's work buffers and sizes (no LLR stream, no sb)
  bool ensure_llr();                                     // the LLR stream d_e, allocated on first use
  // HBM bytes of this plan's work buffers (+ the softbuffer arena, + the LLR stream), as DevBuf::ensure rounds them
  size_t work_bytes(bool with_sb, bool with_llr);
  // split runs (mi_dl_batch_run_split): the front end's hand-off to the back-end stream, and the back end's completion,
  // which the batch's next run or re-plan waits for (the workspace is reused)
  hipEvent_t split_ev = nullptr, back_ev = nullptr;
  bool back_pending = false;
  // enqueue on st a wait for the last split run's back end, if one is pending; false on a HIP error
  bool order_after_split(hipStream_t st) {
    if (!back_pending) return true;
    back_pending = false;
    return hip_ok(hipStreamWaitEvent(st, back_ev, 0), "wait");
  }
  // stage mask bit i = stage i (MI_DL_STAGE_*).  sb_override: external softbuffer arena.  back: the stream of the
  // TDEC and TB stages (split run), nullptr = all on st
  int run(const void* d_iq, hipStream_t st, uint32_t stage_mask, float* sb_override, const hipStream_t* back = nullptr);
  // raw code-block decoding: scatter d into the softbuffer layout, then the turbo kernel
  int run_codeblocks(const float* d_in, hipStream_t st);
  int stage_ms(float* ms, uint32_t* nruns);   // average over the runs since profile_reset()
  void profile_reset() { ev_used = 0; }
};

}  // namespace mi
