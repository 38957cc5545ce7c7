/*
 * mi_dl.h -- batched MI355X LTE downlink PDSCH receiver (C ABI, no torch types).
 *
 * The batched extension SURVEY.md 8b asks for beside the per-TTI srsLTE API of
 * include/srslte/srslte.h: N subframes (IQ resident in HBM) are taken through
 *   OFDM RX -> CRS channel estimation -> equalisation -> soft demap -> descrambling ->
 *   rate de-matching + HARQ combining -> max-log-MAP turbo decoding -> TB CRC -> payload
 * by a fixed sequence of gfx950 kernels on one HIP stream.  The per-subframe work is what
 * srsUE's phch_worker performs per TTI through srslte_ue_dl_decode_fft_estimate and
 * srslte_pdsch_decode_rnti (/root/reference/ue/src/phy/phch_worker.cc:254, :347-348).
 *
 * Multi-GPU: one process per GPU, each with its own batch (subframes are independent; no
 * collective on the data path).  All functions return 0 on success and a negative value on
 * error, like the srsLTE API (SRSLTE_SUCCESS / SRSLTE_ERROR).
 */
#ifndef MI_DL_H
#define MI_DL_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MI_DL_MAX_PRB 110

typedef struct {
  uint32_t cell_id;      /* N_ID^cell */
  uint32_t nof_prb;      /* 6, 15, 25, 50, 75, 100 */
  uint32_t nof_ports;    /* 1 or 2 CRS ports */
  uint32_t sf_idx;       /* 0..9 */
  uint32_t cfi;          /* 1..3 (control symbols) */
  uint32_t tm;           /* 1 = single port, 2 = transmit diversity (SFBC) */
  uint32_t nl_td;        /* N_L used by rate matching for TM2 (36.212 5.1.4.1.2: 2) */
  uint32_t rnti;
  uint32_t rv;           /* redundancy version 0..3 */
  uint32_t tbs;          /* transport block size, bits */
  uint32_t Qm;           /* 2, 4, 6 */
  uint32_t new_tb;       /* 1 = first transmission (softbuffer overwritten), 0 = HARQ combine */
  /* allocated PRBs.  If every entry is 0 or 1, a non-zero entry = PRB used in both slots (localized).
   * Otherwise bit 0 / bit 1 of entry p = PRB p used in slot 0 / slot 1 (distributed VRB, 36.211 6.2.3.2:
   * srslte_ra_dl_grant_t.prb_idx[0] / [1]); the RE gather follows 36.211 6.3.5 per slot. */
  uint8_t  prb_mask[MI_DL_MAX_PRB];
} mi_dl_sf_cfg_t;

/* stages, for mi_dl_batch_stage_ms */
enum { MI_DL_STAGE_OFDM = 0, MI_DL_STAGE_CHEST, MI_DL_STAGE_DEMAP, MI_DL_STAGE_RM, MI_DL_STAGE_TDEC,
       MI_DL_STAGE_TB, MI_DL_NSTAGES };

/* buffers that can be downloaded for parity checks */
enum { MI_DL_BUF_GRID = 0, MI_DL_BUF_CE, MI_DL_BUF_LLR, MI_DL_BUF_PAYLOAD, MI_DL_BUF_TB_CRC, MI_DL_BUF_TB_ITS,
       MI_DL_BUF_METRICS, MI_DL_BUF_CB_ITS, MI_DL_BUF_CB_CRC,
       MI_DL_BUF_SOFTBUFFER /* the batch's HARQ softbuffer arena (group layout, dl_common.h sb_group_floats) */ };

#define MI_DL_FLAG_PROFILE 1u  /* record HIP events around every stage of every run */
/* turbo decoder arithmetic.  Default (and MI_DL_FLAG_TDEC_I16): the int16 decoder of srsLTE's SSE
 * design (srslte_tdec_sse, what srsUE runs on SSE4.1 hosts: reference CMakeLists.txt:58-68 adds
 * -DLV_HAVE_SSE), fixed-point contract in DESIGN.md 4.5.  MI_DL_FLAG_TDEC_GEN: the float
 * srsLTE-gen decoder (srslte_tdec_gen, the non-SSE build).  Both are bit-exact to their oracle. */
#define MI_DL_FLAG_TDEC_I16 2u
#define MI_DL_FLAG_TDEC_GEN 4u
/* IQ input in UHD's sc16 wire format (int16 I/Q, fc32 = sc16 / 32768) instead of fc32: half the
 * bytes over PCIe for host-resident IQ; the OFDM stage converts on load (exact). */
#define MI_DL_FLAG_IQ_SC16 8u
/* turbo decoder schedule (int16 arithmetic only; results are identical either way).  Default: the
 * latency form (one workgroup per code block, exact trellis segments) when the batch
 * holds at most MI_TDEC_WIN_AUTO_CBS code blocks, else one code block per lane of 64-lane wavefronts.
 * MI_DL_FLAG_TDEC_WIN / MI_DL_FLAG_TDEC_LANE force one of them. */
#define MI_DL_FLAG_TDEC_WIN  16u
#define MI_DL_FLAG_TDEC_LANE 32u
#define MI_TDEC_WIN_AUTO_CBS 1024u
/* Keep the LLR stream (MI_DL_BUF_LLR) of a full run.  By default a run that includes both the DEMAP and
 * the RM stage fuses them: rate de-matching computes each LLR from the grid and channel estimates (the
 * same arithmetic, demap_body.h) and the LLR stream is never written.  Runs of RM without DEMAP read the
 * LLR buffer (e.g. uploaded by the caller). */
#define MI_DL_FLAG_KEEP_LLR  64u
/* Lane-per-code-block turbo decoder in the crossed schedule: two wavefronts per 64-code-block group, the
 * forward and backward recursions of each half-iteration run concurrently and meet in the middle
 * (bit-identical outputs, tdec_body.h).  Without MI_DL_FLAG_TDEC_X / MI_DL_FLAG_TDEC_LANE the int16 lane
 * form is always crossed (the float one below 2 groups per SIMD); MI_DL_FLAG_TDEC_LANE alone = one
 * wavefront per group. */
#define MI_DL_FLAG_TDEC_X    128u
/* with MI_DL_FLAG_TDEC_X: force the crossed kernel's recompute form (metric windows recomputed per step,
 * 92 VGPRs, 5 waves per SIMD; int16 decoder).  Default: chosen when the batch's wavefronts fit in one
 * round at 5 but not at 4 waves per SIMD. */
#define MI_DL_FLAG_TDEC_XR   256u
/* int16 decoder, lane form with TWO code blocks per lane: the trellis metrics of a code block of group A
 * (low 16 bits) and of the same lane of an equal-K group B (high 16 bits) in one register, advanced by
 * packed int16 instructions (half the VALU instructions per code block), crossed schedule; bit-identical
 * outputs (tdec_p2_body.h) */
#define MI_DL_FLAG_TDEC_P2   512u
/* compact channel estimates: the channel-estimation stage writes, per port, only the 4 pilot symbols'
 * frequency-interpolated rows ([port][4][12 N_RB] at the subframe's ce offset) and the fused demap stage
 * interpolates each RE's estimate in time from them with the chest kernel's own expression -- identical
 * LLRs, 10 of 14 rows of channel-estimate traffic written and read never.  Batch throughput mode: the
 * batch's ce buffer then does not hold the full estimates (no MI_DL_FLAG_KEEP_LLR, no mi_dl_ctrl_* on it).
 * A run whose stage mask includes DEMAP but not CHEST after a compact estimation fails (returns -1,
 * mi_dl_last_error says why) instead of reading rows that were never written. */
#define MI_DL_FLAG_CE_COMPACT 1024u
/* waterfall compaction (packed decoder, CRC early stop): the re-compaction rounds after the first decode each dense
 * pair with 8 wavefronts, one per trellis segment, made exact by fix-up rounds instead of the crossed
 * pair of wavefronts: a shorter chain for more wavefronts.  Results identical.  Pays when the batch runs alone (one
 * stream, waterfall: +6 %); beside other streams' work the extra wavefronts cost more than the shorter chain saves
 * (4 streams: -2 %), so it is off by default. */
#define MI_DL_FLAG_TDEC_SEG  2048u

typedef struct mi_dl_batch mi_dl_batch_t;

/* Plans a batch (host work + device allocation, once).  max_its: turbo iteration cap
 * (srslte_sch_set_max_noi), early stop on the code-block CRC as srsLTE does. */
mi_dl_batch_t *mi_dl_batch_create(const mi_dl_sf_cfg_t *cfgs, uint32_t n_sf, uint32_t max_its, uint32_t flags);
void   mi_dl_batch_destroy(mi_dl_batch_t *b);
/* IQ layout: subframe i starts at sample (cf32) mi_dl_batch_iq_offset(b, i) */
size_t mi_dl_batch_iq_offset(const mi_dl_batch_t *b, uint32_t sf);
size_t mi_dl_batch_iq_samples(const mi_dl_batch_t *b);
size_t mi_dl_batch_payload_offset(const mi_dl_batch_t *b, uint32_t sf);
size_t mi_dl_batch_bytes(const mi_dl_batch_t *b, int which);       /* size of a downloadable buffer */
size_t mi_dl_batch_offset(const mi_dl_batch_t *b, int which, uint32_t sf);  /* element offset per subframe */
/* Enqueue the whole receive chain on `stream` (a hipStream_t; NULL = default stream).
 * d_iq: device pointer to cf32 IQ, mi_dl_batch_iq_samples() samples.  Asynchronous. */
int    mi_dl_batch_run(mi_dl_batch_t *b, const void *d_iq, void *stream);
/* Run only the stages in stage_mask (bit i = MI_DL_STAGE_i) -- e.g. RM|TDEC|TB after
 * mi_dl_batch_upload(MI_DL_BUF_LLR) to decode given soft bits (parity tests). */
int    mi_dl_batch_run_stages(mi_dl_batch_t *b, const void *d_iq, void *stream, uint32_t stage_mask);
/* The whole chain with its front end (OFDM, channel estimation, demap + rate de-matching) on front_stream and its
 * back end (turbo decoding, TB CRC) on back_stream, ordered by events the batch owns: the back end waits for this
 * run's front end, and the batch's next run or re-plan (split or not, on any stream) waits for this back end (the
 * workspace is reused).  The run is complete when back_stream is; downloads synchronise it.  With the two streams on complementary CU shares
 * (mi_stream_create_cu_share) and several batches in flight, rate de-matching never shares a CU with the turbo
 * decoder: the headline step is 7.96-8.08 ms on every MI355X sampled, where whole runs on plain streams vary from
 * 7.86 to 8.35 ms by box.  front_stream == back_stream is mi_dl_batch_run.  Results are those of
 * mi_dl_batch_run. */
int    mi_dl_batch_run_split(mi_dl_batch_t *b, const void *d_iq, void *front_stream, void *back_stream);
/* Blocking copy of host data into a batch buffer (grid / ce / LLR injection for parity tests). */
int    mi_dl_batch_upload(mi_dl_batch_t *b, int which, const void *host, size_t bytes);
/* Blocking copy of a result buffer to host memory (synchronises the batch's last stream). */
int    mi_dl_batch_download(mi_dl_batch_t *b, int which, void *host, size_t bytes);
/* Device pointer of a result buffer (for zero-copy consumers). */
void  *mi_dl_batch_device_ptr(mi_dl_batch_t *b, int which);
/* Per-stage device time in ms, averaged over the runs since the last profile reset
 * (MI_DL_FLAG_PROFILE: HIP events recorded on the run's stream around every stage; synchronises). */
int    mi_dl_batch_stage_ms(mi_dl_batch_t *b, float *ms /* MI_DL_NSTAGES */, uint32_t *nruns);
void   mi_dl_batch_profile_reset(mi_dl_batch_t *b);
/* Algorithmic HBM bytes of one run (SURVEY.md 8d definitions) */
double mi_dl_batch_algo_bytes(const mi_dl_batch_t *b, int which_stage /* -1 = compulsory total */);
uint32_t mi_dl_batch_n_codeblocks(const mi_dl_batch_t *b);
/* turbo schedule of the batch: 1 = latency form (MI_DL_FLAG_TDEC_WIN rules), 2 = lane per code block in
 * the crossed schedule (two wavefronts per group), 3 = the same in its recompute form, 4 = two code blocks
 * per lane (packed int16, crossed), 0 = lane per code block, one wavefront per group */
int    mi_dl_batch_turbo_win(const mi_dl_batch_t *b);
/* 1 when schedule 4 runs with waterfall compaction: iteration 0 over every group pair, then the code blocks
 * whose CRC failed gathered into dense continuation pairs for the remaining iterations (early stop,
 * max_its > 1, one code-block size; the environment variable MI_TDEC_COMPACT=0 disables it for A/B runs) */
int    mi_dl_batch_turbo_compact(const mi_dl_batch_t *b);
uint32_t mi_dl_batch_n_groups(const mi_dl_batch_t *b);
/* groups whose rate de-matching runs in the direct form (every valid lane a new TB with one rank table, one
 * k0 rank, one modulation, E <= N_v: each LLR written straight to its softbuffer row); the others gather per
 * circular-buffer position.  The environment variable MI_RM_DIRECT=0 (read when the batch is created) disables
 * the direct form for A/B runs; the softbuffer is bit-identical either way. */
uint32_t mi_dl_batch_rm_direct_groups(const mi_dl_batch_t *b);
/* Waterfall compaction's schedule source.  With compaction the first launch chooses between two exact schedules
 * (store the iteration-0 extrinsic rows and re-compact per iteration, or not; and the size of the gather grid) from
 * the continuation counts of THIS batch's earlier runs, read back without a wait -- so by default the timing of a run
 * depends on the batch's history (its results never do).  mode: -1 = from the history (default); 0 = fixed "few
 * code blocks continue" (the high-SNR schedule); 1 = fixed "waterfall" (the low-SNR schedule).  A fixed mode makes
 * the schedule of every run a function of the call alone.  mi_dl_batch_reset_history forgets the recorded counts
 * (the next run of mode -1 schedules as a fresh batch). */
int    mi_dl_batch_set_tdec_history(mi_dl_batch_t *b, int mode);   /* 0 = ok, -1 = bad mode */
void   mi_dl_batch_reset_history(mi_dl_batch_t *b);

/* ---- streaming re-planning (srsUE re-derives the grant every TTI: phch_worker.cc:297 -> :337).
 * The planner is split from the device: mi_dl_plan_build runs the whole host planning of a batch (RE lists,
 * scrambling words, segmentation, 64-lane grouping, rate-matching work lists) with NO HIP call, so host
 * threads can plan step i+1 while the GPU decodes step i; mi_dl_batch_replan then swaps the built plan into a
 * batch and enqueues its table upload on `stream` -- ordered after the batch's earlier work on that stream,
 * so the caller passes the stream the batch runs on.  The plan object keeps its lookup caches (scrambling
 * words per (RNTI, sf, G), CRS per cell, per-K tables: srslte_ue_dl_set_rnti's pregeneration) across builds,
 * and after a replan it holds the batch's previous plan, ready to be rebuilt.  One plan object per planning
 * thread; a batch's work buffers only grow (a larger plan reallocates them, synchronously).
 * HARQ continuity across a replan, per 64-lane group: the softbuffer rows of a code block are where the plan puts
 * them, so soft combining (new_tb = 0 lanes) carries over for every group the new plan lays out exactly as the old
 * one did (same group index, K, N_cb, first lane and softbuffer offset, and the same code-block-to-lane assignment
 * in its 64 lanes -- e.g. the same grant with a new rv), whatever happens to the other groups.  A group whose layout
 * differs and that holds a retransmission lane has its softbuffer region cleared (every value RX_NULL, as
 * srslte_softbuffer_rx_reset), so such a lane combines with nothing rather than with another code block's rows --
 * srsLTE's softbuffer is per HARQ process, and a change of another subframe's grant does not touch it.  (New
 * transmissions overwrite their rows; rows another layout left are settled by the kernels.)  When the new plan needs a
 * larger softbuffer arena, the arena grows keeping its contents (a device copy; the new tail is RX_NULL), so the
 * unchanged groups keep combining across the growth too. */
typedef struct mi_dl_plan mi_dl_plan_t;
mi_dl_plan_t *mi_dl_plan_create(void);
void   mi_dl_plan_destroy(mi_dl_plan_t *p);
int    mi_dl_plan_build(mi_dl_plan_t *p, const mi_dl_sf_cfg_t *cfgs, uint32_t n_sf);   /* host only; 0 = ok */
int    mi_dl_batch_replan(mi_dl_batch_t *b, mi_dl_plan_t *p, void *stream);          /* 0 = ok */
/* HBM a batch holds: its work buffers, softbuffer arena, descriptor tables and twiddles (the LLR stream only once a
 * run or a buffer access needed it: the default fused demap never does).  mi_dl_plan_device_bytes: the work buffers
 * and softbuffer a batch of a built plan would allocate with these max_its / flags -- host only, no HIP call that
 * allocates; a deployer sizes workspaces per GPU with it (4 workspaces of 12,500 subframes). */
size_t mi_dl_batch_device_bytes(mi_dl_batch_t *b);
size_t mi_dl_plan_device_bytes(const mi_dl_plan_t *p, uint32_t max_its, uint32_t flags);

/* ---- raw turbo code-block decoding (the srslte_tdec_* contract; BASELINE configs[0] =
 * srsLTE turbodecoder_test).  n_cb code blocks of size K; decoder input per block = 3(K+4) fp32
 * LLRs in triplet order d0_k d1_k d2_k with the 36.212 tail layout, LLR > 0 => bit 1 (device
 * memory, [n_cb][3(K+4)]).  max_its iterations; early_stop on the block CRC (24A if crc24a, else
 * 24B) or a fixed iteration count.  Decisions: K/8 bytes per block, MSB first. */
typedef struct mi_tdec_batch mi_tdec_batch_t;
mi_tdec_batch_t *mi_tdec_create(uint32_t K, uint32_t n_cb, uint32_t max_its, int early_stop, int crc24a,
                                uint32_t flags);
void   mi_tdec_destroy(mi_tdec_batch_t *b);
int    mi_tdec_run(mi_tdec_batch_t *b, const float *d_in, void *stream);
int    mi_tdec_download(mi_tdec_batch_t *b, uint8_t *bits /* n_cb*K/8 */, uint32_t *its, uint32_t *crc_ok);
int    mi_tdec_stage_ms(mi_tdec_batch_t *b, float *ms /* MI_DL_NSTAGES */, uint32_t *nruns);
void   mi_tdec_profile_reset(mi_tdec_batch_t *b);
double mi_tdec_algo_bytes(const mi_tdec_batch_t *b);
int    mi_tdec_turbo_win(const mi_tdec_batch_t *b);
/* 36.212 5.1.3 turbo encoder (host): bits[K] -> d[3(K+4)] triplet order, 2 = <NULL> filler */
int    mi_turbo_encode(const uint8_t *bits, uint32_t K, uint32_t F, uint8_t *d);

/* ---- synthetic transmitter (eNB side, host) used to build benchmark input ------------------
 * Mirrors srsLTE's PDSCH encode chain: CRC24A, segmentation, turbo code, rate matching,
 * scrambling, QAM, SFBC, RE mapping + CRS + PCFICH, IFFT (1/sqrt N) + CP, flat per-port
 * channel h and AWGN at snr_db per RE (>= 200 => noiseless).  iq: 2 * 15 N floats. */
int    mi_tx_subframe(const mi_dl_sf_cfg_t *cfg, const uint8_t *tb, const float *h_re_im /* 2*ports */,
                      float snr_db, uint64_t noise_seed, float *iq);
int    mi_sf_len(uint32_t nof_prb);
/* number of PDSCH bits G of a configuration (RE count x Qm, 36.211 6.3.5 / 6.4) */
int    mi_pdsch_G(const mi_dl_sf_cfg_t *cfg);

/* ---- DL control channels ----------------------------------------------
 * PCFICH -> CFI, PDCCH soft bits and DCI blind search (srslte_pdcch_extract_llr +
 * srslte_ue_dl_find_dl_dci / _find_ul_dci) over the grid and channel estimates a batch's front end
 * left in HBM.  Per subframe the search uses that subframe's cfg.rnti and cfg.cfi; PHICH resources
 * phich_ng = 0..3 (Ng = 1/6, 1/2, 1, 2; normal duration).  run() enqueues four kernels (stage mask:
 * 1 PCFICH, 2 PDCCH soft bits, 4 blind search, 8 PHICH); result() returns the first DCI of the
 * subframe in srsLTE's search order (one DCI size over all candidates of a space at a time): `ul` 0 =
 * DL for a C-RNTI (UE-specific L = 1, 2, 4, 8 with 1A then 1, common L = 4, 8 with 1A), 1 = UL format 0,
 * 2 = DL for an SI/RA/P-RNTI (common space only, 1A then 1C).  format: 0 = 0, 1 = 1, 2 = 1A, 3 = 1C.
 * Returns 1 found, 0 not found, -1 error.  PHICH (srslte_ue_dl_decode_phich, phch_worker.cc:381): set_phich() sets per subframe the
 * UL grant's lowest PRB index and DMRS cyclic shift (36.213 9.1.2; default 0, 0), phich() returns the
 * HARQ indicator (1 ACK, 0 NACK, -1 error) and its soft value (> 0 favours ACK). */
typedef struct mi_dl_ctrl mi_dl_ctrl_t;
mi_dl_ctrl_t *mi_dl_ctrl_create(mi_dl_batch_t *b, uint32_t phich_ng);
void          mi_dl_ctrl_destroy(mi_dl_ctrl_t *c);
int           mi_dl_ctrl_run(mi_dl_ctrl_t *c, void *stream);
int           mi_dl_ctrl_run_stages(mi_dl_ctrl_t *c, uint32_t mask, void *stream);
int           mi_dl_ctrl_result(mi_dl_ctrl_t *c, uint32_t sf, int ul, uint32_t *cfi, uint32_t *format, uint32_t *L,
                                uint32_t *ncce, uint8_t *bits /* 64 */, uint32_t *nbits);
size_t        mi_dl_ctrl_llr_floats(const mi_dl_ctrl_t *c);
size_t        mi_dl_ctrl_llr_offset(const mi_dl_ctrl_t *c, uint32_t sf);
uint32_t      mi_dl_ctrl_n_cce(const mi_dl_ctrl_t *c, uint32_t sf);
/* copy PDCCH soft bits between host and device (upload != 0: host -> device) */
int           mi_dl_ctrl_llr(mi_dl_ctrl_t *c, float *host, size_t n, int upload);
int           mi_dl_ctrl_set_phich(mi_dl_ctrl_t *c, const uint32_t *i_lowest, const uint32_t *n_dmrs);
int           mi_dl_ctrl_phich(mi_dl_ctrl_t *c, uint32_t sf, float *soft);

/* ---- sync front end ----------------------------------------------------
 * The data-parallel part of srslte_ue_sync_zerocopy (phch_recv.cc:321): PSS timing + N_ID_2 search,
 * the PSS CFO estimate, SSS detection (N_ID_1, subframe 0 or 5) and CFO correction, batched over
 * device-resident IQ (cf32 offsets in samples).  pss(): window i starts at d_iq[off[i]], candidate
 * lags 0..nlag-1 (the PSS symbol's useful part, N samples, starting at the lag), N_ID_2 candidates in
 * nid2_mask (bit u); rho = |sum x conj(p)|^2 / (E_x E_p); cfo in subcarrier spacings (|cfo| < 1).
 * sss(): subframe i starts at d_iq[sf_off[i]].  correct(): len samples of d_src[src_off[i]] rotated
 * by exp(-j 2 pi cfo[i] n / N) into d_dst[dst_off[i]] (enqueued on stream); pss / sss are synchronous.
 * mi_tx_sync adds the PSS / SSS of subframes 0 and 5 to a subframe's IQ (synthetic transmitter). */
typedef struct mi_sync mi_sync_t;
typedef struct { uint32_t nid2, lag; float rho, cfo; } mi_pss_result_t;
typedef struct { uint32_t nid1, sf5; float score; } mi_sss_result_t;
mi_sync_t *mi_sync_create(uint32_t nof_prb);
void       mi_sync_destroy(mi_sync_t *s);
uint32_t   mi_sync_fft_size(const mi_sync_t *s);
int        mi_sync_pss(mi_sync_t *s, const void *d_iq, const uint64_t *off, uint32_t n, uint32_t nlag,
                       uint32_t nid2_mask, mi_pss_result_t *out, void *stream);
int        mi_sync_sss(mi_sync_t *s, const void *d_iq, const uint64_t *sf_off, const uint32_t *nid2, const float *cfo,
                       uint32_t n, mi_sss_result_t *out, void *stream);
int        mi_sync_correct(mi_sync_t *s, const void *d_src, const uint64_t *src_off, void *d_dst,
                           const uint64_t *dst_off, const float *cfo, uint32_t n, uint32_t len, void *stream);
int        mi_tx_sync(uint32_t cell_id, uint32_t nof_prb, uint32_t sf_idx, float amp, float *iq);

/* ---- host-IQ streaming pipeline -------------------------------------
 * Double buffering for IQ that arrives in host memory (srsUE's sync thread writes the worker's
 * buffer, phch_recv.cc:321-322): two batches of the same configuration, one copy stream and one
 * compute stream.  submit() enqueues the H2D copy of host_iq (mi_dl_batch_iq_samples cf32, or sc16
 * with MI_DL_FLAG_IQ_SC16, batch
 * layout; pinned memory from mi_host_alloc for full PCIe rate) into the free slot behind that
 * slot's previous decode, then the decode behind the copy, and returns the slot (0/1) without
 * blocking: the copy of one batch overlaps the decode of the other.  wait() blocks until the slot's
 * decode is done; its outputs (mi_dl_pipe_batch + mi_dl_batch_download/device_ptr) stay valid
 * until the slot is submitted again, i.e. for one further submit(). */
typedef struct mi_dl_pipe mi_dl_pipe_t;
mi_dl_pipe_t  *mi_dl_pipe_create(const mi_dl_sf_cfg_t *cfgs, uint32_t n_sf, uint32_t max_its, uint32_t flags);
void           mi_dl_pipe_destroy(mi_dl_pipe_t *p);
int            mi_dl_pipe_submit(mi_dl_pipe_t *p, const void *host_iq);   /* slot, or -1 */
int            mi_dl_pipe_wait(mi_dl_pipe_t *p, int slot);
mi_dl_batch_t *mi_dl_pipe_batch(mi_dl_pipe_t *p, int slot);
/* page-locked host memory (hipHostMalloc) for IQ buffers */
void  *mi_host_alloc(size_t bytes);
void   mi_host_free(void *p);

/* ---- device / runtime helpers ------------------------------------------------------------ */
int    mi_device_count(void);
int    mi_set_device(int dev);
const char *mi_last_error(void);
/* A stream of the current device restricted to a share of its compute units (hipExtStreamCreateWithCUMask): CU i
 * belongs to the share when i mod 8 lies in [first, first + count), so a share spans every XCD; count = 8 gives a
 * plain non-blocking stream on all CUs.  (A masked stream is a blocking stream: it orders with the null stream.)
 * Release with mi_stream_destroy. */
int    mi_stream_create_cu_share(uint32_t first, uint32_t count, void **stream);
int    mi_stream_destroy(void *stream);

#ifdef __cplusplus
}
#endif
#endif
