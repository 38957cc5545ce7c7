// tdec.hip -- turbo decoder launch: one 64-lane wavefront per group of code blocks of equal K
// (tdec_body.h holds the per-lane algorithm and its bit-exactness contract with the oracle).
#include "kernels.h"
#include "tb_body.h"
#include "tdec_body.h"
#include "tdec_p2_body.h"

namespace mi {

struct TdecOut {            // per code block (lane index li) results
  uint8_t* cb_bytes;        // [li][CB_BYTES_STRIDE] packed decisions
  uint32_t* its;            // iterations used
  uint32_t* crc_ok;         // CB CRC verdict of the last iteration
  uint32_t* tb_part;        // partial TB-CRC24A register (tb_kernel combines them)
  uint8_t* payload;         // packed decoder, PDSCH batches: payload bytes written in place (MiLaneDesc pay_st /
                            // pay_n), no code-block rows; nullptr = rows
};
// the packed decoder's output of one half: the code block's payload run, or its row; crc24a bit 1 = the code
// block carries the TB CRC (tdec_p2_check)
__device__ inline void p2_out(TdecArgsP2& a, int h, const TdecOut& out, uint32_t li, const MiLaneDesc& ld) {
  a.out_bytes = out.payload ? out.payload : out.cb_bytes;
  a.cb_off[h] = out.payload ? ld.pay_st : li * CB_BYTES_STRIDE;
  a.crc24a[h] = ld.crc24a | (ld.tbcrc << 1);
}

// crossed schedule (tdec_body.h tdec_lane_x): wave 0 = F, wave 1 = B of the same 64 code blocks
struct TdecExecGpu {
  static constexpr bool SHARED = true;
  int wave;
  uint32_t* xcrc;   // LDS [2][64] partial CB-CRC registers
  template <class F, class B>
  __device__ void run(F f, B b) {
    if (wave == 0) f(); else b();
    __syncthreads();
  }
  __device__ uint32_t crc_combine(uint32_t v, int lane) {
    xcrc[wave * LANES + lane] = v;
    __syncthreads();
    return v ^ xcrc[(wave ^ 1) * LANES + lane];
  }
};

template <bool Q16, bool X, bool RC = false>
__device__ __forceinline__ void tdec_group(const float* __restrict__ sb, const uint32_t* __restrict__ wm,
                                           float* __restrict__ scratch, uint8_t* __restrict__ dec, const TdecOut& out,
                                           const MiGroupDesc* __restrict__ groups,
                                           const MiLaneDesc* __restrict__ lanes, const MiKTab* __restrict__ ktabs,
                                           const uint32_t* __restrict__ kdata, uint32_t max_its,
                                           uint32_t early_stop) {
  // CRC24A byte table in LDS (one entry per lane group of 4), for the TB-CRC partial of each lane
  __shared__ uint32_t crc8[256];
  __shared__ uint32_t xcrc[X ? 2 * LANES : 1];
  for (uint32_t b = threadIdx.x; b < 256; b += blockDim.x) crc8[b] = crc24_byte_entry(b, CRC24A_POLY);
  __syncthreads();
  const MiGroupDesc g = groups[blockIdx.x];
  const MiKTab kt = ktabs[g.ktab];
  const int lane = threadIdx.x % LANES;
  const uint32_t li = g.lane0 + lane;
  const MiLaneDesc ld = lanes[li];
  if (!ld.valid) return;
  TdecArgs a;
  a.sb = sb + g.sb_off;
  a.wm = wm + (size_t)blockIdx.x * WM_STRIDE;
  a.zrow = g.Ncb;
  a.q16 = reinterpret_cast<int16_t*>(scratch + g.scratch_off) + q16_elem_off(g.K);
  a.pos = kdata + kt.pos_off;
  a.pi = kdata + kt.pi_off;
  a.crc_a = kdata + kt.crca_off;
  a.crc_b = kdata + kt.crcb_off;
  a.crc8 = crc8;
  a.scr = scratch + g.scratch_off;
  a.dec = dec + g.dec_off;
  a.cb_bytes = out.cb_bytes + (size_t)li * CB_BYTES_STRIDE;
  a.K = g.K;
  a.F = ld.F;
  a.max_its = max_its;
  a.early_stop = early_stop;
  a.crc24a = ld.crc24a;
  if constexpr (X) {
    TdecExecGpu ex{(int)(threadIdx.x / LANES), xcrc};
    TdecLaneResult r = tdec_lane_x<Q16, RC>(a, lane, ex);
    __syncthreads();   // wave B's decisions are visible to wave F, which packs them
    if (ex.wave) return;
    out.its[li] = r.its;
    out.crc_ok[li] = r.crc_ok;
    out.tb_part[li] = tdec_pack(a, lane);
  } else {
    const TdecLaneResult r = tdec_lane<Q16>(a, lane);
    out.its[li] = r.its;
    out.crc_ok[li] = r.crc_ok;
    out.tb_part[li] = r.tb_part;
  }
}

// window masks of the sparse softbuffer rows: one thread per 4-step window (12 decoder inputs) of a
// group; bit i = row pos[12w + i] is materialised (dl_common.h sb_group_floats).  zero (if set): the continuation's
// count, reset here for launch_tdec_cont (one launch fewer on the stream, between the decoder and its assign kernel)
__global__ __launch_bounds__(256) void rowmask_kernel(const float* __restrict__ sb, uint32_t* __restrict__ wm,
                                                     const MiGroupDesc* __restrict__ groups,
                                                     const MiKTab* __restrict__ ktabs,
                                                     const uint32_t* __restrict__ kdata, uint32_t* zero) {
  if (zero && !(blockIdx.x | blockIdx.y | threadIdx.x)) *zero = 0u;
  const MiGroupDesc g = groups[blockIdx.y];
  const uint32_t w = blockIdx.x * 256 + threadIdx.x;
  if (w > g.K / BETA_W) return;
  const uint8_t* map = reinterpret_cast<const uint8_t*>(sb + g.sb_off + sb_map_off(g.Ncb));
  wm[(size_t)blockIdx.y * WM_STRIDE + w] = tdec_window_mask(map, kdata + ktabs[g.ktab].pos_off, w);
}

void launch_rowmask(const float* sb, uint32_t* wm, const MiGroupDesc* groups, const MiKTab* ktabs,
                    const uint32_t* kdata, uint32_t n_groups, uint32_t* zero, hipStream_t st) {
  if (!n_groups) return;
  hipLaunchKernelGGL(rowmask_kernel, dim3((WM_STRIDE + 255) / 256, n_groups), dim3(256), 0, st, sb, wm, groups,
                     ktabs, kdata, zero);
}

// float decoder
__global__ __launch_bounds__(64) void tdec_kernel_gen(const float* __restrict__ sb, const uint32_t* __restrict__ wm, float* __restrict__ scratch,
                                                     uint8_t* __restrict__ dec, TdecOut out,
                                                     const MiGroupDesc* __restrict__ groups,
                                                     const MiLaneDesc* __restrict__ lanes,
                                                     const MiKTab* __restrict__ ktabs, const uint32_t* __restrict__ kdata,
                                                     uint32_t max_its, uint32_t early_stop) {
  tdec_group<false, false>(sb, wm, scratch, dec, out, groups, lanes, ktabs, kdata, max_its, early_stop);
}
// int16 decoder: held to 3 waves per SIMD (<= 168 VGPRs), enough to keep every group of a 12,500-subframe batch
// resident (2,540 waves on 1,024 SIMDs)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3)))
void tdec_kernel_i16(const float* __restrict__ sb, const uint32_t* __restrict__ wm, float* __restrict__ scratch, uint8_t* __restrict__ dec, TdecOut out,
                     const MiGroupDesc* __restrict__ groups, const MiLaneDesc* __restrict__ lanes,
                     const MiKTab* __restrict__ ktabs, const uint32_t* __restrict__ kdata, uint32_t max_its,
                     uint32_t early_stop) {
  tdec_group<true, false>(sb, wm, scratch, dec, out, groups, lanes, ktabs, kdata, max_its, early_stop);
}
// crossed schedule: two wavefronts per group (same register budget per wave)
__global__ __launch_bounds__(128) void tdec_kernel_genx(const float* __restrict__ sb, const uint32_t* __restrict__ wm,
                                                       float* __restrict__ scratch, uint8_t* __restrict__ dec,
                                                       TdecOut out, const MiGroupDesc* __restrict__ groups,
                                                       const MiLaneDesc* __restrict__ lanes,
                                                       const MiKTab* __restrict__ ktabs,
                                                       const uint32_t* __restrict__ kdata, uint32_t max_its,
                                                       uint32_t early_stop) {
  tdec_group<false, true>(sb, wm, scratch, dec, out, groups, lanes, ktabs, kdata, max_its, early_stop);
}
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(4)))
void tdec_kernel_i16x(const float* __restrict__ sb, const uint32_t* __restrict__ wm, float* __restrict__ scratch,
                      uint8_t* __restrict__ dec, TdecOut out, const MiGroupDesc* __restrict__ groups,
                      const MiLaneDesc* __restrict__ lanes, const MiKTab* __restrict__ ktabs,
                      const uint32_t* __restrict__ kdata, uint32_t max_its, uint32_t early_stop) {
  tdec_group<true, true>(sb, wm, scratch, dec, out, groups, lanes, ktabs, kdata, max_its, early_stop);
}
// crossed, metric windows recomputed per step: 92 VGPRs, 5 waves per SIMD
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(5)))
void tdec_kernel_i16xr(const float* __restrict__ sb, const uint32_t* __restrict__ wm, float* __restrict__ scratch,
                       uint8_t* __restrict__ dec, TdecOut out, const MiGroupDesc* __restrict__ groups,
                       const MiLaneDesc* __restrict__ lanes, const MiKTab* __restrict__ ktabs,
                       const uint32_t* __restrict__ kdata, uint32_t max_its, uint32_t early_stop) {
  tdec_group<true, true, true>(sb, wm, scratch, dec, out, groups, lanes, ktabs, kdata, max_its, early_stop);
}

// ---- two code blocks per lane (packed int16, tdec_p2_body.h): one workgroup of two wavefronts (the
// crossed schedule) per PAIR of equal-K groups; pairs[2p] = group A, pairs[2p + 1] = group B or
// 0xFFFFFFFF (an unpaired group: the high halves carry no code block)
struct TdecP2ExecGpu {
  static constexpr bool SHARED = true;
  int wave;
  uint32_t* xs;   // LDS [64]: wave F's per-lane code-block CRC verdicts
  template <class F, class B>
  __device__ __forceinline__ void run(F f, B b) {
    if (wave == 0) f(); else b();
    __syncthreads();
  }
  // wave F's value of this lane, on both waves
  __device__ __forceinline__ uint32_t share(uint32_t v, int lane) {
    if (wave == 0) xs[lane] = v;
    __syncthreads();
    const uint32_t r = xs[lane];
    __syncthreads();   // xs is reused by the next exchange
    return r;
  }
  __device__ bool pack_wave() const { return wave == 0; }
};

// 3 waves per SIMD (<= 168 VGPRs): the headline's 1,270 pairs (2,540 wavefronts) resident in one round
constexpr int P2_WAVES = 3;
// 16-step spans (tdec_p2_body.h P2_CKS) hold a wavefront's stash in LDS; ONE: a one-iteration launch, whose passes never
// stash DEC1's a-priori rows (30 rows per wavefront instead of 38: room for the other streams' rate de-matching)
// FIXED: several iterations without early stop (configs[0]): the q rows are created in iteration 0
template <bool ONE, bool FIXED = false>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(P2_WAVES)))
void tdec_kernel_p2x(const float* __restrict__ sb, const uint32_t* __restrict__ wm, float* __restrict__ scratch,
                     uint8_t* __restrict__ dec, TdecOut out, const MiGroupDesc* __restrict__ groups,
                     const MiLaneDesc* __restrict__ lanes, const MiKTab* __restrict__ ktabs,
                     const uint32_t* __restrict__ kdata, const uint32_t* __restrict__ pairs, uint32_t max_its,
                     uint32_t early_stop, uint32_t no_w) {
  __shared__ uint32_t crc8[256], crc8b[256];
  __shared__ uint32_t xs[LANES];
  __shared__ uint32_t stash[2][(ONE ? P2_STASH_ROWS_FIRST : P2_STASH_ROWS) * LANES];
  for (uint32_t b = threadIdx.x; b < 256; b += blockDim.x) {
    crc8[b] = crc24_byte_entry(b, CRC24A_POLY);
    crc8b[b] = crc24_byte_entry(b, CRC24B_POLY);
  }
  __syncthreads();
  const uint32_t ga = pairs[2 * blockIdx.x], gbi = pairs[2 * blockIdx.x + 1];
  const bool paired = gbi != 0xFFFFFFFFu;
  const uint32_t gb = paired ? gbi : ga;
  const MiGroupDesc gA = groups[ga], gB = groups[gb];
  const MiKTab kt = ktabs[gA.ktab];
  const int lane = threadIdx.x % LANES;
  const uint32_t li[2] = {gA.lane0 + lane, gB.lane0 + lane};
  const MiLaneDesc l0 = lanes[li[0]], l1 = lanes[li[1]];
  TdecArgsP2 a;
  a.live = (l0.valid ? 1u : 0u) | (paired && l1.valid ? 2u : 0u);
  if (!a.live) return;   // the same on both wavefronts: no barrier is left waiting
  a.sb[0] = sb + gA.sb_off;
  a.sb[1] = sb + gB.sb_off;
  a.wm[0] = wm + (size_t)ga * WM_STRIDE;
  a.wm[1] = wm + (size_t)gb * WM_STRIDE;
  a.zrow[0] = gA.Ncb;
  a.zrow[1] = gB.Ncb;
  const uint32_t K = gA.K;
  a.scr = reinterpret_cast<uint32_t*>(scratch + gA.scratch_off);   // spans both groups' scratch (plan.cpp)
  a.q = a.scr + (size_t)(4 * K + 8) * LANES;
  a.pos = kdata + kt.pos_off;
  a.pi = kdata + kt.pi_off;
  a.crc8 = crc8;
  a.crc8b = crc8b;
  a.dec = dec + gA.dec_off;
  p2_out(a, 0, out, li[0], l0);
  if (a.live & 2u) p2_out(a, 1, out, li[1], l1);
  else p2_out(a, 1, out, li[0], l0);
  a.to_payload = out.payload != nullptr;
  a.K = K;
  a.F[0] = l0.F;
  a.F[1] = paired ? l1.F : l0.F;
  a.max_its = max_its;
  a.early_stop = early_stop;
  a.cont_w = 0;
  a.no_w = no_w;   // a one-iteration first launch whose continuation re-forms the w rows (launch_tdec_p2)
  TdecP2ExecGpu ex{(int)(threadIdx.x / LANES), xs};
  a.stash = stash[ex.wave];
  const TdecP2Result r = tdec_p2_lane<false, P2_CKS, ONE, FIXED ? 0u : TDEC_MKQ_IT>(a, lane, ex);
  if (ex.wave) return;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    if (!((a.live >> h) & 1u)) continue;
    out.its[li[h]] = r.its[h];
    out.crc_ok[li[h]] = r.crc_ok[h];
    out.tb_part[li[h]] = r.tb_part[h];
  }
}

void launch_tdec_p2(const float* sb, const uint32_t* wm, float* scratch, uint8_t* dec, uint8_t* cb_bytes,
                    uint32_t* cb_its, uint32_t* cb_crc, uint32_t* cb_tbp, const MiGroupDesc* groups,
                    const MiLaneDesc* lanes, const MiKTab* ktabs, const uint32_t* ktab_data, const uint32_t* pairs,
                    uint32_t n_pairs, uint32_t max_its, uint32_t early_stop, uint8_t* payload, bool no_w,
                    hipStream_t st) {
  if (!n_pairs) return;
  const TdecOut out{cb_bytes, cb_its, cb_crc, cb_tbp, payload};
  // a one-iteration launch (the compacted path's first, beside other streams' rate de-matching): the smaller stash
  if (max_its > 1 && !early_stop)
    hipLaunchKernelGGL((tdec_kernel_p2x<false, true>), dim3(n_pairs), dim3(128), 0, st, sb, wm, scratch, dec, out,
                       groups, lanes, ktabs, ktab_data, pairs, max_its, early_stop, 0u);
  else if (max_its > 1)
    hipLaunchKernelGGL(tdec_kernel_p2x<false>, dim3(n_pairs), dim3(128), 0, st, sb, wm, scratch, dec, out, groups,
                       lanes, ktabs, ktab_data, pairs, max_its, early_stop, 0u);
  else
    hipLaunchKernelGGL(tdec_kernel_p2x<true>, dim3(n_pairs), dim3(128), 0, st, sb, wm, scratch, dec, out, groups,
                       lanes, ktabs, ktab_data, pairs, max_its, early_stop, (uint32_t)no_w);
}

// ---- waterfall compaction (tdec_p2_body.h P2ContSrc): one K, early stop, iteration 0 done by
// tdec_kernel_p2x (max_its 1).  cont[0] = number of continuing code blocks, cont[1 ..] = their lane indices;
// continuation pair p holds cont[1 + 128 p + 64 h + lane] in half h of lane `lane`.  cap = the capacity of a list
// (n_groups x 64 entries): one run never claims more (each valid lane continues at most once), and every kernel below
// clamps a count it reads from memory to it and writes no slot beyond it, so two runs of one workspace racing on two
// unordered streams (a caller error: a batch runs on one stream at a time) cannot take a kernel out of its buffers
__device__ __forceinline__ uint32_t cont_count(const uint32_t* list, uint32_t cap) { return min(list[0], cap); }
// 1. one wavefront per group: the lanes whose code block failed its CRC claim consecutive slots
__global__ __launch_bounds__(64) void tdec_cont_assign_kernel(const MiGroupDesc* __restrict__ groups,
                                                              const MiLaneDesc* __restrict__ lanes,
                                                              const uint32_t* __restrict__ cb_crc, uint32_t* cont,
                                                              uint32_t cap) {
  const uint32_t lane = threadIdx.x, li = groups[blockIdx.x].lane0 + lane;
  const bool act = lanes[li].valid && !cb_crc[li];
  const uint64_t m = __ballot(act);
  if (!m) return;
  const int lead = __ffsll((unsigned long long)m) - 1;
  uint32_t base = 0;
  if ((int)lane == lead) base = atomicAdd(cont, (uint32_t)__popcll(m));
  base = __shfl(base, lead);
  const uint32_t slot = base + __popcll(m & ((1ull << lane) - 1ull));
  if (act && slot < cap) cont[1 + slot] = li;
}

// 1'. a re-compaction round (waterfall, tdec_p2_body.h): one wavefront per 64 slots of the previous round's list; its
// code blocks whose CRC still fails claim consecutive slots of the next list, which records each one's lane index and
// its previous slot (src: where the gather finds its state)
__global__ __launch_bounds__(64) void tdec_cont_assign2_kernel(const uint32_t* __restrict__ prev,
                                                               const uint32_t* __restrict__ cb_crc, uint32_t* next,
                                                               uint32_t* __restrict__ src, uint32_t cap) {
  const uint32_t lane = threadIdx.x, d = blockIdx.x * LANES + lane, n = cont_count(prev, cap);
  if (blockIdx.x * LANES >= n) return;   // the whole wavefront
  const uint32_t li = d < n ? prev[1 + d] : 0u;
  const bool act = d < n && !cb_crc[li];
  const uint64_t m = __ballot(act);
  if (!m) return;
  const int lead = __ffsll((unsigned long long)m) - 1;
  uint32_t base = 0;
  if ((int)lane == lead) base = atomicAdd(next, (uint32_t)__popcll(m));
  base = __shfl(base, lead);
  const uint32_t slot = base + __popcll(m & ((1ull << lane) - 1ull));
  if (act && slot < cap) {
    next[1 + slot] = li;
    src[slot] = d;
  }
}

// 2. the gather, grid-stride over tasks (continuation pair, 8 q windows) and (continuation pair, 96 rows of iteration 0's
// state: the x2 rows (DEC1 outputs, at K) when the first launch stored no w rows -- the continuation re-runs DEC2 --,
// else its w rows (at 0)); lane = continuation lane, both halves
constexpr uint32_t CONT_QW = 8, CONT_WR = 96;
__global__ __launch_bounds__(256) void tdec_cont_gather_kernel(const float* __restrict__ sb,
                                                               const uint32_t* __restrict__ wm,
                                                               const float* __restrict__ scratch,
                                                               const MiGroupDesc* __restrict__ groups,
                                                               const uint32_t* __restrict__ pos,
                                                               const uint32_t* __restrict__ cont,
                                                               uint32_t* __restrict__ cscr, size_t pair_u32, uint32_t K,
                                                               uint32_t w_stored, uint32_t cap) {
  const uint32_t n = cont_count(cont, cap), np = (n + 2 * LANES - 1) / (2 * LANES), lane = threadIdx.x % LANES;
  const uint32_t nqw = p2_cont_qwins(K), nqt = (nqw + CONT_QW - 1) / CONT_QW, per = nqt + (K + CONT_WR - 1) / CONT_WR;
  for (uint32_t u = blockIdx.x * 4 + threadIdx.x / LANES; u < np * per; u += gridDim.x * 4) {
    const uint32_t p = u / per, c = u % per;
    P2ContSrc s[2] = {};
    uint32_t live = 0;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t d = p * 2 * LANES + h * LANES + lane;
      if (d >= n) continue;
      const uint32_t li = cont[1 + d], g = li / LANES;   // plan.cpp: group g = lanes 64 g .. 64 g + 63
      live |= 1u << h;
      s[h].sb = sb + groups[g].sb_off;
      s[h].wm = wm + (size_t)g * WM_STRIDE;
      s[h].scr = reinterpret_cast<const uint32_t*>(scratch + groups[g & ~1u].scratch_off);   // pairs (2j, 2j + 1)
      s[h].ls = li % LANES;
      s[h].hs = g & 1u;
    }
    uint32_t* dst = cscr + (size_t)p * pair_u32;
    if (c < nqt) {
      uint32_t* dq = dst + (size_t)(4 * K + 8) * LANES;
      for (uint32_t w = c * CONT_QW; w < min(nqw, (c + 1) * CONT_QW); w++) {
        uint32_t q[3 * BETA_W];
        p2_cont_qwin(s, live, pos, w, q);
#pragma unroll
        for (int i = 0; i < 3 * BETA_W; i++) dq[(size_t)(3 * BETA_W * w + i) * LANES + lane] = q[i];
      }
    } else {
      const uint32_t k0 = (c - nqt) * CONT_WR, k1 = min(K, k0 + CONT_WR);
      if (w_stored) {
#pragma unroll 8
        for (uint32_t k = k0; k < k1; k++) dst[(size_t)k * LANES + lane] = p2_cont_wrow(s, live, k);
      } else {
#pragma unroll 8
        for (uint32_t k = k0; k < k1; k++) dst[(size_t)(K + k) * LANES + lane] = p2_cont_xrow(s, live, K, k);
      }
    }
  }
}

// 2'. a re-compaction round's gather: every packed row of the state iteration it0 reads (the q rows and the w rows
// the previous round's DEC2 stored), dense pairs -> dense pairs; grid-stride over (pair, 96-row chunk)
__global__ __launch_bounds__(256) void tdec_cont_gather2_kernel(const uint32_t* __restrict__ prev, size_t prev_u32,
                                                                const uint32_t* __restrict__ cont,
                                                                const uint32_t* __restrict__ src,
                                                                uint32_t* __restrict__ dst, size_t dst_u32, uint32_t K,
                                                                uint32_t cap) {
  const uint32_t n = cont_count(cont, cap), np = (n + 2 * LANES - 1) / (2 * LANES), lane = threadIdx.x % LANES;
  const uint32_t nq = 3 * (K + 4), per = (K + CONT_WR - 1) / CONT_WR + (nq + CONT_WR - 1) / CONT_WR;
  for (uint32_t u = blockIdx.x * 4 + threadIdx.x / LANES; u < np * per; u += gridDim.x * 4) {
    const uint32_t p = u / per, c = u % per, nwc = (K + CONT_WR - 1) / CONT_WR;
    P2ContSrc s[2] = {};
    uint32_t live = 0;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t d = p * 2 * LANES + h * LANES + lane;
      if (d >= n) continue;
      const uint32_t e = src[d];   // the previous round's slot: pair e / 128, half (e / 64) % 2, lane e % 64
      live |= 1u << h;
      s[h].scr = prev + (size_t)(e / (2 * LANES)) * prev_u32;
      s[h].ls = e % LANES;
      s[h].hs = (e / LANES) & 1u;
    }
    uint32_t* dp = dst + (size_t)p * dst_u32;
    // rows [r0, r1): the w rows (at 0) or the q rows (at 4K + 8)
    const size_t base = c < nwc ? 0 : (size_t)(4 * K + 8);
    const uint32_t r0 = (c < nwc ? c : c - nwc) * CONT_WR, r1 = min(c < nwc ? K : nq, r0 + CONT_WR);
#pragma unroll 8
    for (uint32_t r = r0; r < r1; r++) dp[(base + r) * LANES + lane] = p2_cont_drow(s, live, base + r);
  }
}

// 3. iterations it0 .. it_end - 1 of the continuing code blocks, dense pairs (pair stride pair_u32, decision rows
// dec_stride bytes apart), checkpoints every CKS steps (tdec_p2_body.h P2C_CKS, P2C_CKS_LATE).  (A 2-waves-per-SIMD
// register budget of its own, with q-row loads 2-3 windows ahead, measured neutral on 4 streams: profiles/r4/ab_cont_pf)
template <int CKS>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(P2_WAVES)))
void tdec_kernel_p2c(uint32_t* __restrict__ cscr, uint8_t* __restrict__ cdec, TdecOut out,
                     const MiLaneDesc* __restrict__ lanes, const uint32_t* __restrict__ kdata, MiKTab kt,
                     const uint32_t* __restrict__ cont, size_t pair_u32, size_t dec_stride, uint32_t K, uint32_t max_its,
                     uint32_t w_stored, uint32_t it0, uint32_t it_end, uint32_t cap) {
  __shared__ uint32_t crc8[256], crc8b[256];
  static_assert(CKS != 16, "the continuation has no LDS stash (16-step spans measured slower here: profiles/r5/ab_misc)");
  __shared__ uint32_t xs[LANES];
  const uint32_t n = cont_count(cont, cap), p = blockIdx.x;
  if ((size_t)p * 2 * LANES >= n) return;   // the whole workgroup
  for (uint32_t b = threadIdx.x; b < 256; b += blockDim.x) {
    crc8[b] = crc24_byte_entry(b, CRC24A_POLY);
    crc8b[b] = crc24_byte_entry(b, CRC24B_POLY);
  }
  __syncthreads();
  const int lane = threadIdx.x % LANES;
  const uint32_t d0 = p * 2 * LANES + lane, d1 = d0 + LANES;
  TdecArgsP2 a{};
  a.live = (d0 < n ? 1u : 0u) | (d1 < n ? 2u : 0u);
  if (!a.live) return;   // the same on both wavefronts
  const uint32_t li[2] = {cont[1 + d0], (a.live & 2u) ? cont[1 + d1] : cont[1 + d0]};
  const MiLaneDesc l0 = lanes[li[0]], l1 = lanes[li[1]];
  a.scr = cscr + (size_t)p * pair_u32;
  a.q = a.scr + (size_t)(4 * K + 8) * LANES;
  a.pos = kdata + kt.pos_off;
  a.pi = kdata + kt.pi_off;
  a.crc8 = crc8;
  a.crc8b = crc8b;
  a.dec = cdec + (size_t)p * dec_stride;
  p2_out(a, 0, out, li[0], l0);
  p2_out(a, 1, out, li[1], l1);
  a.to_payload = out.payload != nullptr;
  a.K = K;
  a.F[0] = l0.F;
  a.F[1] = l1.F;
  a.max_its = max_its;
  a.early_stop = 1;
  a.cont_w = w_stored;
  a.it0 = it0;
  a.it_end = it_end;
  TdecP2ExecGpu ex{(int)(threadIdx.x / LANES), xs};
  const TdecP2Result r = tdec_p2_lane<true, CKS>(a, lane, ex);
  if (ex.wave) return;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    if (!((a.live >> h) & 1u)) continue;
    out.its[li[h]] = r.its[h];
    out.crc_ok[li[h]] = r.crc_ok[h];
    out.tb_part[li[h]] = r.tb_part[h];
  }
}

// 3'. a re-compaction round after the first, segmented (tdec_p2_body.h p2s_*): one workgroup of S wavefronts per dense
// pair, wavefront j owning trellis segment j of every pass; the boundaries are made exact by fix-up rounds (a
// workgroup-wide OR decides whether another round runs).  One iteration (it0), w rows gathered (cont_w).
// one constituent decoder of a segmented pair: first passes, then fix-up rounds until no boundary changes (every wave
// joins every barrier; the neighbour's vector is read before the round's barrier, the fix-up writes after it)
template <bool DEC2>
__device__ __forceinline__ void p2s_half(const TdecArgsP2& a, int lane, uint32_t wave, const P2Seg& g, const P2SegVecs& V) {
  const bool mine = wave < g.nseg;
  if (mine) p2s_bwd_first<DEC2>(a, lane, g, V);
  __syncthreads();
  for (;;) {
    P2 nb[8];
    const bool act = mine && wave + 1 < g.nseg;
    if (act) p2s_vld(V.bend, wave + 1, lane, nb);
    __syncthreads();
    const bool ch = act ? p2s_bwd_fix<DEC2>(a, lane, g, V, nb) : false;
    if (!__syncthreads_or(ch)) break;
  }
  if (mine) p2s_fwd_first<DEC2>(a, lane, g, V);
  __syncthreads();
  for (;;) {
    P2 na[8];
    const bool act = mine && wave > 0;
    if (act) p2s_vld(V.aend, wave - 1, lane, na);
    __syncthreads();
    const bool ch = act ? p2s_fwd_fix<DEC2>(a, lane, g, V, na) : false;
    if (!__syncthreads_or(ch)) break;
  }
}

template <int S>
__global__ __launch_bounds__(64 * S) __attribute__((amdgpu_waves_per_eu(P2_WAVES)))
void tdec_kernel_p2s(uint32_t* __restrict__ cscr, uint8_t* __restrict__ cdec, TdecOut out,
                     const MiLaneDesc* __restrict__ lanes, const uint32_t* __restrict__ kdata, MiKTab kt,
                     const uint32_t* __restrict__ cont, size_t pair_u32, size_t dec_stride, uint32_t K, uint32_t max_its,
                     uint32_t it0, uint32_t cap) {
  __shared__ uint32_t crc8[256], crc8b[256];
  __shared__ uint32_t vecs[4][S * P2_CKW * LANES];
  const uint32_t n = cont_count(cont, cap), p = blockIdx.x;
  if ((size_t)p * 2 * LANES >= n) return;   // the whole workgroup
  for (uint32_t b = threadIdx.x; b < 256; b += blockDim.x) {
    crc8[b] = crc24_byte_entry(b, CRC24A_POLY);
    crc8b[b] = crc24_byte_entry(b, CRC24B_POLY);
  }
  __syncthreads();
  const int lane = threadIdx.x % LANES;
  const uint32_t wave = threadIdx.x / LANES;
  const uint32_t d0 = p * 2 * LANES + lane, d1 = d0 + LANES;
  TdecArgsP2 a{};
  a.live = (d0 < n ? 1u : 0u) | (d1 < n ? 2u : 0u);   // dead halves decode zeros, consistently (no early exit: barriers)
  const uint32_t li[2] = {d0 < n ? cont[1 + d0] : cont[1 + p * 2 * LANES],
                          d1 < n ? cont[1 + d1] : (d0 < n ? cont[1 + d0] : cont[1 + p * 2 * LANES])};
  const MiLaneDesc l0 = lanes[li[0]], l1 = lanes[li[1]];
  a.scr = cscr + (size_t)p * pair_u32;
  a.q = a.scr + (size_t)(4 * K + 8) * LANES;
  a.pos = kdata + kt.pos_off;
  a.pi = kdata + kt.pi_off;
  a.crc8 = crc8;
  a.crc8b = crc8b;
  a.dec = cdec + (size_t)p * dec_stride;
  p2_out(a, 0, out, li[0], l0);
  p2_out(a, 1, out, li[1], l1);
  a.to_payload = out.payload != nullptr;
  a.K = K;
  a.F[0] = l0.F;
  a.F[1] = l1.F;
  a.max_its = max_its;
  a.early_stop = 1;
  a.cont_w = 1;
  a.it0 = it0;
  a.it_end = it0 + 1;
  // (built field by field: a const aggregate of LDS addresses becomes a static initializer the backend cannot emit)
  P2SegVecs V;
  V.bvec = vecs[0];
  V.bend = vecs[1];
  V.avec = vecs[2];
  V.aend = vecs[3];
  const P2Seg g = p2s_seg(K, S, wave);
  p2s_half<false>(a, lane, wave, g, V);
  p2s_half<true>(a, lane, wave, g, V);
  if (wave || !a.live) return;   // wave 0: the check pass over the decision rows and the outputs
  uint32_t tbp[2] = {0u, 0u};
  const uint32_t ok = tdec_p2_check(a, lane, a.live, tbp);
#pragma unroll
  for (int h = 0; h < 2; h++) {
    if (!((a.live >> h) & 1u)) continue;
    out.its[li[h]] = it0 + 1;
    out.crc_ok[li[h]] = (ok >> h) & 1u;
    out.tb_part[li[h]] = tbp[h];
  }
}

bool launch_tdec_cont(const float* sb, const uint32_t* wm, float* scratch, size_t scr_pair_u32, uint8_t* dec,
                      uint8_t* cb_bytes, uint32_t* cb_its, uint32_t* cb_crc, uint32_t* cb_tbp, const MiGroupDesc* groups,
                      const MiLaneDesc* lanes, const uint32_t* ktab_data, const MiKTab& kt, uint32_t n_groups, uint32_t* cont,
                      uint32_t* cscr, uint8_t* cdec, uint32_t max_pairs, size_t pair_u32, uint32_t K, uint32_t max_its,
                      uint32_t gather_wgs, uint8_t* payload, bool w_stored, bool rounds, uint32_t* h_count,
                      uint32_t seg, bool cont_zeroed, hipStream_t st) {
  if (!n_groups || !max_pairs) return true;
  const TdecOut out{cb_bytes, cb_its, cb_crc, cb_tbp, payload};
  const size_t nl = (size_t)n_groups * LANES + 1;   // one list: count + lane indices
  uint32_t* lists[2] = {cont, cont + nl};
  uint32_t* src = cont + 2 * nl;
  if (!cont_zeroed && hipMemsetAsync(cont, 0, 4, st) != hipSuccess) return false;
  const uint32_t cap = n_groups * LANES;
  hipLaunchKernelGGL(tdec_cont_assign_kernel, dim3(n_groups), dim3(64), 0, st, groups, lanes, cb_crc, cont, cap);
  if (h_count && hipMemcpyAsync(h_count, cont, 4, hipMemcpyDeviceToHost, st) != hipSuccess) return false;
  hipLaunchKernelGGL(tdec_cont_gather_kernel, dim3(gather_wgs), dim3(256), 0, st, sb, wm, scratch, groups,
                     ktab_data + kt.pos_off, cont, cscr, pair_u32, K, (uint32_t)w_stored, cap);
  const size_t cdec_stride = (size_t)K * LANES;
  if (!rounds) {   // one launch for iterations 1 .. max_its - 1 (each pair until its slowest code block stops)
    hipLaunchKernelGGL(tdec_kernel_p2c<P2C_CKS>, dim3(max_pairs), dim3(128), 0, st, cscr, cdec, out, lanes,
                       ktab_data, kt, cont,
                       pair_u32, cdec_stride, K, max_its, (uint32_t)w_stored, 1u, max_its, cap);
    return true;
  }
  // re-compaction: one iteration per round, the code blocks still failing gathered into fewer dense pairs for the
  // next.  The pair buffers alternate between the continuation scratch and the groups' own scratch (free after the
  // first gather; group pair j's region holds dense pair j: 2 (2K + 8 (K/4 + 1)) >= 7K + 20 rows of 64 lanes)
  uint32_t* bufs[2] = {cscr, reinterpret_cast<uint32_t*>(scratch)};
  const size_t strides[2] = {pair_u32, scr_pair_u32};
  uint8_t* decs[2] = {cdec, dec};
  const size_t dstrides[2] = {cdec_stride, 2 * cdec_stride};
  for (uint32_t it = 1; it < max_its; it++) {
    const int b = (int)((it - 1) & 1u), l = b;
    if (it > 1) {
      if (hipMemsetAsync(lists[l], 0, 4, st) != hipSuccess) return false;
      hipLaunchKernelGGL(tdec_cont_assign2_kernel, dim3(2 * max_pairs), dim3(64), 0, st, lists[l ^ 1], cb_crc, lists[l],
                         src, cap);
      hipLaunchKernelGGL(tdec_cont_gather2_kernel, dim3(gather_wgs), dim3(256), 0, st, bufs[b ^ 1], strides[b ^ 1],
                         lists[l], src, bufs[b], strides[b], K, cap);
    }
    // each round's count, for the next run's grids (h_count[it - 1]: the list this round decodes)
    if (it > 1 && h_count && it <= CONT_HIST &&
        hipMemcpyAsync(h_count + it - 1, lists[l], 4, hipMemcpyDeviceToHost, st) != hipSuccess)
      return false;
    if (it > 1 && seg == 8)   // the late rounds segmented: seg wavefronts per pair (tdec_kernel_p2s)
      hipLaunchKernelGGL(tdec_kernel_p2s<8>, dim3(max_pairs), dim3(512), 0, st, bufs[b], decs[b], out, lanes, ktab_data,
                         kt, lists[l], strides[b], dstrides[b], K, max_its, it, cap);
    else if (it > 1 && seg == 4)
      hipLaunchKernelGGL(tdec_kernel_p2s<4>, dim3(max_pairs), dim3(256), 0, st, bufs[b], decs[b], out, lanes, ktab_data,
                         kt, lists[l], strides[b], dstrides[b], K, max_its, it, cap);
    else if (it > 1)
      hipLaunchKernelGGL(tdec_kernel_p2c<P2C_CKS_LATE>, dim3(max_pairs), dim3(128), 0, st, bufs[b], decs[b], out, lanes,
                         ktab_data, kt, lists[l], strides[b], dstrides[b], K, max_its, 1u, it, it + 1, cap);
    else
      hipLaunchKernelGGL(tdec_kernel_p2c<P2C_CKS>, dim3(max_pairs), dim3(128), 0, st, bufs[b], decs[b], out,
                         lanes, ktab_data, kt, lists[l], strides[b], dstrides[b], K, max_its,
                         (uint32_t)(w_stored || it > 1), it, it + 1, cap);
  }
  return true;
}

void launch_tdec(const float* sb, const uint32_t* wm, float* scratch, uint8_t* dec, uint8_t* cb_bytes, uint32_t* cb_its, uint32_t* cb_crc,
                 uint32_t* cb_tbp, const MiGroupDesc* groups, const MiLaneDesc* lanes, const MiKTab* ktabs,
                 const uint32_t* ktab_data, uint32_t n_groups, uint32_t max_its, uint32_t early_stop, bool q16,
                 int crossed, hipStream_t st) {
  if (!n_groups) return;
  const TdecOut out{cb_bytes, cb_its, cb_crc, cb_tbp, nullptr};
  if (crossed == 2 && q16) {
    hipLaunchKernelGGL(tdec_kernel_i16xr, dim3(n_groups), dim3(128), 0, st, sb, wm, scratch, dec, out, groups, lanes,
                       ktabs, ktab_data, max_its, early_stop);
    return;
  }
  if (crossed) {
    if (q16)
      hipLaunchKernelGGL(tdec_kernel_i16x, dim3(n_groups), dim3(128), 0, st, sb, wm, scratch, dec, out, groups, lanes,
                         ktabs, ktab_data, max_its, early_stop);
    else
      hipLaunchKernelGGL(tdec_kernel_genx, dim3(n_groups), dim3(128), 0, st, sb, wm, scratch, dec, out, groups, lanes,
                         ktabs, ktab_data, max_its, early_stop);
    return;
  }
  if (q16)
    hipLaunchKernelGGL(tdec_kernel_i16, dim3(n_groups), dim3(64), 0, st, sb, wm, scratch, dec, out, groups, lanes, ktabs,
                       ktab_data, max_its, early_stop);
  else
    hipLaunchKernelGGL(tdec_kernel_gen, dim3(n_groups), dim3(64), 0, st, sb, wm, scratch, dec, out, groups, lanes, ktabs,
                       ktab_data, max_its, early_stop);
}

}  // namespace mi
