// tdec_body.h -- max-log-MAP turbo decoder, one code block per lane (gfx950 wavefront = 64 CBs).
//
// Replaces srslte_tdec_reset / srslte_tdec_iteration / srslte_tdec_decision + the CRC early stop
// of srsLTE's decode_tb, reached from srslte_pdsch_decode_rnti (/root/reference/ue/src/phy/
// phch_worker.cc:347-348) with the iteration cap of srslte_sch_set_max_noi (phch_worker.cc:88).
//
// Layout (MI355X-first): the 64 code blocks of a group share K, so every memory index is
// wave-uniform -- the QPP interleaver Pi(k) and the circular-buffer position of each d-stream bit
// come from scalar tables, and a wave-instruction touches 64 consecutive floats [index][lane]:
// fully coalesced 256-B accesses even for the interleaved decoder.  The lane reads its systematic
// and parity LLRs straight out of the HARQ softbuffer (rate de-matching fused into the loads).
// The full-length backward recursion is kept exact by storing beta every BETA_W steps and
// recomputing the window in registers during the forward pass, so decisions and extrinsics are
// bit-identical to the oracle (oracle/o_fec.c documents the operation order reproduced here).
//
// Latency hiding: each pass walks windows of BETA_W steps; the loads of window j+1 (and its beta
// checkpoint) are issued before window j is computed (software pipelining, no data-dependent
// branches around loads), and the code-block CRC is accumulated during the last half-iteration
// from a per-K table of single-bit CRC contributions (CRC is linear over GF(2)), so no separate
// CRC pass re-reads the decisions.
//
// Two arithmetic modes (template parameter Q16), both bit-exact against their oracle:
//  * Q16 = false: srsLTE-gen float decoder (oracle or_decode_cb);
//  * Q16 = true : the int16 "SSE" decoder (oracle or_decode_cb16, CPU baseline or_simd_decode_cb):
//    inputs quantised q(x) = clamp(rint(32 x), +-511), DEC2 systematic clamped to +-1535, extrinsic
//    w = clamp(llr2 - xs2, +-1023).  Every metric is then an integer of magnitude < 2^15, which
//    fp32 adds/subs/max represent exactly, so the same register code reproduces the int16 decoder.
#pragma once
#include <string.h>

#include <type_traits>

#include "dl_common.h"

#ifndef MI_HD
#define MI_HD __host__ __device__
#endif
#include "p2.h"

namespace mi {

// trellis of the 36.212 PCCC constituent encoder: s = 4 s1 + 2 s2 + s3
MI_HD constexpr int tr_next(int s, int u) { return (((u ^ (s >> 1) ^ s) & 1) << 2) | (s >> 1); }
MI_HD constexpr int tr_par(int s, int u) { return ((u ^ (s >> 1) ^ s) ^ (s >> 2) ^ s) & 1; }
// predecessor (state, input) pairs of state sp: prev states have s>>1 == sp & 3
MI_HD constexpr int tr_prev_s(int sp, int j) { return ((sp & 3) << 1) | j; }
MI_HD constexpr int tr_prev_u(int sp, int j) {
  return ((sp >> 2) ^ (tr_prev_s(sp, j) >> 1) ^ tr_prev_s(sp, j)) & 1;
}

struct TdecArgs {
  const float* sb;        // group softbuffer [Ncb][64] + zero row Ncb (dl_common.h sb_group_floats)
  const uint32_t* wm;     // [K/4 + 1] window masks (rowmask_kernel): bit i of wm[w] = the softbuffer
                          // row of decoder input 12w + i is materialised (else its value is 0)
  uint32_t zrow;          // row index of the group's all-zero softbuffer row (= Ncb)
  int16_t* q16;           // group quantised decoder inputs [3(K+4)][64], natural order (int16 decoder;
                          // written by the first pass of the first iteration, read by all others)
  const uint32_t* pos;    // [3(K+4)] circular-buffer position of decoder input t = 3k+i
  const uint32_t* pi;     // [K]
  const uint32_t* crc_a;  // [K] CRC24A contribution of a 1 at bit i (x^(K-1-i+24) mod g)
  const uint32_t* crc_b;  // [K] same for CRC24B
  const uint32_t* crc8;   // [256] byte table of CRC24A (register update of one message byte)
  float* scr;             // group scratch: w [K][64], llr1 [K][64], checkpoints [(K/4+1)][64][8]
  uint8_t* dec;           // [K][64] decision bytes
  uint8_t* cb_bytes;      // this lane's packed output row (K/8 bytes, MSB first)
  uint32_t K, F, max_its, early_stop, crc24a;
};

// the code block's own CRC register, accumulated by linearity during DEC2's forward pass (early stop)
struct TdecCrc { uint32_t cb; };
struct TdecLaneResult { uint32_t its; uint32_t crc_ok; uint32_t tb_part; };


// The trellis steps below are generic over the metric type T: float (both scalar decoders: the float
// srsLTE-gen one and the int16 one computing on integer-valued fp32) or P2 (p2.h: two code blocks' int16
// metrics in one register, tdec_p2_body.h).  gam(0, 0, ...) is the additive identity (no add is emitted).
template <class T>
MI_HD inline T gam(int u, int z, T lu, T lp, T luz) {
  return u ? (z ? luz : lu) : (z ? lp : Metric<T>::zero());
}

// State-metric normalisation (subtract state 0).  The float decoder normalises every step, as the
// srsLTE-gen order it reproduces does (its rounding depends on magnitudes).  In the int16 design every
// metric is an exact integer and an LLR is a difference of two maxima over alpha + gamma + beta, so
// adding a constant to all states of alpha_k or beta_k never changes an LLR: the int16 decoder
// normalises once per window (before a checkpoint is stored, at the end of each forward window) --
// values then grow by at most 4 x (1535 + 1023 + 511) within a window, far inside fp32's exact range
// -- and its LLRs, extrinsics and decisions stay bit-identical to the per-step oracle.
template <bool NORM, class T>
MI_HD inline void norm8(T (&v)[8]) {
  if constexpr (NORM) {
    const T v0 = v[0];
#pragma unroll
    for (int s = 0; s < 8; s++) v[s] = v[s] - v0;
  }
}

// one backward step: beta_k from beta_{k+1} (NORM: normalised)
template <bool NORM = true, class T>
MI_HD inline void beta_step(const T (&bn)[8], T xs, T xp, T (&bk)[8]) {
  const T luz = xs + xp;
  T m[8];
#pragma unroll
  for (int s = 0; s < 8; s++) {
    const int z0 = tr_par(s, 0), z1 = tr_par(s, 1);
    T b0 = z0 ? bn[tr_next(s, 0)] + gam(0, z0, xs, xp, luz) : bn[tr_next(s, 0)];
    T b1 = bn[tr_next(s, 1)] + gam(1, z1, xs, xp, luz);
    m[s] = fmaxf(b0, b1);
  }
  if constexpr (NORM) {
#pragma unroll
    for (int s = 0; s < 8; s++) bk[s] = m[s] - m[0];
  } else {
#pragma unroll
    for (int s = 0; s < 8; s++) bk[s] = m[s];
  }
}

// The packed int16 decoder (P2) takes each 8-term maximum of the LLR as two interleaved chains joined at the end
// (half the dependent depth); an integer maximum is exact in any order.  The float decoders keep their single chains
// (fmaxf's choice between -0 and +0 could depend on the order).
template <class T>
constexpr bool LLR_TREE = std::is_same<T, P2>::value;

// one forward step: llr_k and alpha_{k+1} from alpha_k, beta_{k+1} (NORM: alpha normalised)
// (max(-inf, t) = t exactly, so the maxima start from the first term)
template <bool NORM = true, class T>
MI_HD inline T alpha_step(T (&al)[8], const T (&bn)[8], T xs, T xp) {
  const T luz = xs + xp;
  T c[8][2], m0 = T{}, m1 = T{}, t8[2][8];
#pragma unroll
  for (int s = 0; s < 8; s++) {
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int z = tr_par(s, u);
      c[s][u] = (u || z) ? tadd_a(al[s], gam(u, z, xs, xp, luz)) : al[s];
      T t = tadd_a(c[s][u], bn[tr_next(s, u)]);
      t8[u][s] = t;
      if constexpr (!LLR_TREE<T>) {
        if (u) m1 = s ? fmaxf(m1, t) : t; else m0 = s ? fmaxf(m0, t) : t;
      }
    }
  }
  if constexpr (LLR_TREE<T>) {   // two interleaved chains per maximum (llr_step)
    m0 = fmaxf(fmaxf(fmaxf(t8[0][0], t8[0][2]), fmaxf(t8[0][4], t8[0][6])), fmaxf(fmaxf(t8[0][1], t8[0][3]), fmaxf(t8[0][5], t8[0][7])));
    m1 = fmaxf(fmaxf(fmaxf(t8[1][0], t8[1][2]), fmaxf(t8[1][4], t8[1][6])), fmaxf(fmaxf(t8[1][1], t8[1][3]), fmaxf(t8[1][5], t8[1][7])));
  }
  T llr = m1 - m0;
  T na[8];
#pragma unroll
  for (int sp = 0; sp < 8; sp++)
    na[sp] = fmaxf(c[tr_prev_s(sp, 0)][tr_prev_u(sp, 0)], c[tr_prev_s(sp, 1)][tr_prev_u(sp, 1)]);
  if constexpr (NORM) {
#pragma unroll
    for (int s = 0; s < 8; s++) al[s] = na[s] - na[0];
  } else {
#pragma unroll
    for (int s = 0; s < 8; s++) al[s] = na[s];
  }
  return llr;
}

// Row access [row][64 lanes].  On the GPU every row stream is read/written with buffer instructions:
// a scalar resource descriptor on the stream base, the row offset (wave-uniform) in soffset and the
// lane's byte offset in one VGPR shared by all accesses -- no per-access 64-bit address arithmetic
// and no address registers held across the pipelined windows (plain global pointers compile to
// one v_lshl_add_u64 + a VGPR pair per load on gfx950).  The host emulation indexes directly.
// Offsets are 32-bit: every stream is addressed from its group's base (< 6 MB).
// The compile-time row delta goes into the wave-uniform soffset, not the lane offset: in the VGPR form LICM hoisted
// every distinct (lane + crow * 64) * size out of the window loops -- one loop-invariant VGPR per row delta, live
// across the whole pass -- instead of leaving the constant in the instruction's immediate offset.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ inline __amdgpu_buffer_rsrc_t row_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
// row = wave-uniform row (soffset), crow = compile-time row delta (folded into the instruction's
// immediate offset): consecutive rows of one window share a single soffset SGPR
template <class T>
__device__ inline T row_ld(const T* base, size_t row, int lane, uint32_t crow = 0) {
  const uint32_t so = ((uint32_t)row + crow) * (uint32_t)(LANES * sizeof(T));
  const uint32_t vo = (uint32_t)lane * (uint32_t)sizeof(T);
  if constexpr (sizeof(T) == 4)
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(row_rsrc(base), vo, so, 0));
  else if constexpr (sizeof(T) == 2)
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b16(row_rsrc(base), vo, so, 0));
  else
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b8(row_rsrc(base), vo, so, 0));
}
template <class T>
__device__ inline void row_st(T* base, size_t row, int lane, T v, uint32_t crow = 0) {
  const uint32_t so = ((uint32_t)row + crow) * (uint32_t)(LANES * sizeof(T));
  const uint32_t vo = (uint32_t)lane * (uint32_t)sizeof(T);
  if constexpr (sizeof(T) == 4)
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), row_rsrc(base), vo, so, 0);
  else if constexpr (sizeof(T) == 2)
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, v), row_rsrc(base), vo, so, 0);
  else
    __builtin_amdgcn_raw_buffer_store_b8(__builtin_bit_cast(uint8_t, v), row_rsrc(base), vo, so, 0);
}
#else
template <class T>
MI_HD inline T row_ld(const T* base, size_t row, int lane, uint32_t crow = 0) {
  return base[(row + crow) * LANES + (uint32_t)lane];
}
template <class T>
MI_HD inline void row_st(T* base, size_t row, int lane, T v, uint32_t crow = 0) {
  base[(row + crow) * LANES + (uint32_t)lane] = v;
}
#endif

// Where the int16 decoder reads its channel inputs from (the float decoder always uses SRC_SB):
//   SRC_SB  the fp32 softbuffer through the position table, quantised at use
//   SRC_MKQ (DEC1 only) the backward pass reads the softbuffer, quantises all three streams and
//           writes the q rows; the forward pass reads the q rows
//   SRC_Q   the int16 q rows [3(K+4)][64] (2-byte rows, natural order, no position table)
// The q rows are created in iteration TDEC_MKQ_IT (1 = only once a second iteration is needed:
// a one-iteration decode never pays for them).
enum { SRC_SB = 0, SRC_MKQ = 1, SRC_Q = 2 };
constexpr uint32_t TDEC_MKQ_IT = 1;
// software-pipelining depth (windows ahead) of a pass, by where it reads its channel inputs: the
// softbuffer passes 1 (ping-pong), the q-row passes 2 (three buffers).  Same-box A/B (ab_pf,
// ab_tord): 2 for every pass made the one-iteration headline 3 % slower and the 8-iteration
// configs[0] 6-10 % faster.
constexpr int TDEC_PF_SB = 1, TDEC_PF_Q = 2;

// Raw loaded values of one window of BETA_W steps, kept exactly as loaded (softbuffer floats or
// int16 words as int) and converted only when the window is computed, so that the loads of the next
// window stay in flight while the current one is computed.
//   DEC1: s0 = systematic, s1 = parity 1, r0 = w            (FIRST: w = 0, not loaded)
//   DEC2: s0 = parity 2,   r0 = llr1[pi], r1 = w[pi]         (FIRST: w = 0, not loaded)
//   (s0/s1: softbuffer floats via the position table, or int16 q[3k+i] rows in int16 mode)
//   ck  : the raw record of the checkpoint closing the window (forward pass only)
//   f0..f2: the three softbuffer inputs of a step, in the int16 decoder's first pass only
template <bool Q16>
struct TdecWin {
  using R = typename std::conditional<Q16, int32_t, float>::type;
  R s0[BETA_W], s1[BETA_W];
  R r0[BETA_W], r1[BETA_W];
  uint32_t ck[8];   // raw checkpoint (row layout: states 1..7 as loaded; record layout: the packed record)
  float f0[BETA_W], f1[BETA_W], f2[BETA_W];
};

// scratch streams (w, llr1, beta checkpoints): fp32 rows, or int16 rows in int16 mode (every stored
// value is an integer inside +-26598, see above); both views share the row layout
// element view of scratch row 0 of a stream starting `row0` rows into the scratch
template <bool Q16>
MI_HD inline const float* scr_at(const float* scr, size_t row0) {
  if constexpr (Q16) return reinterpret_cast<const float*>(reinterpret_cast<const int16_t*>(scr) + row0 * LANES);
  else return scr + row0 * LANES;
}
template <bool Q16>
MI_HD inline float* scr_at(float* scr, size_t row0) { return const_cast<float*>(scr_at<Q16>((const float*)scr, row0)); }
template <bool Q16>
MI_HD inline typename TdecWin<Q16>::R scr_raw(const float* scr, size_t row, int lane, uint32_t crow = 0) {
  if constexpr (Q16) return (int32_t)row_ld(reinterpret_cast<const int16_t*>(scr), row, lane, crow);
  else return row_ld(scr, row, lane, crow);
}
template <bool Q16>
MI_HD inline float scr_cvt(typename TdecWin<Q16>::R x) { return (float)x; }
template <bool Q16>
MI_HD inline void scr_st(float* scr, size_t row, int lane, float v, uint32_t crow = 0) {
  if constexpr (Q16) row_st(reinterpret_cast<int16_t*>(scr), row, lane, (int16_t)(int32_t)v, crow);
  else row_st(scr, row, lane, v, crow);
}

// softbuffer rows in decoder-input order (dl_common.h): decoder input t is row t; the QPP interleaver and the CRC
// contributions come from the per-K tables
#define MI_PI(a, k) ((a).pi[k])
#define MI_CRC(a, pk) ((a).crc24a ? (a).crc_a[pk] : (a).crc_b[pk])
// window mask of decoder inputs 12w .. 12w+11 (tail: w = K/4): bit i = row pos[12w+i] materialised
MI_HD inline uint32_t tdec_window_mask(const uint8_t* map, const uint32_t* pos, uint32_t w) {
  uint32_t m = 0;
  for (uint32_t i = 0; i < 12; i++) m |= (uint32_t)(map[pos[12 * w + i]] != 0) << i;
  return m;
}
// the mask of window w (a scalar load, batched with the window's position-table loads)
MI_HD inline uint32_t wmask(const TdecArgs& a, uint32_t w) { return a.wm[w]; }
// softbuffer float of decoder input t0 + dt (t0 = 12 w, m = wmask(w)): materialised rows are read; an
// unmaterialised row is 0 without HBM traffic -- the group's zero row is read instead (one scalar select; the row
// stays cache-resident).  Same-box A/B (gpurun_out ab_sparse2, profiles/r3/ab_oob): reading out of the buffer
// descriptor's range instead (the hardware returns 0) measured slower for both decoders.
// The row indices of window inputs t0 .. t0 + 11 (the tail's 12 inputs start at 3 K = 12 (K / 4)).
struct PosW { uint32_t v[12]; };
#define MI_POSW(a, t0) pos_window(t0)
MI_HD inline PosW pos_window(uint32_t t0) {
  PosW P;
#pragma unroll
  for (int j = 0; j < 12; j++) P.v[j] = t0 + (uint32_t)j;
  return P;
}
template <bool Q16>
MI_HD inline float sb_in(const TdecArgs& a, uint32_t m, const PosW& P, uint32_t dt, int lane) {
  const bool on = (m >> dt) & 1u;
  return row_ld(a.sb, on ? P.v[dt] : a.zrow, lane);
}

// raw decoder input t (= 3k + i): softbuffer float at position pos[t], or the int16 q row t
template <bool Q16>
MI_HD inline typename TdecWin<Q16>::R dec_in(const TdecArgs& a, uint32_t m, const PosW& P, uint32_t t0, uint32_t dt,
                                             int lane) {
  if constexpr (Q16) return (int32_t)row_ld(a.q16, t0, lane, dt);
  else return sb_in<Q16>(a, m, P, dt, lane);
}

template <bool DEC2, bool FIRST, bool Q16, bool SQ>
MI_HD inline void tdec_load_window(const TdecArgs& a, int lane, uint32_t base, TdecWin<Q16>& r) {
  const float* llr1 = scr_at<Q16>(a.scr, a.K);
  const uint32_t m = (Q16 && SQ) ? 0u : wmask(a, base / BETA_W);
  PosW P{};
  if constexpr (!(Q16 && SQ)) P = MI_POSW(a, 3 * base);
#pragma unroll
  for (int i = 0; i < BETA_W; i++) {
    const uint32_t k = base + i;
    if (!DEC2) {
      if constexpr (Q16 && !SQ) {
        r.f0[i] = sb_in<Q16>(a, m, P, 3 * i, lane);
        r.f1[i] = sb_in<Q16>(a, m, P, 3 * i + 1, lane);
      } else {
        r.s0[i] = dec_in<Q16>(a, m, P, 3 * base, 3 * i, lane);
        r.s1[i] = dec_in<Q16>(a, m, P, 3 * base, 3 * i + 1, lane);
      }
      r.r0[i] = FIRST ? 0 : scr_raw<Q16>(a.scr, base, lane, i);
    } else {
      const uint32_t pk = MI_PI(a, k);
      if constexpr (Q16 && !SQ) r.f0[i] = sb_in<Q16>(a, m, P, 3 * i + 2, lane);
      else r.s0[i] = dec_in<Q16>(a, m, P, 3 * base, 3 * i + 2, lane);
      r.r0[i] = scr_raw<Q16>(llr1, pk, lane);
      r.r1[i] = FIRST ? 0 : scr_raw<Q16>(a.scr, pk, lane);
    }
  }
}

// int16 decoder, q-creating pass (DEC1 backward of iteration TDEC_MKQ_IT): the three softbuffer
// inputs of each step through the position table (+ w); the window computation quantises them and
// writes the q rows
template <bool FIRST, bool Q16>
MI_HD inline void tdec_load_window_sb(const TdecArgs& a, int lane, uint32_t base, TdecWin<Q16>& r) {
  const uint32_t m = wmask(a, base / BETA_W);
  const PosW P = MI_POSW(a, 3 * base);
#pragma unroll
  for (int i = 0; i < BETA_W; i++) {
    r.f0[i] = sb_in<Q16>(a, m, P, 3 * i, lane);
    r.f1[i] = sb_in<Q16>(a, m, P, 3 * i + 1, lane);
    r.f2[i] = sb_in<Q16>(a, m, P, 3 * i + 2, lane);
    r.r0[i] = FIRST ? 0 : scr_raw<Q16>(a.scr, base, lane, i);
  }
}

// Checkpoint c (beta, or in the crossed schedule's first half alpha, at step c * BETA_W) holds states
// 1..7 (state 0 is 0 after normalisation) in a slot of 8 rows' worth of elements at row ck0 + 8 c.
// Two layouts (REC):
//  * rows (single-wave kernel): state s in row ck0 + 8 c + s - 1, seven 128-B (int16) / 256-B row
//    accesses per checkpoint, 14 / 28 B per lane;
//  * record (crossed kernel): [c][lane][8] elements, one 128-bit access per lane (two in float mode),
//    16 / 32 B per lane.  Same-box A/B (`profiles/r1/ab_ck/`): the record saves ~6 memory instructions
//    per trellis step and is 5.6 % faster on configs[2] (0.4 groups per SIMD), but moves 1/7 more
//    checkpoint bytes and was 0.8 % slower at the headline's 2.5 groups per SIMD -- so each kernel
//    keeps the layout that suits the occupancy it is chosen for.
// Checkpoints are taken where every state is reachable (k <= K for beta, k >= 4 for alpha), so no
// -inf is ever stored.
template <bool Q16, bool REC>
MI_HD inline void ck_store(float* scr, size_t ck0, uint32_t c, int lane, const float (&b)[8]) {
  if constexpr (!REC) {
#pragma unroll
    for (int s = 1; s < 8; s++) scr_st<Q16>(scr, ck0 + (size_t)c * 8, lane, b[s], s - 1);
    return;
  }
  constexpr uint32_t NW = Q16 ? 4 : 8, ESZ = Q16 ? 2 : 4;
  uint32_t w[NW];
  if constexpr (Q16) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t lo = (uint16_t)(int16_t)(int32_t)b[2 * k + 1];
      const uint32_t hi = k < 3 ? (uint32_t)(uint16_t)(int16_t)(int32_t)b[2 * k + 2] : 0u;
      w[k] = lo | (hi << 16);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 7; k++) w[k] = __builtin_bit_cast(uint32_t, b[k + 1]);
    w[7] = 0u;
  }
  const uint32_t so = (uint32_t)((ck0 * LANES + (size_t)c * 8 * LANES) * ESZ), vo = (uint32_t)lane * 8 * ESZ;
#if defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rs = row_rsrc(scr);
#pragma unroll
  for (uint32_t q = 0; q < NW / 4; q++)
    __builtin_amdgcn_raw_buffer_store_b128(u4{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]}, rs, vo + 16 * q, so, 0);
#else
  memcpy(reinterpret_cast<char*>(scr) + so + vo, w, sizeof(w));
#endif
}
template <bool Q16, bool REC>
MI_HD inline void ck_load_raw(const float* scr, size_t ck0, uint32_t c, int lane, TdecWin<Q16>& r) {
  if constexpr (!REC) {
#pragma unroll
    for (int s = 1; s < 8; s++) {
      const auto v = scr_raw<Q16>(scr, ck0 + (size_t)c * 8, lane, s - 1);
      r.ck[s - 1] = __builtin_bit_cast(uint32_t, v);
    }
    return;
  }
  constexpr uint32_t NW = Q16 ? 4 : 8, ESZ = Q16 ? 2 : 4;
  const uint32_t so = (uint32_t)((ck0 * LANES + (size_t)c * 8 * LANES) * ESZ), vo = (uint32_t)lane * 8 * ESZ;
#if defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rs = row_rsrc(scr);
#pragma unroll
  for (uint32_t q = 0; q < NW / 4; q++) {
    const u4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 16 * q, so, 0);
    r.ck[4 * q] = v.x; r.ck[4 * q + 1] = v.y; r.ck[4 * q + 2] = v.z; r.ck[4 * q + 3] = v.w;
  }
#else
  memcpy(r.ck, reinterpret_cast<const char*>(scr) + so + vo, NW * 4);
#endif
}
// state s (1..7) of a raw checkpoint
template <bool Q16, bool REC>
MI_HD inline float ck_state(const uint32_t* ck, int s) {
  if constexpr (!REC) return Q16 ? (float)(int32_t)ck[s - 1] : __builtin_bit_cast(float, ck[s - 1]);
  else if constexpr (Q16) return (float)(int16_t)(uint16_t)(ck[(s - 1) >> 1] >> (16 * ((s - 1) & 1)));
  else return __builtin_bit_cast(float, ck[s - 1]);
}

// decoder inputs (xs, xp) of step base+i from the raw window (filler: known-zero bits)
template <bool Q16, bool SQ>
MI_HD inline float chan0(const TdecWin<Q16>& r, int i) {
  if constexpr (Q16 && !SQ) return q16f(r.f0[i]);
  else return scr_cvt<Q16>(r.s0[i]);
}
template <bool Q16, bool SQ>
MI_HD inline float chan1(const TdecWin<Q16>& r, int i) {
  if constexpr (Q16 && !SQ) return q16f(r.f1[i]);
  else return scr_cvt<Q16>(r.s1[i]);
}
template <bool DEC2, bool Q16, bool SQ>
MI_HD inline void tdec_xs_xp(const TdecWin<Q16>& r, int i, uint32_t k, uint32_t F, float& xs, float& xp) {
  constexpr float FILL = Q16 ? -I16_CI : FILLER_LLR;   // q(FILLER_LLR) = -511
  if (!DEC2) {
    const bool fill = k < F;
    xs = (fill ? FILL : chan0<Q16, SQ>(r, i)) + scr_cvt<Q16>(r.r0[i]);
    xp = fill ? FILL : chan1<Q16, SQ>(r, i);
  } else {
    const float d = scr_cvt<Q16>(r.r0[i]) - scr_cvt<Q16>(r.r1[i]);
    xs = Q16 ? clampf(d, I16_CX) : d;
    xp = chan0<Q16, SQ>(r, i);
  }
}

// per-step outputs: DEC1 stores llr1; DEC2 updates w, stores the decision and folds it into the CRC
template <bool DEC2, bool Q16>
MI_HD inline void tdec_emit(const TdecArgs& a, int lane, uint32_t base, int i, float llr, float xs,
                            const TdecWin<Q16>& w, TdecCrc& crc) {
  const uint32_t k = base + i;
  if (!DEC2) {
    scr_st<Q16>(scr_at<Q16>(a.scr, a.K), base, lane, llr, i);           // llr1
  } else {
    const uint32_t pk = MI_PI(a, k);
    scr_st<Q16>(a.scr, pk, lane,                                         // w update
                Q16 ? clampf(llr - xs, I16_CW)
                    : scr_cvt<Q16>(w.r1[i]) + (llr - scr_cvt<Q16>(w.r0[i])));
    const bool bit = llr > 0.0f;
    row_st(a.dec, pk, lane, (uint8_t)(bit ? 1 : 0));                    // decision
    const uint32_t tt = MI_CRC(a, pk);
    crc.cb ^= bit ? tt : 0u;                                            // CB CRC by linearity
  }
}

// backward steps of one window (steps base+W-1 .. base); beta_0 is computed but never used
template <bool DEC2, bool Q16, bool SQ>
MI_HD inline void tdec_beta_window(const TdecWin<Q16>& w, uint32_t base, uint32_t F, float (&b)[8]) {
#pragma unroll
  for (int i = BETA_W - 1; i >= 0; i--) {
    float xs, xp, nb[8];
    tdec_xs_xp<DEC2, Q16, SQ>(w, i, base + i, F, xs, xp);
    beta_step<!Q16>(b, xs, xp, nb);
#pragma unroll
    for (int s = 0; s < 8; s++) b[s] = nb[s];
  }
  norm8<Q16>(b);
}

// the same for the int16 decoder's first pass: quantise the window's softbuffer inputs, store them as
// q rows 3k..3k+2 (read by every later pass), then the backward steps
template <bool Q16>
MI_HD inline void tdec_beta_window_mkq(const TdecArgs& a, int lane, const TdecWin<Q16>& w, uint32_t base,
                                       float (&b)[8]) {
  constexpr float FILL = -I16_CI;
#pragma unroll
  for (int i = BETA_W - 1; i >= 0; i--) {
    const float q0 = q16f(w.f0[i]), q1 = q16f(w.f1[i]), q2 = q16f(w.f2[i]);
    row_st(a.q16, 3 * base, lane, (int16_t)q0, 3 * i);
    row_st(a.q16, 3 * base, lane, (int16_t)q1, 3 * i + 1);
    row_st(a.q16, 3 * base, lane, (int16_t)q2, 3 * i + 2);
    const bool fill = base + i < a.F;
    float nb[8];
    beta_step<!Q16>(b, (fill ? FILL : q0) + scr_cvt<Q16>(w.r0[i]), fill ? FILL : q1, nb);
#pragma unroll
    for (int s = 0; s < 8; s++) b[s] = nb[s];
  }
  norm8<Q16>(b);
}

// forward steps of one window: beta_{base+1..base+W} recomputed in registers from the window's
// closing checkpoint, then alpha and the LLRs
template <bool DEC2, bool Q16, bool SQ, bool REC = false>
MI_HD inline void tdec_alpha_window(const TdecArgs& a, int lane, const TdecWin<Q16>& w, uint32_t base, float (&al)[8],
                                    TdecCrc& crc) {
  float xs[BETA_W], xp[BETA_W];
#pragma unroll
  for (int i = 0; i < BETA_W; i++) tdec_xs_xp<DEC2, Q16, SQ>(w, i, base + i, a.F, xs[i], xp[i]);
  float bw[BETA_W][8];
  bw[BETA_W - 1][0] = 0.0f;
#pragma unroll
  for (int s = 1; s < 8; s++) bw[BETA_W - 1][s] = ck_state<Q16, REC>(w.ck, s);
#pragma unroll
  for (int i = BETA_W - 2; i >= 0; i--) beta_step<!Q16>(bw[i + 1], xs[i + 1], xp[i + 1], bw[i]);
#pragma unroll
  for (int i = 0; i < BETA_W; i++)
    tdec_emit<DEC2, Q16>(a, lane, base, i, alpha_step<!Q16>(al, bw[i], xs[i], xp[i]), xs[i], w, crc);
  norm8<Q16>(al);
}

// One constituent decoder (half iteration).  Backward pass: beta over the 3 tail steps and then the
// K info steps, checkpointed every BETA_W steps.  Forward pass: per window the beta values are
// recomputed from the window's closing checkpoint, alpha and the LLRs follow.  Both passes are
// software-pipelined PF windows deep: PF = 2 unrolls by three windows with rotating buffers A/B/C
// (the loads of window j+2 are issued before window j is computed; the passes may exit after any
// window of the rotation), PF = 1 by two with ping-pong buffers (K is a multiple of 8 for every LTE
// code block size, so the window count K/4 is even and that loop has no remainder).
template <bool DEC2, bool FIRST, bool Q16, int SRC>
MI_HD inline void tdec_half(const TdecArgs& a, int lane, TdecCrc& crc) {
  constexpr bool MKQ = Q16 && !DEC2 && SRC == SRC_MKQ;   // backward pass: softbuffer -> q rows
  constexpr bool SQB = Q16 && SRC == SRC_Q;              // backward pass reads q rows
  constexpr bool SQF = Q16 && SRC != SRC_SB;             // forward pass reads q rows
  constexpr int PF = SRC == SRC_SB ? TDEC_PF_SB : TDEC_PF_Q;
  const uint32_t K = a.K, F = a.F, nw = K / BETA_W;
  const size_t ck = (size_t)2 * K;  // beta checkpoints (row)
  const float NINF = -INFINITY;
  float b[8];
#pragma unroll
  for (int s = 0; s < 8; s++) b[s] = s ? NINF : 0.0f;
  {
    const uint32_t t0 = 3 * K + (DEC2 ? 6 : 0), tm = (Q16 && SQB) ? 0u : wmask(a, nw);
    const PosW PT = MI_POSW(a, 3 * K);   // unused (and not loaded) when the tail comes from q rows
    float tx[3], tp[3];
    if constexpr (MKQ) {
      // all 12 tail inputs (both constituent codes) quantised into their q rows
      float tq[12];
#pragma unroll
      for (int j = 0; j < 12; j++) tq[j] = q16f(sb_in<Q16>(a, tm, PT, j, lane));
#pragma unroll
      for (int j = 0; j < 12; j++) row_st(a.q16, 3 * K, lane, (int16_t)tq[j], j);
#pragma unroll
      for (int j = 0; j < 3; j++) { tx[j] = tq[2 * j]; tp[j] = tq[2 * j + 1]; }
    } else if constexpr (Q16 && !SQB) {
#pragma unroll
      for (int j = 0; j < 3; j++) {
        tx[j] = q16f(sb_in<Q16>(a, tm, PT, t0 - 3 * K + 2 * j, lane));
        tp[j] = q16f(sb_in<Q16>(a, tm, PT, t0 - 3 * K + 2 * j + 1, lane));
      }
    } else {
#pragma unroll
      for (int j = 0; j < 3; j++) {
        tx[j] = scr_cvt<Q16>(dec_in<Q16>(a, tm, PT, 3 * K, t0 - 3 * K + 2 * j, lane));
        tp[j] = scr_cvt<Q16>(dec_in<Q16>(a, tm, PT, 3 * K, t0 - 3 * K + 2 * j + 1, lane));
      }
    }
#pragma unroll
    for (int j = 2; j >= 0; j--) {
      float nb[8];
      beta_step<!Q16>(b, tx[j], tp[j], nb);
#pragma unroll
      for (int s = 0; s < 8; s++) b[s] = nb[s];
    }
    norm8<Q16>(b);
  }
  ck_store<Q16, false>(a.scr, ck, nw, lane, b);
  // ---- backward pass (window j closes with checkpoint j; window 0's betas are not stored)
  auto load = [&](uint32_t w, TdecWin<Q16>& r) {
    if constexpr (MKQ) tdec_load_window_sb<FIRST, Q16>(a, lane, w * BETA_W, r);
    else tdec_load_window<DEC2, FIRST, Q16, SQB>(a, lane, w * BETA_W, r);
  };
  auto beta = [&](const TdecWin<Q16>& r, uint32_t w) {
    if constexpr (MKQ) tdec_beta_window_mkq<Q16>(a, lane, r, w * BETA_W, b);
    else tdec_beta_window<DEC2, Q16, SQB>(r, w * BETA_W, F, b);
  };
  auto fload = [&](uint32_t w, TdecWin<Q16>& r) {
    tdec_load_window<DEC2, FIRST, Q16, SQF>(a, lane, w * BETA_W, r);
    ck_load_raw<Q16, false>(a.scr, ck, w + 1, lane, r);
  };
  float al[8];
#pragma unroll
  for (int s = 0; s < 8; s++) al[s] = s ? NINF : 0.0f;
  if constexpr (PF >= 2) {
    // three rotating buffers: the loads of window j-2 are issued before window j is computed, so two
    // windows of compute cover each load's latency (out-of-range window indices are clamped: harmless
    // reloads at the ends)
    TdecWin<Q16> A, B, C;
    const int last = (int)nw - 1;
    auto lo = [](int w) { return (uint32_t)(w > 0 ? w : 0); };
    auto hi = [last](int w) { return (uint32_t)(w < last ? w : last); };
    load(last, A);
    load(lo(last - 1), B);
    for (int j = last;; j -= 3) {
      load(lo(j - 2), C);
      beta(A, j);
      if (j == 0) break;
      ck_store<Q16, false>(a.scr, ck, j, lane, b);
      load(lo(j - 3), A);
      beta(B, j - 1);
      if (j == 1) break;
      ck_store<Q16, false>(a.scr, ck, j - 1, lane, b);
      load(lo(j - 4), B);
      beta(C, j - 2);
      if (j == 2) break;
      ck_store<Q16, false>(a.scr, ck, j - 2, lane, b);
    }
    // ---- forward pass: window j closes with checkpoint j + 1
    fload(0, A);
    fload(1, B);
    for (int j = 0;; j += 3) {
      fload(hi(j + 2), C);
      tdec_alpha_window<DEC2, Q16, SQF>(a, lane, A, j * BETA_W, al, crc);
      if (j == last) break;
      fload(hi(j + 3), A);
      tdec_alpha_window<DEC2, Q16, SQF>(a, lane, B, (j + 1) * BETA_W, al, crc);
      if (j + 1 == last) break;
      fload(hi(j + 4), B);
      tdec_alpha_window<DEC2, Q16, SQF>(a, lane, C, (j + 2) * BETA_W, al, crc);
      if (j + 2 == last) break;
    }
  } else {
    TdecWin<Q16> A, B;
    load(nw - 1, A);
    for (uint32_t j = nw - 1;; j -= 2) {
      load(j - 1, B);
      beta(A, j);
      ck_store<Q16, false>(a.scr, ck, j, lane, b);
      load(j >= 3 ? j - 2 : 1, A);   // last round: a harmless reload
      beta(B, j - 1);
      if (j == 1) break;
      ck_store<Q16, false>(a.scr, ck, j - 1, lane, b);
    }
    // ---- forward pass: windows 0 (A), 1 (B), ...; window j closes with checkpoint j + 1
    fload(0, A);
    for (uint32_t j = 0; j < nw; j += 2) {
      fload(j + 1, B);
      tdec_alpha_window<DEC2, Q16, SQF>(a, lane, A, j * BETA_W, al, crc);
      fload(j + 2 < nw ? j + 2 : nw - 1, A);   // last round: a harmless reload
      tdec_alpha_window<DEC2, Q16, SQF>(a, lane, B, (j + 1) * BETA_W, al, crc);
    }
  }
}

// ---- crossed schedule: two wavefronts per group --------------------------------------------------
// The lane-per-code-block kernel runs ~2.5 wavefronts per SIMD at the headline batch (2,540 groups on
// 1,024 SIMDs) and is latency-bound: each wave walks 4 K dependent trellis steps per iteration.  The
// crossed schedule gives every group a second wavefront on the same 64 code blocks and splits each
// half-iteration at the middle window h = K / 8 (windows of BETA_W steps, nw = K / 4 of them):
//   phase 1  wave F: alpha over windows 0 .. h-1 (no outputs), alpha checkpoints in slots 1 .. h-1
//            wave B: tail + beta over windows nw-1 .. h, beta checkpoints in slots h+1 .. nw
//   phase 2  wave F: the usual forward pass over windows h .. nw-1 (beta recomputed per window from
//            the checkpoints wave B left), LLRs of steps K/2 .. K-1
//            wave B: backward over windows h-1 .. 0, alpha recomputed per window from wave F's
//            checkpoints, LLRs of steps 0 .. K/2-1
// Both recursions stay exact full-length recursions (only the traversal order changes) and every LLR
// is computed from the same alpha_k, beta_{k+1} and branch metrics with the same operations, so
// outputs are bit-identical to tdec_lane's (and the oracle's).  Alpha and beta checkpoints occupy
// disjoint slots of the one checkpoint stream (alpha_k for k >= 4 has every state reachable: no -inf
// is stored), and the phases only exchange data through checkpoints, so one barrier per phase orders
// them; within a phase the two waves write disjoint rows (steps k < K/2 vs k >= K/2, and pi is a
// permutation for the DEC2 rows).  The host emulation runs the phases of both waves in turn.

// the alpha update of alpha_step without the LLR (identical operations)
template <bool NORM = true, class T>
MI_HD inline void alpha_fwd(T (&al)[8], T xs, T xp) {
  const T luz = xs + xp;
  T c[8][2];
#pragma unroll
  for (int s = 0; s < 8; s++)
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int z = tr_par(s, u);
      c[s][u] = (u || z) ? tadd_a(al[s], gam(u, z, xs, xp, luz)) : al[s];
    }
  T na[8];
#pragma unroll
  for (int sp = 0; sp < 8; sp++)
    na[sp] = fmaxf(c[tr_prev_s(sp, 0)][tr_prev_u(sp, 0)], c[tr_prev_s(sp, 1)][tr_prev_u(sp, 1)]);
  if constexpr (NORM) {
#pragma unroll
    for (int s = 0; s < 8; s++) al[s] = na[s] - na[0];
  } else {
#pragma unroll
    for (int s = 0; s < 8; s++) al[s] = na[s];
  }
}
// the LLR of alpha_step without the alpha update (identical operations)
// REACH: the alpha states that are reachable (bit s); the others are left out of the maxima (for the
// packed int16 decoder's first trellis steps, where "-inf" is a finite stand-in, tdec_p2_body.h)
template <uint32_t REACH = 0xFFu, class T>
MI_HD inline T llr_step(const T (&al)[8], const T (&bn)[8], T xs, T xp) {
  if constexpr (LLR_TREE<T>) {
    // packed int16: the same terms, each maximum as two interleaved chains (states of even / odd rank among the
    // reachable ones) joined at the end: half the dependent depth, two more live accumulators
    const T luz = xs + xp;
    T m[2][2] = {};
    int n = 0;
#pragma unroll
    for (int s = 0; s < 8; s++) {
      if (!((REACH >> s) & 1u)) continue;
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const int z = tr_par(s, u);
        // alpha + (gamma + beta): one saturating add per term, the gamma + beta sums free of the alpha chain
        const T t = tadd_a(al[s], (u || z) ? gam(u, z, xs, xp, luz) + bn[tr_next(s, u)] : bn[tr_next(s, u)]);
        m[u][n & 1] = n < 2 ? t : fmaxf(m[u][n & 1], t);
      }
      n++;
    }
    const T m1 = n > 1 ? fmaxf(m[1][0], m[1][1]) : m[1][0], m0 = n > 1 ? fmaxf(m[0][0], m[0][1]) : m[0][0];
    return m1 - m0;
  }
  const T luz = xs + xp;
  T m0 = T{}, m1 = T{};
  bool f0 = true, f1 = true;
#pragma unroll
  for (int s = 0; s < 8; s++) {
    if (!((REACH >> s) & 1u)) continue;
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int z = tr_par(s, u);
      const T t = tadd_a((u || z) ? tadd_a(al[s], gam(u, z, xs, xp, luz)) : al[s], bn[tr_next(s, u)]);
      if (u) { m1 = f1 ? t : fmaxf(m1, t); f1 = false; }
      else { m0 = f0 ? t : fmaxf(m0, t); f0 = false; }
    }
  }
  return m1 - m0;
}

// phase-1 window of wave F: alpha only (regular inputs, or the q-creating first pass)
template <bool DEC2, bool Q16, bool SQ>
MI_HD inline void tdec_alpha_only_window(const TdecWin<Q16>& w, uint32_t base, uint32_t F, float (&al)[8]) {
#pragma unroll
  for (int i = 0; i < BETA_W; i++) {
    float xs, xp;
    tdec_xs_xp<DEC2, Q16, SQ>(w, i, base + i, F, xs, xp);
    alpha_fwd<!Q16>(al, xs, xp);
  }
  norm8<Q16>(al);
}
template <bool Q16>
MI_HD inline void tdec_alpha_only_window_mkq(const TdecArgs& a, int lane, const TdecWin<Q16>& w, uint32_t base,
                                             float (&al)[8]) {
  constexpr float FILL = -I16_CI;
#pragma unroll
  for (int i = 0; i < BETA_W; i++) {
    const float q0 = q16f(w.f0[i]), q1 = q16f(w.f1[i]), q2 = q16f(w.f2[i]);
    row_st(a.q16, 3 * base, lane, (int16_t)q0, 3 * i);
    row_st(a.q16, 3 * base, lane, (int16_t)q1, 3 * i + 1);
    row_st(a.q16, 3 * base, lane, (int16_t)q2, 3 * i + 2);
    const bool fill = base + i < a.F;
    alpha_fwd<!Q16>(al, (fill ? FILL : q0) + scr_cvt<Q16>(w.r0[i]), fill ? FILL : q1);
  }
  norm8<Q16>(al);
}

// phase-2 window of wave B: backward steps emitting the LLRs (beta carried in b); the alpha each step
// needs is recomputed from the window's opening checkpoint (window 0: the known start state) -- i steps
// for step i, 6 alpha steps per window instead of 3 kept in registers: the 32 VGPRs of a stored alpha
// window were what held the crossed kernel to 4 waves per SIMD.  Recomputation is the same
// deterministic recursion, so the values are identical.
#if defined(__HIP_DEVICE_COMPILE__)
#define MI_OPAQUE8(v) do { _Pragma("unroll") for (int s_ = 0; s_ < 8; s_++) asm volatile("" : "+v"((v)[s_])); } while (0)
#else
#define MI_OPAQUE8(v) do { } while (0)
#endif
template <bool DEC2, bool Q16, bool SQ>
MI_HD inline void tdec_beta_emit_window(const TdecArgs& a, int lane, const TdecWin<Q16>& w, uint32_t base,
                                        float (&b)[8], TdecCrc& crc) {
  float xs[BETA_W], xp[BETA_W];
#pragma unroll
  for (int i = 0; i < BETA_W; i++) tdec_xs_xp<DEC2, Q16, SQ>(w, i, base + i, a.F, xs[i], xp[i]);
  auto ck = [&](float (&v)[8]) {
    v[0] = 0.0f;
#pragma unroll
    for (int s = 1; s < 8; s++) v[s] = base ? ck_state<Q16, true>(w.ck, s) : -INFINITY;
    MI_OPAQUE8(v);
  };
  auto emit_back = [&](const float (&ai)[8], int i) {
    tdec_emit<DEC2, Q16>(a, lane, base, i, llr_step(ai, b, xs[i], xp[i]), xs[i], w, crc);
    float nb[8];
    beta_step<!Q16>(b, xs[i], xp[i], nb);
#pragma unroll
    for (int s = 0; s < 8; s++) b[s] = nb[s];
  };
  // two-level: alpha_{base+2} kept, 4 recursion steps per window (every step's alpha from the checkpoint: 6)
  float a2[8];
  ck(a2);
  alpha_fwd<!Q16>(a2, xs[0], xp[0]);
  alpha_fwd<!Q16>(a2, xs[1], xp[1]);
  {
    float ai[8];
#pragma unroll
    for (int s = 0; s < 8; s++) ai[s] = a2[s];
    alpha_fwd<!Q16>(ai, xs[2], xp[2]);
    emit_back(ai, 3);
  }
  emit_back(a2, 2);
  {
    float ai[8];
    ck(ai);
    alpha_fwd<!Q16>(ai, xs[0], xp[0]);
    emit_back(ai, 1);
  }
  {
    float ai[8];
    ck(ai);
    emit_back(ai, 0);
  }
  norm8<Q16>(b);
}

// phase-2 window of wave B, register form (4 waves per SIMD): alpha of the window recomputed from its opening checkpoint (window 0:
// the known start state), then backward steps emitting the LLRs (beta carried in b)
template <bool DEC2, bool Q16, bool SQ, bool REC = true>
MI_HD inline void tdec_beta_emit_window_reg(const TdecArgs& a, int lane, const TdecWin<Q16>& w, uint32_t base,
                                        float (&b)[8], TdecCrc& crc) {
  float xs[BETA_W], xp[BETA_W];
#pragma unroll
  for (int i = 0; i < BETA_W; i++) tdec_xs_xp<DEC2, Q16, SQ>(w, i, base + i, a.F, xs[i], xp[i]);
  float aw[BETA_W][8];
  aw[0][0] = 0.0f;
#pragma unroll
  for (int s = 1; s < 8; s++) aw[0][s] = base ? ck_state<Q16, REC>(w.ck, s) : -INFINITY;
#pragma unroll
  for (int i = 0; i < BETA_W - 1; i++) {
#pragma unroll
    for (int s = 0; s < 8; s++) aw[i + 1][s] = aw[i][s];
    alpha_fwd<!Q16>(aw[i + 1], xs[i], xp[i]);
  }
#pragma unroll
  for (int i = BETA_W - 1; i >= 0; i--) {
    tdec_emit<DEC2, Q16>(a, lane, base, i, llr_step(aw[i], b, xs[i], xp[i]), xs[i], w, crc);
    float nb[8];
    beta_step<!Q16>(b, xs[i], xp[i], nb);
#pragma unroll
    for (int s = 0; s < 8; s++) b[s] = nb[s];
  }
  norm8<Q16>(b);
}

// the forward window of the crossed kernel: like tdec_alpha_window, but the beta each step needs is
// recomputed from the window's closing checkpoint (3 - i steps for step i) instead of keeping the 4
// recomputed vectors in registers (same values, 6 beta steps per window instead of 3)
static_assert(BETA_W == 4, "the recompute-form windows below are written for 4-step windows");
template <bool DEC2, bool Q16, bool SQ>
MI_HD inline void tdec_alpha_window_rc(const TdecArgs& a, int lane, const TdecWin<Q16>& w, uint32_t base,
                                       float (&al)[8], TdecCrc& crc) {
  // two-level: beta_{base+2} (= bw[1]) is kept, bw[0] / bw[2] are one step from bw[1] / the checkpoint,
  // bw[3] is the checkpoint -- 4 recursion steps per window, 8 extra VGPRs
  float xs[BETA_W], xp[BETA_W];
#pragma unroll
  for (int i = 0; i < BETA_W; i++) tdec_xs_xp<DEC2, Q16, SQ>(w, i, base + i, a.F, xs[i], xp[i]);
  auto ck = [&](float (&v)[8]) {
    v[0] = 0.0f;
#pragma unroll
    for (int s = 1; s < 8; s++) v[s] = ck_state<Q16, true>(w.ck, s);
    MI_OPAQUE8(v);
  };
  auto bstep = [&](float (&v)[8], int j) {
    float nb[8];
    beta_step<!Q16>(v, xs[j], xp[j], nb);
#pragma unroll
    for (int s = 0; s < 8; s++) v[s] = nb[s];
  };
  float b1[8];
  ck(b1);
  bstep(b1, 3);
  bstep(b1, 2);   // b1 = bw[1] = beta_{base+2}
  {
    float bi[8];
#pragma unroll
    for (int s = 0; s < 8; s++) bi[s] = b1[s];
    bstep(bi, 1);   // bw[0]
    tdec_emit<DEC2, Q16>(a, lane, base, 0, alpha_step<!Q16>(al, bi, xs[0], xp[0]), xs[0], w, crc);
  }
  tdec_emit<DEC2, Q16>(a, lane, base, 1, alpha_step<!Q16>(al, b1, xs[1], xp[1]), xs[1], w, crc);
  {
    float bi[8];
    ck(bi);
    bstep(bi, 3);   // bw[2]
    tdec_emit<DEC2, Q16>(a, lane, base, 2, alpha_step<!Q16>(al, bi, xs[2], xp[2]), xs[2], w, crc);
  }
  {
    float bi[8];
    ck(bi);         // bw[3]
    tdec_emit<DEC2, Q16>(a, lane, base, 3, alpha_step<!Q16>(al, bi, xs[3], xp[3]), xs[3], w, crc);
  }
  norm8<Q16>(al);
}

// software-pipelined walk over n windows widx(0), widx(1), ...: PF = 1 ping-pong buffers (loads one
// window ahead), PF = 2 three rotating buffers (two ahead); the last rounds reload the last window
// (harmless)
template <int PF, class Win, class Idx, class Load, class Run>
MI_HD inline void pipe_windows(int n, Idx widx, Load load, Run run) {
  if (n <= 0) return;
  auto at = [&](int i) { return widx(i < n ? i : n - 1); };
  if constexpr (PF >= 3) {
    // PF + 1 buffers in a ring, the rotation unrolled so every buffer index is a compile-time constant
    // (the windows stay in registers); the loads of window i + PF are issued before window i is computed
    constexpr int NB = PF + 1;
    Win buf[NB];
#pragma unroll
    for (int b = 0; b < PF; b++) load(at(b), buf[b]);
    for (int i = 0;; i += NB) {
#pragma unroll
      for (int b = 0; b < NB; b++) {
        load(at(i + b + PF), buf[(b + PF) % NB]);
        run(buf[b], at(i + b));
        if (i + b + 1 >= n) return;
      }
    }
  } else if constexpr (PF == 2) {
    Win A, B, C;
    load(at(0), A);
    load(at(1), B);
    for (int i = 0;; i += 3) {
      load(at(i + 2), C);
      run(A, at(i));
      if (i + 1 >= n) break;
      load(at(i + 3), A);
      run(B, at(i + 1));
      if (i + 2 >= n) break;
      load(at(i + 4), B);
      run(C, at(i + 2));
      if (i + 3 >= n) break;
    }
  } else {
    Win A, B;
    load(at(0), A);
    for (int i = 0;; i += 2) {
      load(at(i + 1), B);
      run(A, at(i));
      if (i + 1 >= n) break;
      load(at(i + 2), A);
      run(B, at(i + 1));
      if (i + 2 >= n) break;
    }
  }
}

// pipelining depth of the crossed schedule's q-row passes (twice the waves hide more latency, and the
// three-buffer rotation spills at the 128-VGPR budget of 4 waves per SIMD)
constexpr int TDEC_XPF_Q = 1;
// the four phase bodies of one constituent decoder (same source modes as tdec_half)
template <bool DEC2, bool FIRST, bool Q16, int SRC, bool RC>
struct TdecX {
  static constexpr bool MKQ = Q16 && !DEC2 && SRC == SRC_MKQ;
  static constexpr bool SQB = Q16 && SRC == SRC_Q;
  static constexpr bool SQF = Q16 && SRC != SRC_SB;
  static constexpr int PF = SRC == SRC_SB ? TDEC_PF_SB : TDEC_XPF_Q;
  using Win = TdecWin<Q16>;

  MI_HD static void load1(const TdecArgs& a, int lane, uint32_t w, Win& r) {
    if constexpr (MKQ) tdec_load_window_sb<FIRST, Q16>(a, lane, w * BETA_W, r);
    else tdec_load_window<DEC2, FIRST, Q16, SQB>(a, lane, w * BETA_W, r);
  }
  // wave F, phase 1: alpha_0 .. alpha_{K/2}
  MI_HD static void f1(const TdecArgs& a, int lane, float (&al)[8]) {
    const uint32_t h = a.K / (2 * BETA_W);
    const size_t ck = (size_t)2 * a.K;
#pragma unroll
    for (int s = 0; s < 8; s++) al[s] = s ? -INFINITY : 0.0f;
    pipe_windows<PF, Win>(
        (int)h, [](int i) { return (uint32_t)i; }, [&](uint32_t w, Win& r) { load1(a, lane, w, r); },
        [&](const Win& r, uint32_t w) {
          if (w) ck_store<Q16, true>(a.scr, ck, w, lane, al);
          if constexpr (MKQ) tdec_alpha_only_window_mkq<Q16>(a, lane, r, w * BETA_W, al);
          else tdec_alpha_only_window<DEC2, Q16, SQB>(r, w * BETA_W, a.F, al);
        });
  }
  // wave F, phase 2: forward pass over windows h .. nw-1 (LLRs of steps K/2 .. K-1)
  MI_HD static void f2(const TdecArgs& a, int lane, float (&al)[8], TdecCrc& crc) {
    const uint32_t nw = a.K / BETA_W, h = nw / 2;
    const size_t ck = (size_t)2 * a.K;
    pipe_windows<PF, Win>(
        (int)(nw - h), [h](int i) { return h + (uint32_t)i; },
        [&](uint32_t w, Win& r) {
          tdec_load_window<DEC2, FIRST, Q16, SQF>(a, lane, w * BETA_W, r);
          ck_load_raw<Q16, true>(a.scr, ck, w + 1, lane, r);
        },
        [&](const Win& r, uint32_t w) {
          if constexpr (RC) tdec_alpha_window_rc<DEC2, Q16, SQF>(a, lane, r, w * BETA_W, al, crc);
          else tdec_alpha_window<DEC2, Q16, SQF, true>(a, lane, r, w * BETA_W, al, crc);
        });
  }
  // wave B, phase 1: tail, then beta_{K} .. beta_{K/2}
  MI_HD static void b1(const TdecArgs& a, int lane, float (&b)[8]) {
    const uint32_t K = a.K, nw = K / BETA_W, h = nw / 2;
    const size_t ck = (size_t)2 * K;
#pragma unroll
    for (int s = 0; s < 8; s++) b[s] = s ? -INFINITY : 0.0f;
    {
      const uint32_t t0 = 3 * K + (DEC2 ? 6 : 0), tm = SQB ? 0u : wmask(a, nw);
      const PosW PT = MI_POSW(a, 3 * K);
      float tx[3], tp[3];
      if constexpr (MKQ) {
        float tq[12];
#pragma unroll
        for (int j = 0; j < 12; j++) tq[j] = q16f(sb_in<Q16>(a, tm, PT, j, lane));
#pragma unroll
        for (int j = 0; j < 12; j++) row_st(a.q16, 3 * K, lane, (int16_t)tq[j], j);
#pragma unroll
        for (int j = 0; j < 3; j++) { tx[j] = tq[2 * j]; tp[j] = tq[2 * j + 1]; }
      } else if constexpr (Q16 && !SQB) {
#pragma unroll
        for (int j = 0; j < 3; j++) {
          tx[j] = q16f(sb_in<Q16>(a, tm, PT, t0 - 3 * K + 2 * j, lane));
          tp[j] = q16f(sb_in<Q16>(a, tm, PT, t0 - 3 * K + 2 * j + 1, lane));
        }
      } else {
#pragma unroll
        for (int j = 0; j < 3; j++) {
          tx[j] = scr_cvt<Q16>(dec_in<Q16>(a, tm, PT, 3 * K, t0 - 3 * K + 2 * j, lane));
          tp[j] = scr_cvt<Q16>(dec_in<Q16>(a, tm, PT, 3 * K, t0 - 3 * K + 2 * j + 1, lane));
        }
      }
#pragma unroll
      for (int j = 2; j >= 0; j--) {
        float nb[8];
        beta_step<!Q16>(b, tx[j], tp[j], nb);
#pragma unroll
        for (int s = 0; s < 8; s++) b[s] = nb[s];
      }
      norm8<Q16>(b);
    }
    ck_store<Q16, true>(a.scr, ck, nw, lane, b);
    pipe_windows<PF, Win>(
        (int)(nw - h), [nw](int i) { return nw - 1 - (uint32_t)i; }, [&](uint32_t w, Win& r) { load1(a, lane, w, r); },
        [&](const Win& r, uint32_t w) {
          if constexpr (MKQ) tdec_beta_window_mkq<Q16>(a, lane, r, w * BETA_W, b);
          else tdec_beta_window<DEC2, Q16, SQB>(r, w * BETA_W, a.F, b);
          if (w > h) ck_store<Q16, true>(a.scr, ck, w, lane, b);
        });
  }
  // wave B, phase 2: windows h-1 .. 0 backward (LLRs of steps 0 .. K/2-1)
  MI_HD static void b2(const TdecArgs& a, int lane, float (&b)[8], TdecCrc& crc) {
    const uint32_t h = a.K / (2 * BETA_W);
    const size_t ck = (size_t)2 * a.K;
    pipe_windows<PF, Win>(
        (int)h, [h](int i) { return h - 1 - (uint32_t)i; },
        [&](uint32_t w, Win& r) {
          tdec_load_window<DEC2, FIRST, Q16, SQF>(a, lane, w * BETA_W, r);
          ck_load_raw<Q16, true>(a.scr, ck, w, lane, r);   // window 0: slot 0 is loaded but not used
        },
        [&](const Win& r, uint32_t w) {
          if constexpr (RC) tdec_beta_emit_window<DEC2, Q16, SQF>(a, lane, r, w * BETA_W, b, crc);
          else tdec_beta_emit_window_reg<DEC2, Q16, SQF>(a, lane, r, w * BETA_W, b, crc);
        });
  }
};

// one half-iteration in the crossed schedule: ex.run(f, b) runs wave F's and wave B's phase body and
// then orders them (GPU: each wave its own, then a workgroup barrier; host: both in turn)
template <bool DEC2, bool FIRST, bool Q16, int SRC, bool RC, class Exec>
MI_HD inline void tdec_xhalf(const TdecArgs& a, int lane, Exec& ex, TdecCrc& cF, TdecCrc& cB) {
  using X = TdecX<DEC2, FIRST, Q16, SRC, RC>;
  float mF[8], mBs[8];
  float(&mB)[8] = Exec::SHARED ? mF : mBs;   // GPU: each wave holds only its own metric
  ex.run([&] { X::f1(a, lane, mF); }, [&] { X::b1(a, lane, mB); });
  ex.run([&] { X::f2(a, lane, mF, cF); }, [&] { X::b2(a, lane, mB, cB); });
}

// the iteration loop of tdec_lane in the crossed schedule (same source-mode sequence); the code-block
// CRC is the XOR of both waves' partial registers (ex.crc_combine), so both waves stop together
// RC: metric windows recomputed per step instead of held in registers (92 VGPRs: 5 waves per SIMD, for
// batches that fit then; more VALU per wave, so the register form is faster when fewer waves are needed)
template <bool Q16, bool RC, class Exec>
MI_HD inline TdecLaneResult tdec_lane_x(const TdecArgs& a, int lane, Exec& ex) {
  TdecLaneResult r{0, 0, 0};
  for (uint32_t it = 0; it < a.max_its; it++) {
    TdecCrc cF{0}, cB{0};
    constexpr uint32_t MK = Q16 ? TDEC_MKQ_IT : 0xffffffffu;
    if (it == 0) {
      if (MK == 0) {
        tdec_xhalf<false, true, Q16, SRC_MKQ, RC>(a, lane, ex, cF, cB);
        tdec_xhalf<true, true, Q16, SRC_Q, RC>(a, lane, ex, cF, cB);
      } else {
        tdec_xhalf<false, true, Q16, SRC_SB, RC>(a, lane, ex, cF, cB);
        tdec_xhalf<true, true, Q16, SRC_SB, RC>(a, lane, ex, cF, cB);
      }
    } else if (it < MK) {
      tdec_xhalf<false, false, Q16, SRC_SB, RC>(a, lane, ex, cF, cB);
      tdec_xhalf<true, false, Q16, SRC_SB, RC>(a, lane, ex, cF, cB);
    } else if (it == MK) {
      tdec_xhalf<false, false, Q16, SRC_MKQ, RC>(a, lane, ex, cF, cB);
      tdec_xhalf<true, false, Q16, SRC_Q, RC>(a, lane, ex, cF, cB);
    } else {
      tdec_xhalf<false, false, Q16, SRC_Q, RC>(a, lane, ex, cF, cB);
      tdec_xhalf<true, false, Q16, SRC_Q, RC>(a, lane, ex, cF, cB);
    }
    r.its = it + 1;
    r.crc_ok = ex.crc_combine(cF.cb ^ cB.cb, lane) == 0;
    if (a.early_stop && r.crc_ok) break;
  }
  return r;
}

// pack the final decisions MSB first; the bytes of the TB payload part (after filler, before the CB
// CRC when C > 1) also run through a byte-wise CRC24A: the code block's partial TB-CRC register
// (tb_kernel combines the partials, tb_body.h)
MI_HD inline uint32_t tdec_pack(const TdecArgs& a, int lane) {
  const uint32_t b0 = a.F / 8, b1 = a.K / 8 - (a.crc24a ? 0 : 3);
  uint32_t tb = 0;
  for (uint32_t j = 0; j < a.K / 8; j++) {
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) v |= (uint32_t)row_ld(a.dec, 8 * j + q, lane) << (7 - q);
    a.cb_bytes[j] = (uint8_t)v;
    if (j >= b0 && j < b1) tb = ((tb << 8) & 0xFFFFFFu) ^ a.crc8[((tb >> 16) ^ v) & 0xFFu];
  }
  return tb;
}

struct TdecExecHost {
  static constexpr bool SHARED = false;
  template <class F, class B>
  void run(F f, B b) { f(); b(); }
  uint32_t crc_combine(uint32_t v, int) { return v; }
};

template <bool Q16>
MI_HD inline TdecLaneResult tdec_lane(const TdecArgs& a, int lane) {
  TdecLaneResult r{0, 0, 0};
  for (uint32_t it = 0; it < a.max_its; it++) {
    TdecCrc crc{0};
    constexpr uint32_t MK = Q16 ? TDEC_MKQ_IT : 0xffffffffu;   // iteration creating the q rows
    if (it == 0) {
      if (MK == 0) {
        tdec_half<false, true, Q16, SRC_MKQ>(a, lane, crc);
        tdec_half<true, true, Q16, SRC_Q>(a, lane, crc);
      } else {
        tdec_half<false, true, Q16, SRC_SB>(a, lane, crc);
        tdec_half<true, true, Q16, SRC_SB>(a, lane, crc);
      }
    } else if (it < MK) {
      tdec_half<false, false, Q16, SRC_SB>(a, lane, crc);
      tdec_half<true, false, Q16, SRC_SB>(a, lane, crc);
    } else if (it == MK) {
      tdec_half<false, false, Q16, SRC_MKQ>(a, lane, crc);
      tdec_half<true, false, Q16, SRC_Q>(a, lane, crc);
    } else {
      tdec_half<false, false, Q16, SRC_Q>(a, lane, crc);
      tdec_half<true, false, Q16, SRC_Q>(a, lane, crc);
    }
    r.its = it + 1;
    r.crc_ok = crc.cb == 0;
    if (a.early_stop && r.crc_ok) break;
  }
  r.tb_part = tdec_pack(a, lane);
  return r;
}

}  // namespace mi
