// tdec_p2_body.h -- the int16 max-log-MAP turbo decoder with TWO code blocks per lane (packed int16).
//
// Same algorithm, schedule and bit-exactness contract as the crossed lane decoder of tdec_body.h
// (tdec_lane_x, register form), with the trellis metrics of two code blocks in one 32-bit register
// (p2.h): lane l of a pair of 64-lane groups A and B of equal K carries code block (A, l) in the low
// and (B, l) in the high 16 bits, so every add / subtract / maximum of the recursions is one
// v_pk_*_16 instruction for two code blocks -- half the VALU instructions per code block -- and every
// scratch / q-row / checkpoint access moves both code blocks' values in one memory instruction.  Two
// wavefronts (F and B, the crossed schedule) run each pair: 2,540 wavefronts for the headline's 2,540
// groups instead of 5,080.
//
// Exactness: every value the int16 decoder forms is an integer inside the int16 range (bounds in
// oracle/o_fec.c: normalised metrics +-3R, R = 2046; with the once-per-window normalisation of
// tdec_body.h a candidate alpha + gamma + beta stays inside +-14R = +-28644 and an LLR inside +-13R),
// so the wrapping packed adds are exact.  The one exception is the "-inf" of the unreachable start
// states.  Beta (the tail's start) uses the finite -16384 (p2.h Metric<P2>::ninf), which loses every maximum of
// the beta recursion against a reachable state.  Alpha (the trellis start) uses -32768 (Metric<P2>::ninf_alpha)
// and every add that takes an alpha metric saturates (p2.h tadd_a: v_pk_add_i16 with clamp, the same rate), so an
// unreachable state also drops out of the LLR maxima of steps 0, 1 and 2 (the only ones with unreachable alpha
// states), exactly as -inf would.  The forward terms are (alpha + gamma) + beta, both adds saturating: at step k <= 2 an
// unreachable candidate is at most -32768 + (k + 1) R + beta(s') and a reachable one at least -(k + 1) R + beta(s''),
// and beta's spread over the states is at most 3R (any state reaches any other in 3 steps, oracle/o_fec.c), so the
// unreachable one is lower by at least 32768 - (2k + 5) R >= 14,354.  The backward terms (llr_step) are
// alpha + (gamma + beta), one saturating add (the gamma + beta sums stay off the alpha chain): there the spread of
// gamma + beta is at most 4R and the margin 32768 - (2k + 4) R >= 16,400.  Reachable values never reach the clamp
// (+-14R), where the saturating and the wrapping add agree.  One code path therefore serves window 0 and every other
// window (no REACH-masked LLR variants: the specialised copies held the kernel's register peak).
//
// Per-code-block early stop: a lane iterates while either of its code blocks is undecided.  After each
// iteration one pass over the decision rows (tdec_p2_check, on wave F) packs the bytes of every code block
// still iterating and runs them through two byte-wise CRC24 registers: the code block's own CRC (CRC24B,
// or CRC24A for a one-code-block TB: remainder 0 = pass, the early-stop test) and the partial TB CRC24A
// of its payload bytes (tb_kernel combines them).  A code block that stops keeps the bytes of its last
// pass; later iterations of its partner never touch its outputs; iteration counts are per code block.
// Outputs (packed bytes, iterations, CRC verdict, partial TB-CRC register) are identical to the
// one-code-block-per-lane kernels and to the oracle's int16 decoder (or_decode_cb16).
//
// The DEC2 passes carry each step's interleaver index pi(k) from the window's loads to its stores in
// scalar registers (TdecWinP2::pk): no table load, and no wait on one, between a step's arithmetic and
// its outputs.
#pragma once
#include "tdec_body.h"

namespace mi {

// the packed decoder's phase bodies are large enough for the inliner to outline them as calls (register saves through
// scratch at every call): force them inline
#define MI_P2_INL MI_HD __attribute__((always_inline)) inline

struct TdecArgsP2 {
  const float* sb[2];     // the two groups' softbuffers (dl_common.h sb_group_floats layout)
  const uint32_t* wm[2];  // their window masks (rowmask_kernel)
  uint32_t zrow[2];       // their all-zero rows
  uint32_t* q;            // packed q rows [3 (K + 4)][64] (lo = group A, hi = group B)
  const uint32_t* pos;    // [3 (K + 4)]
  const uint32_t* pi;     // [K]
  const uint32_t* crc8;   // [256] CRC24A byte table (LDS on the GPU)
  const uint32_t* crc8b;  // [256] CRC24B byte table
  uint32_t* scr;          // pair scratch, u32 rows: w [K][64], llr1 [K][64], checkpoints [(K/4 + 1)][64][7]
  uint8_t* dec;           // [K][64] decision bytes, bit h = code block of half h
  uint8_t* out_bytes;     // wave-uniform: the code-block rows, or -- flag to_payload -- the TB payload buffer
  uint32_t cb_off[2];     // each half's packed output: byte j of the code block at out_bytes + cb_off[h] + j - skip,
  uint32_t to_payload;    // skip = 0 (its row: every byte) or F/8 (payload: its bytes j >= F/8 from its first
                          // payload byte); p2_run_off.  (32-bit offsets: the per-lane state across the trellis is 2
                          // registers, not 6)
  uint32_t K, F[2], max_its, early_stop;
  uint32_t crc24a[2];     // bit 0: C == 1 (CB CRC = TB CRC24A); bit 1: the code block carries the TB CRC
  uint32_t live;          // bit h: half h holds a code block (padding lanes / an unpaired group: 0)
  uint32_t no_w;          // wave-uniform: DEC2 stores no extrinsic rows w (a one-iteration launch: nothing reads
                          // them -- the compaction continuation re-runs DEC2 of iteration 0 instead, tdec_p2_lane)
  uint32_t cont_w;        // continuation only: iteration 0's w rows were gathered (no DEC2 re-run)
  uint32_t it0, it_end;   // continuation only: this launch runs iterations it0 .. it_end - 1 (a round of the
                          // re-compacted waterfall: one iteration; the one-shot continuation: 1 .. max_its - 1)
  uint32_t* stash;        // this wave's P2_STASH_ROWS x 64 words of LDS (16-step checkpoints, TdecP2X; host: a buffer)
};
struct TdecP2Result { uint32_t its[2], crc_ok[2], tb_part[2]; };
// the offset of half h's byte j = 0 from out_bytes: byte j of its run is out_bytes[p2_run_off(a, h) + j].  Signed and
// added only with j (>= F/8 in the run): the first code block of a TB at payload offset 0 has a negative one, and no
// pointer before the buffer is ever formed
MI_HD inline int64_t p2_run_off(const TdecArgsP2& a, int h) {
  return (int64_t)a.cb_off[h] - (int64_t)(a.to_payload ? a.F[h] / 8 : 0u);
}

// decoder-input quantiser q(x) = clamp(rint(32 x), +-511) of two floats, packed.  Device: fma(x, 32,
// 1.5 * 2^23) rounds 32 x to the nearest (even) integer in the low mantissa bits (|32 x| < 2^22; beyond,
// the clamp gives +-511 either way), med3 clamps in that domain, and the low 16 bits of the two results
// are the two's-complement int16 values, packed by one byte permute.
MI_HD inline P2 q16_pair(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float M = 12582912.0f;
  const float ya = __builtin_amdgcn_fmed3f(__builtin_fmaf(a, 32.0f, M), M - I16_CI, M + I16_CI);
  const float yb = __builtin_amdgcn_fmed3f(__builtin_fmaf(b, 32.0f, M), M - I16_CI, M + I16_CI);
  return p2_from_bits(__builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, yb), __builtin_bit_cast(uint32_t, ya),
                                            0x05040100u));
#else
  return p2_make((int)q16f(a), (int)q16f(b));
#endif
}

// DEC2's systematic input x2(k) = clamp(llr1(k) - w(k)) (tdec_body.h) is formed by DEC1 when it emits
// step k -- w(k) is the a-priori row DEC1 has just read in natural order, and it is still the value DEC2
// would read at row pi(k): DEC2 rewrites that row only after reading it -- and stored in the llr1 rows, so
// DEC2 loads one interleaved row per step instead of two (identical integers)
// raw loads of one window (BETA_W steps), converted only at use (software pipelining, tdec_body.h):
//   q-row passes: s0 / s1 = packed q rows;  softbuffer passes: a0/b0, a1/b1 = groups A / B floats
//   DEC1: s0 = systematic, s1 = parity 1, r0 = w;   DEC2: s0 = parity 2, r0 = x2 = llr1[pi] (the x2 rows)
//   MKQ (DEC1, the q-creating pass): a0..a2 / b0..b2 = the three streams of both groups
struct TdecWinP2 {
  uint32_t s0[BETA_W], s1[BETA_W];
  float a0[BETA_W], b0[BETA_W], a1[BETA_W], b1[BETA_W], a2[BETA_W], b2[BETA_W];
  uint32_t r0[BETA_W];
  uint32_t pk[BETA_W];   // DEC2: pi(k) of the window's steps (wave-uniform: scalar registers)
  uint32_t ck[7];
};

MI_HD inline uint32_t p2_wmask(const TdecArgsP2& a, int h, uint32_t w) { return a.wm[h][w]; }
// softbuffer row of decoder input 12 w + dt of half h (tdec_body.h sb_in: unmaterialised rows from the zero row)
MI_HD inline float p2_sb_in(const TdecArgsP2& a, int h, uint32_t m, const PosW& P, uint32_t dt, int lane) {
  return row_ld(a.sb[h], ((m >> dt) & 1u) ? P.v[dt] : a.zrow[h], lane);
}
#define MI_P2_SB_PAIR(A, B, M, DT) (A = p2_sb_in(a, 0, ma, P, DT, lane), B = p2_sb_in(a, 1, mb, P, DT, lane))
template <bool DEC2, bool FIRST, bool SQ>
MI_HD inline void p2_load_window(const TdecArgsP2& a, int lane, uint32_t base, TdecWinP2& r) {
  const uint32_t* llr1 = a.scr + (size_t)a.K * LANES;
  const uint32_t ma = SQ ? 0u : p2_wmask(a, 0, base / BETA_W), mb = SQ ? 0u : p2_wmask(a, 1, base / BETA_W);
  PosW P{};
  if constexpr (!SQ) P = MI_POSW(a, 3 * base);
#pragma unroll
  for (int i = 0; i < BETA_W; i++) {
    const uint32_t k = base + i;
    if (!DEC2) {
      if constexpr (SQ) {
        r.s0[i] = row_ld(a.q, 3 * base, lane, 3 * i);
        r.s1[i] = row_ld(a.q, 3 * base, lane, 3 * i + 1);
      } else {
        MI_P2_SB_PAIR(r.a0[i], r.b0[i], ma, 3 * i);
        MI_P2_SB_PAIR(r.a1[i], r.b1[i], ma, 3 * i + 1);
      }
      r.r0[i] = FIRST ? 0u : row_ld(a.scr, base, lane, i);
    } else {
      const uint32_t pk = MI_PI(a, k);
      r.pk[i] = pk;
      if constexpr (SQ) {
        r.s0[i] = row_ld(a.q, 3 * base, lane, 3 * i + 2);
      } else {
        MI_P2_SB_PAIR(r.a0[i], r.b0[i], ma, 3 * i + 2);
      }
      r.r0[i] = row_ld(llr1, pk, lane);
    }
  }
}
template <bool FIRST>
MI_HD inline void p2_load_window_mkq(const TdecArgsP2& a, int lane, uint32_t base, TdecWinP2& r) {
  const uint32_t ma = p2_wmask(a, 0, base / BETA_W), mb = p2_wmask(a, 1, base / BETA_W);
  const PosW P = MI_POSW(a, 3 * base);
#pragma unroll
  for (int i = 0; i < BETA_W; i++) {
    r.a0[i] = p2_sb_in(a, 0, ma, P, 3 * i, lane);
    r.b0[i] = p2_sb_in(a, 1, mb, P, 3 * i, lane);
    r.a1[i] = p2_sb_in(a, 0, ma, P, 3 * i + 1, lane);
    r.b1[i] = p2_sb_in(a, 1, mb, P, 3 * i + 1, lane);
    r.a2[i] = p2_sb_in(a, 0, ma, P, 3 * i + 2, lane);
    r.b2[i] = p2_sb_in(a, 1, mb, P, 3 * i + 2, lane);
    r.r0[i] = FIRST ? 0u : row_ld(a.scr, base, lane, i);
  }
}

// checkpoint record c: states 1..7 of both code blocks (state 0 is 0), [c][lane][7] u32 -- one 128-bit and
// one 96-bit access per lane, the 64 lanes' records one contiguous 1,792-B run (no padding word: an
// eighth of the checkpoint traffic saved)
constexpr uint32_t P2_CKW = 7;
MI_HD inline void p2_ck_store(uint32_t* scr, size_t ck0, uint32_t c, int lane, const P2 (&b)[8]) {
  uint32_t w[P2_CKW];
#pragma unroll
  for (int k = 0; k < 7; k++) w[k] = p2_bits(b[k + 1]);
  const uint32_t so = (uint32_t)((ck0 * LANES + (size_t)c * P2_CKW * LANES) * 4), vo = (uint32_t)lane * (4 * P2_CKW);
#if defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  typedef uint32_t u3 __attribute__((ext_vector_type(3)));
  const __amdgpu_buffer_rsrc_t rs = row_rsrc(scr);
  __builtin_amdgcn_raw_buffer_store_b128(u4{w[0], w[1], w[2], w[3]}, rs, vo, so, 0);
  __builtin_amdgcn_raw_buffer_store_b96(u3{w[4], w[5], w[6]}, rs, vo + 16, so, 0);
#else
  memcpy(reinterpret_cast<char*>(scr) + so + vo, w, sizeof(w));
#endif
}
MI_HD inline void p2_ck_load_to(const uint32_t* scr, size_t ck0, uint32_t c, int lane, uint32_t (&ck)[P2_CKW]) {
  const uint32_t so = (uint32_t)((ck0 * LANES + (size_t)c * P2_CKW * LANES) * 4), vo = (uint32_t)lane * (4 * P2_CKW);
#if defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  typedef uint32_t u3 __attribute__((ext_vector_type(3)));
  const __amdgpu_buffer_rsrc_t rs = row_rsrc(scr);
  const u4 v0 = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, 0);
  const u3 v1 = __builtin_amdgcn_raw_buffer_load_b96(rs, vo + 16, so, 0);
  ck[0] = v0.x; ck[1] = v0.y; ck[2] = v0.z; ck[3] = v0.w;
  ck[4] = v1.x; ck[5] = v1.y; ck[6] = v1.z;
#else
  memcpy(ck, reinterpret_cast<const char*>(scr) + so + vo, sizeof(ck));
#endif
}
MI_HD inline void p2_ck_load(const uint32_t* scr, size_t ck0, uint32_t c, int lane, TdecWinP2& r) {
  p2_ck_load_to(scr, ck0, c, lane, r.ck);
}
MI_HD inline void p2_ck_vec(const uint32_t (&ck)[7], P2 (&v)[8]) {
  v[0] = Metric<P2>::zero();
#pragma unroll
  for (int s = 1; s < 8; s++) v[s] = p2_from_bits(ck[s - 1]);
}
MI_HD inline void p2_ck_vec(const TdecWinP2& r, P2 (&v)[8]) { p2_ck_vec(r.ck, v); }

// decoder inputs (xs, xp) of step base + i; filler bits (k < F, known zeros; F < 64) of each half get
// q(FILLER_LLR) = -511 in the systematic and parity-1 inputs
template <bool SQ>
MI_HD inline P2 p2_chan0(const TdecWinP2& r, int i) { return SQ ? p2_from_bits(r.s0[i]) : q16_pair(r.a0[i], r.b0[i]); }
template <bool SQ>
MI_HD inline P2 p2_chan1(const TdecWinP2& r, int i) { return SQ ? p2_from_bits(r.s1[i]) : q16_pair(r.a1[i], r.b1[i]); }
MI_HD inline P2 p2_fill(P2 x, uint32_t k, const TdecArgsP2& a) {
  const int FILL = -(int)I16_CI;
  return p2_make(k < a.F[0] ? FILL : p2_lo(x), k < a.F[1] ? FILL : p2_hi(x));
}
template <bool DEC2, bool SQ>
MI_HD inline void p2_xs_xp(const TdecArgsP2& a, const TdecWinP2& r, int i, uint32_t base, P2& xs, P2& xp) {
  if (!DEC2) {
    P2 c0 = p2_chan0<SQ>(r, i), c1 = p2_chan1<SQ>(r, i);
    if (base < 64) {   // wave-uniform: only the first 16 windows can hold filler bits
      c0 = p2_fill(c0, base + i, a);
      c1 = p2_fill(c1, base + i, a);
    }
    xs = c0 + p2_from_bits(r.r0[i]);
    xp = c1;
  } else {
    xs = p2_from_bits(r.r0[i]);
    xp = p2_chan0<SQ>(r, i);
  }
}

// per-step outputs (tdec_body.h tdec_emit): DEC1 stores x2 = clamp(llr1 - w) in the llr1 rows (xs = the step's
// a-priori w); DEC2 updates w at row pi(k) (pk, carried from the window's loads) and stores
// the two decision bits there (the code-block CRCs are taken from the decision rows after the iteration:
// tdec_p2_check)
template <bool DEC2>
MI_HD inline void p2_emit(const TdecArgsP2& a, int lane, uint32_t base, int i, uint32_t pk, P2 llr, P2 xs) {
  if (!DEC2) {
    row_st(a.scr + (size_t)a.K * LANES, base, lane, p2_bits(p2_clamp(llr - xs, (int)I16_CX)), i);
  } else {
    if (!a.no_w) row_st(a.scr, pk, lane, p2_bits(p2_clamp(llr - xs, (int)I16_CW)));
    const uint32_t ng = p2_bits(Metric<P2>::zero() - llr);   // sign bits 15 / 31: llr > 0 per half
    // decision byte: half 0's bit at bit 0, half 1's at bit 4 (the check pass packs 4 rows with 3 shift-ors)
    const uint32_t b0 = (ng >> 15) & 1u, b1 = ng >> 31;
    row_st(a.dec, pk, lane, (uint8_t)(b0 | (b1 << 4)));
  }
}

// ---- window bodies (the register form of tdec_body.h's crossed schedule) --------------------------
// wave F, phase 1: alpha only
template <bool DEC2, bool SQ>
MI_HD inline void p2_alpha_only_window(const TdecArgsP2& a, const TdecWinP2& w, uint32_t base, P2 (&al)[8]) {
#pragma unroll
  for (int i = 0; i < BETA_W; i++) {
    P2 xs, xp;
    p2_xs_xp<DEC2, SQ>(a, w, i, base, xs, xp);
    alpha_fwd<false>(al, xs, xp);
  }
  norm8<true>(al);
}
// the q-creating first pass (DEC1): quantise the window's three streams of both groups, store the packed
// q rows, then the steps
MI_HD inline void p2_store_q(const TdecArgsP2& a, int lane, const TdecWinP2& w, uint32_t base, int i, P2& q0, P2& q1) {
  q0 = q16_pair(w.a0[i], w.b0[i]);
  q1 = q16_pair(w.a1[i], w.b1[i]);
  const P2 q2 = q16_pair(w.a2[i], w.b2[i]);
  row_st(a.q, 3 * base, lane, p2_bits(q0), 3 * i);
  row_st(a.q, 3 * base, lane, p2_bits(q1), 3 * i + 1);
  row_st(a.q, 3 * base, lane, p2_bits(q2), 3 * i + 2);
}
MI_HD inline void p2_mkq_xs_xp(const TdecArgsP2& a, const TdecWinP2& w, uint32_t base, int i, P2 q0, P2 q1, P2& xs,
                               P2& xp) {
  if (base < 64) {
    q0 = p2_fill(q0, base + i, a);
    q1 = p2_fill(q1, base + i, a);
  }
  xs = q0 + p2_from_bits(w.r0[i]);
  xp = q1;
}
MI_HD inline void p2_alpha_only_window_mkq(const TdecArgsP2& a, int lane, const TdecWinP2& w, uint32_t base,
                                           P2 (&al)[8]) {
#pragma unroll
  for (int i = 0; i < BETA_W; i++) {
    P2 q0, q1, xs, xp;
    p2_store_q(a, lane, w, base, i, q0, q1);
    p2_mkq_xs_xp(a, w, base, i, q0, q1, xs, xp);
    alpha_fwd<false>(al, xs, xp);
  }
  norm8<true>(al);
}
// wave B, phase 1: beta only
template <bool DEC2, bool SQ>
MI_HD inline void p2_beta_window(const TdecArgsP2& a, const TdecWinP2& w, uint32_t base, P2 (&b)[8]) {
#pragma unroll
  for (int i = BETA_W - 1; i >= 0; i--) {
    P2 xs, xp, nb[8];
    p2_xs_xp<DEC2, SQ>(a, w, i, base, xs, xp);
    beta_step<false>(b, xs, xp, nb);
#pragma unroll
    for (int s = 0; s < 8; s++) b[s] = nb[s];
  }
  norm8<true>(b);
}
MI_HD inline void p2_beta_window_mkq(const TdecArgsP2& a, int lane, const TdecWinP2& w, uint32_t base, P2 (&b)[8]) {
#pragma unroll
  for (int i = BETA_W - 1; i >= 0; i--) {
    P2 q0, q1, xs, xp, nb[8];
    p2_store_q(a, lane, w, base, i, q0, q1);
    p2_mkq_xs_xp(a, w, base, i, q0, q1, xs, xp);
    beta_step<false>(b, xs, xp, nb);
#pragma unroll
    for (int s = 0; s < 8; s++) b[s] = nb[s];
  }
  norm8<true>(b);
}
// the emit's last operand: DEC2 its systematic input xs, DEC1 (x2 form) the step's a-priori w
template <bool DEC2>
MI_HD inline P2 p2_emit_x(const TdecWinP2& w, const P2 (&xs)[BETA_W], int i) {
  if constexpr (DEC2) return xs[i];
  else return p2_from_bits(w.r0[i]);
}
// wave F, phase 2: beta_{base+1..base+4} recomputed from the closing checkpoint, then alpha + LLRs
template <bool DEC2, bool SQ>
MI_HD inline void p2_alpha_window(const TdecArgsP2& a, int lane, const TdecWinP2& w, uint32_t base, P2 (&al)[8]) {
  P2 xs[BETA_W], xp[BETA_W];
#pragma unroll
  for (int i = 0; i < BETA_W; i++) p2_xs_xp<DEC2, SQ>(a, w, i, base, xs[i], xp[i]);
  P2 bw[BETA_W][8];
  p2_ck_vec(w, bw[BETA_W - 1]);
#pragma unroll
  for (int i = BETA_W - 2; i >= 0; i--) beta_step<false>(bw[i + 1], xs[i + 1], xp[i + 1], bw[i]);
#pragma unroll
  for (int i = 0; i < BETA_W; i++)
    p2_emit<DEC2>(a, lane, base, i, w.pk[i], alpha_step<false>(al, bw[i], xs[i], xp[i]), p2_emit_x<DEC2>(w, xs, i));
  norm8<true>(al);
}
// wave B, phase 2: alpha of the window recomputed from its opening checkpoint (FIRST_WIN, window 0: the start
// state), then backward steps emitting the LLRs (the unreachable start states drop out of the maxima by
// themselves: p2.h tadd_a)
template <bool DEC2, bool SQ, bool FIRST_WIN>
MI_HD inline void p2_beta_emit_window(const TdecArgsP2& a, int lane, const TdecWinP2& w, uint32_t base, P2 (&b)[8]) {
  P2 xs[BETA_W], xp[BETA_W];
#pragma unroll
  for (int i = 0; i < BETA_W; i++) p2_xs_xp<DEC2, SQ>(a, w, i, base, xs[i], xp[i]);
  P2 aw[BETA_W][8];
  if constexpr (FIRST_WIN) {
#pragma unroll
    for (int s = 0; s < 8; s++) aw[0][s] = s ? Metric<P2>::ninf_alpha() : Metric<P2>::zero();
  } else {
    p2_ck_vec(w, aw[0]);
  }
#pragma unroll
  for (int i = 0; i < BETA_W - 1; i++) {
#pragma unroll
    for (int s = 0; s < 8; s++) aw[i + 1][s] = aw[i][s];
    alpha_fwd<false>(aw[i + 1], xs[i], xp[i]);
  }
#pragma unroll
  for (int i = BETA_W - 1; i >= 0; i--) {
    const P2 llr = llr_step(aw[i], b, xs[i], xp[i]);
    p2_emit<DEC2>(a, lane, base, i, w.pk[i], llr, p2_emit_x<DEC2>(w, xs, i));
    P2 nb[8];
    beta_step<false>(b, xs[i], xp[i], nb);
#pragma unroll
    for (int s = 0; s < 8; s++) b[s] = nb[s];
  }
  norm8<true>(b);
}

// ---- 8-step checkpoint spacing -------------------------------------------------------------------
// The phase-1 passes store a checkpoint every second window (8 steps) and the phase-2 passes walk PAIRS
// of windows between them: half the checkpoint stores and loads (8 of the ~35 B per code block and
// step), and each pair's loads are issued once the previous pair's inputs are converted, so they are in
// flight for 8 steps of compute with a single raw buffer.  The 8 metric vectors a pair needs are
// recomputed by halving (the checkpoint, the vector 4 steps in, normalised, then 2 and 1 steps from
// those): 12 recursion steps per 8 instead of 6, in the same 4 live vectors as the 4-step register
// form.  Every LLR still takes its alpha and beta at most 3 unnormalised steps from a normalised vector
// and the running metrics are normalised after every 4 steps exactly as before, so the int16 bounds
// (p2.h) and every output are unchanged; only the traversal of the recomputation differs.
// scheduling fences keep the pair's recomputation in program order (left alone, the scheduler interleaves
// the independent metric chains and the next pair's loads, and the live vectors exceed the register budget)
#if defined(__HIP_DEVICE_COMPILE__)
#define MI_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define MI_SCHED_FENCE() ((void)0)
#endif
struct TdecWin8P2 {
  TdecWinP2 lo, hi;
  uint32_t ck[P2_CKW];
};
struct TdecX8P2 {
  P2 xs[2 * BETA_W], xp[2 * BETA_W];
  uint32_t pk[2 * BETA_W];   // DEC2: pi(k) of the pair's steps
  P2 w[2 * BETA_W];          // DEC1, x2 form: the steps' a-priori w (the emit's operand)
};

template <bool DEC2, bool SQ>
MI_HD inline void p2_cvt8(const TdecArgsP2& a, const TdecWin8P2& r, uint32_t base, TdecX8P2& x) {
#pragma unroll
  for (int i = 0; i < BETA_W; i++) p2_xs_xp<DEC2, SQ>(a, r.lo, i, base, x.xs[i], x.xp[i]);
#pragma unroll
  for (int i = 0; i < BETA_W; i++) p2_xs_xp<DEC2, SQ>(a, r.hi, i, base + BETA_W, x.xs[BETA_W + i], x.xp[BETA_W + i]);
  if constexpr (DEC2) {
#pragma unroll
    for (int i = 0; i < BETA_W; i++) {
      x.pk[i] = r.lo.pk[i];
      x.pk[BETA_W + i] = r.hi.pk[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < BETA_W; i++) {
      x.w[i] = p2_from_bits(r.lo.r0[i]);
      x.w[BETA_W + i] = p2_from_bits(r.hi.r0[i]);
    }
  }
}
template <bool DEC2>
MI_HD inline P2 p2_emit_x8(const TdecX8P2& x, int i) {
  if constexpr (DEC2) return x.xs[i];
  else return x.w[i];
}
// the default argument of a window body's precomputed vector (unused unless HAVE4)
MI_HD inline const P2 (&p2_no_vec())[8] {
  static constexpr P2 v[8] = {};
  return v;
}
#define P2_NO_VEC p2_no_vec()
MI_HD inline void p2_cp8(P2 (&d)[8], const P2 (&s)[8]) {
#pragma unroll
  for (int k = 0; k < 8; k++) d[k] = s[k];
}
// the start of a recomputation chain: an opaque copy, so GVN cannot merge the recomputed chain with the
// chain that produced the same values earlier (which would keep every intermediate vector live: the
// register form this layout avoids)
MI_HD inline void p2_cp8_opaque(P2 (&d)[8], const P2 (&s)[8]) {
  p2_cp8(d, s);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
  for (int k = 0; k < 8; k++) asm volatile("" : "+v"(d[k].v));
#endif
}
// v <- the backward recursion through steps hi .. lo (inputs x[hi] down to x[lo])
template <int HI, int LO>
MI_HD inline void p2_beta_run(P2 (&v)[8], const TdecX8P2& x) {
#pragma unroll
  for (int i = HI; i >= LO; i--) {
    P2 nb[8];
    beta_step<false>(v, x.xs[i], x.xp[i], nb);
    p2_cp8(v, nb);
  }
}
// v <- the forward recursion through steps lo .. hi
template <int LO, int HI>
MI_HD inline void p2_alpha_run(P2 (&v)[8], const TdecX8P2& x) {
#pragma unroll
  for (int i = LO; i <= HI; i++) alpha_fwd<false>(v, x.xs[i], x.xp[i]);
}
MI_HD inline void p2_opaque8(P2 (&d)[8]) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
  for (int k = 0; k < 8; k++) asm volatile("" : "+v"(d[k].v));
#endif
}
// a recomputation chain that starts from vector s.  DIRECT: its first step reads s itself (no copy) and an empty asm on
// that step's result keeps GVN from merging the rest of the chain with another one -- at most one chain per source
// vector starts this way (the others from an opaque copy), so no two chains compute the same first step; 8 v_mov less
// per chain, but the copies also anchor the scheduler, and without them the kernels whose registers are full spill
// (the one-iteration kernel takes DIRECT: -64 v_mov per 16-step span, 149 -> 168 VGPRs, no spill in its loops;
// same box: its launch 6.13 -> 6.01 ms, 4-stream headline +1.7 %, profiles/r5/ab_direct)
template <int HI, int LO, bool DIRECT>
MI_HD inline void p2_beta_run_from(P2 (&v)[8], const P2 (&s)[8], const TdecX8P2& x) {
  if constexpr (DIRECT) {
    P2 nb[8];
    beta_step<false>(s, x.xs[HI], x.xp[HI], nb);
    p2_cp8(v, nb);
    p2_opaque8(v);
    if constexpr (HI > LO) p2_beta_run<HI - 1, LO>(v, x);
  } else {
    p2_cp8_opaque(v, s);
    p2_beta_run<HI, LO>(v, x);
  }
}
template <int LO, int HI, bool DIRECT>
MI_HD inline void p2_alpha_run_from(P2 (&v)[8], const P2 (&s)[8], const TdecX8P2& x) {
  if constexpr (DIRECT) {
    p2_cp8(v, s);
    alpha_fwd<false>(v, x.xs[LO], x.xp[LO]);
    p2_opaque8(v);
    if constexpr (HI > LO) p2_alpha_run<LO + 1, HI>(v, x);
  } else {
    p2_cp8_opaque(v, s);
    p2_alpha_run<LO, HI>(v, x);
  }
}
// wave F, phase 2, one pair: B(j) = beta_{base + j}, B(8) = the checkpoint; LLR i from alpha_i and B(i + 1).
// HAVE4: B(4) was computed on the way (a 16-step span's upper pair, TdecP2X::f2) and comes in B4in
template <bool DEC2, bool HAVE4 = false, bool DIRECT = false>
MI_HD inline void p2_alpha_window8(const TdecArgsP2& a, int lane, const TdecX8P2& x, const P2 (&B8)[8], uint32_t base,
                                   P2 (&al)[8], const P2 (&B4in)[8] = P2_NO_VEC) {
#define emit(I, BN) \
  p2_emit<DEC2>(a, lane, base, I, x.pk[I], alpha_step<false>(al, BN, x.xs[I], x.xp[I]), p2_emit_x8<DEC2>(x, I))
  if constexpr (DIRECT) {
    // sequential chains, every recomputed vector kept until its LLR (round 6): B(4) from B8 (or B4in), then B(3), B(2),
    // B(1) one step each from the last; after the first four LLRs B(7), B(6), B(5) the same way from B8 -- 10 recursion
    // steps per pair (6 with HAVE4) instead of 12 (8), one metric vector more live (5 instead of 4).  The chain to B(4)
    // and the one to B(7) start with the same step from B8, so the second starts from an opaque copy (GVN would
    // otherwise keep the first chain's B(7), B(6), B(5) live through the first four LLRs)
    P2 V4[8], V3[8], V2[8], V1[8];
    if constexpr (HAVE4) {
      p2_cp8_opaque(V4, B4in);
    } else {
      p2_beta_run_from<7, 4, true>(V4, B8, x);
      norm8<true>(V4);
    }
    p2_beta_run_from<3, 3, true>(V3, V4, x);
    p2_beta_run_from<2, 2, true>(V2, V3, x);
    p2_beta_run_from<1, 1, true>(V1, V2, x);
    MI_SCHED_FENCE();
    emit(0, V1);
    MI_SCHED_FENCE();
    emit(1, V2);
    MI_SCHED_FENCE();
    emit(2, V3);
    MI_SCHED_FENCE();
    emit(3, V4);
    norm8<true>(al);
    P2 V7[8], V6[8], V5[8];
    if constexpr (HAVE4) {
      p2_beta_run_from<7, 7, true>(V7, B8, x);
    } else {
      p2_cp8_opaque(V7, B8);
      p2_beta_run<7, 7>(V7, x);
    }
    p2_beta_run_from<6, 6, true>(V6, V7, x);
    p2_beta_run_from<5, 5, true>(V5, V6, x);
    MI_SCHED_FENCE();
    emit(4, V5);
    MI_SCHED_FENCE();
    emit(5, V6);
    MI_SCHED_FENCE();
    emit(6, V7);
    MI_SCHED_FENCE();
    emit(7, B8);
    norm8<true>(al);
    return;
  }
  P2 B4[8], Bm[8], Bt[8];
  // chains from B8: B(4) (without HAVE4) directly, B(6) and B(7) from copies; from B(4): B(3) directly, B(2) from a
  // copy; B(1) and B(5) directly from B(2) and B(6)
  if constexpr (HAVE4) {
    p2_cp8_opaque(B4, B4in);   // (opaque: also anchors the scheduler -- a plain copy costs 5 VGPRs here)
  } else {
    p2_beta_run_from<7, 4, DIRECT>(B4, B8, x);
    norm8<true>(B4);
  }
  p2_cp8_opaque(Bm, B4);
  p2_beta_run<3, 2>(Bm, x);   // B(2)
  p2_beta_run_from<1, 1, DIRECT>(Bt, Bm, x);   // B(1)
  MI_SCHED_FENCE();
  emit(0, Bt);
  MI_SCHED_FENCE();
  emit(1, Bm);
  p2_beta_run_from<3, 3, DIRECT>(Bt, B4, x);   // B(3)
  MI_SCHED_FENCE();
  emit(2, Bt);
  MI_SCHED_FENCE();
  emit(3, B4);
  norm8<true>(al);
  if constexpr (HAVE4) {
    p2_beta_run_from<7, 6, DIRECT>(Bm, B8, x);   // B(6): B8's only direct chain here
  } else {
    p2_cp8_opaque(Bm, B8);
    p2_beta_run<7, 6>(Bm, x);   // B(6)
  }
  p2_beta_run_from<5, 5, DIRECT>(Bt, Bm, x);   // B(5)
  MI_SCHED_FENCE();
  emit(4, Bt);
  MI_SCHED_FENCE();
  emit(5, Bm);
  p2_cp8_opaque(Bt, B8);
  p2_beta_run<7, 7>(Bt, x);   // B(7)
  MI_SCHED_FENCE();
  emit(6, Bt);
  MI_SCHED_FENCE();
  emit(7, B8);
  norm8<true>(al);
#undef emit
}
// LLR of step I from alpha_I (av) and the running beta_{I + 1}, then beta_I
template <bool DEC2, int I>
MI_HD inline void p2_llr_emit_back(const TdecArgsP2& a, int lane, const TdecX8P2& x, const P2 (&av)[8], uint32_t base,
                                   P2 (&b)[8]) {
  const P2 llr = llr_step(av, b, x.xs[I], x.xp[I]);
  p2_emit<DEC2>(a, lane, base, I, x.pk[I], llr, p2_emit_x8<DEC2>(x, I));
  P2 nb[8];
  beta_step<false>(b, x.xs[I], x.xp[I], nb);
  p2_cp8(b, nb);
}
// wave B, phase 2, one pair: A(j) = alpha_{base + j}, A(0) = the checkpoint (pair 0: the start state);
// LLR i from A(i) and beta_{base + i + 1} (the running b).  HAVE4: A(4) was computed on the way (a 16-step span's lower
// pair, TdecP2X::b2) and comes in A4in
template <bool DEC2, bool HAVE4 = false, bool DIRECT = false>
MI_HD inline void p2_beta_emit_window8(const TdecArgsP2& a, int lane, const TdecX8P2& x, const P2 (&A0)[8],
                                       uint32_t base, P2 (&b)[8], const P2 (&A4in)[8] = P2_NO_VEC) {
#define emit(I, AV) p2_llr_emit_back<DEC2, I>(a, lane, x, AV, base, b)
  if constexpr (DIRECT) {
    // the mirror of p2_alpha_window8's sequential chains: A(4) from A0 (or A4in), A(5), A(6), A(7) one step each; after
    // the LLRs of steps 7..4, A(1), A(2), A(3) from A0 (an opaque copy when the chain to A(4) started from A0 too)
    P2 V4[8], V5[8], V6[8], V7[8];
    if constexpr (HAVE4) {
      p2_cp8_opaque(V4, A4in);
    } else {
      p2_alpha_run_from<0, 3, true>(V4, A0, x);
      norm8<true>(V4);
    }
    p2_alpha_run_from<4, 4, true>(V5, V4, x);
    p2_alpha_run_from<5, 5, true>(V6, V5, x);
    p2_alpha_run_from<6, 6, true>(V7, V6, x);
    MI_SCHED_FENCE();
    emit(7, V7);
    MI_SCHED_FENCE();
    emit(6, V6);
    MI_SCHED_FENCE();
    emit(5, V5);
    MI_SCHED_FENCE();
    emit(4, V4);
    norm8<true>(b);
    P2 V1[8], V2[8], V3[8];
    if constexpr (HAVE4) {
      p2_alpha_run_from<0, 0, true>(V1, A0, x);
    } else {
      p2_cp8_opaque(V1, A0);
      p2_alpha_run<0, 0>(V1, x);
    }
    p2_alpha_run_from<1, 1, true>(V2, V1, x);
    p2_alpha_run_from<2, 2, true>(V3, V2, x);
    MI_SCHED_FENCE();
    emit(3, V3);
    MI_SCHED_FENCE();
    emit(2, V2);
    MI_SCHED_FENCE();
    emit(1, V1);
    MI_SCHED_FENCE();
    emit(0, A0);
    norm8<true>(b);
    return;
  }
  P2 A4[8], Am[8], At[8];
  // the mirror of p2_alpha_window8: from A0, A(4) (without HAVE4) directly, A(2) and A(1) from copies; from A(4), A(5)
  // directly, A(6) from a copy; A(7) and A(3) directly from A(6) and A(2)
  if constexpr (HAVE4) {
    p2_cp8_opaque(A4, A4in);   // (opaque: also anchors the scheduler -- a plain copy costs 5 VGPRs here)
  } else {
    p2_alpha_run_from<0, 3, DIRECT>(A4, A0, x);
    norm8<true>(A4);
  }
  p2_cp8_opaque(Am, A4);
  p2_alpha_run<4, 5>(Am, x);   // A(6)
  p2_alpha_run_from<6, 6, DIRECT>(At, Am, x);   // A(7)
  MI_SCHED_FENCE();
  emit(7, At);
  MI_SCHED_FENCE();
  emit(6, Am);
  p2_alpha_run_from<4, 4, DIRECT>(At, A4, x);   // A(5)
  MI_SCHED_FENCE();
  emit(5, At);
  MI_SCHED_FENCE();
  emit(4, A4);
  norm8<true>(b);
  if constexpr (HAVE4) {
    p2_alpha_run_from<0, 1, DIRECT>(Am, A0, x);   // A(2): A0's only direct chain here
  } else {
    p2_cp8_opaque(Am, A0);
    p2_alpha_run<0, 1>(Am, x);   // A(2)
  }
  p2_alpha_run_from<2, 2, DIRECT>(At, Am, x);   // A(3)
  MI_SCHED_FENCE();
  emit(3, At);
  MI_SCHED_FENCE();
  emit(2, Am);
  p2_cp8_opaque(At, A0);
  p2_alpha_run<0, 0>(At, x);   // A(1)
  MI_SCHED_FENCE();
  emit(1, At);
  MI_SCHED_FENCE();
  emit(0, A0);
  norm8<true>(b);
#undef emit
}

// ---- pipelining depths and checkpoint spacings -----------------------------------------------------
// q-row passes keep one window of loads in flight (two: 17 VGPRs spilled at the 3-waves-per-SIMD budget); the
// softbuffer passes follow tdec_body.h.  The check pass keeps two decision-row chunks in flight (three: 38 VGPRs
// spilled).
constexpr int P2_PF_Q = 1, P2_PF_SB = TDEC_PF_SB, P2_PF_CHK = 2;
// Checkpoint spacing (steps) of tdec_kernel_p2x: 16-step spans (the LDS stash below) in every launch.  Measured (round 5,
// profiles/r5/ab_ck16): 16-step spans cut the traffic of a headline launch from 22.8 to 19.5 GB (2.00 -> 1.70 x
// algorithmic) and leave its isolated time as it was (the decoder follows its instruction stream); configs[0] (8
// iterations) gains 9 %: 16.1 -> 17.6 Gbps.  Beside other streams' rate de-matching the stash's LDS matters: 38 rows per
// wavefront (19 KB per workgroup) left one co-resident rate de-matching workgroup per CU instead of three (4-stream
// headline -2 %); a one-iteration launch (the headline, the waterfall's first) never stashes DEC1's a-priori rows, and
// at 30 rows (15 KB) the 4-stream headline is unchanged (112.6 vs 112.8 Gbps over four interleaved pairs) and the
// waterfall gains 1 % (65.0 vs 64.4); without the quarter-point vector (23 rows, 12 KB) the 4 recomputed steps per
// span cost more than the LDS saves (111.3-112.1 Gbps).
constexpr int P2_CKS = 16;
// The waterfall continuation (tdec_kernel_p2c) runs few wavefronts (0.74 per SIMD at the 21.5 dB bench point), each a
// lone chain, so its spacing is a parameter of its own.  Its first round keeps 8-step checkpoints: 4-step ones (6
// recursion steps per 8 instead of 12) shorten a lone chain (one stream, same box: waterfall tdec 21.95 -> 21.25 ms)
// but move twice the checkpoint bytes, and beside the other streams' batches that costs more than it saves (4
// streams: 56.7-57.2 Gbps with 8-step checkpoints, 53.0-53.8 with 4-step ones; profiles/r4/ab_cont_ck).  The later
// re-compaction rounds hold a few dozen pairs, far below the HBM rate, and take 4-step checkpoints
// (profiles/r4/ab_ck_late: one stream waterfall tdec 18.58-18.61 -> 18.32 ms, headline unchanged).
constexpr int P2C_CKS = 8, P2C_CKS_LATE = 4;

// ---- 16-step checkpoint spacing (CKS = 16) ------------------------------------------------------
// Phase 1 stores a checkpoint every fourth window and phase 2 walks SPANS of four windows (two pairs) between them:
// half the checkpoint bytes of the 8-step form (20 of the ~141 KB per code block and iteration at the headline).  A
// span's midpoint vector -- the checkpoint the 8-step form would have loaded -- is recomputed on the way:
//   wave F (forward, closing checkpoint B16): the upper pair's inputs arrive first; B8 = 8 backward steps from B16,
//     normalised after each window exactly as phase 1 normalises before it stores a checkpoint; then the lower pair
//     runs against B8 and the upper pair against B16;
//   wave B (backward, opening checkpoint A0): the lower pair's inputs arrive first; A8 = 8 forward steps from A0,
//     normalised per window; then the upper pair runs against A8 and the lower pair against A0.
// The pair processed last needs inputs that were converted two pair-steps earlier: they wait in this wave's LDS stash
// (xs, xp, the DEC1 a-priori w: 24 rows of 64 words, + the span's checkpoint vector: 7 rows), not in registers (the
// 8-step form already uses the 168-VGPR budget of 3 waves per SIMD) and not re-read from HBM.  B8 / A8 are exactly
// the vectors phase 1 would have stored (the same deterministic recursion from the same normalised vector over the
// same inputs), and every pair then runs p2_alpha_window8 / p2_beta_emit_window8 as in the 8-step form, so every
// output is unchanged.  The quarter-point vector (B12 / A4) is normalised on the way to the midpoint and is the first
// vector the pair processed last recomputes: it is stashed too (7 more rows), so the extra cost is 4 recursion steps
// per 16 in phase 2 (28 + 16 instead of 24 + 16).
// Stash rows: xs, xp (2 x 8), the span's checkpoint vector (7), the quarter-point vector (7), DEC1's a-priori w (8;
// never in a one-iteration launch, whose passes are all FIRST: P2_STASH_ROWS_FIRST)
constexpr uint32_t P2_STASH_V = 2 * 2 * BETA_W, P2_STASH_V4 = P2_STASH_V + P2_CKW, P2_STASH_W = P2_STASH_V4 + P2_CKW,
                   P2_STASH_ROWS = P2_STASH_W + 2 * BETA_W, P2_STASH_ROWS_FIRST = P2_STASH_W;
MI_HD inline void p2_stash_st(uint32_t* st, uint32_t row, int lane, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  ((__attribute__((address_space(3))) uint32_t*)st)[row * LANES + (uint32_t)lane] = v;   // ds_write_b32: LDS
#else
  st[row * LANES + (uint32_t)lane] = v;
#endif
}
MI_HD inline uint32_t p2_stash_ld(const uint32_t* st, uint32_t row, int lane) {
#if defined(__HIP_DEVICE_COMPILE__)
  return ((const __attribute__((address_space(3))) uint32_t*)st)[row * LANES + (uint32_t)lane];
#else
  return st[row * LANES + (uint32_t)lane];
#endif
}
// park a pair's converted inputs and two normalised vectors (state 0 is 0): the span's checkpoint and the vector 4
// steps into the pair
template <bool DEC2, bool FIRST>
MI_HD inline void p2_stash_put(uint32_t* st, int lane, const TdecX8P2& x, const P2 (&v)[8], const P2 (&v4)[8]) {
#pragma unroll
  for (int i = 0; i < 2 * BETA_W; i++) {
    p2_stash_st(st, i, lane, p2_bits(x.xs[i]));
    p2_stash_st(st, 2 * BETA_W + i, lane, p2_bits(x.xp[i]));
    if constexpr (!DEC2 && !FIRST) p2_stash_st(st, P2_STASH_W + i, lane, p2_bits(x.w[i]));
  }
#pragma unroll
  for (int s = 1; s < 8; s++) {
    p2_stash_st(st, P2_STASH_V + s - 1, lane, p2_bits(v[s]));
    p2_stash_st(st, P2_STASH_V4 + s - 1, lane, p2_bits(v4[s]));
  }
}
// ... and take them back: DEC2's interleaver indices pi(k) (wave-uniform) come from the table again
template <bool DEC2, bool FIRST>
MI_HD inline void p2_stash_get(const TdecArgsP2& a, const uint32_t* st, int lane, uint32_t base, TdecX8P2& x,
                               P2 (&v)[8], P2 (&v4)[8]) {
#pragma unroll
  for (int i = 0; i < 2 * BETA_W; i++) {
    x.xs[i] = p2_from_bits(p2_stash_ld(st, i, lane));
    x.xp[i] = p2_from_bits(p2_stash_ld(st, 2 * BETA_W + i, lane));
    if constexpr (DEC2) x.pk[i] = MI_PI(a, base + i);
    else x.w[i] = FIRST ? Metric<P2>::zero() : p2_from_bits(p2_stash_ld(st, P2_STASH_W + i, lane));
  }
  v[0] = v4[0] = Metric<P2>::zero();
#pragma unroll
  for (int s = 1; s < 8; s++) {
    v[s] = p2_from_bits(p2_stash_ld(st, P2_STASH_V + s - 1, lane));
    v4[s] = p2_from_bits(p2_stash_ld(st, P2_STASH_V4 + s - 1, lane));
  }
}
// the tail's start vector (beta, wrapping adds) and the trellis start state (alpha, saturating adds: p2.h)
MI_HD inline void p2_start(P2 (&v)[8]) {
#pragma unroll
  for (int s = 0; s < 8; s++) v[s] = s ? Metric<P2>::ninf() : Metric<P2>::zero();
}
MI_HD inline void p2_start_alpha(P2 (&v)[8]) {
#pragma unroll
  for (int s = 0; s < 8; s++) v[s] = s ? Metric<P2>::ninf_alpha() : Metric<P2>::zero();
}

// the four phase bodies of one constituent decoder (tdec_body.h TdecX, register form)
// CKS: checkpoint spacing in steps (4, 8 or 16); PFQ: windows of q-row loads in flight.  The first launch takes
// P2_CKS / P2_PF_Q, the waterfall continuation its own (tdec_p2_lane)
template <bool DEC2, bool FIRST, int SRC, int CKS = P2_CKS, int PFQ = P2_PF_Q, bool DIRECT = false>
struct TdecP2X {
  static constexpr bool MKQ = !DEC2 && SRC == SRC_MKQ;
  static constexpr bool SQB = SRC == SRC_Q;    // backward-side passes read q rows
  static constexpr bool SQF = SRC != SRC_SB;   // forward-side passes read q rows
  static constexpr int PF = SRC == SRC_SB ? P2_PF_SB : PFQ;
  using Win = TdecWinP2;

  // Phase 2's traversal: wave F walks windows h .. nw - 1 upwards as 16-step spans (CKS = 16), then 8-step pairs,
  // then a lone last window; wave B walks windows h - 1 .. 0 downwards the same way (a lone window 0 last).  The
  // checkpoints phase 1 stores are exactly the ones these read: beta at every span / pair / window end above h (and
  // at nw, from the tail), alpha at every span / pair start below h except window 0 (the start state).
  MI_HD static uint32_t spans(uint32_t n) { return CKS == 16 ? n / 4 : 0u; }
  MI_HD static bool beta_ck(uint32_t w, uint32_t h, uint32_t nw) {   // h < w < nw
    if constexpr (CKS == 4) return true;
    const uint32_t w1 = h + 4 * spans(nw - h);
    return w <= w1 ? ((w - h) & 3u) == 0 : ((w - w1) & 1u) == 0;
  }
  MI_HD static bool alpha_ck(uint32_t w, uint32_t h) {   // 0 < w < h
    if constexpr (CKS == 4) return true;
    const uint32_t wlo = h - 4 * spans(h);
    return w >= wlo ? ((h - w) & 3u) == 0 : ((wlo - w) & 1u) == 0;
  }
  // a pair's loads: windows w0, w0 + 1 and (CK) the checkpoint in slot c
  MI_HD static void load8(const TdecArgsP2& a, int lane, uint32_t w0, uint32_t c, bool with_ck, TdecWin8P2& r) {
    p2_load_window<DEC2, FIRST, SQF>(a, lane, w0 * BETA_W, r.lo);
    p2_load_window<DEC2, FIRST, SQF>(a, lane, (w0 + 1) * BETA_W, r.hi);
    if (with_ck) p2_ck_load_to(a.scr, (size_t)2 * a.K, c, lane, r.ck);
  }

  MI_HD static void load1(const TdecArgsP2& a, int lane, uint32_t w, Win& r) {
    if constexpr (MKQ) p2_load_window_mkq<FIRST>(a, lane, w * BETA_W, r);
    else p2_load_window<DEC2, FIRST, SQB>(a, lane, w * BETA_W, r);
  }
  // wave F, phase 1: alpha_0 .. alpha_{K/2}, the alpha checkpoints phase 2 of wave B reads
  MI_P2_INL static void f1(const TdecArgsP2& a, int lane, P2 (&al)[8]) {
    const uint32_t h = a.K / (2 * BETA_W);
    const size_t ck = (size_t)2 * a.K;
    p2_start_alpha(al);
    pipe_windows<PF, Win>(
        (int)h, [](int i) { return (uint32_t)i; }, [&](uint32_t w, Win& r) { load1(a, lane, w, r); },
        [&](const Win& r, uint32_t w) {
          if (w && alpha_ck(w, h)) p2_ck_store(a.scr, ck, w, lane, al);
          if constexpr (MKQ) p2_alpha_only_window_mkq(a, lane, r, w * BETA_W, al);
          else p2_alpha_only_window<DEC2, SQB>(a, r, w * BETA_W, al);
        });
  }
  // wave F, phase 2: windows h .. nw - 1, LLRs of steps K/2 .. K - 1
  MI_P2_INL static void f2(const TdecArgsP2& a, int lane, P2 (&al)[8]) {
    const uint32_t nw = a.K / BETA_W, h = nw / 2;
    const size_t ck = (size_t)2 * a.K;
    if constexpr (CKS >= 8) {
      const uint32_t ns = spans(nw - h), w1 = h + 4 * ns;
      if (ns) {
        // span j: windows w0 .. w0 + 3 (w0 = h + 4 j), closing checkpoint w0 + 4.  The upper pair (and the checkpoint)
        // is loaded first; the loads of the next span's upper pair are in flight through this span's two pairs
        TdecWin8P2 r;
        load8(a, lane, h + 2, h + 4, true, r);
        for (uint32_t j = 0; j < ns; j++) {
          const uint32_t w0 = h + 4 * j;
          TdecX8P2 x;
          P2 B16[8], B8[8];
          p2_cvt8<DEC2, SQF>(a, r, (w0 + 2) * BETA_W, x);
          p2_ck_vec(r.ck, B16);
          MI_SCHED_FENCE();
          load8(a, lane, w0, 0, false, r);   // the lower pair
          MI_SCHED_FENCE();
          p2_beta_run_from<7, 4, true>(B8, B16, x);   // B16's only chain in registers (the stash keeps B16)
          norm8<true>(B8);   // B12: the upper pair's "B(4)", stashed with its inputs
          p2_stash_put<DEC2, FIRST>(a.stash, lane, x, B16, B8);
          p2_beta_run<3, 0>(B8, x);
          norm8<true>(B8);
          MI_SCHED_FENCE();
          p2_cvt8<DEC2, SQF>(a, r, w0 * BETA_W, x);
          MI_SCHED_FENCE();
          const uint32_t wn = j + 1 < ns ? w0 + 6 : w0 + 2;   // the last span reloads its upper pair (unused)
          load8(a, lane, wn, wn + 2, true, r);
          MI_SCHED_FENCE();
          p2_alpha_window8<DEC2, false, DIRECT>(a, lane, x, B8, w0 * BETA_W, al);
          MI_SCHED_FENCE();
          p2_stash_get<DEC2, FIRST>(a, a.stash, lane, (w0 + 2) * BETA_W, x, B16, B8);
          p2_alpha_window8<DEC2, true, DIRECT>(a, lane, x, B16, (w0 + 2) * BETA_W, al, B8);
        }
      }
      // pairs (w1 + 2j, w1 + 2j + 1), beta checkpoint w1 + 2j + 2; an odd count leaves window nw - 1 alone
      const uint32_t n = nw - w1, np = n / 2;
      if (np) {
        TdecWin8P2 r;
        load8(a, lane, w1, w1 + 2, true, r);
        for (uint32_t j = 0; j < np; j++) {
          const uint32_t w0 = w1 + 2 * j;
          TdecX8P2 x;
          P2 B8[8];
          p2_cvt8<DEC2, SQF>(a, r, w0 * BETA_W, x);
          p2_ck_vec(r.ck, B8);
          MI_SCHED_FENCE();
          const uint32_t wn = j + 1 < np ? w0 + 2 : w0;   // the last pair reloads itself (unused)
          load8(a, lane, wn, wn + 2, true, r);
          MI_SCHED_FENCE();
          p2_alpha_window8<DEC2, false, DIRECT>(a, lane, x, B8, w0 * BETA_W, al);
        }
      }
      if (n & 1u) {
        Win r;
        p2_load_window<DEC2, FIRST, SQF>(a, lane, (nw - 1) * BETA_W, r);
        p2_ck_load(a.scr, ck, nw, lane, r);
        p2_alpha_window<DEC2, SQF>(a, lane, r, (nw - 1) * BETA_W, al);
      }
    } else {
      pipe_windows<PF, Win>(
          (int)(nw - h), [h](int i) { return h + (uint32_t)i; },
          [&](uint32_t w, Win& r) {
            p2_load_window<DEC2, FIRST, SQF>(a, lane, w * BETA_W, r);
            p2_ck_load(a.scr, ck, w + 1, lane, r);
          },
          [&](const Win& r, uint32_t w) { p2_alpha_window<DEC2, SQF>(a, lane, r, w * BETA_W, al); });
    }
  }
  // wave B, phase 1: tail, then beta_K .. beta_{K/2}, the beta checkpoints phase 2 of wave F reads
  MI_P2_INL static void b1(const TdecArgsP2& a, int lane, P2 (&b)[8]) {
    const uint32_t K = a.K, nw = K / BETA_W, h = nw / 2;
    const size_t ck = (size_t)2 * K;
    p2_start(b);
    {
      const uint32_t t0 = 3 * K + (DEC2 ? 6 : 0);
      P2 tx[3], tp[3];
      if constexpr (MKQ) {
        // all 12 tail inputs (both constituent codes) quantised into their q rows
        const uint32_t ma = p2_wmask(a, 0, nw), mb = p2_wmask(a, 1, nw);
        const PosW PT = MI_POSW(a, 3 * K);
#pragma unroll
        for (int j = 0; j < 12; j++) {
          const P2 q = q16_pair(p2_sb_in(a, 0, ma, PT, j, lane), p2_sb_in(a, 1, mb, PT, j, lane));
          row_st(a.q, 3 * K, lane, p2_bits(q), j);
          if (j < 6) { if (j & 1) tp[j / 2] = q; else tx[j / 2] = q; }
        }
      } else if constexpr (!SQB) {
        const uint32_t ma = p2_wmask(a, 0, nw), mb = p2_wmask(a, 1, nw);
        const PosW PT = MI_POSW(a, 3 * K);
#pragma unroll
        for (int j = 0; j < 3; j++) {
          const uint32_t d = t0 - 3 * K + 2 * j;
          tx[j] = q16_pair(p2_sb_in(a, 0, ma, PT, d, lane), p2_sb_in(a, 1, mb, PT, d, lane));
          tp[j] = q16_pair(p2_sb_in(a, 0, ma, PT, d + 1, lane), p2_sb_in(a, 1, mb, PT, d + 1, lane));
        }
      } else {
#pragma unroll
        for (int j = 0; j < 3; j++) {
          tx[j] = p2_from_bits(row_ld(a.q, t0, lane, 2 * j));
          tp[j] = p2_from_bits(row_ld(a.q, t0, lane, 2 * j + 1));
        }
      }
#pragma unroll
      for (int j = 2; j >= 0; j--) {
        P2 nb[8];
        beta_step<false>(b, tx[j], tp[j], nb);
#pragma unroll
        for (int s = 0; s < 8; s++) b[s] = nb[s];
      }
      norm8<true>(b);
    }
    p2_ck_store(a.scr, ck, nw, lane, b);
    pipe_windows<PF, Win>(
        (int)(nw - h), [nw](int i) { return nw - 1 - (uint32_t)i; }, [&](uint32_t w, Win& r) { load1(a, lane, w, r); },
        [&](const Win& r, uint32_t w) {
          if constexpr (MKQ) p2_beta_window_mkq(a, lane, r, w * BETA_W, b);
          else p2_beta_window<DEC2, SQB>(a, r, w * BETA_W, b);
          if (w > h && beta_ck(w, h, nw)) p2_ck_store(a.scr, ck, w, lane, b);
        });
  }
  // wave B, phase 2: windows h - 1 .. 0 backward, LLRs of steps 0 .. K/2 - 1
  MI_P2_INL static void b2(const TdecArgsP2& a, int lane, P2 (&b)[8]) {
    const uint32_t h = a.K / (2 * BETA_W);
    const size_t ck = (size_t)2 * a.K;
    if constexpr (CKS >= 8) {
      const uint32_t ns = spans(h), wlo = h - 4 * ns;
      if (ns) {
        // span j: windows w0 .. w0 + 3 (w0 = h - 4 j - 4), opening checkpoint w0 (w0 = 0: the start state).  The lower
        // pair (and the checkpoint) is loaded first
        TdecWin8P2 r;
        load8(a, lane, h - 4, h - 4, true, r);   // w0 = 0: slot 0 is loaded but not used
        for (uint32_t j = 0; j < ns; j++) {
          const uint32_t w0 = h - 4 * j - 4;
          TdecX8P2 x;
          P2 A0[8], A8[8];
          p2_cvt8<DEC2, SQF>(a, r, w0 * BETA_W, x);
          if (w0) p2_ck_vec(r.ck, A0);
          else p2_start_alpha(A0);
          MI_SCHED_FENCE();
          load8(a, lane, w0 + 2, 0, false, r);   // the upper pair
          MI_SCHED_FENCE();
          p2_alpha_run_from<0, 3, true>(A8, A0, x);   // A0's only chain in registers (the stash keeps A0)
          norm8<true>(A8);   // A4: the lower pair's "A(4)", stashed with its inputs
          p2_stash_put<DEC2, FIRST>(a.stash, lane, x, A0, A8);
          p2_alpha_run<4, 7>(A8, x);
          norm8<true>(A8);
          MI_SCHED_FENCE();
          p2_cvt8<DEC2, SQF>(a, r, (w0 + 2) * BETA_W, x);
          MI_SCHED_FENCE();
          const uint32_t wn = j + 1 < ns ? w0 - 4 : w0;   // the last span reloads its lower pair (unused)
          load8(a, lane, wn, wn, true, r);
          MI_SCHED_FENCE();
          p2_beta_emit_window8<DEC2, false, DIRECT>(a, lane, x, A8, (w0 + 2) * BETA_W, b);
          MI_SCHED_FENCE();
          p2_stash_get<DEC2, FIRST>(a, a.stash, lane, w0 * BETA_W, x, A0, A8);
          p2_beta_emit_window8<DEC2, true, DIRECT>(a, lane, x, A0, w0 * BETA_W, b, A8);
        }
      }
      // pairs (wlo - 2j - 2, wlo - 2j - 1), alpha checkpoint wlo - 2j - 2 (0: the start state); an odd wlo leaves
      // window 0 alone
      const uint32_t np = wlo / 2;
      if (np) {
        TdecWin8P2 r;
        load8(a, lane, wlo - 2, wlo - 2, true, r);   // w0 = 0: slot 0 is loaded but not used
        for (uint32_t j = 0; j < np; j++) {
          const uint32_t w0 = wlo - 2 * j - 2;
          TdecX8P2 x;
          P2 A0[8];
          p2_cvt8<DEC2, SQF>(a, r, w0 * BETA_W, x);
          if (w0) p2_ck_vec(r.ck, A0);
          else p2_start_alpha(A0);
          MI_SCHED_FENCE();
          const uint32_t wn = j + 1 < np ? w0 - 2 : w0;   // the last pair reloads itself (unused)
          load8(a, lane, wn, wn, true, r);
          MI_SCHED_FENCE();
          p2_beta_emit_window8<DEC2, false, DIRECT>(a, lane, x, A0, w0 * BETA_W, b);
        }
      }
      if (wlo & 1u) {
        Win r;
        p2_load_window<DEC2, FIRST, SQF>(a, lane, 0, r);
        p2_beta_emit_window<DEC2, SQF, true>(a, lane, r, 0, b);
      }
    } else {
      pipe_windows<PF, Win>(
          (int)h, [h](int i) { return h - 1 - (uint32_t)i; },
          [&](uint32_t w, Win& r) {
            p2_load_window<DEC2, FIRST, SQF>(a, lane, w * BETA_W, r);
            p2_ck_load(a.scr, ck, w, lane, r);   // window 0: slot 0 is loaded but not used
          },
          [&](const Win& r, uint32_t w) {
            if (w) p2_beta_emit_window<DEC2, SQF, false>(a, lane, r, w * BETA_W, b);
            else p2_beta_emit_window<DEC2, SQF, true>(a, lane, r, 0, b);
          });
    }
  }
};

template <bool DEC2, bool FIRST, int SRC, int CKS = P2_CKS, int PFQ = P2_PF_Q, bool DIRECT = false, class Exec>
MI_P2_INL void tdec_p2_xhalf(const TdecArgsP2& a, int lane, Exec& ex) {
  using X = TdecP2X<DEC2, FIRST, SRC, CKS, PFQ, DIRECT>;
  P2 mF[8], mBs[8];
  P2(&mB)[8] = Exec::SHARED ? mF : mBs;   // GPU: each wave holds only its own metric
  ex.run([&] { X::f1(a, lane, mF); }, [&] { X::b1(a, lane, mB); });
  ex.run([&] { X::f2(a, lane, mF); }, [&] { X::b2(a, lane, mB); });
}

// The pass after an iteration (wave F; tdec_body.h tdec_pack is the one-code-block form): for every half in
// `act` (still iterating), pack its decision bits MSB first into its output row, run the bytes through the
// code block's own CRC register -- CRC24A for a one-code-block TB, else CRC24B, the register of the whole
// K-bit block (filler bits included, as the oracle checks it) is 0 iff the CRC passes -- and through the
// partial TB CRC24A of its payload bytes F/8 .. K/8 - (CB CRC ? 3 : 0) that tb_kernel combines.  Returns
// bit h = half h's code-block CRC passed.  (The byte-wise register of a K-bit block equals the XOR of the
// per-bit contributions crc_a / crc_b[k] the one-code-block kernels accumulate: CRC is linear.)
// The payload bytes go out as aligned dword stores (a byte store per payload byte and half put 64 code blocks' lines
// under every store instruction for one byte each: 0.5 ms of a 6.6 ms launch, profiles/r4/diag_pay).
// Measured and not kept: the pass split over both waves (wave B waits at the barrier otherwise; the registers combine
// by linearity, R(A || B) = R(A) x^(8 |B|) ^ R(B)): more scalar spills, one stream 6.47-6.51 -> 6.50-6.65 ms, four
// streams 112.3-113.0 -> 110.5-110.9 Gbps (profiles/r4/ab_split_chk), although the pass alone costs 0.45 ms.
struct P2CrcRegs { uint32_t cb[2], tb[2]; };
MI_P2_INL uint32_t tdec_p2_check(const TdecArgsP2& a, int lane, uint32_t act, uint32_t (&tbp)[2]) {
  uint32_t bl[2], bh[2];
  P2CrcRegs g{{0u, 0u}, {0u, 0u}};
  const uint32_t* ct[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    bl[h] = a.F[h] / 8;
    bh[h] = a.K / 8 - ((a.crc24a[h] & 1u) ? 0 : 3);
    ct[h] = (a.crc24a[h] & 1u) ? a.crc8 : a.crc8b;
  }
  const uint32_t nb = a.K / 8, c1 = (nb + 3) / 4;
  constexpr uint32_t c0 = 0;
  // the decision rows of 4 bytes (32 rows) per chunk, P2_PF_CHK chunks' loads in flight ahead of the chunk whose
  // bits are used (the trellis registers are dead here); rows past K are clamped to row K - 1 and their bytes never
  // used
  struct Chunk { uint32_t d[32]; };
  auto load = [&](uint32_t c, Chunk& dd) {
#pragma unroll
    for (int q = 0; q < 32; q++) {
      const uint32_t row = 32 * c + (uint32_t)q;
      dd.d[q] = row_ld(a.dec, row < a.K ? row : a.K - 1, lane);
    }
  };
  // payload bytes of half h: j in [jlo, jhi) -- F/8 .. the CB CRC, less the TB CRC where the code block carries it
  // (tb_kernel's run) -- at out_bytes[p2_run_off(a, h) + j]; every byte of a code-block row otherwise
  // run[h] = m | (jlo + m) << 4 | (jhi + m) << 16 (one register per half; m = the misalignment of byte 0 of the run,
  // the same for every chunk; byte j lies in the run iff jlo + m <= j + m < jhi + m)
  uint32_t rng[2], wprev[2] = {0u, 0u};
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint32_t jlo = a.to_payload ? bl[h] : 0u, jhi = a.to_payload ? bh[h] - 3 * ((a.crc24a[h] >> 1) & 1u) : nb;
    const uint32_t m = ((uint32_t)(uintptr_t)a.out_bytes + (uint32_t)p2_run_off(a, h)) & 3u;   // (mod 4: wraps)
    rng[h] = m | ((jlo + m) << 4) | ((jhi + m) << 16);
  }
  auto run = [&](const Chunk& dd, uint32_t c) {
    uint32_t w[2] = {0u, 0u};   // the chunk's 4 bytes per half, little-endian (byte 4c in bits 0..7)
#pragma unroll
    for (int jj = 0; jj < 4; jj++) {
      const uint32_t j = 4 * c + (uint32_t)jj;
      if (j >= nb) break;   // wave-uniform
      // rows 8 jj .. 8 jj + 7, MSB first: four rows at a time give half 0's 4 bits in bits 3..0 and half 1's in 7..4
      // (decision byte = b0 | b1 << 4, p2_emit)
      const uint32_t* r8 = &dd.d[8 * jj];
      const uint32_t xa = (r8[0] << 3) | (r8[1] << 2) | (r8[2] << 1) | r8[3];
      const uint32_t xb = (r8[4] << 3) | (r8[5] << 2) | (r8[6] << 1) | r8[7];
      const uint32_t v0 = ((xa & 0xFu) << 4) | (xb & 0xFu), v1 = (xa & 0xF0u) | (xb >> 4);
      w[0] |= v0 << (8 * jj);
      w[1] |= v1 << (8 * jj);
      g.cb[0] = ((g.cb[0] << 8) & 0xFFFFFFu) ^ ct[0][((g.cb[0] >> 16) ^ v0) & 0xFFu];
      g.cb[1] = ((g.cb[1] << 8) & 0xFFFFFFu) ^ ct[1][((g.cb[1] >> 16) ^ v1) & 0xFFu];
      if (j >= bl[0] && j < bh[0]) g.tb[0] = ((g.tb[0] << 8) & 0xFFFFFFu) ^ a.crc8[((g.tb[0] >> 16) ^ v0) & 0xFFu];
      if (j >= bl[1] && j < bh[1]) g.tb[1] = ((g.tb[1] << 8) & 0xFFFFFFu) ^ a.crc8[((g.tb[1] >> 16) ^ v1) & 0xFFu];
    }
#pragma unroll
    for (int h = 0; h < 2; h++) {
      if (!((act >> h) & 1u)) continue;
      const int64_t off = p2_run_off(a, h);   // byte j at out_bytes[off + j], j in the run
      // aligned dword stores: the chunk's bytes sit at 4c + m .. 4c + m + 3 (mod 4); it completes the dword at 4c - m
      // (the previous chunk's last m bytes and its first 4 - m), written whole when it lies inside the run and the
      // previous chunk is in this range; the bytes of a dword that is not (the run's and the range's edges) go one
      // by one.  Every byte is written exactly once, only inside the run (the neighbouring code blocks' bytes are
      // untouched).
      const uint32_t m = rng[h] & 3u, lo = (rng[h] >> 4) & 0xFFFu, hi = rng[h] >> 16;
      // the dword at byte 4c - m, i.e. at 4c .. 4c + 3 in the shifted index
      const bool full0 = c > c0 && 4 * c >= lo && 4 * c + 4 <= hi;
      const bool full1 = c + 1 < c1 && 4 * c + 4 >= lo && 4 * c + 8 <= hi;   // the next chunk writes it
      if (full0) {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t v = m ? __builtin_amdgcn_alignbyte(w[h], wprev[h], 4 - m) : w[h];
#else
        const uint32_t v = m ? (uint32_t)((((uint64_t)w[h] << 32) | wprev[h]) >> (8 * (4 - m))) : w[h];
#endif
        *reinterpret_cast<uint32_t*>(a.out_bytes + (off + (int64_t)(4 * c) - (int64_t)m)) = v;
      }
      // uncovered bytes lie in the range's first 3 chunks (jlo + m < 11) and its last 5 (hi >= nb - 6), a
      // wave-uniform test
      if (c < c0 + 3 || c + 5 >= c1) {
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const uint32_t j = 4 * c + (uint32_t)b;
          const bool covered = (uint32_t)b < 4 - m ? full0 : full1;
          if (j + m >= lo && j + m < hi && !covered) a.out_bytes[off + (int64_t)j] = (uint8_t)(w[h] >> (8 * b));
        }
      }
      wprev[h] = w[h];
    }
  };
  if (c1 > c0)
    pipe_windows<P2_PF_CHK, Chunk>((int)c1, [](int i) { return (uint32_t)i; }, load, run);
  if (act & 1u) tbp[0] = g.tb[0];
  if (act & 2u) tbp[1] = g.tb[1];
  return (g.cb[0] == 0u ? 1u : 0u) | (g.cb[1] == 0u ? 2u : 0u);
}

// the iteration loop (tdec_body.h tdec_lane_x's source-mode sequence) with per-code-block stopping.
// ex.pack_wave is true on the wave that runs tdec_p2_check (GPU: wave F, after the iteration's barrier;
// host: always); ex.share hands its verdicts to the other wave.  With early stop off (configs[0]'s fixed
// iteration count) only the last iteration's pass runs.
// CONT (waterfall compaction, tdec.hip): the code blocks continue from iteration 1 in a dense continuation
// pair whose q rows and extrinsic rows were gathered after iteration 0 -- every pass reads q rows.
// CKS: the checkpoint spacing of every pass (the first launch: P2_CKS; the continuation: P2C_CKS or
// P2C_CKS_LATE, tdec.hip tdec_kernel_p2c)
// ONE: a launch of one iteration (a.max_its == 1; tdec.hip tdec_kernel_p2x<true>): only iteration 0's passes are built.
// MK: the iteration whose DEC1 pass creates the packed q rows (TDEC_MKQ_IT: only once a second iteration runs; 0 for a
// fixed iteration count without early stop -- configs[0] -- where every later iteration reads them: +2.9 %,
// profiles/r5/ab_misc)
template <bool CONT = false, int CKS = P2_CKS, bool ONE = false, uint32_t MK = TDEC_MKQ_IT, class Exec>
MI_P2_INL TdecP2Result tdec_p2_lane(const TdecArgsP2& a, int lane, Exec& ex) {
  TdecP2Result r{{0u, 0u}, {0u, 0u}, {0u, 0u}};
  uint32_t active = a.live & 3u;
  if constexpr (ONE && !CONT) {
    tdec_p2_xhalf<false, true, SRC_SB, CKS, P2_PF_Q, true>(a, lane, ex);   // direct recomputation chains
    tdec_p2_xhalf<true, true, SRC_SB, CKS, P2_PF_Q, true>(a, lane, ex);
    uint32_t ok = 0u;
    if (ex.pack_wave()) ok = tdec_p2_check(a, lane, active, r.tb_part);
    ok = ex.share(ok, lane);
#pragma unroll
    for (int h = 0; h < 2; h++) {
      if (!((active >> h) & 1u)) continue;
      r.its[h] = 1u;
      r.crc_ok[h] = (ok >> h) & 1u;
    }
    return r;
  }
  // CONT: iteration 0 ran with no_w (no extrinsic rows); its DEC2 pass is re-run here from the gathered q rows
  // and DEC1 outputs (x2 rows) -- the same integers as in iteration 0 -- to form the w rows iteration 1 reads
  if constexpr (CONT)
    if (!a.cont_w && a.it0 == 1) tdec_p2_xhalf<true, false, SRC_Q, CKS>(a, lane, ex);
  for (uint32_t it = CONT ? a.it0 : 0u; it < (CONT ? a.it_end : a.max_its) && active; it++) {
    if constexpr (CONT) {
      tdec_p2_xhalf<false, false, SRC_Q, CKS>(a, lane, ex);
      tdec_p2_xhalf<true, false, SRC_Q, CKS>(a, lane, ex);
    } else if (it == 0) {
      if (MK == 0) {
        // fixed iteration count (configs[0]): direct recomputation chains in every pass -- 20 VGPRs spill, but only
        // around the iteration loop; span loops -7.5 % VALU, one launch 29.8-29.9 -> 27.9 ms (profiles/r6/ab_fixed)
        tdec_p2_xhalf<false, true, SRC_MKQ, CKS, P2_PF_Q, true>(a, lane, ex);
        tdec_p2_xhalf<true, true, SRC_Q, CKS, P2_PF_Q, true>(a, lane, ex);
      } else {
        tdec_p2_xhalf<false, true, SRC_SB, CKS>(a, lane, ex);
        tdec_p2_xhalf<true, true, SRC_SB, CKS>(a, lane, ex);
      }
    } else if (it < MK) {
      tdec_p2_xhalf<false, false, SRC_SB, CKS>(a, lane, ex);
      tdec_p2_xhalf<true, false, SRC_SB, CKS>(a, lane, ex);
    } else if (it == MK) {
      tdec_p2_xhalf<false, false, SRC_MKQ, CKS>(a, lane, ex);
      tdec_p2_xhalf<true, false, SRC_Q, CKS>(a, lane, ex);
    } else {
      tdec_p2_xhalf<false, false, SRC_Q, CKS, P2_PF_Q, MK == 0>(a, lane, ex);
      tdec_p2_xhalf<true, false, SRC_Q, CKS, P2_PF_Q, MK == 0>(a, lane, ex);
    }
    const bool last = it + 1 == a.max_its;
    uint32_t ok = 0u;
    if (a.early_stop || last) {   // wave-uniform
      if (ex.pack_wave()) ok = tdec_p2_check(a, lane, active, r.tb_part);
      ok = ex.share(ok, lane);
    }
    uint32_t stop = 0u;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      if (!((active >> h) & 1u)) continue;
      r.its[h] = it + 1;
      r.crc_ok[h] = (ok >> h) & 1u;
      if ((a.early_stop && r.crc_ok[h]) || last) stop |= 1u << h;
    }
    active &= ~stop;
  }
  return r;
}

// ---- waterfall compaction (tdec.hip tdec_cont_*, emu.cpp) ---------------------------------------------
// At 21.5 dB most code blocks pass their CRC after iteration 0 and the lanes that go on iterate in
// sparse wavefronts (a pair's cost is its slowest code block).  With early stop the decode therefore runs
// iteration 0 over all pairs, then gathers the code blocks whose CRC failed into dense continuation
// pairs and runs iterations 1.. there (tdec_p2_lane<true>).  The gather builds exactly the state
// iteration 1 reads: the packed q rows that the SRC_MKQ pass would create (window masks applied:
// unmaterialised rows are the group's zero row, i.e. q = 0) and the iteration-0 extrinsic rows w -- formed by
// re-running iteration 0's DEC2 pass on the gathered iteration-0 DEC1 outputs (x2 rows), because the
// one-iteration first launch stores no w rows (no_w: 12 KB per code block less at the headline, where no code
// block continues); llr1, checkpoints and decisions are rewritten by every iteration.  The two halves of a lane never interact,
// so which code blocks share a continuation lane does not change any result.
// Continuation pair layout = the pair scratch layout: w rows at 0, q rows at (4K + 8) rows.  The gather
// goes by q window (12 rows: one window-mask word per source) and by w row.
struct P2ContSrc {
  const float* sb;      // the code block's group softbuffer
  const uint32_t* wm;   // the group's window masks
  const uint32_t* scr;  // the scratch of the group's pair (w rows: packed, this code block = half hs)
  uint32_t ls, hs;      // lane in the group, half in the pair
};
MI_HD inline uint32_t p2_cont_qwins(uint32_t K) { return K / BETA_W + 1; }   // 3 (K + 4) q rows, incl. the tail
// q rows 12 w .. 12 w + 11 of one continuation lane (both halves), packed
MI_HD inline void p2_cont_qwin(const P2ContSrc (&s)[2], uint32_t live, const uint32_t* pos, uint32_t w,
                               uint32_t (&q)[3 * BETA_W]) {
  uint32_t m[2];
#pragma unroll
  for (int h = 0; h < 2; h++) m[h] = ((live >> h) & 1u) ? s[h].wm[w] : 0u;
  float v[3 * BETA_W][2];
#pragma unroll
  for (int i = 0; i < 3 * BETA_W; i++) {
    const size_t row = 3 * BETA_W * w + i;   // rows in decoder-input order
#pragma unroll
    for (int h = 0; h < 2; h++) v[i][h] = ((m[h] >> i) & 1u) ? s[h].sb[row * LANES + s[h].ls] : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 3 * BETA_W; i++) q[i] = p2_bits(q16_pair(v[i][0], v[i][1]));
}
// packed row `row` of one continuation lane from its sources' packed rows (each half's 16 bits from its source pair's
// row, half hs): the w rows (at 0) after a first launch that stored them, and every row of a re-compaction round
MI_HD inline uint32_t p2_cont_drow(const P2ContSrc (&s)[2], uint32_t live, size_t row) {
  uint32_t w[2];
#pragma unroll
  for (int h = 0; h < 2; h++)
    w[h] = ((live >> h) & 1u) ? (s[h].scr[row * LANES + s[h].ls] >> (16 * s[h].hs)) & 0xFFFFu : 0u;
  return w[0] | (w[1] << 16);
}
MI_HD inline uint32_t p2_cont_wrow(const P2ContSrc (&s)[2], uint32_t live, uint32_t k) { return p2_cont_drow(s, live, k); }
// x2 row k (the llr1 rows, at K) of one continuation lane: each half's 16-bit iteration-0 DEC1 output from its
// source pair's packed row
MI_HD inline uint32_t p2_cont_xrow(const P2ContSrc (&s)[2], uint32_t live, uint32_t K, uint32_t k) {
  uint32_t w[2];
#pragma unroll
  for (int h = 0; h < 2; h++)
    w[h] = ((live >> h) & 1u) ? (s[h].scr[(size_t)(K + k) * LANES + s[h].ls] >> (16 * s[h].hs)) & 0xFFFFu : 0u;
  return w[0] | (w[1] << 16);
}

// ---- segmented continuation: the late re-compaction rounds of the waterfall (tdec.hip tdec_kernel_p2s) ----------
// A round after the first holds a few dozen dense pairs (21.5 dB: 84, then 19), far under one wavefront per SIMD, and
// each pair's iteration is a lone chain of 4 x K/2 dependent trellis steps per wavefront in the crossed schedule
// (~3 ms whatever the pair count).  Here one dense pair is decoded by S wavefronts, wavefront j owning the trellis
// segment [a, e) = [j L, min((j + 1) L, K)) (L a multiple of 8 steps) in BOTH recursions of both constituent
// decoders -- a chain of 4 K / S steps -- and the segments are made exact exactly as the latency form's threads are
// (tdec_win_body.h): in the int16 design a recursion started from a GUESSED normalised vector reproduces the true one
// from the first step where the two coincide, so
//   backward: every segment runs beta from a guess (the last one from the tail) and stores a checkpoint every 8 steps
//     and its left-end vector; then fix-up rounds: a segment whose right neighbour's left-end vector differs from
//     the vector it started from restarts from it and re-walks until a recomputed vector EQUALS the stored one (all
//     lanes: the re-walk is wave-uniform) or its left end changes (the next round re-checks its left neighbour);
//   forward: the same with alpha (the first segment from the start state), emitting the half-iteration's outputs
//     (DEC1: x2 rows; DEC2: extrinsic rows and decision bytes) from alpha and the final betas; a fix-up re-emits
//     exactly the steps whose alpha changed.
// Rounds end when no boundary changed (a workgroup-wide OR).  Every value that survives is the full-length
// recursion's, so the outputs equal tdec_p2_lane<true>'s (and the oracle's).  Checkpoints: beta at step 8c in slot c,
// alpha at step 8c in slot K/8 + 1 + c of the pair's checkpoint region (interior steps of a segment only: both fit its
// K/4 + 1 slots); the boundary vectors live in LDS (4 x [S][7][64] words): bvec[j] = the beta segment j started
// from (at e), bend[j] = its beta at a; avec[j] / aend[j] = its alpha at a / at e.
constexpr uint32_t P2S_SPAN = 2 * BETA_W;   // checkpoint spacing of both directions (steps)
struct P2Seg { uint32_t j, nseg, a, e; };
MI_HD inline P2Seg p2s_seg(uint32_t K, uint32_t S, uint32_t j) {
  const uint32_t L = (K + P2S_SPAN * S - 1) / (P2S_SPAN * S) * P2S_SPAN;
  P2Seg g;
  g.j = j;
  g.nseg = (K + L - 1) / L;
  g.a = j * L < K ? j * L : K;
  g.e = g.a + L < K ? g.a + L : K;
  return g;
}
// wave-uniform: every lane's predicate (GPU: all active lanes; host: the one lane emulated)
MI_HD inline bool p2_all(bool v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_ballot_w64(!v) == 0;
#else
  return v;
#endif
}
MI_HD inline bool p2_vec_eq(const P2 (&x)[8], const P2 (&y)[8]) {
  bool eq = true;
#pragma unroll
  for (int s = 1; s < 8; s++) eq = eq && p2_bits(x[s]) == p2_bits(y[s]);   // state 0 is 0 in both
  return eq;
}
// boundary vector j of an LDS array [S][7][64] (state 0 is 0)
MI_HD inline void p2s_vst(uint32_t* v, uint32_t j, int lane, const P2 (&x)[8]) {
#pragma unroll
  for (int s = 1; s < 8; s++) p2_stash_st(v, j * P2_CKW + (uint32_t)(s - 1), lane, p2_bits(x[s]));
}
MI_HD inline void p2s_vld(const uint32_t* v, uint32_t j, int lane, P2 (&x)[8]) {
  x[0] = Metric<P2>::zero();
#pragma unroll
  for (int s = 1; s < 8; s++) x[s] = p2_from_bits(p2_stash_ld(v, j * P2_CKW + (uint32_t)(s - 1), lane));
}
MI_HD inline void p2_zero8(P2 (&x)[8]) {
#pragma unroll
  for (int s = 0; s < 8; s++) x[s] = Metric<P2>::zero();
}
struct P2SegVecs { uint32_t *bvec, *bend, *avec, *aend; };
// the 8 steps 8c .. 8c + 7 of a continuation pass (q rows), converted
template <bool DEC2>
MI_P2_INL void p2s_load(const TdecArgsP2& a, int lane, uint32_t c, TdecX8P2& x) {
  TdecWin8P2 r;
  p2_load_window<DEC2, false, true>(a, lane, c * P2S_SPAN, r.lo);
  p2_load_window<DEC2, false, true>(a, lane, c * P2S_SPAN + BETA_W, r.hi);
  p2_cvt8<DEC2, true>(a, r, c * P2S_SPAN, x);
}
MI_HD inline void p2s_beta8(P2 (&b)[8], const TdecX8P2& x) {   // beta_{8c} from beta_{8c+8}, normalised per window
  p2_beta_run<7, 4>(b, x);
  norm8<true>(b);
  p2_beta_run<3, 0>(b, x);
  norm8<true>(b);
}
MI_HD inline void p2s_ck_get(const TdecArgsP2& a, uint32_t slot, int lane, P2 (&v)[8]) {
  uint32_t ck[P2_CKW];
  p2_ck_load_to(a.scr, (size_t)2 * a.K, slot, lane, ck);
  p2_ck_vec(ck, v);
}
// backward: the first pass of segment g (from the tail or a zero guess)
template <bool DEC2>
MI_P2_INL void p2s_bwd_first(const TdecArgsP2& a, int lane, const P2Seg& g, const P2SegVecs& V) {
  P2 b[8];
  if (g.j + 1 == g.nseg) {
    // beta_K from the three tail steps (TdecP2X::b1, q rows)
    const uint32_t t0 = 3 * a.K + (DEC2 ? 6 : 0);
    p2_start(b);
#pragma unroll
    for (int j = 2; j >= 0; j--) {
      P2 nb[8];
      beta_step<false>(b, p2_from_bits(row_ld(a.q, t0, lane, 2 * j)), p2_from_bits(row_ld(a.q, t0, lane, 2 * j + 1)), nb);
      p2_cp8(b, nb);
    }
    norm8<true>(b);
  } else {
    p2_zero8(b);
  }
  p2s_vst(V.bvec, g.j, lane, b);
  for (uint32_t c = g.e / P2S_SPAN; c-- > g.a / P2S_SPAN;) {
    TdecX8P2 x;
    p2s_load<DEC2>(a, lane, c, x);
    p2s_beta8(b, x);
    if (c > g.a / P2S_SPAN) p2_ck_store(a.scr, (size_t)2 * a.K, c, lane, b);
  }
  p2s_vst(V.bend, g.j, lane, b);
}
// backward fix-up of segment g (g.j + 1 < g.nseg) from its right neighbour's left-end vector nb: true when its own
// left-end vector changed
template <bool DEC2>
MI_P2_INL bool p2s_bwd_fix(const TdecArgsP2& a, int lane, const P2Seg& g, const P2SegVecs& V, const P2 (&nb)[8]) {
  P2 b[8];
  p2s_vld(V.bvec, g.j, lane, b);
  if (p2_all(p2_vec_eq(b, nb))) return false;
  p2s_vst(V.bvec, g.j, lane, nb);
  p2_cp8(b, nb);
  for (uint32_t c = g.e / P2S_SPAN; c-- > g.a / P2S_SPAN;) {
    TdecX8P2 x;
    p2s_load<DEC2>(a, lane, c, x);
    p2s_beta8(b, x);
    P2 old[8];
    const bool inner = c > g.a / P2S_SPAN;
    if (inner) p2s_ck_get(a, c, lane, old);
    else p2s_vld(V.bend, g.j, lane, old);
    if (p2_all(p2_vec_eq(old, b))) return false;   // merged: every earlier vector of the segment is already exact
    if (inner) p2_ck_store(a.scr, (size_t)2 * a.K, c, lane, b);
    else p2s_vst(V.bend, g.j, lane, b);
  }
  return true;
}
// forward over the steps 8c .. 8c + 7 with the outputs: the closing beta from the checkpoint or the segment's bvec
template <bool DEC2>
MI_P2_INL void p2s_fwd8(const TdecArgsP2& a, int lane, const P2Seg& g, const P2SegVecs& V, uint32_t c, P2 (&al)[8]) {
  TdecX8P2 x;
  p2s_load<DEC2>(a, lane, c, x);
  P2 B8[8];
  if (c + 1 < g.e / P2S_SPAN) p2s_ck_get(a, c + 1, lane, B8);
  else p2s_vld(V.bvec, g.j, lane, B8);
  p2_alpha_window8<DEC2>(a, lane, x, B8, c * P2S_SPAN, al);
}
template <bool DEC2>
MI_P2_INL void p2s_fwd_first(const TdecArgsP2& a, int lane, const P2Seg& g, const P2SegVecs& V) {
  P2 al[8];
  if (g.j == 0) p2_start_alpha(al);
  else p2_zero8(al);
  p2s_vst(V.avec, g.j, lane, al);
  const uint32_t K8 = a.K / P2S_SPAN;
  for (uint32_t c = g.a / P2S_SPAN; c < g.e / P2S_SPAN; c++) {
    p2s_fwd8<DEC2>(a, lane, g, V, c, al);
    if (c + 1 < g.e / P2S_SPAN) p2_ck_store(a.scr, (size_t)2 * a.K, K8 + 1 + c + 1, lane, al);
  }
  p2s_vst(V.aend, g.j, lane, al);
}
// forward fix-up of segment g (g.j > 0) from its left neighbour's right-end vector na: re-emits the steps whose alpha
// changed; true when its own right-end vector changed
template <bool DEC2>
MI_P2_INL bool p2s_fwd_fix(const TdecArgsP2& a, int lane, const P2Seg& g, const P2SegVecs& V, const P2 (&na)[8]) {
  P2 al[8];
  p2s_vld(V.avec, g.j, lane, al);
  if (p2_all(p2_vec_eq(al, na))) return false;
  p2s_vst(V.avec, g.j, lane, na);
  p2_cp8(al, na);
  const uint32_t K8 = a.K / P2S_SPAN;
  for (uint32_t c = g.a / P2S_SPAN; c < g.e / P2S_SPAN; c++) {
    p2s_fwd8<DEC2>(a, lane, g, V, c, al);
    P2 old[8];
    const bool inner = c + 1 < g.e / P2S_SPAN;
    if (inner) p2s_ck_get(a, K8 + 1 + c + 1, lane, old);
    else p2s_vld(V.aend, g.j, lane, old);
    if (p2_all(p2_vec_eq(old, al))) return false;
    if (inner) p2_ck_store(a.scr, (size_t)2 * a.K, K8 + 1 + c + 1, lane, al);
    else p2s_vst(V.aend, g.j, lane, al);
  }
  return true;
}
// one constituent decoder of one lane on the host: the segments in turn, rounds until no boundary changes -- the
// GPU kernel's schedule with its barriers (tdec.hip tdec_kernel_p2s), for the test emulation
template <bool DEC2>
inline void p2s_half_host(const TdecArgsP2& a, int lane, uint32_t S, const P2SegVecs& V) {
  const uint32_t nseg = p2s_seg(a.K, S, 0).nseg;
  for (uint32_t j = 0; j < nseg; j++) p2s_bwd_first<DEC2>(a, lane, p2s_seg(a.K, S, j), V);
  for (bool ch = true; ch;) {
    ch = false;
    P2 nb[64][8];
    for (uint32_t j = 0; j + 1 < nseg; j++) p2s_vld(V.bend, j + 1, lane, nb[j]);
    for (uint32_t j = 0; j + 1 < nseg; j++) ch = p2s_bwd_fix<DEC2>(a, lane, p2s_seg(a.K, S, j), V, nb[j]) || ch;
  }
  for (uint32_t j = 0; j < nseg; j++) p2s_fwd_first<DEC2>(a, lane, p2s_seg(a.K, S, j), V);
  for (bool ch = true; ch;) {
    ch = false;
    P2 na[64][8];
    for (uint32_t j = 1; j < nseg; j++) p2s_vld(V.aend, j - 1, lane, na[j]);
    for (uint32_t j = 1; j < nseg; j++) ch = p2s_fwd_fix<DEC2>(a, lane, p2s_seg(a.K, S, j), V, na[j]) || ch;
  }
}

struct TdecP2ExecHost {
  static constexpr bool SHARED = false;
  template <class F, class B>
  void run(F f, B b) { f(); b(); }
  uint32_t share(uint32_t v, int) { return v; }
  bool pack_wave() const { return true; }
};

}  // namespace mi
