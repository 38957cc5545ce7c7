// tdec_win_body.h -- the int16 max-log-MAP turbo decoder with ONE code block per workgroup: the
// trellis is cut into segments, one per thread, and the segments are decoded in parallel with EXACT
// boundary metrics (the latency path: a single subframe's 13 code blocks on 13 CUs instead of 13
// lanes of one wavefront).  Same algorithm and arithmetic as tdec_body.h's int16 mode (srsLTE's SSE
// decoder design, oracle or_decode_cb16), bit-identical extrinsics, decisions and iteration counts.
//
// Replaces, like tdec_body.h, srslte_tdec_reset / _iteration / _decision + the CRC early stop reached
// from srslte_pdsch_decode_rnti (/root/reference/ue/src/phy/phch_worker.cc:347-348), with the cap of
// srslte_sch_set_max_noi (phch_worker.cc:88).
//
// Why segments can be exact.  In the int16 design every state metric is an integer and each
// recursion step is max-plus: beta_k(s) = max(beta_{k+1}(s0) + g0, beta_{k+1}(s1) + g1).  Adding a
// constant to all states of a metric vector adds it to every later vector and cancels in every LLR
// (a difference of two maxima), so only the normalised vector (state 0 subtracted) matters.  A
// segment started from a GUESSED boundary vector therefore produces exactly the true normalised
// metrics from the first step at which its vector coincides with the true one -- and once that
// happens, every later step coincides too (same inputs, same deterministic recursion).  So:
//   1. every segment runs from a guess (the outer segments from the true trellis boundary: alpha_0 =
//      state 0, beta_K from the tail bits) and stores its normalised vectors every 4 steps
//      (checkpoints) and its final boundary vector;
//   2. fix-up rounds: a segment whose neighbour's boundary vector differs from the one it started
//      from restarts from the neighbour's vector and re-walks its windows until the recomputed vector
//      EQUALS the stored checkpoint (exact integer compare: from there on nothing changes) or the
//      segment end (then its own boundary changed and the next segment re-checks);
//   3. rounds repeat until no boundary changed.  The last round leaves every checkpoint equal to the
//      full-length recursion's normalised vector, and the forward pass re-emits exactly the outputs
//      whose alpha changed.  Worst case (no two paths ever merge) is the serial walk; at any useful
//      SNR vectors merge within a few trellis steps, so a half-iteration costs ~2 segment lengths.
// The float (srsLTE-gen) decoder normalises every step with rounding that depends on magnitudes --
// not shift-invariant -- so it keeps the one-lane-per-code-block kernel (tdec_body.h).
//
// Layout: the whole code block lives in LDS (q inputs, pi, DEC2 input d, extrinsic w, decisions,
// beta/alpha checkpoints as int16: all normalised metrics lie within +-6138, oracle/o_fec.c).
// Segment j = thread j covers steps [j S, min((j+1) S, K)), S a multiple of the 4-step window.
#pragma once
#include "tb_body.h"
#include "tdec_body.h"

namespace mi {

constexpr int WIN_MAXP = 512;   // threads (segments) per code block, at most

// per code block state (LDS on the GPU; host arrays in the test emulation)
struct WinCb {
  int16_t* q;        // [3K + 12] quantised decoder inputs, natural (triplet) order; DEC1's systematic and
                     // parity of filler steps k < F replaced by the filler value
  uint16_t* pi;      // [K] QPP interleaver
  int16_t* d;        // [K] DEC2 systematic input clamp(llr1 - w, CX), written by DEC1 at step k
  int16_t* w;        // [K] extrinsic, written by DEC2 at pi(k)
  uint8_t* dec;      // [K] decisions, written by DEC2 at pi(k)
  int16_t* bck;      // [(K/4 + 1) * 8] beta checkpoints: beta at step 4v, normalised (state 0 = 0)
  int16_t* ack;      // [(K/4 + 1) * 8] alpha checkpoints: alpha at step 4v
  int16_t* bend;     // [nseg * 8] beta at each segment's first step (its left boundary)
  int16_t* aend;     // [nseg * 8] alpha after each segment's last step (its right boundary)
  uint8_t* lmap;     // [Ncb, rounded to 16] the group's softbuffer row map, staged for win_load only (on
                     // the GPU it borrows the checkpoint arrays, unused until the first half-iteration)
  uint32_t K, S, nseg;
};

MI_HD inline void win_geometry(uint32_t K, uint32_t P, uint32_t& S, uint32_t& nseg) {
  S = (((K + P - 1) / P) + 3) / 4 * 4;
  nseg = (K + S - 1) / S;
}
// LDS bytes of one code block of size K with P threads (tdec_win.hip lays the arrays out in this order)
MI_HD inline uint32_t win_lds_bytes(uint32_t K, uint32_t P) {
  const uint32_t ck = (K / 4 + 1) * 16;
  return ((3 * K + 12) * 2 + 15) / 16 * 16 + K * 2 + K * 2 + K * 2 + (K + 15) / 16 * 16 + 2 * ck + 2 * P * 16;
}

// ---- metric vectors <-> int16 checkpoints ------------------------------------------------------
MI_HD inline void ck_put(int16_t* c, const float (&v)[8]) {
#pragma unroll
  for (int s = 0; s < 8; s++) c[s] = (int16_t)fmaxf(v[s], -32768.0f);   // -inf only at alpha_0 (never read)
}
MI_HD inline void ck_get(const int16_t* c, float (&v)[8]) {
#pragma unroll
  for (int s = 0; s < 8; s++) v[s] = (float)c[s];
}
MI_HD inline bool ck_eq(const int16_t* c, const float (&v)[8]) {
  bool eq = true;
#pragma unroll
  for (int s = 1; s < 8; s++) eq = eq && ((float)c[s] == v[s]);
  return eq;
}

// ---- window inputs ------------------------------------------------------------------------------
// DEC1 step k: xs = q[3k] + w[k], xp = q[3k+1].  DEC2 step k: xs = d[pi(k)], xp = q[3k+2].
template <bool DEC2>
MI_HD inline void win_inputs(const WinCb& c, uint32_t base, float (&xs)[4], float (&xp)[4], uint32_t (&pk)[4]) {
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t k = base + i;
    if (!DEC2) {
      pk[i] = k;
      xs[i] = (float)c.q[3 * k] + (float)c.w[k];
      xp[i] = (float)c.q[3 * k + 1];
    } else {
      pk[i] = c.pi[k];
      xs[i] = (float)c.d[pk[i]];
      xp[i] = (float)c.q[3 * k + 2];
    }
  }
}

// backward over one window: beta_{base} from beta_{base+4} (normalised once, as tdec_body.h's int16 mode)
MI_HD inline void win_beta(const float (&xs)[4], const float (&xp)[4], float (&b)[8]) {
#pragma unroll
  for (int i = 3; i >= 0; i--) {
    float nb[8];
    beta_step<false>(b, xs[i], xp[i], nb);
#pragma unroll
    for (int s = 0; s < 8; s++) b[s] = nb[s];
  }
  norm8<true>(b);
}

// forward over one window: beta_{base+1..base+4} from the closing checkpoint, alpha and the outputs
//   DEC1: d[k] = clamp(llr1 - w[k], CX)      DEC2: w[pi(k)] = clamp(llr2 - xs, CW), dec[pi(k)] = llr2 > 0
template <bool DEC2>
MI_HD inline void win_alpha(const WinCb& c, uint32_t base, const float (&xs)[4], const float (&xp)[4],
                            const uint32_t (&pk)[4], const float (&bclose)[8], float (&al)[8]) {
  float bw[4][8];
#pragma unroll
  for (int s = 0; s < 8; s++) bw[3][s] = bclose[s];
#pragma unroll
  for (int i = 2; i >= 0; i--) beta_step<false>(bw[i + 1], xs[i + 1], xp[i + 1], bw[i]);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const float llr = alpha_step<false>(al, bw[i], xs[i], xp[i]);
    if (!DEC2) {
      c.d[base + i] = (int16_t)clampf(llr - (float)c.w[base + i], I16_CX);
    } else {
      c.w[pk[i]] = (int16_t)clampf(llr - xs[i], I16_CW);
      c.dec[pk[i]] = llr > 0.0f ? 1 : 0;
    }
  }
  norm8<true>(al);
}

// beta_K of a constituent decoder from its three tail steps (DEC1: q[3K..3K+5], DEC2: q[3K+6..3K+11])
template <bool DEC2>
MI_HD inline void win_tail_beta(const WinCb& c, float (&b)[8]) {
  const uint32_t t0 = 3 * c.K + (DEC2 ? 6 : 0);
#pragma unroll
  for (int s = 0; s < 8; s++) b[s] = s ? -INFINITY : 0.0f;
#pragma unroll
  for (int j = 2; j >= 0; j--) {
    float nb[8];
    beta_step<false>(b, (float)c.q[t0 + 2 * j], (float)c.q[t0 + 2 * j + 1], nb);
#pragma unroll
    for (int s = 0; s < 8; s++) b[s] = nb[s];
  }
  norm8<true>(b);
}

MI_HD inline void win_seg(const WinCb& c, uint32_t j, uint32_t& a, uint32_t& b) {
  a = j * c.S;
  b = a + c.S < c.K ? a + c.S : c.K;
}

// ---- backward pass ------------------------------------------------------------------------------
// Segment j owns bck[v] for a/4 < v <= b/4 (bck[b/4] = the start vector it used) and bend[j].
// First pass: from the trellis end (last segment) or an all-zero guess.
template <bool DEC2>
MI_HD inline void win_bwd_first(const WinCb& c, uint32_t j) {
  uint32_t a, e;
  win_seg(c, j, a, e);
  float b[8];
  if (j == c.nseg - 1) win_tail_beta<DEC2>(c, b);
  else
    for (int s = 0; s < 8; s++) b[s] = 0.0f;
  ck_put(c.bck + (e / 4) * 8, b);
  for (uint32_t v = e / 4; v-- > a / 4;) {
    float xs[4], xp[4];
    uint32_t pk[4];
    win_inputs<DEC2>(c, 4 * v, xs, xp, pk);
    win_beta(xs, xp, b);
    if (v > a / 4) ck_put(c.bck + v * 8, b);
  }
  ck_put(c.bend + j * 8, b);
}
// Fix-up: nb = the right neighbour's bend (read before the round's barrier).  Returns true when this
// segment's own left boundary changed (the left neighbour must re-check in the next round).
template <bool DEC2>
MI_HD inline bool win_bwd_fix(const WinCb& c, uint32_t j, const float (&nb)[8]) {
  uint32_t a, e;
  win_seg(c, j, a, e);
  if (ck_eq(c.bck + (e / 4) * 8, nb)) return false;
  ck_put(c.bck + (e / 4) * 8, nb);
  float b[8];
  for (int s = 0; s < 8; s++) b[s] = nb[s];
  for (uint32_t v = e / 4; v-- > a / 4;) {
    float xs[4], xp[4];
    uint32_t pk[4];
    win_inputs<DEC2>(c, 4 * v, xs, xp, pk);
    win_beta(xs, xp, b);
    int16_t* slot = v > a / 4 ? c.bck + v * 8 : c.bend + j * 8;
    if (ck_eq(slot, b)) return false;   // merged with the stored (already exact from here) metrics
    ck_put(slot, b);
  }
  return true;
}

// ---- forward pass (emits the half-iteration's outputs) ---------------------------------------------
// Segment j owns ack[v] for a/4 <= v < b/4 (ack[a/4] = the start vector it used) and aend[j].
template <bool DEC2>
MI_HD inline void win_fwd_first(const WinCb& c, uint32_t j) {
  uint32_t a, e;
  win_seg(c, j, a, e);
  float al[8];
  for (int s = 0; s < 8; s++) al[s] = j == 0 ? (s ? -INFINITY : 0.0f) : 0.0f;
  ck_put(c.ack + (a / 4) * 8, al);
  for (uint32_t v = a / 4; v < e / 4; v++) {
    float xs[4], xp[4], bc[8];
    uint32_t pk[4];
    win_inputs<DEC2>(c, 4 * v, xs, xp, pk);
    ck_get(c.bck + (v + 1) * 8, bc);
    win_alpha<DEC2>(c, 4 * v, xs, xp, pk, bc, al);
    if (v + 1 < e / 4) ck_put(c.ack + (v + 1) * 8, al);
  }
  ck_put(c.aend + j * 8, al);
}
template <bool DEC2>
MI_HD inline bool win_fwd_fix(const WinCb& c, uint32_t j, const float (&na)[8]) {
  uint32_t a, e;
  win_seg(c, j, a, e);
  if (ck_eq(c.ack + (a / 4) * 8, na)) return false;
  ck_put(c.ack + (a / 4) * 8, na);
  float al[8];
  for (int s = 0; s < 8; s++) al[s] = na[s];
  for (uint32_t v = a / 4; v < e / 4; v++) {
    float xs[4], xp[4], bc[8];
    uint32_t pk[4];
    win_inputs<DEC2>(c, 4 * v, xs, xp, pk);
    ck_get(c.bck + (v + 1) * 8, bc);
    win_alpha<DEC2>(c, 4 * v, xs, xp, pk, bc, al);
    int16_t* slot = v + 1 < e / 4 ? c.ack + (v + 1) * 8 : c.aend + j * 8;
    if (ck_eq(slot, al)) return false;   // merged: every later output of this segment is unchanged
    ck_put(slot, al);
  }
  return true;
}

// ---- load / CRC / packing (cooperative loops over the code block, thread t of P) ----------------------
// decoder inputs of the lane `lane` of a group softbuffer (rate de-matching's layout, dl_common.h):
// q(x) of the materialised rows, 0 for the others; filler steps k < F: DEC1 systematic/parity = -511
// load, step 1: the group's row map (one byte per circular-buffer position) into c.lmap, 16-byte
// pieces (the map region is 256-byte aligned and rounded up to 256 bytes, dl_common.h)
MI_HD inline void win_load_map(const WinCb& c, uint32_t t, uint32_t P, const float* sbg, uint32_t Ncb) {
  const uint8_t* map = reinterpret_cast<const uint8_t*>(sbg + sb_map_off(Ncb));
  for (uint32_t i = 16 * t; i < Ncb; i += 16 * P) {
#if defined(__HIP_DEVICE_COMPILE__)
    *reinterpret_cast<uint4*>(c.lmap + i) = *reinterpret_cast<const uint4*>(map + i);
#else
    memcpy(c.lmap + i, map + i, 16);
#endif
  }
}
// load, step 2 (after a barrier): walk the circular buffer in position order -- row p of this lane
// (0 when the row is not materialised, c.lmap) goes, quantised, to decoder input ipos[p] in LDS.  The
// position-table and softbuffer loads of a batch are independent (one round trip per batch of B per
// thread) and consecutive threads read consecutive rows.  (Gathering in decoder order -- position,
// then map, then value: three dependent loads, B = 8 -- was 53 us of a 174 us single-subframe decode.)
// tab = the position table pos (rows in decoder-input order: row t is read whatever its state and kept when its
// position pos[t] is materialised -- the row and table loads stay independent)
MI_HD inline void win_load(const WinCb& c, uint32_t t, uint32_t P, const float* sbg, const uint32_t* tab,
                           const uint32_t* pi32, uint32_t lane, uint32_t F) {
  constexpr uint32_t B = 24;   // independent loads per thread and round (72 measured the same)
  const uint32_t T = 3 * (c.K + 4);
  for (uint32_t t0 = t; t0 < T; t0 += B * P) {
    uint32_t pp[B];
    float xx[B];
#pragma unroll
    for (uint32_t b = 0; b < B; b++) {
      const uint32_t i = t0 + b * P;
      pp[b] = i < T ? tab[i] : 0u;
      xx[b] = i < T ? sbg[(size_t)i * LANES + lane] : 0.0f;
    }
#pragma unroll
    for (uint32_t b = 0; b < B; b++) {
      const uint32_t i = t0 + b * P;
      if (i >= T) continue;
      float x = c.lmap[pp[b]] ? q16f(xx[b]) : 0.0f;
      if (i < 3 * F && i % 3 != 2) x = -I16_CI;
      c.q[i] = (int16_t)x;
    }
  }
  for (uint32_t k = t; k < c.K; k += P) {
    c.pi[k] = (uint16_t)pi32[k];
    c.w[k] = 0;
  }
}

// this thread's share of the code-block CRC register of the decisions (XOR of the per-bit table)
MI_HD inline uint32_t win_crc_part(const WinCb& c, uint32_t t, uint32_t P, const uint32_t* tab) {
  uint32_t r = 0;
  for (uint32_t i = t; i < c.K; i += P) r ^= c.dec[i] ? tab[i] : 0u;
  return r;
}

// pack decisions MSB first (bytes t, t + P, ...) into the code block's output row
MI_HD inline void win_pack(const WinCb& c, uint32_t t, uint32_t P, uint8_t* out) {
  for (uint32_t j = t; j < c.K / 8; j += P) {
    uint32_t v = 0;
    for (int q = 0; q < 8; q++) v |= (uint32_t)c.dec[8 * j + q] << (7 - q);
    out[j] = (uint8_t)v;
  }
}
// this thread's term of the partial TB-CRC24A register over payload bytes [b0, b1) (tdec_body.h's
// tb_part): its contiguous chunk through the byte table, shifted by the bytes after it
MI_HD inline uint32_t win_tb_term(const WinCb& c, uint32_t t, uint32_t P, const uint8_t* out, uint32_t b0, uint32_t b1,
                                  const uint32_t* crc8) {
  if (b1 <= b0) return 0;
  const uint32_t n = b1 - b0, per = (n + P - 1) / P, s = b0 + t * per;
  if (s >= b1) return 0;
  const uint32_t e = s + per < b1 ? s + per : b1;
  uint32_t r = 0;
  for (uint32_t j = s; j < e; j++) r = ((r << 8) & 0xFFFFFFu) ^ crc8[((r >> 16) ^ out[j]) & 0xFFu];
  return r ? gf24_mulmod(r, gf24_xpow8(b1 - e, CRC24A_POLY), CRC24A_POLY) : 0u;
}

}  // namespace mi
