// ul_common.h -- shared host/device definitions of the UL PUSCH transmit path:
// what srsUE reaches through srslte_ue_ul_cfg_grant + srslte_ue_ul_pusch_encode_rnti_softbuffer
// (/root/reference/ue/src/phy/phch_worker.cc:551-560).  Spec: 36.212 5.2.2 (UL-SCH: CRC24A,
// segmentation, CRC24B, turbo code, rate matching, channel interleaver without UCI), 36.211 5.3
// (scrambling, modulation, transform precoding, mapping), 5.5.2.1 (PUSCH DMRS), 5.6 (SC-FDMA).
#pragma once
#include "dl_common.h"

// one PUSCH transmission (one subframe of one UE)
struct MiUlTx {
  uint64_t iq_off;       // float2 offset of its output subframe (15 N samples)
  uint32_t N, W;         // FFT size, 12 N_RB^UL
  uint32_t n_prb, M, Qm; // first PRB, M = 12 L_prb subcarriers, bits per symbol
  uint32_t n_prb1;       // first PRB of slot 1 (= n_prb without frequency hopping)
  uint32_t sym_off;      // byte offset of its 12 M coded symbols (Qm bits each, first bit = MSB)
  uint32_t scr_off;      // uint32 offset of its scrambling words (36.211 5.3.1, G bits)
  uint32_t pay_off;      // byte offset of its TB payload
  uint32_t tbs;
  uint32_t q[2], ncs[2]; // DMRS root index q and cyclic shift n_cs of slots 0 / 1 (5.5.2.1)
  uint32_t nzc;          // Zadoff-Chu length (largest prime < M)
  uint32_t fact;         // radix list of the M-point DFT, 4 bits per stage (first stage lowest)
  uint32_t fact_n;       // same for the N-point SC-FDMA transform
  uint32_t twm_off, twn_off;   // float2 offsets of exp(-2 pi i t / M) and exp(-2 pi i t / N) tables
  float scale;           // output amplitude factor (1; srslte_ue_ul_set_normalization)
  float cfo;             // frequency shift applied to the output, subcarriers (0; srslte_ue_ul_set_cfo)
  uint32_t q_ack;        // HARQ-ACK coded symbols Q'_ACK (0 = none)
  uint32_t ack_nblk;     // symbols in the encoded ACK block (1 or 3), repeated over the Q'_ACK symbols
  uint32_t ack_sym[3];   // the block's symbols: 2 bits per coded bit, bit b at bits 2b (0/1, 2 = x, 3 = y)
  uint32_t q_ri;         // RI coded symbols Q'_RI (0 = none), placed like HARQ-ACK in columns {1, 4, 7, 10}
  uint32_t ri_nblk;      // symbols in the encoded RI block (1 or 3)
  uint32_t ri_sym[3];    // as ack_sym
  uint32_t q_cqi;        // CQI coded symbols Q'_CQI at the head of the multiplexed sequence (uploaded with the plan)
};

// one UL-SCH code block
struct MiUlCb {
  uint32_t tx, K, F, C, r, E, r0, Nv;
  uint32_t byte0;        // first byte of (TB || CRC24A) it carries
  uint32_t nbytes;       // bytes of (TB || CRC24A) it carries (K - F - 24 [C > 1]) / 8
  uint32_t sym0;         // first coded symbol within the transmission (rate-matching output / Qm)
  uint32_t pi_off;       // uint32 offset of the QPP table [K]
  uint32_t sel_off;      // uint32 offset of the selection table [Nv]: the d-stream index t = 3k + i
                         // of the n-th non-null circular-buffer position (36.212 5.1.4.1.2 inverted)
};

namespace mi {
constexpr int UL_THREADS = 256;
constexpr int UL_NMAX = 2048;     // largest SC-FDMA transform
constexpr int UL_MMAX = 1320;     // 12 x 110 PRB
}  // namespace mi
