// dl_common.h -- shared host/device definitions for the MI355X LTE DL PDSCH path.
//
// The path replaces what srsUE reaches through srslte_ue_dl_decode_fft_estimate and
// srslte_pdsch_decode_rnti (/root/reference/ue/src/phy/phch_worker.cc:254, :347-348).
// Everything here is spec arithmetic (3GPP TS 36.211 / 36.212 / 36.213) shared by the host
// planner and the gfx950 kernels.
#pragma once
#include <stdint.h>
#if defined(MI_EMU)
// host-only emulation build (tests): plain C++ stand-ins for the HIP vector type / qualifiers
#include <math.h>
#define __host__
#define __device__
struct float2 { float x, y; };
inline float2 make_float2(float a, float b) { return float2{a, b}; }
#else
#include <hip/hip_runtime.h>
#endif

namespace mi {

constexpr int NRB_MAX = 110;
constexpr int NSYMB = 14;            // normal CP, symbols per subframe
constexpr int KMAX = 6144;           // largest turbo code block
constexpr int NCB_MAX = 3 * 32 * ((KMAX + 4 + 31) / 32);   // 18528
constexpr int LANES = 64;            // code blocks per wavefront group (one CB per lane)
constexpr int BETA_W = 4;            // beta register window of the turbo kernel
// channel estimation: CRS pilot symbols of a port-0/1 subframe and the linear time interpolation /
// extrapolation of the pilot symbols' rows to symbol l (chest.hip writes it, the compact-estimate consumers
// recompute it: one table and one expression, so both give the same floats)
constexpr int CE_PL[4] = {0, 4, 7, 11};
__host__ __device__ constexpr int ce_ia(int l) { return l <= 4 ? 0 : (l <= 7 ? 1 : 2); }
__host__ __device__ constexpr float ce_tt_of(int l) {
  return (float)(l - CE_PL[ce_ia(l)]) / (float)(CE_PL[ce_ia(l) + 1] - CE_PL[ce_ia(l)]);
}
constexpr float CE_TT[NSYMB] = {ce_tt_of(0), ce_tt_of(1), ce_tt_of(2), ce_tt_of(3), ce_tt_of(4), ce_tt_of(5), ce_tt_of(6),
                                ce_tt_of(7), ce_tt_of(8), ce_tt_of(9), ce_tt_of(10), ce_tt_of(11), ce_tt_of(12), ce_tt_of(13)};
// CE_TT[l] for a run-time l without a table load: quarters are exact, thirds are the table's constants
__host__ __device__ inline float ce_tt(int l) {
  return l <= 4 ? 0.25f * (float)l : l == 5 ? CE_TT[5] : l == 6 ? CE_TT[6] : l == 7 ? 1.0f : 0.25f * (float)(l - 7);
}
__host__ __device__ inline float2 ce_time_interp(float2 a, float2 b, float tt) {
  return make_float2(__builtin_fmaf(tt, b.x - a.x, a.x), __builtin_fmaf(tt, b.y - a.y, a.y));
}
constexpr int TDEC_CK_MIN = 4;   // scratch sizing: one checkpoint slot per BETA_W-step window (the decoders use a subset)
constexpr float FILLER_LLR = -10000.0f;
constexpr int RM_CHUNK = 128;  // circular-buffer positions per rate-dematch workgroup
constexpr int WM_STRIDE = KMAX / BETA_W + 4;   // turbo window masks per group (rowmask_kernel)

__host__ __device__ inline int symbol_sz(uint32_t nof_prb) {
  return nof_prb <= 6 ? 128 : nof_prb <= 15 ? 256 : nof_prb <= 25 ? 512 : nof_prb <= 50 ? 1024
       : nof_prb <= 75 ? 1536 : nof_prb <= 110 ? 2048 : -1;
}
__host__ __device__ inline int cp_len(int N, int l_in_slot) { return (l_in_slot == 0 ? 160 : 144) * N / 2048; }
__host__ __device__ inline int sf_len(int N) { return 15 * N; }
// sample offset of the useful part of OFDM symbol l (0..13) inside the subframe
__host__ __device__ inline int symbol_offset(int N, int l) {
  int slot = l / 7, lp = l % 7;
  int off = slot * (15 * N / 2);
  for (int q = 0; q < lp; q++) off += cp_len(N, q) + N;
  return off + cp_len(N, lp);
}
// FFT bin of grid subcarrier k (DC skipped), 36.211 6.12
__host__ __device__ inline int sc_bin(int k, int W, int N) { return k < W / 2 ? N - W / 2 + k : k - W / 2 + 1; }

// 36.212 5.1.4.1.1 inter-column permutation
__host__ __device__ inline uint32_t subblock_perm(uint32_t c) {
  // bit-reversal of the 5-bit column index
  return ((c & 1) << 4) | ((c & 2) << 2) | (c & 4) | ((c & 8) >> 2) | ((c & 16) >> 4);
}

}  // namespace mi

// --------------------------------------------------------------------------------------------
// Device-side descriptors built by the host planner (plan.cpp) and read by the kernels.
// --------------------------------------------------------------------------------------------
struct MiCellDesc {          // one per distinct (cell id, nof_prb, nof_ports)
  uint32_t id, nof_prb, nof_ports, N, W;
  uint32_t crs_off;          // float2 offset of CRS table [20 ns][2 l'][220]
};

struct MiPdschDesc {         // one per distinct PDSCH mapping (cell, cfi, sf, prb mask, Qm, tm, rnti)
  uint32_t cell;             // index into MiCellDesc
  uint32_t sf_idx, nre, Qm, tm, G;
  uint32_t re_off;           // offset into the RE index table (uint32 grid indices)
  uint32_t scr_off;          // offset into scrambling word table (uint32 words, bit i = word[i/32] >> (i%32))
};

struct MiSfDesc {            // one per subframe of the batch
  uint64_t iq_off;           // float2 offset into the IQ batch buffer
  uint64_t grid_off;         // float2 offset into grid buffer (ce uses nof_ports * same stride)
  uint64_t ce_off;
  uint64_t e_off;            // float offset into the LLR buffer
  uint32_t pdsch;            // MiPdschDesc index
  uint32_t cell;             // MiCellDesc index
  uint32_t sf_idx;
  uint32_t tb;               // TB index
};

struct MiLaneDesc {          // one per code block (lane of a group)
  uint64_t e_off;            // float offset of this CB's E LLRs
  uint32_t E;
  uint32_t r0;               // number of non-null circular-buffer positions before k0(rv)
  uint32_t Nv;               // non-null circular-buffer positions (depends on K and F)
  uint32_t F;                // filler bits (only CB 0 of a TB may have F > 0)
  uint32_t rank_off;         // int32 offset of this (K, F)'s rank table [Ncb] (-1 = <NULL>), followed
                             // by the rank at every RM_CHUNK-th position [Ncb / RM_CHUNK + 2]
  uint32_t new_tb;           // 1 = first transmission (overwrite softbuffer), 0 = combine
  uint32_t crc24a;           // 1 when C == 1 (code-block CRC is the TB CRC24A)
  uint32_t tb;               // owning TB
  uint32_t valid;            // 0 for padding lanes of a partial group
  // where the code block's payload bytes go (PDSCH batches): CB bytes F/8 .. are payload bytes pay_st ..
  // (tb_kernel's copy; the packed decoder writes them there directly), up to the CB CRC and, when the code
  // block carries it (tbcrc = 1: C == 1 or the last code block), the TB CRC
  uint32_t pay_st, tbcrc;
  uint32_t pad;
};

struct MiLaneSrc {           // one per code block: where the fused demap stage finds its LLRs' inputs
  uint64_t goff, coff;       // float2 offsets of its subframe's grid and port-0 channel estimates
  uint32_t c1;               // port 1's estimates at c0 + c1 (NSYMB x W)
  uint32_t re, scr;          // offsets of the PDSCH RE list and scrambling words
  uint32_t qm, tm2;          // bits per symbol, SFBC
  uint32_t eb;               // LLR index of the code block's first LLR within its subframe
  uint32_t wdiv;             // floor(2^32 / W) + 1: RE index / W = __umulhi(re, wdiv) (compact estimates)
};

struct MiGroupDesc {         // one per wavefront group of <= 64 code blocks of equal K
  uint32_t K, Ncb;
  uint32_t lane0;            // first MiLaneDesc index (64 consecutive entries)
  uint32_t ktab;             // K-table index (pos / pi tables)
  uint64_t sb_off;           // float offset of the group's softbuffer region (mi::sb_group_floats: rows, zero row, map)
  uint64_t scratch_off;      // float offset of the group's turbo scratch (w, llr1, beta ckpt)
  uint64_t dec_off;          // byte offset of decision bytes [K][64]
};

// a direct group of rate de-matching (rm.hip, Plan::rm_direct): what rm_direct_map_kernel needs
struct MiRmDirect {
  uint32_t lane0, Ncb;
  uint32_t sb64;             // the group's softbuffer offset / 64 floats
  uint32_t rrow_off;         // uint32 offset of the (K, F) rank -> softbuffer row table [N_v] in kdata
  uint32_t r0, Nv;           // the lanes' common k0 rank and non-null position count
  uint32_t emax_kind;        // largest E of the group's lanes | (Qm + 8 TM2) << 24
  uint32_t rank_off;         // the (K, F) rank table (kdata)
};

struct MiKTab {              // per K, device resident
  uint32_t K, Ncb;
  uint32_t pos_off;          // uint32 offset: pos[3*(K+4)] circular-buffer position of d_i(k)
  uint32_t pi_off;           // uint32 offset: pi[K]
  uint32_t crca_off;         // uint32 offset: CRC24A contribution of a single 1 at bit i, [K]
  uint32_t crcb_off;         // uint32 offset: same for CRC24B
  uint32_t ipos_off;         // uint32 offset: ipos[Ncb] decoder input index of circular-buffer position p
                             // (the inverse of pos; 0xFFFFFFFF at dummy / null positions)
};

namespace mi {
// ---- int16 ("SSE") turbo arithmetic (oracle/oracle.h OR_I16_*, contract in tdec_body.h) ----------
constexpr float I16_SCALE = 32.0f, I16_CI = 511.0f, I16_CX = 1535.0f, I16_CW = 1023.0f;
__host__ __device__ inline float clampf(float x, float c) { return fminf(fmaxf(x, -c), c); }
// decoder-input quantiser q(x) = clamp(rint(32 x), +-511)
__host__ __device__ inline float q16f(float x) { return clampf(rintf(x * I16_SCALE), I16_CI); }
// In int16 mode a group's scratch (sized in floats for the float decoder) holds int16 streams: w [K],
// llr1 [K], beta checkpoints [(K/4 + 1)][64 lanes][8] (tdec_body.h ck_store), then from this int16 element index
// the quantised decoder inputs q [3 (K + 4)][64] in natural (triplet) order, written by the decoder's
// first pass from the softbuffer and read by every later pass.  Fits: 3K + 12 <= 2K + 8 (K/4 + 1) for K >= 4.
__host__ __device__ inline size_t q16_elem_off(uint32_t K) {
  return (size_t)LANES * (2 * K + 8 * (K / TDEC_CK_MIN + 1));
}
}  // namespace mi

namespace mi {
// ---- softbuffer region of one group (sparse rows) -------------------------------------------------
// [Ncb][64] fp32 rows, then one all-zero row (row index Ncb), then the row map: one byte per
// circular-buffer position, 1 = the row holds the values of all 64 lanes ("materialised"), 0 = every
// lane's value there is 0 (RX_NULL / never received).  The rate de-matcher writes only rows that
// receive an LLR (or must keep a HARQ history) and rewrites the map; the turbo decoder fetches
// unmaterialised rows from the zero row (L2-resident) instead of HBM.  Punctured positions never
// cost HBM traffic and a reset only needs the map cleared.
// Softbuffer rows in decoder-input order: the value of circular-buffer position p lives in row ipos[p] -- the decoder
// input index t it feeds (MiKTab::ipos_off; dummy positions have none and are never materialised) -- so the turbo
// decoder reads rows t = 3 k + stream in sequence, with no position table on its path; rate de-matching does the
// mapping once when it writes.  The row map stays indexed by position p.
// (An int16 mirror of the rows, written beside them by rate de-matching for the decoder, was measured in round 4 and
// dropped: tdec -8 % but rate de-matching +20 %, the 4-stream headline -3 %; profiles/r4/ab_mirror.)
__host__ __device__ inline size_t sb_map_off(uint32_t Ncb) { return (size_t)(Ncb + 1) * LANES; }   // floats
__host__ __device__ inline size_t sb_group_floats(uint32_t Ncb) {   // a multiple of 64 floats (256 B)
  return sb_map_off(Ncb) + (size_t)((Ncb + 255) / 256) * LANES;
}
}  // namespace mi

struct MiTbDesc {            // one per transport block
  uint32_t tbs, C, Kp, Km, Cm, F;
  uint32_t cb_list;          // offset into the lane-index list: C entries, CB r -> MiLaneDesc index
  uint32_t pay_off;          // byte offset into payload buffer
  uint32_t crc_mul;          // kdata offset of C multipliers x^(8 bytes after CB r) mod g24A (tb_kernel)
};
