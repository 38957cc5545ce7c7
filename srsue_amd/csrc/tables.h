// tables.h -- host-side spec tables and index maps (36.211 / 36.212 / 36.213) for the planner.
#pragma once
#include <stdint.h>
#include <vector>

namespace mi {

struct CbSegm { uint32_t C, Cp, Cm, Kp, Km, F, B; };

int qpp_params(uint32_t K, uint32_t* f1, uint32_t* f2);           // 36.212 Table 5.1.3-3
bool cb_size_valid(uint32_t K);
int cbsegm(uint32_t tbs, CbSegm* s);                                // 36.212 5.1.2
int tbs_from_idx(uint32_t i_tbs, uint32_t nof_prb);                 // 36.213 Table 7.1.7.2.1-1 (N_PRB 1..110)
int mcs_to_itbs(uint32_t mcs, uint32_t* qm);                        // 36.213 Table 7.1.7.1-1
uint32_t rm_E(uint32_t G, uint32_t C, uint32_t Qm, uint32_t NL, uint32_t r);   // 36.212 5.1.4.1.2
uint32_t ncb_of(uint32_t K);
uint32_t k0_of(uint32_t K, uint32_t rv);
// circular-buffer maps of one code block size: pos[t] for decoder input t = 3k + i, and the rank
// table (number of non-null positions before p, -1 for <NULL>) for F filler bits.
void cb_pos_table(uint32_t K, std::vector<uint32_t>& pos);
void cb_rank_table(uint32_t K, uint32_t F, std::vector<int32_t>& rank, uint32_t* Nv);
void qpp_table(uint32_t K, std::vector<uint32_t>& pi);
// CRC register of a K-bit message holding a single 1 at bit i (zero init): x^(K-1-i+24) mod g
void crc_bit_table(uint32_t K, uint32_t poly, std::vector<uint32_t>& t);
// 36.211 7.2 Gold sequence, packed 32 bits per word (bit i at word[i/32] bit i%32)
void gold_words(uint32_t c_init, uint32_t nbits, uint32_t* words);
void gold_bits(uint32_t c_init, uint32_t nbits, uint8_t* bits);
// 36.211 6.10.1.1 CRS r_{l,ns}(m), m < 220 (interleaved re, im)
void crs_seq(uint32_t id, uint32_t ns, uint32_t l, float* re_im);
// PDSCH RE membership / list (36.211 6.3.5 mapping order), grid index l * 12 N_RB + k
int ctrl_symbols(uint32_t nof_prb, uint32_t cfi);
bool is_pdsch_re(uint32_t id, uint32_t nof_prb, uint32_t nof_ports, uint32_t cfi, uint32_t sf, uint32_t l, uint32_t k);
// prb_mask: bit s of entry p = PRB p used in slot s when any entry is >= 2 (distributed VRB), else
// non-zero = used in both slots
uint32_t pdsch_re_list(uint32_t id, uint32_t nof_prb, uint32_t nof_ports, uint32_t cfi, uint32_t sf,
                       const uint8_t* prb_mask, std::vector<uint32_t>& re);
// PCFICH REs (36.211 6.7.4) in symbol 0, and scrambling init (36.211 6.7.1)
void pcfich_k(uint32_t id, uint32_t nof_prb, uint32_t* k16);
uint32_t pcfich_cinit(uint32_t id, uint32_t sf);
void cfi_codeword(uint32_t cfi, uint8_t* b32);                       // 36.212 Table 5.3.4-1

// ---- DL control: 36.211 6.2.4 / 6.7.4 / 6.8.5 / 6.9.3, 36.212 5.1.4.2 / 5.3.3,
// 36.213 9.1.1.  Same restatement as oracle/o_ctrl.c (which documents the spec walk-through).
uint32_t phich_ngroups(uint32_t nof_prb, uint32_t ng);               // ng: 0..3 = Ng 1/6, 1/2, 1, 2
// PHICH (36.213 9.1.2 FDD): group / orthogonal sequence of an UL grant; the group's 12 symbol-0 REs
void phich_calc(uint32_t nof_prb, uint32_t ng, uint32_t I_lowest, uint32_t n_dmrs, uint32_t* group, uint32_t* seq);
int phich_res(uint32_t id, uint32_t nof_prb, uint32_t ng, uint32_t group, uint32_t* re12);
inline uint32_t phich_cinit(uint32_t id, uint32_t sf) { return (sf + 1) * (2 * id + 1) * 512 + id; }
// PDCCH REGs (not PCFICH / PHICH) in 6.8.5 mapping order, 4 RE indices each; returns N_REG
uint32_t pdcch_regs(uint32_t id, uint32_t nof_prb, uint32_t ng, uint32_t cfi, std::vector<uint32_t>* re4);
// logical quadruplet carried by each physical REG (quadruplet sub-block interleaver + shift by N_ID)
void pdcch_quad_perm(uint32_t M, uint32_t id, std::vector<uint32_t>& log_of_reg);
enum { DCI_0 = 0, DCI_1 = 1, DCI_1A = 2, DCI_1C = 3 };
uint32_t dci_size(int format, uint32_t nof_prb);
// ---- DL resource allocation (36.213 7.1.6, 36.211 6.2.3.2) -------------------------------------
uint32_t ceil_log2(uint32_t x);
uint32_t rbg_size(uint32_t nof_prb);                       // Table 7.1.6.1-1
uint32_t n_gap(uint32_t nof_prb, bool gap2);               // Table 6.2.3.2-1 (0: not defined)
uint32_t n_vrb_dist(uint32_t nof_prb, bool gap2);          // N_VRB^DL of the distributed mapping
// PRB of distributed VRB n_vrb in slot 0 / 1; -1 outside N_VRB^DL
int vrb_to_prb(uint32_t nof_prb, bool gap2, uint32_t n_vrb, uint32_t slot);
uint32_t dci1c_rba_bits(uint32_t nof_prb);
int tbs_1c(uint32_t i_tbs);                                // Table 7.1.7.2.3-1, -1 for I_TBS > 31
// circular-buffer rank of each coded bit p of the rate-1/3 tail-biting code (d0 | d1 | d2, D each):
// e_k lands on the position of rank k mod 3D
void conv_rank_table(uint32_t D, std::vector<uint32_t>& rank);
// 36.213 9.1.1 candidates (L, first CCE) in search order; returns the count (<= 16)
int search_space(uint32_t n_cce, uint32_t sf, uint16_t rnti, bool common, uint32_t* L, uint32_t* ncce);

}  // namespace mi
