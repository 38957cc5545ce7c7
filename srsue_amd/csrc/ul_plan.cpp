// ul_plan.cpp -- UL PUSCH planner (see ul_plan.h).  Spec arithmetic: 36.212 5.2.2 / 5.1.2-5.1.4,
// 36.211 5.3 / 5.5.1 / 5.5.2.1 / 5.6; the oracle (oracle/o_ul.c) restates the same clauses for the tests.
#include "ul_plan.h"

#include <math.h>

#include "plan.h"   // set_error

namespace mi {

static const uint32_t N1_DMRS[8] = {0, 2, 3, 4, 6, 8, 9, 10};   // 36.211 Table 5.5.2.1.1-2 (cyclicShift)
static const uint32_t N2_DMRS[8] = {0, 6, 3, 4, 2, 8, 10, 9};   // 36.211 Table 5.5.2.1.1-1 (DCI format 0)

// 36.213 Table 8.6.3-1: beta_offset^HARQ-ACK x 8 for I_offset^HARQ-ACK = 0..14
static const uint32_t BETA8_ACK[15] = {16, 20, 25, 32, 40, 50, 64, 80, 101, 127, 160, 248, 400, 640, 1008};

static bool prime(uint32_t n) {
  if (n < 2) return false;
  for (uint32_t d = 2; d * d <= n; d++)
    if (n % d == 0) return false;
  return true;
}

int ul_dmrs_params(const mi_ul_cfg_t& c, uint32_t ns, uint32_t* q, uint32_t* nzc, uint32_t* ncs) {
  const uint32_t M = 12 * c.L_prb, fss = (c.cell_id + c.delta_ss) % 30;
  if (M < 12 || ns >= 20) return -1;
  uint32_t fgh = 0;
  if (c.group_hopping) {               // 5.5.1.3: c_init = floor(N_ID / 30)
    std::vector<uint8_t> g(160);
    gold_bits(c.cell_id / 30, 160, g.data());
    for (int i = 0; i < 8; i++) fgh += (uint32_t)g[8 * ns + i] << i;
    fgh %= 30;
  }
  const uint32_t u = (fgh + fss) % 30;
  // sequence hopping (5.5.1.4) and n_PRS (5.5.2.1.1) share c_init = floor(N_ID / 30) 2^5 + f_ss
  std::vector<uint8_t> s(8 * 7 * 20);
  gold_bits((c.cell_id / 30) * 32 + fss, 8 * 7 * 20, s.data());
  const uint32_t v = (M >= 72 && !c.group_hopping && c.sequence_hopping) ? s[ns] : 0;
  uint32_t prs = 0;
  for (int i = 0; i < 8; i++) prs += (uint32_t)s[8 * 7 * ns + i] << i;
  *ncs = (N1_DMRS[c.cyclic_shift & 7] + N2_DMRS[c.n_dmrs2 & 7] + prs) % 12;
  if (M < 36) {   // L_prb = 1, 2: the tabulated base sequences of group u (5.5.1.2), marked by N_ZC = 0
    *nzc = 0;
    *q = u;
    return 0;
  }
  uint32_t N = M - 1;
  while (!prime(N)) N--;
  *nzc = N;
  const double qb = (double)N * (u + 1) / 31.0;
  const uint32_t odd = (uint32_t)floor(2.0 * qb) & 1u;
  *q = (uint32_t)floor(qb + 0.5) + (odd ? (uint32_t)-(int32_t)v : v);
  return 0;
}

uint32_t ul_radix_plan(uint32_t n) {
  uint32_t plan = 0, st = 0;
  auto push = [&](uint32_t r) { plan |= r << (4 * st++); };
  while (n % 8 == 0 && n != 16 && n != 32 && st < 8) { push(8); n /= 8; }   // 16 / 32: 4 x 4, 8 x 4
  while (n % 4 == 0 && st < 8) { push(4); n /= 4; }
  while (n % 2 == 0 && st < 8) { push(2); n /= 2; }
  while (n % 3 == 0 && st < 8) { push(3); n /= 3; }
  while (n % 5 == 0 && st < 8) { push(5); n /= 5; }
  return n == 1 ? plan : 0;
}

// 36.212 Table 5.2.2.6.4-1 by columns: bit 31 - i of RM32_COL[n] = M_{i,n}
static const uint32_t RM32_COL[11] = {0xFFFFFFFFu, 0xCC95A5D2u, 0x5A7089BEu, 0x39CC64B6u, 0x07C3E38Eu, 0x003FF07Eu,
                                      0x2671B8CEu, 0x0DAF22D6u, 0x371843BEu, 0x62ED85B2u, 0xFFFF0F42u};
// 36.213 Table 8.6.3-2 (RI, I 0..12) and Table 8.6.3-3 (CQI, I 2..15), x 8
static const uint32_t BETA8_RI[13] = {10, 13, 16, 20, 25, 32, 40, 50, 64, 80, 101, 127, 160};
static const uint32_t BETA8_CQI[16] = {0, 0, 9, 10, 11, 13, 14, 16, 18, 20, 23, 25, 28, 32, 40, 50};

void ul_cqi_code(const uint8_t* o, uint32_t O, uint32_t Q, std::vector<uint8_t>& q) {
  q.assign(Q, 0);
  if (O <= 11) {   // b = sum_n o_n M_{., n}, q_i = b_(i mod 32)
    uint32_t w = 0;
    for (uint32_t n = 0; n < O; n++)
      if (o[n] & 1u) w ^= RM32_COL[n];
    for (uint32_t i = 0; i < Q; i++) q[i] = (uint8_t)((w >> (31 - (i & 31))) & 1u);
    return;
  }
  // CRC8 g = D^8 + D^7 + D^4 + D^3 + D + 1, then the rate-1/3 tail-biting code (5.1.3.1: generators 133,
  // 171, 165 octal, register preloaded with the last six bits) and its rate matching (5.1.4.2)
  const uint32_t D = O + 8;
  std::vector<uint8_t> c(o, o + O);
  uint32_t r = 0;
  for (uint32_t i = 0; i < O; i++) {
    const uint32_t fb = ((r >> 7) ^ o[i]) & 1u;
    r = ((r << 1) & 0xFFu) ^ (fb ? 0x9Bu : 0u);
  }
  for (int i = 7; i >= 0; i--) c.push_back((uint8_t)((r >> i) & 1u));
  static const uint32_t G[3] = {0133, 0171, 0165};
  std::vector<uint8_t> d(3 * D);
  uint32_t win = 0;   // bit 6 - j = c_{k-j} (the generators' MSB taps the current bit); preload c_{D-1} .. c_{D-6}
  for (uint32_t j = 1; j <= 6; j++) win |= (uint32_t)c[D - j] << (7 - j);
  for (uint32_t k = 0; k < D; k++) {
    win = (win >> 1) | ((uint32_t)c[k] << 6);
    for (int i = 0; i < 3; i++) d[i * D + k] = (uint8_t)(__builtin_popcount(win & G[i]) & 1);
  }
  std::vector<uint32_t> rank, inv(3 * D);
  conv_rank_table(D, rank);   // rank of each coded bit in the circular buffer
  for (uint32_t p = 0; p < 3 * D; p++) inv[rank[p]] = p;
  for (uint32_t k = 0; k < Q; k++) q[k] = d[inv[k % (3 * D)]];
}

// HARQ-ACK / RI block of Tables 5.2.2.6-1..-4 as modulation symbols (2 bits per coded bit: 0/1, 2 = x, 3 = y):
// 1 bit [o0 y x ..], 2 bits [o0 o1 x ..][o2 o0 x ..][o1 o2 x ..]; returns the symbol count
static uint32_t uci_block(uint32_t len, uint32_t v, uint32_t Qm, uint32_t* out) {
  const uint32_t o0 = v & 1u, o1 = (v >> 1) & 1u, o2 = o0 ^ o1, X = 2, Y = 3;
  auto sym = [&](uint32_t a, uint32_t b) {   // [a b x x ...]
    uint32_t w = a | (b << 2);
    for (uint32_t k = 2; k < Qm; k++) w |= X << (2 * k);
    return w;
  };
  if (len == 1) {
    out[0] = sym(o0, Y);
    return 1;
  }
  out[0] = sym(o0, o1);
  out[1] = sym(o2, o0);
  out[2] = sym(o1, o2);
  return 3;
}

int UlPlan::build(const mi_ul_cfg_t* cfgs, uint32_t n) {
  txs.clear(); cbs.clear(); kdata.clear(); scr.clear(); tw.clear(); tb_cb0.clear(); cqi_syms.clear(); cqi_off.clear();
  pi_off.clear(); tw_off.clear(); sel_off.clear();
  payload_bytes = sym_bytes = iq_samples = 0;
  algo_bytes = 0;
  auto twiddles = [&](uint32_t len) {
    auto it = tw_off.find(len);
    if (it != tw_off.end()) return it->second;
    const uint32_t off = (uint32_t)(tw.size() / 2);
    auto& tc = tw_cache[len];   // computed once per length (cos / sin of 2,048 + 1,200 points: ~0.1 ms)
    if (tc.empty())
      for (uint32_t t = 0; t < len; t++) {
        tc.push_back((float)cos(-2.0 * M_PI * t / len));
        tc.push_back((float)sin(-2.0 * M_PI * t / len));
      }
    tw.insert(tw.end(), tc.begin(), tc.end());
    tw_off[len] = off;
    return off;
  };
  for (uint32_t i = 0; i < n; i++) {
    const mi_ul_cfg_t& c = cfgs[i];
    const int N = symbol_sz(c.nof_prb);
    if (N < 0 || c.nof_prb == 0 || c.sf_idx > 9 || c.L_prb < 1 || c.n_prb + c.L_prb > c.nof_prb || (c.hop && c.n_prb1 + c.L_prb > c.nof_prb) ||
        (c.Qm != 2 && c.Qm != 4 && c.Qm != 6) || c.tbs == 0 || c.tbs % 8 || c.rv > 3) {
      set_error("invalid UL configuration (L_prb >= 1, allocation inside the cell, Qm 2/4/6, byte-aligned TBS)");
      return -1;
    }
    MiUlTx t{};
    t.N = (uint32_t)N;
    t.W = 12 * c.nof_prb;
    t.n_prb = c.n_prb;
    t.n_prb1 = c.hop ? c.n_prb1 : c.n_prb;
    t.M = 12 * c.L_prb;
    t.Qm = c.Qm;
    t.scale = 1.0f;
    t.cfo = 0.0f;
    t.fact = ul_radix_plan(t.M);
    t.fact_n = ul_radix_plan(t.N);
    if (!t.fact || !t.fact_n) {
      set_error("L_prb must be 2^a 3^b 5^c (36.211 5.3.3)");
      return -1;
    }
    for (uint32_t s = 0; s < 2; s++)
      if (ul_dmrs_params(c, 2 * c.sf_idx + s, &t.q[s], &t.nzc, &t.ncs[s])) {
        set_error("DMRS parameters");
        return -1;
      }
    t.twm_off = twiddles(t.M);
    t.twn_off = twiddles(t.N);
    CbSegm sg;
    if (cbsegm(c.tbs, &sg)) {
      set_error("segmentation");
      return -1;
    }
    uint64_t sumK = 0;
    for (uint32_t r = 0; r < sg.C; r++) sumK += r < sg.Cm ? sg.Km : sg.Kp;
    // RI and CQI on PUSCH (36.212 5.2.2.6): Q'_RI = min(ceil(O M 12 beta / sum K_r), 4 M); Q'_CQI =
    // min(ceil((O + L) M 12 beta / sum K_r), 12 M - Q'_RI), L = 8 (CRC) for O > 11
    if (c.ri_len > 2 || (c.ri_len && c.I_offset_ri > 12) || c.cqi_len > 64 ||
        (c.cqi_len && (c.I_offset_cqi < 2 || c.I_offset_cqi > 15))) {
      set_error("UCI on PUSCH: RI 0..2 bits (beta index 0..12), CQI 0..64 bits (beta index 2..15)");
      return -1;
    }
    auto qprime = [&](uint64_t bits, uint32_t beta8, uint64_t cap) {
      const uint64_t q = (bits * t.M * 12 * beta8 + 8 * sumK - 1) / (8 * sumK);
      return (uint32_t)(q < cap ? q : cap);
    };
    t.q_ri = c.ri_len ? qprime(c.ri_len, BETA8_RI[c.I_offset_ri], 4ull * t.M) : 0;
    t.q_cqi = c.cqi_len ? qprime(c.cqi_len + (c.cqi_len > 11 ? 8 : 0), BETA8_CQI[c.I_offset_cqi], 12ull * t.M - t.q_ri) : 0;
    cqi_off.push_back((uint32_t)cqi_syms.size());
    if (t.q_cqi) {
      std::vector<uint8_t> qb;
      ul_cqi_code(c.cqi, c.cqi_len, t.q_cqi * c.Qm, qb);
      for (uint32_t k = 0; k < t.q_cqi; k++) {
        uint32_t v = 0;
        for (uint32_t b = 0; b < c.Qm; b++) v = (v << 1) | qb[k * c.Qm + b];
        cqi_syms.push_back((uint8_t)v);
      }
    }
    // UL-SCH data bits: the 12 data symbols' cells less the CQI and RI ones (normal CP, no SRS)
    const uint32_t G = (12 * t.M - t.q_cqi - t.q_ri) * c.Qm;
    t.iq_off = iq_samples;
    iq_samples += 15 * (size_t)N;
    t.pay_off = (uint32_t)payload_bytes;
    payload_bytes += c.tbs / 8;
    t.sym_off = (uint32_t)sym_bytes;
    sym_bytes += 12 * (size_t)t.M;
    t.tbs = c.tbs;
    t.scr_off = (uint32_t)scr.size();
    const uint32_t n_scr = 12 * t.M * c.Qm;   // 36.211 5.3.1 scrambles every coded bit of the subframe (UCI too)
    {
      const auto key = std::make_pair((c.rnti << 14) | (c.sf_idx << 9) | c.cell_id, n_scr);
      auto it = scr_cache.find(key);
      if (it == scr_cache.end()) {
        if (scr_cache.size() >= SCR_CACHE_MAX) scr_cache.clear();
        std::vector<uint32_t> wv((n_scr + 31) / 32 + 1, 0u);
        gold_words(key.first, n_scr, wv.data());
        it = scr_cache.emplace(key, std::move(wv)).first;
      }
      scr.insert(scr.end(), it->second.begin(), it->second.end());
    }
    // segmentation of (TB || CRC24A), 36.212 5.1.2 (sg above); the data follow the CQI symbols in g (5.2.2.7)
    tb_cb0.push_back((uint32_t)cbs.size());
    uint32_t byte0 = 0, sym = t.q_cqi;
    for (uint32_t r = 0; r < sg.C; r++) {
      MiUlCb b{};
      b.tx = i;
      b.K = r < sg.Cm ? sg.Km : sg.Kp;
      b.F = r == 0 ? sg.F : 0;
      b.C = sg.C;
      b.r = r;
      b.E = rm_E(G, sg.C, c.Qm, 1, r);
      b.byte0 = byte0;
      b.nbytes = (b.K - b.F - (sg.C > 1 ? 24 : 0)) / 8;
      byte0 += b.nbytes;
      b.sym0 = sym;
      sym += b.E / c.Qm;
      if (!pi_off.count(b.K)) {
        auto& pi = pi_cache[b.K];
        if (pi.empty()) qpp_table(b.K, pi);
        pi_off[b.K] = (uint32_t)kdata.size();
        kdata.insert(kdata.end(), pi.begin(), pi.end());
      }
      b.pi_off = pi_off[b.K];
      const auto key = std::make_pair(b.K, b.F);
      SelTab& st = sel_cache[key];
      if (st.sel.empty()) {   // selection table and per-rv start ranks of (K, F), kept across builds
        std::vector<uint32_t> pos;
        std::vector<int32_t> rank;
        uint32_t Nv = 0;
        cb_pos_table(b.K, pos);
        cb_rank_table(b.K, b.F, rank, &Nv);
        st.sel.assign(Nv, 0);
        for (uint32_t tt = 0; tt < pos.size(); tt++)
          if (rank[pos[tt]] >= 0) st.sel[(uint32_t)rank[pos[tt]]] = tt;
        for (uint32_t rv = 0; rv < 4; rv++) {   // rank of the first non-null position at or after k0(rv)
          const uint32_t k0 = k0_of(b.K, rv);
          uint32_t cnt = 0;
          for (uint32_t p = 0; p < k0 && p < rank.size(); p++) cnt += rank[p] >= 0 ? 1 : 0;
          st.r0[rv] = cnt % Nv;
        }
      }
      if (!sel_off.count(key)) {
        sel_off[key] = (uint32_t)kdata.size();
        kdata.insert(kdata.end(), st.sel.begin(), st.sel.end());
      }
      b.sel_off = sel_off[key];
      b.Nv = (uint32_t)st.sel.size();
      b.r0 = st.r0[c.rv];
      cbs.push_back(b);
    }
    // HARQ-ACK on PUSCH (36.212 5.2.2.6): Q'_ACK = min(ceil(O M 12 beta / sum K_r), 4 M), encoded block
    // of Tables 5.2.2.6-1 / -2 (x / y placeholders), inserted by the modulation kernel
    if (c.ack_len) {
      if (c.ack_len > 2) {
        set_error("HARQ-ACK on PUSCH: 1 or 2 bits");
        return -1;
      }
      const uint64_t num = (uint64_t)c.ack_len * t.M * 12 * BETA8_ACK[c.I_offset_ack > 14 ? 14 : c.I_offset_ack];
      const uint64_t qp = (num + 8 * sumK - 1) / (8 * sumK);
      t.q_ack = (uint32_t)(qp < 4ull * t.M ? qp : 4ull * t.M);
      t.ack_nblk = uci_block(c.ack_len, c.ack, c.Qm, t.ack_sym);
    }
    if (c.ri_len) t.ri_nblk = uci_block(c.ri_len, c.ri, c.Qm, t.ri_sym);   // Tables 5.2.2.6-3 / -4
    if (byte0 != c.tbs / 8 + 3 || sym != 12 * t.M - t.q_ri) {
      set_error("UL planner: segmentation / rate-matching bookkeeping");
      return -1;
    }
    txs.push_back(t);
    algo_bytes += (double)c.tbs / 8 + 15.0 * N * 8;
  }
  tb_cb0.push_back((uint32_t)cbs.size());
  return 0;
}

}  // namespace mi

// 36.211 5.3.4, PUSCH hopping type 2 (include/mi_ul.h documents the mapping)
extern "C" int mi_ul_hop_type2(uint32_t nof_prb, uint32_t n_ho, uint32_t n_sb, int intra, uint32_t cell_id,
                               uint32_t n_vrb, uint32_t L, uint32_t ns, uint32_t current_tx_nb) {
  if (n_sb < 1 || n_sb > 4 || L < 1 || ns >= 20 || n_vrb + L > nof_prb) return -1;
  const uint32_t ho = n_ho + (n_ho & 1u);                 // N~_HO
  const uint32_t nsb_rb = n_sb == 1 ? nof_prb : (nof_prb > ho + (nof_prb & 1u) ? (nof_prb - ho - (nof_prb & 1u)) / n_sb : 0);
  const uint32_t shift = n_sb == 1 ? 0u : ho / 2;
  if (nsb_rb == 0) return -1;
  const uint32_t i = intra ? ns : ns / 2;
  std::vector<uint8_t> c(10 * 20 + 10);
  mi::gold_bits(cell_id, (uint32_t)c.size(), c.data());
  // f_hop(i) = (f_hop(i - 1) + sum_{k = 10 i + 1}^{10 i + 9} c(k) 2^(k - (10 i + 1))) mod N_sb       (N_sb = 2)
  //          = (f_hop(i - 1) + (sum ...) mod (N_sb - 1) + 1) mod N_sb                            (N_sb > 2)
  uint32_t fhop = 0;
  for (uint32_t j = 0; j <= i && n_sb > 1; j++) {
    uint32_t sum = 0;
    for (uint32_t k = 10 * j + 1; k <= 10 * j + 9; k++) sum += (uint32_t)c[k] << (k - (10 * j + 1));
    fhop = n_sb == 2 ? (fhop + sum) % n_sb : (fhop + sum % (n_sb - 1) + 1) % n_sb;
  }
  const uint32_t fm = n_sb > 1 ? c[10 * i] : intra ? (i & 1u) : (current_tx_nb & 1u);
  uint32_t lo = 0xFFFFFFFFu, hi = 0;
  for (uint32_t v = n_vrb; v < n_vrb + L; v++) {
    if (v < shift) return -1;
    const uint32_t vt = v - shift;
    if (vt >= nsb_rb * n_sb) return -1;
    const uint32_t pt = (vt + fhop * nsb_rb + ((nsb_rb - 1) - 2 * (vt % nsb_rb)) * fm) % (nsb_rb * n_sb);
    const uint32_t p = pt + shift;
    lo = p < lo ? p : lo;
    hi = p > hi ? p : hi;
  }
  if (hi - lo + 1 != L || hi >= nof_prb) return -1;
  return (int)lo;
}

