// tx.cpp -- synthetic eNB-side PDSCH transmitter (host C++), the input generator of bench.py.
//
// Produces what srsUE's radio hands to phch_worker (/root/reference/ue/src/phy/phch_recv.cc:321
// -> phch_worker.cc:254): one subframe of cf32 IQ carrying a known transport block.  Chain:
// CRC24A -> segmentation (+CRC24B) -> PCCC turbo code -> sub-block interleaving + bit selection
// -> Gold scrambling -> Gray QAM -> (SFBC for 2 ports) -> RE mapping with CRS and PCFICH ->
// IFFT scaled 1/sqrt(N) + cyclic prefix -> flat per-port channel + AWGN.  36.211 / 36.212.
#include <math.h>
#include <string.h>

#include <vector>

#include "dl_common.h"
#include "mi_dl.h"
#include "tables.h"
#include "sync.h"

namespace mi {

static uint64_t sm64(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// 8-state RSC step (g0 = 1 + D^2 + D^3 feedback, g1 = 1 + D + D^3): returns parity, updates state
static inline int rsc(int& s, int u) {
  const int a = u ^ ((s >> 1) & 1) ^ (s & 1);
  const int z = a ^ ((s >> 2) & 1) ^ (s & 1);
  s = (a << 2) | (s >> 1);
  return z;
}

// d: 3(K+4) entries, 0/1 or 2 = <NULL>
void turbo_encode(const uint8_t* c, uint32_t K, uint32_t F, uint8_t* d) {
  std::vector<uint32_t> pi;
  qpp_table(K, pi);
  int s1 = 0, s2 = 0;
  for (uint32_t k = 0; k < K; k++) {
    d[3 * k] = c[k];
    d[3 * k + 1] = (uint8_t)rsc(s1, c[k]);
    d[3 * k + 2] = (uint8_t)rsc(s2, c[pi[k]]);
  }
  uint8_t t[12];
  for (int j = 0; j < 3; j++) {   // termination: input = feedback so the register fills with 0
    const int u1 = ((s1 >> 1) ^ s1) & 1;
    t[2 * j] = (uint8_t)u1; t[2 * j + 1] = (uint8_t)rsc(s1, u1);
    const int u2 = ((s2 >> 1) ^ s2) & 1;
    t[6 + 2 * j] = (uint8_t)u2; t[6 + 2 * j + 1] = (uint8_t)rsc(s2, u2);
  }
  memcpy(d + 3 * K, t, 12);
  for (uint32_t k = 0; k < F; k++) d[3 * k] = d[3 * k + 1] = 2;
}

static void rate_match(const uint8_t* d, uint32_t K, uint32_t E, uint32_t rv, uint8_t* e) {
  std::vector<uint32_t> pos;
  cb_pos_table(K, pos);
  const uint32_t Ncb = ncb_of(K);
  std::vector<int32_t> w(Ncb, -1);
  for (uint32_t t = 0; t < 3 * (K + 4); t++)
    if (d[t] != 2) w[pos[t]] = d[t];
  const uint32_t k0 = k0_of(K, rv);
  for (uint32_t k = 0, j = 0; k < E; j++) {
    const int32_t v = w[(k0 + j) % Ncb];
    if (v >= 0) e[k++] = (uint8_t)v;
  }
}

static inline double pam(int b0, int b1, int b2, uint32_t Qm) {
  if (Qm == 2) return (1 - 2 * b0) * 0.70710678118654752440;
  if (Qm == 4) return (1 - 2 * b0) * (1 + 2 * b1) / sqrt(10.0);
  return (1 - 2 * b0) * (4 - (1 - 2 * b1) * (2 - (1 - 2 * b2))) / sqrt(42.0);
}
static void modulate(const uint8_t* b, uint32_t Qm, double* re, double* im) {
  *re = pam(b[0], Qm > 2 ? b[2] : 0, Qm > 4 ? b[4] : 0, Qm);
  *im = pam(b[1], Qm > 2 ? b[3] : 0, Qm > 4 ? b[5] : 0, Qm);
}

// Stockham radix-2/3 inverse DFT (unnormalised), double precision, table twiddles
static void idft(std::vector<double>& a, int N) {
  std::vector<double> b(2 * N), tc(N), ts(N);
  for (int t = 0; t < N; t++) { tc[t] = cos(2.0 * M_PI * t / N); ts[t] = sin(2.0 * M_PI * t / N); }
  int Ns = 1;
  std::vector<int> rad;
  int m = N;
  while (m % 3 == 0) { rad.push_back(3); m /= 3; }
  while (m > 1) { rad.push_back(2); m /= 2; }
  for (int R : rad) {
    for (int j = 0; j < N / R; j++) {
      double vr[3], vi[3];
      const int k = j % Ns;
      for (int r = 0; r < R; r++) {
        const double xr = a[2 * (j + r * N / R)], xi = a[2 * (j + r * N / R) + 1];
        const int t = (k * r * (N / (Ns * R))) % N;
        vr[r] = xr * tc[t] - xi * ts[t];
        vi[r] = xr * ts[t] + xi * tc[t];
      }
      const int base = (j / Ns) * Ns * R + k;
      for (int q = 0; q < R; q++) {
        double sr = 0, si = 0;
        for (int r = 0; r < R; r++) {
          const int t = (q * r * (N / R)) % N;
          sr += vr[r] * tc[t] - vi[r] * ts[t];
          si += vr[r] * ts[t] + vi[r] * tc[t];
        }
        b[2 * (base + q * Ns)] = sr;
        b[2 * (base + q * Ns) + 1] = si;
      }
    }
    a.swap(b);
    Ns *= R;
  }
}

int tx_subframe(const mi_dl_sf_cfg_t* c, const uint8_t* tb, const float* h, float snr_db, uint64_t seed, float* iq) {
  const int N = symbol_sz(c->nof_prb);
  if (N < 0 || c->tbs == 0 || c->tbs % 8 || (c->tm == 2 && c->nof_ports != 2)) return -1;
  const uint32_t W = 12 * c->nof_prb, P = c->nof_ports, A = c->tbs, Qm = c->Qm;
  // transport block + CRC24A
  std::vector<uint8_t> b(A + 24);
  for (uint32_t i = 0; i < A; i++) b[i] = (tb[i / 8] >> (7 - i % 8)) & 1;
  {
    uint32_t crc = 0;
    for (uint32_t i = 0; i < A; i++) {
      const uint32_t fb = ((crc >> 23) ^ b[i]) & 1u;
      crc = ((crc << 1) & 0xFFFFFFu) ^ (fb ? 0x864CFBu : 0u);
    }
    for (int i = 0; i < 24; i++) b[A + i] = (crc >> (23 - i)) & 1;
  }
  CbSegm sg;
  if (cbsegm(A, &sg)) return -1;
  std::vector<uint32_t> re;
  const uint32_t nre = pdsch_re_list(c->cell_id, c->nof_prb, P, c->cfi, c->sf_idx, c->prb_mask, re);
  if (c->tm == 2 && (nre & 1)) return -1;
  const uint32_t G = nre * Qm, NL = c->tm == 2 ? (c->nl_td ? c->nl_td : 2) : 1;
  std::vector<uint8_t> f(G), cb(KMAX), d(3 * (KMAX + 4));
  uint32_t pb = 0, pf = 0;
  for (uint32_t r = 0; r < sg.C; r++) {
    const uint32_t K = r < sg.Cm ? sg.Km : sg.Kp, F = r == 0 ? sg.F : 0, L = sg.C > 1 ? 24 : 0;
    for (uint32_t k = 0; k < K - L; k++) cb[k] = k < F ? 0 : b[pb++];
    if (L) {
      uint32_t crc = 0;
      for (uint32_t k = 0; k < K - L; k++) {
        const uint32_t fb = ((crc >> 23) ^ cb[k]) & 1u;
        crc = ((crc << 1) & 0xFFFFFFu) ^ (fb ? 0x800063u : 0u);
      }
      for (int i = 0; i < 24; i++) cb[K - L + i] = (crc >> (23 - i)) & 1;
    }
    turbo_encode(cb.data(), K, F, d.data());
    const uint32_t E = rm_E(G, sg.C, Qm, NL, r);
    rate_match(d.data(), K, E, c->rv, f.data() + pf);
    pf += E;
  }
  std::vector<uint8_t> cs(G + 32);
  gold_bits((c->rnti << 14) | (c->sf_idx << 9) | c->cell_id, G, cs.data());
  for (uint32_t i = 0; i < G; i++) f[i] ^= cs[i];

  std::vector<double> grid((size_t)P * NSYMB * W * 2, 0.0);
  auto at = [&](uint32_t p, uint32_t idx) -> double* { return &grid[((size_t)p * NSYMB * W + idx) * 2]; };
  const double s2 = 0.70710678118654752440;
  auto put_sfbc = [&](double x0r, double x0i, double x1r, double x1i, uint32_t ia, uint32_t ib) {
    double* y = at(0, ia); y[0] = s2 * x0r; y[1] = s2 * x0i;
    y = at(1, ia); y[0] = -s2 * x1r; y[1] = s2 * x1i;
    y = at(0, ib); y[0] = s2 * x1r; y[1] = s2 * x1i;
    y = at(1, ib); y[0] = s2 * x0r; y[1] = -s2 * x0i;
  };
  for (uint32_t i = 0; i < nre; i += (c->tm == 2 ? 2 : 1)) {
    double xr, xi;
    modulate(&f[(size_t)i * Qm], Qm, &xr, &xi);
    if (c->tm != 2) {
      double* y = at(0, re[i]); y[0] = xr; y[1] = xi;
    } else {
      double yr, yi;
      modulate(&f[(size_t)(i + 1) * Qm], Qm, &yr, &yi);
      put_sfbc(xr, xi, yr, yi, re[i], re[i + 1]);
    }
  }
  float rs[4 * NRB_MAX];
  for (uint32_t p = 0; p < P; p++)
    for (uint32_t l = 0; l < (uint32_t)NSYMB; l++) {
      const uint32_t lp = l % 7;
      if (lp != 0 && lp != 4) continue;
      const uint32_t v = p == 0 ? (lp == 0 ? 0 : 3) : (lp == 0 ? 3 : 0), off = (v + c->cell_id % 6) % 6;
      crs_seq(c->cell_id, 2 * c->sf_idx + l / 7, lp, rs);
      for (uint32_t m = 0; m < 2 * c->nof_prb; m++) {
        double* y = at(p, l * W + 6 * m + off);
        y[0] = rs[2 * (m + NRB_MAX - c->nof_prb)];
        y[1] = rs[2 * (m + NRB_MAX - c->nof_prb) + 1];
      }
    }
  if (c->cfi >= 1 && c->cfi <= 3) {
    uint8_t cw[32], sc[32];
    uint32_t kk[16];
    cfi_codeword(c->cfi, cw);
    gold_bits(pcfich_cinit(c->cell_id, c->sf_idx), 32, sc);
    for (int i = 0; i < 32; i++) cw[i] ^= sc[i];
    pcfich_k(c->cell_id, c->nof_prb, kk);
    for (int i = 0; i < 16; i += (P == 2 ? 2 : 1)) {
      double xr, xi;
      modulate(cw + 2 * i, 2, &xr, &xi);
      if (P == 1) {
        double* y = at(0, kk[i]); y[0] = xr; y[1] = xi;
      } else {
        double yr, yi;
        modulate(cw + 2 * (i + 1), 2, &yr, &yi);
        put_sfbc(xr, xi, yr, yi, kk[i], kk[i + 1]);
      }
    }
  }
  const int SF = sf_len(N);
  std::vector<double> acc((size_t)SF * 2, 0.0), X(2 * N);
  const double nrm = 1.0 / sqrt((double)N);
  for (uint32_t p = 0; p < P; p++) {
    double hr = h ? h[2 * p] : (p == 0 ? 1.0 : 0.0), hi = h ? h[2 * p + 1] : 0.0;
    size_t pos = 0;
    for (int l = 0; l < NSYMB; l++) {
      std::fill(X.begin(), X.end(), 0.0);
      for (uint32_t k = 0; k < W; k++) {
        const int bin = sc_bin((int)k, (int)W, N);
        X[2 * bin] = *at(p, l * W + k);
        X[2 * bin + 1] = *(at(p, l * W + k) + 1);
      }
      idft(X, N);
      const int cp = cp_len(N, l % 7);
      for (int n = 0; n < cp + N; n++) {
        const int src = n < cp ? N - cp + n : n - cp;
        const double sr = X[2 * src] * nrm, si = X[2 * src + 1] * nrm;
        acc[2 * pos] += hr * sr - hi * si;
        acc[2 * pos + 1] += hr * si + hi * sr;
        pos++;
      }
    }
  }
  const double sigma = snr_db >= 200.0f ? 0.0 : sqrt(pow(10.0, -snr_db / 10.0) / 2.0);
  uint64_t st = seed;
  for (int n = 0; n < SF; n++) {
    double nr = 0, ni = 0;
    if (sigma > 0) {
      const double u1 = ((double)(sm64(st) >> 11) + 0.5) * (1.0 / 9007199254740992.0);
      const double u2 = ((double)(sm64(st) >> 11) + 0.5) * (1.0 / 9007199254740992.0);
      const double rr = sqrt(-2.0 * log(u1));
      nr = rr * cos(2 * M_PI * u2) * sigma;
      ni = rr * sin(2 * M_PI * u2) * sigma;
    }
    iq[2 * n] = (float)(acc[2 * n] + nr);
    iq[2 * n + 1] = (float)(acc[2 * n + 1] + ni);
  }
  return 0;
}

}  // namespace mi

extern "C" int mi_tx_subframe(const mi_dl_sf_cfg_t* cfg, const uint8_t* tb, const float* h_re_im, float snr_db,
                              uint64_t noise_seed, float* iq) {
  return mi::tx_subframe(cfg, tb, h_re_im, snr_db, noise_seed, iq);
}
extern "C" int mi_turbo_encode(const uint8_t* bits, uint32_t K, uint32_t F, uint8_t* d) {
  if (!mi::cb_size_valid(K) || F >= K) return -1;
  mi::turbo_encode(bits, K, F, d);
  return 0;
}
extern "C" int mi_pdsch_G(const mi_dl_sf_cfg_t* c) {
  if (!c || mi::symbol_sz(c->nof_prb) < 0) return -1;
  std::vector<uint32_t> re;
  return (int)(mi::pdsch_re_list(c->cell_id, c->nof_prb, c->nof_ports, c->cfi, c->sf_idx, c->prb_mask, re) * c->Qm);
}
// PSS (symbol 6) + SSS (symbol 5) of subframes 0 / 5 (36.211 6.11), amplitude amp per RE, added to the
// subframe's IQ through the same 1/sqrt(N) OFDM modulation as the PDSCH (a direct 62-bin IDFT)
extern "C" int mi_tx_sync(uint32_t cell_id, uint32_t nof_prb, uint32_t sf_idx, float amp, float* iq) {
  if (sf_idx != 0 && sf_idx != 5) return 0;
  const int Ni = mi::symbol_sz(nof_prb);
  if (Ni < 0 || !iq || cell_id > 503) return -1;
  const uint32_t N = (uint32_t)Ni;
  float2 pss[62];
  float sss[62];
  mi::pss_seq(cell_id % 3, pss);
  mi::sss_seq(cell_id / 3, cell_id % 3, sf_idx == 5, sss);
  const double nrm = amp / sqrt((double)N);
  for (uint32_t l = 5; l <= 6; l++) {
    const uint32_t cp = (uint32_t)mi::cp_len((int)N, (int)(l % 7)), s0 = (uint32_t)mi::symbol_offset((int)N, (int)l) - cp;
    for (uint32_t n = 0; n < N; n++) {
      double re = 0, im = 0;
      for (uint32_t m = 0; m < 62; m++) {
        const double dr = l == 6 ? pss[m].x : sss[m], di = l == 6 ? pss[m].y : 0.0;
        const double ph = 2.0 * M_PI * (double)((uint64_t)mi::sync_bin(m, nof_prb, N) * n % N) / N;
        re += dr * cos(ph) - di * sin(ph);
        im += dr * sin(ph) + di * cos(ph);
      }
      re *= nrm;
      im *= nrm;
      iq[2 * (s0 + cp + n)] += (float)re;
      iq[2 * (s0 + cp + n) + 1] += (float)im;
      if (n >= N - cp) {   // cyclic prefix
        iq[2 * (s0 + n - (N - cp))] += (float)re;
        iq[2 * (s0 + n - (N - cp)) + 1] += (float)im;
      }
    }
  }
  return 1;
}

extern "C" int mi_sf_len(uint32_t nof_prb) {
  const int N = mi::symbol_sz(nof_prb);
  return N < 0 ? -1 : mi::sf_len(N);
}
