// tb_body.h -- transport-block assembly and CRC24A (36.212 5.1.1 / 5.1.2), the tail of
// srslte_pdsch_decode_rnti (/root/reference/ue/src/phy/phch_worker.cc:347-348): code-block bits
// without filler and CB CRC are concatenated, the TB CRC24A is checked (return 0 <=> CRC ok) and
// the payload is packed MSB-first into bytes (srsUE treats it as bytes: ue/src/mac/demux.cc:180).
//
// The TB CRC is linear over GF(2): the turbo decoder accumulates, per code block, the register
// contribution of its decided payload bits (TdecLaneResult::tb_part, per-K table crc_p), and the TB
// register is XOR_r tb_part_r * x^(bits after code block r) mod g (CRC(A||B) = CRC(A) x^|B| + CRC(B))
// -- no pass over the TB bytes.
#pragma once
#include "dl_common.h"
#ifndef MI_HD
#define MI_HD __host__ __device__
#endif

namespace mi {

constexpr uint32_t CRC24A_POLY = 0x864CFBu;
constexpr uint32_t CRC24B_POLY = 0x800063u;

MI_HD inline uint32_t crc24_bytes(const uint8_t* p, uint32_t n, uint32_t poly) {
  uint32_t crc = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t byte = p[i];
    for (int b = 7; b >= 0; b--) {
      const uint32_t fb = ((crc >> 23) ^ (byte >> b)) & 1u;
      crc = ((crc << 1) & 0xFFFFFFu) ^ (fb ? poly : 0u);
    }
  }
  return crc;
}

// CRC register after one message byte b from the zero state (byte-table entry)
MI_HD inline uint32_t crc24_byte_entry(uint32_t b, uint32_t poly) {
  uint32_t c = b << 16;
  for (int i = 0; i < 8; i++) c = ((c << 1) & 0xFFFFFFu) ^ ((c & 0x800000u) ? poly : 0u);
  return c;
}

// a * b mod (x^24 + poly) over GF(2)
MI_HD inline uint32_t gf24_mulmod(uint32_t a, uint32_t b, uint32_t poly) {
  uint32_t r = 0;
  for (int i = 23; i >= 0; i--) {
    r <<= 1;
    if (r & 0x1000000u) r ^= 0x1000000u | poly;
    if ((b >> i) & 1u) r ^= a;
  }
  return r;
}

// x^(8 n) mod (x^24 + poly)
MI_HD inline uint32_t gf24_xpow8(uint32_t n, uint32_t poly) {
  uint32_t res = 1, base = 0x100u;
  while (n) {
    if (n & 1u) res = gf24_mulmod(res, base, poly);
    base = gf24_mulmod(base, base, poly);
    n >>= 1;
  }
  return res;
}

// payload bytes code block r contributes to the TB (after filler, without the CB CRC)
MI_HD inline uint32_t tb_cb_nbytes(const MiTbDesc& t, uint32_t r) {
  const uint32_t Kr = r < t.Cm ? t.Km : t.Kp;
  return Kr / 8 - (r == 0 ? t.F / 8 : 0) - (t.C > 1 ? 3 : 0);
}

// code block r's term of the TB CRC24A register
MI_HD inline uint32_t tb_crc_term(const MiTbDesc& t, uint32_t r, uint32_t part) {
  uint32_t after = 0;
  for (uint32_t j = r + 1; j < t.C; j++) after += tb_cb_nbytes(t, j);
  return gf24_mulmod(part, gf24_xpow8(after, CRC24A_POLY), CRC24A_POLY);
}

}  // namespace mi
