/*
 * srslte/utils/bit.h -- the srsLTE 1.0 bit utilities srsUE uses beside the PHY: MAC PDU fields
 * (reference ue/src/mac/pdu.cc:776,791 through srslte/srslte.h), the MIB payload handed to the MAC
 * (ue/src/phy/phch_recv.cc:220) and RRC (ue/src/upper/rrc.cc:32).  Bits are one per byte (0/1),
 * MSB first; srslte_bit_pack / _unpack advance the caller's cursor by nof_bits.
 * Implemented in srsue_amd/csrc/srslte_util.cpp.
 */
#ifndef SRSLTE_MI355X_BIT_H
#define SRSLTE_MI355X_BIT_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
void srslte_bit_pack_vector(uint8_t *unpacked, uint8_t *packed, int nof_bits);
void srslte_bit_unpack_vector(uint8_t *packed, uint8_t *unpacked, int nof_bits);
uint32_t srslte_bit_pack(uint8_t **bits, int nof_bits);
void srslte_bit_unpack(uint32_t value, uint8_t **bits, int nof_bits);
#ifdef __cplusplus
}
#endif
#endif
