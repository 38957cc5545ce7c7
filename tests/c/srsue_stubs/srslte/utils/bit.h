/* TEST STUB (compile check only): srsLTE bit utilities srsUE's MAC includes (reference
 * ue/hdr/mac/pdu.h, <srslte/utils/bit.h>).  Not part of the DL drop-in. */
#pragma once
#include <stdint.h>
void srslte_bit_pack_vector(uint8_t *unpacked, uint8_t *packed, int nof_bits);
void srslte_bit_unpack_vector(uint8_t *packed, uint8_t *unpacked, int nof_bits);
uint32_t srslte_bit_pack(uint8_t **bits, int nof_bits);
void srslte_bit_unpack(uint32_t value, uint8_t **bits, int nof_bits);
