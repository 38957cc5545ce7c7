// tb.hip -- transport-block assembly + parallel CRC24A + payload packing (see tb_body.h).
// One 256-thread workgroup per TB; the TB bytes are staged in LDS for the CRC pass.
#include "kernels.h"
#include "tb_body.h"

namespace mi {

constexpr uint32_t TB_MAX_BYTES = 12288;   // >= (max TBS + 24) / 8 for one layer, 110 PRB

__global__ __launch_bounds__(256) void tb_kernel(const uint8_t* __restrict__ cb_bytes, uint8_t* __restrict__ payload,
                                                uint32_t* __restrict__ tb_ok, uint32_t* __restrict__ tb_its,
                                                const uint32_t* __restrict__ cb_its,
                                                const MiTbDesc* __restrict__ tbs,
                                                const uint32_t* __restrict__ cb_list) {
  __shared__ uint8_t buf[TB_MAX_BYTES];
  __shared__ uint32_t red[4];
  const MiTbDesc t = tbs[blockIdx.x];
  const uint32_t* lanes = cb_list + t.cb_list;
  const uint32_t nbytes = (t.tbs + 24) / 8, pbytes = t.tbs / 8;
  for (uint32_t j = threadIdx.x; j < nbytes; j += 256) {
    uint32_t r, off;
    tb_byte_src(t, j, r, off);
    const uint8_t v = cb_bytes[(size_t)lanes[r] * CB_BYTES_STRIDE + off];
    buf[j] = v;
    if (j < pbytes) payload[t.pay_off + j] = v;
  }
  __syncthreads();
  const uint32_t seg = (nbytes + 255) / 256;
  const uint32_t b0 = threadIdx.x * seg;
  uint32_t c = 0;
  if (b0 < nbytes) {
    const uint32_t n = (b0 + seg <= nbytes) ? seg : nbytes - b0;
    c = crc24_bytes(buf + b0, n, CRC24A_POLY);
    c = gf24_mulmod(c, gf24_xpow8(nbytes - b0 - n, CRC24A_POLY), CRC24A_POLY);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c ^= __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t crc = red[0] ^ red[1] ^ red[2] ^ red[3];
    uint32_t its = 0;
    for (uint32_t r = 0; r < t.C; r++) its = cb_its[lanes[r]] > its ? cb_its[lanes[r]] : its;
    tb_ok[blockIdx.x] = crc == 0;
    tb_its[blockIdx.x] = its;
  }
}

void launch_tb(const uint8_t* cb_bytes, uint8_t* payload, uint32_t* tb_crc_ok, uint32_t* tb_its, const uint32_t* cb_its,
               const MiTbDesc* tbs, uint32_t n_tb, const uint32_t* cb_list, hipStream_t st) {
  if (!n_tb) return;
  hipLaunchKernelGGL(tb_kernel, dim3(n_tb), dim3(256), 0, st, cb_bytes, payload, tb_crc_ok, tb_its, cb_its, tbs,
                     cb_list);
}

}  // namespace mi
