// tb.hip -- transport-block assembly + CRC24A check + payload packing (see tb_body.h).
// One 256-thread workgroup per TB: the payload bytes are copied code block by code block (each code
// block's payload is a contiguous, byte-aligned run of the TB), and the TB CRC is combined from the
// turbo decoder's per-code-block partial registers -- no pass over the TB bytes.
#include "kernels.h"
#include "tb_body.h"

namespace mi {

__global__ __launch_bounds__(256) void tb_kernel(const uint8_t* __restrict__ cb_bytes, uint8_t* __restrict__ payload,
                                                uint32_t* __restrict__ tb_ok, uint32_t* __restrict__ tb_its,
                                                const uint32_t* __restrict__ cb_its,
                                                const uint32_t* __restrict__ cb_tbp,
                                                const MiTbDesc* __restrict__ tbs,
                                                const uint32_t* __restrict__ cb_list) {
  const MiTbDesc t = tbs[blockIdx.x];
  const uint32_t* lanes = cb_list + t.cb_list;
  const uint32_t pbytes = t.tbs / 8;
  // wavefront w copies code blocks w, w + 4, ...: each block's start in the TB is arithmetic, so the
  // blocks' loads are independent (no serial chain over the code blocks)
  const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  for (uint32_t r = wv; r < t.C; r += 4) {
    uint32_t start = 0;
    for (uint32_t j = 0; j < r; j++) start += tb_cb_nbytes(t, j);
    const uint32_t n = tb_cb_nbytes(t, r);
    const uint8_t* src = cb_bytes + (size_t)lanes[r] * CB_BYTES_STRIDE + (r == 0 ? t.F / 8 : 0);
    uint8_t* dst = payload + t.pay_off + start;
    for (uint32_t j = ln; j < n && start + j < pbytes; j += 64) dst[j] = src[j];
  }
  if (threadIdx.x < 64) {
    uint32_t c = 0, its = 0;
    for (uint32_t r = threadIdx.x; r < t.C; r += 64) {
      c ^= tb_crc_term(t, r, cb_tbp[lanes[r]]);
      its = cb_its[lanes[r]] > its ? cb_its[lanes[r]] : its;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      c ^= __shfl_xor(c, o, 64);
      const uint32_t oi = __shfl_xor(its, o, 64);
      its = oi > its ? oi : its;
    }
    if (threadIdx.x == 0) {
      tb_ok[blockIdx.x] = c == 0;
      tb_its[blockIdx.x] = its;
    }
  }
}

void launch_tb(const uint8_t* cb_bytes, uint8_t* payload, uint32_t* tb_crc_ok, uint32_t* tb_its, const uint32_t* cb_its,
               const uint32_t* cb_tbp, const MiTbDesc* tbs, uint32_t n_tb, const uint32_t* cb_list, hipStream_t st) {
  if (!n_tb) return;
  hipLaunchKernelGGL(tb_kernel, dim3(n_tb), dim3(256), 0, st, cb_bytes, payload, tb_crc_ok, tb_its, cb_its, cb_tbp,
                     tbs, cb_list);
}

}  // namespace mi
