// tb.hip -- transport-block assembly + CRC24A check + payload packing (see tb_body.h).
// One workgroup per TB (16 wavefronts for small batches, 4 for large ones): each code block's payload is a contiguous, byte-aligned run of the
// TB whose start is arithmetic, so every wavefront copies whole code blocks with one batch of
// independent loads per lane, and the TB CRC is combined from the turbo decoder's per-code-block partial
// registers with planner-precomputed multipliers -- no pass over the TB bytes.
#include "kernels.h"
#include "tb_body.h"

namespace mi {

constexpr uint32_t TB_MAX_C = 128;   // code blocks per TB (LTE: at most 64)
constexpr int TB_BATCH = 12;          // independent byte loads in flight per lane (a code block: <= 765 bytes)

template <uint32_t TB_NW>   // wavefronts per TB
__global__ __launch_bounds__(64 * TB_NW) void tb_kernel(const uint8_t* __restrict__ cb_bytes, uint8_t* __restrict__ payload,
                                                uint32_t* __restrict__ tb_ok, uint32_t* __restrict__ tb_its,
                                                const uint32_t* __restrict__ cb_its,
                                                const uint32_t* __restrict__ cb_tbp,
                                                const MiTbDesc* __restrict__ tbs,
                                                const uint32_t* __restrict__ cb_list,
                                                const uint32_t* __restrict__ kdata, uint32_t copy) {
  __shared__ uint32_t s_start[TB_MAX_C + 1], s_src[TB_MAX_C];
  const MiTbDesc t = tbs[blockIdx.x];
  const uint32_t* lanes = cb_list + t.cb_list;
  const uint32_t pbytes = t.tbs / 8, tid = threadIdx.x;
  // payload start of each code block's byte run (closed form) and where its bytes sit in cb_bytes
  for (uint32_t r = tid; r <= t.C; r += 64 * TB_NW) {
    const uint32_t nm = r < t.Cm ? r : t.Cm;
    s_start[r] = nm * (t.Km / 8) + (r - nm) * (t.Kp / 8) - (r ? t.F / 8 : 0) - (t.C > 1 ? 3 * r : 0);
    if (r < t.C) s_src[r] = lanes[r] * CB_BYTES_STRIDE + (r == 0 ? t.F / 8 : 0);
  }
  __syncthreads();
  // copy: wavefront w copies code blocks w, w + TB_NW, ...; a code block's bytes (<= 765) are one batch
  // of TB_BATCH independent loads per lane, issued before the stores (a byte-per-iteration loop
  // serialised one load round trip per 64 bytes: 30 us for one TB)
  const uint32_t wv = tid >> 6, ln = tid & 63;
  for (uint32_t r = wv; copy && r < t.C; r += TB_NW) {   // copy = 0: the packed decoder wrote the payload
    const uint32_t st0 = s_start[r], n = s_start[r + 1] - st0, src = s_src[r];
    for (uint32_t j0 = ln; j0 < n; j0 += 64u * TB_BATCH) {
      uint8_t v[TB_BATCH];
#pragma unroll
      for (int k = 0; k < TB_BATCH; k++) {
        const uint32_t j = j0 + 64u * k;
        if (j < n && st0 + j < pbytes) v[k] = cb_bytes[(size_t)src + j];
      }
#pragma unroll
      for (int k = 0; k < TB_BATCH; k++) {
        const uint32_t j = j0 + 64u * k;
        if (j < n && st0 + j < pbytes) payload[t.pay_off + st0 + j] = v[k];
      }
    }
  }
  if (tid < 64) {
    // TB CRC24A from the code blocks' partial registers: term r = part_r x^(8 bytes after r) mod g
    // (multipliers precomputed by the planner, tb_body.h tb_crc_term)
    uint32_t c = 0, its = 0;
    for (uint32_t r = tid; r < t.C; r += 64) {
      c ^= gf24_mulmod(cb_tbp[lanes[r]], kdata[t.crc_mul + r], CRC24A_POLY);
      its = cb_its[lanes[r]] > its ? cb_its[lanes[r]] : its;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      c ^= __shfl_xor(c, o, 64);
      const uint32_t oi = __shfl_xor(its, o, 64);
      its = oi > its ? oi : its;
    }
    if (tid == 0) {
      tb_ok[blockIdx.x] = c == 0;
      tb_its[blockIdx.x] = its;
    }
  }
}

void launch_tb(const uint8_t* cb_bytes, uint8_t* payload, uint32_t* tb_crc_ok, uint32_t* tb_its, const uint32_t* cb_its,
               const uint32_t* cb_tbp, const MiTbDesc* tbs, uint32_t n_tb, const uint32_t* cb_list,
               const uint32_t* kdata, bool copy, hipStream_t st) {
  if (!n_tb) return;
  // small batches (per-TTI latency): 16 wavefronts, all code blocks of a 20 MHz TB in one round;
  // large batches: 4 wavefronts per TB, the batch itself fills the GPU (16 measured 50 % slower there)
  if (n_tb < 1024)
    hipLaunchKernelGGL(tb_kernel<16>, dim3(n_tb), dim3(1024), 0, st, cb_bytes, payload, tb_crc_ok, tb_its, cb_its,
                       cb_tbp, tbs, cb_list, kdata, (uint32_t)copy);
  else
    hipLaunchKernelGGL(tb_kernel<4>, dim3(n_tb), dim3(256), 0, st, cb_bytes, payload, tb_crc_ok, tb_its, cb_its,
                       cb_tbp, tbs, cb_list, kdata, (uint32_t)copy);
}

}  // namespace mi
