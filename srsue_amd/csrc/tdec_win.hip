// tdec_win.hip -- latency form of the int16 turbo decoder: one code block per workgroup, its trellis
// split into exact segments, one per thread (algorithm and exactness argument in tdec_win_body.h).
// Used for batches too small to fill the GPU with 64-code-block wavefronts (a single subframe: 13
// code blocks = one fifth of ONE wavefront in the lane-per-code-block kernel).
#include "kernels.h"
#include "tdec_win_body.h"

namespace mi {

struct TdecWinOut {
  uint8_t* cb_bytes;
  uint32_t* its;
  uint32_t* crc_ok;
  uint32_t* tb_part;
};

template <int P>
__device__ __forceinline__ uint32_t block_xor(uint32_t v, uint32_t* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v ^= (uint32_t)__shfl_xor((int)v, o, 64);
  const uint32_t t = threadIdx.x;
  if ((t & 63) == 0) red[t >> 6] = v;
  __syncthreads();
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < P / 64; i++) r ^= red[i];
  __syncthreads();
  return r;
}

// one constituent decoder over all segments: first passes + fix-up rounds, backward then forward
template <bool DEC2>
__device__ __forceinline__ void win_half(const WinCb& c, uint32_t t) {
  if (t < c.nseg) win_bwd_first<DEC2>(c, t);
  __syncthreads();
  for (;;) {
    const bool act = t + 1 < c.nseg;
    float nb[8];
    if (act) ck_get(c.bend + (t + 1) * 8, nb);
    __syncthreads();
    const bool ch = act ? win_bwd_fix<DEC2>(c, t, nb) : false;
    if (!__syncthreads_or(ch)) break;
  }
  if (t < c.nseg) win_fwd_first<DEC2>(c, t);
  __syncthreads();
  for (;;) {
    const bool act = t > 0 && t < c.nseg;
    float na[8];
    if (act) ck_get(c.aend + (t - 1) * 8, na);
    __syncthreads();
    const bool ch = act ? win_fwd_fix<DEC2>(c, t, na) : false;
    if (!__syncthreads_or(ch)) break;
  }
}

template <int P>
__global__ __launch_bounds__(P) void tdec_win_kernel(const float* __restrict__ sb, TdecWinOut out,
                                                     const MiGroupDesc* __restrict__ groups,
                                                     const MiLaneDesc* __restrict__ lanes,
                                                     const MiKTab* __restrict__ ktabs,
                                                     const uint32_t* __restrict__ kdata, uint32_t max_its,
                                                     uint32_t early_stop) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ uint32_t crc8[256];
  __shared__ uint32_t red[P / 64];
  const uint32_t li = blockIdx.x;
  const MiLaneDesc ld = lanes[li];
  if (!ld.valid) return;
  const MiGroupDesc g = groups[li / LANES];
  const MiKTab kt = ktabs[g.ktab];
  const uint32_t t = threadIdx.x, K = g.K;
  WinCb c;
  c.K = K;
  win_geometry(K, P, c.S, c.nseg);
  unsigned char* p = smem;
  c.q = reinterpret_cast<int16_t*>(p);   p += ((3 * K + 12) * 2 + 15) / 16 * 16;
  c.pi = reinterpret_cast<uint16_t*>(p); p += K * 2;
  c.d = reinterpret_cast<int16_t*>(p);   p += K * 2;
  c.w = reinterpret_cast<int16_t*>(p);   p += K * 2;
  c.dec = p;                             p += (K + 15) / 16 * 16;
  c.bck = reinterpret_cast<int16_t*>(p); p += (K / 4 + 1) * 16;
  c.ack = reinterpret_cast<int16_t*>(p); p += (K / 4 + 1) * 16;
  c.bend = reinterpret_cast<int16_t*>(p); p += P * 16;
  c.aend = reinterpret_cast<int16_t*>(p);
  c.lmap = reinterpret_cast<uint8_t*>(c.bck);   // bck + ack: 2 (K/4 + 1) 16 bytes >= Ncb rounded to 16
  for (uint32_t b = t; b < 256; b += P) crc8[b] = crc24_byte_entry(b, CRC24A_POLY);
  win_load_map(c, t, P, sb + g.sb_off, g.Ncb);
  __syncthreads();
  win_load(c, t, P, sb + g.sb_off, kdata + kt.pos_off, kdata + kt.pi_off, li % LANES, ld.F);
  __syncthreads();
  const uint32_t* tab = kdata + (ld.crc24a ? kt.crca_off : kt.crcb_off);
  uint32_t its = 0, ok = 0;
  for (uint32_t it = 0; it < max_its; it++) {
    win_half<false>(c, t);
    __syncthreads();
    win_half<true>(c, t);
    __syncthreads();
    ok = block_xor<P>(win_crc_part(c, t, P, tab), red) == 0;
    its = it + 1;
    if (early_stop && ok) break;
  }
  // pack into LDS (the d stream is free now), then the output row and the partial TB-CRC register
  uint8_t* pk = reinterpret_cast<uint8_t*>(c.d);
  win_pack(c, t, P, pk);
  __syncthreads();
  uint8_t* row = out.cb_bytes + (size_t)li * CB_BYTES_STRIDE;
  for (uint32_t j = t; j < K / 8; j += P) row[j] = pk[j];
  const uint32_t b0 = ld.F / 8, b1 = K / 8 - (ld.crc24a ? 0 : 3);
  const uint32_t tbp = block_xor<P>(win_tb_term(c, t, P, pk, b0, b1, crc8), red);
  if (t == 0) {
    out.its[li] = its;
    out.crc_ok[li] = ok;
    out.tb_part[li] = tbp;
  }
}

template <int P>
static void launch_win_p(const float* sb, const TdecWinOut& out, const MiGroupDesc* groups, const MiLaneDesc* lanes,
                         const MiKTab* ktabs, const uint32_t* kdata, uint32_t n_lanes, uint32_t max_k,
                         uint32_t max_its, uint32_t early_stop, hipStream_t st) {
  const uint32_t lds = win_lds_bytes(max_k, P);
  static bool attr = false;   // idempotent; the attribute is per function
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&tdec_win_kernel<P>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)win_lds_bytes(KMAX, P));
    attr = true;
  }
  hipLaunchKernelGGL(tdec_win_kernel<P>, dim3(n_lanes), dim3(P), lds, st, sb, out, groups, lanes, ktabs, kdata, max_its,
                     early_stop);
}

void launch_tdec_win(const float* sb, uint8_t* cb_bytes, uint32_t* cb_its, uint32_t* cb_crc, uint32_t* cb_tbp,
                     const MiGroupDesc* groups, const MiLaneDesc* lanes, const MiKTab* ktabs, const uint32_t* kdata,
                     uint32_t n_lanes, uint32_t max_k, uint32_t max_its, uint32_t early_stop, uint32_t threads,
                     hipStream_t st) {
  if (!n_lanes) return;
  const TdecWinOut out{cb_bytes, cb_its, cb_crc, cb_tbp};
  if (threads <= 64)
    launch_win_p<64>(sb, out, groups, lanes, ktabs, kdata, n_lanes, max_k, max_its, early_stop, st);
  else if (threads <= 128)
    launch_win_p<128>(sb, out, groups, lanes, ktabs, kdata, n_lanes, max_k, max_its, early_stop, st);
  else if (threads <= 256)
    launch_win_p<256>(sb, out, groups, lanes, ktabs, kdata, n_lanes, max_k, max_its, early_stop, st);
  else
    launch_win_p<512>(sb, out, groups, lanes, ktabs, kdata, n_lanes, max_k, max_its, early_stop, st);
}

}  // namespace mi
