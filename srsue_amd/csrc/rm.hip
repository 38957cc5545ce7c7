// rm.hip -- rate de-matching + HARQ combine into the group-interleaved softbuffer [Ncb][64 lanes].
//
// Semantics: rm_body.h (bit-identical to the serial srslte_rm_turbo_rx loop).  MI355X layout: one
// 256-thread workgroup owns RM_CHUNK circular-buffer positions of one 64-code-block group.  The
// positions of a chunk receive a contiguous run of each code block's LLRs (the non-null ranks of
// the chunk, modulo N_v), so the workgroup first stages, per lane, that run of e into an LDS tile
// with coalesced loads (consecutive threads on consecutive LLRs of one code block), then every
// wavefront combines one position for all 64 lanes: softbuffer rows are read and written as 256-B
// coalesced rows and the LLRs come from LDS (row stride RM_CHUNK + 1 floats: conflict-free column
// reads).  No integer division in the loops: ranks are rebased with one conditional add.
// Repetition beyond N_v (E > N_v, low code rates) adds the further copies from HBM in order.
//
// Sparse rows (dl_common.h sb_group_floats): a row is written only when some lane receives an LLR
// there or a combining lane keeps a materialised history; each wavefront owns 32 consecutive rows,
// whose map bytes it reads and rewrites with one 32-byte access (the bits live in a scalar register
// in between).  A chunk that receives nothing and holds nothing exits after its first barrier.
// Punctured positions of a first transmission (60 % of the circular buffer at MCS 28) thus cost no
// HBM traffic, here or in the decoder.
#include "demap_body.h"
#include "kernels.h"
#include "rm_body.h"

namespace mi {

// wavefronts per workgroup of the general (non-direct) chunks and the waves per SIMD their registers must allow (80
// VGPRs, 3 groups per CU); direct chunks run 8-wavefront workgroups at 8 waves per SIMD (4 per CU).  Same box, configs[4]
// mix on one stream (profiles/r3/ab_rm_split/ab_g8*): general chunks 977 us with 4-wavefront groups (122 VGPRs, 4 waves
// per SIMD), 918 us with 8 at 6 waves per SIMD, 1,121 us at 8 (45 VGPRs spilled)
constexpr int RM_GENERAL_NW = 8, RM_GENERAL_WPE = 6, RM_DIRECT_WPE = 8;

// workgroup shape: RM_NW wavefronts per chunk, each owning RM_CHUNK / RM_NW = 32 consecutive positions
// in the combine and 64 / RM_NW code-block rows (2 row-segments each) in the staging
constexpr int RM_NW = RM_CHUNK / 32;
static_assert(RM_CHUNK == 128 || RM_CHUNK == 256, "rm.hip: 128- or 256-position chunks");

// Fused demap -> rate de-matching (MI_DL_FLAG_KEEP_LLR off): instead of reading the LLR stream e, the
// staging computes each LLR from the grid and channel estimates (demap_body.h, the arithmetic of
// demap_kernel): the 90,000 LLRs of a 20 MHz subframe are never written to or read from HBM.
struct RmFuse {
  const float2* grid;
  const float2* ce;
  const MiLaneSrc* src;      // per lane of the launch (group.lane0 + lane), built by the planner
  const uint32_t* re_tab;
  const uint32_t* scr_tab;
  float noise;
  uint32_t compact;          // MI_DL_FLAG_CE_COMPACT: ce holds the 4 pilot rows [port][4][W] per subframe
};

// channel estimate of port plane cp at RE index ra (= l W + k): full estimates are read; compact ones are
// interpolated in time from the two pilot rows around symbol l with chest.hip's expression (identical floats)
__device__ __forceinline__ float2 ce_at(const RmFuse& f, const MiLaneSrc& src, const float2* cp, uint32_t ra) {
  if (!f.compact) return cp[ra];
  const uint32_t W = src.c1 / NSYMB, l = __umulhi(ra, src.wdiv), k = ra - l * W;
  const int ia = ce_ia((int)l);
  return ce_time_interp(cp[ia * W + k], cp[(ia + 1) * W + k], ce_tt((int)l));
}

// All LLRs of one demap unit (TM1: one RE, QM LLRs; TM2: one SFBC RE pair, 2 QM LLRs), descrambled, into
// the tile positions of [ga, gb): demap_kernel's arithmetic (demap_body.h).  Split in three so that the
// uniform-modulation kernel can software-pipeline units: the RE-table and scrambling-word loads, the
// grid / channel-estimate loads they address, and the arithmetic.
struct UnitIdx {
  uint32_t ra, rb;   // RE indices (rb: TM2 only)
  uint32_t s0, s1;   // the scrambling words holding the unit's first and last bit
};
struct UnitIn {
  float2 r0, r1, h00, h01, h10, h11;   // TM1: r0, h00
  uint32_t s0, s1;
};
template <int QM, bool TM2>
__device__ __forceinline__ UnitIdx fused_idx(const RmFuse& f, const MiLaneSrc& src, uint32_t u) {
  constexpr uint32_t U = QM * (TM2 ? 2 : 1);
  const uint32_t* re = f.re_tab + src.re;
  const uint32_t* scr = f.scr_tab + src.scr;
  UnitIdx x;
  x.ra = re[TM2 ? 2 * u : u];
  x.rb = TM2 ? re[2 * u + 1] : 0u;
  const uint32_t bit0 = u * U;
  x.s0 = scr[bit0 >> 5];
  x.s1 = scr[(bit0 + U - 1) >> 5];
  return x;
}
template <bool TM2>
__device__ __forceinline__ UnitIn fused_data(const RmFuse& f, const MiLaneSrc& src, const UnitIdx& x) {
  const float2* g = f.grid + src.goff;
  const float2* c0 = f.ce + src.coff;
  UnitIn d;
  d.r0 = g[x.ra];
  d.h00 = ce_at(f, src, c0, x.ra);
  if constexpr (TM2) {
    const float2* c1 = c0 + (f.compact ? 4 * (src.c1 / NSYMB) : src.c1);
    d.r1 = g[x.rb];
    d.h01 = ce_at(f, src, c0, x.rb);
    d.h10 = ce_at(f, src, c1, x.ra);
    d.h11 = ce_at(f, src, c1, x.rb);
  }
  d.s0 = x.s0;
  d.s1 = x.s1;
  return d;
}
// the U = Qm (TM1) or 2 Qm (TM2) descrambled LLRs of unit u, in LLR order
template <int QM, bool TM2>
__device__ __forceinline__ void fused_llrs(const RmFuse& f, const UnitIn& d, uint32_t u, float* out) {
  float2 x[2];
  if constexpr (!TM2) x[0] = eq_single(d.r0, d.h00, f.noise);
  else eq_sfbc(d.r0, d.r1, d.h00, d.h01, d.h10, d.h11, &x[0], &x[1]);
  constexpr int NS = TM2 ? 2 : 1, U = QM * NS;
  float l[U];
#pragma unroll
  for (int k = 0; k < NS; k++) {
    demap_dim<QM>(x[k].x, l + k * QM);
    demap_dim<QM>(x[k].y, l + k * QM + 1);
  }
  const uint32_t bit0 = u * U, w0 = bit0 >> 5;
#pragma unroll
  for (int b = 0; b < U; b++) {
    const uint32_t i = bit0 + b;
    const uint32_t word = (i >> 5) == w0 ? d.s0 : d.s1;
    out[b] = ((word >> (i & 31)) & 1u) ? -l[b] : l[b];
  }
}
// ... into the tile positions of [ga, gb)
template <int QM, bool TM2>
__device__ __forceinline__ void fused_compute(const RmFuse& f, const UnitIn& d, uint32_t u, uint32_t ga, uint32_t gb,
                                              uint32_t ta, float* tile) {
  constexpr int U = QM * (TM2 ? 2 : 1);
  float v[U];
  fused_llrs<QM, TM2>(f, d, u, v);
  const uint32_t bit0 = u * U;
#pragma unroll
  for (int b = 0; b < U; b++) {
    const uint32_t i = bit0 + b;
    if (i >= ga && i < gb) tile[ta + (i - ga)] = v[b];
  }
}
template <int QM, bool TM2>
__device__ __forceinline__ void fused_unit(const RmFuse& f, const MiLaneSrc& src, uint32_t u, uint32_t ga, uint32_t gb,
                                           uint32_t ta, float* tile) {
  fused_compute<QM, TM2>(f, fused_data<TM2>(f, src, fused_idx<QM, TM2>(f, src, u)), u, ga, gb, ta, tile);
}

__device__ __forceinline__ void fused_unit_any(const RmFuse& f, const MiLaneSrc& src, uint32_t u, uint32_t ga,
                                               uint32_t gb, uint32_t ta, float* tile) {
  switch (src.qm + 8 * src.tm2) {
    case 2: fused_unit<2, false>(f, src, u, ga, gb, ta, tile); break;
    case 4: fused_unit<4, false>(f, src, u, ga, gb, ta, tile); break;
    case 6: fused_unit<6, false>(f, src, u, ga, gb, ta, tile); break;
    case 10: fused_unit<2, true>(f, src, u, ga, gb, ta, tile); break;
    case 12: fused_unit<4, true>(f, src, u, ga, gb, ta, tile); break;
    default: fused_unit<6, true>(f, src, u, ga, gb, ta, tile); break;
  }
}

// LLR gi of a lane's subframe, alone (repetition beyond N_v, low code rates only): the single-bit
// form of the same arithmetic (demap_body.h demap_llr)
__device__ __forceinline__ float fused_llr(const RmFuse& f, const MiLaneSrc& src, uint32_t gi) {
  MiPdschDesc pd{};
  pd.tm = src.tm2 ? 2 : 1;
  const float2* g = f.grid + src.goff;
  const float2* c0 = f.ce + src.coff;
  const float2* c1 = c0 + src.c1;
  const uint32_t* re = f.re_tab + src.re;
  const uint32_t* scr = f.scr_tab + src.scr;
  switch (src.qm) {
    case 2: return demap_llr<2>(pd, gi, g, c0, c1, re, scr, f.noise);
    case 4: return demap_llr<4>(pd, gi, g, c0, c1, re, scr, f.noise);
    default: return demap_llr<6>(pd, gi, g, c0, c1, re, scr, f.noise);
  }
}

// FQ / FT: the batch's common modulation order and transmission mode (FQ = 0: mixed, per-unit switch).
// NW / DIR: wavefronts per workgroup; DIR = every item is a direct group's chunk (those run
// as 8-wavefront workgroups -- the same tile, each wavefront staging 8 rows and storing 16 ranks -- in a
// launch of their own, whose instantiation carries none of the general combine's registers)
template <bool FUSED, int FQ = 0, bool FT = false, int NW = RM_NW, bool DIR = false>
__global__ __launch_bounds__(64 * NW, DIR ? RM_DIRECT_WPE : (NW == 8 ? RM_GENERAL_WPE : 1)) void rm_combine_kernel(const float* __restrict__ e, float* __restrict__ sb,
                                                        const MiGroupDesc* __restrict__ groups,
                                                        const MiLaneDesc* __restrict__ lanes,
                                                        const uint32_t* __restrict__ kdata, RmFuse fz,
                                                        const uint32_t* __restrict__ items,
                                                        const uint4* __restrict__ recs,
                                                        const MiKTab* __restrict__ ktabs) {
  constexpr int NSEG = 2 * LANES / NW;   // (row, segment) LLR runs per wavefront in the staging
  __shared__ float tile[LANES][RM_CHUNK + 1];
  __shared__ uint32_t s_j0[LANES], s_nr[LANES], s_nv[LANES], s_E[LANES];
  __shared__ uint64_t s_eoff[LANES];
  __shared__ uint32_t s_comb, s_new;
  __shared__ uint32_t s_dra, s_dnr;   // direct groups: the chunk's first rank and rank count (every lane's)
  // fused staging: per-lane sources, and per wavefront NSEG (row, segment) LLR runs -> demap units
  __shared__ MiLaneSrc s_src[FUSED ? LANES : 1];
  __shared__ uint32_t rs_ga[FUSED ? NW : 1][NSEG], rs_gb[FUSED ? NW : 1][NSEG],
      rs_ta[FUSED ? NW : 1][NSEG], rs_u0[FUSED ? NW : 1][NSEG], rs_pre[FUSED ? NW : 1][NSEG + 1];
  // the work item: (group, chunk) from the planner's work list, or the 2-D grid.  With the list, each workgroup
  // reads one 16-B record {lane0, Ncb | chunk << 16, softbuffer offset / 64, ipos offset} (Plan::rm_recs): the
  // group descriptor is folded in, one dependent global load less at the head of every chunk's chain
  uint32_t lane0, Ncb, ci, ipos_off;
  uint64_t sb_off;
  bool direct = DIR;   // a Plan::rm_direct group: r.w is its rank -> row table
  if (recs) {
    const uint4 r = recs[blockIdx.x];
    lane0 = r.x;
    Ncb = r.y & 0x7FFFu;
    direct = DIR || ((r.y >> 15) & 1u);
    ci = r.y >> 16;
    sb_off = (uint64_t)r.z * LANES;
    ipos_off = r.w;
  } else {
    uint32_t gi = blockIdx.y;
    ci = blockIdx.x;
    if (items) {
      const uint32_t it = items[blockIdx.x];
      gi = it >> 9;
      ci = it & 511u;
    }
    const MiGroupDesc g = groups[gi];
    lane0 = g.lane0;
    Ncb = g.Ncb;
    sb_off = g.sb_off;
    ipos_off = ktabs[g.ktab].ipos_off;
  }
  const uint32_t pa = ci * RM_CHUNK;
  if (pa >= Ncb) return;
  const uint32_t tid = threadIdx.x;
  float* sbg = sb + sb_off;
  uint8_t* map = reinterpret_cast<uint8_t*>(sbg + sb_map_off(Ncb)) + pa;   // map rounded up to 256 B
  int busy = 0;
  if (tid < LANES) {
    const MiLaneDesc ld = lanes[lane0 + tid];
    uint32_t j0 = 0, nr = 0, ra = 0;
    if (ld.valid) {
      const uint32_t* ch = kdata + ld.rank_off + Ncb;
      ra = ch[pa / RM_CHUNK];
      nr = ch[pa / RM_CHUNK + 1] - ra;
      j0 = ra >= ld.r0 ? ra - ld.r0 : ra + ld.Nv - ld.r0;   // LLR index of the chunk's first rank
    }
    s_j0[tid] = j0; s_nr[tid] = nr; s_nv[tid] = ld.Nv; s_E[tid] = ld.E;
    if constexpr (FUSED) {
      const MiLaneSrc src = fz.src[lane0 + tid];
      s_src[tid] = src;
      s_eoff[tid] = src.eb;   // LLR index of the code block's first LLR within its subframe
    } else {
      s_eoff[tid] = ld.e_off;
    }
    // does any LLR of this lane land in the chunk (LLR indices j0 .. j0+nr-1 mod Nv against [0, E))?
    busy = nr > 0 && (ld.E >= ld.Nv || j0 < ld.E || j0 + nr > ld.Nv);
    const uint64_t comb = __ballot(ld.valid && !ld.new_tb), fresh = __ballot(ld.valid && ld.new_tb);
    if (tid == 0) { s_comb = comb != 0; s_new = fresh != 0; }
    if (direct && fresh && tid == (uint32_t)(__ffsll((unsigned long long)fresh) - 1)) {
      s_dra = ra;
      s_dnr = nr;
    }
    if (ci == 0) sbg[(size_t)Ncb * LANES + tid] = 0.0f;   // the group's zero row
  }
  if (tid < RM_CHUNK / 4 && !direct) busy |= reinterpret_cast<const uint32_t*>(map)[tid] != 0;
  // nothing received and nothing materialised: the chunk stays all-zero, no HBM traffic
  if (!__syncthreads_or(busy)) return;
  // stage: tile[l][t] = e_l[(j0 + t) mod Nv] (0 beyond E), t < nr; a wavefront per code-block row,
  // all of a wavefront's loads issued before its LDS writes
  constexpr int ROWS = LANES / NW, PER = RM_CHUNK / 64;
  if constexpr (FUSED) {
    // Every LLR computed from grid + ce, one demap unit (an RE, or an SFBC RE pair: all its Qm or 2 Qm
    // LLRs, as demap_kernel computes them) per thread and step.  Wavefront w owns code-block rows
    // l = w + NW r; each row's LLR run (j0 + t) mod Nv, t < nr, clipped to [0, E), is at most two
    // contiguous runs (row-segments); the units of the wavefront's NSEG row-segments are dealt to its 64
    // threads flat, so all threads work and their loads are independent.
    const uint32_t w = tid >> 6, q = tid & 63;
#pragma unroll
    for (int r = 0; r < ROWS; r++)
      for (uint32_t t = q; t < RM_CHUNK; t += 64) tile[w + NW * r][t] = 0.0f;
    uint32_t nu = 0;
    if (q < NSEG) {
      const uint32_t l = w + NW * (q >> 1), seg = q & 1;
      const uint32_t j0 = s_j0[l], nr = s_nr[l], nv = s_nv[l], E = s_E[l];
      const uint32_t ta = seg ? nv - j0 : 0, tb = seg ? nr : (nr < nv - j0 ? nr : nv - j0);
      uint32_t ga = 0, gb = 0, u0 = 0;
      if (ta < tb) {
        const uint32_t ja = seg ? 0 : j0, jf = ja + (tb - ta), jb = jf < E ? jf : E;
        if (ja < jb) {
          const uint32_t U = s_src[l].qm * (s_src[l].tm2 ? 2 : 1), eb = (uint32_t)s_eoff[l];
          ga = eb + ja;
          gb = eb + jb;
          u0 = ga / U;
          nu = (gb - 1) / U - u0 + 1;
        }
      }
      rs_ga[w][q] = ga; rs_gb[w][q] = gb; rs_ta[w][q] = ta; rs_u0[w][q] = u0;
    }
    // units before each row-segment: inclusive wavefront scan of nu (lanes >= NSEG contribute 0)
    uint32_t incl = nu;
#pragma unroll
    for (int d = 1; d < NSEG; d <<= 1) {
      const uint32_t t = __shfl_up(incl, d, 64);
      if (q >= (uint32_t)d) incl += t;
    }
    if (q < NSEG) rs_pre[w][q + 1] = incl;
    if (q == 0) rs_pre[w][0] = 0;
    const uint32_t total = __shfl(incl, NSEG - 1, 64);
    __syncthreads();
    auto locate = [&](uint32_t fi) {   // row-segment rs with rs_pre[rs] <= fi < rs_pre[rs + 1]
      uint32_t lo = 0, hi = NSEG;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (rs_pre[w][mid] <= fi) lo = mid; else hi = mid;
      }
      return lo;
    };
    if constexpr (FQ != 0 && DIR) {
      // direct 8-wavefront form: ~3 units per thread, one unit after the other; occupancy hides latency (the
      // three-stage pipeline below measured 2.44-2.49 ms against 2.34-2.40 here, same box)
      for (uint32_t fi = q; fi < total; fi += 64) {
        const uint32_t lo = locate(fi), l = w + NW * (lo >> 1);
        fused_unit<FQ, FT>(fz, s_src[l], rs_u0[w][lo] + (fi - rs_pre[w][lo]), rs_ga[w][lo], rs_gb[w][lo], rs_ta[w][lo],
                           tile[l]);
      }
    } else if constexpr (FQ != 0) {
      // uniform modulation: three-stage software pipeline over the thread's units (fi, fi + 64, ...):
      // the RE-table / scrambling loads run two units ahead, the grid / channel-estimate loads one
      // unit ahead, so each unit's two dependent HBM round trips overlap earlier units' arithmetic
      uint32_t fi = q;
      if (fi < total) {
        uint32_t loA = locate(fi), uA = rs_u0[w][loA] + (fi - rs_pre[w][loA]);
        UnitIn dA = fused_data<FT>(fz, s_src[w + NW * (loA >> 1)], fused_idx<FQ, FT>(fz, s_src[w + NW * (loA >> 1)], uA));
        uint32_t loB = 0, uB = 0;
        UnitIdx iB{};
        if (fi + 64 < total) {
          loB = locate(fi + 64);
          uB = rs_u0[w][loB] + (fi + 64 - rs_pre[w][loB]);
          iB = fused_idx<FQ, FT>(fz, s_src[w + NW * (loB >> 1)], uB);
        }
        for (;; fi += 64) {
          const bool hasB = fi + 64 < total, hasC = fi + 128 < total;
          UnitIn dB{};
          if (hasB) dB = fused_data<FT>(fz, s_src[w + NW * (loB >> 1)], iB);
          uint32_t loC = 0, uC = 0;
          UnitIdx iC{};
          if (hasC) {
            loC = locate(fi + 128);
            uC = rs_u0[w][loC] + (fi + 128 - rs_pre[w][loC]);
            iC = fused_idx<FQ, FT>(fz, s_src[w + NW * (loC >> 1)], uC);
          }
          fused_compute<FQ, FT>(fz, dA, uA, rs_ga[w][loA], rs_gb[w][loA], rs_ta[w][loA], tile[w + NW * (loA >> 1)]);
          if (!hasB) break;
          loA = loB; uA = uB; dA = dB;
          loB = loC; uB = uC; iB = iC;
        }
      }
    } else {
      for (uint32_t fi = q; fi < total; fi += 64) {
        const uint32_t lo = locate(fi), l = w + NW * (lo >> 1);
        fused_unit_any(fz, s_src[l], rs_u0[w][lo] + (fi - rs_pre[w][lo]), rs_ga[w][lo], rs_gb[w][lo], rs_ta[w][lo],
                       tile[l]);
      }
    }
  } else {
  {
    float v[ROWS][PER];
    const uint32_t w = tid >> 6, q = tid & 63;
#pragma unroll
    for (int r = 0; r < ROWS; r++) {
      const uint32_t l = w + NW * r;
      const uint32_t nr = s_nr[l], nv = s_nv[l], E = s_E[l];
      const float* el = e + s_eoff[l];
#pragma unroll
      for (int c = 0; c < PER; c++) {
        const uint32_t t = q + 64 * c;
        uint32_t j = s_j0[l] + t;
        if (j >= nv) j -= nv;
        v[r][c] = (t < nr && j < E) ? el[j] : 0.0f;
      }
    }
#pragma unroll
    for (int r = 0; r < ROWS; r++)
#pragma unroll
      for (int c = 0; c < PER; c++) tile[w + NW * r][q + 64 * c] = v[r][c];
  }
  }
  __syncthreads();
  // combine: wavefront w owns the NP consecutive positions pw .. pw+NP-1, one row (64 lanes) each
  constexpr int NP = RM_CHUNK / NW;
  const int lane = (int)(tid & 63), wave = (int)(tid >> 6);
  if (direct) {
    // rank-driven stores: wavefront w owns tile columns (ranks s_dra + t) t = NP w .. NP w + NP - 1
    const uint32_t t0 = NP * (uint32_t)wave, nr = s_dnr;
    const uint32_t nt = nr > t0 ? min(nr - t0, (uint32_t)NP) : 0u;
    const uint32_t rowv = (uint32_t)lane < nt ? kdata[ipos_off + s_dra + t0 + lane] : 0u;
    const bool lvalid = s_E[lane] != 0u;   // valid lanes receive E > 0 LLRs
#pragma unroll
    for (int i = 0; i < NP; i++) {
      const uint32_t row = (uint32_t)__builtin_amdgcn_readlane((int)rowv, i);
      if ((uint32_t)i < nt && lvalid) sbg[(size_t)row * LANES + lane] = 0.0f + tile[lane][t0 + i];
    }
    return;
  }
  const uint32_t pw = pa + NP * (uint32_t)wave, np = Ncb > pw ? min(Ncb - pw, (uint32_t)NP) : 0u;
  const MiLaneDesc ld = lanes[lane0 + lane];
  const int32_t* rank = reinterpret_cast<const int32_t*>(kdata + ld.rank_off);
  const uint32_t* ch = kdata + ld.rank_off + Ncb;
  const uint32_t ra = ld.valid ? ch[pa / RM_CHUNK] : 0;
  const uint32_t j0 = s_j0[lane], nv = ld.Nv, E = ld.E;
  const bool rep = E > nv, comb = s_comb, fresh = s_new;
  // materialised-before bits of the wave's rows (wave-uniform)
  const uint32_t was_m = (uint32_t)__ballot(lane < NP && (uint32_t)lane < np && map[NP * wave + lane] != 0);
  // the softbuffer rows of the wave's positions (decoder-input order, dl_common.h): lane i < NP holds ipos[pw + i], read
  // back wave-uniform per position (dummy positions are never written)
  const uint32_t rowv = (uint32_t)lane < np ? kdata[ipos_off + pw + lane] : pw + (uint32_t)lane;
  auto row_of = [&](int i) -> size_t {
    return (size_t)(uint32_t)__builtin_amdgcn_readlane((int)rowv, i);
  };
  int32_t rk[NP];
  float old[NP];
#pragma unroll
  for (int i = 0; i < NP; i++) {
    const uint32_t p = pw + i;
    rk[i] = (ld.valid && (uint32_t)i < np) ? rank[p] : -2;
    old[i] = (((was_m >> i) & 1u) && ld.valid && !ld.new_tb) ? sbg[row_of(i) * LANES + lane] : 0.0f;
  }
  uint32_t mat_m = 0;
#pragma unroll
  for (int i = 0; i < NP; i++) {
    if ((uint32_t)i >= np) continue;   // uniform: only the group's last wavefront has np < NP
    float v = old[i];
    bool c = false;
    if (rk[i] >= 0) {
      const uint32_t t = (uint32_t)rk[i] - ra;
      uint32_t j = j0 + t;
      if (j >= nv) j -= nv;
      if (j < E) { v = v + tile[lane][t]; c = true; }
      if (rep) {
        if constexpr (FUSED) {
          for (j += nv; j < E; j += nv) v = v + fused_llr(fz, s_src[lane], (uint32_t)s_eoff[lane] + j);
        } else {
          for (j += nv; j < E; j += nv) v = v + e[ld.e_off + j];
        }
      }
    }
    const bool any = __ballot(c) != 0, was = (was_m >> i) & 1u;
    const bool mat = any || (was && comb);   // row holds data after this launch
    if (mat && (any || !was || fresh) && ld.valid) sbg[row_of(i) * LANES + lane] = v;
    mat_m |= (uint32_t)mat << i;
  }
  if ((uint32_t)lane < np) map[NP * wave + lane] = (uint8_t)((mat_m >> lane) & 1u);
}

// Chunks where no lane receives an LLR (the planner's idle list; 60 % of a first transmission's
// circular buffer at MCS 28): one thread per chunk reads its 128 map bytes and normally finds them all
// zero.  Rows still materialised from an earlier run are settled exactly as rm_combine_kernel would
// settle them (nothing is received, so v = old): in a group with combining lanes the row stays
// materialised and its fresh lanes are zeroed, otherwise the row is dropped from the map.
__global__ __launch_bounds__(256) void rm_idle_kernel(float* __restrict__ sb, const MiGroupDesc* __restrict__ groups,
                                                     const MiLaneDesc* __restrict__ lanes,
                                                     const uint32_t* __restrict__ items, uint32_t n,
                                                     const MiKTab* __restrict__ ktabs, const uint32_t* __restrict__ kdata) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t it = items[i];
  const MiGroupDesc g = groups[it >> 9];
  const uint32_t pa = (it & 511u) * RM_CHUNK;
  if (pa >= g.Ncb) return;
  float* sbg = sb + g.sb_off;
  uint8_t* map = reinterpret_cast<uint8_t*>(sbg + sb_map_off(g.Ncb)) + pa;
  const uint4* m4 = reinterpret_cast<const uint4*>(map);
  uint32_t any = 0;
#pragma unroll
  for (int k = 0; k < RM_CHUNK / 16; k++) {
    const uint4 v = m4[k];
    any |= v.x | v.y | v.z | v.w;
  }
  if (!any) return;
  uint64_t fresh = 0;
  bool comb = false;
  for (int l = 0; l < LANES; l++) {
    const MiLaneDesc ld = lanes[g.lane0 + l];
    if (!ld.valid) continue;
    if (ld.new_tb) fresh |= 1ull << l; else comb = true;
  }
  const uint32_t np = min((uint32_t)RM_CHUNK, g.Ncb - pa);
  for (uint32_t p = 0; p < np; p++) {
    if (!map[p]) continue;
    if (!comb) { map[p] = 0; continue; }
    const size_t row = kdata[ktabs[g.ktab].ipos_off + pa + p];   // rows in decoder-input order (dl_common.h)
    for (int l = 0; l < LANES; l++)
      if ((fresh >> l) & 1u) sbg[row * LANES + l] = 0.0f;
  }
}

// ---- direct groups (Plan::rm_direct) ---------------------------------------------------------------
// Groups whose valid lanes all start a new TB with one rank table, one k0 rank and E <= N_v: every received
// circular-buffer position gets exactly one LLR, LLR j of every lane at rank (r0 + j) mod N_v.  Their busy
// chunks run rm_combine_kernel's staging unchanged, then a rank-driven store phase: tile column t is rank
// ra + t for every lane, so a wavefront reads the rows of its 32 ranks with one coalesced load of the
// (K, F) rank -> row table and stores each as a 256-B row (0.0f + LLR; 0.0f past a lane's E, where the tile
// holds 0) -- no rank / map loads, no ballots.  Their row maps and zero rows come from rm_direct_map_kernel
// (materialised iff some lane receives the position), so their idle chunks need no rm_idle_kernel and no
// stale row of an earlier plan survives.  (A lane-per-code-block form without the LDS transpose, one demap
// unit per lane and wavefront, measured 6.6 ms against 3.85: 64 code blocks' scattered grid / estimate loads
// per instruction, profiles/r3/ab_rm_direct.)
// the direct groups' row maps and zero rows: RM_DIRECT_MAPB workgroups per group stride over its positions
constexpr uint32_t RM_DIRECT_MAPB = 8;
__global__ __launch_bounds__(256) void rm_direct_map_kernel(float* __restrict__ sb, const uint32_t* __restrict__ kdata,
                                                           const MiRmDirect* __restrict__ dgs) {
  const MiRmDirect d = dgs[blockIdx.x / RM_DIRECT_MAPB];
  const uint32_t part = blockIdx.x % RM_DIRECT_MAPB;
  float* sbg = sb + (size_t)d.sb64 * LANES;
  if (part == 0 && threadIdx.x < LANES) sbg[(size_t)d.Ncb * LANES + threadIdx.x] = 0.0f;   // the zero row
  uint8_t* map = reinterpret_cast<uint8_t*>(sbg + sb_map_off(d.Ncb));
  const int32_t* rank = reinterpret_cast<const int32_t*>(kdata + d.rank_off);
  const uint32_t emax = d.emax_kind & 0xFFFFFFu;
  for (uint32_t p = part * 256 + threadIdx.x; p < d.Ncb; p += RM_DIRECT_MAPB * 256) {
    const int32_t rk = rank[p];
    uint32_t j = (uint32_t)rk + d.Nv - d.r0;   // the LLR index the position receives
    if (j >= d.Nv) j -= d.Nv;
    map[p] = (rk >= 0 && j < emax) ? 1 : 0;
  }
}

void launch_rm_direct_maps(float* sb, const uint32_t* ktab_data, const MiRmDirect* dgs, uint32_t ndg, hipStream_t st) {
  if (ndg)
    hipLaunchKernelGGL(rm_direct_map_kernel, dim3(ndg * RM_DIRECT_MAPB), dim3(256), 0, st, sb, ktab_data, dgs);
}

// the chunk work list (busy items with the combine kernel, idle items with rm_idle_kernel), or without
// one (n_items = 0) every chunk of every group through the combine kernel
static dim3 rm_grid(const uint32_t* items, uint32_t n_busy, uint32_t n_groups, uint32_t max_ncb) {
  return items ? dim3(n_busy) : dim3((max_ncb + RM_CHUNK - 1) / RM_CHUNK, n_groups);
}
static void rm_idle(float* sb, const MiGroupDesc* groups, const MiLaneDesc* lanes, const uint32_t* items,
                    uint32_t n_busy, uint32_t n_items, const MiKTab* ktabs, const uint32_t* kdata, hipStream_t st) {
  if (items && n_items > n_busy)
    hipLaunchKernelGGL(rm_idle_kernel, dim3((n_items - n_busy + 255) / 256), dim3(256), 0, st, sb, groups, lanes,
                       items + n_busy, n_items - n_busy, ktabs, kdata);
}

// the direct groups' chunks lead the busy items (Plan::rm_dbusy): they run in their own 8-wavefront launch, the
// general chunks after them
void launch_rm_combine(const float* e, float* sb, const MiGroupDesc* groups, const MiLaneDesc* lanes,
                       const MiKTab* ktabs, const uint32_t* ktab_data, uint32_t n_groups, uint32_t max_ncb,
                       const uint32_t* items, const uint4* recs, uint32_t n_busy, uint32_t n_dbusy, uint32_t n_items,
                       hipStream_t st) {
  if (!n_groups) return;
  if (items && !n_busy) items = nullptr;
  rm_idle(sb, groups, lanes, items, n_busy, n_items, ktabs, ktab_data, st);
  uint32_t skip = 0;
  if (items && n_dbusy) {
    hipLaunchKernelGGL((rm_combine_kernel<false, 0, false, 8, true>), dim3(n_dbusy), dim3(512), 0, st, e, sb, groups,
                       lanes, ktab_data, RmFuse{}, items, recs, ktabs);
    skip = n_dbusy;
    if (skip == n_busy) return;
  }
  hipLaunchKernelGGL((rm_combine_kernel<false, 0, false, RM_GENERAL_NW>), rm_grid(items, n_busy - skip, n_groups, max_ncb),
                     dim3(64 * RM_GENERAL_NW), 0, st, e,
                     sb, groups, lanes, ktab_data, RmFuse{}, items ? items + skip : nullptr,
                     items ? recs + skip : nullptr, ktabs);
}

void launch_rm_fused(const float2* grid, const float2* ce, const MiLaneSrc* lane_src, const uint32_t* re_tab,
                     const uint32_t* scr_tab, float noise, float* sb, const MiGroupDesc* groups, const MiLaneDesc* lanes,
                     const MiKTab* ktabs, const uint32_t* ktab_data, uint32_t n_groups, uint32_t max_ncb, uint32_t unit_kind,
                     const uint32_t* items, const uint4* recs, uint32_t n_busy, uint32_t n_dbusy, uint32_t n_items,
                     bool compact_ce, hipStream_t st) {
  if (!n_groups) return;
  if (items && !n_busy) items = nullptr;
  rm_idle(sb, groups, lanes, items, n_busy, n_items, ktabs, ktab_data, st);
  const RmFuse fz{grid, ce, lane_src, re_tab, scr_tab, noise, (uint32_t)compact_ce};
  uint32_t skip = 0;
  if (items && n_dbusy) {
#define MI_RM_LAUNCH(...) \
  hipLaunchKernelGGL((__VA_ARGS__), dim3(n_dbusy), dim3(512), 0, st, nullptr, sb, groups, lanes, ktab_data, fz, items, \
                     recs, ktabs)
    switch (unit_kind) {   // Qm + 8 * (TM2)
      case 2: MI_RM_LAUNCH(rm_combine_kernel<true, 2, false, 8, true>); break;
      case 4: MI_RM_LAUNCH(rm_combine_kernel<true, 4, false, 8, true>); break;
      case 6: MI_RM_LAUNCH(rm_combine_kernel<true, 6, false, 8, true>); break;
      case 10: MI_RM_LAUNCH(rm_combine_kernel<true, 2, true, 8, true>); break;
      case 12: MI_RM_LAUNCH(rm_combine_kernel<true, 4, true, 8, true>); break;
      case 14: MI_RM_LAUNCH(rm_combine_kernel<true, 6, true, 8, true>); break;
      default: MI_RM_LAUNCH(rm_combine_kernel<true, 0, false, 8, true>); break;
    }
#undef MI_RM_LAUNCH
    skip = n_dbusy;
    if (skip == n_busy) return;
  }
  const dim3 g = rm_grid(items, n_busy - skip, n_groups, max_ncb);
  const uint32_t* it = items ? items + skip : nullptr;
  const uint4* rc = items ? recs + skip : nullptr;
#define MI_RM_LAUNCH(...) \
  hipLaunchKernelGGL((__VA_ARGS__), g, dim3(64 * RM_GENERAL_NW), 0, st, nullptr, sb, groups, lanes, ktab_data, fz, \
                     it, rc, ktabs)
  constexpr int GNW = RM_GENERAL_NW;
  switch (unit_kind) {   // Qm + 8 * (TM2)
    case 2: MI_RM_LAUNCH(rm_combine_kernel<true, 2, false, GNW>); break;
    case 4: MI_RM_LAUNCH(rm_combine_kernel<true, 4, false, GNW>); break;
    case 6: MI_RM_LAUNCH(rm_combine_kernel<true, 6, false, GNW>); break;
    case 10: MI_RM_LAUNCH(rm_combine_kernel<true, 2, true, GNW>); break;
    case 12: MI_RM_LAUNCH(rm_combine_kernel<true, 4, true, GNW>); break;
    case 14: MI_RM_LAUNCH(rm_combine_kernel<true, 6, true, GNW>); break;
    default: MI_RM_LAUNCH(rm_combine_kernel<true, 0, false, GNW>); break;
  }
#undef MI_RM_LAUNCH
}

}  // namespace mi
