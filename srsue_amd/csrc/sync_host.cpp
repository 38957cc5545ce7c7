// sync_host.cpp -- host side of the sync front end (sync.h): PSS/SSS sequences (36.211 6.11), the
// time-domain PSS templates of a bandwidth, the SyncEngine that batches the GPU searches, and the
// mi_sync_* C ABI (include/mi_dl.h).
#include <math.h>
#include <string.h>

#include "kernels.h"
#include "sync.h"

namespace mi {

void pss_seq(uint32_t nid2, float2* d) {
  const double u = nid2 % 3 == 0 ? 25 : nid2 % 3 == 1 ? 29 : 34;
  for (int n = 0; n < 62; n++) {
    const double ph = n < 31 ? -M_PI * u * n * (n + 1) / 63.0 : -M_PI * u * (n + 1) * (n + 2) / 63.0;
    d[n] = make_float2((float)cos(ph), (float)sin(ph));
  }
}

void sss_seq(uint32_t nid1, uint32_t nid2, uint32_t sf5, float* d) {
  auto mseq = [](uint32_t taps, int* s) {   // x(i+5) = x(i) + sum of tapped x(i+t), t in 1..4
    int x[31] = {0, 0, 0, 0, 1};
    for (int i = 0; i < 26; i++) {
      int v = x[i];
      for (int t = 1; t <= 4; t++) if ((taps >> t) & 1u) v ^= x[i + t];
      x[i + 5] = v;
    }
    for (int i = 0; i < 31; i++) s[i] = 1 - 2 * x[i];
  };
  int st[31], ct[31], zt[31];
  mseq(1u << 2, st);
  mseq(1u << 3, ct);
  mseq((1u << 1) | (1u << 2) | (1u << 4), zt);
  const uint32_t qp = nid1 / 30, q = (nid1 + qp * (qp + 1) / 2) / 30, mp = nid1 + q * (q + 1) / 2;
  const uint32_t m0 = mp % 31, m1 = (m0 + mp / 31 + 1) % 31;
  for (uint32_t n = 0; n < 31; n++) {
    const int s0 = st[(n + m0) % 31], s1 = st[(n + m1) % 31], c0 = ct[(n + nid2) % 31], c1 = ct[(n + nid2 + 3) % 31];
    const int z0 = zt[(n + m0 % 8) % 31], z1 = zt[(n + m1 % 8) % 31];
    d[2 * n] = (float)(sf5 ? s1 * c0 : s0 * c0);
    d[2 * n + 1] = (float)(sf5 ? s0 * c1 * z1 : s1 * c1 * z0);
  }
}

uint32_t sync_bin(uint32_t m, uint32_t nof_prb, uint32_t N) {
  const uint32_t W = 12 * nof_prb, k = m - 31 + W / 2;
  return k < W / 2 ? N - W / 2 + k : k - W / 2 + 1;
}

int SyncEngine::init(uint32_t prb) {
  const int n = symbol_sz(prb);
  if (n < 0) { set_error("sync: nof_prb"); return -1; }
  nof_prb = prb;
  N = (uint32_t)n;
  std::vector<float2> t(3 * (size_t)N);
  for (uint32_t u = 0; u < 3; u++) {   // p[n] = (1/sqrt N) sum_m d(m) exp(+j 2 pi b(m) n / N)
    float2 d[62];
    pss_seq(u, d);
    for (uint32_t i = 0; i < N; i++) {
      double re = 0, im = 0;
      for (uint32_t m = 0; m < 62; m++) {
        const double ph = 2.0 * M_PI * (double)((uint64_t)sync_bin(m, prb, N) * i % N) / N;
        re += d[m].x * cos(ph) - d[m].y * sin(ph);
        im += d[m].x * sin(ph) + d[m].y * cos(ph);
      }
      t[u * N + i] = make_float2((float)(re / sqrt((double)N)), (float)(im / sqrt((double)N)));
    }
  }
  return (d_tmpl.ensure(t.size() * sizeof(float2)) &&
          hip_ok(hipMemcpy(d_tmpl.p, t.data(), t.size() * sizeof(float2), hipMemcpyHostToDevice), "H2D"))
             ? 0
             : -1;
}

template <class T>
static bool up_sync(DevBuf& b, const std::vector<T>& v, hipStream_t st) {
  return b.ensure(std::max<size_t>(v.size(), 1) * sizeof(T)) &&
         (v.empty() || hip_ok(hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st), "H2D"));
}

int SyncEngine::pss(const float2* iq, const std::vector<MiPssJob>& jobs, hipStream_t st) {
  pres.resize(jobs.size());
  if (jobs.empty()) return 0;
  if (!up_sync(d_pjobs, jobs, st) || !d_pres.ensure(jobs.size() * sizeof(MiPssRes))) return -1;
  uint32_t max_nlag = 0;
  for (const MiPssJob& j : jobs) max_nlag = std::max(max_nlag, j.nlag);
  launch_pss_search(iq, d_tmpl.as<float2>(), d_pjobs.as<MiPssJob>(), d_pres.as<MiPssRes>(), (uint32_t)jobs.size(), N,
                    max_nlag, st);
  return (hip_ok(hipGetLastError(), "pss launch") &&
          hip_ok(hipMemcpyAsync(pres.data(), d_pres.p, pres.size() * sizeof(MiPssRes), hipMemcpyDeviceToHost, st), "D2H") &&
          hip_ok(hipStreamSynchronize(st), "sync"))
             ? 0
             : -1;
}

int SyncEngine::sss(const float2* iq, const std::vector<MiSssJob>& jobs, hipStream_t st) {
  sres.resize(jobs.size());
  if (jobs.empty()) return 0;
  if (!up_sync(d_sjobs, jobs, st) || !d_sres.ensure(jobs.size() * sizeof(MiSssRes))) return -1;
  launch_sss_detect(iq, d_sjobs.as<MiSssJob>(), d_sres.as<MiSssRes>(), (uint32_t)jobs.size(), N, nof_prb,
                    (uint32_t)symbol_offset((int)N, 5), (uint32_t)symbol_offset((int)N, 6), st);
  return (hip_ok(hipGetLastError(), "sss launch") &&
          hip_ok(hipMemcpyAsync(sres.data(), d_sres.p, sres.size() * sizeof(MiSssRes), hipMemcpyDeviceToHost, st), "D2H") &&
          hip_ok(hipStreamSynchronize(st), "sync"))
             ? 0
             : -1;
}

int SyncEngine::correct(const float2* src, float2* dst, const std::vector<MiCfoJob>& jobs, uint32_t len, hipStream_t st) {
  if (jobs.empty()) return 0;
  if (!up_sync(d_cjobs, jobs, st)) return -1;
  launch_cfo_correct(src, dst, d_cjobs.as<MiCfoJob>(), (uint32_t)jobs.size(), len, N, st);
  return hip_ok(hipGetLastError(), "cfo launch") ? 0 : -1;
}

}  // namespace mi

// ---- C ABI (include/mi_dl.h) -----------------------------------------------------------------
struct mi_sync {
  mi::SyncEngine e;
};

extern "C" {

mi_sync_t* mi_sync_create(uint32_t nof_prb) {
  auto* s = new mi_sync();
  if (s->e.init(nof_prb)) { delete s; return nullptr; }
  return s;
}
void mi_sync_destroy(mi_sync_t* s) { delete s; }
uint32_t mi_sync_fft_size(const mi_sync_t* s) { return s ? s->e.N : 0; }

int mi_sync_pss(mi_sync_t* s, const void* d_iq, const uint64_t* off, uint32_t n, uint32_t nlag, uint32_t nid2_mask,
                mi_pss_result_t* out, void* stream) {
  if (!s || !d_iq || (n && (!off || !out)) || nlag == 0 || (nid2_mask & 7u) == 0) {
    mi::set_error("mi_sync_pss: arguments");
    return -1;
  }
  std::vector<mi::MiPssJob> jobs(n);
  for (uint32_t i = 0; i < n; i++) jobs[i] = mi::MiPssJob{off[i], nlag, nid2_mask & 7u};
  if (s->e.pss(reinterpret_cast<const float2*>(d_iq), jobs, reinterpret_cast<hipStream_t>(stream))) return -1;
  for (uint32_t i = 0; i < n; i++) {
    out[i].nid2 = s->e.pres[i].nid2;
    out[i].lag = s->e.pres[i].lag;
    out[i].rho = s->e.pres[i].rho;
    out[i].cfo = s->e.pres[i].cfo;
  }
  return 0;
}

int mi_sync_sss(mi_sync_t* s, const void* d_iq, const uint64_t* sf_off, const uint32_t* nid2, const float* cfo,
                uint32_t n, mi_sss_result_t* out, void* stream) {
  if (!s || !d_iq || (n && (!sf_off || !nid2 || !cfo || !out))) { mi::set_error("mi_sync_sss: arguments"); return -1; }
  std::vector<mi::MiSssJob> jobs(n);
  for (uint32_t i = 0; i < n; i++) jobs[i] = mi::MiSssJob{sf_off[i], nid2[i] % 3, cfo[i]};
  if (s->e.sss(reinterpret_cast<const float2*>(d_iq), jobs, reinterpret_cast<hipStream_t>(stream))) return -1;
  for (uint32_t i = 0; i < n; i++) {
    out[i].nid1 = s->e.sres[i].nid1;
    out[i].sf5 = s->e.sres[i].sf5;
    out[i].score = s->e.sres[i].score;
  }
  return 0;
}

int mi_sync_correct(mi_sync_t* s, const void* d_src, const uint64_t* src_off, void* d_dst, const uint64_t* dst_off,
                    const float* cfo, uint32_t n, uint32_t len, void* stream) {
  if (!s || !d_src || !d_dst || (n && (!src_off || !dst_off || !cfo))) {
    mi::set_error("mi_sync_correct: arguments");
    return -1;
  }
  std::vector<mi::MiCfoJob> jobs(n);
  for (uint32_t i = 0; i < n; i++) jobs[i] = mi::MiCfoJob{src_off[i], dst_off[i], cfo[i], 0};
  return s->e.correct(reinterpret_cast<const float2*>(d_src), reinterpret_cast<float2*>(d_dst), jobs, len,
                      reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"
