// PMC calibration: FETCH_SIZE / WRITE_SIZE of gfx950 for the access widths the DL chain uses.
// Each kernel reads (or writes) exactly BYTES bytes of a buffer far larger than the Infinity Cache, once,
// coalesced: a wave instruction covers 64 consecutive elements of the access width (b8 .. b128).  Run under
//   rocprofv3 --pmc FETCH_SIZE -- ./pmc_calib      and      rocprofv3 --pmc WRITE_SIZE -- ./pmc_calib
// and compare the counter (KiB) with the byte count each kernel prints (MI355X_MICROARCH.md: FETCH_SIZE reports
// half the bytes of 16-B-per-lane streaming reads; other widths are uncalibrated).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <class T>
__global__ __launch_bounds__(256) void rd(const T* __restrict__ p, size_t n, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const T v = __builtin_nontemporal_load(p + i);
    acc = acc * 33u + (uint32_t)v;
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc;   // 4 B per thread: negligible beside the buffer
}
template <class T>
__global__ __launch_bounds__(256) void rd_plain(const T* __restrict__ p, size_t n, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    acc = acc * 33u + (uint32_t)p[i];
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
}
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void rd128(const u4* __restrict__ p, size_t n, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const u4 v = p[i];
    acc = acc * 33u + (v.x ^ v.y ^ v.z ^ v.w);
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
}
template <class T>
__global__ __launch_bounds__(256) void wr(T* __restrict__ p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = (T)i;
}
// half-row writes: 64 lanes x 2 B = 128 B of every 256-B row (the int16 mirror's pattern beside fp32 rows)
__global__ __launch_bounds__(256) void wr16_rows(uint16_t* __restrict__ p, size_t rows) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < rows * 64; i += (size_t)gridDim.x * 256)
    p[(i / 64) * 128 + (i % 64)] = (uint16_t)i;
}

// rows of 64 lanes x sizeof(T) in a random order (every row once): wave w of the grid reads rows w, w + nw, ...
// through a multiplicative permutation -- the turbo decoder's [row][lane] accesses at interleaved rows
template <class T>
__global__ __launch_bounds__(256) void rd_rows(const T* __restrict__ p, uint32_t rows, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  const uint32_t lane = threadIdx.x & 63, nw = gridDim.x * 4;
  for (uint32_t r = blockIdx.x * 4 + threadIdx.x / 64; r < rows; r += nw) {
    const uint32_t row = (uint32_t)(((uint64_t)r * 2654435761ull) % rows);   // rows is odd-free power of 2: a permutation
    acc = acc * 33u + (uint32_t)p[(size_t)row * 64 + lane];
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
}
// the same with U independent rows in flight per wave (unrolled), and random-row writes: the achievable bandwidth of
// the turbo decoder's access pattern with more memory-level parallelism
template <class T, int U>
__global__ __launch_bounds__(256) void rd_rows_mlp(const T* __restrict__ p, uint32_t rows, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  const uint32_t lane = threadIdx.x & 63, nw = gridDim.x * 4;
  for (uint32_t r = (blockIdx.x * 4 + threadIdx.x / 64) * U; r < rows; r += nw * U) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t row = (uint32_t)(((uint64_t)(r + u) * 2654435761ull) % rows);
      v[u] = p[(size_t)row * 64 + lane];
    }
#pragma unroll
    for (int u = 0; u < U; u++) acc = acc * 33u + (uint32_t)v[u];
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
}
template <class T>
__global__ __launch_bounds__(256) void wr_rows(T* __restrict__ p, uint32_t rows) {
  const uint32_t lane = threadIdx.x & 63, nw = gridDim.x * 4;
  for (uint32_t r = blockIdx.x * 4 + threadIdx.x / 64; r < rows; r += nw) {
    const uint32_t row = (uint32_t)(((uint64_t)r * 2654435761ull) % rows);
    p[(size_t)row * 64 + lane] = (T)(r + lane);
  }
}
// partial-line stores: 16 B of every 128-B line (lanes 0-3 of a wave's 64 x 4 B, i.e. 4 lanes per 256 B)
__global__ __launch_bounds__(256) void wr_partial(uint32_t* __restrict__ p, size_t lines) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < lines * 4; i += (size_t)gridDim.x * 256)
    p[(i / 4) * 32 + (i % 4)] = (uint32_t)i;
}

int main() {
  const size_t BYTES = (size_t)2 << 30;   // 2 GiB: 8x the Infinity Cache
  void* buf;
  uint32_t* sink;
  if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
  if (hipMalloc(&sink, 8 << 20) != hipSuccess) return 1;
  (void)hipMemset(buf, 1, BYTES);
  (void)hipDeviceSynchronize();
  const int G = 256 * 8;
  printf("bytes per kernel: %zu (%.1f KiB)\n", BYTES, BYTES / 1024.0);
  for (int rep = 0; rep < 2; rep++) {
    rd<uint8_t><<<G, 256>>>((const uint8_t*)buf, BYTES, sink);
    rd<uint16_t><<<G, 256>>>((const uint16_t*)buf, BYTES / 2, sink);
    rd<uint32_t><<<G, 256>>>((const uint32_t*)buf, BYTES / 4, sink);
    rd<uint64_t><<<G, 256>>>((const uint64_t*)buf, BYTES / 8, sink);
    rd_plain<uint16_t><<<G, 256>>>((const uint16_t*)buf, BYTES / 2, sink);
    rd_plain<uint32_t><<<G, 256>>>((const uint32_t*)buf, BYTES / 4, sink);
    rd_plain<uint64_t><<<G, 256>>>((const uint64_t*)buf, BYTES / 8, sink);
    rd128<<<G, 256>>>((const u4*)buf, BYTES / 16, sink);
    wr<uint8_t><<<G, 256>>>((uint8_t*)buf, BYTES);
    wr<uint16_t><<<G, 256>>>((uint16_t*)buf, BYTES / 2);
    wr<uint32_t><<<G, 256>>>((uint32_t*)buf, BYTES / 4);
    wr<uint64_t><<<G, 256>>>((uint64_t*)buf, BYTES / 8);
    wr16_rows<<<G, 256>>>((uint16_t*)buf, BYTES / 256);   // writes BYTES / 2
    rd_rows<uint32_t><<<G, 256>>>((const uint32_t*)buf, (uint32_t)(BYTES / 256), sink);   // reads BYTES
    rd_rows<uint16_t><<<G, 256>>>((const uint16_t*)buf, (uint32_t)(BYTES / 128), sink);   // reads BYTES
    rd_rows<uint8_t><<<G, 256>>>((const uint8_t*)buf, (uint32_t)(BYTES / 64), sink);     // reads BYTES
    wr_partial<<<G, 256>>>((uint32_t*)buf, BYTES / 128);   // writes BYTES / 8
    rd_rows_mlp<uint32_t, 8><<<G, 256>>>((const uint32_t*)buf, (uint32_t)(BYTES / 256), sink);   // reads BYTES
    rd_rows_mlp<uint32_t, 16><<<G, 256>>>((const uint32_t*)buf, (uint32_t)(BYTES / 256), sink);
    rd_rows_mlp<uint32_t, 8><<<G / 4, 256>>>((const uint32_t*)buf, (uint32_t)(BYTES / 256), sink);   // 2 waves/SIMD
    rd_rows_mlp<uint16_t, 8><<<G, 256>>>((const uint16_t*)buf, (uint32_t)(BYTES / 128), sink);
    rd_rows_mlp<uint64_t, 8><<<G, 256>>>((const uint64_t*)buf, (uint32_t)(BYTES / 512), sink);
    wr_rows<uint32_t><<<G, 256>>>((uint32_t*)buf, (uint32_t)(BYTES / 256));   // writes BYTES
    wr_rows<uint8_t><<<G, 256>>>((uint8_t*)buf, (uint32_t)(BYTES / 64));      // writes BYTES
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("done (wr16_rows writes %zu bytes, wr_partial %zu)\n", BYTES / 2, BYTES / 8);
  return 0;
}
