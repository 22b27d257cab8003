// scan.hpp — device-wide exclusive prefix sum over u64 counts (block item
// counts -> item_start, encoded block sizes -> block offsets).
// Three small launches: per-tile reduce, scan of tile sums, per-tile scan
// (one, for a single tile).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.hpp"

namespace lsmgpu {

constexpr int kScanThreads = 256;
constexpr int kScanPerThread = 8;
constexpr int kScanTile = kScanThreads * kScanPerThread;  // 2048

__device__ __forceinline__ uint64_t block_excl_scan_u64(uint64_t v, uint64_t* sh /*[kScanThreads/64]*/,
                                                        uint64_t& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint64_t incl = wave_incl_scan_u64(v);
  if (lane == 63) sh[wid] = incl;
  __syncthreads();
  uint64_t wbase = 0, tot = 0;
  for (int i = 0; i < kScanThreads / 64; ++i) {
    uint64_t s = sh[i];
    if (i < wid) wbase += s;
    tot += s;
  }
  __syncthreads();
  total = tot;
  return wbase + incl - v;
}

// A thread's kScanPerThread inputs: one vector load when all are in range
// (the inputs are 256-B aligned workspace arrays), else one at a time.
template <class T>
__device__ __forceinline__ void scan_load(const T* in, uint64_t base, uint64_t n, uint64_t (&v)[kScanPerThread]) {
  typedef T vec_t __attribute__((ext_vector_type(kScanPerThread)));
  if (base + kScanPerThread <= n) {
    const vec_t x = *(const __attribute__((address_space(1))) vec_t*)(in + base);
#pragma unroll
    for (int i = 0; i < kScanPerThread; ++i) v[i] = x[i];
  } else {
#pragma unroll
    for (int i = 0; i < kScanPerThread; ++i) v[i] = base + i < n ? in[base + i] : 0;
  }
}

template <class T>
__global__ __launch_bounds__(kScanThreads) void scan_tile_reduce(const T* __restrict__ in, uint64_t n,
                                                                 uint64_t* __restrict__ tile_sums) {
  __shared__ uint64_t sh[kScanThreads / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPerThread;
  uint64_t v[kScanPerThread];
  scan_load(in, base, n, v);
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) s += v[i];
  uint64_t total;
  block_excl_scan_u64(s, sh, total);
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

// Single workgroup: exclusive scan of the tile sums in place, kScanPerThread
// consecutive tiles per thread (one pass for up to kScanTile tiles: 2048 tiles
// of 2048 inputs each).
static __global__ __launch_bounds__(kScanThreads) void scan_tile_sums(uint64_t* __restrict__ sums, uint64_t n_tiles) {
  __shared__ uint64_t sh[kScanThreads / 64];
  uint64_t carry = 0;
  for (uint64_t b0 = 0; b0 < n_tiles; b0 += kScanTile) {
    const uint64_t base = b0 + (uint64_t)threadIdx.x * kScanPerThread;
    uint64_t v[kScanPerThread];
    scan_load(sums, base, n_tiles, v);
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanPerThread; ++i) s += v[i];
    uint64_t total;
    uint64_t ex = carry + block_excl_scan_u64(s, sh, total);
#pragma unroll
    for (int i = 0; i < kScanPerThread; ++i) {
      if (base + i < n_tiles) sums[base + i] = ex;
      ex += v[i];
    }
    carry += total;
  }
}
// Out(i, prefix) is called for i in [0, n] with the exclusive prefix.  Each
// thread reads its inputs before its first Out call, so Out may overwrite in[i].
// tile_offsets == nullptr: a single tile (no tile sums to add).
template <class T, class Out>
__global__ __launch_bounds__(kScanThreads) void scan_tile_apply(const T* in, uint64_t n,
                                                                const uint64_t* __restrict__ tile_offsets,
                                                                Out out) {
  __shared__ uint64_t sh[kScanThreads / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPerThread;
  uint64_t v[kScanPerThread];
  scan_load(in, base, n, v);
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) s += v[i];
  uint64_t total;
  uint64_t ex = block_excl_scan_u64(s, sh, total) + (tile_offsets ? tile_offsets[blockIdx.x] : 0);
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) {
    if (base + i < n) out(base + i, ex);
    if (base + i == n - 1) out(n, ex + v[i]);
    ex += v[i];
  }
}

inline uint64_t scan_tiles(uint64_t n) { return (n + kScanTile - 1) / kScanTile; }

// The tile pre-passes of a scan with more than one tile (per-tile reduce, scan of
// the tile sums into tmp); *offs = tmp then, else null (a single tile needs none).
template <class T>
inline hipError_t launch_scan_tile_offsets(const T* in, uint64_t n, uint64_t* tmp, hipStream_t st,
                                           const uint64_t** offs) {
  const uint64_t tiles = scan_tiles(n);
  *offs = nullptr;
  if (tiles == 1) return hipSuccess;  // (a batch of <= 2048 blocks: one launch, not three of ~4.5 us each)
  hipLaunchKernelGGL(scan_tile_reduce<T>, dim3((uint32_t)tiles), dim3(kScanThreads), 0, st, in, n, tmp);
  hipLaunchKernelGGL(scan_tile_sums, dim3(1), dim3(kScanThreads), 0, st, tmp, tiles);
  *offs = tmp;
  return hipGetLastError();
}

// Enqueue the scan (u64 or u32 inputs, u64 prefixes); `tmp` holds scan_tiles(n) u64.  n >= 1.
template <class T, class Out>
inline hipError_t launch_excl_scan(const T* in, uint64_t n, uint64_t* tmp, Out out, hipStream_t st) {
  const uint64_t* offs;
  hipError_t e = launch_scan_tile_offsets(in, n, tmp, st, &offs);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((scan_tile_apply<T, Out>), dim3((uint32_t)scan_tiles(n)), dim3(kScanThreads), 0, st, in, n, offs,
                     out);
  return hipGetLastError();
}
}  // namespace lsmgpu
