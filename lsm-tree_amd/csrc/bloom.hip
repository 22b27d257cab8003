// bloom.hip — the table's standard Bloom filter on the device
// (src/table/filter/standard_bloom/, written by FullFilterWriter,
// src/table/writer/filter/full.rs:47-92, probed by Table::point_read through
// StandardBloomFilterReader::contains_hash, standard_bloom/mod.rs:100-120).
//
//   hash64_keys_kernel    Builder::get_hash = hash64 = xxh3_64 (builder.rs:172-175,
//                         src/hash.rs:2-4): lane per key, straight from the key arena.
//   bloom_init_kernel     Builder::build's header (builder.rs:33-53) + zeroed bit array.
//   bloom_set_kernel      set_with_hash (builder.rs:154-170): lane per hash, k
//                         double-hashed bit positions, one 32-bit atomicOr each.
//   bloom_contains_kernel contains_hash: lane per probe, early exit on a clear bit.
//
// Layout in HBM: the filter is the exact byte image Builder::build returns
// (22-byte header, then m/8 bytes, bit i = byte i/8 mask 0x80 >> i%8), so the
// set kernel ORs into the 32-bit word holding byte 22 + i/8.  Work per key is
// k scattered 4-byte atomics into a filter that is ~1.2 MB per million keys
// (BitsPerKey(10)), which lives in L2: the build is atomic-throughput bound,
// the probe latency bound; neither is an HBM-streaming kernel.
#include <hip/hip_runtime.h>

#include "decode.hpp"
#include "device_common.hpp"
#include "lsmgpu.h"

namespace lsmgpu {

constexpr uint32_t kBloomHdr = 22;  // magic 4 + filter type 1 + hash type 1 + m u64 + k u64
constexpr uint64_t kBloomMaxK = LSM_BLOOM_MAX_K;

__device__ __forceinline__ uint64_t bloom_secondary(uint64_t h1) {  // builder.rs:10-13
  return (h1 >> 32) * 0x517cc1b727220a95ULL;
}

__global__ __launch_bounds__(256) void hash64_keys_kernel(const uint8_t* __restrict__ keys,
                                                          const uint64_t* __restrict__ key_off, uint64_t n,
                                                          uint64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t o = key_off[i], e = key_off[i + 1];
  const uint8_t* b = keys + (o & ~15ULL);
  const uint32_t p = (uint32_t)(o & 15);
  out[i] = xxh3_64_any((uint32_t)(e - o), BaseReader8{b, p}, BaseReader64{b, p});
}

__global__ __launch_bounds__(256) void bloom_init_kernel(uint32_t* __restrict__ filter, uint64_t m, uint64_t k,
                                                         uint64_t words) {
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += (uint64_t)gridDim.x * blockDim.x) {
    // bytes 0..23: "LSM\x03", filter type 0, hash type 0, m u64 LE, k u64 LE, first two bit bytes 0
    const uint32_t v = w == 0   ? 0x034D534Cu
                       : w == 1 ? (uint32_t)(m << 16)
                       : w == 2 ? (uint32_t)(m >> 16)
                       : w == 3 ? (uint32_t)(m >> 48) | (uint32_t)(k << 16)
                       : w == 4 ? (uint32_t)(k >> 16)
                       : w == 5 ? (uint32_t)(k >> 48)
                                : 0u;
    filter[w] = v;
  }
}

__global__ __launch_bounds__(256) void bloom_set_kernel(const uint64_t* __restrict__ hashes, uint64_t n, uint64_t m,
                                                        uint32_t k, uint32_t* __restrict__ filter) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  uint64_t h1 = hashes[j], h2 = bloom_secondary(h1);
  for (uint32_t i = 1; i <= k; ++i) {
    const uint64_t idx = h1 % m;
    const uint64_t byte = kBloomHdr + (idx >> 3);
    atomicOr(filter + (byte >> 2), (0x80u >> (idx & 7)) << (8 * (byte & 3)));
    h1 += h2;
    h2 *= i;
  }
}

__global__ __launch_bounds__(256) void bloom_contains_kernel(const uint8_t* __restrict__ filter, uint64_t len,
                                                             const uint64_t* __restrict__ hashes, uint64_t n,
                                                             uint8_t* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  // StandardBloomFilterReader::new (mod.rs:36-86), re-read by every lane from one cached line
  uint64_t m = 0, k = 0;
#pragma unroll
  for (int b = 7; b >= 0; --b) {
    m = (m << 8) | filter[6 + b];
    k = (k << 8) | filter[14 + b];
  }
  const bool ok = filter[0] == 'L' && filter[1] == 'S' && filter[2] == 'M' && filter[3] == 3 && filter[4] == 0 &&
                  filter[5] == 0 && m > 0 && (m + 7) / 8 <= len - kBloomHdr &&
                  k <= kBloomMaxK;  // bounded probe loop (a garbage k must not spin a wave)
  if (!ok) {
    out[j] = LSM_BLOOM_BAD_FILTER;
    return;
  }
  const uint8_t* bits = filter + kBloomHdr;
  uint64_t h1 = hashes[j], h2 = bloom_secondary(h1);
  uint8_t r = 1;
  for (uint64_t i = 1; i <= k; ++i) {
    const uint64_t idx = h1 % m;
    if (!(bits[idx >> 3] & (0x80u >> (idx & 7)))) {
      r = 0;
      break;
    }
    h1 += h2;
    h2 *= i;
  }
  out[j] = r;
}

static inline uint32_t grid_for(uint64_t n) { return (uint32_t)((n + 255) / 256); }

}  // namespace lsmgpu

using namespace lsmgpu;

namespace {
constexpr float kLn2 = 0.693147180559945309417232121458176568f;  // std::f32::consts::LN_2
uint64_t f32_to_usize(float x) {  // Rust `as usize`: truncate, NaN/negative -> 0, saturate
  if (!(x > 0.0f)) return 0;
  if (x >= 18446744073709551616.0f) return UINT64_MAX;
  return (uint64_t)x;
}
}  // namespace

extern "C" {

uint64_t lsm_bloom_calculate_m(uint64_t n, float fpr) {  // builder.rs:128-151
  const float numerator = (float)n * logf(fpr);
  const float m = -(numerator / (kLn2 * kLn2));
  return f32_to_usize(ceilf(m / 8.0f) * 8.0f);
}

int lsm_bloom_shape(uint64_t n, int policy, float value, uint64_t* m, uint64_t* k) {
  if (!m || !k || n == 0) return LSM_BAD_ARG;  // assert!(n > 0)
  if (policy == LSM_BLOOM_BITS_PER_KEY) {      // Builder::with_bpk, builder.rs:91-126
    if (!(value > 0.0f)) return LSM_BAD_ARG;    // assert!(bpk > 0.0)
    const uint64_t mm = n * f32_to_usize(value);
    const uint64_t kk = f32_to_usize(value * kLn2);
    *m = f32_to_usize(ceilf((float)mm / 8.0f)) * 8;
    *k = kk < 1 ? 1 : kk;
    return LSM_OK;
  }
  if (policy == LSM_BLOOM_FP_RATE) {  // Builder::with_fp_rate, builder.rs:58-85
    const float fpr = value >= 0.0000001f ? value : 0.0000001f;
    const uint64_t mm = lsm_bloom_calculate_m(n, fpr);
    const uint64_t kk = f32_to_usize((float)(mm / n) * kLn2);
    *m = mm;
    *k = kk < 1 ? 1 : kk;
    return LSM_OK;
  }
  return LSM_BAD_ARG;
}

uint64_t lsm_bloom_filter_size(uint64_t m) { return kBloomHdr + (m + 7) / 8; }

int lsm_hash64_keys(const uint8_t* d_keys, const uint64_t* d_key_off, uint64_t n, uint64_t* d_out, void* stream) {
  if (n == 0) return LSM_OK;
  if (!d_keys || !d_key_off || !d_out || ((uintptr_t)d_keys & 15)) return LSM_BAD_ARG;
  hipLaunchKernelGGL(hash64_keys_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, d_keys, d_key_off, n,
                     d_out);
  return lsmgpu::hip_status(hipGetLastError(), __func__);
}

int lsm_bloom_build(const uint64_t* d_hashes, uint64_t n, uint64_t m, uint64_t k, uint8_t* d_filter,
                    uint64_t filter_cap, void* stream) {
  const uint64_t len = lsm_bloom_filter_size(m);
  const uint64_t words = (len + 3) / 4;
  if (!d_filter || m == 0 || (m & 7) || k == 0 || k > kBloomMaxK || ((uintptr_t)d_filter & 3) ||
      filter_cap < words * 4 || (n && !d_hashes))
    return LSM_BAD_ARG;
  const hipStream_t st = (hipStream_t)stream;
  const uint64_t g = words / 256 + 1;
  hipLaunchKernelGGL(bloom_init_kernel, dim3((uint32_t)(g < 8192 ? g : 8192)), dim3(256), 0, st, (uint32_t*)d_filter, m,
                     k, words);
  if (n)
    hipLaunchKernelGGL(bloom_set_kernel, dim3(grid_for(n)), dim3(256), 0, st, d_hashes, n, m, (uint32_t)k,
                       (uint32_t*)d_filter);
  return lsmgpu::hip_status(hipGetLastError(), __func__);
}

int lsm_bloom_contains(const uint8_t* d_filter, uint64_t filter_len, const uint64_t* d_hashes, uint64_t n,
                       uint8_t* d_out, void* stream) {
  if (n == 0) return LSM_OK;
  if (!d_filter || !d_hashes || !d_out || filter_len < kBloomHdr) return LSM_BAD_ARG;
  hipLaunchKernelGGL(bloom_contains_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, d_filter,
                     filter_len, d_hashes, n, d_out);
  return lsmgpu::hip_status(hipGetLastError(), __func__);
}

}  // extern "C"
