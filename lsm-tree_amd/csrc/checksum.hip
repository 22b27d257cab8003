// checksum.hip — batched xxh3_128 (hash128, src/hash.rs:7-9) of arbitrary
// byte ranges in HBM: one wave per range, the wave-cooperative long path from
// device_common.hpp.  Used by tests to pin the device XXH3 against
// python-xxhash / the reference KATs, and available to callers that checksum
// ranges themselves (e.g. Block::write_into of externally built payloads).
#include <hip/hip_runtime.h>

#include "decode.hpp"
#include "device_common.hpp"
#include "lsmgpu.h"

namespace lsmgpu {

__global__ __launch_bounds__(64) void xxh3_128_batch_kernel(const uint8_t* __restrict__ data,
                                                            const uint64_t* __restrict__ off, uint32_t n,
                                                            uint64_t* __restrict__ out) {
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  const uint64_t o = off[i], e = off[i + 1];
  const uint8_t* base = data + (o & ~15ULL);
  uint64_t lo, hi;
  xxh3_128_wave(base, (uint32_t)(o & 15), (uint32_t)(e - o), &kLongSecret, lo, hi);
  if (threadIdx.x == 0) {
    out[2 * i] = lo;
    out[2 * i + 1] = hi;
  }
}

__global__ __launch_bounds__(64) void xxh3_file_short_kernel(const uint8_t* __restrict__ data, uint64_t len,
                                                             uint64_t* __restrict__ out) {
  const uint8_t* base = data - ((uintptr_t)data & 15);
  uint64_t lo, hi;
  xxh3_128_wave(base, (uint32_t)((uintptr_t)data & 15), (uint32_t)len, &kLongSecret, lo, hi);
  if (threadIdx.x == 0) {
    out[0] = lo;
    out[1] = hi;
  }
}

hipError_t launch_xxh3_128_batch(const uint8_t* data, const uint64_t* off, uint32_t n, uint64_t* out,
                                 hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(xxh3_128_batch_kernel, dim3(n), dim3(64), 0, st, data, off, n, out);
  return hipGetLastError();
}

// ---- whole-file xxh3_128 (ChecksummedWriter, src/checksum.rs:59-96: the
// streaming digest equals the one-shot xxh3_128 of the file,
// tests/table_full_file_checksum.rs:26-31).  One input of any length, spread
// over the whole GPU: the per-KiB contributions of the XXH3 long loop do not
// depend on the accumulators, so K1 computes them for every KiB block in
// parallel (wave per KiB, 64 B per KiB into the workspace) and K2 (one wave)
// runs the serial scramble chain, the tail stripes and the merge.
__global__ __launch_bounds__(256) void xxh3_file_contrib_kernel(const uint8_t* __restrict__ data, uint64_t nb,
                                                                uint64_t* __restrict__ contrib) {
  const int lane = threadIdx.x & 63;
  const int q = lane & 3, s = lane >> 2;
  const LongSecret* ls = &kLongSecret;
  const uint64_t k0 = ls->acc[s + 2 * q], k1 = ls->acc[s + 2 * q + 1];
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
  for (uint64_t n = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); n < nb; n += waves) {
    const uint64_t a = (uint64_t)(uintptr_t)(data + n * 1024);
    const Win16 w = read_win16(reinterpret_cast<const uint8_t*>(a & ~15ULL), (uint32_t)(a & 15) + 16 * lane);
    uint64_t c0 = 0, c1 = 0;
    stripe_part(w, k0, k1, c0, c1);
    c0 = quad_group_sum64(c0);
    c1 = quad_group_sum64(c1);
    if (lane < 4) {
      contrib[8 * n + 2 * q] = c0;
      contrib[8 * n + 2 * q + 1] = c1;
    }
  }
}

__global__ __launch_bounds__(64) void xxh3_file_finish_kernel(const uint8_t* __restrict__ data, uint64_t len,
                                                              const uint64_t* __restrict__ contrib,
                                                              uint64_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int q = lane & 3, s = lane >> 2;
  const LongSecret* ls = &kLongSecret;
  const uint64_t k0 = ls->acc[s + 2 * q], k1 = ls->acc[s + 2 * q + 1];
  uint64_t a0 = q == 0 ? (uint64_t)P32_3 : q == 1 ? P64_2 : q == 2 ? P64_4 : P64_5;
  uint64_t a1 = q == 0 ? P64_1 : q == 1 ? P64_3 : q == 2 ? (uint64_t)P32_2 : (uint64_t)P32_1;
  const uint64_t scr0 = ls->acc[16 + 2 * q], scr1 = ls->acc[16 + 2 * q + 1];
  const uint64_t nb = (len - 1) / 1024;
  uint64_t n = 0;
  // The chain is one wave's dependent VALU work; feeding it straight from HBM
  // stalls on load latency every few steps.  Instead the whole wave streams
  // the contributions of kChunk KiB blocks (16 KiB) into registers one chunk
  // ahead, parks them in LDS, and the chain reads LDS only.
  constexpr uint32_t kChunk = 256;
  __shared__ u32x4 stage[kChunk * 4];  // 64 B of contributions per KiB block
  const uint64_t nchunks = nb / kChunk;
  const u32x4* src = reinterpret_cast<const u32x4*>(contrib);
  u32x4 r[16];
  if (nchunks) {
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = __builtin_nontemporal_load(&src[i * 64 + lane]);
  }
  for (uint64_t c = 0; c < nchunks; ++c) {
#pragma unroll
    for (int i = 0; i < 16; ++i) stage[i * 64 + lane] = r[i];
    __syncthreads();
    if (c + 1 < nchunks) {
      const u32x4* nx = src + (c + 1) * kChunk * 4;
#pragma unroll
      for (int i = 0; i < 16; ++i) r[i] = __builtin_nontemporal_load(&nx[i * 64 + lane]);
    }
    const uint64_t* st = reinterpret_cast<const uint64_t*>(stage);
#pragma unroll 8
    for (uint32_t u = 0; u < kChunk; ++u) {
      const uint64_t c0 = st[8 * u + 2 * q], c1 = st[8 * u + 2 * q + 1];
      a0 = xxh3_scr(a0, c0, scr0);
      a1 = xxh3_scr(a1, c1, scr1);
    }
    __syncthreads();
  }
  n = nchunks * kChunk;
  for (; n + 4 <= nb; n += 4) {  // contributions of four KiB blocks in flight per step
    uint64_t c[8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      c[2 * u] = contrib[8 * (n + u) + 2 * q];
      c[2 * u + 1] = contrib[8 * (n + u) + 2 * q + 1];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a0 = xxh3_scr(a0, c[2 * u], scr0);
      a1 = xxh3_scr(a1, c[2 * u + 1], scr1);
    }
  }
  for (; n < nb; ++n) {
    a0 = xxh3_scr(a0, contrib[8 * n + 2 * q], scr0);
    a1 = xxh3_scr(a1, contrib[8 * n + 2 * q + 1], scr1);
  }
  {  // tail stripes of the last (partial) KiB block, then the last stripe (secret + 121)
    const uint64_t tail0 = nb * 1024;
    const uint32_t nb_stripes = (uint32_t)(((len - 1) - tail0) / 64);
    uint64_t c0 = 0, c1 = 0;
    if ((uint32_t)s < nb_stripes) {
      const uint64_t a = (uint64_t)(uintptr_t)(data + tail0);
      const Win16 w = read_win16(reinterpret_cast<const uint8_t*>(a & ~15ULL), (uint32_t)(a & 15) + 16 * lane);
      stripe_part(w, k0, k1, c0, c1);
    }
    if (lane < 4) {
      const uint64_t a = (uint64_t)(uintptr_t)(data + len - 64);
      const Win16 w = read_win16(reinterpret_cast<const uint8_t*>(a & ~15ULL), (uint32_t)(a & 15) + 16 * lane);
      stripe_part(w, ls->last[2 * q], ls->last[2 * q + 1], c0, c1);
    }
    a0 += quad_group_sum64(c0);
    a1 += quad_group_sum64(c1);
  }
  uint64_t tlo = mul_fold64(a0 ^ ls->mlo[2 * q], a1 ^ ls->mlo[2 * q + 1]);
  uint64_t thi = mul_fold64(a0 ^ ls->mhi[2 * q], a1 ^ ls->mhi[2 * q + 1]);
  tlo += shfl_xor64(tlo, 1);
  thi += shfl_xor64(thi, 1);
  tlo += shfl_xor64(tlo, 2);
  thi += shfl_xor64(thi, 2);
  if (lane == 0) {
    out[0] = xxh3_avalanche(len * P64_1 + tlo);
    out[1] = xxh3_avalanche(~(len * P64_2) + thi);
  }
}

size_t xxh3_file_workspace_size(uint64_t len) { return len > 240 ? ((len - 1) / 1024) * 64 + 256 : 256; }

hipError_t launch_xxh3_128_file(const uint8_t* data, uint64_t len, uint64_t* out, void* ws, hipStream_t st) {
  if (len <= 240) {  // short paths: one wave
    hipLaunchKernelGGL(xxh3_file_short_kernel, dim3(1), dim3(64), 0, st, data, len, out);
    return hipGetLastError();
  }
  const uint64_t nb = (len - 1) / 1024;
  uint64_t* contrib = (uint64_t*)ws;
  if (nb) {
    const uint64_t wgs = (nb + 3) / 4;
    hipLaunchKernelGGL(xxh3_file_contrib_kernel, dim3((uint32_t)(wgs < 65536 ? wgs : 65536)), dim3(256), 0, st, data,
                       nb, contrib);
  }
  hipLaunchKernelGGL(xxh3_file_finish_kernel, dim3(1), dim3(64), 0, st, data, len, contrib, out);
  return hipGetLastError();
}

}  // namespace lsmgpu

extern "C" size_t lsm_xxh3_128_file_workspace_size(uint64_t len) { return lsmgpu::xxh3_file_workspace_size(len); }

extern "C" int lsm_xxh3_128_file(const uint8_t* d_data, uint64_t len, uint64_t* d_out, void* d_workspace,
                                 size_t workspace_bytes, void* stream) {
  if (!d_out || (len && !d_data)) return LSM_BAD_ARG;
  if (len > 240 && (!d_workspace || workspace_bytes < lsmgpu::xxh3_file_workspace_size(len))) return LSM_BAD_ARG;
  const hipError_t e = lsmgpu::launch_xxh3_128_file(d_data, len, d_out, d_workspace, (hipStream_t)stream);
  return lsmgpu::hip_status(e, "lsm_xxh3_128_file");
}
