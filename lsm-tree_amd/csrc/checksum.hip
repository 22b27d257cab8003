// checksum.hip — batched xxh3_128 (hash128, src/hash.rs:7-9) of arbitrary
// byte ranges in HBM: one wave per range, the wave-cooperative long path from
// device_common.hpp.  Used by tests to pin the device XXH3 against
// python-xxhash / the reference KATs, and available to callers that checksum
// ranges themselves (e.g. Block::write_into of externally built payloads).
#include <hip/hip_runtime.h>

#include <stddef.h>

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

hipError_t launch_xxh3_128_batch(const uint8_t* data, const uint64_t* off, uint32_t n, uint64_t* out,
                                 hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(xxh3_128_batch_kernel, dim3(n), dim3(64), 0, st, data, off, n, out);
  return hipGetLastError();
}

// ---- whole-file xxh3_128 as a resumable stream (ChecksummedWriter,
// src/checksum.rs:59-96: every write() feeds a running Xxh3Default, whose
// digest128 equals the one-shot xxh3_128 of the file,
// tests/table_full_file_checksum.rs:26-31).
//
// The running state lives in device memory (Xxh3Stream).  XXH3's long loop
// consumes the input in 1 KiB blocks: each block adds a contribution to the 8
// accumulators that does not depend on them (16 stripes), then scrambles
// them.  A block is consumed only once at least one byte follows it (a final
// full KiB is the tail of the one-shot algorithm, never scrambled), so the
// state keeps 1..1024 pending bytes, plus the 64 bytes before them for the
// last stripe (input[len-64 .. len) may reach back into consumed data).
// update(data, len) = K1 the contributions of every KiB block of
// pending || data that can be consumed (whole GPU, wave per KiB) + K2 the
// serial scramble chains over them (8 single-wave workgroups, accumulator k
// on workgroup k) + K3 the new pending / history bytes.  digest() = tail stripes + last stripe + merge
// (one wave), the state is left unchanged.
struct alignas(16) Xxh3Stream {
  uint64_t acc[8];
  uint64_t total;      // bytes fed so far
  uint32_t pending;    // bytes in buf (1..1024 once total > 0)
  uint32_t magic;      // kStreamMagic after init
  uint8_t pad[48];
  uint8_t hist[64];    // the 64 bytes just before buf (valid once a KiB block was consumed)
  uint8_t buf[1024];   // pending bytes
  uint8_t slack[64];   // readable past buf (window reads)
};
static_assert(sizeof(Xxh3Stream) == 1280 && offsetof(Xxh3Stream, hist) == 128 && offsetof(Xxh3Stream, buf) == 192,
              "Xxh3Stream layout: hist immediately precedes buf");
constexpr uint32_t kStreamMagic = 0x58583353u;  // "S3XX"

// workgroup i initialises states[i]
__global__ __launch_bounds__(64) void xxh3_stream_init_kernel(Xxh3Stream* states) {
  Xxh3Stream* st = states + blockIdx.x;
  const int lane = threadIdx.x;
  uint64_t a0, a1;
  xxh3_acc_init(lane & 3, a0, a1);
  if (lane < 4) {
    st->acc[2 * lane] = a0;
    st->acc[2 * lane + 1] = a1;
  }
  if (lane == 0) {
    st->total = 0;
    st->pending = 0;
    st->magic = kStreamMagic;
  }
}

// KiB blocks of pending || data that this update consumes: all but the last
// (partial or full) KiB of the combined input.
__device__ __forceinline__ uint64_t stream_blocks(uint32_t pending, uint64_t len) {
  const uint64_t t = (uint64_t)pending + len;
  return t ? (t - 1) / 1024 : 0;
}

// The 16 bytes at offset o of pending || data.
__device__ __forceinline__ Win16 stream_window(const Xxh3Stream* __restrict__ st, uint32_t pend,
                                               const uint8_t* __restrict__ data, uint64_t o) {
  if (o >= pend) {
    const uint64_t a = (uint64_t)(uintptr_t)(data + (o - pend));
    return read_win16(reinterpret_cast<const uint8_t*>(a & ~15ULL), (uint32_t)(a & 15));
  }
  if (o + 16 <= pend) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(st->buf + o);
    return Win16{(uint64_t)v.x | ((uint64_t)v.y << 32), (uint64_t)v.z | ((uint64_t)v.w << 32)};
  }
  uint64_t lo = 0, hi = 0;  // the 16 bytes straddle the end of the pending bytes
  for (uint32_t i = 0; i < 16; ++i) {
    const uint64_t x = o + i < pend ? st->buf[o + i] : data[o + i - pend];
    if (i < 8) lo |= x << (8 * i);
    else hi |= x << (8 * (i - 8));
  }
  return Win16{lo, hi};
}

// K1: wave per consumable KiB block j of pending || data; lane l reduces bytes
// [1024 j + 16 l, +16) (stripe l >> 2, accumulator pair l & 3).
__global__ __launch_bounds__(256) void xxh3_stream_contrib_kernel(const Xxh3Stream* __restrict__ st,
                                                                  const uint8_t* __restrict__ data, uint64_t len,
                                                                  uint64_t* __restrict__ contrib) {
  const int lane = threadIdx.x & 63;
  const int q = lane & 3, s = lane >> 2;
  const LongSecret* ls = &kLongSecret;
  const uint64_t k0 = ls->acc[s + 2 * q], k1 = ls->acc[s + 2 * q + 1];
  const uint32_t pend = st->pending;
  const uint64_t nb = stream_blocks(pend, len);
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
  for (uint64_t n = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); n < nb; n += waves) {
    const uint64_t o = n * 1024 + 16 * lane;  // offset in pending || data
    const Win16 w = stream_window(st, pend, data, o);
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

// K2: 8 single-wave workgroups; workgroup k carries accumulator k over this
// update's KiB blocks.
__global__ __launch_bounds__(64) void xxh3_stream_chain_kernel(Xxh3Stream* __restrict__ st, uint64_t len,
                                                                const uint64_t* __restrict__ contrib) {
  const uint32_t k = blockIdx.x;
  const uint64_t nb = stream_blocks(st->pending, len);
  if (!nb) return;
  const uint64_t x = xxh3_chain_wave(contrib, nb, k, st->acc[k], kLongSecret.acc[16 + k]);
  if (threadIdx.x == 0) st->acc[k] = x;
}

// K3: the new pending bytes (and the 64 before them) into the state: all
// reads first, a barrier, then the writes (the new history may come from the
// old pending bytes).
__device__ __forceinline__ void stream_buffer_wg(Xxh3Stream* __restrict__ st, const uint8_t* __restrict__ data,
                                                 uint64_t len) {
  const uint32_t tid = threadIdx.x;
  const uint32_t pend = st->pending;
  const uint64_t nb = stream_blocks(pend, len);
  const uint64_t t = (uint64_t)pend + len;
  uint8_t v[3] = {0, 0, 0};
  uint32_t cnt, dst0;
  uint64_t src0;
  if (nb) {  // hist || buf = (pending || data)[1024 nb - 64, t)
    src0 = nb * 1024 - 64;
    cnt = (uint32_t)(t - src0);
    dst0 = 0;
  } else {   // append to the pending bytes
    src0 = pend;
    cnt = (uint32_t)len;
    dst0 = 64 + pend;
  }
#pragma unroll
  for (uint32_t r = 0; r < 3; ++r) {
    const uint32_t i = tid + 512 * r;
    if (i < cnt) {
      const uint64_t x = src0 + i;
      v[r] = x < pend ? st->buf[x] : data[x - pend];
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < 3; ++r) {
    const uint32_t i = tid + 512 * r;
    if (i < cnt) st->hist[dst0 + i] = v[r];  // (hist[64 + j] is buf[j])
  }
  if (tid == 0) {
    st->pending = nb ? (uint32_t)(t - nb * 1024) : (uint32_t)t;
    st->total += len;
  }
}

__global__ __launch_bounds__(512) void xxh3_stream_buffer_kernel(Xxh3Stream* __restrict__ st,
                                                                 const uint8_t* __restrict__ data, uint64_t len) {
  stream_buffer_wg(st, data, len);
}

// digest128 (Xxh3Default::digest128): the tail stripes of the pending bytes,
// the last stripe (64 bytes ending at the input's end: hist || buf), the
// merge and the avalanche.  One wave; the state is not modified.
__device__ __forceinline__ void stream_digest_wave(const Xxh3Stream* __restrict__ st, uint64_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int q = lane & 3, s = lane >> 2;
  const LongSecret* ls = &kLongSecret;
  const uint8_t* sb = reinterpret_cast<const uint8_t*>(st);
  const uint64_t len = st->total;
  const uint32_t pend = st->pending;
  const uint32_t buf = (uint32_t)offsetof(Xxh3Stream, buf);
  uint64_t lo, hi;
  if (len <= 240) {  // short paths: every byte is still pending
    xxh3_128_wave(sb, buf, (uint32_t)len, ls, lo, hi);
  } else {
    uint64_t a0 = st->acc[2 * q], a1 = st->acc[2 * q + 1];
    const uint32_t nb_stripes = (pend - 1) / 64;
    uint64_t c0 = 0, c1 = 0;
    if ((uint32_t)s < nb_stripes)
      stripe_part(read_win16(sb, buf + 16 * lane), ls->acc[s + 2 * q], ls->acc[s + 2 * q + 1], c0, c1);
    if (lane < 4) stripe_part(read_win16(sb, buf + pend - 64 + 16 * lane), ls->last[2 * q], ls->last[2 * q + 1], c0, c1);
    a0 += quad_group_sum64(c0);
    a1 += quad_group_sum64(c1);
    uint64_t tlo = mul_fold64(a0 ^ ls->mlo[2 * q], a1 ^ ls->mlo[2 * q + 1]);
    uint64_t thi = mul_fold64(a0 ^ ls->mhi[2 * q], a1 ^ ls->mhi[2 * q + 1]);
    tlo += shfl_xor64(tlo, 1);
    thi += shfl_xor64(thi, 1);
    tlo += shfl_xor64(tlo, 2);
    thi += shfl_xor64(thi, 2);
    lo = xxh3_avalanche(len * P64_1 + tlo);
    hi = xxh3_avalanche(~(len * P64_2) + thi);
  }
  if (lane == 0) {
    out[0] = lo;
    out[1] = hi;
  }
}

__global__ __launch_bounds__(64) void xxh3_stream_digest_kernel(const Xxh3Stream* __restrict__ st,
                                                                uint64_t* __restrict__ out) {
  stream_digest_wave(st, out);
}

constexpr uint32_t kChainLds = 96 * 1024;

size_t xxh3_stream_workspace_size(uint64_t len) { return 64 * (len / 1024 + 2) + 256; }

hipError_t launch_xxh3_stream_update(Xxh3Stream* st, const uint8_t* data, uint64_t len, uint64_t* contrib,
                                     hipStream_t s) {
  if (len == 0) return hipSuccess;
  const uint64_t kmax = (len + 1023) / 1024 + 1;  // blocks of pending (<= 1024) || data, at most
  const uint64_t wgs = (kmax + 3) / 4;
  hipLaunchKernelGGL(xxh3_stream_contrib_kernel, dim3((uint32_t)(wgs < 65536 ? wgs : 65536)), dim3(256), 0, s, st,
                     data, len, contrib);
  // (an unused 96 KiB LDS request: one chain workgroup per CU, no two chains share a SIMD)
  static uint64_t attr_done = 0;
  hipError_t e = set_lds_attr((const void*)xxh3_stream_chain_kernel, kChainLds, &attr_done);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(xxh3_stream_chain_kernel, dim3(8), dim3(64), kChainLds, s, st, len, contrib);
  hipLaunchKernelGGL(xxh3_stream_buffer_kernel, dim3(1), dim3(512), 0, s, st, data, len);
  return hipGetLastError();
}

// ---- many running states in one launch sequence (a flush or compaction that
// rotates through several tables, src/table/multi_writer.rs:181-257, each
// with its own ChecksummedWriter, src/checksum.rs:59-96).  State i (states[i],
// back to back) is fed data[off[i] .. off[i+1]).  The KiB blocks every state
// consumes are numbered in one space (bpre = exclusive prefix of the per-state
// counts), so one contribution launch covers all states, one chain launch runs
// 8 chains per state side by side, one buffer launch moves every state's
// pending bytes.
constexpr uint32_t kBatchWgBlocks = 64;  // consecutive global KiB blocks per contribution workgroup

__device__ __forceinline__ bool batch_state_ok(const Xxh3Stream* st, const uint64_t* off, uint32_t i) {
  return st->magic == kStreamMagic && off[i + 1] >= off[i];
}

// B0: per-state status and KiB block counts, exclusive prefix over the batch
// (one workgroup, chunks of 1024 states).  A batch whose blocks exceed the
// workspace (total_len below the real byte count) is rejected whole.
__global__ __launch_bounds__(1024) void xxh3_batch_plan_kernel(const Xxh3Stream* __restrict__ states, uint32_t n,
                                                               const uint64_t* __restrict__ off, uint64_t cap_blocks,
                                                               uint64_t total_len, uint64_t* __restrict__ bpre,
                                                               int32_t* __restrict__ status) {
  __shared__ uint64_t wsum[16];
  __shared__ uint64_t carry_s;
  __shared__ unsigned long long bytes_s;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) carry_s = 0, bytes_s = 0;
  __syncthreads();
  for (uint32_t c = 0; c < n; c += 1024) {
    const uint32_t i = c + tid;
    uint64_t nb = 0, len = 0;
    if (i < n) {
      const bool ok = batch_state_ok(states + i, off, i);
      len = off[i + 1] >= off[i] ? off[i + 1] - off[i] : 0;  // (every range counts against total_len)
      nb = ok ? stream_blocks(states[i].pending, len) : 0;
      status[i] = ok ? (int32_t)LSM_OK : (int32_t)LSM_BAD_ARG;
    }
    const uint64_t incl = wave_incl_scan_u64(nb);
    const uint64_t lsum = wave_incl_scan_u64(len);
    if (lane == 63) atomicAdd(&bytes_s, (unsigned long long)lsum);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint64_t base = carry_s, tot = 0;
    for (uint32_t w = 0; w < 16; ++w) {
      base += w < wave ? wsum[w] : 0;
      tot += wsum[w];
    }
    if (i < n) bpre[i] = base + incl - nb;
    __syncthreads();
    if (tid == 0) carry_s += tot;
    __syncthreads();
  }
  if (tid == 0) bpre[n] = carry_s;
  // (uniform) a caller error: the ranges hold more bytes than total_len (or
  // more KiB blocks than the workspace was sized for): nothing is updated
  if (bytes_s > total_len || carry_s > cap_blocks) {
    for (uint32_t i = tid; i < n; i += 1024) status[i] = LSM_BAD_ARG;
    if (tid == 0) bpre[n] = 0;
  }
}

// B1: contributions of global KiB block g (state i = the last with bpre[i] <= g);
// a workgroup takes kBatchWgBlocks consecutive blocks, one state search each.
__global__ __launch_bounds__(256) void xxh3_batch_contrib_kernel(const Xxh3Stream* __restrict__ states, uint32_t n,
                                                                 const uint8_t* __restrict__ data,
                                                                 const uint64_t* __restrict__ off,
                                                                 const uint64_t* __restrict__ bpre,
                                                                 const int32_t* __restrict__ status,
                                                                 uint64_t* __restrict__ contrib) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = threadIdx.x >> 6;
  const int q = lane & 3, s = lane >> 2;
  const LongSecret* ls = &kLongSecret;
  const uint64_t k0 = ls->acc[s + 2 * q], k1 = ls->acc[s + 2 * q + 1];
  const uint64_t total = bpre[n];
  const uint64_t g0 = (uint64_t)blockIdx.x * kBatchWgBlocks;
  if (g0 >= total) return;
  // the state of block g0: last i with bpre[i] <= g0 (bpre[0] = 0)
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (bpre[mid] <= g0) lo = mid;
    else hi = mid;
  }
  uint32_t i = lo;
  const uint64_t g1 = min(total, g0 + kBatchWgBlocks);
  for (uint64_t g = g0 + wave; g < g1; g += 4) {
    while (bpre[i + 1] <= g) ++i;  // (states with no blocks are passed over)
    if (status[i] != LSM_OK) continue;  // (bad states have no blocks; defensive)
    const Xxh3Stream* st = states + i;
    const uint32_t pend = st->pending;
    const uint8_t* d = data + off[i];
    const uint64_t o = (g - bpre[i]) * 1024 + 16 * lane;  // offset in pending || data of state i
    const Win16 w = stream_window(st, pend, d, o);
    uint64_t c0 = 0, c1 = 0;
    stripe_part(w, k0, k1, c0, c1);
    c0 = quad_group_sum64(c0);
    c1 = quad_group_sum64(c1);
    if (lane < 4) {
      contrib[8 * g + 2 * q] = c0;
      contrib[8 * g + 2 * q + 1] = c1;
    }
  }
}

// B2: workgroup 8 i + k carries accumulator k of state i.
__global__ __launch_bounds__(64) void xxh3_batch_chain_kernel(Xxh3Stream* __restrict__ states,
                                                              const uint64_t* __restrict__ bpre,
                                                              const int32_t* __restrict__ status,
                                                              const uint64_t* __restrict__ contrib) {
  const uint32_t i = blockIdx.x >> 3, k = blockIdx.x & 7;
  if (status[i] != LSM_OK) return;
  const uint64_t nb = bpre[i + 1] - bpre[i];
  if (!nb) return;
  Xxh3Stream* st = states + i;
  const uint64_t x = xxh3_chain_wave(contrib + 8 * bpre[i], nb, k, st->acc[k], kLongSecret.acc[16 + k]);
  if (threadIdx.x == 0) st->acc[k] = x;
}

// B3: workgroup i = xxh3_stream_buffer_kernel for state i.
__global__ __launch_bounds__(512) void xxh3_batch_buffer_kernel(Xxh3Stream* __restrict__ states,
                                                                const uint8_t* __restrict__ data,
                                                                const uint64_t* __restrict__ off,
                                                                const int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x;
  if (status[i] != LSM_OK) return;  // (uniform)
  stream_buffer_wg(states + i, data + off[i], off[i + 1] - off[i]);
}

// KiB blocks the batch may consume, at most: sum over states of len_i / 1024 + 1.
static uint64_t batch_cap_blocks(uint32_t n, uint64_t total_len) { return total_len / 1024 + 2ULL * n; }

size_t xxh3_stream_batch_workspace_size(uint32_t n, uint64_t total_len) {
  return 8 * ((size_t)n + 1) + 256 + 64 * batch_cap_blocks(n, total_len) + 256;
}

hipError_t launch_xxh3_stream_update_batch(Xxh3Stream* states, uint32_t n, const uint8_t* data, const uint64_t* off,
                                           uint64_t total_len, int32_t* status, void* ws, hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t* bpre = (uint64_t*)ws;
  uint64_t* contrib = (uint64_t*)((uint8_t*)ws + ((8 * ((size_t)n + 1) + 255) & ~(size_t)255));
  const uint64_t cap = batch_cap_blocks(n, total_len);
  hipLaunchKernelGGL(xxh3_batch_plan_kernel, dim3(1), dim3(1024), 0, s, states, n, off, cap, total_len, bpre,
                     status);
  const uint64_t wgs = (cap + kBatchWgBlocks - 1) / kBatchWgBlocks;
  if (wgs > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(xxh3_batch_contrib_kernel, dim3((uint32_t)wgs), dim3(256), 0, s, states, n, data, off, bpre,
                     status, contrib);
  // (a 40 KiB LDS request: at most four chain workgroups per CU, so the 8 n
  // chains spread over the CUs' SIMDs instead of queueing on a few CUs)
  static uint64_t attr_done = 0;
  hipError_t e = set_lds_attr((const void*)xxh3_batch_chain_kernel, 40 * 1024, &attr_done);
  if (e != hipSuccess) return e;
  if ((uint64_t)n * 8 > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(xxh3_batch_chain_kernel, dim3(8 * n), dim3(64), 40 * 1024, s, states, bpre, status, contrib);
  hipLaunchKernelGGL(xxh3_batch_buffer_kernel, dim3(n), dim3(512), 0, s, states, data, off, status);
  return hipGetLastError();
}

__global__ __launch_bounds__(64) void xxh3_batch_digest_kernel(const Xxh3Stream* __restrict__ states,
                                                               uint64_t* __restrict__ out) {
  stream_digest_wave(states + blockIdx.x, out + 2 * blockIdx.x);
}

size_t xxh3_file_workspace_size(uint64_t len) { return sizeof(Xxh3Stream) + xxh3_stream_workspace_size(len); }

// One-shot whole-file checksum: a stream in the workspace, one update, digest.
hipError_t launch_xxh3_128_file(const uint8_t* data, uint64_t len, uint64_t* out, void* ws, hipStream_t s) {
  Xxh3Stream* st = (Xxh3Stream*)ws;
  uint64_t* contrib = (uint64_t*)((uint8_t*)ws + sizeof(Xxh3Stream));
  hipLaunchKernelGGL(xxh3_stream_init_kernel, dim3(1), dim3(64), 0, s, st);
  hipError_t e = launch_xxh3_stream_update(st, data, len, contrib, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(xxh3_stream_digest_kernel, dim3(1), dim3(64), 0, s, st, out);
  return hipGetLastError();
}

}  // namespace lsmgpu

extern "C" size_t lsm_xxh3_128_file_workspace_size(uint64_t len) { return lsmgpu::xxh3_file_workspace_size(len); }

extern "C" int lsm_xxh3_128_file(const uint8_t* d_data, uint64_t len, uint64_t* d_out, void* d_workspace,
                                 size_t workspace_bytes, void* stream) {
  if (!d_out || (len && !d_data)) return LSM_BAD_ARG;
  if (!d_workspace || ((uintptr_t)d_workspace & 15) || workspace_bytes < lsmgpu::xxh3_file_workspace_size(len))
    return LSM_BAD_ARG;
  const hipError_t e = lsmgpu::launch_xxh3_128_file(d_data, len, d_out, d_workspace, (hipStream_t)stream);
  return lsmgpu::hip_status(e, "lsm_xxh3_128_file");
}

extern "C" size_t lsm_xxh3_128_stream_state_size(void) { return sizeof(lsmgpu::Xxh3Stream); }

extern "C" int lsm_xxh3_128_stream_init(void* d_state, void* stream) {
  if (!d_state || ((uintptr_t)d_state & 15)) return LSM_BAD_ARG;
  hipLaunchKernelGGL(lsmgpu::xxh3_stream_init_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     (lsmgpu::Xxh3Stream*)d_state);
  return lsmgpu::hip_status(hipGetLastError(), "lsm_xxh3_128_stream_init");
}

extern "C" size_t lsm_xxh3_128_stream_workspace_size(uint64_t len) { return lsmgpu::xxh3_stream_workspace_size(len); }

extern "C" int lsm_xxh3_128_stream_update(void* d_state, const uint8_t* d_data, uint64_t len, void* d_workspace,
                                          size_t workspace_bytes, void* stream) {
  if (!d_state || ((uintptr_t)d_state & 15) || (len && !d_data)) return LSM_BAD_ARG;
  if (len && (!d_workspace || workspace_bytes < lsmgpu::xxh3_stream_workspace_size(len))) return LSM_BAD_ARG;
  const hipError_t e = lsmgpu::launch_xxh3_stream_update((lsmgpu::Xxh3Stream*)d_state, d_data, len,
                                                         (uint64_t*)d_workspace, (hipStream_t)stream);
  return lsmgpu::hip_status(e, "lsm_xxh3_128_stream_update");
}

extern "C" int lsm_xxh3_128_stream_digest(const void* d_state, uint64_t* d_out, void* stream) {
  if (!d_state || ((uintptr_t)d_state & 15) || !d_out) return LSM_BAD_ARG;
  hipLaunchKernelGGL(lsmgpu::xxh3_stream_digest_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     (const lsmgpu::Xxh3Stream*)d_state, d_out);
  return lsmgpu::hip_status(hipGetLastError(), "lsm_xxh3_128_stream_digest");
}

extern "C" int lsm_xxh3_128_stream_init_batch(void* d_states, uint32_t n, void* stream) {
  if (!n) return LSM_OK;
  if (!d_states || ((uintptr_t)d_states & 15)) return LSM_BAD_ARG;
  hipLaunchKernelGGL(lsmgpu::xxh3_stream_init_kernel, dim3(n), dim3(64), 0, (hipStream_t)stream,
                     (lsmgpu::Xxh3Stream*)d_states);
  return lsmgpu::hip_status(hipGetLastError(), "lsm_xxh3_128_stream_init_batch");
}

extern "C" size_t lsm_xxh3_128_stream_batch_workspace_size(uint32_t n, uint64_t total_len) {
  return lsmgpu::xxh3_stream_batch_workspace_size(n, total_len);
}

extern "C" int lsm_xxh3_128_stream_update_batch(void* d_states, uint32_t n, const uint8_t* d_data,
                                                const uint64_t* d_off, uint64_t total_len, int32_t* d_status,
                                                void* d_workspace, size_t workspace_bytes, void* stream) {
  if (!n) return LSM_OK;
  if (!d_states || ((uintptr_t)d_states & 15) || !d_off || !d_status || (total_len && !d_data)) return LSM_BAD_ARG;
  if (!d_workspace || ((uintptr_t)d_workspace & 15) ||
      workspace_bytes < lsmgpu::xxh3_stream_batch_workspace_size(n, total_len))
    return LSM_BAD_ARG;
  const hipError_t e = lsmgpu::launch_xxh3_stream_update_batch((lsmgpu::Xxh3Stream*)d_states, n, d_data, d_off,
                                                               total_len, d_status, d_workspace, (hipStream_t)stream);
  return lsmgpu::hip_status(e, "lsm_xxh3_128_stream_update_batch");
}

extern "C" int lsm_xxh3_128_stream_digest_batch(const void* d_states, uint32_t n, uint64_t* d_out, void* stream) {
  if (!n) return LSM_OK;
  if (!d_states || ((uintptr_t)d_states & 15) || !d_out) return LSM_BAD_ARG;
  hipLaunchKernelGGL(lsmgpu::xxh3_batch_digest_kernel, dim3(n), dim3(64), 0, (hipStream_t)stream,
                     (const lsmgpu::Xxh3Stream*)d_states, d_out);
  return lsmgpu::hip_status(hipGetLastError(), "lsm_xxh3_128_stream_digest_batch");
}
