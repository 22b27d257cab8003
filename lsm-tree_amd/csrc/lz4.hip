// lz4.hip — Block::from_reader / from_file for CompressionType::Lz4
// (src/table/block/mod.rs:87-128, :131-182): header checks, xxh3_128 verify of
// the stored (compressed) payload, then lz4_flex::decompress_into of the LZ4
// block format into header.uncompressed_length bytes (mod.rs:104-118).
//
// LZ4 decode is a serial chain of sequences, so the unit of parallelism is the
// block: one wave per block.  The wave stages the compressed payload into its
// own LDS slice (coalesced dword loads), every lane walks the token stream
// redundantly from LDS (wave-uniform control flow, broadcast reads), and the
// literal and match copies are spread over the 64 lanes inside an LDS output
// slice (a match with offset < 64 is copied in offset-sized rounds, so every
// source byte is already written).  The decoded block is then stored to HBM.
//   lz4_small_kernel  4 waves/workgroup, 5 KiB in + 5 KiB out per wave (the
//                     4 KiB data-block class; 4 workgroups = 16 waves per CU:
//                     160 -> 269 GiB/s over 8 KiB slices at 8 waves per CU).
//   lz4_large_kernel  1 wave/workgroup, 72 KiB in + 80 KiB out (16/64 KiB
//                     blocks); anything larger is decoded by lane 0 straight
//                     in HBM (rare: only oversize blocks).
#include <hip/hip_runtime.h>
#include "fill.hpp"

#include "block_format.hpp"
#include "decode.hpp"
#include "device_common.hpp"
#include "lsmgpu.h"
#include "scan.hpp"

namespace lsmgpu {

constexpr int32_t kLz4Deferred = -1;  // small kernel -> large kernel hand-off

// Wave-uniform LZ4 block decode from an LDS input slice (dword-staged, payload
// at byte `sh`, readable 8 bytes past its end) into an LDS output slice;
// returns the number of bytes written or -1 (Error::Decompress).  The parse
// chain is one 8-byte window read per sequence in the common case: the window
// read at a sequence's offset field also holds the next token.
__device__ __forceinline__ uint64_t lds_read8(const uint32_t* w, uint32_t p) {
  const uint32_t a = p >> 2, s = p & 3u;
  const uint32_t d0 = w[a], d1 = w[a + 1], d2 = w[a + 2];
  const uint32_t lo = s ? alignbyte(d1, d0, s) : d0, hi = s ? alignbyte(d2, d1, s) : d1;
  // wave-uniform by construction (every lane reads the same bytes): move it to
  // SGPRs so the walk's bounds checks and loops are scalar branches
  // (readfirstlane returns int: widen through uint32_t, or bit 31 of lo would sign-fill the high word)
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(lo) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(hi) << 32);
}

__device__ __forceinline__ uint32_t lds_read1(const uint8_t* in, uint32_t p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)in[p]);
}

__device__ __forceinline__ int64_t lz4_wave_decode(const uint32_t* lin, uint32_t sh, uint32_t n, uint8_t* out,
                                                   uint32_t cap, int lane) {
  const uint8_t* in = reinterpret_cast<const uint8_t*>(lin) + sh;
  uint32_t ip = 0, op = 0;
  if (n == 0) return -1;
  uint64_t win = lds_read8(lin, sh);  // bytes at ip
  for (;;) {
    if (ip >= n) return -1;
    const uint32_t token = (uint32_t)win & 0xFFu;
    uint32_t lit = token >> 4, hp = ip + 1;
    if (lit == 15) {
      uint32_t b;
      do {
        if (hp >= n) return -1;
        b = lds_read1(in, hp++);
        lit += b;
      } while (b == 255);
    }
    if (lit > n - hp || lit > cap - op) return -1;
    for (uint32_t j = lane; j < lit; j += 64) out[op + j] = in[hp + j];
    ip = hp + lit;
    op += lit;
    if (ip == n) return op;
    if (n - ip < 2) return -1;
    const uint64_t w2 = lds_read8(lin, sh + ip);  // offset, then (usually) the next token
    const uint32_t off = (uint32_t)w2 & 0xFFFFu;
    ip += 2;
    if (off == 0 || off > op) return -1;
    uint32_t ml = (token & 15u) + 4;
    if ((token & 15u) == 15) {
      uint32_t b;
      do {
        if (ip >= n) return -1;
        b = lds_read1(in, ip++);
        ml += b;
      } while (b == 255);
      win = lds_read8(lin, sh + ip);
    } else {
      win = w2 >> 16;
    }
    if (ml > cap - op) return -1;
    const uint32_t step = off < 64 ? off : 64;
    for (uint32_t c = 0; c < ml; c += step) {
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // previous round's bytes before this round's reads
      const uint32_t j = c + lane;
      if (lane < step && j < ml) out[op + j] = out[op + j - off];
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    op += ml;
  }
}

// Serial fallback for blocks larger than the LDS stages: lane 0, in HBM.
__device__ int64_t lz4_serial_decode(const uint8_t* in, uint64_t n, uint8_t* out, uint64_t cap) {
  uint64_t ip = 0, op = 0;
  if (n == 0) return -1;
  for (;;) {
    if (ip >= n) return -1;
    const uint32_t token = in[ip++];
    uint64_t lit = token >> 4;
    if (lit == 15) {
      uint32_t b;
      do {
        if (ip >= n) return -1;
        b = in[ip++];
        lit += b;
      } while (b == 255);
    }
    if (lit > n - ip || lit > cap - op) return -1;
    for (uint64_t j = 0; j < lit; ++j) out[op + j] = in[ip + j];
    ip += lit;
    op += lit;
    if (ip == n) return (int64_t)op;
    if (n - ip < 2) return -1;
    const uint64_t off = (uint64_t)in[ip] | ((uint64_t)in[ip + 1] << 8);
    ip += 2;
    if (off == 0 || off > op) return -1;
    uint64_t ml = (token & 15u) + 4;
    if ((token & 15u) == 15) {
      uint32_t b;
      do {
        if (ip >= n) return -1;
        b = in[ip++];
        ml += b;
      } while (b == 255);
    }
    if (ml > cap - op) return -1;
    for (uint64_t j = 0; j < ml; ++j) out[op + j] = out[op + j - off];
    op += ml;
  }
}

struct Lz4Block {
  const uint8_t* base;  // 16-aligned
  uint32_t hb;          // header position in base
  uint32_t data_len;
  uint32_t raw_len;
  uint8_t* dst;
};

// Header + payload checksum (Block::from_reader, mod.rs:92-102); wave-uniform.
// frame = 0 (payload only) or kHdrLen (lsm_lz4_decompress_framed: the payload
// follows a frame header written by lz4_write_frame_header).
__device__ __forceinline__ int32_t lz4_check_block(const uint8_t* blocks, const uint64_t* block_off, const uint64_t* out_off,
                                   uint8_t* out, uint32_t i, uint32_t frame, Lz4Block& b) {
  const uint64_t o = block_off[i], e = block_off[i + 1];
  b.base = blocks + (o & ~15ULL);
  b.hb = (uint32_t)(o & 15);
  HeaderInfo h;
  int32_t st = check_header(b.base, b.hb, e - o, h);
  if (st != ST_OK) return st;
  if ((uint64_t)h.data_length != e - o - kHdrLen) return ST_TRUNCATED;
  b.data_len = __builtin_amdgcn_readfirstlane(h.data_length);  // wave-uniform: keep the walk scalar
  b.raw_len = __builtin_amdgcn_readfirstlane(read_u32_unaligned(b.base, b.hb + 25));  // uncompressed_length, header.rs:101
  if ((uint64_t)b.raw_len + frame != out_off[i + 1] - out_off[i]) return ST_OVERFLOW;
  uint64_t lo, hi;
  xxh3_128_wave(b.base, b.hb + kHdrLen, b.data_len, &kLongSecret, lo, hi);
  if (lo != h.ck_lo || hi != h.ck_hi) return ST_CKSUM;
  b.dst = out + out_off[i] + frame;
  return ST_OK;
}

template <uint32_t kIn, uint32_t kOut>
__device__ __forceinline__ int32_t lz4_stage_and_decode(const Lz4Block& b, uint32_t* lin, uint8_t* lout, int lane) {
  // coalesced dword window [a0, a0 + 4*words) covering the payload
  const uint32_t p0 = b.hb + kHdrLen, a0 = p0 & ~3u, sh = p0 - a0;
  const uint32_t words = (sh + b.data_len + 3) / 4;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(b.base + a0);
  for (uint32_t w = lane; w < words; w += 64) lin[w] = src[w];
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const int64_t got = lz4_wave_decode(lin, sh, b.data_len, lout, kOut, lane);
  if (got != (int64_t)b.raw_len) return LSM_DECOMPRESS;
  // dword stores to HBM: head bytes up to the first aligned dword, then dwords
  // built from two aligned LDS dwords (alignbyte), then the tail bytes
  const uint32_t len = b.raw_len;
  uint32_t head = (4u - (uint32_t)((uintptr_t)b.dst & 3)) & 3u;
  if (head > len) head = len;
  if ((uint32_t)lane < head) b.dst[lane] = lout[lane];
  const uint32_t body = (len - head) >> 2, s = head & 3u;
  const uint32_t* l32 = reinterpret_cast<const uint32_t*>(lout);
  uint32_t* d32 = reinterpret_cast<uint32_t*>(b.dst + head);
  for (uint32_t w = lane; w < body; w += 64) {
    const uint32_t a = (head >> 2) + w;  // head < 4, so a = w; kept general
    d32[w] = s ? alignbyte(l32[a + 1], l32[a], s) : l32[a];
  }
  for (uint32_t j = head + 4 * body + lane; j < len; j += 64) b.dst[j] = lout[j];
  return ST_OK;
}

// Frame header of lsm_lz4_decompress_framed for block i (one lane): the
// stored header with data_length = uncompressed_length and the header checksum
// recomputed over the new first 29 bytes (header.rs:83-109), so the frame is a
// well-formed uncompressed block whose payload checksum field still names the
// stored bytes (decoded with LSM_DECODE_PAYLOAD_VERIFIED).  Written only once
// the block's decompression has succeeded; a block that failed (payload
// checksum, Error::Decompress, length mismatch) gets an all-zero frame header
// instead, so a decode of the frames reports BAD_MAGIC for it on its own even
// if the caller never merges the decompress statuses.  Blocks whose plan gave
// no frame (failed header) have nothing to write.
__device__ __forceinline__ void lz4_write_frame_header(const uint8_t* blocks, const uint64_t* block_off, uint32_t i,
                                                       uint8_t* out, const uint64_t* out_off, bool ok) {
  const uint64_t fo = out_off[i];
  if (out_off[i + 1] - fo < kHdrLen) return;
  uint32_t h[12] = {0};  // 29 header bytes + the readers' 12-byte over-read
  uint8_t* hp = reinterpret_cast<uint8_t*>(h);
  if (ok) {
    const uint64_t o = block_off[i];
    const uint8_t* base = blocks + (o & ~15ULL);
    const uint32_t hb = (uint32_t)(o & 15);
    for (uint32_t j = 0; j < 21; ++j) hp[j] = base[hb + j];  // magic, type, stored checksum
    const uint32_t ul = read_u32_unaligned(base, hb + 25);
    for (uint32_t j = 0; j < 4; ++j) hp[21 + j] = hp[25 + j] = (uint8_t)(ul >> (8 * j));
    uint64_t lo, hi;
    xxh3_128_short(29, BaseReader8{hp, 0}, BaseReader64{hp, 0}, lo, hi);
    for (uint32_t j = 0; j < 4; ++j) hp[29 + j] = (uint8_t)(lo >> (8 * j));
  }
  for (uint32_t j = 0; j < kHdrLen; ++j) out[fo + j] = hp[j];
}

constexpr uint32_t kSmallIn = 5120, kSmallOut = 5120;  // 40 KiB per 4-wave workgroup: 4 per CU
constexpr uint32_t kLargeIn = 72 * 1024, kLargeOut = 80 * 1024;

__global__ __launch_bounds__(256) void lz4_small_kernel(const uint8_t* __restrict__ blocks,
                                                        const uint64_t* __restrict__ block_off, uint32_t n,
                                                        uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off,
                                                        int32_t* __restrict__ status, uint32_t frame) {
  __shared__ uint32_t s_in[4][kSmallIn / 4];
  __shared__ uint8_t s_out[4][kSmallOut];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t i = blockIdx.x * 4 + wv;
  if (i >= n) return;
  Lz4Block b;
  int32_t st = lz4_check_block(blocks, block_off, out_off, out, i, frame, b);
  if (st == ST_OK) {
    const uint32_t sh = (b.hb + kHdrLen) & 3u;
    if (b.data_len + sh + 12 > kSmallIn || b.raw_len > kSmallOut)  // +12: dword window + 8-byte reads
      st = kLz4Deferred;
    else
      st = lz4_stage_and_decode<kSmallIn, kSmallOut>(b, s_in[wv], s_out[wv], lane);
  }
  if (lane == 0) {
    if (frame && st != kLz4Deferred) lz4_write_frame_header(blocks, block_off, i, out, out_off, st == ST_OK);
    status[i] = st;
  }
}

__global__ __launch_bounds__(64) void lz4_large_kernel(const uint8_t* __restrict__ blocks,
                                                       const uint64_t* __restrict__ block_off, uint32_t n,
                                                       uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off,
                                                       int32_t* __restrict__ status, const uint32_t* __restrict__ list,
                                                       const uint32_t* __restrict__ count, uint32_t frame) {
  extern __shared__ uint32_t s_dyn[];
  const int lane = threadIdx.x;
  const uint32_t total = *count;
  for (uint32_t li = blockIdx.x; li < total; li += gridDim.x) {
    const uint32_t i = list[li];
    Lz4Block b;
    int32_t st = lz4_check_block(blocks, block_off, out_off, out, i, frame, b);
    if (st == ST_OK) {
      const uint32_t sh = (b.hb + kHdrLen) & 3u;
      if (b.data_len + sh + 12 <= kLargeIn && b.raw_len <= kLargeOut) {
        st = lz4_stage_and_decode<kLargeIn, kLargeOut>(b, s_dyn, reinterpret_cast<uint8_t*>(s_dyn + kLargeIn / 4), lane);
      } else {
        int64_t got = 0;
        if (lane == 0) got = lz4_serial_decode(b.base + b.hb + kHdrLen, b.data_len, b.dst, b.raw_len);
        got = __shfl(got, 0);
        st = got == (int64_t)b.raw_len ? ST_OK : LSM_DECOMPRESS;
      }
    }
    if (lane == 0) {
      if (frame) lz4_write_frame_header(blocks, block_off, i, out, out_off, st == ST_OK);
      status[i] = st;
    }
  }
}

__global__ __launch_bounds__(256) void lz4_collect_deferred(int32_t* __restrict__ status, uint32_t n,
                                                            uint32_t* __restrict__ list, uint32_t* __restrict__ count) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n && status[i] == kLz4Deferred) list[atomicAdd(count, 1u)] = i;
}

// Output plan (lane per block): the uncompressed_length of every block whose
// header verifies (magic, type, header checksum, data_length == handle), as
// Block::from_reader only sizes its buffer after Header::decode_from has
// passed (block/mod.rs:91-112); 0 for a failing header or a length above the
// caller's cap (that block then reports its header status, or OVERFLOW).
__global__ __launch_bounds__(256) void lz4_plan_kernel(const uint8_t* __restrict__ blocks,
                                                       const uint64_t* __restrict__ block_off, uint32_t n,
                                                       uint64_t max_raw, uint32_t frame, uint64_t* __restrict__ raw) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t o = block_off[i], e = block_off[i + 1];
  const uint8_t* base = blocks + (o & ~15ULL);
  const uint32_t hb = (uint32_t)(o & 15);
  HeaderInfo h;
  uint64_t len = 0;
  if (e >= o && check_header(base, hb, e - o, h) == ST_OK && (uint64_t)h.data_length == e - o - kHdrLen) {
    len = read_u32_unaligned(base, hb + 25);  // uncompressed_length, header.rs:101
    len = len > max_raw ? 0 : len + frame;
  }
  raw[i] = len;
}

struct Lz4OffOut {
  uint64_t* off;
  __device__ void operator()(uint64_t i, uint64_t prefix) const { off[i] = prefix; }
};

// lsm_lz4_plan_capped: an output larger than the caller's arena leaves every
// range empty (each block whose header verifies then reports LSM_OVERFLOW).
// One workgroup: every thread reads the total before any range is cleared.
__global__ __launch_bounds__(1024) void lz4_cap_kernel(uint64_t* __restrict__ off, uint32_t n, uint64_t cap) {
  const bool over = off[n] > cap;
  __syncthreads();
  if (!over) return;
  for (uint64_t i = threadIdx.x; i <= n; i += 1024) off[i] = 0;
}

}  // namespace lsmgpu

using namespace lsmgpu;

extern "C" size_t lsm_lz4_plan_workspace_size(uint32_t n_blocks) {
  return ((size_t)n_blocks * 8 + 255) / 256 * 256 + (scan_tiles(n_blocks ? n_blocks : 1) * 8 + 255) / 256 * 256;
}

static int lz4_plan(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks, uint64_t max_block_bytes,
                    uint64_t* d_out_off, void* d_workspace, size_t workspace_bytes, void* stream, uint32_t frame) {
  if (n_blocks == 0) return LSM_OK;
  if (!d_blocks || !d_block_off || !d_out_off || !d_workspace || ((uintptr_t)d_blocks & 15) ||
      workspace_bytes < lsm_lz4_plan_workspace_size(n_blocks))
    return LSM_BAD_ARG;
  const hipStream_t st = (hipStream_t)stream;
  uint64_t* raw = (uint64_t*)d_workspace;
  uint64_t* tiles = (uint64_t*)((uint8_t*)d_workspace + ((size_t)n_blocks * 8 + 255) / 256 * 256);
  hipLaunchKernelGGL(lz4_plan_kernel, dim3((n_blocks + 255) / 256), dim3(256), 0, st, d_blocks, d_block_off, n_blocks,
                     max_block_bytes, frame, raw);
  hipError_t e = launch_excl_scan(raw, n_blocks, tiles, Lz4OffOut{d_out_off}, st);
  return hip_status(e != hipSuccess ? e : hipGetLastError(), "lsm_lz4_plan_output");
}

extern "C" size_t lsm_lz4_workspace_size(uint32_t n_blocks) { return 16 + (size_t)n_blocks * 4; }

extern "C" int lsm_lz4_plan_output(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                                   uint64_t max_block_bytes, uint64_t* d_out_off, void* d_workspace,
                                   size_t workspace_bytes, void* stream) {
  return lz4_plan(d_blocks, d_block_off, n_blocks, max_block_bytes, d_out_off, d_workspace, workspace_bytes, stream, 0);
}

extern "C" int lsm_lz4_plan_framed(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                                   uint64_t max_block_bytes, uint64_t* d_out_off, void* d_workspace,
                                   size_t workspace_bytes, void* stream) {
  return lz4_plan(d_blocks, d_block_off, n_blocks, max_block_bytes, d_out_off, d_workspace, workspace_bytes, stream,
                  kHdrLen);
}

extern "C" int lsm_lz4_plan_capped(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                                   uint64_t max_block_bytes, int framed, uint64_t out_cap, uint64_t* d_out_off,
                                   void* d_workspace, size_t workspace_bytes, void* stream) {
  const int rc = lz4_plan(d_blocks, d_block_off, n_blocks, max_block_bytes, d_out_off, d_workspace, workspace_bytes,
                          stream, framed ? kHdrLen : 0);
  if (rc != LSM_OK || n_blocks == 0) return rc;
  hipLaunchKernelGGL(lz4_cap_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, d_out_off, n_blocks, out_cap);
  return hip_status(hipGetLastError(), "lsm_lz4_plan_capped");
}

static int lz4_decompress(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks, uint8_t* d_out,
                          const uint64_t* d_out_off, int32_t* d_status, void* d_workspace, size_t workspace_bytes,
                          void* stream, uint32_t frame) {
  if (n_blocks == 0) return LSM_OK;
  if (!d_blocks || !d_block_off || !d_out || !d_out_off || !d_status || !d_workspace ||
      ((uintptr_t)d_blocks & 15) || workspace_bytes < lsm_lz4_workspace_size(n_blocks))
    return LSM_BAD_ARG;
  const hipStream_t st = (hipStream_t)stream;
  uint32_t* count = (uint32_t*)d_workspace;
  uint32_t* list = count + 4;
  hipError_t e = fill_words_async(count, 1, 0, st);
  if (e != hipSuccess) return hip_status(e, "lsm_lz4_decompress_blocks");
  hipLaunchKernelGGL(lz4_small_kernel, dim3((n_blocks + 3) / 4), dim3(256), 0, st, d_blocks, d_block_off, n_blocks,
                     d_out, d_out_off, d_status, frame);
  hipLaunchKernelGGL(lz4_collect_deferred, dim3((n_blocks + 255) / 256), dim3(256), 0, st, d_status, n_blocks, list,
                     count);
  static uint64_t attr_done = 0;
  if ((e = set_lds_attr((const void*)lz4_large_kernel, kLargeIn + kLargeOut, &attr_done)) != hipSuccess)
    return hip_status(e, "lsm_lz4_decompress_blocks");
  const uint32_t grid = n_blocks < 1024 ? n_blocks : 1024;
  hipLaunchKernelGGL(lz4_large_kernel, dim3(grid), dim3(64), kLargeIn + kLargeOut, st, d_blocks, d_block_off,
                     n_blocks, d_out, d_out_off, d_status, list, count, frame);
  return hip_status(hipGetLastError(), "lsm_lz4_decompress_blocks");
}

extern "C" int lsm_lz4_decompress_blocks(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                                         uint8_t* d_out, const uint64_t* d_out_off, int32_t* d_status,
                                         void* d_workspace, size_t workspace_bytes, void* stream) {
  return lz4_decompress(d_blocks, d_block_off, n_blocks, d_out, d_out_off, d_status, d_workspace, workspace_bytes,
                        stream, 0);
}

extern "C" int lsm_lz4_decompress_framed(const uint8_t* d_blocks, const uint64_t* d_block_off, uint32_t n_blocks,
                                         uint8_t* d_out, const uint64_t* d_out_off, int32_t* d_status,
                                         void* d_workspace, size_t workspace_bytes, void* stream) {
  return lz4_decompress(d_blocks, d_block_off, n_blocks, d_out, d_out_off, d_status, d_workspace, workspace_bytes,
                        stream, kHdrLen);
}
