// device_common.hpp — gfx950 device building blocks for the SST block codec.
//
// * XXH3-64 / XXH3-128 (seed 0, default secret): the per-lane short paths
//   (<= 240 B, used for the 29-byte header checksum, hash-index keys and tiny
//   payloads) and a WAVE-COOPERATIVE long path (> 240 B) for block payloads:
//   one 64-lane wave covers one 1 KiB XXH3 block per step (lane l owns bytes
//   [16l, 16l+16) = stripe l>>2, accumulator pair 2(l&3), 2(l&3)+1), the 16
//   stripe contributions are summed with a 4-step xor butterfly and every
//   lane applies the per-KiB scramble to its own accumulator pair.
//   Reference call sites: src/hash.rs:2-9, src/table/block/mod.rs:70,94,141,
//   src/table/block/header.rs:83-109, hash_index/mod.rs:35-41.
// * LEB128 (varint-rs) decoding from a 16-byte register window.
// * Unaligned 16-byte windows over LDS or global bytes (aligned dword reads +
//   v_alignbyte_b32), wave scans.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lds_dma.hpp"

namespace lsmgpu {

constexpr int kWave = 64;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Explicit global-address-space access.  Generic (flat) pointers compile to
// flat_load/flat_store, which count on lgkmcnt as well as vmcnt: every LDS
// wait after a flat store would also wait for the store to reach memory.
template <class T>
__device__ __forceinline__ void gstore(T* p, uint64_t i, T v) {
  ((__attribute__((address_space(1))) T*)p)[i] = v;
}
template <class T>
__device__ __forceinline__ T gload(const T* p, uint64_t i) {
  return ((const __attribute__((address_space(1))) T*)p)[i];
}
// A trivially copyable struct element by explicit global loads (gload cannot
// copy a struct through an address-space-qualified lvalue).
template <class T>
__device__ __forceinline__ T gload_pod(const T* p, uint64_t i) {
  static_assert(sizeof(T) % 8 == 0, "8-byte multiple");
  T r;
  const __attribute__((address_space(1))) uint64_t* src = (const __attribute__((address_space(1))) uint64_t*)(p + i);
  uint64_t* dst = reinterpret_cast<uint64_t*>(&r);
#pragma unroll
  for (uint32_t k = 0; k < sizeof(T) / 8; ++k) dst[k] = src[k];
  return r;
}
constexpr uint32_t kHdrLen = 33;
constexpr uint32_t kTrailerLen = 31;
constexpr uint8_t kTrailerMarker = 0xFF;
constexpr uint8_t kHashFree = 254;
constexpr uint8_t kHashConflict = 255;
constexpr uint32_t kHashMaxPointers = 254;

enum : int32_t {
  ST_OK = 0, ST_BAD_MAGIC = 1, ST_BAD_TYPE = 2, ST_HDR_CKSUM = 3, ST_CKSUM = 4, ST_PARSE = 5,
  ST_OVERFLOW = 6, ST_TYPE_MISMATCH = 7, ST_TRUNCATED = 8, ST_UNSUPPORTED = 9, ST_BAD_ARG = 10,
  ST_INCOMPLETE = 13  // LSM_INCOMPLETE: a streamed chain gave up waiting; the fallback pass re-verifies the block
};

// ---------------------------------------------------------------- XXH3 consts
constexpr uint32_t P32_1 = 0x9E3779B1U, P32_2 = 0x85EBCA77U, P32_3 = 0xC2B2AE3DU;

// One XXH3 accumulator step of the long loop's scramble (XXH3_scrambleAcc)
// after adding the KiB block's contribution c: x = a + c;
// ((x ^ (x >> 47)) ^ s) * PRIME32_1.  x >> 47 < 2^17 only touches the low
// word, and the multiply by a 32-bit prime is one 32x32+64 mad: a short
// dependent chain for the serial per-KiB scramble.
__host__ __device__ __forceinline__ uint64_t xxh3_scr(uint64_t a, uint64_t c, uint64_t s) {
  const uint64_t x = a + c;
  const uint32_t hi = (uint32_t)(x >> 32);
  const uint32_t lo = (uint32_t)x ^ (hi >> 15) ^ (uint32_t)s;
  const uint32_t hs = hi ^ (uint32_t)(s >> 32);
  return (uint64_t)lo * P32_1 + ((uint64_t)(hs * P32_1) << 32);
}
constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ULL, P64_2 = 0xC2B2AE3D27D4EB4FULL,
                   P64_3 = 0x165667B19E3779F9ULL, P64_4 = 0x85EBCA77C2B2AE63ULL,
                   P64_5 = 0x27D4EB2F165667C5ULL, PMX1 = 0x165667919E3779F9ULL,
                   PMX2 = 0x9FB21C651E98DF25ULL;

// The default 192-byte XXH3 secret as little-endian u64 at every byte offset
// the algorithm reads is obtained from this table with constant offsets only,
// so the compiler folds them into immediates.
struct Secret {
  static constexpr uint8_t b[192] = {
      0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
      0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
      0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
      0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
      0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
      0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
      0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
      0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
      0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
      0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
      0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
      0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
  };
  static constexpr uint64_t u64(int o) {
    return (uint64_t)b[o] | ((uint64_t)b[o + 1] << 8) | ((uint64_t)b[o + 2] << 16) |
           ((uint64_t)b[o + 3] << 24) | ((uint64_t)b[o + 4] << 32) | ((uint64_t)b[o + 5] << 40) |
           ((uint64_t)b[o + 6] << 48) | ((uint64_t)b[o + 7] << 56);
  }
  static constexpr uint32_t u32(int o) {
    return (uint32_t)b[o] | ((uint32_t)b[o + 1] << 8) | ((uint32_t)b[o + 2] << 16) |
           ((uint32_t)b[o + 3] << 24);
  }
};

// Secret words for the wave long path (runtime-indexed -> constant memory).
struct LongSecret {
  uint64_t acc[24];   // u64 at byte 8j, j = 0..23 (stripe keys: stripe s, acc i -> acc[s+i])
  uint64_t last[8];   // u64 at byte 121 + 8i (last stripe, XXH_SECRET_LASTACC_START = 7)
  uint64_t mlo[8];    // u64 at byte 11 + 8i  (mergeAccs low)
  uint64_t mhi[8];    // u64 at byte 117 + 8i (mergeAccs high)
};
constexpr LongSecret make_long_secret() {
  LongSecret ls{};
  for (int j = 0; j < 24; ++j) ls.acc[j] = Secret::u64(8 * j);
  for (int i = 0; i < 8; ++i) {
    ls.last[i] = Secret::u64(121 + 8 * i);
    ls.mlo[i] = Secret::u64(11 + 8 * i);
    ls.mhi[i] = Secret::u64(117 + 8 * i);
  }
  return ls;
}
// One copy per translation unit (no -fgpu-rdc).
static __constant__ LongSecret kLongSecret = make_long_secret();

__device__ __forceinline__ uint64_t mul_fold64(uint64_t a, uint64_t b) {
  return (a * b) ^ __umul64hi(a, b);
}
__device__ __forceinline__ uint64_t xxh64_avalanche(uint64_t h) {
  h ^= h >> 33; h *= P64_2; h ^= h >> 29; h *= P64_3; h ^= h >> 32;
  return h;
}
__device__ __forceinline__ uint64_t xxh3_avalanche(uint64_t h) {
  h ^= h >> 37; h *= PMX1; h ^= h >> 32;
  return h;
}
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

// ------------------------------------------------- byte access (LDS / global)
// `base` is 16-byte aligned (an LDS image base or a global span base); all
// reads are aligned dwords, unaligned views are assembled with v_alignbyte.
__device__ __forceinline__ uint32_t ld32(const uint8_t* base, uint32_t aligned_off) {
  return *reinterpret_cast<const uint32_t*>(base + aligned_off);
}
__device__ __forceinline__ uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t shift) {
  return __builtin_amdgcn_alignbyte(hi, lo, shift);
}
__device__ __forceinline__ uint8_t ld8(const uint8_t* base, uint32_t off) { return base[off]; }

struct Win16 {
  uint64_t lo, hi;
};
// 16 bytes at base[pos..pos+16) (reads up to 4 bytes past pos+16).
__device__ __forceinline__ Win16 read_win16(const uint8_t* base, uint32_t pos) {
  const uint32_t a = pos & ~3u, s = pos & 3u;
  uint32_t d0 = ld32(base, a), d1 = ld32(base, a + 4), d2 = ld32(base, a + 8),
           d3 = ld32(base, a + 12), d4 = ld32(base, a + 16);
  uint32_t e0 = alignbyte(d1, d0, s), e1 = alignbyte(d2, d1, s), e2 = alignbyte(d3, d2, s),
           e3 = alignbyte(d4, d3, s);
  return {(uint64_t)e0 | ((uint64_t)e1 << 32), (uint64_t)e2 | ((uint64_t)e3 << 32)};
}
// read_win16 with the dword-aligned offset a and the shift s split out, for
// loops that step a window by whole dwords: a + constant folds into the
// ds_read offsets, and the alignment is computed once per loop, not per window.
__device__ __forceinline__ Win16 read_win16_split(const uint8_t* base, uint32_t a, uint32_t s) {
  const uint32_t d0 = ld32(base, a), d1 = ld32(base, a + 4), d2 = ld32(base, a + 8), d3 = ld32(base, a + 12),
                 d4 = ld32(base, a + 16);
  return {(uint64_t)alignbyte(d1, d0, s) | ((uint64_t)alignbyte(d2, d1, s) << 32),
          (uint64_t)alignbyte(d3, d2, s) | ((uint64_t)alignbyte(d4, d3, s) << 32)};
}
// The same from an LDS pointer (explicit address space: ds_read even where
// the compiler cannot tell that a generic pointer is LDS).
__device__ __forceinline__ Win16 read_win16_lds(const uint8_t* base_generic, uint32_t pos) {
  const __attribute__((address_space(3))) uint32_t* b =
      (const __attribute__((address_space(3))) uint32_t*)(const __attribute__((address_space(3))) uint8_t*)base_generic;
  const uint32_t a = pos >> 2, s = pos & 3u;
  const uint32_t d0 = b[a], d1 = b[a + 1], d2 = b[a + 2], d3 = b[a + 3], d4 = b[a + 4];
  return {(uint64_t)alignbyte(d1, d0, s) | ((uint64_t)alignbyte(d2, d1, s) << 32),
          (uint64_t)alignbyte(d3, d2, s) | ((uint64_t)alignbyte(d4, d3, s) << 32)};
}
__device__ __forceinline__ uint32_t read_u32_unaligned(const uint8_t* base, uint32_t pos) {
  const uint32_t a = pos & ~3u, s = pos & 3u;
  return alignbyte(ld32(base, a + 4), ld32(base, a), s);
}
__device__ __forceinline__ uint64_t read_u64_unaligned(const uint8_t* base, uint32_t pos) {
  const uint32_t a = pos & ~3u, s = pos & 3u;
  const uint32_t d0 = ld32(base, a), d1 = ld32(base, a + 4), d2 = ld32(base, a + 8);
  return (uint64_t)alignbyte(d1, d0, s) | ((uint64_t)alignbyte(d2, d1, s) << 32);
}
__device__ __forceinline__ uint16_t read_u16_unaligned(const uint8_t* base, uint32_t pos) {
  return (uint16_t)(read_u32_unaligned(base, pos) & 0xFFFF);
}

// Drop the low n bytes (0 <= n <= 16) of a 128-bit window.
__device__ __forceinline__ void win_shift(Win16& w, uint32_t n) {
  if (n >= 16) {
    w.lo = w.hi = 0;
    return;
  }
  if (n >= 8) {
    w.lo = w.hi;
    w.hi = 0;
    n -= 8;
  }
  if (n) {
    w.lo = (w.lo >> (8 * n)) | (w.hi << (64 - 8 * n));
    w.hi >>= 8 * n;
  }
}

// LEB128 (varint-rs VarintReader) from the low bytes of a window.
// Returns the byte length (1..max_bytes) or 0 if the varint does not
// terminate within min(max_bytes, avail) bytes.  Value is truncated to the
// type width by the caller's mask (`as $type` in varint-rs).
__device__ __forceinline__ uint32_t leb_decode(const Win16& w, uint32_t max_bytes, uint32_t avail,
                                                uint64_t& v) {
  const uint64_t msb = 0x8080808080808080ULL;
  uint64_t stop = ~w.lo & msb;
  uint32_t n;
  if (stop) {
    n = (uint32_t)(__builtin_ctzll(stop) >> 3) + 1;  // 1..8
  } else {
    uint64_t stop2 = ~w.hi & 0x8080ULL;              // bytes 9, 10
    n = stop2 ? 9 + (uint32_t)(__builtin_ctzll(stop2) >> 3) : 99;
  }
  if (n > max_bytes || n > avail) return 0;
  uint64_t x = w.lo;
  if (n < 8) x &= (1ULL << (8 * n)) - 1;
  // compact 7-bit groups: 8 x 7 -> 56 bits
  x = ((x & 0x7F007F007F007F00ULL) >> 1) | (x & 0x007F007F007F007FULL);
  x = ((x & 0x3FFF00003FFF0000ULL) >> 2) | (x & 0x00003FFF00003FFFULL);
  x = ((x & 0x0FFFFFFF00000000ULL) >> 4) | (x & 0x000000000FFFFFFFULL);
  if (n > 8) {
    x |= (w.hi & 0x7FULL) << 56;
    if (n > 9) x |= (w.hi & 0x7F00ULL) << 55;  // bits 63..69 (only bit 63 survives)
  }
  v = x;
  return n;
}

// ------------------------------------------------- XXH3 per-lane short paths
// Input bytes come from a caller-supplied reader R: R(off) -> u64 at byte off
// (unaligned little-endian), R8(off) -> byte.
template <class R8, class R64>
__device__ __forceinline__ void xxh3_128_short(uint32_t len, R8 rb, R64 r64, uint64_t& out_lo,
                                               uint64_t& out_hi) {
  using S = Secret;
  if (len == 0) {
    out_lo = xxh64_avalanche(S::u64(64) ^ S::u64(72));
    out_hi = xxh64_avalanche(S::u64(80) ^ S::u64(88));
    return;
  }
  if (len <= 3) {
    uint32_t c1 = rb(0), c2 = rb(len >> 1), c3 = rb(len - 1);
    uint32_t cl = (c1 << 16) | (c2 << 24) | c3 | (len << 8);
    uint32_t ch = rotl32(bswap32(cl), 13);
    out_lo = xxh64_avalanche((uint64_t)cl ^ (uint64_t)(S::u32(0) ^ S::u32(4)));
    out_hi = xxh64_avalanche((uint64_t)ch ^ (uint64_t)(S::u32(8) ^ S::u32(12)));
    return;
  }
  if (len <= 8) {
    uint32_t in_lo = (uint32_t)r64(0), in_hi = (uint32_t)r64(len - 4);
    uint64_t keyed = (in_lo + ((uint64_t)in_hi << 32)) ^ (S::u64(16) ^ S::u64(24));
    uint64_t m = P64_1 + ((uint64_t)len << 2);
    uint64_t lo = keyed * m, hi = __umul64hi(keyed, m);
    hi += lo << 1;
    lo ^= hi >> 3;
    lo ^= lo >> 35;
    lo *= PMX2;
    lo ^= lo >> 28;
    out_lo = lo;
    out_hi = xxh3_avalanche(hi);
    return;
  }
  if (len <= 16) {
    uint64_t in_lo = r64(0), in_hi = r64(len - 8);
    uint64_t k = in_lo ^ in_hi ^ (S::u64(32) ^ S::u64(40));
    uint64_t mlo = k * P64_1, mhi = __umul64hi(k, P64_1);
    mlo += (uint64_t)(len - 1) << 54;
    in_hi ^= S::u64(48) ^ S::u64(56);
    mhi += in_hi + (uint64_t)(uint32_t)in_hi * (uint64_t)(P32_2 - 1);
    mlo ^= bswap64(mhi);
    uint64_t hlo = mlo * P64_2, hhi = __umul64hi(mlo, P64_2);
    hhi += mhi * P64_2;
    out_lo = xxh3_avalanche(hlo);
    out_hi = xxh3_avalanche(hhi);
    return;
  }
  auto mix16 = [&](uint32_t io, int so, uint64_t seed) {
    return mul_fold64(r64(io) ^ (S::u64(so) + seed), r64(io + 8) ^ (S::u64(so + 8) - seed));
  };
  uint64_t alo = (uint64_t)len * P64_1, ahi = 0;
  auto mix32 = [&](uint32_t i1, uint32_t i2, int so, uint64_t seed) {
    alo += mix16(i1, so, seed);
    alo ^= r64(i2) + r64(i2 + 8);
    ahi += mix16(i2, so + 16, seed);
    ahi ^= r64(i1) + r64(i1 + 8);
  };
  if (len <= 128) {
    if (len > 32) {
      if (len > 64) {
        if (len > 96) mix32(48, len - 64, 96, 0);
        mix32(32, len - 48, 64, 0);
      }
      mix32(16, len - 32, 32, 0);
    }
    mix32(0, len - 16, 0, 0);
  } else {  // 129..240
#pragma unroll
    for (int i = 32; i < 160; i += 32) mix32(i - 32, i - 16, i - 32, 0);
    alo = xxh3_avalanche(alo);
    ahi = xxh3_avalanche(ahi);
#pragma unroll
    for (int i = 160; i <= 240; i += 32)
      if ((uint32_t)i <= len) mix32(i - 32, i - 16, 3 + i - 160, 0);
    mix32(len - 16, len - 32, 136 - 17 - 16, 0);
  }
  uint64_t hlo = alo + ahi;
  uint64_t hhi = alo * P64_1 + ahi * P64_4 + (uint64_t)len * P64_2;
  out_lo = xxh3_avalanche(hlo);
  out_hi = 0 - xxh3_avalanche(hhi);
}

// XXH3-64 of 0..16 bytes (reads offsets < len only, r64 at offsets <= 8).
template <class R8, class R64>
__device__ __forceinline__ uint64_t xxh3_64_le16(uint32_t len, R8 rb, R64 r64) {
  using S = Secret;
  if (len == 0) return xxh64_avalanche(S::u64(56) ^ S::u64(64));
  if (len <= 3) {
    uint32_t c1 = rb(0), c2 = rb(len >> 1), c3 = rb(len - 1);
    uint32_t combined = (c1 << 16) | (c2 << 24) | c3 | (len << 8);
    return xxh64_avalanche((uint64_t)combined ^ (uint64_t)(S::u32(0) ^ S::u32(4)));
  }
  if (len <= 8) {
    uint32_t in1 = (uint32_t)r64(0), in2 = (uint32_t)r64(len - 4);
    uint64_t h = (in2 + ((uint64_t)in1 << 32)) ^ (S::u64(8) ^ S::u64(16));
    h ^= rotl64(h, 49) ^ rotl64(h, 24);
    h *= PMX2;
    h ^= (h >> 35) + len;
    h *= PMX2;
    return h ^ (h >> 28);
  }
  if (len <= 16) {
    uint64_t lo = r64(0) ^ (S::u64(24) ^ S::u64(32));
    uint64_t hi = r64(len - 8) ^ (S::u64(40) ^ S::u64(48));
    uint64_t acc = len + bswap64(lo) + hi + mul_fold64(lo, hi);
    return xxh3_avalanche(acc);
  }
  return 0;  // (len > 16: not this function's range)
}
// Readers over a 16-byte register window (the key's first 16 bytes).
struct WinReader8 {
  uint64_t lo, hi;
  __device__ __forceinline__ uint32_t operator()(uint32_t o) const {
    return (uint32_t)((o < 8 ? lo >> (8 * o) : hi >> (8 * (o - 8))) & 0xFF);
  }
};
struct WinReader64 {  // o <= 8
  uint64_t lo, hi;
  __device__ __forceinline__ uint64_t operator()(uint32_t o) const {
    return o == 0 ? lo : o >= 8 ? hi : (lo >> (8 * o)) | (hi << (64 - 8 * o));
  }
};

template <class R8, class R64>
__device__ __forceinline__ uint64_t xxh3_64_short(uint32_t len, R8 rb, R64 r64) {
  using S = Secret;
  if (len <= 16) return xxh3_64_le16(len, rb, r64);
  auto mix16 = [&](uint32_t io, int so) {
    return mul_fold64(r64(io) ^ S::u64(so), r64(io + 8) ^ S::u64(so + 8));
  };
  uint64_t acc = (uint64_t)len * P64_1;
  if (len <= 128) {
    if (len > 32) {
      if (len > 64) {
        if (len > 96) {
          acc += mix16(48, 96);
          acc += mix16(len - 64, 112);
        }
        acc += mix16(32, 64);
        acc += mix16(len - 48, 80);
      }
      acc += mix16(16, 32);
      acc += mix16(len - 32, 48);
    }
    acc += mix16(0, 0);
    acc += mix16(len - 16, 16);
    return xxh3_avalanche(acc);
  }
  // 129..240
#pragma unroll
  for (int i = 0; i < 8; ++i) acc += mix16(16 * i, 16 * i);
  acc = xxh3_avalanche(acc);
  const uint32_t rounds = len / 16;
#pragma unroll
  for (int i = 8; i < 15; ++i)
    if ((uint32_t)i < rounds) acc += mix16(16 * i, 16 * (i - 8) + 3);
  acc += mix16(len - 16, 136 - 17);
  return xxh3_avalanche(acc);
}

// Generic byte reader over a (possibly unaligned) byte pointer, for per-lane
// hashing of keys in global memory (hash index) — byte loads, any alignment.
struct PtrReader {
  const uint8_t* p;
  __device__ __forceinline__ uint32_t operator()(uint32_t o) const { return p[o]; }
};
struct PtrReader64 {
  const uint8_t* p;
  __device__ __forceinline__ uint64_t operator()(uint32_t o) const {
    uint64_t v = 0;
#pragma unroll
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[o + i];
    return v;
  }
};


// ------------------------------------------------- XXH3-128 wave long path
// 16 bytes of the input at byte offset o (relative to the aligned base),
// with input start alignment folded in: see read_win16.
struct WaveHashState {
  uint64_t a0, a1;  // accumulators 2(l&3), 2(l&3)+1 (every lane of a quad group holds them)
};

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int mask) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  lo = __shfl_xor((int)lo, mask);
  hi = __shfl_xor((int)hi, mask);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// Contribution of one 16-byte chunk (lane's part of a stripe) to its pair.
__device__ __forceinline__ void stripe_part(const Win16& w, uint64_t k0, uint64_t k1, uint64_t& c0,
                                            uint64_t& c1) {
  uint64_t x0 = w.lo ^ k0, x1 = w.hi ^ k1;
  c0 += (uint64_t)(uint32_t)x0 * (x0 >> 32) + w.hi;  // acc[w0] += mul(k0) ; acc[w0] (=w1^1) += v1
  c1 += (uint64_t)(uint32_t)x1 * (x1 >> 32) + w.lo;  // acc[w1] += mul(k1) ; acc[w1] (=w0^1) += v0
}

// Sum of v over the 16 lanes that share (lane & 3): two DPP row rotates
// (within each 16-lane row) + gfx950 v_permlane16_swap / v_permlane32_swap
// (across rows) — all VALU, no LDS round trips.
// (row rotates and quad perms read an in-range lane for every lane, so the
// bound-control form needs no zeroed "old" operand: one VALU per move, not two)
__device__ __forceinline__ uint32_t dpp_ror4(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x124, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_ror8(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, true);
}
__device__ __forceinline__ uint64_t quad_group_sum64(uint64_t v) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  v += (uint64_t)dpp_ror4(lo) | ((uint64_t)dpp_ror4(hi) << 32);
  lo = (uint32_t)v; hi = (uint32_t)(v >> 32);
  v += (uint64_t)dpp_ror8(lo) | ((uint64_t)dpp_ror8(hi) << 32);
  lo = (uint32_t)v; hi = (uint32_t)(v >> 32);
  {
    const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    v = ((uint64_t)a[0] | ((uint64_t)b[0] << 32)) + ((uint64_t)a[1] | ((uint64_t)b[1] << 32));
  }
  lo = (uint32_t)v; hi = (uint32_t)(v >> 32);
  {
    const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    v = ((uint64_t)a[0] | ((uint64_t)b[0] << 32)) + ((uint64_t)a[1] | ((uint64_t)b[1] << 32));
  }
  return v;
}

// XXH3-128 of base[pos .. pos+len), len > 240, computed by the whole wave
// (all 64 lanes must call it with identical arguments).  `base` 16-aligned.
__device__ __forceinline__ void xxh3_128_wave_long(const uint8_t* base, uint32_t pos, uint32_t len,
                                                   const LongSecret* __restrict__ ls, uint64_t& out_lo,
                                                   uint64_t& out_hi) {
  const int lane = threadIdx.x & 63;
  const int q = lane & 3;          // accumulator pair index
  const int s = lane >> 2;         // stripe in block
  const uint64_t k0 = ls->acc[s + 2 * q], k1 = ls->acc[s + 2 * q + 1];
  // XXH3 initial accumulators {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1}
  uint64_t a0 = q == 0 ? (uint64_t)P32_3 : q == 1 ? P64_2 : q == 2 ? P64_4 : P64_5;
  uint64_t a1 = q == 0 ? P64_1 : q == 1 ? P64_3 : q == 2 ? (uint64_t)P32_2 : (uint64_t)P32_1;
  const uint64_t scr0 = ls->acc[16 + 2 * q], scr1 = ls->acc[16 + 2 * q + 1];  // secret + 128
  const uint32_t nb_blocks = (len - 1) / 1024;
  // The per-KiB contributions do not depend on the accumulators, so two
  // KiB blocks are loaded and reduced together; only the scramble is serial.
  uint32_t n = 0;
  const uint32_t la = (pos + 16 * lane) & ~3u, lsh = (pos + 16 * lane) & 3u;  // (one shift for every window)
  for (; n + 2 <= nb_blocks; n += 2) {
    const Win16 wa = read_win16_split(base, la + n * 1024, lsh);
    const Win16 wb = read_win16_split(base, la + n * 1024 + 1024, lsh);
    uint64_t c0 = 0, c1 = 0, d0 = 0, d1 = 0;
    stripe_part(wa, k0, k1, c0, c1);
    stripe_part(wb, k0, k1, d0, d1);
    c0 = quad_group_sum64(c0);
    c1 = quad_group_sum64(c1);
    d0 = quad_group_sum64(d0);
    d1 = quad_group_sum64(d1);
    a0 = xxh3_scr(a0, c0, scr0);
    a1 = xxh3_scr(a1, c1, scr1);
    a0 = xxh3_scr(a0, d0, scr0);
    a1 = xxh3_scr(a1, d1, scr1);
  }
  if (n < nb_blocks) {
    const Win16 w = read_win16_split(base, la + n * 1024, lsh);
    uint64_t c0 = 0, c1 = 0;
    stripe_part(w, k0, k1, c0, c1);
    c0 = quad_group_sum64(c0);
    c1 = quad_group_sum64(c1);
    a0 = xxh3_scr(a0, c0, scr0);
    a1 = xxh3_scr(a1, c1, scr1);
  }
  {
    const uint32_t tail0 = nb_blocks * 1024;
    const uint32_t nb_stripes = ((len - 1) - tail0) / 64;
    uint64_t c0 = 0, c1 = 0;
    if ((uint32_t)s < nb_stripes) {
      Win16 w = read_win16(base, pos + tail0 + 16 * lane);
      stripe_part(w, k0, k1, c0, c1);
    }
    if (lane < 4) {  // last stripe: input[len-64 .. len), secret + 121
      Win16 w = read_win16(base, pos + len - 64 + 16 * lane);
      stripe_part(w, ls->last[2 * q], ls->last[2 * q + 1], c0, c1);
    }
    a0 += quad_group_sum64(c0);
    a1 += quad_group_sum64(c1);
  }
  // mergeAccs: lane pair q holds acc[2q], acc[2q+1]
  uint64_t tlo = mul_fold64(a0 ^ ls->mlo[2 * q], a1 ^ ls->mlo[2 * q + 1]);
  uint64_t thi = mul_fold64(a0 ^ ls->mhi[2 * q], a1 ^ ls->mhi[2 * q + 1]);
  tlo += shfl_xor64(tlo, 1);
  thi += shfl_xor64(thi, 1);
  tlo += shfl_xor64(tlo, 2);
  thi += shfl_xor64(thi, 2);
  out_lo = xxh3_avalanche((uint64_t)len * P64_1 + tlo);
  out_hi = xxh3_avalanche(~((uint64_t)len * P64_2) + thi);
}

__device__ __forceinline__ uint64_t u64_of(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }
// Lanes with lane bit `bit` clear keep a's sum over the lane pair (lane, lane ^ 2^bit),
// the others b's (bit 5: v_permlane32_swap, bit 4: v_permlane16_swap).
template <int kBit>
__device__ __forceinline__ uint64_t pair_swap_sum64(uint64_t a, uint64_t b) {
  const uint32_t alo = (uint32_t)a, ahi = (uint32_t)(a >> 32), blo = (uint32_t)b, bhi = (uint32_t)(b >> 32);
  if constexpr (kBit == 5) {
    const auto l = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
    return u64_of(l[0], h[0]) + u64_of(l[1], h[1]);
  } else {
    const auto l = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
    return u64_of(l[0], h[0]) + u64_of(l[1], h[1]);
  }
}

// XXH3 contributions of cnt <= kB (4 or 8) KiB blocks n0 .. n0 + cnt - 1 of
// base[pos ..] (kLds: an LDS image, else HBM) by one wave (lane l: bytes [16 l, 16 l + 16) of each, stripe
// l >> 2, accumulator pair l & 3) into contrib[8 n ..].  The 16-lane sums of
// all of them as one reduce-scatter: lane bits 5 and 4 by permlane32 /
// permlane16 swaps (each halves the values a lane holds), then DPP row
// rotates (kB = 8: bit 3 a scatter, bit 2 a sum; kB = 4: both sums): about
// 10 VALU per KiB block against 32 for a quad_group_sum64 pair.
template <int kB, bool kLds, bool kAgent = false>
__device__ __forceinline__ void xxh3_kib_contribs_b(const uint8_t* base, uint32_t pos, uint32_t n0, uint32_t cnt,
                                                    uint64_t k0, uint64_t k1, uint64_t* contrib) {
  static_assert(kB == 4 || kB == 8, "batch");
  const int lane = threadIdx.x & 63, q = lane & 3;
  uint64_t c0[kB], c1[kB];
#pragma unroll
  for (int j = 0; j < kB; ++j) {
    c0[j] = c1[j] = 0;
    if ((uint32_t)j < cnt) {
      const uint32_t at = pos + (n0 + j) * 1024 + 16 * lane;
      const Win16 w = kLds ? read_win16_lds(base, at) : read_win16(base, at);
      stripe_part(w, k0, k1, c0[j], c1[j]);
    }
  }
  constexpr int h5 = kB / 2, h4 = kB / 4;
#pragma unroll
  for (int j = 0; j < h5; ++j) {  // lanes with bit 5 set keep block j + h5
    c0[j] = pair_swap_sum64<5>(c0[j], c0[j + h5]);
    c1[j] = pair_swap_sum64<5>(c1[j], c1[j + h5]);
  }
#pragma unroll
  for (int j = 0; j < h4; ++j) {  // bit 4 set: j + h4
    c0[j] = pair_swap_sum64<4>(c0[j], c0[j + h4]);
    c1[j] = pair_swap_sum64<4>(c1[j], c1[j + h4]);
  }
  uint64_t x0, x1;
  uint32_t n;
  if constexpr (kB == 8) {  // bit 3 set: block 1 of the remaining two
    const bool b3 = (lane & 8) != 0;
    auto lvl3 = [&](uint64_t a, uint64_t b) {
      const uint64_t keep = b3 ? b : a, send = b3 ? a : b;
      return keep + u64_of(dpp_ror8((uint32_t)send), dpp_ror8((uint32_t)(send >> 32)));
    };
    x0 = lvl3(c0[0], c0[1]);
    x1 = lvl3(c1[0], c1[1]);
    n = ((lane >> 5) & 1) * 4 + ((lane >> 4) & 1) * 2 + ((lane >> 3) & 1);
  } else {
    x0 = c0[0] + u64_of(dpp_ror8((uint32_t)c0[0]), dpp_ror8((uint32_t)(c0[0] >> 32)));
    x1 = c1[0] + u64_of(dpp_ror8((uint32_t)c1[0]), dpp_ror8((uint32_t)(c1[0] >> 32)));
    n = ((lane >> 5) & 1) * 2 + ((lane >> 4) & 1);
  }
  // (row_ror:4 hands lane i the value of lane i - 4 of its row: the partner for lanes with bit 2 set)
  x0 += u64_of(dpp_ror4((uint32_t)x0), dpp_ror4((uint32_t)(x0 >> 32)));
  x1 += u64_of(dpp_ror4((uint32_t)x1), dpp_ror4((uint32_t)(x1 >> 32)));
  const bool st = kB == 8 ? (lane & 4) != 0 : (lane & 12) == 4;
  if (st && n < cnt) {
    if (kAgent) {  // agent-scope stores (written through the XCD's L2): read by another XCD in this launch
      __hip_atomic_store(&contrib[8 * (uint64_t)(n0 + n) + 2 * q], x0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&contrib[8 * (uint64_t)(n0 + n) + 2 * q + 1], x1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      contrib[8 * (uint64_t)(n0 + n) + 2 * q] = x0;
      contrib[8 * (uint64_t)(n0 + n) + 2 * q + 1] = x1;
    }
  }
}

// XXH3-128 long path split across the waves of a workgroup.  The per-KiB
// contributions of the accumulate loop do not depend on the accumulators, so
// wave w of nw reduces runs of B = 4 consecutive KiB blocks (starting at B w,
// B (w + nw), ...) into contrib[8 n ..]; after a workgroup barrier one wave
// runs the serial scramble chain over them and the tail
// (xxh3_128_wave_finish).  len > 240; kLds: base is LDS.  With `ready`, KiB block n's
// contribution is published to a concurrent xxh3_128_wave_finish by
// ready[n] = tag (LDS, workgroup release).
template <bool kLds = true, bool kAgent = false>
__device__ __forceinline__ void xxh3_kib_contribs(const uint8_t* base, uint32_t pos, uint32_t len,
                                                  const LongSecret* __restrict__ ls, uint64_t* contrib, uint32_t w,
                                                  uint32_t nw, uint32_t* ready = nullptr, uint32_t tag = 0) {
  const int lane = threadIdx.x & 63;
  const int q = lane & 3, s = lane >> 2;
  const uint64_t k0 = ls->acc[s + 2 * q], k1 = ls->acc[s + 2 * q + 1];
  const uint32_t nb_blocks = (len - 1) / 1024;
  constexpr uint32_t B = 4;
  for (uint32_t n0 = B * w; n0 < nb_blocks; n0 += B * nw) {
    const uint32_t cnt = min(B, nb_blocks - n0);
    xxh3_kib_contribs_b<B, kLds, kAgent>(base, pos, n0, cnt, k0, k1, contrib);
    if (ready) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      if ((uint32_t)lane < cnt) __hip_atomic_store(&ready[n0 + lane], tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}

// With `ready`, the chain consumes the contributions as xxh3_kib_contribs
// publishes them (waits for ready[n] == tag).
// XXH3-128 long path, wave-level pieces: the initial accumulators of lane
// quad position q (pair 2q, 2q+1), and the tail (the stripes after the last
// full KiB block, the last stripe) + merge + avalanche after the chain.
__device__ __forceinline__ void xxh3_acc_init(int q, uint64_t& a0, uint64_t& a1) {
  a0 = q == 0 ? (uint64_t)P32_3 : q == 1 ? P64_2 : q == 2 ? P64_4 : P64_5;
  a1 = q == 0 ? P64_1 : q == 1 ? P64_3 : q == 2 ? (uint64_t)P32_2 : (uint64_t)P32_1;
}
__device__ __forceinline__ void xxh3_wave_tail_merge(const uint8_t* base, uint32_t pos, uint32_t len,
                                                     const LongSecret* __restrict__ ls, uint64_t a0, uint64_t a1,
                                                     uint64_t& out_lo, uint64_t& out_hi) {
  const int lane = threadIdx.x & 63;
  const int q = lane & 3;
  const int s = lane >> 2;
  const uint64_t k0 = ls->acc[s + 2 * q], k1 = ls->acc[s + 2 * q + 1];
  const uint32_t nb_blocks = (len - 1) / 1024;
  {
    const uint32_t tail0 = nb_blocks * 1024;
    const uint32_t nb_stripes = ((len - 1) - tail0) / 64;
    uint64_t c0 = 0, c1 = 0;
    if ((uint32_t)s < nb_stripes) {
      Win16 w = read_win16(base, pos + tail0 + 16 * lane);
      stripe_part(w, k0, k1, c0, c1);
    }
    if (lane < 4) {  // last stripe: input[len-64 .. len), secret + 121
      Win16 w = read_win16(base, pos + len - 64 + 16 * lane);
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
  out_lo = xxh3_avalanche((uint64_t)len * P64_1 + tlo);
  out_hi = xxh3_avalanche(~((uint64_t)len * P64_2) + thi);
}

// The serial scramble chain of accumulator k (this wave) over n >= 1 KiB
// blocks' contributions c[8 i + k], from the accumulator value acc.  One
// dependent VALU chain per wave: the 8 accumulators are independent, so 8
// single-wave workgroups (on different SIMDs) run them side by side; a wave
// holding two chains issues twice the quarter-rate multiplies per step and is
// slower per step than two waves (scripts/exp/chain_exp.cpp: 1 chain / wave
// 53 cycles per KiB, 2 chains / wave 79, the one-wave lane-quad chain 133).
// Step i: acc = scramble(acc + c_i); the addition of c_{i+1} is folded into
// the addend of the next multiply: y = lo' * P32_1 + (c_{i+1} + (hs * P32_1 << 32)).
// Contributions arrive 64 steps per coalesced load, kDepth loads in flight,
// and reach the chain by v_readlane.
template <int kDepth = 8>
__device__ __forceinline__ uint64_t xxh3_chain_wave(const uint64_t* __restrict__ c, uint64_t n, uint32_t k,
                                                     uint64_t acc, uint64_t s) {
  const int lane = threadIdx.x & 63;
  const uint32_t s_lo = (uint32_t)s, s_hi = (uint32_t)(s >> 32);
  // y = acc + c_0, lane-varying by construction (+0): keeps the chain in VGPRs (VALU)
  uint64_t y = acc + c[k] + __builtin_amdgcn_mbcnt_lo(0, 0);
  auto step = [&](uint64_t cn) {  // y = scramble(y) + cn
    const uint32_t hi = (uint32_t)(y >> 32);
    const uint32_t lo = (uint32_t)y ^ (hi >> 15) ^ s_lo;
    const uint32_t hs = hi ^ s_hi;
    y = (uint64_t)lo * P32_1 + (cn + ((uint64_t)(hs * P32_1) << 32));
  };
  const uint64_t* cn = c + 8;  // the contributions that follow c_0
  const uint64_t m = n - 1, full = m / 64;
  uint64_t buf[kDepth];
#pragma unroll
  for (int d = 0; d < kDepth; ++d) buf[d] = (uint64_t)d < full ? cn[8 * (64 * d + lane) + k] : 0;
  for (uint64_t b = 0; b < full; ++b) {
    const uint32_t lo = (uint32_t)buf[0], hi = (uint32_t)(buf[0] >> 32);
#pragma unroll
    for (int d = 0; d + 1 < kDepth; ++d) buf[d] = buf[d + 1];
    buf[kDepth - 1] = b + kDepth < full ? cn[8 * (64 * (b + kDepth) + lane) + k] : 0;
#pragma unroll
    for (int t = 0; t < 64; ++t)
      step((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo, t) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, t) << 32));
  }
  {
    const uint64_t n0 = full * 64;
    const uint64_t cl = n0 + lane < m ? cn[8 * (n0 + lane) + k] : 0;
    const uint32_t lo = (uint32_t)cl, hi = (uint32_t)(cl >> 32);
    for (uint32_t t = 0; n0 + t < m; ++t)
      step((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo, (int)t) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, (int)t) << 32));
  }
  step(0);  // the last block's scramble, nothing added after it
  return y;
}

// The eight scramble chains of one block on one wave: lane k = lane & 7 runs
// accumulator k (lanes 8.. repeat lanes 0..7), y = scramble(y) + c_i over the
// block's n >= 1 contribution rows (64 B each, row i = c[8 i .. 8 i + 7]) from
// acc, and returns scramble(y).  The instruction stream is that of one chain
// (xxh3_chain_wave needs eight waves on eight SIMDs for the same work), with
// no v_readlane: rows arrive by LDS-DMA into ring (kRing KiB of this wave's
// LDS), 16 rows per wave instruction, kRing instructions in flight (counted
// vmcnt, lds_dma.hpp), and each lane reads its accumulator's word with one
// ds_read_b64 per step, a chunk ahead of its steps.
struct ChainNoWait {
  __device__ __forceinline__ void operator()(uint64_t) const {}
};
// wait(q): called (wave-uniform) before chunk q's rows are fetched; a caller
// whose rows are produced in the same launch waits there until they are.
template <uint32_t kRing = 16, class Wait = ChainNoWait>
__device__ __forceinline__ uint64_t xxh3_chain8(const uint64_t* __restrict__ c, uint64_t n_in, uint64_t acc, uint64_t s,
                                                uint8_t* ring, Wait wait = Wait{}) {
  static_assert(kRing >= 2 && kRing <= 32, "chunks in flight");
  const uint32_t lane = threadIdx.x & 63, k = lane & 7;
  const uint32_t s_lo = (uint32_t)s, s_hi = (uint32_t)(s >> 32);
  // every compiler-visible load waited for here: the waits the compiler would
  // put in the loop (it does not see the DMA) would drain the ring
  asm volatile("" ::"v"(s_lo), "v"(s_hi), "v"(acc));
  const uint64_t n = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(n_in >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)n_in);
  const uint64_t nc = (n + 15) / 16;  // 1-KiB chunks of 16 rows
  const uint8_t* src = reinterpret_cast<const uint8_t*>(c);
  const uint32_t rbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)ring;
  auto dma = [&](uint64_t q, uint32_t slot) {  // (past the last chunk: the last one again, so the count stays)
    const uint64_t qq = q < nc ? q : nc - 1;
    if (q < nc) wait(qq);
    if (16 * qq + lane / 4 < n) dma16<false>(src + 1024 * qq + 16 * lane, rbase + 1024 * slot);
  };
  const __attribute__((address_space(3))) uint64_t* rw =
      (const __attribute__((address_space(3))) uint64_t*)ring + k;  // row r of slot q: rw[128 q + 8 r]
  uint64_t y;
  const uint32_t p1 = __builtin_amdgcn_readfirstlane(P32_1);
  auto step = [&](uint64_t cn) {  // y = scramble(y) + cn: two quarter-rate multiplies, five plain ops
    const uint32_t hi = (uint32_t)(y >> 32);
    const uint32_t lo = (uint32_t)y ^ (hi >> 15) ^ s_lo;
    uint32_t hm;  // (asm: left to itself the compiler spends a third v_mad_u64_u32 on the 64-bit addend)
    asm("v_mul_lo_u32 %0, %1, %2" : "=v"(hm) : "v"(hi ^ s_hi), "s"(p1));
    const uint64_t add = ((uint64_t)(hm + (uint32_t)(cn >> 32)) << 32) | (uint32_t)cn;
    uint64_t cc;  // (the carry-out nobody reads)
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(y), "=s"(cc) : "v"(lo), "s"(p1), "v"(add));
  };
#pragma unroll
  for (uint32_t q = 0; q < kRing; ++q) dma(q, q);
  // rows of two chunks in registers, ping-pong (no copies): one chunk's steps
  // run while the next one's rows come out of the ring
  uint64_t A[16], B[16];
  vm_wait<kRing - 1>();  // chunk 0
#pragma unroll
  for (int r = 0; r < 16; ++r) A[r] = rw[8 * r];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  dma(kRing, 0);
  y = acc + A[0];  // row 0 seeds y
  // in flight at chunk q: chunks q + 1 .. q + kRing; read chunk q + 1 into nb,
  // the steps of chunk q (cb) from row r0, then chunk q + 1's slot refilled
  auto chunk = [&](uint64_t* cb, uint64_t* nb, uint64_t q, int r0) {
    const uint32_t ns = (uint32_t)((q + 1) % kRing);
    vm_wait<kRing - 1>();
#pragma unroll
    for (int r = 0; r < 16; ++r) nb[r] = rw[128 * ns + 8 * r];
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (r >= r0) step(cb[r]);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(y)::"memory");  // (y ties the wait to the steps)
    dma(q + 1 + kRing, ns);
  };
  auto tail = [&](const uint64_t* cb, uint32_t r0, uint32_t rn) {
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r)
      if (r >= r0 && r < rn) step(cb[r]);
  };
  const uint64_t full = n / 16;  // whole chunks
  const uint32_t rn = (uint32_t)(n - 16 * full);
  if (full == 0) {
    tail(A, 1, rn);
  } else {
    chunk(A, B, 0, 1);
    uint64_t q = 1;
    for (; q + 2 <= full; q += 2) {
      chunk(B, A, q, 0);
      chunk(A, B, q + 1, 0);
    }
    if (q < full) {
      chunk(B, A, q, 0);
      tail(A, 0, rn);
    } else {
      tail(B, 0, rn);
    }
  }
  vm_wait<0>();  // (no DMA may land in the ring after this chain)
  step(0);       // the last block's scramble, nothing added after it
  return y;
}

template <uint32_t kBatch = 8>
__device__ __forceinline__ void xxh3_128_wave_finish(const uint8_t* base, uint32_t pos, uint32_t len,
                                                     const LongSecret* __restrict__ ls, const uint64_t* contrib,
                                                     uint64_t& out_lo, uint64_t& out_hi,
                                                     const uint32_t* ready = nullptr, uint32_t tag = 0) {
  const int q = threadIdx.x & 3;
  uint64_t a0, a1;
  xxh3_acc_init(q, a0, a1);
  const uint64_t scr0 = ls->acc[16 + 2 * q], scr1 = ls->acc[16 + 2 * q + 1];
  const uint32_t nb_blocks = (len - 1) / 1024;
  // the serial chain: kBatch KiB blocks' contributions read ahead of their
  // steps.  The flag and contribution reads are unconditional (no branch, so
  // no wait, between them): past the last KiB block they read LDS beyond the
  // arrays (the callers' stage follows), and those values are not used.
  for (uint32_t n0 = 0; n0 < nb_blocks; n0 += kBatch) {
    uint64_t c0[kBatch], c1[kBatch];
    if (ready) {  // (every lane reads the same flags: the loop is wave-uniform)
      for (;;) {
        uint32_t f[kBatch];
#pragma unroll
        for (uint32_t t = 0; t < kBatch; ++t)
          f[t] = __hip_atomic_load(&ready[n0 + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        bool all = true;
#pragma unroll
        for (uint32_t t = 0; t < kBatch; ++t) all &= (n0 + t >= nb_blocks) | (f[t] == tag);
        if (all) break;
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    }
#pragma unroll
    for (uint32_t t = 0; t < kBatch; ++t) {
      c0[t] = contrib[8 * (n0 + t) + 2 * q];
      c1[t] = contrib[8 * (n0 + t) + 2 * q + 1];
    }
#pragma unroll
    for (uint32_t t = 0; t < kBatch; ++t) {
      if (n0 + t < nb_blocks) {
        a0 = xxh3_scr(a0, c0[t], scr0);
        a1 = xxh3_scr(a1, c1[t], scr1);
      }
    }
  }
  xxh3_wave_tail_merge(base, pos, len, ls, a0, a1, out_lo, out_hi);
}

// Window-backed readers for the per-lane short path over an aligned base.
struct BaseReader8 {
  const uint8_t* base;
  uint32_t pos;
  __device__ __forceinline__ uint32_t operator()(uint32_t o) const { return base[pos + o]; }
};
struct BaseReader64 {
  const uint8_t* base;
  uint32_t pos;
  __device__ __forceinline__ uint64_t operator()(uint32_t o) const {
    const uint32_t p = pos + o, a = p & ~3u, s = p & 3u;
    uint32_t d0 = ld32(base, a), d1 = ld32(base, a + 4), d2 = ld32(base, a + 8);
    return (uint64_t)alignbyte(d1, d0, s) | ((uint64_t)alignbyte(d2, d1, s) << 32);
  }
};

// Row-cooperative XXH3-128 (> 240 B): the 16 lanes of one DPP row hash one
// input, so a wave hashes four blocks at once.  Lane r = lane & 15 owns bytes
// [256t + 16r, +16) of each KiB block (t = 0..3): stripe 4t + (r >> 2),
// accumulator pair q = r & 3.  The per-KiB reduction is two DPP row rotates.
__device__ __forceinline__ uint64_t row_quad_sum64(uint64_t v) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  v += (uint64_t)dpp_ror4(lo) | ((uint64_t)dpp_ror4(hi) << 32);
  lo = (uint32_t)v; hi = (uint32_t)(v >> 32);
  v += (uint64_t)dpp_ror8(lo) | ((uint64_t)dpp_ror8(hi) << 32);
  return v;
}
// sum over the 4 lanes of each quad (DPP quad_perm [1,0,3,2] then [2,3,0,1])
__device__ __forceinline__ uint64_t quad_sum64(uint64_t v) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  v += (uint64_t)(uint32_t)__builtin_amdgcn_mov_dpp((int)lo, 0xB1, 0xF, 0xF, true) |
       ((uint64_t)(uint32_t)__builtin_amdgcn_mov_dpp((int)hi, 0xB1, 0xF, 0xF, true) << 32);
  lo = (uint32_t)v; hi = (uint32_t)(v >> 32);
  v += (uint64_t)(uint32_t)__builtin_amdgcn_mov_dpp((int)lo, 0x4E, 0xF, 0xF, true) |
       ((uint64_t)(uint32_t)__builtin_amdgcn_mov_dpp((int)hi, 0x4E, 0xF, 0xF, true) << 32);
  return v;
}

__device__ __forceinline__ void xxh3_128_row_long(const uint8_t* base, uint32_t pos, uint32_t len,
                                                  const LongSecret* __restrict__ ls, uint64_t& out_lo,
                                                  uint64_t& out_hi) {
  const int r = threadIdx.x & 15;
  const int q = r & 3, s = r >> 2;
  uint64_t k0[4], k1[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    k0[t] = ls->acc[4 * t + s + 2 * q];
    k1[t] = ls->acc[4 * t + s + 2 * q + 1];
  }
  uint64_t a0 = q == 0 ? (uint64_t)P32_3 : q == 1 ? P64_2 : q == 2 ? P64_4 : P64_5;
  uint64_t a1 = q == 0 ? P64_1 : q == 1 ? P64_3 : q == 2 ? (uint64_t)P32_2 : (uint64_t)P32_1;
  const uint64_t scr0 = ls->acc[16 + 2 * q], scr1 = ls->acc[16 + 2 * q + 1];
  const uint32_t nb_blocks = (len - 1) / 1024;
  for (uint32_t n = 0; n < nb_blocks; ++n) {
    Win16 w[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) w[t] = read_win16(base, pos + n * 1024 + 256 * t + 16 * r);
    uint64_t c0 = 0, c1 = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) stripe_part(w[t], k0[t], k1[t], c0, c1);
    c0 = row_quad_sum64(c0);
    c1 = row_quad_sum64(c1);
    a0 = xxh3_scr(a0, c0, scr0);
    a1 = xxh3_scr(a1, c1, scr1);
  }
  {
    const uint32_t tail0 = nb_blocks * 1024;
    const uint32_t nb_stripes = ((len - 1) - tail0) / 64;
    uint64_t c0 = 0, c1 = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if ((uint32_t)(4 * t + s) < nb_stripes) {
        const Win16 w = read_win16(base, pos + tail0 + 256 * t + 16 * r);
        stripe_part(w, k0[t], k1[t], c0, c1);
      }
    }
    if (r < 4) {  // last stripe: input[len-64 .. len), secret + 121
      const Win16 w = read_win16(base, pos + len - 64 + 16 * r);
      stripe_part(w, ls->last[2 * q], ls->last[2 * q + 1], c0, c1);
    }
    a0 += row_quad_sum64(c0);
    a1 += row_quad_sum64(c1);
  }
  uint64_t tlo = mul_fold64(a0 ^ ls->mlo[2 * q], a1 ^ ls->mlo[2 * q + 1]);
  uint64_t thi = mul_fold64(a0 ^ ls->mhi[2 * q], a1 ^ ls->mhi[2 * q + 1]);
  tlo = quad_sum64(tlo);
  thi = quad_sum64(thi);
  out_lo = xxh3_avalanche((uint64_t)len * P64_1 + tlo);
  out_hi = xxh3_avalanche(~((uint64_t)len * P64_2) + thi);
}

// Register-lean variant of xxh3_128_row_long for kernels that run 4 waves per
// SIMD: the stripe secret words are read from an LDS copy of LongSecret as
// they are needed and one 16-byte window is in flight per step (occupancy
// hides the LDS latency instead of registers).
__device__ __forceinline__ void xxh3_128_row_long_lean(const uint8_t* base, uint32_t pos, uint32_t len,
                                                       const LongSecret* ls, uint64_t& out_lo, uint64_t& out_hi) {
  const int r = threadIdx.x & 15;
  const int q = r & 3, s = r >> 2;
  uint64_t a0 = q == 0 ? (uint64_t)P32_3 : q == 1 ? P64_2 : q == 2 ? P64_4 : P64_5;
  uint64_t a1 = q == 0 ? P64_1 : q == 1 ? P64_3 : q == 2 ? (uint64_t)P32_2 : (uint64_t)P32_1;
  const uint32_t nb_blocks = (len - 1) / 1024;
  const uint64_t* acc = ls->acc + s + 2 * q;
  const uint32_t wa = (pos + 16 * r) & ~3u, wsh = (pos + 16 * r) & 3u;  // (every window of the lane shares the shift)
  for (uint32_t n = 0; n < nb_blocks; ++n) {
    uint64_t c0 = 0, c1 = 0;
#pragma unroll 2
    for (int t = 0; t < 4; ++t) {
      const Win16 w = read_win16_split(base, wa + n * 1024 + 256 * t, wsh);
      stripe_part(w, acc[4 * t], acc[4 * t + 1], c0, c1);
    }
    c0 = row_quad_sum64(c0);
    c1 = row_quad_sum64(c1);
    a0 = xxh3_scr(a0, c0, ls->acc[16 + 2 * q]);
    a1 = xxh3_scr(a1, c1, ls->acc[16 + 2 * q + 1]);
  }
  {
    const uint32_t tail0 = nb_blocks * 1024;
    const uint32_t nb_stripes = ((len - 1) - tail0) / 64;
    uint64_t c0 = 0, c1 = 0;
#pragma unroll 1
    for (int t = 0; t < 4; ++t) {
      if ((uint32_t)(4 * t + s) < nb_stripes) {
        const Win16 w = read_win16_split(base, wa + tail0 + 256 * t, wsh);
        stripe_part(w, acc[4 * t], acc[4 * t + 1], c0, c1);
      }
    }
    if (r < 4) {  // last stripe: input[len-64 .. len), secret + 121
      const Win16 w = read_win16(base, pos + len - 64 + 16 * r);
      stripe_part(w, ls->last[2 * q], ls->last[2 * q + 1], c0, c1);
    }
    a0 += row_quad_sum64(c0);
    a1 += row_quad_sum64(c1);
  }
  uint64_t tlo = mul_fold64(a0 ^ ls->mlo[2 * q], a1 ^ ls->mlo[2 * q + 1]);
  uint64_t thi = mul_fold64(a0 ^ ls->mhi[2 * q], a1 ^ ls->mhi[2 * q + 1]);
  tlo = quad_sum64(tlo);
  thi = quad_sum64(thi);
  out_lo = xxh3_avalanche((uint64_t)len * P64_1 + tlo);
  out_hi = xxh3_avalanche(~((uint64_t)len * P64_2) + thi);
}

// Octet XXH3-128 (> 240 B): the 8 lanes of an aligned lane octet hash one
// input, so a wave hashes eight blocks at once.  Lane r = lane & 7 owns
// accumulator pair q = r >> 1 (acc[2q], acc[2q+1]) over stripes 2i + h of
// every KiB, h = r & 1 (interleaved, so an octet reads 128 contiguous bytes
// per step: no bank conflict between its halves).  Per KiB the two halves of
// a pair meet in ONE DPP quad-perm step; each lane reads its 16-byte window
// and its two secret words (one ds_read2_b64) per stripe.  All 8 lanes of the
// octet must be active.
template <int kCtrl>
__device__ __forceinline__ uint64_t mov_dpp64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, kCtrl, 0xF, 0xF, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), kCtrl, 0xF, 0xF, true);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ void xxh3_128_oct_long(const uint8_t* base, uint32_t pos, uint32_t len,
                                                  const LongSecret* ls, uint64_t& out_lo, uint64_t& out_hi) {
  const int r = threadIdx.x & 7;
  const int q = r >> 1, h = r & 1;
  uint64_t a0 = q == 0 ? (uint64_t)P32_3 : q == 1 ? P64_2 : q == 2 ? P64_4 : P64_5;
  uint64_t a1 = q == 0 ? P64_1 : q == 1 ? P64_3 : q == 2 ? (uint64_t)P32_2 : (uint64_t)P32_1;
  const uint64_t scr0 = ls->acc[16 + 2 * q], scr1 = ls->acc[16 + 2 * q + 1];
  const uint64_t* key = ls->acc + h + 2 * q;  // stripe 2i + h, pair q -> key[2i], key[2i + 1]
  const uint32_t nb_blocks = (len - 1) / 1024;
  const uint32_t lpos = pos + 64 * h + 16 * q;  // stripe h of KiB 0, this lane's 16 bytes
  for (uint32_t n = 0; n < nb_blocks; ++n) {
    uint64_t c0 = 0, c1 = 0;
#pragma unroll 4
    for (int i = 0; i < 8; ++i) {
      const Win16 w = read_win16(base, lpos + 1024 * n + 128 * i);
      stripe_part(w, key[2 * i], key[2 * i + 1], c0, c1);
    }
    c0 += mov_dpp64<0xB1>(c0);  // quad_perm [1,0,3,2]: the other half of the pair
    c1 += mov_dpp64<0xB1>(c1);
    a0 = xxh3_scr(a0, c0, scr0);
    a1 = xxh3_scr(a1, c1, scr1);
  }
  {
    const uint32_t tail0 = nb_blocks * 1024;
    const uint32_t nb_stripes = ((len - 1) - tail0) / 64;
    uint64_t c0 = 0, c1 = 0;
#pragma unroll 1
    for (uint32_t i = 0; i < 8; ++i) {
      if (2 * i + h < nb_stripes) {
        const Win16 w = read_win16(base, lpos + tail0 + 128 * i);
        stripe_part(w, key[2 * i], key[2 * i + 1], c0, c1);
      }
    }
    if (h == 0) {  // last stripe: input[len-64 .. len), secret + 121
      const Win16 w = read_win16(base, pos + len - 64 + 16 * q);
      stripe_part(w, ls->last[2 * q], ls->last[2 * q + 1], c0, c1);
    }
    a0 += c0 + mov_dpp64<0xB1>(c0);
    a1 += c1 + mov_dpp64<0xB1>(c1);
  }
  uint64_t tlo = mul_fold64(a0 ^ ls->mlo[2 * q], a1 ^ ls->mlo[2 * q + 1]);
  uint64_t thi = mul_fold64(a0 ^ ls->mhi[2 * q], a1 ^ ls->mhi[2 * q + 1]);
  tlo += mov_dpp64<0x4E>(tlo);   // quad_perm [2,3,0,1]: pairs q ^ 1
  thi += mov_dpp64<0x4E>(thi);
  tlo += mov_dpp64<0x141>(tlo);  // row_half_mirror: the other quad of the octet (h-symmetric)
  thi += mov_dpp64<0x141>(thi);
  out_lo = xxh3_avalanche((uint64_t)len * P64_1 + tlo);
  out_hi = xxh3_avalanche(~((uint64_t)len * P64_2) + thi);
}

__device__ __forceinline__ void xxh3_128_row(const uint8_t* base, uint32_t pos, uint32_t len,
                                             uint64_t& lo, uint64_t& hi) {
  if (len > 240) {
    xxh3_128_row_long(base, pos, len, &kLongSecret, lo, hi);
  } else {
    xxh3_128_short(len, BaseReader8{base, pos}, BaseReader64{base, pos}, lo, hi);
  }
}

// XXH3-128 of base[pos..pos+len) for any len: long inputs use the whole wave
// (wave-uniform len required), short inputs are computed by every lane
// redundantly (results identical in all lanes).
__device__ __forceinline__ void xxh3_128_wave(const uint8_t* base, uint32_t pos, uint32_t len,
                                              const LongSecret* ls, uint64_t& lo, uint64_t& hi) {
  if (len > 240) {
    xxh3_128_wave_long(base, pos, len, ls, lo, hi);
  } else {
    xxh3_128_short(len, BaseReader8{base, pos}, BaseReader64{base, pos}, lo, hi);
  }
}

// Per-lane XXH3-64 for inputs > 240 B (hash-index keys longer than 240 B;
// rare).  Scalar restatement of hashLong + mergeAccs on one lane.
template <class R64>
__device__ __noinline__ uint64_t xxh3_64_long_lane(uint32_t len, R64 r64, const LongSecret* ls) {
  uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
  auto stripe = [&](uint32_t off, const uint64_t* key) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t v = r64(off + 8 * i);
      const uint64_t x = v ^ key[i];
      acc[i ^ 1] += v;
      acc[i] += (uint64_t)(uint32_t)x * (x >> 32);
    }
  };
  const uint32_t nb = (len - 1) / 1024;
  for (uint32_t n = 0; n < nb; ++n) {
    for (uint32_t s = 0; s < 16; ++s) stripe(n * 1024 + 64 * s, ls->acc + s);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      acc[i] = xxh3_scr(acc[i], 0, ls->acc[16 + i]);
    }
  }
  const uint32_t ns = ((len - 1) - nb * 1024) / 64;
  for (uint32_t s = 0; s < ns; ++s) stripe(nb * 1024 + 64 * s, ls->acc + s);
  stripe(len - 64, ls->last);
  uint64_t r = (uint64_t)len * P64_1;
#pragma unroll
  for (int i = 0; i < 4; ++i) r += mul_fold64(acc[2 * i] ^ ls->mlo[2 * i], acc[2 * i + 1] ^ ls->mlo[2 * i + 1]);
  return xxh3_avalanche(r);
}

template <class R8, class R64>
__device__ __forceinline__ uint64_t xxh3_64_any(uint32_t len, R8 rb, R64 r64) {
  if (len > 240) return xxh3_64_long_lane(len, r64, &kLongSecret);
  return xxh3_64_short(len, rb, r64);
}

// ------------------------------------------------------------ wave helpers
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up((int)v, d);
    if (lane >= d) v += t;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t lo = __shfl_up((int)(uint32_t)v, d), hi = __shfl_up((int)(uint32_t)(v >> 32), d);
    uint64_t t = (uint64_t)lo | ((uint64_t)hi << 32);
    if (lane >= d) v += t;
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_bcast_u32(uint32_t v, int src) { return __shfl((int)v, src); }
__device__ __forceinline__ uint64_t wave_bcast_u64(uint64_t v, int src) {
  uint32_t lo = __shfl((int)(uint32_t)v, src), hi = __shfl((int)(uint32_t)(v >> 32), src);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
// per-lane source lane (ds_bpermute)
__device__ __forceinline__ uint64_t wave_shfl_u64(uint64_t v, int src) { return wave_bcast_u64(v, src); }
// wave-uniform source lane (v_readlane -> SGPR)
__device__ __forceinline__ uint32_t wave_readlane_u32(uint32_t v, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)src);
}
__device__ __forceinline__ uint64_t wave_readlane_u64(uint64_t v, uint32_t src) {
  return (uint64_t)wave_readlane_u32((uint32_t)v, src) | ((uint64_t)wave_readlane_u32((uint32_t)(v >> 32), src) << 32);
}

}  // namespace lsmgpu
