// encode.hip — batched SST block encode on gfx950.
//
// Replaces, per block, DataBlock::encode_into / IndexBlock::encode_into
// (src/table/data_block/mod.rs:523-549, src/table/index_block/mod.rs:110-127,
// Encoder src/table/block/encoder.rs:84-164, Trailer trailer.rs:78-173) and
// Block::write_into (src/table/block/mod.rs:45-84, CompressionType::None):
// the payload xxh3_128 and the 33-byte header are fused into the same pass.
//
// Pipeline (all on one stream, DESIGN.md "Encode kernels"):
//   E1  size pass, one wave per block: per item (lane) the shared prefix
//       with the restart head (encoder.rs:140-143) and the record length;
//       wave scan -> records bytes, binary-index step, hash-index size.
//   S   device exclusive scan of block sizes -> d_block_off (packed output).
//   E2  write pass, one wave per block: key/value spans staged HBM->LDS in
//       coalesced 16 B/lane sweeps, each lane assembles its record in the LDS
//       payload image (dword stores inside records, byte stores at seams),
//       binary index, hash index (LDS min/max atomics reproduce the
//       order-independent FREE/idx/CONFLICT rule, hash_index/builder.rs:64-110),
//       trailer, wave xxh3_128 over the image, header, then one coalesced
//       16 B/lane copy-out to the block's place in the packed output.
//   E3  same algorithm straight on HBM for blocks whose staging does not fit
//       the LDS budget (grid-stride over a device list).
#include <hip/hip_runtime.h>

#include <math.h>

#include "block_format.hpp"
#include "encode.hpp"
#include "scan.hpp"

namespace lsmgpu {

constexpr uint32_t kPlanLarge = 1, kPlanBad = 2;
constexpr uint32_t kE2Budget = 24 * 1024;  // LDS bytes per E2 wave
constexpr uint32_t kE3HashChunk = 4096;    // buckets per LDS pass in E3

struct alignas(16) BlockPlan {
  uint32_t recs;      // bytes of all records
  uint32_t bin_len;   // restart heads
  uint32_t hash_w;    // buckets written (0 = no hash index in the block)
  uint32_t step_flags;  // step (2|4) | flags << 8
};

__device__ __forceinline__ uint32_t leb_len(uint64_t v) {
  const uint32_t bits = 64 - __builtin_clzll(v | 1);
  return (bits + 6) / 7;
}

// hash_index/builder.rs:39-63: (item_count as f32 * ratio) as u32, at least 1
__device__ __host__ __forceinline__ uint32_t bucket_count(uint64_t n, float ratio) {
  if (!(ratio > 0.0f)) return 0;
  const float prod = (float)n * ratio;
  uint32_t b;
  if (!(prod > 0.0f)) b = 0;
  else if (prod >= 4294967296.0f) b = 0xFFFFFFFFu;
  else b = (uint32_t)prod;
  return b < 1 ? 1 : b;
}

__device__ __forceinline__ Win16 read_win16_at(const uint8_t* base, uint64_t off) {
  return read_win16(base + (off & ~3ULL), (uint32_t)(off & 3));
}

// longest_shared_prefix_length, src/table/util.rs:125-130
__device__ __forceinline__ uint32_t lcp_global(const uint8_t* keys, uint64_t a, uint64_t b, uint32_t n) {
  uint32_t k = 0;
  while (k < n) {
    const Win16 wa = read_win16_at(keys, a + k), wb = read_win16_at(keys, b + k);
    const uint64_t x0 = wa.lo ^ wb.lo, x1 = wa.hi ^ wb.hi;
    if (x0) return min(n, k + (uint32_t)(__builtin_ctzll(x0) >> 3));
    if (x1) return min(n, k + 8 + (uint32_t)(__builtin_ctzll(x1) >> 3));
    k += 16;
  }
  return n;
}

struct EncodeParams {
  lsm_items it;
  const uint32_t* starts;
  uint32_t n_blocks;
  uint32_t ri;
  float ratio;
  uint32_t type;
  uint8_t* out;
  uint64_t out_cap;
  uint64_t* block_off;
  int32_t* status;
  uint16_t* shared;     // [n_items]
  uint64_t* sizes;      // [n_blocks]
  BlockPlan* plans;     // [n_blocks]
  uint32_t* large_list; // [n_blocks]
  uint32_t* large_count;
};

__device__ __forceinline__ bool is_index(const EncodeParams& P) { return P.type == 1; }

// Record length of item i (j = index within its block); sh = shared prefix.
__device__ __forceinline__ uint64_t record_len(const EncodeParams& P, uint64_t i, uint32_t j, uint32_t klen,
                                               uint32_t sh, bool& bad) {
  const uint64_t seq = P.it.seqno[i];
  if (is_index(P)) {
    return 1 + leb_len(P.it.handle_off[i]) + leb_len(P.it.handle_size[i]) + leb_len(seq) + leb_len(klen) + klen;
  }
  const uint32_t vt = P.it.vtype[i];
  if (!valid_vtype(vt)) bad = true;
  uint64_t rec = 1 + leb_len(seq);
  if (j % P.ri == 0) rec += leb_len(klen) + klen;
  else rec += leb_len(sh) + leb_len(klen - sh) + (klen - sh);
  if (!is_tombstone(vt)) {
    const uint64_t vl = P.it.val_off[i + 1] - P.it.val_off[i];
    if (vl > 0xFFFFFFFFULL) bad = true;
    rec += leb_len(vl) + vl;
  }
  return rec;
}

// LDS staging need of a block for E2 (see layout in encode_write_kernel).
__device__ __forceinline__ uint64_t e2_need(const EncodeParams& P, uint32_t s, uint32_t e, uint64_t total,
                                            uint32_t hash_w) {
  const uint64_t ka = (uint64_t)(uintptr_t)P.it.keys + P.it.key_off[s];
  const uint64_t kb = (uint64_t)(uintptr_t)P.it.keys + P.it.key_off[e];
  uint64_t need = ((kb + 15) & ~15ULL) - (ka & ~15ULL) + 32;
  if (!is_index(P)) {
    const uint64_t va = (uint64_t)(uintptr_t)P.it.vals + P.it.val_off[s];
    const uint64_t vb = (uint64_t)(uintptr_t)P.it.vals + P.it.val_off[e];
    need += ((vb + 15) & ~15ULL) - (va & ~15ULL) + 32;
  }
  need += ((total + 16 + 15) & ~15ULL) + 32;
  need += 8ULL * ((hash_w + 3) & ~3u);
  return need;
}

// ---------------------------------------------------------------- E1: sizes
__global__ __launch_bounds__(256) void encode_sizes_kernel(EncodeParams P) {
  const int lane = threadIdx.x & 63;
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= P.n_blocks) return;
  const uint32_t s = P.starts[b], e = P.starts[b + 1];
  const uint32_t ri = is_index(P) ? 1 : P.ri;
  bool bad = e <= s;
  const uint32_t n = bad ? 0 : e - s;
  uint64_t carry = 0, last_head = 0;
  const uint32_t lh = n ? ((n - 1) / ri) * ri : 0;
  for (uint32_t c = 0; c < n; c += kWave) {
    const uint32_t j = c + lane;
    uint64_t rec = 0;
    if (j < n) {
      const uint64_t i = (uint64_t)s + j;
      const uint64_t ko = P.it.key_off[i];
      const uint64_t kl64 = P.it.key_off[i + 1] - ko;
      if (kl64 > 0xFFFF) bad = true;
      const uint32_t klen = (uint32_t)min(kl64, (uint64_t)0xFFFF);
      uint32_t sh = 0;
      if (!is_index(P) && j % ri != 0) {
        const uint64_t h = (uint64_t)s + (j / ri) * ri;
        const uint64_t hko = P.it.key_off[h];
        const uint32_t hkl = (uint32_t)min(P.it.key_off[h + 1] - hko, (uint64_t)0xFFFF);
        sh = lcp_global(P.it.keys, hko, ko, min(hkl, klen));
      }
      if (!is_index(P)) P.shared[i] = (uint16_t)sh;
      rec = record_len(P, i, j, klen, sh, bad);
    }
    const uint64_t incl = wave_incl_scan_u64(rec);
    if (lh >= c && lh < c + kWave) last_head = carry + wave_bcast_u64(incl - rec, lh - c);
    carry += wave_bcast_u64(incl, 63);
  }
  bad = __ballot(bad) != 0;
  if (lane != 0) return;
  BlockPlan pl;
  const uint32_t bin_len = n ? (n + ri - 1) / ri : 0;
  const uint32_t step = last_head <= 0xFFFF ? 2 : 4;
  const uint32_t buckets = is_index(P) ? 0 : bucket_count(n, P.ratio);
  const uint32_t hash_w = (buckets > 0 && bin_len <= kHashMaxPointers) ? buckets : 0;
  const uint64_t payload = carry + 1 + (uint64_t)bin_len * step + hash_w + kTrailerLen;
  const uint64_t total = kHdrLen + payload;
  if (carry > 0xFFFFFFF0ULL || total > 0xFFFFFF00ULL) bad = true;
  uint32_t flags = 0;
  if (bad) {
    flags = kPlanBad;
    P.status[b] = ST_BAD_ARG;
  } else if (e2_need(P, s, e, total, hash_w) > kE2Budget) {
    flags = kPlanLarge;
    const uint32_t slot = atomicAdd(P.large_count, 1u);
    P.large_list[slot] = b;
  }
  pl.recs = (uint32_t)carry;
  pl.bin_len = bin_len;
  pl.hash_w = hash_w;
  pl.step_flags = step | (flags << 8);
  P.plans[b] = pl;
  P.sizes[b] = bad ? 0 : total;
}

// ------------------------------------------------------- record assembly
// Byte sink over a 4-aligned base: dword stores for bytes wholly inside the
// caller's record, byte stores at the seams shared with neighbour records.
struct ByteWriter {
  uint8_t* dst;
  uint32_t pos;
  uint64_t acc;
  uint32_t nacc;
  __device__ __forceinline__ void init(uint8_t* d, uint32_t p) { dst = d; pos = p; acc = 0; nacc = 0; }
  __device__ __forceinline__ void drain() {
    while (nacc && (pos & 3)) {
      dst[pos++] = (uint8_t)acc;
      acc >>= 8;
      --nacc;
    }
    if (nacc >= 4) {
      *reinterpret_cast<uint32_t*>(dst + pos) = (uint32_t)acc;
      acc >>= 32;
      nacc -= 4;
      pos += 4;
    }
  }
  __device__ __forceinline__ void byte(uint32_t b) {
    acc |= (uint64_t)(b & 0xFF) << (8 * nacc);
    ++nacc;
    if (nacc >= 4) drain();
  }
  __device__ __forceinline__ void word(uint32_t v, uint32_t n) {  // n in 1..4 low bytes of v
    if (n < 4) v &= (1u << (8 * n)) - 1;
    acc |= (uint64_t)v << (8 * nacc);
    nacc += n;
    if (nacc >= 4) drain();
  }
  __device__ __forceinline__ void leb(uint64_t v) {  // varint-rs write_*_varint
    while (v >= 0x80) {
      byte((uint32_t)(v & 0x7F) | 0x80);
      v >>= 7;
    }
    byte((uint32_t)v);
  }
  // n bytes from src_base[src_pos ..) (4-aligned base, any src_pos)
  __device__ __forceinline__ void copy(const uint8_t* src_base, uint32_t src_pos, uint32_t n) {
    uint32_t k = 0;
    for (; k + 4 <= n; k += 4) word(read_u32_unaligned(src_base, src_pos + k), 4);
    if (k < n) word(read_u32_unaligned(src_base, src_pos + k), n - k);
  }
  __device__ __forceinline__ void finish() {
    while (nacc) {
      dst[pos++] = (uint8_t)acc;
      acc >>= 8;
      --nacc;
    }
  }
};

// Source of item bytes: either staged LDS images or global arenas.
struct ItemSrc {
  const uint8_t* kbase;  // 16-aligned
  uint64_t kshift;       // key i is at kbase + key_off[i] - kshift
  const uint8_t* vbase;
  uint64_t vshift;
};

__device__ __forceinline__ void write_record(const EncodeParams& P, const ItemSrc& src, uint64_t i, uint32_t j,
                                             uint32_t ri, uint8_t* dst, uint32_t dpos) {
  ByteWriter w;
  w.init(dst, dpos);
  const uint64_t ko = P.it.key_off[i];
  const uint32_t klen = (uint32_t)(P.it.key_off[i + 1] - ko);
  const uint64_t seq = P.it.seqno[i];
  const uint64_t kp = ko - src.kshift;  // position relative to kbase
  const uint8_t* kb = src.kbase + (kp & ~15ULL);
  const uint32_t kq = (uint32_t)(kp & 15);
  if (is_index(P)) {  // block_handle.rs:134-156
    w.byte(0);
    w.leb(P.it.handle_off[i]);
    w.leb(P.it.handle_size[i]);
    w.leb(seq);
    w.leb(klen);
    w.copy(kb, kq, klen);
    w.finish();
    return;
  }
  const uint32_t vt = P.it.vtype[i];
  w.byte(vt);
  w.leb(seq);
  if (j % ri == 0) {  // encode_full_into, data_block/mod.rs:195-219
    w.leb(klen);
    w.copy(kb, kq, klen);
  } else {            // encode_truncated_into, data_block/mod.rs:221-264
    const uint32_t sh = P.shared[i];
    w.leb(sh);
    w.leb(klen - sh);
    w.copy(kb, kq + sh, klen - sh);
  }
  if (!is_tombstone(vt)) {
    const uint64_t vo = P.it.val_off[i];
    const uint32_t vl = (uint32_t)(P.it.val_off[i + 1] - vo);
    w.leb(vl);
    const uint64_t vp = vo - src.vshift;
    w.copy(src.vbase + (vp & ~15ULL), (uint32_t)(vp & 15), vl);
  }
  w.finish();
}

__device__ __forceinline__ void store_le(uint8_t* dst, uint32_t pos, uint64_t v, uint32_t n) {
  for (uint32_t k = 0; k < n; ++k) dst[pos + k] = (uint8_t)(v >> (8 * k));
}

// Hash-index bucket of a key (hash_index/mod.rs:35-41).
__device__ __forceinline__ uint32_t key_bucket(const ItemSrc& src, const EncodeParams& P, uint64_t i,
                                               uint32_t buckets) {
  const uint64_t ko = P.it.key_off[i];
  const uint32_t klen = (uint32_t)(P.it.key_off[i + 1] - ko);
  const uint64_t kp = ko - src.kshift;
  const uint8_t* kb = src.kbase + (kp & ~15ULL);
  const uint32_t kq = (uint32_t)(kp & 15);
  const uint64_t h = xxh3_64_any(klen, BaseReader8{kb, kq}, BaseReader64{kb, kq});
  return (uint32_t)(h % buckets);
}

// Marker, binary index entries are written by the record loop; this writes
// the hash-index bytes (given final min/max per bucket) and the trailer.
__device__ __forceinline__ uint32_t bucket_byte(uint32_t lo, uint32_t hi) {
  return lo == 0xFFFFFFFFu ? kHashFree : (lo == hi ? lo : kHashConflict);
}

__device__ __forceinline__ void write_trailer_bytes(uint8_t* dst, uint32_t tp, uint32_t ri, uint32_t step,
                                                    uint32_t bin_len, uint32_t bin_off, uint32_t hash_w,
                                                    uint32_t hash_off, uint32_t items) {
  // trailer.rs:118-163, lanes 0..30 write one byte each
  const int lane = threadIdx.x & 63;
  if (lane >= (int)kTrailerLen) return;
  uint32_t v;
  const int k = lane;
  if (k == 0) v = ri;
  else if (k == 1) v = step;
  else if (k < 6) v = bin_len >> (8 * (k - 2));
  else if (k < 10) v = bin_off >> (8 * (k - 6));
  else if (k < 14) v = hash_w >> (8 * (k - 10));
  else if (k < 18) v = hash_off >> (8 * (k - 14));
  else if (k == 18) v = 1;       // prefix truncation on
  else if (k < 27) v = 0;        // fixed key/value size (unused)
  else v = items >> (8 * (k - 27));
  dst[tp + k] = (uint8_t)v;
}

// Header::encode_into (header.rs:80-112): lanes 0..32 write one byte each.
__device__ __forceinline__ void write_header_bytes(uint8_t* dst, uint32_t hp, uint32_t type, uint64_t ck_lo,
                                                   uint64_t ck_hi, uint32_t plen) {
  uint64_t w0 = 0x034D534CULL | ((uint64_t)type << 32) | (ck_lo << 40);
  uint64_t w1 = (ck_lo >> 24) | (ck_hi << 40);
  uint64_t w2 = (ck_hi >> 24) | ((uint64_t)plen << 40);
  uint64_t w3 = ((uint64_t)plen >> 24) | ((uint64_t)plen << 8);
  auto r64 = [&](uint32_t o) -> uint64_t {  // LE u64 at byte o of w0..w3 (o <= 24)
    const uint32_t q = o >> 3, sft = (o & 7) * 8;
    const uint64_t a = q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : w3;
    const uint64_t b = q == 0 ? w1 : q == 1 ? w2 : q == 2 ? w3 : 0;
    return sft ? (a >> sft) | (b << (64 - sft)) : a;
  };
  auto r8 = [&](uint32_t o) -> uint32_t { return (uint32_t)(r64(o) & 0xFF); };
  uint64_t hlo, hhi;
  xxh3_128_short(29, r8, r64, hlo, hhi);
  const int lane = threadIdx.x & 63;
  if (lane < 29) dst[hp + lane] = (uint8_t)r8(lane);
  else if (lane < 33) dst[hp + lane] = (uint8_t)((uint32_t)hlo >> (8 * (lane - 29)));
}

// ------------------------------------------------------ E2: LDS write pass
__global__ __launch_bounds__(64) void encode_write_kernel(EncodeParams P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const BlockPlan pl = P.plans[b];
  const uint32_t flags = pl.step_flags >> 8, step = pl.step_flags & 0xFF;
  if (flags) return;  // large (E3) or rejected
  const uint64_t dst_off = P.block_off[b], dst_end = P.block_off[b + 1];
  if (dst_end > P.out_cap) {
    if (lane == 0) P.status[b] = ST_OVERFLOW;
    return;
  }
  const uint32_t s = P.starts[b], e = P.starts[b + 1], n = e - s;
  const uint32_t ri = is_index(P) ? 1 : P.ri;
  const uint32_t total = (uint32_t)(dst_end - dst_off);
  const uint32_t plen = total - kHdrLen;

  // ---- LDS layout: [keys span][vals span][image][hash lo][hash hi]
  const uint64_t ka = (uint64_t)(uintptr_t)P.it.keys + P.it.key_off[s];
  const uint64_t kb = (uint64_t)(uintptr_t)P.it.keys + P.it.key_off[e];
  const uint64_t k0 = ka & ~15ULL;
  const uint32_t kbytes = (uint32_t)(((kb + 15) & ~15ULL) - k0);
  uint8_t* kimg = smem;
  uint32_t cur = kbytes + 32;
  uint8_t* vimg = smem + cur;
  uint64_t v0 = 0;
  uint32_t vbytes = 0;
  if (!is_index(P)) {
    const uint64_t va = (uint64_t)(uintptr_t)P.it.vals + P.it.val_off[s];
    const uint64_t vb = (uint64_t)(uintptr_t)P.it.vals + P.it.val_off[e];
    v0 = va & ~15ULL;
    vbytes = (uint32_t)(((vb + 15) & ~15ULL) - v0);
    cur += vbytes + 32;
  }
  uint8_t* img = smem + cur;
  const uint64_t dabs = (uint64_t)(uintptr_t)P.out + dst_off;
  const uint32_t pad = (uint32_t)(dabs & 15);
  cur += ((pad + total + 15) & ~15u) + 32;
  uint32_t* hlo = reinterpret_cast<uint32_t*>(smem + cur);
  uint32_t* hhi = hlo + ((pl.hash_w + 3) & ~3u);

  // ---- stage key / value spans HBM -> LDS
  {
    const u32x4* src = reinterpret_cast<const u32x4*>(k0);
    u32x4* dst = reinterpret_cast<u32x4*>(kimg);
    for (uint32_t c = lane; c < (kbytes >> 4); c += kWave) dst[c] = src[c];
    if (vbytes) {
      const u32x4* vs = reinterpret_cast<const u32x4*>(v0);
      u32x4* vd = reinterpret_cast<u32x4*>(vimg);
      uint32_t c = lane;
      for (; c + 3 * kWave < (vbytes >> 4); c += 4 * kWave) {
        u32x4 a0 = vs[c], a1 = vs[c + kWave], a2 = vs[c + 2 * kWave], a3 = vs[c + 3 * kWave];
        vd[c] = a0; vd[c + kWave] = a1; vd[c + 2 * kWave] = a2; vd[c + 3 * kWave] = a3;
      }
      for (; c < (vbytes >> 4); c += kWave) vd[c] = vs[c];
    }
    for (uint32_t k = lane; k < pl.hash_w; k += kWave) {
      hlo[k] = 0xFFFFFFFFu;
      hhi[k] = 0;
    }
  }
  __syncthreads();
  ItemSrc src;
  src.kbase = kimg;
  src.kshift = k0 - (uint64_t)(uintptr_t)P.it.keys;
  src.vbase = vimg;
  src.vshift = v0 - (uint64_t)(uintptr_t)P.it.vals;
  const uint32_t p0 = pad + kHdrLen;  // payload start in the image
  const uint32_t bin_off = pl.recs + 1;

  // ---- records (+ binary index entries, hash-index votes)
  uint32_t carry = 0;
  for (uint32_t c = 0; c < n; c += kWave) {
    const uint32_t j = c + lane;
    uint32_t rec = 0;
    uint64_t i = (uint64_t)s + j;
    if (j < n) {
      bool bad = false;
      const uint32_t klen = (uint32_t)(P.it.key_off[i + 1] - P.it.key_off[i]);
      rec = (uint32_t)record_len(P, i, j, klen, is_index(P) ? 0 : P.shared[i], bad);
    }
    const uint32_t incl = wave_incl_scan_u32(rec);
    const uint32_t roff = carry + incl - rec;
    if (j < n) {
      write_record(P, src, i, j, ri, img, p0 + roff);
      if (j % ri == 0) store_le(img, p0 + bin_off + (j / ri) * step, roff, step);
      if (pl.hash_w) {
        const uint32_t bk = key_bucket(src, P, i, pl.hash_w);
        const uint32_t ridx = j / ri;
        atomicMin(&hlo[bk], ridx);
        atomicMax(&hhi[bk], ridx);
      }
    }
    carry += wave_bcast_u32(incl, 63);
  }
  __syncthreads();
  if (lane == 0) img[p0 + pl.recs] = kTrailerMarker;
  const uint32_t hash_off = pl.hash_w ? bin_off + pl.bin_len * step : 0;
  for (uint32_t k = lane; k < pl.hash_w; k += kWave) img[p0 + hash_off + k] = (uint8_t)bucket_byte(hlo[k], hhi[k]);
  write_trailer_bytes(img, p0 + plen - kTrailerLen, ri, step, pl.bin_len, bin_off, pl.hash_w, hash_off, n);
  __syncthreads();
  // ---- fused checksum + header
  uint64_t ck_lo, ck_hi;
  xxh3_128_wave(img, p0, plen, &kLongSecret, ck_lo, ck_hi);
  write_header_bytes(img, pad, P.type, ck_lo, ck_hi, plen);
  __syncthreads();
  // ---- image -> HBM (16 B per lane; the two edge granules byte-wise)
  const uint32_t chunks = (pad + total + 15) >> 4;
  uint8_t* gdst = reinterpret_cast<uint8_t*>(dabs & ~15ULL);
  for (uint32_t c = lane; c < chunks; c += kWave) {
    const uint32_t lo = c * 16, hi = lo + 16;
    if (lo >= pad && hi <= pad + total) {
      reinterpret_cast<u32x4*>(gdst)[c] = reinterpret_cast<const u32x4*>(img)[c];
    } else {
      for (uint32_t k = max(lo, pad); k < min(hi, pad + total); ++k) gdst[k] = img[k];
    }
  }
  if (lane == 0) P.status[b] = ST_OK;
}

// ----------------------------------------------------- E3: HBM write pass
__global__ __launch_bounds__(64) void encode_large_kernel(EncodeParams P) {
  __shared__ uint32_t hlo[kE3HashChunk], hhi[kE3HashChunk];
  const int lane = threadIdx.x;
  const uint32_t count = *P.large_count;
  for (uint32_t li = blockIdx.x; li < count; li += gridDim.x) {
    const uint32_t b = P.large_list[li];
    const BlockPlan pl = P.plans[b];
    const uint32_t step = pl.step_flags & 0xFF;
    const uint64_t dst_off = P.block_off[b], dst_end = P.block_off[b + 1];
    if (dst_end > P.out_cap) {
      if (lane == 0) P.status[b] = ST_OVERFLOW;
      continue;
    }
    const uint32_t s = P.starts[b], e = P.starts[b + 1], n = e - s;
    const uint32_t ri = is_index(P) ? 1 : P.ri;
    const uint32_t total = (uint32_t)(dst_end - dst_off);
    const uint32_t plen = total - kHdrLen;
    const uint64_t dabs = (uint64_t)(uintptr_t)P.out + dst_off;
    uint8_t* img = reinterpret_cast<uint8_t*>(dabs & ~15ULL);
    const uint32_t pad = (uint32_t)(dabs & 15);
    const uint32_t p0 = pad + kHdrLen;
    const uint32_t bin_off = pl.recs + 1;
    ItemSrc src;
    src.kbase = P.it.keys; src.kshift = 0; src.vbase = P.it.vals; src.vshift = 0;
    uint32_t carry = 0;
    for (uint32_t c = 0; c < n; c += kWave) {
      const uint32_t j = c + lane;
      uint32_t rec = 0;
      const uint64_t i = (uint64_t)s + j;
      if (j < n) {
        bool bad = false;
        const uint32_t klen = (uint32_t)(P.it.key_off[i + 1] - P.it.key_off[i]);
        rec = (uint32_t)record_len(P, i, j, klen, is_index(P) ? 0 : P.shared[i], bad);
      }
      const uint32_t incl = wave_incl_scan_u32(rec);
      const uint32_t roff = carry + incl - rec;
      if (j < n) {
        write_record(P, src, i, j, ri, img, p0 + roff);
        if (j % ri == 0) store_le(img, p0 + bin_off + (j / ri) * step, roff, step);
      }
      carry += wave_bcast_u32(incl, 63);
    }
    const uint32_t hash_off = pl.hash_w ? bin_off + pl.bin_len * step : 0;
    for (uint32_t base = 0; base < pl.hash_w; base += kE3HashChunk) {
      const uint32_t lim = min(kE3HashChunk, pl.hash_w - base);
      for (uint32_t k = lane; k < lim; k += kWave) { hlo[k] = 0xFFFFFFFFu; hhi[k] = 0; }
      __syncthreads();
      for (uint32_t j = lane; j < n; j += kWave) {
        const uint32_t bk = key_bucket(src, P, (uint64_t)s + j, pl.hash_w);
        if (bk >= base && bk < base + lim) {
          atomicMin(&hlo[bk - base], j / ri);
          atomicMax(&hhi[bk - base], j / ri);
        }
      }
      __syncthreads();
      for (uint32_t k = lane; k < lim; k += kWave) img[p0 + hash_off + base + k] = (uint8_t)bucket_byte(hlo[k], hhi[k]);
      __syncthreads();
    }
    if (lane == 0) img[p0 + pl.recs] = kTrailerMarker;
    write_trailer_bytes(img, p0 + plen - kTrailerLen, ri, step, pl.bin_len, bin_off, pl.hash_w, hash_off, n);
    __threadfence();  // make this wave's HBM writes visible to its own re-reads below
    __syncthreads();
    uint64_t ck_lo, ck_hi;
    xxh3_128_wave(img, p0, plen, &kLongSecret, ck_lo, ck_hi);
    write_header_bytes(img, pad, P.type, ck_lo, ck_hi, plen);
    if (lane == 0) P.status[b] = ST_OK;
    __syncthreads();
  }
}

struct BlockOffOut {
  uint64_t* off;
  __device__ void operator()(uint64_t i, uint64_t prefix) const { off[i] = prefix; }
};

static size_t al256(size_t x) { return (x + 255) / 256 * 256; }

size_t encode_workspace_size(uint64_t n_items, uint32_t n_blocks) {
  return al256(n_items * 2) + al256((size_t)n_blocks * 8) + al256((size_t)n_blocks * sizeof(BlockPlan)) +
         al256((size_t)n_blocks * 4) + 256 + al256(scan_tiles(n_blocks) * 8);
}

uint64_t encode_bound(uint64_t n_items, uint32_t n_blocks, uint64_t key_bytes, uint64_t val_bytes,
                      const lsm_block_params* params) {
  const float ratio = params ? params->hash_ratio : 0.0f;
  uint64_t hash = 0;
  if (ratio > 0.0f) hash = (uint64_t)ceil((double)n_items * (double)ratio) + n_blocks;
  return 29ULL * n_items + key_bytes + val_bytes + 4ULL * n_items + hash +
         (uint64_t)n_blocks * (kHdrLen + 1 + kTrailerLen + 16) + 64;
}

hipError_t launch_encode(const lsm_items& items, const uint32_t* starts, uint32_t n_blocks,
                         const lsm_block_params& params, uint8_t* out, uint64_t out_cap, uint64_t* block_off,
                         int32_t* status, void* ws, hipStream_t st) {
  EncodeParams P;
  P.it = items;
  P.starts = starts;
  P.n_blocks = n_blocks;
  P.ri = params.block_type == 1 ? 1 : params.restart_interval;
  P.ratio = params.block_type == 1 ? 0.0f : params.hash_ratio;
  P.type = params.block_type;
  P.out = out;
  P.out_cap = out_cap;
  P.block_off = block_off;
  P.status = status;
  uint8_t* w = (uint8_t*)ws;
  P.shared = (uint16_t*)w; w += al256(items.n_items * 2);
  P.sizes = (uint64_t*)w; w += al256((size_t)n_blocks * 8);
  P.plans = (BlockPlan*)w; w += al256((size_t)n_blocks * sizeof(BlockPlan));
  P.large_list = (uint32_t*)w; w += al256((size_t)n_blocks * 4);
  P.large_count = (uint32_t*)w; w += 256;
  uint64_t* tiles = (uint64_t*)w;
  hipError_t e = hipMemsetAsync(P.large_count, 0, 16, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(encode_sizes_kernel, dim3((n_blocks + 3) / 4), dim3(256), 0, st, P);
  e = launch_excl_scan(P.sizes, n_blocks, tiles, BlockOffOut{block_off}, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(encode_write_kernel, dim3(n_blocks), dim3(64), kE2Budget, st, P);
  hipLaunchKernelGGL(encode_large_kernel, dim3(1024), dim3(64), 0, st, P);
  return hipGetLastError();
}

}  // namespace lsmgpu
