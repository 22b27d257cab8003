// block_format.hpp — device-side parsing of the v3 block format
// (header, trailer, DataBlock / IndexBlock records).
//
// Reference layout (fjall-rs/lsm-tree 3.1.9):
//   header   src/table/block/header.rs:49-169   [LSM\x03][type][xxh3_128 LE][data_len][uncomp_len][hdr_cksum]
//   trailer  src/table/block/trailer.rs:78-173  [ri][step][bin_len][bin_off][hash_len][hash_off][1][0][0u16][0][0u32][item_count]
//   records  src/table/data_block/mod.rs:27-191 (parse_full / parse_truncated)
//            src/table/index_block/block_handle.rs:175-206 (KeyedBlockHandle::parse_full)
// Validation rules are identical to oracle/block.c (the reference panics on
// malformed payloads; we return LSM_PARSE).
#pragma once

#include "device_common.hpp"

namespace lsmgpu {

struct ItemFields {
  uint64_t seqno;
  uint64_t handle_off;
  uint32_t key_off, val_off, val_len;
  uint16_t key_len, prefix_len;
  uint8_t vtype;
};

// Cursor over the record area [0, end) of a payload that starts at byte
// offset p0 of a 16-aligned base (LDS image or global span).  Keeps a
// 16-byte register window and refills it with one aligned LDS/global read
// burst when a field could straddle it.
struct Cursor {
  const uint8_t* base;
  uint32_t p0, pos, end, avail;
  Win16 w;

  __device__ __forceinline__ void init(const uint8_t* b, uint32_t payload0, uint32_t start, uint32_t rec_end) {
    base = b; p0 = payload0; pos = start; end = rec_end; avail = 0; w.lo = w.hi = 0;
  }
  __device__ __forceinline__ void refill() {
    w = read_win16(base, p0 + pos);
    avail = 16;
  }
  __device__ __forceinline__ void ensure(uint32_t need) {
    if (avail < need) refill();
  }
  __device__ __forceinline__ uint32_t left() const { return end - pos; }
  __device__ __forceinline__ bool byte(uint32_t& b) {
    if (pos >= end) return false;
    ensure(1);
    b = (uint32_t)(w.lo & 0xFF);
    win_shift(w, 1);
    avail -= 1;
    pos += 1;
    return true;
  }
  // varint-rs read_*_varint: at most max_bytes, value masked to the type width
  __device__ __forceinline__ bool varint(uint32_t max_bytes, uint64_t mask, uint64_t& v) {
    ensure(max_bytes);
    const uint32_t lim = min(max_bytes, left());
    const uint32_t n = leb_decode(w, max_bytes, lim, v);
    if (!n) return false;
    v &= mask;
    win_shift(w, n);
    avail -= n;
    pos += n;
    return true;
  }
  __device__ __forceinline__ bool skip(uint64_t n) {
    if (n > (uint64_t)left()) return false;
    if (n < avail) {
      win_shift(w, (uint32_t)n);
      avail -= (uint32_t)n;
    } else {
      avail = 0;
    }
    pos += (uint32_t)n;
    return true;
  }
};

__device__ __forceinline__ bool valid_vtype(uint32_t t) { return t == 0 || t == 1 || t == 2 || t == 4; }
__device__ __forceinline__ bool is_tombstone(uint32_t t) { return t == 1 || t == 2; }

// parse_full / parse_truncated, src/table/data_block/mod.rs:58-191.
__device__ __forceinline__ bool parse_data_record(Cursor& c, bool restart, uint32_t base_key_off,
                                                  ItemFields& f) {
  uint32_t vt;
  if (!c.byte(vt) || !valid_vtype(vt)) return false;  // 0xFF marker inside an interval -> error
  uint64_t seq, shared = 0, klen, vl = 0;
  if (!c.varint(10, ~0ULL, seq)) return false;
  if (!restart && !c.varint(3, 0xFFFF, shared)) return false;
  if (!c.varint(3, 0xFFFF, klen)) return false;
  const uint32_t key_off = c.pos;
  if (!restart && (uint64_t)base_key_off + shared > c.end) return false;
  if (!c.skip(klen)) return false;
  if (!is_tombstone(vt) && !c.varint(5, 0xFFFFFFFFULL, vl)) return false;
  const uint32_t val_off = c.pos;
  if (!c.skip(vl)) return false;
  f.seqno = seq;
  f.handle_off = 0;
  f.key_off = key_off;
  f.key_len = (uint16_t)klen;
  f.prefix_len = (uint16_t)shared;
  f.val_off = val_off;
  f.val_len = (uint32_t)vl;
  f.vtype = (uint8_t)vt;
  return true;
}

// KeyedBlockHandle::parse_full, src/table/index_block/block_handle.rs:175-206.
__device__ __forceinline__ bool parse_index_record(Cursor& c, ItemFields& f) {
  uint32_t m;
  if (!c.byte(m) || m != 0) return false;
  uint64_t off, size, seq, klen;
  if (!c.varint(10, ~0ULL, off)) return false;
  if (!c.varint(5, 0xFFFFFFFFULL, size)) return false;
  if (!c.varint(10, ~0ULL, seq)) return false;
  if (!c.varint(3, 0xFFFF, klen)) return false;
  const uint32_t key_off = c.pos;
  if (!c.skip(klen)) return false;
  f.seqno = seq;
  f.handle_off = off;
  f.key_off = key_off;
  f.key_len = (uint16_t)klen;
  f.prefix_len = 0;
  f.val_off = c.pos;
  f.val_len = (uint32_t)size;
  f.vtype = 0;
  return true;
}

// Parsed trailer (trailer.rs:118-163) + the structural checks of oracle read_trailer.
struct TrailerInfo {
  uint32_t ri, step, bin_len, bin_off, hash_len, hash_off, item_count, rec_end;
};

__device__ __forceinline__ int32_t read_trailer(const uint8_t* base, uint32_t p0, uint32_t plen,
                                                TrailerInfo& t) {
  if (plen < kTrailerLen + 1) return ST_PARSE;
  const uint32_t tp = p0 + plen - kTrailerLen;
  const uint32_t w0 = read_u32_unaligned(base, tp);
  t.ri = w0 & 0xFF;
  t.step = (w0 >> 8) & 0xFF;
  t.bin_len = read_u32_unaligned(base, tp + 2);
  t.bin_off = read_u32_unaligned(base, tp + 6);
  t.hash_len = read_u32_unaligned(base, tp + 10);
  t.hash_off = read_u32_unaligned(base, tp + 14);
  t.item_count = read_u32_unaligned(base, tp + 27);
  if (t.ri == 0 || (t.step != 2 && t.step != 4) || t.bin_len == 0 || t.bin_off == 0) return ST_PARSE;
  if ((uint64_t)t.bin_off + (uint64_t)t.bin_len * t.step > (uint64_t)(plen - kTrailerLen)) return ST_PARSE;
  if ((read_u32_unaligned(base, p0 + t.bin_off - 1) & 0xFF) != kTrailerMarker) return ST_PARSE;
  if ((uint64_t)t.bin_len != ((uint64_t)t.item_count + t.ri - 1) / t.ri) return ST_PARSE;
  t.rec_end = t.bin_off - 1;
  return ST_OK;
}

__device__ __forceinline__ uint32_t bin_get(const uint8_t* base, uint32_t p0, const TrailerInfo& t,
                                            uint32_t i) {  // binary_index/reader.rs:30-48
  const uint32_t q = p0 + t.bin_off + i * t.step;
  const uint32_t v = read_u32_unaligned(base, q);
  return t.step == 2 ? (v & 0xFFFF) : v;
}

// Header::decode_from (header.rs:116-169) on base[hb .. hb+len).  On success
// fills the payload checksum, type and data_length.
struct HeaderInfo {
  uint64_t ck_lo, ck_hi;
  uint32_t data_length;
  uint32_t type;
};
__device__ __forceinline__ int32_t check_header(const uint8_t* base, uint32_t hb, uint64_t len,
                                                HeaderInfo& h) {
  if (len < 4) return ST_TRUNCATED;
  const uint32_t magic = read_u32_unaligned(base, hb);
  if (magic != 0x034D534CU) return ST_BAD_MAGIC;  // "LSM\x03", file.rs:8
  if (len < 5) return ST_TRUNCATED;
  h.type = read_u32_unaligned(base, hb + 4) & 0xFF;
  if (h.type > 3) return ST_BAD_TYPE;
  if (len < kHdrLen) return ST_TRUNCATED;
  uint64_t lo, hi;
  xxh3_128_short(29, BaseReader8{base, hb}, BaseReader64{base, hb}, lo, hi);
  if ((uint32_t)lo != read_u32_unaligned(base, hb + 29)) return ST_HDR_CKSUM;
  BaseReader64 r{base, hb};
  h.ck_lo = r(5);
  h.ck_hi = r(13);
  h.data_length = read_u32_unaligned(base, hb + 21);
  return ST_OK;
}

}  // namespace lsmgpu
