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

// ---------------------------------------------------------------- fast path
// The common record header (vtype, seqno <= 7 LEB bytes, shared <= 3 LEB
// bytes, 1-byte key length) lies in the 8 bytes at the record start, read as
// aligned dwords + v_alignbyte (measured faster than unaligned ds_read_b64 /
// b128 on gfx950) and decoded with bit tricks, then one dependent read at
// start + header + key length for a 1-2 byte value length.  Any other shape
// (seqno >= 2^49, key length >= 128, value length >= 2^14) takes the Cursor.
// Loads may run up to 138 bytes past the record start; callers guarantee that
// many readable bytes (LDS stage padding) or clamp (see parse_data_fast).
__device__ __forceinline__ uint64_t leb_val8(uint64_t x, uint32_t n) {  // n in 1..8
  if (n < 8) x &= (1ULL << (8 * n)) - 1;
  x = ((x & 0x7F007F007F007F00ULL) >> 1) | (x & 0x007F007F007F007FULL);
  x = ((x & 0x3FFF00003FFF0000ULL) >> 2) | (x & 0x00003FFF00003FFFULL);
  x = ((x & 0x0FFFFFFF00000000ULL) >> 4) | (x & 0x000000000FFFFFFFULL);
  return x;
}
__device__ __forceinline__ uint32_t ctz64(uint64_t t) {  // 64 for t == 0
  return t ? (uint32_t)__builtin_ctzll(t) : 64u;
}

struct RecHead {
  uint32_t vt, hdr, klen, q, e1, e2;
  bool ok;  // header in the fast shape (vtype not checked)
};
__device__ __forceinline__ RecHead rec_head(uint64_t h, bool restart) {
  RecHead r;
  r.vt = (uint32_t)(h & 0xFF);
  // LEB terminators (MSB clear) among bytes 1..7: seqno, [shared], key length
  const uint64_t t1 = ~h & 0x8080808080808000ULL;
  r.e1 = ctz64(t1);
  const uint64_t t2 = t1 & (t1 - 1);
  r.e2 = restart ? r.e1 : ctz64(t2);
  const uint64_t t3 = restart ? t2 : t2 & (t2 - 1);
  const uint32_t e3 = ctz64(t3);
  r.ok = t3 != 0 && e3 - r.e2 == 8 && (restart || r.e2 - r.e1 <= 24);
  r.klen = (uint32_t)(h >> (r.ok ? e3 - 7 : 0)) & 0x7F;
  r.hdr = (e3 >> 3) + 1;
  r.q = r.hdr + r.klen;  // <= 136
  return r;
}
// two bytes at offset q (q <= 14) of the window, branch-free
__device__ __forceinline__ uint32_t win16_u16(const Win16& w, uint32_t q) {
  const uint32_t d0 = (uint32_t)w.lo, d1 = (uint32_t)(w.lo >> 32), d2 = (uint32_t)w.hi, d3 = (uint32_t)(w.hi >> 32);
  const uint32_t qi = q >> 2;
  const uint32_t lo = qi == 0 ? d0 : qi == 1 ? d1 : qi == 2 ? d2 : d3;
  const uint32_t hi = qi == 0 ? d1 : qi == 1 ? d2 : qi == 2 ? d3 : 0u;
  return alignbyte(hi, lo, q & 3) & 0xFFFF;
}
// value length from the two bytes at start + q; false = longer varint
__device__ __forceinline__ bool rec_vlen(uint32_t z, bool tomb, uint32_t& n4, uint32_t& vl) {
  const bool two = (z & 0x80) != 0;
  n4 = tomb ? 0 : (two ? 2 : 1);
  vl = tomb ? 0 : (two ? ((z & 0x7F) | ((z >> 1) & 0x3F80)) : (z & 0x7F));
  return tomb || (z & 0x8080) != 0x8080;
}

// Full record parse.  Returns 1 = parsed, 0 = Cursor path, -1 = malformed
// (same outcomes as oracle parse_data_item).  Payload-relative positions.
// Branch-free: both loads are unconditional (clamped to the marker, so they
// stay inside the block) and every field is computed before classifying.
__device__ __forceinline__ int parse_data_fast(const uint8_t* base, uint32_t p0, uint32_t pos, uint32_t end,
                                               bool restart, uint32_t base_key_off, ItemFields& f,
                                               uint32_t& next) {
  const uint64_t h = read_u64_unaligned(base, p0 + min(pos, end));  // >= 33 block bytes follow the marker
  const RecHead r = rec_head(h, restart);
  const bool tomb = is_tombstone(r.vt);
  const uint32_t z = read_u16_unaligned(base, p0 + min(pos + r.q, end));
  uint32_t n4, vl;
  const bool vl_ok = rec_vlen(z, tomb, n4, vl);
  const uint64_t seq = leb_val8(h >> 8, r.e1 >> 3);
  const uint32_t shared =
      restart ? 0u : (uint32_t)leb_val8(h >> min(r.e1 + 1, 63u), (r.e2 - r.e1) >> 3) & 0xFFFF;
  const uint32_t val_off = pos + r.q + n4;
  const bool bad = (pos + r.hdr > end) || (!restart && (uint64_t)base_key_off + shared > end) ||
                   (pos + r.q + n4 > end) || ((uint64_t)val_off + vl > end);
  f.seqno = seq;
  f.handle_off = 0;
  f.key_off = pos + r.hdr;
  f.key_len = (uint16_t)r.klen;
  f.prefix_len = (uint16_t)shared;
  f.val_off = val_off;
  f.val_len = vl;
  f.vtype = (uint8_t)r.vt;
  next = val_off + vl;
  const bool fast = r.ok && vl_ok;
  return (pos >= end || !valid_vtype(r.vt)) ? -1 : (!fast ? 0 : (bad ? -1 : 1));
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

// (mbase: where the marker byte before the binary index is read, when base is
// a staged copy of the trailer bytes only)
__device__ __forceinline__ int32_t read_trailer(const uint8_t* base, uint32_t p0, uint32_t plen,
                                                TrailerInfo& t, const uint8_t* mbase = nullptr) {
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
  if ((read_u32_unaligned(mbase ? mbase : base, p0 + t.bin_off - 1) & 0xFF) != kTrailerMarker) return ST_PARSE;
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
// Header fields and the structural checks before the header checksum
// (header.rs:116-169 order); check_header adds the checksum.
__device__ __forceinline__ int32_t check_header_fields(const uint8_t* base, uint32_t hb, uint64_t len,
                                                       HeaderInfo& h) {
  if (len < 4) return ST_TRUNCATED;
  const uint32_t magic = read_u32_unaligned(base, hb);
  if (magic != 0x034D534CU) return ST_BAD_MAGIC;  // "LSM\x03", file.rs:8
  if (len < 5) return ST_TRUNCATED;
  h.type = read_u32_unaligned(base, hb + 4) & 0xFF;
  if (h.type > 3) return ST_BAD_TYPE;
  if (len < kHdrLen) return ST_TRUNCATED;
  BaseReader64 r{base, hb};
  h.ck_lo = r(5);
  h.ck_hi = r(13);
  h.data_length = read_u32_unaligned(base, hb + 21);
  return ST_OK;
}
// header checksum: low 32 bits of xxh3_128 over the first 29 header bytes
__device__ __forceinline__ bool header_cksum_ok(const uint8_t* base, uint32_t hb) {
  uint64_t lo, hi;
  xxh3_128_short(29, BaseReader8{base, hb}, BaseReader64{base, hb}, lo, hi);
  return (uint32_t)lo == read_u32_unaligned(base, hb + 29);
}
__device__ __forceinline__ int32_t check_header(const uint8_t* base, uint32_t hb, uint64_t len,
                                                HeaderInfo& h) {
  const int32_t st = check_header_fields(base, hb, len, h);
  if (st != ST_OK) return st;
  return header_cksum_ok(base, hb) ? ST_OK : ST_HDR_CKSUM;
}

}  // namespace lsmgpu
