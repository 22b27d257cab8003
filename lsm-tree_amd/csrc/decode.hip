// decode.hip — batched SST block decode on gfx950 (the north-star hot path).
//
// Replaces, per block, Block::from_file (header decode + xxh3_128 verify,
// src/table/block/mod.rs:131-182), the load_block type check
// (src/table/util.rs:79-86) and the full forward DataBlock::iter() /
// IndexBlock::iter() (src/table/block/decoder.rs:442-483) over a whole batch.
//
// Launch shape: 4-wave workgroups, four per CU.  Workgroup w
// owns blocks [w*BPW, (w+1)*BPW) and walks them in GROUPS — the longest run of
// consecutive blocks that fits the 33.75 KiB LDS stage (consecutive blocks are
// contiguous on disk, so a group is one contiguous span):
//   1. lane j of every wave holds block j's handle and item range;
//   2. all waves copy the span HBM -> LDS with global_load_lds_dwordx4;
//   3. wave 0: lane j checks block j's header fields and trailer, a wave scan
//      numbers the restart intervals of the group;
//   4. phase A on one wave (lane = restart interval) walks record boundaries
//      only, while the other waves verify the payload xxh3_128 (16-lane DPP
//      rows) and the header checksums;
//   5. phase B on all waves (thread = record) parses and validates every
//      field and stores the parsed-item SoA with coalesced global stores.
// Blocks larger than the stage, index blocks and rare record shapes go to
// decode_deferred_staged_kernel (one block per 4-wave workgroup, LEB cursor).
#include <hip/hip_runtime.h>

#include "block_format.hpp"
#include "decode.hpp"
#include "fill.hpp"
#include "lds_dma.hpp"
#include "scan.hpp"

namespace lsmgpu {

// Diagnostic-only flags (lsm_decode_tuning.flags high bits, honoured only by
// -DLSM_DIAG builds; the release library rejects them with LSM_BAD_ARG): drop
// one phase to price it in a profile.  Outputs are NOT valid with them set.

// (16 blocks x 80 B of block metadata: the LDS this frees lets the stage hold
// two 17 KB blocks of the 16 KiB random-key class, or nine 4 KiB blocks,
// inside the 40 KiB that keeps four workgroups per CU)
constexpr uint32_t kMaxGroup = 16;  // blocks per staged group
// Internal status: the block needs the general path (index block, a record
// shape the straight-line parsers do not take, a block larger than the
// stage).  The group kernel lists it for decode_big_kernel, which hands on
// what it cannot take (index blocks, rare shapes, blocks beyond its stage) to
// decode_deferred_staged_kernel, the general path with the LEB cursor; that
// one writes the final status.
constexpr int32_t ST_DEFER = 0x7F;
constexpr uint32_t kStagePad = 256;  // readable LDS bytes past the span (fast parsers read <= 138)

// Record descriptor (one u64 per group item, LDS), written by phase A, read
// by phase B: image offsets of the record start, of where it must end (the
// next record's start, or the interval's end for its last record) and of its
// restart head's key; [48,53) group block, 53 restart head, 54 valid,
// [55,58) seqno bytes and [58,60) shared bytes of a header shape phase A has
// verified (0 = not verified: phase B decodes the header itself).
// Two layouts: kWide = false for stages < 64 KiB (16-bit image offsets),
// kWide = true for the big-block kernel's stage (17-bit offsets; the end is
// kept as its distance from the start, clamped to 2^15 - 1: longer than any
// record the straight-line parsers take, so a clamped end can only mismatch).
template <bool kWide>
struct RecLayout {
  static constexpr int kPosBits = kWide ? 17 : 16;
  static constexpr uint32_t kPosMask = (1u << kPosBits) - 1;
  static constexpr int kKeyShift = 32, kBlockShift = 32 + kPosBits;
  static constexpr uint64_t kRestart = 1ULL << (kBlockShift + 5), kValid = 1ULL << (kBlockShift + 6);
  static constexpr int kN1Shift = kBlockShift + 7, kN2Shift = kBlockShift + 10;
  __device__ static __forceinline__ uint32_t lo(uint32_t a, uint32_t end) {
    return kWide ? a | (min(end - a, 0x7FFFu) << 17) : a | (end << 16);
  }
  __device__ static __forceinline__ uint32_t start(uint64_t d) { return (uint32_t)d & kPosMask; }
  __device__ static __forceinline__ uint32_t end(uint64_t d) {
    return kWide ? ((uint32_t)d & kPosMask) + (((uint32_t)d >> 17) & 0x7FFF) : (uint32_t)d >> 16;
  }
};
static_assert(RecLayout<true>::kN2Shift + 2 <= 64 && RecLayout<false>::kN2Shift + 2 <= 64, "descriptor bits");

struct alignas(16) BlockMeta {
  // first 16 bytes: what phase B needs per record (one ds_read_b128)
  uint32_t p0;        // image / span offset of the payload (header offset + 33)
  uint32_t rec_end;   // image / span offset of the 0xFF trailer marker
  int32_t st;         // lsm_status
  uint32_t type;
  uint64_t ck_lo, ck_hi;
  uint32_t hb;        // byte offset of the header in the image / span
  uint32_t len;       // handle size (header + payload)
  uint32_t ri, step, bin_len, bin_off, item_count;
  uint32_t item0;     // first output index relative to the group base
  uint32_t chain0;    // exclusive prefix of restart intervals in the group
  int32_t hdr_st;     // header-level status before the header checksum (gates hashing)
  uint16_t ck_bad;    // payload checksum mismatch
  uint16_t hck_bad;   // header checksum mismatch
};
static_assert(sizeof(BlockMeta) == 80, "BlockMeta layout");

// The kernel's DecodeParams in the kernarg segment.  Out-of-line helpers take
// this pointer: taking the address of the by-value kernel parameter instead
// makes the compiler copy it to scratch and reload its fields from there
// (vmcnt waits in the hot loops).
typedef const __attribute__((address_space(4))) DecodeParams* KArgs;
__device__ __forceinline__ KArgs kargs() { return (KArgs)__builtin_amdgcn_kernarg_segment_ptr(); }
__device__ __forceinline__ DecodeParams load_params(KArgs Pk) {
  DecodeParams P;
  __builtin_memcpy(&P, (const void*)Pk, sizeof(P));
  return P;
}

__device__ __forceinline__ void wave_sync() {
  // Single-wave workgroups: LDS operations of a wave complete in order, so a
  // compiler barrier is all cross-lane LDS hand-offs need (no s_barrier, and
  // no vmcnt(0) drain of the output stores as __syncthreads would imply).
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops
// (lgkmcnt), not for its global stores, which __syncthreads' release fence
// would drain (vmcnt(0)) before every phase.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// compact (lsm_decode_blocks16): key_off / val_off / val_len are uint16_t
// arrays; every block that reaches a store has a payload <= 65535 bytes
// (meta_trailer), so the payload-relative values fit.
__device__ __forceinline__ void emit_global(const lsm_parsed_items& o, uint64_t i, const ItemFields& f,
                                            uint64_t seqno_add, bool compact) {
  if (o.seqno) gstore(o.seqno, i, f.seqno + seqno_add);
  if (compact) {
    if (o.key_off) gstore(reinterpret_cast<uint16_t*>(o.key_off), i, (uint16_t)f.key_off);
    if (o.val_off) gstore(reinterpret_cast<uint16_t*>(o.val_off), i, (uint16_t)f.val_off);
    if (o.val_len) gstore(reinterpret_cast<uint16_t*>(o.val_len), i, (uint16_t)f.val_len);
  } else {
    if (o.key_off) gstore(o.key_off, i, f.key_off);
    if (o.val_off) gstore(o.val_off, i, f.val_off);
    if (o.val_len) gstore(o.val_len, i, f.val_len);
  }
  if (o.key_len) gstore(o.key_len, i, f.key_len);
  if (o.prefix_len) gstore(o.prefix_len, i, f.prefix_len);
  if (o.vtype) gstore(o.vtype, i, f.vtype);
  if (o.handle_off) gstore(o.handle_off, i, f.handle_off);
}

// Lane-level: header checks in oracle order (header.rs:116-169).
__device__ __forceinline__ void meta_header(const uint8_t* base, uint32_t hb, uint64_t len, BlockMeta& m) {
  HeaderInfo h;
  m.hb = hb;
  m.p0 = hb + kHdrLen;
  m.rec_end = 0;
  m.len = (uint32_t)len;
  m.st = (len > 0xFFFFFF00ULL) ? ST_TRUNCATED : check_header(base, hb, len, h);
  m.ck_lo = h.ck_lo;
  m.ck_hi = h.ck_hi;
  m.type = h.type;
  m.item_count = h.data_length;  // stash data_length until meta_trailer
  m.chain0 = 0;
}

// Staged kernel: the same without the header checksum (the hash waves check it).
__device__ __forceinline__ void meta_header_fields(const uint8_t* base, uint32_t hb, uint64_t len, BlockMeta& m) {
  HeaderInfo h;
  m.hb = hb;
  m.p0 = hb + kHdrLen;
  m.rec_end = 0;
  m.len = (uint32_t)len;
  m.st = (len > 0xFFFFFF00ULL) ? ST_TRUNCATED : check_header_fields(base, hb, len, h);
  m.ck_lo = h.ck_lo;
  m.ck_hi = h.ck_hi;
  m.type = h.type;
  m.item_count = h.data_length;  // stash data_length until meta_trailer
  m.chain0 = 0;
}

// After the payload checksum: data_length, expected type, trailer structure.
// compact output (lsm_decode_blocks16): index blocks (u64 handle offsets) and
// payloads over 65535 bytes cannot be stored in 16 bits: LSM_UNSUPPORTED,
// decided here, after every header check and before the trailer is read.
__device__ __forceinline__ void meta_trailer(const uint8_t* base, int32_t expect_type, uint32_t cap, BlockMeta& m,
                                             bool compact, const uint8_t* mbase = nullptr) {
  if (m.st != ST_OK) return;
  const uint32_t plen = m.len - kHdrLen;
  if (m.item_count != plen) { m.st = ST_TRUNCATED; return; }   // data_length vs handle
  if (expect_type >= 0 && (int32_t)m.type != expect_type) { m.st = ST_TYPE_MISMATCH; return; }
  if (m.type == 2) { m.st = ST_UNSUPPORTED; return; }          // filter blocks are not KV blocks
  if (compact && (m.type == 1 || plen > 0xFFFFu)) { m.st = ST_UNSUPPORTED; return; }
  TrailerInfo t;
  int32_t st = read_trailer(base, m.hb + kHdrLen, plen, t, mbase);
  if (st == ST_OK && m.type == 1 && t.ri != 1) st = ST_PARSE;   // index blocks: restart interval 1
  if (st == ST_OK && t.item_count > cap) st = ST_OVERFLOW;
  m.st = st;
  if (st != ST_OK) return;
  m.ri = t.ri; m.step = t.step; m.bin_len = t.bin_len; m.bin_off = t.bin_off;
  m.item_count = t.item_count; m.rec_end = m.p0 + t.rec_end;
}

__device__ __forceinline__ TrailerInfo trailer_of(const BlockMeta& m) {
  TrailerInfo t;
  t.ri = m.ri; t.step = m.step; t.bin_len = m.bin_len; t.bin_off = m.bin_off;
  t.item_count = m.item_count; t.rec_end = m.rec_end - m.p0;
  t.hash_len = 0; t.hash_off = 0;
  return t;
}

// Rare record shapes (long varints) through the general LEB cursor; kept out
// of line so the hot loops stay small in the instruction cache.
__device__ __noinline__ bool parse_data_slow(const uint8_t* base, uint32_t p0, uint32_t pos, uint32_t end,
                                             bool restart, uint32_t base_key, ItemFields* f, uint32_t* next) {
  Cursor c;
  c.init(base, p0, pos, end);
  if (!parse_data_record(c, restart, base_key, *f)) return false;
  *next = c.pos;
  return true;
}
__device__ __noinline__ bool parse_index_slow(const uint8_t* base, uint32_t p0, uint32_t pos, uint32_t end,
                                              ItemFields* f, uint32_t* next) {
  Cursor c;
  c.init(base, p0, pos, end);
  if (!parse_index_record(c, *f)) return false;
  *next = c.pos;
  return true;
}

// Full parse of one record at pos; returns next position or false.
__device__ __forceinline__ bool parse_record(const uint8_t* base, uint32_t p0, uint32_t pos, const TrailerInfo& t,
                                             uint32_t type, bool restart, uint32_t base_key, ItemFields& f,
                                             uint32_t& next) {
  ItemFields tmp;  // only the out-of-line paths take an address (keeps f in registers)
  uint32_t tnext;
  bool ok;
  if (type == 1) {
    ok = parse_index_slow(base, p0, pos, t.rec_end, &tmp, &tnext);
  } else {
    const int rc = parse_data_fast(base, p0, pos, t.rec_end, restart, base_key, f, next);
    if (rc > 0) return true;
    if (rc < 0) return false;
    ok = parse_data_slow(base, p0, pos, t.rec_end, restart, base_key, &tmp, &tnext);
  }
  f = tmp;
  next = tnext;
  return ok;
}

// Out-of-line record walk that returns in registers (no address-taken
// locals: results passed through scratch would put vmcnt waits — which also
// drain the output stores — on the hot loops).  0 = malformed, else
// bit 63 | key_off << 32 | next (payload-relative).
__device__ __noinline__ uint64_t data_slow_next(const uint8_t* base, uint32_t p0, uint32_t pos, uint32_t end,
                                                bool restart, uint32_t base_key) {
  Cursor c;
  c.init(base, p0, pos, end);
  ItemFields f;
  if (!parse_data_record(c, restart, base_key, f)) return 0;
  return (1ULL << 63) | ((uint64_t)f.key_off << 32) | c.pos;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

template <class RL>
__device__ __forceinline__ uint64_t rec_desc(uint32_t a, uint32_t end, uint32_t key, uint64_t tag) {
  return (uint64_t)RL::lo(a, end) | ((uint64_t)key << RL::kKeyShift) | tag;
}

// Predicted header shape of a non-restart record: n1 seqno bytes, n2 shared
// bytes, 1 key-length byte.  msk = MSB bits of header bytes 1..hdr-1, pat =
// where their LEB terminators must be; a record matches iff (~h & msk) == pat.
struct Shape {
  uint32_t hdr, kshift;
  uint64_t msk, pat;
  uint64_t bits;  // descriptor shape bits
};
template <class RL>
__device__ __forceinline__ Shape make_shape(uint32_t n1, uint32_t n2) {
  Shape s;
  s.bits = ((uint64_t)n1 << RL::kN1Shift) | ((uint64_t)n2 << RL::kN2Shift);
  s.hdr = n1 + n2 + 2;  // <= 8
  s.kshift = 8 * (s.hdr - 1);
  s.msk = 0x8080808080808000ULL & (s.hdr >= 8 ? ~0ULL : ((1ULL << (8 * s.hdr)) - 1));
  s.pat = (0x80ULL << (8 * n1)) | (0x80ULL << (8 * (n1 + n2))) | (0x80ULL << (8 * (s.hdr - 1)));
  return s;
}

// Value length from the two bytes z after the key; ok = 1-2 byte varint.
__device__ __forceinline__ void rec_value(uint32_t vt, uint32_t z, uint32_t& n4, uint32_t& vl, bool& ok) {
  const bool tomb = vt - 1u < 2u;
  const bool two = (z & 0x80) != 0;
  ok = tomb || (z & 0x8080) != 0x8080;
  n4 = tomb ? 0 : (two ? 2 : 1);
  vl = tomb ? 0 : (two ? ((z & 0x7F) | ((z >> 1) & 0x3F80)) : (z & 0x7F));
}

// Record length from the key length and the two bytes z after the key
// (1-2 byte value length; tombstones carry none).
__device__ __forceinline__ uint32_t rec_len(uint32_t vt, uint32_t q, uint32_t z) {
  const bool tomb = vt - 1u < 2u;
  const bool two = (z & 0x80) != 0;
  const uint32_t vl = two ? ((z & 0x7F) | ((z >> 1) & 0x3F80)) : (z & 0x7F);
  return q + (tomb ? 0u : vl + 1u + (two ? 1u : 0u));
}

// Phase A: lane = restart interval.  Walks record BOUNDARIES only and writes
// one descriptor per record; phase B parses every record in full and checks
// that it ends exactly where its descriptor says, so a boundary computed
// here from a malformed record can only turn into a PARSE status.  The step
// is kept short because it runs as one wave's serial instruction stream:
// the key length is read at the PREDICTED header length (the previous
// record's shape, checked with one mask compare) and the value length from
// the same 16-byte LDS window; only a shape change, a long key suffix or a
// long varint leaves the straight path.  The loop is wave-uniform: lanes
// past their interval's end store to rec[dummy].
template <bool kWide = false>
__device__ __forceinline__ void phase_a(const uint8_t* img, BlockMeta* meta, const uint8_t* owner, uint64_t* rec,
                                        uint32_t c_first, uint32_t c_step, uint32_t total, uint32_t dummy) {
  typedef RecLayout<kWide> RL;
  const int lane = threadIdx.x & (kWave - 1);
  for (uint32_t c0 = c_first; c0 < total; c0 += c_step) {
    const uint32_t c = c0 + lane;
    const bool live = c < total;
    const uint32_t j = live ? owner[c] : 0;
    const BlockMeta& m = meta[j];
    const TrailerInfo t = trailer_of(m);
    const uint32_t p0 = m.p0, rec_end = m.rec_end;
    const uint32_t r = live ? c - m.chain0 : 0;
    const bool last_iv = r + 1 == t.bin_len;
    const uint32_t s_rel = bin_get(img, p0, t, r);
    const uint32_t e_rel = last_iv ? t.rec_end : bin_get(img, p0, t, r + 1);
    // records lie before the marker; the first one at payload offset 0
    bool ok = s_rel < t.rec_end && e_rel <= t.rec_end && (r != 0 || s_rel == 0);
    const uint32_t count = (live && ok) ? (last_iv ? t.item_count - r * t.ri : t.ri) : 0;
    if (live && !ok) atomicCAS(&meta[j].st, ST_OK, ST_PARSE);
    const uint32_t ib0 = m.item0 + r * t.ri;
    const uint64_t tag = ((uint64_t)j << RL::kBlockShift) | RL::kValid;
    const uint32_t stop = p0 + e_rel;
    uint32_t a = p0 + (ok ? s_rel : 0), key = a;
    const uint32_t max_count = __builtin_amdgcn_readfirstlane(wave_max_u32(count));
    if (!max_count) continue;
    Shape sp;
    bool defer = false;  // a record shape the straight path does not take: whole block to the general path
    {  // restart head (full key: the value length is read separately)
      const Win16 w = read_win16(img, a);
      const RecHead hd = rec_head(w.lo, true);
      const uint32_t nxt = a + rec_len(hd.vt, hd.q, read_u16_unaligned(img, a + hd.q));
      key = a + hd.hdr;
      sp = make_shape<RL>(min(hd.e1 >> 3, 5u), 1);
      defer = count > 1 && !(hd.ok && valid_vtype(hd.vt));
      const bool act = count > 0 && !defer;
      if (count > 1 && act) ok = nxt < rec_end;
      const uint64_t rbits = (count > 1) ? ((uint64_t)(hd.e1 >> 3) << RL::kN1Shift) : 0;  // verified only if walked
      rec[act ? ib0 : dummy] = rec_desc<RL>(a, count == 1 ? stop : nxt, key, tag | RL::kRestart | rbits);
      a = (act && ok) ? nxt : a;
    }
    // The straight-line step, kept short because it is one wave's serial
    // instruction stream: the key length is read at the header length of the
    // previous record's shape and the value length at its key end (both
    // loads issued together); a shape or key-length change takes the rare
    // branch.  No bounds bookkeeping here: positions are clamped to the
    // marker and phase B rejects any record that does not end where its
    // descriptor says.
    uint32_t qp = 0;
    uint32_t hi = (uint32_t)((((uint64_t)key << RL::kKeyShift) | tag | sp.bits) >> 32);
    const uint32_t dmy = dummy;
    for (uint32_t jj = 1; jj < max_count; ++jj) {
      const uint64_t h = read_u64_unaligned(img, a);
      uint32_t z = read_u16_unaligned(img, a + qp);
      const uint32_t klen = (uint32_t)(h >> sp.kshift) & 0x7F;
      uint32_t q = sp.hdr + klen;
      uint32_t vt = (uint32_t)h & 0xFF;
      if (((~h & sp.msk) != sp.pat) | (q != qp)) {  // rare: header shape or key length changed
        const RecHead hd = rec_head(h, false);
        if (hd.ok) sp = make_shape<RL>(hd.e1 >> 3, (hd.e2 - hd.e1) >> 3);
        defer = defer || (jj < count && !hd.ok);  // seqno >= 2^49, shared >= 2^21 or key length >= 128
        q = hd.q;
        z = read_u16_unaligned(img, a + q);
        qp = q;
        hi = (uint32_t)((((uint64_t)key << RL::kKeyShift) | tag | sp.bits) >> 32);
      }
      const uint32_t nxt = min(a + rec_len(vt, q, z), rec_end);
      const bool act = jj < count && !defer;
      const uint32_t end = jj + 1 == count ? stop : nxt;
      rec[act ? ib0 + jj : dmy] = ((uint64_t)hi << 32) | (uint64_t)RL::lo(a, end);
      a = act ? nxt : a;
    }
    if (defer) meta[j].st = ST_DEFER;                             // wins over PARSE
    else if (count && !ok) atomicCAS(&meta[j].st, ST_OK, ST_PARSE);  // walked off the record area
  }
}


// parse_data_fast for a record whose header shape (n1 seqno bytes, n2 shared
// bytes, 1-byte key length) phase A has already verified bit for bit.
__device__ __forceinline__ int parse_data_shape(const uint8_t* base, uint32_t p0, uint32_t pos, uint32_t end,
                                                bool restart, uint32_t base_key_off, uint32_t n1, uint32_t n2,
                                                ItemFields& f, uint32_t& next) {
  const uint64_t h = read_u64_unaligned(base, p0 + pos);
  const uint32_t hdr = n1 + (restart ? 0u : n2) + 2;
  const uint32_t klen = (uint32_t)(h >> (8 * (hdr - 1))) & 0x7F;
  const uint32_t q = hdr + klen;
  const uint32_t vt = (uint32_t)h & 0xFF;
  uint32_t n4, vl;
  bool vl_ok;
  rec_value(vt, read_u16_unaligned(base, p0 + min(pos + q, end)), n4, vl, vl_ok);
  const uint32_t shared = restart ? 0u : (uint32_t)leb_val8(h >> (8 * (n1 + 1)), n2) & 0xFFFF;
  const uint32_t val_off = pos + q + n4;
  f.seqno = leb_val8(h >> 8, n1);
  f.handle_off = 0;
  f.key_off = pos + hdr;
  f.key_len = (uint16_t)klen;
  f.prefix_len = (uint16_t)shared;
  f.val_off = val_off;
  f.val_len = vl;
  f.vtype = (uint8_t)vt;
  next = val_off + vl;
  const bool bad = (pos + q + n4 > end) || ((uint64_t)val_off + vl > end) ||
                   (!restart && (uint64_t)base_key_off + shared > end);
  return !valid_vtype(vt) ? -1 : (!vl_ok ? 0 : (bad ? -1 : 1));
}

// The seven data-block fields present (handle_off is an index-block field,
// stored only when requested).
__host__ __device__ __forceinline__ bool all_fields(const lsm_parsed_items& o) {
  return o.seqno && o.key_off && o.val_off && o.val_len && o.key_len && o.prefix_len && o.vtype;
}

template <bool kCompact>
__device__ __forceinline__ void store_fields(const DecodeParams& P, bool all_fields, uint64_t gi,
                                             const ItemFields& f) {
  if (all_fields) {  // every output array present: no per-field null checks
    gstore(P.out.seqno, gi, f.seqno + P.seqno_add);
    if (kCompact) {  // 19 B/item: 16-bit payload offsets and lengths
      gstore(reinterpret_cast<uint16_t*>(P.out.key_off), gi, (uint16_t)f.key_off);
      gstore(reinterpret_cast<uint16_t*>(P.out.val_off), gi, (uint16_t)f.val_off);
      gstore(reinterpret_cast<uint16_t*>(P.out.val_len), gi, (uint16_t)f.val_len);
    } else {
      gstore(P.out.key_off, gi, f.key_off);
      gstore(P.out.val_off, gi, f.val_off);
      gstore(P.out.val_len, gi, f.val_len);
    }
    gstore(P.out.key_len, gi, f.key_len);
    gstore(P.out.prefix_len, gi, f.prefix_len);
    gstore(P.out.vtype, gi, f.vtype);
    if (P.out.handle_off) gstore(P.out.handle_off, gi, f.handle_off);
  } else {
    emit_global(P.out, gi, f, P.seqno_add, kCompact);
  }
}

// Phase B: thread = record.  Full parse + validation of every descriptor
// (the oracle's parse_data_item checks, and the record must end exactly at
// the descriptor's end), then coalesced stores of all fields.
template <bool kAllFields, bool kCompact, bool kWide = false>
__device__ __forceinline__ void phase_b(const DecodeParams& P, const uint8_t* img, BlockMeta* meta,
                                        const uint64_t* rec, uint32_t n_items, uint32_t g_item0, uint32_t tid,
                                        uint32_t nthr) {
  typedef RecLayout<kWide> RL;
  constexpr bool all_fields = kAllFields;
  const bool store = !(kDiagBuild && (P.flags & kDiagSkipStore));
  for (uint32_t i0 = 0; i0 < n_items; i0 += nthr) {
    const uint32_t i = i0 + tid;
    if (i >= n_items) break;
    const uint64_t d = rec[i];
    if (!(d & RL::kValid)) continue;  // not reached: its block has failed
    const uint32_t j = (uint32_t)(d >> RL::kBlockShift) & 31;
    const u32x4 hot = *reinterpret_cast<const u32x4*>(&meta[j]);  // p0, rec_end, st, type
    const uint32_t p0 = hot.x, end = hot.y - p0;
    if ((int32_t)hot.z != ST_OK) continue;  // block already failed: outputs unspecified
    const uint32_t a = RL::start(d) - p0;
    const uint32_t want = RL::end(d) - p0;
    const uint32_t base_key = ((uint32_t)(d >> RL::kKeyShift) & RL::kPosMask) - p0;
    const bool restart = (d & RL::kRestart) != 0;
    const uint64_t gi = (uint64_t)g_item0 + i;
    ItemFields f;
    uint32_t next;
    const uint32_t n1 = (uint32_t)(d >> RL::kN1Shift) & 7, n2 = (uint32_t)(d >> RL::kN2Shift) & 3;
    const int rc = n1 ? parse_data_shape(img, p0, a, end, restart, base_key, n1, n2, f, next)
                      : parse_data_fast(img, p0, a, end, restart, base_key, f, next);
    if (rc > 0 && store) store_fields<kCompact>(P, all_fields, gi, f);
    if (rc == 0) meta[j].st = ST_DEFER;  // wins over PARSE
    else if (rc < 0 || next != want) atomicCAS(&meta[j].st, ST_OK, ST_PARSE);
  }
}

// Records of restart interval r, [start, stop) payload-relative (the binary
// index's entries r, r + 1), parsed from `base`; emit(j, fields).
template <class Emit>
__device__ __forceinline__ bool walk_interval_at(const uint8_t* base, uint32_t p0, const BlockMeta& m,
                                                 const TrailerInfo& t, uint32_t r, uint32_t start, uint32_t stop,
                                                 Emit emit) {
  const bool last = r + 1 == t.bin_len;
  const uint32_t count = last ? t.item_count - r * t.ri : t.ri;
  if (start > t.rec_end || stop > t.rec_end || (r == 0 && start != 0)) return false;
  uint32_t base_key = 0, pos = start;
  ItemFields f;
  for (uint32_t j = 0; j < count; ++j) {
    uint32_t next;
    if (!parse_record(base, p0, pos, t, m.type, j == 0, base_key, f, next)) return false;
    if (j == 0) base_key = f.key_off;
    emit(r * t.ri + j, f);
    pos = next;
  }
  return pos == stop;
}

// Interval walk straight from a span (direct path); emit(j, fields).
template <class Emit>
__device__ __forceinline__ bool walk_interval(const uint8_t* base, uint32_t p0, const BlockMeta& m, uint32_t r,
                                              Emit emit) {
  const TrailerInfo t = trailer_of(m);
  const bool last = r + 1 == t.bin_len;
  const uint32_t start = bin_get(base, p0, t, r);
  const uint32_t stop = last ? t.rec_end : bin_get(base, p0, t, r + 1);
  return walk_interval_at(base, p0, m, t, r, start, stop, emit);
}

// One block straight from HBM (blocks larger than the LDS stage).
__device__ __forceinline__ void decode_block_direct(const DecodeParams& P, uint32_t b, BlockMeta* meta) {
  const int lane = threadIdx.x;
  const uint64_t off = gload(P.block_off, b), end = gload(P.block_off, b + 1);
  const uint8_t* base = P.blocks + (off & ~15ULL);
  const uint32_t hb = (uint32_t)(off & 15);
  const uint64_t len = end >= off ? end - off : 0;
  const uint64_t item_base = gload(P.item_start, b);
  const uint32_t cap = gload(P.item_start, b + 1) - gload(P.item_start, b);
  if (lane == 0) meta_header(base, hb, len, meta[0]);
  wave_sync();
  if (meta[0].st == ST_OK && !(P.flags & LSM_DECODE_PAYLOAD_VERIFIED)) {
    uint64_t lo, hi;
    xxh3_128_wave(base, hb + kHdrLen, meta[0].len - kHdrLen, &kLongSecret, lo, hi);
    if (lane == 0 && (lo != meta[0].ck_lo || hi != meta[0].ck_hi)) meta[0].st = ST_CKSUM;
  }
  wave_sync();
  if (lane == 0) meta_trailer(base, P.expect_type, cap, meta[0], P.compact);
  wave_sync();
  const BlockMeta m = meta[0];
  if (m.st == ST_OK) {
    bool ok = true;
    for (uint32_t r = lane; r < m.bin_len; r += kWave) {
      ok &= walk_interval(base, hb + kHdrLen, m, r,
                          [&](uint32_t j, const ItemFields& f) { emit_global(P.out, item_base + j, f, P.seqno_add, P.compact); });
    }
    if (!ok) atomicCAS(&meta[0].st, ST_OK, ST_PARSE);
  }
  wave_sync();
  if (lane == 0) gstore(P.status, b, meta[0].st);
  wave_sync();
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

// Blocks whose span exceeds this go to the big-block kernel: those larger
// than the stage.  (Half the stage measured slower: the 17 KB blocks of the
// 16 KiB random-key class run at 0.82 TB/s through the big-block kernel, one
// block per iteration, and at 1.42 TB/s here, one block per group.)
__device__ __forceinline__ uint32_t lone_bytes(const DecodeParams& P) { return P.stage_bytes; }

// A group: the longest run of consecutive blocks from b that fits the stage
// (k == 0: block b alone is too large and takes the direct path).  Lane j of
// every wave holds block b+j's handle and item range.
struct Group {
  uint32_t b, k, g_item0, n_items;
  uint64_t span0, span1;
  uint64_t off_j, end_j;
  uint32_t it0_j, it1_j;
};

// offr / itr: lane l holds block_off / item_start of block b_begin + l.
__device__ __forceinline__ Group form_group(const DecodeParams& P, uint32_t b, uint32_t b_begin, uint32_t b_end,
                                            uint32_t gmax, uint64_t offr, uint32_t itr, uint32_t& skip) {
  const int lane = threadIdx.x & (kWave - 1);
  Group G;
  G.b = b;
  const uint32_t li = b - b_begin + lane;
  const bool in_run = b + lane < b_end && (uint32_t)lane < gmax;
  const int s0 = (int)(in_run ? li : 0), s1 = (int)(in_run ? li + 1 : 0);
  G.off_j = wave_shfl_u64(offr, s0);
  G.end_j = wave_shfl_u64(offr, s1);
  G.it0_j = (uint32_t)__shfl((int)itr, s0);
  G.it1_j = (uint32_t)__shfl((int)itr, s1);
  if (!in_run) G.off_j = G.end_j = 0, G.it0_j = G.it1_j = 0;
  const uint64_t off_b = wave_readlane_u64(G.off_j, 0);
  G.g_item0 = wave_readlane_u32(G.it0_j, 0);
  G.span0 = off_b & ~15ULL;
  // lone blocks (lone_block) never join a group: they are listed for the general path up front
  const bool lone = ((G.end_j + 15) & ~15ULL) - (G.off_j & ~15ULL) > lone_bytes(P) ||
                    G.it1_j - G.it0_j > P.tile_items;
  const bool fits = in_run && !lone && G.end_j >= G.off_j && G.off_j >= off_b &&
                    ((G.end_j + 15) & ~15ULL) - G.span0 <= P.stage_bytes && G.it1_j - G.g_item0 <= P.tile_items;
  G.k = (uint32_t)__builtin_ctzll(~__ballot(fits));  // lanes >= gmax never fit
  // (k = 0: the run of lone blocks from b, at least one, passed over at once:
  // 64 huge blocks one form_group at a time took 17 us)
  skip = max(1u, (uint32_t)__builtin_ctzll(~__ballot(in_run && lone)));
  G.span1 = G.k ? (wave_readlane_u64(G.end_j, G.k - 1) + 15) & ~15ULL : G.span0;
  G.n_items = G.k ? wave_readlane_u32(G.it1_j, G.k - 1) - G.g_item0 : 0;
  return G;
}

// Deferred-block list in the workspace: [count u32][pad][index u32 x n_blocks].
__device__ __forceinline__ void defer_block(const DecodeParams& P, uint32_t b) {
  const uint32_t slot = atomicAdd(P.defer_count, 1u);
  gstore(P.defer_list, slot, b);
}
// Wave-level: lanes with `pred` list block b (one atomic per wave, not per block).
__device__ __forceinline__ void defer_blocks_wave(const DecodeParams& P, bool pred, uint32_t b) {
  const uint64_t m = __ballot(pred);
  if (!m) return;
  const int lane = threadIdx.x & (kWave - 1);
  uint32_t base = 0;
  if (lane == (int)__builtin_ctzll(m)) base = atomicAdd(P.defer_count, (uint32_t)__builtin_popcountll(m));
  base = (uint32_t)__shfl((int)base, (int)__builtin_ctzll(m));
  const uint32_t rank = (uint32_t)__builtin_popcountll(m & ((1ULL << lane) - 1));
  if (pred) gstore(P.defer_list, base + rank, b);
}

__device__ __forceinline__ void defer2_block(const DecodeParams& P, uint32_t b) {
  const uint32_t slot = atomicAdd(P.defer2_count, 1u);
  gstore(P.defer2_list, slot, b);
}

// Deferred blocks up to kBigStage bytes (the 16..64 KiB data blocks larger
// than a group stage, and blocks with rare record shapes): one 4-wave
// workgroup per block, the block staged in LDS by LDS-DMA, then wave 0
// verifies the payload checksum while waves 1..3 walk the restart intervals
// (lane = interval) from LDS and store every record; statuses merge in
// oracle order (header, checksum, trailer / parse).  Larger blocks (full
// index blocks) take the HBM path on wave 0.
constexpr uint32_t kBigWaves = 4;
constexpr uint32_t kBigStage = 72 * 1024;

constexpr uint32_t kBigContrib = 256;                        // LDS: contributions, 64 B per KiB
constexpr uint32_t kBigStageOff = kBigContrib + (kBigStage / 1024 + 1) * 64;

// A data or index block larger than the stage (a full block index: ~25 B
// per data block, hundreds of KiB for a 64 MiB table; a data block of the
// writer's up-to-4-MiB targets, writer/mod.rs:193-198), on all four waves of
// the general-path workgroup, through the stage in 64 KiB chunks (staged with
// 7.5 KiB of overlap past the chunk).  Per chunk: all waves compute the
// per-KiB XXH3 contributions of the chunk's KiB blocks, wave 0 carries the
// serial chain across chunks; each thread parses the restart intervals
// (r = tid, tid + 256, ...) that start in the chunk from LDS when the whole
// interval (+ the parsers' read-ahead) is staged, else walks it from HBM.  The
// interval starts come from the binary index in HBM (the block's tail is not
// in the chunk).  Same results as the interval walk of decode_block_direct.
constexpr uint32_t kChunkBytes = 64 * 1024;
constexpr uint32_t kChunkOverlap = 7 * 1024 + 512;
constexpr uint32_t kChunkReadAhead = 192;  // parsers read at most this far past a record start window
static_assert(kChunkBytes + kChunkOverlap + 256 <= kBigStage, "chunk + overlap + pad");

__device__ __forceinline__ void decode_chunked(const DecodeParams& P, uint32_t b, const uint8_t* gbase,
                                               uint32_t span, BlockMeta* meta, uint32_t* cks_bad,
                                               uint64_t* contrib, uint8_t* stage) {
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int lane = tid & (kWave - 1);
  constexpr uint32_t kThreads = kBigWaves * kWave;
  const BlockMeta m = meta[1];
  const TrailerInfo t = trailer_of(m);
  const uint32_t p0 = m.p0;  // span-relative payload start
  const uint32_t plen = m.len - kHdrLen;
  const uint64_t item_base = gload(P.item_start, b);
  const bool hash = !(P.flags & LSM_DECODE_PAYLOAD_VERIFIED);
  const uint32_t nbk = plen > 240 ? (plen - 1) / 1024 : 0;
  uint64_t a0, a1;
  xxh3_acc_init(lane & 3, a0, a1);
  const uint64_t scr0 = kLongSecret.acc[16 + 2 * (lane & 3)], scr1 = kLongSecret.acc[16 + 2 * (lane & 3) + 1];
  const uint32_t nint = t.bin_len;
  auto emit = [&](uint32_t j, const ItemFields& f) { emit_global(P.out, item_base + j, f, P.seqno_add, P.compact); };
  uint32_t r = tid;
  uint32_t s_cur = r < nint ? bin_get(gbase, p0, t, r) : 0xFFFFFFFFu;
  bool ok = true;
  for (uint32_t cs = 0; cs < span; cs += kChunkBytes) {
    const uint32_t ce = min(cs + kChunkBytes, span);
    const uint32_t ss = min(ce + kChunkOverlap, span);  // staged: [cs, ss)
    {
      const uint32_t chunks = (ss - cs + 15) >> 4;
      const uint8_t* src = gbase + cs + 16 * lane;
      for (uint32_t c = wave; c * kWave < chunks; c += kBigWaves)
        if (c * kWave + lane < chunks)
          __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + 1024 * c), (lds_void_t*)(stage + 1024 * c), 16, 0, 0);
    }
    vm_wait<0>();
    lds_barrier();
    const uint8_t* sbase = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(stage) - cs);  // span-relative
    // the KiB blocks that start in this chunk
    const uint32_t n0 = min(nbk, cs > p0 ? (cs - p0 + 1023) / 1024 : 0u);
    const uint32_t n1 = min(nbk, ce > p0 ? (ce - p0 + 1023) / 1024 : 0u);
    if (hash && n1 > n0)
      xxh3_kib_contribs(sbase, p0 + 1024 * n0, (n1 - n0) * 1024 + 1, &kLongSecret, contrib, wave, kBigWaves);
    // the intervals that start in this chunk
    while (r < nint && p0 + s_cur < ce) {
      const bool last = r + 1 == nint;
      const uint32_t stop = last ? t.rec_end : bin_get(gbase, p0, t, r + 1);
      const bool staged = p0 + s_cur >= cs && stop <= t.rec_end && (p0 + stop + kChunkReadAhead <= ss || ss == span);
      ok &= walk_interval_at(staged ? sbase : gbase, p0, m, t, r, s_cur, stop, emit);
      r += kThreads;
      s_cur = r < nint ? bin_get(gbase, p0, t, r) : 0xFFFFFFFFu;
    }
    lds_barrier();
    if (wave == 0 && hash) {  // the chain over this chunk's KiB blocks, in order
      for (uint32_t n = 0; n < n1 - n0; ++n) {
        a0 = xxh3_scr(a0, contrib[8 * n + 2 * (lane & 3)], scr0);
        a1 = xxh3_scr(a1, contrib[8 * n + 2 * (lane & 3) + 1], scr1);
      }
    }
    lds_barrier();  // (the next chunk overwrites the stage and the contributions)
  }
  if (r < nint) ok = false;  // a record start beyond the block
  if (!ok) atomicCAS(&meta[1].st, ST_OK, ST_PARSE);
  if (wave == 0 && hash) {
    uint64_t lo, hi;
    if (plen > 240) xxh3_wave_tail_merge(gbase, p0, plen, &kLongSecret, a0, a1, lo, hi);
    else xxh3_128_wave(gbase, p0, plen, &kLongSecret, lo, hi);
    if (lane == 0) *cks_bad = lo != m.ck_lo || hi != m.ck_hi;
  }
  lds_barrier();
  if (tid == 0) {
    const int32_t st = meta[0].st != ST_OK ? meta[0].st : *cks_bad ? (int32_t)ST_CKSUM : meta[1].st;
    gstore(P.status, b, st);
  }
}

__global__ __launch_bounds__(kBigWaves * kWave) void decode_deferred_staged_kernel(DecodeParams P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  BlockMeta* meta = reinterpret_cast<BlockMeta*>(smem);  // [0] header view, [1] trailer view
  uint32_t* cks_bad = reinterpret_cast<uint32_t*>(smem + 2 * sizeof(BlockMeta));
  uint64_t* contrib = reinterpret_cast<uint64_t*>(smem + kBigContrib);
  uint8_t* stage = smem + kBigStageOff;
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int lane = tid & (kWave - 1);
  const uint32_t n = gload(P.defer_count, 0);
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t b = gload(P.defer_list, i);
    const uint64_t off = gload(P.block_off, b), end = gload(P.block_off, b + 1);
    const uint64_t span0 = off & ~15ULL, span1 = (max(end, off) + 15) & ~15ULL;
    if (span1 - span0 > kBigStage) {  // larger than the stage
      const uint8_t* gbase = P.blocks + span0;
      const uint32_t cap = gload(P.item_start, b + 1) - gload(P.item_start, b);
      if (tid == 0) {
        meta_header(gbase, (uint32_t)(off - span0), end >= off ? end - off : 0, meta[0]);
        meta[1] = meta[0];
        meta_trailer(gbase, P.expect_type, cap, meta[1], P.compact);
        *cks_bad = 0;
      }
      lds_barrier();
      if (meta[0].st == ST_OK && meta[1].st == ST_OK) {  // data / index / meta blocks: chunked through the stage
        decode_chunked(P, b, gbase, (uint32_t)(span1 - span0), meta, cks_bad, contrib, stage);
      } else if (wave == 0) {  // a failing header or trailer: one wave (statuses in oracle order)
        decode_block_direct(P, b, meta);
      }
      lds_barrier();
      continue;
    }
    const uint32_t chunks = (uint32_t)((span1 - span0) >> 4);
    const uint8_t* src = P.blocks + span0 + 16 * lane;
    for (uint32_t c = wave; c * kWave < chunks; c += kBigWaves) {
      if (c * kWave + lane < chunks)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + 1024 * c), (lds_void_t*)(stage + 1024 * c), 16, 0, 0);
    }
    const uint64_t item_base = gload(P.item_start, b);
    const uint32_t cap = gload(P.item_start, b + 1) - (uint32_t)item_base;
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0): this wave's DMA has landed
    lds_barrier();
    const uint32_t hb = (uint32_t)(off & 15);
    if (tid == 0) {
      meta_header(stage, hb, end >= off ? end - off : 0, meta[0]);
      meta[1] = meta[0];
      meta_trailer(stage, P.expect_type, cap, meta[1], P.compact);
      *cks_bad = 0;
    }
    lds_barrier();
    // payload checksum: per-KiB contributions on all waves, then the chain on wave 0
    const bool hdr_ok = meta[0].st == ST_OK && !(P.flags & LSM_DECODE_PAYLOAD_VERIFIED);
    const uint32_t plen = meta[0].len - kHdrLen;
    if (hdr_ok && plen > 240) xxh3_kib_contribs(stage, hb + kHdrLen, plen, &kLongSecret, contrib, wave, kBigWaves);
    lds_barrier();
    if (wave == 0) {
      if (hdr_ok) {
        uint64_t lo, hi;
        if (plen > 240) xxh3_128_wave_finish(stage, hb + kHdrLen, plen, &kLongSecret, contrib, lo, hi);
        else xxh3_128_wave(stage, hb + kHdrLen, plen, &kLongSecret, lo, hi);
        if (lane == 0) *cks_bad = lo != meta[0].ck_lo || hi != meta[0].ck_hi;
      }
    } else {
      const BlockMeta m = meta[1];
      if (m.st == ST_OK) {
        bool ok = true;
        for (uint32_t r = tid - kWave; r < m.bin_len; r += (kBigWaves - 1) * kWave) {
          ok &= walk_interval(stage, hb + kHdrLen, m, r,
                              [&](uint32_t j, const ItemFields& f) { emit_global(P.out, item_base + j, f, P.seqno_add, P.compact); });
        }
        if (!ok) atomicCAS(&meta[1].st, ST_OK, ST_PARSE);
      }
    }
    lds_barrier();
    if (tid == 0) {
      const int32_t st = meta[0].st != ST_OK ? meta[0].st : *cks_bad ? (int32_t)ST_CKSUM : meta[1].st;
      gstore(P.status, b, st);
    }
    lds_barrier();
  }
}

// ---- Blocks larger than the general path's stage across the whole GPU (the
// writer's up-to-4-MiB data blocks, writer/mod.rs:193-198; full block
// indexes): decode_chunked walks such a block on ONE workgroup, chunk by
// chunk.  Here its work is cut into units that any workgroup takes:
//   plan   (decode_huge_plan_kernel, one workgroup, after decode_big_kernel lists them):
//          per huge block the header (incl. its checksum) and trailer views
//          from HBM, its KiB-block and parse-unit counts, prefix sums of both
//          over the list (contributions in the workspace pool: 64 B per KiB)
//   units  (decode_huge_units_kernel, thread per restart interval): per unit
//          the first interval that starts in it and that interval's offset
//   work   (decode_huge_kernel, every CU): units = kHugeWin-byte windows of a
//          block's span.  A unit stages its window (+ kHugeOverlap) in LDS by
//          LDS-DMA, takes the restart intervals that start in it from the unit
//          table (a block whose binary index is not monotone: a 256-way search
//          of the index in HBM, two or three round trips),
//          walks them from LDS (thread per interval, walk_interval_at: every
//          oracle check, the LEB cursor for rare shapes; from HBM when one
//          runs past the staged bytes) and computes the XXH3 contributions
//          of the KiB blocks that start in the window, from LDS too
//   chain  (inside decode_huge_kernel: its first workgroups): one wave per
//          block, the eight accumulator chains on lanes 0..7 (xxh3_chain8)
//          over the KiB contributions as the units publish them (unit-done
//          flags), then the tail merge, the checksum compare and the status
// A block whose header fails, or that no longer fits the pool, goes to the
// general path (defer2) as before: statuses and outputs are the same on both.
constexpr uint32_t kHugeWin = 32 * 1024;  // span bytes per unit
constexpr uint32_t kHugeOverlap = ((8 * 1024 - 256));  // staged past the window (intervals that straddle it)
constexpr uint32_t kHugeStage = kHugeWin + kHugeOverlap;
constexpr uint32_t kHugeMaxIv = 512;                   // intervals per window for phase A / B (else thread walks)
constexpr uint32_t kHugeTile = 32 * 32;  // items per window for phase A / B
constexpr uint32_t kHugeBix = kHugeStage + kStagePad;  // LDS: the window's binary-index entries
constexpr uint32_t kHugeMeta = kHugeBix + 4 * (kHugeMaxIv + 4);
constexpr uint32_t kHugeOwner = kHugeMeta + 80;
constexpr uint32_t kHugeRec = kHugeOwner + kHugeMaxIv;
constexpr uint32_t kHugeLds = 64 + kHugeRec + 8 * (kHugeTile + 1);
constexpr uint32_t kHugeWgsPerCU = 3;  // decode_huge_kernel's residency (3 waves per SIMD, ~51 KB of LDS)
constexpr uint32_t kStreamRing = 12;    // the same for the chain waves inside decode_huge_kernel (4 per workgroup)
// A chain wave gives its block up after this long without progress (s_memrealtime ticks, 100 MHz:
// 5 ms, ~25x a whole 4 MiB decode); the block is then re-verified by the fallback chain pass.
constexpr uint64_t kStreamStallTicks = 500000;
constexpr uint32_t kStreamChainWgs = 16;     // chain workgroups: 64 chain waves (a 1 KiB step of 20 ns each)
constexpr uint32_t kStreamMinUnits = 64;     // stream the chains for batches holding a block of >= 2 MiB
constexpr uint32_t kChainRing = 16;          // the chain kernel's ring (KiB of contribution rows in flight per wave)
constexpr uint32_t kHugeChainGrid = 1024;    // chain kernel workgroups (one block each, grid-stride)
constexpr uint32_t kHugeUnitsGrid = 1024;  // unit-table workgroups (thread per restart interval, grid-stride)

struct HugeRec {
  BlockMeta m;         // header view, trailer fields merged in: m.st = trailer status (header checks passed)
  uint64_t span0, item_base;
  uint64_t acc[8];     // chain results (accumulator k from chain wave k)
  uint32_t b, nbk, accepted, parse_bad;
  uint32_t done, span;  // span: the block's 16-B-aligned byte span
  uint32_t nonmono;     // its binary index is not monotone (units kernel): the units search it
  uint32_t pad;
};
static_assert(sizeof(HugeRec) % 16 == 0, "HugeRec layout");

struct HugeHdr {
  uint64_t total_kib;  // contribution rows over every listed block (each block's padded to 16)
  uint32_t n3;         // listed huge blocks (HugeRec entries)
  uint32_t total_pu;   // work units (kHugeWin windows)
  uint64_t total_iv;   // restart intervals + 1 per parsed block (units kernel threads)
  uint32_t max_npu;    // most units of one accepted block
  uint32_t stream;     // chains inside decode_huge_kernel, streaming behind the units (blocks of >= 2 MiB)
};

// Pool: [HugeHdr | 256][kpre, ppre, ipre: u64 x (n + 1) each][HugeRec x n][contributions, 64 B per KiB
// from the front, each block's rows padded to a multiple of 16 (one 1-KiB chain chunk holds no
// other block's rows)] .. [unit table, 16 B per unit, from the back: entry u at uend[-1 - u]:
// first interval, its payload offset, the unit-done flag].
struct HugeLayout {
  HugeHdr* hdr;
  uint64_t* kpre;
  uint64_t* ppre;
  uint64_t* ipre;
  HugeRec* rec;
  uint64_t* contrib;
  uint4* uend;    // unit u: {first restart interval starting in it, that interval's payload offset, done flag}
  uint64_t rest;  // pool bytes after the fixed part
  bool ok;
};
__host__ __device__ constexpr uint64_t huge_fixed_bytes(uint64_t n) {
  return (256 + 24 * (n + 1) + sizeof(HugeRec) * n + 255) & ~255ULL;
}
__device__ __forceinline__ HugeLayout huge_layout(const DecodeParams& P, uint32_t n) {
  HugeLayout L;
  uint8_t* b = P.huge_pool;
  L.hdr = reinterpret_cast<HugeHdr*>(b);
  L.kpre = reinterpret_cast<uint64_t*>(b + 256);
  L.ppre = L.kpre + (n + 1);
  L.ipre = L.ppre + (n + 1);
  L.rec = reinterpret_cast<HugeRec*>(L.ipre + (n + 1));
  const uint64_t fixed = huge_fixed_bytes(n);
  L.contrib = reinterpret_cast<uint64_t*>(b + fixed);
  L.ok = b != nullptr && fixed <= P.huge_pool_bytes;
  L.rest = L.ok ? (P.huge_pool_bytes - fixed) & ~15ULL : 0;
  L.uend = reinterpret_cast<uint4*>(b + fixed + L.rest);
  return L;
}

__device__ __forceinline__ void defer3_block(const DecodeParams& P, uint32_t b) {
  const uint32_t slot = atomicAdd(P.defer3_count, 1u);
  gstore(P.defer3_list, slot, b);
}

// Plan over the huge list, by one workgroup of nthr threads (nthr / 64 <= 16
// waves); sh: 56 u64 of LDS; hstage: kHugePlanStage bytes of LDS per thread.
// Blocks it does not accept go to defer2.
constexpr uint32_t kHugePlanStage = 128;
__device__ void huge_plan(const DecodeParams& P, uint64_t* sh, uint32_t nthr, uint8_t* hstage) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = nthr >> 6;
  const uint32_t n = gload(P.defer3_count, 0);
  const HugeLayout L = huge_layout(P, n);
  if (!L.ok) {  // (uniform) no pool, or too small for the records: the general path takes them all
    for (uint32_t i = tid; i < n; i += nthr) defer2_block(P, gload(P.defer3_list, i));
    if (P.huge_pool && P.huge_pool_bytes >= 256 && tid == 0) {
      L.hdr->n3 = 0;
      L.hdr->total_pu = 0;
      L.hdr->total_kib = 0;
      L.hdr->total_iv = 0;
      L.hdr->max_npu = 0;
      L.hdr->stream = 0;
    }
    return;
  }
  const bool hash = !(P.flags & LSM_DECODE_PAYLOAD_VERIFIED);
  if (tid == 0) sh[48] = 0, sh[49] = 0, sh[50] = 0, sh[51] = 0;
  __syncthreads();
  for (uint32_t c = 0; c < n; c += nthr) {
    const uint32_t i = c + tid;
    uint64_t nbk = 0, npu = 0, niv = 0;
    bool acc = false;
    uint32_t b = 0;
    BlockMeta m{};
    uint64_t span0 = 0, item_base = 0, span = 0;
    if (i < n) {
      b = gload(P.defer3_list, i);
      const uint64_t off = gload(P.block_off, b), end = gload(P.block_off, b + 1);
      span0 = off & ~15ULL;
      item_base = gload(P.item_start, b);
      const uint32_t cap = gload(P.item_start, b + 1) - (uint32_t)item_base;
      const uint8_t* gbase = P.blocks + span0;
      // the header's and the trailer's 64-B windows staged in LDS, all eight loads at once (the
      // checks' serial reads then cost LDS round trips, not HBM ones); the trailer copy is
      // addressed span-relative like gbase, and the marker byte before the binary index is read
      // from HBM (blocks here span more than the 72 KiB stage; the input padding covers the reads)
      uint8_t* hs = hstage + kHugePlanStage * tid;
      const uint64_t tend = (max(end, off) + 15) & ~15ULL;
      {
        const u32x4* gh = reinterpret_cast<const u32x4*>(gbase);
        const u32x4* gt = reinterpret_cast<const u32x4*>(P.blocks + tend - 64);
        u32x4 x[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = gh[q], x[4 + q] = gt[q];
#pragma unroll
        for (int q = 0; q < 8; ++q) reinterpret_cast<u32x4*>(hs)[q] = x[q];
      }
      const uint8_t* tbase = hs + 128 - (tend - span0);  // (span offset o -> hs[128 - (tend - span0) + o])
      meta_header(hs, (uint32_t)(off - span0), end >= off ? end - off : 0, m);
      acc = m.st == ST_OK;  // every header check, its checksum included
      if (acc) {
        const uint32_t plen = m.len - kHdrLen;
        nbk = hash ? (plen - 1) / 1024 : 0;  // (plen > 72 KiB here: the long path)
        meta_trailer(tbase, P.expect_type, cap, m, P.compact, gbase);  // (after the payload checksum in oracle order)
        span = ((max(end, off) + 15) & ~15ULL) - span0;
        npu = (nbk || m.st == ST_OK) ? (span + kHugeWin - 1) / kHugeWin : 0;
        niv = m.st == ST_OK ? trailer_of(m).bin_len + 1 : 0;  // (+1: the units kernel's end-of-block thread)
      }
    }
    const uint64_t nbk16 = (nbk + 15) & ~15ULL;  // (rows padded to whole 1-KiB chain chunks)
    const uint64_t ik = wave_incl_scan_u64(nbk16), ip = wave_incl_scan_u64(npu), ii = wave_incl_scan_u64(niv);
    if (lane == 63) sh[wave] = ik, sh[16 + wave] = ip, sh[32 + wave] = ii;
    __syncthreads();
    uint64_t bk = sh[48], bp = sh[49], bi = sh[50], tk = 0, tp = 0, ti = 0;
    for (uint32_t w = 0; w < nw; ++w) {
      bk += w < wave ? sh[w] : 0;
      bp += w < wave ? sh[16 + w] : 0;
      bi += w < wave ? sh[32 + w] : 0;
      tk += sh[w];
      tp += sh[16 + w];
      ti += sh[32 + w];
    }
    const uint64_t kp = bk + ik - nbk16, pp = bp + ip - npu, ivp = bi + ii - niv;
    if (i < n) {
      // (the pool holds the contributions, front, and unit entries, back, of a prefix of the list)
      acc = acc && 64 * (kp + nbk16) + 16 * (pp + npu) <= L.rest;
      HugeRec* r = L.rec + i;
      r->m = m;
      r->span0 = span0;
      r->item_base = item_base;
      r->b = b;
      r->nbk = (uint32_t)nbk;
      r->accepted = acc;
      r->parse_bad = 0;
      r->done = 0;
      r->span = (uint32_t)span;
      r->nonmono = 0;
      gstore(L.kpre, i, kp);
      gstore(L.ppre, i, pp);
      gstore(L.ipre, i, ivp);
      if (!acc) defer2_block(P, b);
    }
    {  // the most units of an accepted block: one LDS atomic per wave
      const uint32_t mx = wave_max_u32(i < n && acc ? (uint32_t)npu : 0u);
      if (lane == 0 && mx) atomicMax(reinterpret_cast<unsigned int*>(&sh[51]), mx);
    }
    __syncthreads();
    if (tid == 0) sh[48] += tk, sh[49] += tp, sh[50] += ti;
    __syncthreads();
  }
  if (tid == 0) {
    gstore(L.kpre, n, sh[48]);
    gstore(L.ppre, n, sh[49]);
    gstore(L.ipre, n, sh[50]);
    L.hdr->total_kib = sh[48];
    L.hdr->total_pu = (uint32_t)sh[49];
    L.hdr->total_iv = sh[50];
    L.hdr->max_npu = (uint32_t)sh[51];
    L.hdr->stream = (uint32_t)sh[51] >= kStreamMinUnits;
    L.hdr->n3 = n;
  }
}

__global__ __launch_bounds__(1024) void decode_huge_plan_kernel(DecodeParams P) {
  __shared__ uint64_t sh[56];
  extern __shared__ __attribute__((aligned(16))) uint8_t hstage[];  // kHugePlanStage B per thread
  huge_plan(P, sh, 1024, hstage);
}

// Large blocks (SURVEY configs[4]: 16 / 64 KiB data blocks) listed by the
// group kernel: persistent 8-wave workgroups, two per CU (one stage each:
// the other workgroup's decode overlaps this one's DMA).  Per block, after
// the LDS-DMA, three concurrent streams hand off through LDS flags:
//   wave 0      header fields and trailer (lane 0), then phase A over every
//               restart interval (lane = interval), then phase B
//   waves 1..6  the per-KiB XXH3 contributions, each published as it is
//               done, then phase B once phase A has finished
//   wave 7      the serial XXH3 scramble chain over the contributions as they
//               arrive, the tail and the header checksum (raised priority:
//               it is the block's critical path)
// Blocks larger than the stage, with more items than kBigGTile, index blocks
// and rare record shapes go on to the general path (defer2 list).
constexpr uint32_t kBigGWaves = 8;
constexpr uint32_t kBigGStage = 69376;  // 67.75 KiB: a 64 KiB-target block of 69.2 KB plus alignment
constexpr uint32_t kBigGSlot = kBigGStage + kStagePad;
constexpr uint32_t kBigGTile = 832;
constexpr uint32_t kBigGRec = ((kBigGTile + 1) * 8 + 15) & ~15u;
constexpr uint32_t kBigGContrib = (kBigGStage / 1024 + 1) * 64;
constexpr uint32_t kBigGOwner = (kBigGTile + 15) & ~15u;
// Cross-wave hand-offs of one block (tags: the block's list index + 1, so
// nothing is reset between blocks).
struct BigSync {
  uint32_t a_done;  // phase A finished
  uint32_t hck;     // header checksum ok (chain wave)
  uint64_t lo, hi;  // payload xxh3_128 (chain wave)
  uint32_t ready[kBigGStage / 1024 + 1];  // KiB block n's contribution published
};
constexpr uint32_t kBigGSync = (sizeof(BigSync) + 15) & ~15u;
constexpr uint32_t kBigGLds = 80 + kBigGSync + kBigGRec + kBigGOwner + kBigGContrib + kBigGSlot;
constexpr uint32_t kBigGPerCU = 2;
static_assert(kBigGLds * kBigGPerCU <= 160 * 1024, "big-block workgroups per CU");

// A listed block's handle and item range; fits = it takes the stage path.
struct BigBlk {
  uint32_t li, b, it0, it1;
  uint64_t off, end, span0, span1;
  bool fits;
};
__device__ __forceinline__ BigBlk big_blk(const DecodeParams& P, uint32_t li) {
  BigBlk x;
  x.li = li;
  x.b = gload(P.defer_list, li);
  x.off = gload(P.block_off, x.b);
  x.end = gload(P.block_off, x.b + 1);
  x.it0 = gload(P.item_start, x.b);
  x.it1 = gload(P.item_start, x.b + 1);
  x.span0 = x.off & ~15ULL;
  x.span1 = (max(x.end, x.off) + 15) & ~15ULL;
  x.fits = x.end >= x.off && x.span1 - x.span0 <= kBigGStage && x.it1 - x.it0 <= kBigGTile;
  return x;
}

#if defined(LSM_DIAG) && !defined(LSM_DIAG_NOTIME)
// Diagnostic builds: per-phase s_memtime totals of wave 0 of every big-block
// workgroup (read by lsm_diag_decode_phases).
__device__ unsigned long long g_dec_phase[32];
#define DEC_PHASE(i)                                  \
  {                                                   \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    ph[i] += t_ - t_last;                             \
    t_last = t_;                                      \
  }
// Role timer: time since the last phase mark into ph[i], one count into ph[i + 1].
#define DEC_ROLE(i)                                   \
  {                                                   \
    ph[i] += __builtin_amdgcn_s_memtime() - t_last;   \
    ph[(i) + 1] += 1;                                 \
  }
#else
#define DEC_PHASE(i)
#define DEC_ROLE(i)
#endif

template <bool kAllFields, bool kCompact>
__global__ __launch_bounds__(kBigGWaves * kWave) void decode_big_kernel(DecodeParams P) {
#if defined(LSM_DIAG) && !defined(LSM_DIAG_NOTIME)
  uint64_t t_last = __builtin_amdgcn_s_memtime(), ph[8] = {};
  uint32_t nblk = 0;
#endif
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  BlockMeta* meta = reinterpret_cast<BlockMeta*>(smem);
  BigSync* sync = reinterpret_cast<BigSync*>(smem + 80);
  uint64_t* rec = reinterpret_cast<uint64_t*>(smem + 80 + kBigGSync);
  uint8_t* owner = smem + 80 + kBigGSync + kBigGRec;
  uint64_t* contrib = reinterpret_cast<uint64_t*>(smem + 80 + kBigGSync + kBigGRec + kBigGOwner);
  uint8_t* stages = smem + 80 + kBigGSync + kBigGRec + kBigGOwner + kBigGContrib;
  constexpr uint32_t kThreads = kBigGWaves * kWave;
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int lane = tid & (kWave - 1);
  const uint32_t n = gload(P.defer_count, 0);
  // the listed blocks of this workgroup that fit a stage, in list order
  auto next_fit = [&](uint32_t li) -> BigBlk {
    for (;; li += gridDim.x) {
      if (li >= n) {
        BigBlk z{};
        z.li = li;
        z.fits = false;
        return z;
      }
      const BigBlk x = big_blk(P, li);
      if (x.fits) return x;
      if (tid == 0) {  // (workgroup-uniform)
        if (P.huge_pool && x.end >= x.off && x.span1 - x.span0 > kBigStage) defer3_block(P, x.b);
        else defer2_block(P, x.b);
      }
    }
  };
  auto issue_dma = [&](const BigBlk& x, uint8_t* dst) {  // wave w moves 1-KiB pieces w, w + 8, ...
    const uint32_t chunks = (uint32_t)((x.span1 - x.span0) >> 4);
    const uint8_t* src = P.blocks + x.span0 + 16 * lane;
    for (uint32_t c = wave; c * kWave < chunks; c += kBigGWaves)
      if (c * kWave + lane < chunks)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + 1024 * c), (lds_void_t*)(dst + 1024 * c), 16, 0, 0);
  };
  for (uint32_t x = tid; x < kBigGStage / 1024 + 1; x += kThreads) sync->ready[x] = 0;
  if (tid == 0) sync->a_done = 0;
  BigBlk X = next_fit(blockIdx.x);
  if (X.fits) issue_dma(X, stages);
  while (X.fits) {
    uint8_t* stage = stages;
    const uint32_t b = X.b, n_items = X.it1 - X.it0;
    const uint32_t tag = X.li + 1;  // this block's publication tag (list indices only grow)
    for (uint32_t x = tid; x <= n_items; x += kThreads) rec[x] = 0;
    DEC_PHASE(7);
    vm_wait<0>();  // this block's stage (and every earlier store)
    lds_barrier();
    DEC_PHASE(0);
    const uint32_t hb = (uint32_t)(X.off - X.span0);
    const uint64_t hlen = X.end - X.off;
    // the payload checksum as the handle gives it: it counts only if the
    // header's fields check out (then data_length == handle - 33)
    const bool hash = !(P.flags & LSM_DECODE_PAYLOAD_VERIFIED) && !(kDiagBuild && (P.flags & kDiagSkipHash)) &&
                      hlen >= kHdrLen;
    const uint32_t plen = hash ? (uint32_t)hlen - kHdrLen : 0;
    if (wave == kBigGWaves - 1) {
      // the serial XXH3 chain, consuming the contributions as waves 1.. publish
      // them, then the tail and the header checksum (raised priority: the
      // chain is the block's critical path)
      if (hash) {
        __builtin_amdgcn_s_setprio(3);
        uint64_t lo, hi;
        if (plen > 240) xxh3_128_wave_finish(stage, hb + kHdrLen, plen, &kLongSecret, contrib, lo, hi, sync->ready, tag);
        else xxh3_128_wave(stage, hb + kHdrLen, plen, &kLongSecret, lo, hi);
        const bool hck = header_cksum_ok(stage, hb);
        if (lane == 0) {
          sync->lo = lo;
          sync->hi = hi;
          sync->hck = hck;
        }
        __builtin_amdgcn_s_setprio(0);
      }
    } else {
      if (wave == 0) {  // header, trailer, then phase A over every restart interval
        if (lane == 0) {
          BlockMeta m;
          meta_header_fields(stage, hb, hlen, m);
          m.item0 = 0;
          m.hdr_st = m.st;
          m.ck_bad = 0;
          m.hck_bad = 0;
          meta_trailer(stage, P.expect_type, n_items, m, P.compact);
          if (m.st == ST_OK && m.type == 1) m.st = ST_DEFER;  // index blocks: general path
          m.chain0 = 0;
          meta[0] = m;
        }
        wave_sync();
        const uint32_t total = meta[0].st == ST_OK ? meta[0].bin_len : 0;
        for (uint32_t r = lane; r < total; r += kWave) owner[r] = 0;
        wave_sync();
        __builtin_amdgcn_s_setprio(2);  // (the record walk is the block's longest role)
        phase_a<true>(stage, meta, owner, rec, 0, kWave, total, kBigGTile);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        if (lane == 0) __hip_atomic_store(&sync->a_done, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {  // the per-KiB contributions, then wait for phase A
        if (hash && plen > 240)
          xxh3_kib_contribs(stage, hb + kHdrLen, plen, &kLongSecret, contrib, wave - 1, kBigGWaves - 2, sync->ready,
                            tag);
        while (__hip_atomic_load(&sync->a_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != tag)
          __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
      }
      // phase B on waves 0 .. kBigGWaves - 2, under the chain
      if (!(kDiagBuild && (P.flags & kDiagSkipPhaseB)))
        phase_b<kAllFields, kCompact, true>(P, stage, meta, rec, n_items, X.it0, tid, (kBigGWaves - 1) * kWave);
    }
    lds_barrier();
    DEC_PHASE(4);
    const BigBlk Xn = next_fit(X.li + gridDim.x);
    if (tid == 0) {  // statuses in oracle order: header, header checksum, payload checksum, trailer / parse
      const BlockMeta& m = meta[0];
      const bool chk = hash && m.hdr_st == ST_OK;
      const int32_t st = m.hdr_st != ST_OK                              ? m.hdr_st
                         : (chk && !sync->hck)                          ? (int32_t)ST_HDR_CKSUM
                         : (chk && (sync->lo != m.ck_lo || sync->hi != m.ck_hi)) ? (int32_t)ST_CKSUM
                                                                         : m.st;
      if (st == ST_DEFER) defer2_block(P, b);
      else gstore(P.status, b, st);
    }
    lds_barrier();  // (meta / rec / owner / the stage are rewritten for the next block)
    DEC_PHASE(5);
    if (Xn.fits) issue_dma(Xn, stages);
    DEC_PHASE(6);
#if defined(LSM_DIAG) && !defined(LSM_DIAG_NOTIME)
    ++nblk;
#endif
    X = Xn;
  }
#if defined(LSM_DIAG) && !defined(LSM_DIAG_NOTIME)
  if (tid == 0) {
    for (int i = 0; i < 8; ++i) atomicAdd(&g_dec_phase[i], (unsigned long long)ph[i]);
    atomicAdd(&g_dec_phase[15], (unsigned long long)nblk);
  }
#endif
}

// The last i in [0, n) with a[i] <= v (a[0] = 0, nondecreasing): the huge
// block that owns unit / KiB block v (blocks without any are passed over).
__device__ __forceinline__ uint32_t last_le(const uint64_t* a, uint32_t n, uint64_t v) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (gload(a, mid) <= v) lo = mid;
    else hi = mid;
  }
  return lo;
}

// The unit table of the parsed huge blocks: thread per restart interval x of
// block i (plus one past its last), start s_x (span offset).  Unit u (window
// [uW, uW + W)) gets the first interval that starts at or after uW, and that
// interval's payload offset (the bound the window's last walk stops at): x
// writes the units in (floor(s_{x-1} / W), floor(s_x / W)].  For a monotone
// binary index every unit of the block is written once; a block whose index
// is not monotone is flagged, and the work kernel searches its index instead.
__global__ __launch_bounds__(256) void decode_huge_units_kernel(DecodeParams P) {
  __shared__ uint32_t sb;
  const HugeHdr* hp = reinterpret_cast<const HugeHdr*>(P.huge_pool);
  const uint32_t n = hp->n3;
  if (!n) return;
  const HugeLayout L = huge_layout(P, n);
  if (hp->stream)  // this call's unit-done flags start clear (entries inside the pool only)
    for (uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x; u < hp->total_pu && 16 * (u + 1) <= L.rest;
         u += (uint64_t)gridDim.x * 256)
      L.uend[-1 - (int64_t)u].z = 0;
  const uint64_t tiv = hp->total_iv;
  for (uint64_t t0 = (uint64_t)blockIdx.x * 256; t0 < tiv; t0 += (uint64_t)gridDim.x * 256) {
    if (threadIdx.x == 0) sb = last_le(L.ipre, n, t0);
    __syncthreads();
    const uint64_t tt = t0 + threadIdx.x;
    uint32_t i = sb;
    __syncthreads();  // (sb is rewritten in the next round)
    if (tt >= tiv) continue;
    while (i + 1 < n && gload(L.ipre, i + 1) <= tt) ++i;
    HugeRec* r = L.rec + i;
    if (!r->accepted) continue;
    const BlockMeta m = r->m;
    const TrailerInfo t = trailer_of(m);
    const uint32_t x = (uint32_t)(tt - gload(L.ipre, i)), nint = t.bin_len;
    const uint8_t* gbase = P.blocks + r->span0;
    const uint64_t ub = gload(L.ppre, i);
    const int64_t npu = (int64_t)(gload(L.ppre, i + 1) - ub);
    const uint32_t sv = x < nint ? bin_get(gbase, m.p0, t, x) : t.rec_end;  // payload offset
    const uint32_t sp = x > 0 ? bin_get(gbase, m.p0, t, x - 1) : 0;
    if (x > 0 && x < nint && sv < sp) __hip_atomic_store(&r->nonmono, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t ulo = x > 0 ? (int64_t)((m.p0 + (uint64_t)sp) / kHugeWin) + 1 : 0;
    const int64_t uhi = x < nint ? min((int64_t)((m.p0 + (uint64_t)sv) / kHugeWin), npu - 1) : npu - 1;
    for (int64_t u = ulo; u <= uhi; ++u) *reinterpret_cast<uint2*>(&L.uend[-1 - (int64_t)(ub + u)]) = make_uint2(x, sv);
  }
}

// Huge-block work units (see huge_plan): unit u = window c of block i.  Data
// windows whose intervals are all staged take phase A / B (decode_big_kernel's
// record walk: lane = interval for the boundaries, thread = record for the
// fields) on a window view of the block (meta offsets relative to the stage,
// interval numbers absolute, the binary-index entries copied next to the
// stage); others walk their intervals thread by thread.
// Unit-done flags: unit u's entry .z = the call's tag once its records and
// contributions are written.  The contributions are agent-scope stores
// (through the writer XCD's L2), waited for (vmcnt) before the flag store;
// a chain wave reads a 1-KiB chunk of rows (LDS-DMA) only after the flags of
// every unit that writes into it: no L2 of this launch holds a line of the
// chunk before that, and every block's rows are padded to whole chunks.
// ready_upto: units [0, ready_upto) of the block are known done; polls 64
// flags per load.  Returns false (the caller gives the block up) after
// kStreamStallTicks of wall time without progress: a bound in time, not in
// polls, whose length does not depend on the load latency.
__device__ __forceinline__ bool huge_wait_units(const HugeLayout& L, uint64_t ub, uint32_t need, uint32_t tag,
                                                uint32_t npu, uint32_t& ready_upto, bool give_up) {
  const uint32_t lane = threadIdx.x & 63;
  need = min(need, npu);
  if (ready_upto >= need) return true;
  if (give_up) return false;  // (diagnostic builds: kDiagStreamGiveUp)
  uint64_t t_prog = __builtin_amdgcn_s_memrealtime();
  while (ready_upto < need) {
    const uint32_t c = ready_upto + lane;
    const uint32_t f = c < npu ? __hip_atomic_load(&L.uend[-1 - (int64_t)(ub + c)].z, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT)
                               : tag;
    const uint64_t done = __ballot(f == tag);
    const uint32_t adv = (uint32_t)__builtin_ctzll(~done);  // (done == ~0: 64)
    ready_upto = min(npu, ready_upto + (done == ~0ULL ? 64u : adv));
    if (ready_upto < need && adv == 0) {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (now - t_prog > kStreamStallTicks) return false;
      __builtin_amdgcn_s_sleep(2);
    } else {
      t_prog = __builtin_amdgcn_s_memrealtime();
    }
  }
  return true;
}

// One block's chain on this wave, its rows consumed as the units publish
// them, then the tail merge, the checksum compare and the status (oracle
// order: payload checksum, then trailer, then parse) once every unit is done.
__device__ void huge_chain_streamed(const DecodeParams& P, const HugeLayout& L, uint32_t i, uint8_t* ring) {
  const HugeRec* r = L.rec + i;
  const uint32_t lane = threadIdx.x & 63, k = lane & 7, q = lane & 3;
  const bool hash = !(P.flags & LSM_DECODE_PAYLOAD_VERIFIED);
  const BlockMeta m = r->m;
  const uint64_t ub = gload(L.ppre, i);
  const uint32_t npu = (uint32_t)(gload(L.ppre, i + 1) - ub);
  const uint32_t tag = P.huge_tag;
  const bool give_up = kDiagBuild && (P.flags & kDiagStreamGiveUp);
  uint32_t ready_upto = 0;
  bool ok = true;
  int32_t st = ST_OK;
  if (hash) {
    uint64_t a0, a1;
    xxh3_acc_init((int)(k >> 1), a0, a1);
    uint64_t x = (k & 1) ? a1 : a0;
    const uint32_t nbk = r->nbk;
    if (nbk) {
      // chunk c of 16 rows needs the units holding the starts of KiB blocks 16c .. 16c + 15
      auto wait = [&](uint64_t c) {
        const uint64_t last = min((uint64_t)nbk - 1, 16 * c + 15);
        const uint32_t need = (uint32_t)((m.p0 + 1024 * last) / kHugeWin) + 1;
        ok = ok && huge_wait_units(L, ub, need, tag, npu, ready_upto, give_up);
      };
      x = xxh3_chain8<kStreamRing>(L.contrib + 8 * gload(L.kpre, i), nbk, x, kLongSecret.acc[16 + k], ring, wait);
    }
    const uint64_t c0 = wave_shfl_u64(x, (int)(2 * q)), c1 = wave_shfl_u64(x, (int)(2 * q + 1));
    uint64_t lo, hi;
    xxh3_wave_tail_merge(P.blocks + r->span0, m.p0, m.len - kHdrLen, &kLongSecret, c0, c1, lo, hi);
    if (lo != m.ck_lo || hi != m.ck_hi) st = ST_CKSUM;
  }
  ok = ok && huge_wait_units(L, ub, npu, tag, npu, ready_upto, give_up);  // every unit's parse result
  if (st == ST_OK) {
    const uint32_t bad = __hip_atomic_load(&r->parse_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    st = m.st != ST_OK ? m.st : bad ? (int32_t)ST_PARSE : (int32_t)ST_OK;
  }
  // A chain that gave up decides nothing: its rows or parse results may be missing, so it
  // marks the block for decode_huge_chain_kernel, which runs after this kernel has ended
  // (every unit done) and writes the block's real status.
  if (!ok) st = ST_INCOMPLETE;
  if (lane == 0) gstore(P.status, r->b, st);
}

template <bool kAllFields>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void decode_huge_kernel(DecodeParams P, uint32_t chain_wgs) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* stage = smem + 64;
  uint32_t* cnt = reinterpret_cast<uint32_t*>(smem);  // [0, 1]: search counts; [2..]: per-wave partials
  const HugeHdr* hp = reinterpret_cast<const HugeHdr*>(P.huge_pool);
  const uint32_t n = hp->n3;
  if (!n) return;
  const HugeLayout L = huge_layout(P, n);
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const bool hash = !(P.flags & LSM_DECODE_PAYLOAD_VERIFIED);
  const bool stream = hp->stream != 0;
  if (blockIdx.x < chain_wgs) {
    if (!stream) return;  // (decode_huge_chain_kernel runs the chains after this kernel)
    // chain workgroups (dispatched first): wave q = 4 g + w takes blocks q, q + 4 chain_wgs, ...
    uint8_t* ring = smem + 64 + wave * kStreamRing * 1024;
    for (uint32_t i = 4 * blockIdx.x + wave; i < n; i += 4 * chain_wgs)
      if (L.rec[i].accepted) huge_chain_streamed(P, L, i, ring);
    return;
  }
  // Unit order: batches of B = 4 chain_wgs blocks (one per chain wave), window-major
  // inside a batch: virtual unit v = (batch, window c, block in batch), so the blocks
  // of a batch progress together, each chain streams behind its own, and a chain
  // wave's next block (the next batch) is produced while it finishes this one.
  // Without streaming: a run of consecutive units per workgroup (one block search
  // per run, and a window's first interval is the previous window's end).
  const uint32_t pgrid = gridDim.x - chain_wgs, pb = blockIdx.x - chain_wgs;
  const uint32_t B = 4 * chain_wgs, mx = hp->max_npu;
  const uint64_t vtot = stream ? (uint64_t)((n + B - 1) / B) * B * mx : hp->total_pu;
  // (streaming: unit v goes to workgroup v mod pgrid, so the whole grid works along the windows in
  // order and the chains stream behind it; a grid-sized run per workgroup made every window
  // progress at once and the chains wait for their last windows: 4 MiB 0.202 -> 0.256 ms)
  const uint64_t per = stream ? 1 : (vtot + pgrid - 1) / pgrid;
  const uint64_t v_begin = stream ? pb : (uint64_t)pb * per, v_end = stream ? vtot : min(vtot, v_begin + per);
  const uint64_t v_step = stream ? pgrid : 1;
  uint32_t iseq = !stream && v_begin < v_end ? last_le(L.ppre, n, v_begin) : 0;
  uint32_t carry_u = 0xFFFFFFFFu, carry_r = 0;  // unit whose r1 search answer is carry_r (block iseq)
#if defined(LSM_DIAG) && !defined(LSM_DIAG_NOTIME)
  // diagnostic builds: per-phase s_memtime totals of wave 0 (g_dec_phase[8..13], units in [14])
  uint64_t t_last = __builtin_amdgcn_s_memtime(), ph[8] = {};
  uint32_t nunits = 0;
#define HUGE_PHASE(k) DEC_PHASE(k)
#else
#define HUGE_PHASE(k)
#endif
  uint32_t pending = ~0u;  // a processed unit whose done flag is not yet published
  for (uint64_t v = v_begin; v < v_end; v += v_step) {
    HUGE_PHASE(6);
    uint32_t i, wc;
    uint64_t ub;
    if (stream) {
      const uint64_t bw = (uint64_t)B * mx, rem = v % bw;
      i = (uint32_t)(v / bw) * B + (uint32_t)(rem % B);
      wc = (uint32_t)(rem / B);
      if (i >= n) continue;
      if (!L.rec[i].accepted) continue;  // (uniform)
      ub = gload(L.ppre, i);
      if (wc >= gload(L.ppre, i + 1) - ub) continue;  // the block has fewer windows
    } else {
      while (iseq + 1 < n && gload(L.ppre, iseq + 1) <= v) ++iseq, carry_u = 0xFFFFFFFFu;
      i = iseq;
      if (!L.rec[i].accepted) continue;
      ub = gload(L.ppre, i);
      wc = (uint32_t)(v - ub);
    }
    const HugeRec* r = L.rec + i;
    const uint32_t u = (uint32_t)(ub + wc);
    const BlockMeta m = r->m;
    const TrailerInfo t = trailer_of(m);
    const uint32_t span = r->span;
    const uint8_t* gbase = P.blocks + r->span0;
    const uint32_t cs = wc * kHugeWin;
    const uint32_t ce = min(cs + kHugeWin, span), ss = min(ce + kHugeOverlap, span);
    {  // stage [cs, ss): wave w moves 1-KiB pieces w, w + 4, ...
      const uint32_t chunks = (ss - cs + 15) >> 4;
      const uint8_t* src = gbase + cs + 16 * lane;
      for (uint32_t c = wave; c * kWave < chunks; c += 4)
        if (c * kWave + lane < chunks)
          __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + 1024 * c), (lds_void_t*)(stage + 1024 * c), 16, 0, 0);
    }
    // the intervals that start in [cs, ce): [r0, r1), from the unit table, or (a binary index
    // that is not monotone) by a 256-way search of the binary index (HBM)
    const bool parse = m.st == ST_OK;
    const bool table = !r->nonmono;
    uint32_t r0 = 0, r1 = 0, stop1 = 0;  // stop1: payload offset where the window's last interval ends
    if (parse && table) {
      const uint4 e0 = L.uend[-1 - (int64_t)u];
      const bool last = ce == span;
      const uint2 e1 = last ? make_uint2(t.bin_len, t.rec_end) : make_uint2(L.uend[-2 - (int64_t)u].x, L.uend[-2 - (int64_t)u].y);
      r0 = cs == 0 ? 0 : e0.x;
      r1 = last ? t.bin_len : e1.x;
      stop1 = e1.y;
    } else if (parse) {
      const uint32_t nint = t.bin_len, p0 = m.p0;
      uint32_t lo0 = 0, hi0 = nint, lo1 = 0, hi1 = nint;  // r0 in [lo0, hi0], r1 in [lo1, hi1]
      if (carry_u + 1 == u) lo0 = hi0 = carry_r;
      while (hi0 > lo0 || hi1 > lo1) {  // (uniform) each round narrows both ranges 256-fold
        const uint32_t len0 = hi0 - lo0, len1 = hi1 - lo1;
        const uint32_t st0 = (len0 + 255) / 256, st1 = (len1 + 255) / 256;
        const uint32_t x0 = lo0 + tid * st0, x1 = lo1 + tid * st1;
        const bool b0 = x0 < hi0 && p0 + bin_get(gbase, p0, t, x0) < cs;
        const bool b1 = x1 < hi1 && p0 + bin_get(gbase, p0, t, x1) < ce;
        const uint32_t c0 = (uint32_t)__builtin_popcountll(__ballot(b0)), c1 = (uint32_t)__builtin_popcountll(__ballot(b1));
        if (lane == 0) cnt[2 + wave] = c0, cnt[6 + wave] = c1;
        lds_barrier();
        const uint32_t k0 = cnt[2] + cnt[3] + cnt[4] + cnt[5], k1 = cnt[6] + cnt[7] + cnt[8] + cnt[9];
        lds_barrier();
        // k samples lie below the bound (a prefix of them, for monotone starts): the
        // answer is in (lo + (k - 1) st, lo + k st]; with st = 1 the range closes
        if (len0) {
          const uint32_t nlo = k0 ? lo0 + (k0 - 1) * st0 + 1 : lo0;
          hi0 = min(hi0, lo0 + k0 * st0);
          lo0 = min(nlo, hi0);
        }
        if (len1) {
          const uint32_t nlo = k1 ? lo1 + (k1 - 1) * st1 + 1 : lo1;
          hi1 = min(hi1, lo1 + k1 * st1);
          lo1 = min(nlo, hi1);
        }
      }
      // the same bound gives the same answer in the neighbouring unit, and the first
      // / last windows take every interval before / after: each interval is walked
      // at least once even when the binary index is not monotone (its walk then fails)
      r0 = cs == 0 ? 0 : lo0;
      r1 = ce == span ? nint : lo1;
      carry_u = stream ? 0xFFFFFFFFu : u;  // (streaming: the next unit is another block's)
      carry_r = lo1;
    }
    const uint8_t* sbase = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(stage) - cs);  // span-relative
    HUGE_PHASE(0);
    if (parse) {
      const uint64_t item_base = r->item_base;
      const uint32_t p0 = m.p0, ri = t.ri, niv = r1 - r0;
      const uint32_t items_w = niv ? min(r1 * ri, t.item_count) - r0 * ri : 0;
      // phase A / B when every interval of the window is staged (a wave-uniform vote)
      bool fast = m.type != 1 && niv <= kHugeMaxIv && items_w <= kHugeTile;
      if (fast && table) {  // (monotone: every interval of the window ends by stop1)
        fast = r1 == r0 || (stop1 <= t.rec_end && (p0 + stop1 + kChunkReadAhead <= ss || ss == span));
      } else if (fast) {
        bool mine = true;
        for (uint32_t x = r0 + tid; x < r1; x += 256) {
          const uint32_t s_cur = bin_get(gbase, p0, t, x);
          const uint32_t stop = x + 1 == t.bin_len ? t.rec_end : bin_get(gbase, p0, t, x + 1);
          mine = mine && p0 + s_cur >= cs && stop <= t.rec_end && (p0 + stop + kChunkReadAhead <= ss || ss == span);
        }
        if (lane == 0) cnt[10 + wave] = __ballot(!mine) != 0;
        lds_barrier();
        fast = !(cnt[10] | cnt[11] | cnt[12] | cnt[13]);
      }
      uint8_t* bix = smem + 64 + kHugeBix;
      BlockMeta* wmeta = reinterpret_cast<BlockMeta*>(smem + 64 + kHugeMeta);
      uint8_t* owner = smem + 64 + kHugeOwner;
      uint64_t* rec = reinterpret_cast<uint64_t*>(smem + 64 + kHugeRec);
      if (fast) {
        // the entries r0 .. min(r1, nint - 1) as dwords next to the stage
        const uint32_t e1 = min(r1, t.bin_len - 1);
        const uint32_t eb = p0 + t.bin_off + r0 * t.step, elen = (e1 - r0 + 1) * t.step;
        for (uint32_t d = tid; 4 * d < elen; d += 256)
          reinterpret_cast<uint32_t*>(bix)[d] = read_u32_unaligned(gbase, eb + 4 * d);
        for (uint32_t x = tid; x < niv; x += 256) owner[x] = 0;
        for (uint32_t x = tid; x <= items_w; x += 256) rec[x] = 0;
        if (tid == 0) {
          BlockMeta w = m;
          w.p0 = m.p0 - cs;  // stage offsets (the window starts at span offset cs)
          w.rec_end = m.rec_end - cs;
          w.bin_off = kHugeBix - w.p0 - r0 * t.step;  // bin_get(stage, w.p0, r) reads bix[r - r0]
          w.item0 = 0u - r0 * ri;                     // descriptors numbered from the window's first item
          w.chain0 = 0u - r0;                         // phase A's interval c is interval r0 + c
          w.st = ST_OK;
          *wmeta = w;
        }
      }
      HUGE_PHASE(1);
      vm_wait<0>();
      lds_barrier();
      if (tid == 0 && pending != ~0u)  // (streaming) the previous unit: its stores have completed (vmcnt(0) above)
        __hip_atomic_store(&L.uend[-1 - (int64_t)pending].z, P.huge_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      HUGE_PHASE(2);
      // phase A (serial LDS walks: latency) on wave 0, the contributions (VALU) on the
      // other waves meanwhile; without phase A on all four
      const bool split = fast;
      if (fast && (split ? wave == 0 : true)) {
        if (split) __builtin_amdgcn_s_setprio(2);  // (the walk is the unit's longest role)
        phase_a<true>(stage, wmeta, owner, rec, split ? 0 : wave * kWave, split ? kWave : 4 * kWave, niv, kHugeTile);
        __builtin_amdgcn_s_setprio(0);
      }
      HUGE_PHASE(3);
      if (hash && r->nbk && (!split || wave != 0)) {  // the KiB blocks that start in [cs, ce)
        const uint32_t nbk = r->nbk;
        const uint32_t n0 = min(nbk, cs > p0 ? (cs - p0 + 1023) / 1024 : 0u);
        const uint32_t n1 = min(nbk, ce > p0 ? (ce - p0 + 1023) / 1024 : 0u);
        if (n1 > n0) {  // (streaming: agent-scope stores, read by a chain wave of this launch)
          if (stream)
            xxh3_kib_contribs<true, true>(stage, p0 + 1024 * n0 - cs, (n1 - n0) * 1024 + 1, &kLongSecret,
                                          L.contrib + 8 * (gload(L.kpre, i) + n0), split ? wave - 1 : wave, split ? 3 : 4);
          else
            xxh3_kib_contribs(stage, p0 + 1024 * n0 - cs, (n1 - n0) * 1024 + 1, &kLongSecret,
                              L.contrib + 8 * (gload(L.kpre, i) + n0), split ? wave - 1 : wave, split ? 3 : 4);
        }
      }
      HUGE_PHASE(4);
      bool walk = !fast;
      if (fast) {
        lds_barrier();
        phase_b<kAllFields, false, true>(P, stage, wmeta, rec, items_w, (uint32_t)(item_base + r0 * ri), tid, 256);
        lds_barrier();
        const int32_t wst = wmeta->st;
        if (wst == ST_PARSE && tid == 0) atomicOr(const_cast<uint32_t*>(&r->parse_bad), 1u);
        walk = wst == ST_DEFER;  // a record shape the straight-line parsers do not take: the LEB cursor
      }
      if (walk) {
        bool ok = true;
        for (uint32_t x = r0 + tid; x < r1; x += 256) {
          const uint32_t s_cur = bin_get(gbase, p0, t, x);
          const bool last = x + 1 == t.bin_len;
          const uint32_t stop = last ? t.rec_end : bin_get(gbase, p0, t, x + 1);
          const bool staged = p0 + s_cur >= cs && stop <= t.rec_end && (p0 + stop + kChunkReadAhead <= ss || ss == span);
          ok &= walk_interval_at(staged ? sbase : gbase, p0, m, t, x, s_cur, stop, [&](uint32_t j, const ItemFields& f) {
            emit_global(P.out, item_base + j, f, P.seqno_add, P.compact);
          });
        }
        const uint64_t bad = __ballot(!ok);
        if (bad && lane == (uint32_t)__builtin_ctzll(bad)) atomicOr(const_cast<uint32_t*>(&r->parse_bad), 1u);
      }
    } else if (hash && r->nbk) {
      vm_wait<0>();
      lds_barrier();
      if (tid == 0 && pending != ~0u)  // (streaming) the previous unit: its stores have completed (vmcnt(0) above)
        __hip_atomic_store(&L.uend[-1 - (int64_t)pending].z, P.huge_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t p0 = m.p0, nbk = r->nbk;
      const uint32_t n0 = min(nbk, cs > p0 ? (cs - p0 + 1023) / 1024 : 0u);
      const uint32_t n1 = min(nbk, ce > p0 ? (ce - p0 + 1023) / 1024 : 0u);
      if (n1 > n0) {
        if (stream)
          xxh3_kib_contribs<true, true>(stage, p0 + 1024 * n0 - cs, (n1 - n0) * 1024 + 1, &kLongSecret,
                                        L.contrib + 8 * (gload(L.kpre, i) + n0), wave, 4);
        else
          xxh3_kib_contribs(stage, p0 + 1024 * n0 - cs, (n1 - n0) * 1024 + 1, &kLongSecret,
                            L.contrib + 8 * (gload(L.kpre, i) + n0), wave, 4);
      }
    }
    HUGE_PHASE(5);
    lds_barrier();  // (the next unit rewrites the stage)
    // published after the next unit's DMA wait (vmcnt(0): this unit's contribution
    // stores and parse_bad update have completed by then), or after the loop
    if (stream) pending = u;
#if defined(LSM_DIAG) && !defined(LSM_DIAG_NOTIME)
    ++nunits;
#endif
  }
  if (pending != ~0u) {
    vm_wait<0>();
    lds_barrier();
    if (tid == 0) __hip_atomic_store(&L.uend[-1 - (int64_t)pending].z, P.huge_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#if defined(LSM_DIAG) && !defined(LSM_DIAG_NOTIME)
  if (threadIdx.x == 0) {
    for (int k = 0; k < 7; ++k) atomicAdd(&g_dec_phase[8 + k], (unsigned long long)ph[k]);
    atomicAdd(&g_dec_phase[15], (unsigned long long)nunits);
  }
#endif
#undef HUGE_PHASE
}

// Chains of the huge blocks when they do not stream, and, when they stream,
// of the blocks whose streamed chain gave up (status ST_INCOMPLETE; every
// other block returns at once): a single-wave workgroup per block,
// its eight accumulators on lanes 0..7 (xxh3_chain8), then on the same wave
// the tail merge, the checksum compare and the status (oracle order: payload
// checksum, then trailer, then parse).  The contributions cross a kernel
// boundary here; the chain results stay in the wave.
__global__ __launch_bounds__(64) void decode_huge_chain_kernel(DecodeParams P) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[kChainRing * 1024];
  const HugeHdr* hp = reinterpret_cast<const HugeHdr*>(P.huge_pool);
  const uint32_t n = hp->n3;
  if (!n) return;
  const bool streamed = hp->stream != 0;
  if (streamed && kDiagBuild && (P.flags & kDiagNoChainFallback)) return;
  const HugeLayout L = huge_layout(P, n);
  const bool hash = !(P.flags & LSM_DECODE_PAYLOAD_VERIFIED);
  const uint32_t lane = threadIdx.x & 63, k = lane & 7, q = lane & 3;
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const HugeRec* r = L.rec + i;
    if (!r->accepted) continue;
    if (streamed && gload(P.status, r->b) != ST_INCOMPLETE) continue;  // (the streamed chain decided it)
    const BlockMeta m = r->m;
    int32_t st = m.st != ST_OK ? m.st : r->parse_bad ? (int32_t)ST_PARSE : (int32_t)ST_OK;
    if (hash) {
      uint64_t a0, a1;
      xxh3_acc_init((int)(k >> 1), a0, a1);
      uint64_t x = (k & 1) ? a1 : a0;
      if (r->nbk)
        x = xxh3_chain8<kChainRing>(L.contrib + 8 * gload(L.kpre, i), r->nbk, x, kLongSecret.acc[16 + k], ring);
      // lane quad position q takes accumulators 2q, 2q + 1 (lanes 2q, 2q + 1 hold them)
      const uint64_t c0 = wave_shfl_u64(x, (int)(2 * q)), c1 = wave_shfl_u64(x, (int)(2 * q + 1));
      uint64_t lo, hi;
      xxh3_wave_tail_merge(P.blocks + r->span0, m.p0, m.len - kHdrLen, &kLongSecret, c0, c1, lo, hi);
      if (lo != m.ck_lo || hi != m.ck_hi) st = ST_CKSUM;
    }
    if (lane == 0) gstore(P.status, r->b, st);
  }
}

// Workgroup = kGroupWaves waves sharing one LDS stage (default 32 KiB: eight
// 4-KiB blocks, ~32 restart intervals).  Per group:
//   all waves   LDS-DMA of the span (wave w moves 1-KiB pieces w, w+4, ...)
//   wave 0      headers + trailers (lane j = block j), interval numbering
//   wave pa     phase A over all intervals (every lane walks one interval)
//   other waves payload checksums (16-lane DPP rows, four blocks per wave)
//   all waves   phase B (thread = record), coalesced SoA stores
// pa rotates with the group index so the serial walk lands on each SIMD in
// turn.  Phase A needs only the trailer, not the checksum, so it runs
// concurrently with the hash; statuses merge in oracle order at the end.
constexpr uint32_t kGroupWaves = 4;
// 17-bit record descriptors for stages of 64 KiB and more (two 8-wave workgroups per CU)
constexpr bool kDecWide = kDefaultStageBytes >= 65536;

template <bool kAllFields, bool kCompact>
__global__ __launch_bounds__(kGroupWaves * kWave) __attribute__((amdgpu_waves_per_eu(3))) void decode_blocks_kernel(DecodeParams P) {
  // LDS: [meta: G x 80 B][rec: u64 per item + 1 scratch][owner: u8 per item][staged bytes + pad][secret]
#if defined(LSM_DIAG) && !defined(LSM_DIAG_NOTIME)
  uint64_t t_last = __builtin_amdgcn_s_memtime(), ph[16] = {};
#endif
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t gmax = min(kMaxGroup, P.blocks_per_wave);
  BlockMeta* meta = reinterpret_cast<BlockMeta*>(smem);
  uint64_t* rec = reinterpret_cast<uint64_t*>(smem + gmax * (uint32_t)sizeof(BlockMeta));
  uint8_t* owner = reinterpret_cast<uint8_t*>(rec) + ((8 * (P.tile_items + 1) + 15) & ~15u);
  uint8_t* img = owner + ((P.tile_items + 15) & ~15u);
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int lane = tid & (kWave - 1);
  const uint32_t b_begin = blockIdx.x * P.blocks_per_wave;
  const uint32_t b_end = min(b_begin + P.blocks_per_wave, P.n_blocks);
  // the workgroup's handles and item starts, once per wave (blocks_per_wave <= 63)
  uint64_t offr = 0;
  uint32_t itr = 0;
  if (b_begin + lane <= b_end) {
    offr = gload(P.block_off, b_begin + lane);
    itr = gload(P.item_start, b_begin + lane);
  }
  // XXH3 long-path secret words in LDS (read per use by the lean row hash).
  const uint32_t slot_stride = ((P.stage_bytes + 15) & ~15u) + kStagePad;
  LongSecret* ls = reinterpret_cast<LongSecret*>(img + slot_stride);
  if (tid < sizeof(LongSecret) / 8)
    reinterpret_cast<uint64_t*>(ls)[tid] = reinterpret_cast<const uint64_t*>(&kLongSecret)[tid];
  uint32_t iter = 0;
  // Next stageable group at or after bb (larger blocks go to the general path).
  auto next_group = [&](uint32_t bb) -> Group {
    for (;;) {
      if (bb >= b_end) {
        Group z;
        z.b = bb;
        z.k = 0;
        return z;
      }
      uint32_t skip;
      const Group g = form_group(P, bb, b_begin, b_end, gmax, offr, itr, skip);
      if (g.k) return g;
      bb += skip;  // a run of lone blocks: listed for the general path before the loop
    }
  };
  // LDS-DMA of a group's span (wave w moves 1-KiB pieces w, w + 4, ...).
  auto issue_dma = [&](const Group& g, uint8_t* dst) {
    const uint32_t chunks = (kDiagBuild && (P.flags & kDiagSkipDma)) ? 0u : (uint32_t)((g.span1 - g.span0) >> 4);
    const uint8_t* src = P.blocks + g.span0 + 16 * lane;
    for (uint32_t i = wave; i * kWave < chunks; i += kGroupWaves) {
      if (i * kWave + lane < chunks)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + 1024 * i), (lds_void_t*)(dst + 1024 * i), 16, 0, 0);
    }
  };
  // Lone blocks (larger than the stage, or more items than a tile) go to the
  // general path, decode_deferred_staged_kernel (a 72 KiB stage, the block
  // hashed by four waves): listed here, one atomic per workgroup.
  if (wave == 0) {
    const uint64_t nx = wave_shfl_u64(offr, min(lane + 1, kWave - 1));
    const uint32_t ix = (uint32_t)__shfl((int)itr, min(lane + 1, kWave - 1));
    const bool in = b_begin + lane < b_end;
    const bool lone = in && (((nx + 15) & ~15ULL) - (offr & ~15ULL) > lone_bytes(P) || ix - itr > P.tile_items);
    defer_blocks_wave(P, lone, b_begin + lane);
  }
  Group G = next_group(b_begin);
  if (G.k) issue_dma(G, img);
  for (; G.k; ++iter) {
    const uint32_t b = G.b;
    const uint32_t k = G.k;
    uint8_t* const stage = img;
    // ---- 1. this group's span has landed; clear the record descriptors
    for (uint32_t i = tid; i < G.n_items; i += kGroupWaves * kWave) rec[i] = 0;
    vm_wait<0>();
    lds_barrier();
    DEC_PHASE(0);
    const Group Gn = next_group(b + k);
    // ---- 2. wave 0: headers, trailers, restart-interval numbering; owner[c] = block of interval c
    if (wave == 0 && !(kDiagBuild && (P.flags & kDiagSkipHeader))) {
      uint32_t chains = 0;
      BlockMeta m;
      if ((uint32_t)lane < k) {
        meta_header_fields(stage, (uint32_t)(G.off_j - G.span0), G.end_j - G.off_j, m);
        m.item0 = G.it0_j - G.g_item0;
        m.hdr_st = m.st;
        m.ck_bad = 0;
        m.hck_bad = 0;
        meta_trailer(stage, P.expect_type, G.it1_j - G.it0_j, m, P.compact);
        if (m.st == ST_OK && m.type == 1) m.st = ST_DEFER;  // index blocks: general path
        chains = m.st == ST_OK ? m.bin_len : 0;
      }
      const uint32_t incl = wave_incl_scan_u32(chains);
      if ((uint32_t)lane < k) {
        m.chain0 = incl - chains;
        meta[lane] = m;
        for (uint32_t r = 0; r < chains; ++r) owner[m.chain0 + r] = (uint8_t)lane;
      }
    }
    lds_barrier();
    DEC_PHASE(1);
    // ---- 3. phase A on nA waves (64 intervals each)  ||  payload checksums on the others
    {
      const uint32_t total = (kDiagBuild && (P.flags & kDiagSkipParse)) ? 0
                             : meta[k - 1].chain0 + (meta[k - 1].st == ST_OK ? meta[k - 1].bin_len : 0);
      const uint32_t nA = min((total + kWave - 1) / kWave, kGroupWaves - 1);
      const uint32_t role = (wave + kGroupWaves - iter % kGroupWaves) % kGroupWaves;  // rotates per group
      // payload checksums (not when verified upstream: the LZ4 path checks the stored bytes)
      const bool hash = !(kDiagBuild && (P.flags & kDiagSkipHash)) && !(P.flags & LSM_DECODE_PAYLOAD_VERIFIED);
      if (role < nA) {
        phase_a<kDecWide>(stage, meta, owner, rec, role * kWave, nA * kWave, total, P.tile_items);
        DEC_ROLE(8);
      } else if (hash && (k <= kGroupWaves - nA || (k <= (kGroupWaves - nA) * 4 && (role - nA) * 4 + 1 == k))) {
        // few (large) blocks: one wave per block, the 64-lane XXH3 (1 KiB per
        // step); also a wave whose share of the rows below is one block
        // (k = 4 h + 1, e.g. nine 4 KiB blocks on three hash waves): the whole
        // wave hashes it instead of one row with three rows idle
        const uint32_t jb = k <= kGroupWaves - nA ? role - nA : k - 1;
        if (jb < k && meta[jb].hdr_st == ST_OK) {
          const uint32_t hb = meta[jb].hb, plen = meta[jb].len - kHdrLen;
          uint64_t lo, hi;
          xxh3_128_wave(stage, hb + kHdrLen, plen, ls, lo, hi);
          const bool hck = header_cksum_ok(stage, hb);
          if (lane == 0) {
            meta[jb].ck_bad = lo != meta[jb].ck_lo || hi != meta[jb].ck_hi;
            meta[jb].hck_bad = !hck;
          }
        }
        DEC_ROLE(10);
      } else if (hash) {
        const uint32_t rows = (kGroupWaves - nA) * 4;
        for (uint32_t jb = (role - nA) * 4 + (lane >> 4); jb < k; jb += rows) {
          if (meta[jb].hdr_st != ST_OK) continue;
          const uint32_t hb = meta[jb].hb, len = meta[jb].len;
          uint64_t lo, hi;
          const uint32_t plen = len - kHdrLen;
          if (plen > 240) xxh3_128_row_long_lean(stage, hb + kHdrLen, plen, ls, lo, hi);
          else xxh3_128_short(plen, BaseReader8{stage, hb + kHdrLen}, BaseReader64{stage, hb + kHdrLen}, lo, hi);
          const bool hck = header_cksum_ok(stage, hb);
          if ((lane & 15) == 0) {
            meta[jb].ck_bad = lo != meta[jb].ck_lo || hi != meta[jb].ck_hi;
            meta[jb].hck_bad = !hck;
          }
        }
        DEC_ROLE(12);
      }
    }
    lds_barrier();
    DEC_PHASE(2);
    // ---- 4. phase B: thread = record; full parse + validation; coalesced stores
    if (!(kDiagBuild && (P.flags & (kDiagSkipParse | kDiagSkipPhaseB))))
      phase_b<kAllFields, kCompact, kDecWide>(P, stage, meta, rec, G.n_items, G.g_item0, threadIdx.x, blockDim.x);
    lds_barrier();
    DEC_PHASE(3);
    // refill the stage after phase B, before wave 0's status merge (which reads
    // only meta): 0.2-0.8 % faster than after it over five batch shapes
    if (Gn.k) issue_dma(Gn, img);
    if (wave == 0) {
      int32_t st = ST_OK;
      if ((uint32_t)lane < k) {
        const BlockMeta& m = meta[lane];
        st = m.hdr_st != ST_OK ? m.hdr_st
             : m.hck_bad ? (int32_t)ST_HDR_CKSUM
             : m.ck_bad  ? (int32_t)ST_CKSUM
                         : m.st;
        if (st != ST_DEFER) gstore(P.status, b + lane, st);
      }
      defer_blocks_wave(P, (uint32_t)lane < k && st == ST_DEFER, b + lane);
    }
    DEC_PHASE(4);
#if defined(LSM_DIAG) && !defined(LSM_DIAG_NOTIME)
    ph[5] += 1;
    ph[6] += k;
#endif
    G = Gn;
  }
#if defined(LSM_DIAG) && !defined(LSM_DIAG_NOTIME)
  if (lane == 0) {
    for (int i = 0; i < 16; ++i)
      if ((i >= 8 || wave == 0) && ph[i]) atomicAdd(&g_dec_phase[16 + i], (unsigned long long)ph[i]);
  }
#endif
}

// item counts from the trailers (trailer.rs:57-75), same rule as
// oracle/batch.c: 0 unless the handle holds header + a 32-byte minimum payload,
// and at most (payload - 32) / 3 (every record is >= 3 bytes), so a corrupt,
// not-yet-verified trailer cannot reserve more than its bytes could hold.
__device__ __forceinline__ uint64_t trailer_count(const uint8_t* __restrict__ blocks, const uint64_t* __restrict__ off,
                                                  uint32_t b) {
  const uint64_t o = off[b], e = off[b + 1];
  uint64_t c = 0;
  if (e >= o && e - o >= kHdrLen + kTrailerLen + 1) {
    const uint8_t* p = blocks + e - 4;
    c = (uint64_t)p[0] | ((uint64_t)p[1] << 8) | ((uint64_t)p[2] << 16) | ((uint64_t)p[3] << 24);
    const uint64_t most = (e - o - kHdrLen - 32) / 3;  // records are >= 3 bytes each
    c = c < most ? c : most;
  }
  return c;
}

// (workgroup 0 also clears the call's four list counters: no clear launch of their own)
__global__ __launch_bounds__(256) void trailer_counts_kernel(const uint8_t* __restrict__ blocks,
                                                             const uint64_t* __restrict__ off, uint32_t n,
                                                             uint64_t* __restrict__ counts, uint32_t* __restrict__ clear4) {
  if (blockIdx.x == 0 && threadIdx.x < 4) clear4[threadIdx.x] = 0;
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  counts[b] = trailer_count(blocks, off, b);
}

// Batches of at most one scan tile (kScanTile blocks): the counts and their
// exclusive scan into item_start in one workgroup (one launch, not two), and
// the four list counters cleared.
__global__ __launch_bounds__(kScanThreads) void trailer_counts_scan_kernel(const uint8_t* __restrict__ blocks,
                                                                           const uint64_t* __restrict__ off, uint32_t n,
                                                                           uint32_t* __restrict__ item_start, uint64_t cap,
                                                                           uint32_t* __restrict__ clear4) {
  __shared__ uint64_t sh[kScanThreads / 64];
  if (threadIdx.x < 4) clear4[threadIdx.x] = 0;
  const uint32_t base = threadIdx.x * kScanPerThread;
  uint64_t v[kScanPerThread], s = 0;
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) {
    v[i] = base + i < n ? trailer_count(blocks, off, base + i) : 0;
    s += v[i];
  }
  uint64_t total;
  uint64_t ex = block_excl_scan_u64(s, sh, total);
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) {
    if (base + i < n) item_start[base + i] = (uint32_t)(ex < cap ? ex : cap);
    ex += v[i];
    if (base + i + 1 == n) item_start[n] = (uint32_t)(ex < cap ? ex : cap);
  }
}

struct ItemStartOut {
  uint32_t* item_start;
  uint64_t cap;
  __device__ void operator()(uint64_t i, uint64_t prefix) const {
    item_start[i] = (uint32_t)(prefix < cap ? prefix : cap);
  }
};

static size_t counts_bytes(uint32_t n_blocks) { return ((size_t)n_blocks * 8 + 255) / 256 * 256; }
static size_t tiles_bytes(uint32_t n_blocks) { return (scan_tiles(n_blocks) * 8 + 255) / 256 * 256; }
static size_t defer_bytes(uint32_t n_blocks) { return ((size_t)n_blocks * 4 + 255) / 256 * 256; }

// counts | scan tiles | 256 B of counters (defer, defer2, defer3) | three block lists
size_t decode_workspace_size(uint32_t n_blocks) {
  return counts_bytes(n_blocks) + tiles_bytes(n_blocks) + 256 + 3 * defer_bytes(n_blocks);
}

// + the huge-block pool for a batch of blocks_bytes bytes: every huge block
// spans more than kBigStage bytes, contributions 64 B per KiB, unit entries
// 8 B per kHugeWin window (and one more per block).
size_t decode_pool_min_bytes(uint32_t n_blocks) {
  static_assert(huge_fixed_bytes(1) + 64 * 128 == 8704, "the threshold lsmgpu.h documents");
  return ((decode_workspace_size(n_blocks) + 255) & ~(size_t)255) + huge_fixed_bytes(1) + 64 * 128;
}

size_t decode_workspace_size_ex(uint32_t n_blocks, uint64_t blocks_bytes) {
  const uint64_t most = blocks_bytes / kBigStage + 1;
  const uint64_t n3 = most < n_blocks ? most : n_blocks;
  const size_t ex = decode_workspace_size(n_blocks) + huge_fixed_bytes(n3) + 64 * (blocks_bytes / 1024 + 1 + 16 * n3) +
                    16 * (blocks_bytes / kHugeWin + n3 + 1) + 256;
  return ex > decode_pool_min_bytes(n_blocks) ? ex : decode_pool_min_bytes(n_blocks);
}

uint32_t decode_lds_bytes(uint32_t stage_bytes, uint32_t tile_items, uint32_t blocks_per_wave) {
  const uint32_t g = blocks_per_wave < kMaxGroup ? blocks_per_wave : kMaxGroup;
  return g * (uint32_t)sizeof(BlockMeta) + ((8 * (tile_items + 1) + 15) & ~15u) + ((tile_items + 15) & ~15u) +
         ((stage_bytes + 15) & ~15u) + kStagePad + (uint32_t)sizeof(LongSecret);
}

hipError_t launch_decode(const DecodeParams& P0, void* ws, size_t ws_bytes, hipStream_t st) {
  DecodeParams P = P0;
  uint64_t* counts = (uint64_t*)ws;
  uint64_t* tiles = (uint64_t*)((uint8_t*)ws + counts_bytes(P.n_blocks));
  uint8_t* dws = (uint8_t*)ws + counts_bytes(P.n_blocks) + tiles_bytes(P.n_blocks);
  P.defer_count = (uint32_t*)dws;
  P.defer2_count = (uint32_t*)dws + 1;
  P.defer3_count = (uint32_t*)dws + 2;
  P.defer_list = (uint32_t*)(dws + 256);
  P.defer2_list = (uint32_t*)(dws + 256 + defer_bytes(P.n_blocks));
  P.defer3_list = (uint32_t*)(dws + 256 + 2 * defer_bytes(P.n_blocks));
  const size_t base = decode_workspace_size(P.n_blocks);
  const size_t pool0 = (base + 255) & ~(size_t)255;
  // the pool only when the caller asks for it (LSM_DECODE_HUGE_POOL; the ABI checked the size)
  P.huge_pool = (P.flags & LSM_DECODE_HUGE_POOL) && ws_bytes >= decode_pool_min_bytes(P.n_blocks)
                    ? (uint8_t*)ws + pool0 : nullptr;
  P.huge_pool_bytes = P.huge_pool ? ws_bytes - pool0 : 0;
  hipError_t e = hipSuccess;
  if (P.flags & LSM_DECODE_ITEM_START_VALID) {
    if ((e = fill_words_async(dws, 4, 0, st)) != hipSuccess) return e;
  } else if (scan_tiles(P.n_blocks) == 1) {  // (the counts kernel clears the list counters)
    hipLaunchKernelGGL(trailer_counts_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, P.blocks, P.block_off,
                       P.n_blocks, P.item_start_w, P.item_cap, (uint32_t*)dws);
  } else {
    hipLaunchKernelGGL(trailer_counts_kernel, dim3((P.n_blocks + 255) / 256), dim3(256), 0, st, P.blocks,
                       P.block_off, P.n_blocks, counts, (uint32_t*)dws);
    if ((e = launch_excl_scan(counts, P.n_blocks, tiles, ItemStartOut{P.item_start_w, P.item_cap}, st)) != hipSuccess)
      return e;
  }
  const uint32_t lds = decode_lds_bytes(P.stage_bytes, P.tile_items, P.blocks_per_wave);
  const bool all = all_fields(P.out);
  // kernel variants: every field present or not, 32- or 16-bit offsets
  const int variant = (all ? 1 : 0) | (P.compact ? 2 : 0);
  const void* const group_k[4] = {(const void*)decode_blocks_kernel<false, false>,
                                  (const void*)decode_blocks_kernel<true, false>,
                                  (const void*)decode_blocks_kernel<false, true>,
                                  (const void*)decode_blocks_kernel<true, true>};
  const void* const big_k[4] = {(const void*)decode_big_kernel<false, false>, (const void*)decode_big_kernel<true, false>,
                                (const void*)decode_big_kernel<false, true>, (const void*)decode_big_kernel<true, true>};
  if (lds > 64 * 1024) {
    static uint64_t done[4] = {};
    if ((e = set_lds_attr(group_k[variant], 160 * 1024, &done[variant])) != hipSuccess) return e;
  }
  const uint32_t grid = (P.n_blocks + P.blocks_per_wave - 1) / P.blocks_per_wave;
  void* args[] = {&P};
  if ((e = hipLaunchKernel(group_k[variant], dim3(grid), dim3(kGroupWaves * kWave), args, lds, st)) != hipSuccess)
    return e;
  // listed blocks: the big-block kernel (two workgroups per CU), then the
  // general path for what it hands on (its list read as defer_count / defer_list)
  static int cu_count[64] = {};  // per device (benign race: every writer stores the same count)
  int dev = 0;
  if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
  int n_cu = dev < 64 ? __atomic_load_n(&cu_count[dev], __ATOMIC_RELAXED) : 0;
  if (!n_cu) {
    if ((e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
    if (dev < 64) __atomic_store_n(&cu_count[dev], n_cu, __ATOMIC_RELAXED);
  }
  const uint32_t bgrid = min(P.n_blocks, (uint32_t)n_cu * kBigGPerCU);
  if (bgrid) {
    static uint64_t done_bg[4] = {};
    if ((e = set_lds_attr(big_k[variant], kBigGLds, &done_bg[variant])) != hipSuccess) return e;
    if ((e = hipLaunchKernel(big_k[variant], dim3(bgrid), dim3(kBigGWaves * kWave), args, kBigGLds, st)) != hipSuccess)
      return e;
  }
  if (P.huge_pool && bgrid) {  // the huge blocks the big-block kernel listed: plan (rejects go to defer2)
    static uint64_t done_hp = 0;
    if ((e = set_lds_attr((const void*)decode_huge_plan_kernel, 1024 * kHugePlanStage, &done_hp)) != hipSuccess) return e;
    hipLaunchKernelGGL(decode_huge_plan_kernel, dim3(1), dim3(1024), 1024 * kHugePlanStage, st, P);
  }
  const uint32_t dgrid = P.n_blocks < 1024 ? P.n_blocks : 1024;
  if (dgrid) {
    DecodeParams P2 = P;
    P2.defer_count = P.defer2_count;
    P2.defer_list = P.defer2_list;
    static uint64_t done_big = 0;
    const uint32_t big = kBigStageOff + kBigStage + kStagePad;
    if ((e = set_lds_attr((const void*)decode_deferred_staged_kernel, big, &done_big)) != hipSuccess) return e;
    hipLaunchKernelGGL(decode_deferred_staged_kernel, dim3(dgrid), dim3(kBigWaves * kWave), big, st, P2);
  }
  if (P.huge_pool && bgrid) {
    P.huge_tag = 1;  // (the units kernel clears the flags first)
    const void* hk = all ? (const void*)decode_huge_kernel<true> : (const void*)decode_huge_kernel<false>;
    static uint64_t done_hk[2] = {};
    if ((e = set_lds_attr(hk, kHugeLds, &done_hk[all ? 1 : 0])) != hipSuccess) return e;
    hipLaunchKernelGGL(decode_huge_units_kernel, dim3(kHugeUnitsGrid), dim3(256), 0, st, P);
    // chain workgroups first (four blocks each, at most one per CU), then the units
    uint32_t chain_wgs = min((P.n_blocks + 3) / 4, kStreamChainWgs);
    void* hargs[] = {&P, &chain_wgs};
    // unit workgroups: as many as are resident beside the chain workgroups (one wave of
    // workgroups: no partly filled last wave; 256 KiB / 1 MiB decode 0.229 / 0.202 -> 0.220 / 0.196 ms
    // against a 2048-workgroup grid)
    const uint32_t ugrid = max(64u, kHugeWgsPerCU * (uint32_t)n_cu - chain_wgs);
    if ((e = hipLaunchKernel(hk, dim3(chain_wgs + ugrid), dim3(256), hargs, kHugeLds, st)) != hipSuccess) return e;
    // (when streamed: only the blocks whose chain gave up, LSM_INCOMPLETE; the others return at once)
    hipLaunchKernelGGL(decode_huge_chain_kernel, dim3(kHugeChainGrid), dim3(64), 0, st, P);
  }
  return hipGetLastError();
}

}  // namespace lsmgpu

#if defined(LSM_DIAG) && !defined(LSM_DIAG_NOTIME)
// Diagnostic builds only: copy out and clear the big-block kernel's phase totals.
// Entries 16..31 are the group kernel's (wave 0 per group, role timers summed over waves).
extern "C" int lsm_diag_decode_phases(uint64_t* out32) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out32, HIP_SYMBOL(lsmgpu::g_dec_phase), 32 * sizeof(uint64_t)) != hipSuccess) return -1;
  static const uint64_t z[32] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(lsmgpu::g_dec_phase), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
