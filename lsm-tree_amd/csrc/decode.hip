// decode.hip — batched SST block decode on gfx950 (the north-star hot path).
//
// Replaces, per block, Block::from_file (header decode + xxh3_128 verify,
// src/table/block/mod.rs:131-182), the load_block type check
// (src/table/util.rs:79-86) and the full forward DataBlock::iter() /
// IndexBlock::iter() (src/table/block/decoder.rs:442-483) over a whole batch.
//
// Launch shape (DESIGN.md "Decode kernel"): one 64-lane wave per workgroup,
// wave w owns blocks [w*BPW, (w+1)*BPW) and walks them in GROUPS — the longest
// run of consecutive blocks that fits the LDS stage (consecutive blocks are
// contiguous on disk, so a group is one contiguous span):
//   1. lane j holds block j's handle and item range in registers;
//   2. the span is copied HBM -> LDS with global_load_lds_dwordx4 (1 KiB per
//      wave instruction), one wait per group;
//   3. lane j checks block j's header (magic, type, 29-byte xxh3 checksum);
//   4. the four 16-lane DPP rows hash four payloads at a time (xxh3_128);
//   5. lane j reads block j's trailer, a wave scan numbers the restart
//      intervals of the group;
//   6. phase A: lane = restart interval, walks record boundaries only;
//   7. phase B: lane = record, parses and validates every field and stores
//      the parsed-item SoA with coalesced global stores.
// Blocks larger than the stage take decode_block_direct (same parsers on HBM).
#include <hip/hip_runtime.h>

#include "block_format.hpp"
#include "decode.hpp"
#include "lds_dma.hpp"
#include "scan.hpp"

namespace lsmgpu {

// Diagnostic-only flags (lsm_decode_tuning.flags high bits): drop one phase to
// price it in a profile.  Outputs are NOT valid with any of them set.
constexpr uint32_t kDiagSkipHash = 0x100, kDiagSkipParse = 0x200, kDiagSkipStore = 0x400,
                   kDiagSkipPhaseB = 0x800, kDiagHalfWalk = 0x1000, kPrioA = 0x4000, kRingNt = 0x20000;

constexpr uint32_t kMaxGroup = 32;  // blocks per staged group
// Internal status: the block needs the general path (index block, a record
// shape the straight-line parsers do not take, a block larger than the
// stage).  The main kernel lists it; decode_deferred_kernel re-decodes it
// from HBM with the LEB cursor and writes the final status.
constexpr int32_t ST_DEFER = 0x7F;
constexpr uint32_t kStagePad = 256;  // readable LDS bytes past the span (fast parsers read <= 138)

// Record descriptor (one u64 per group item, LDS), written by phase A, read
// by phase B: image offsets of the record start, of where it must end (the
// next record's start, or the interval's end for its last record) and of its
// restart head's key; [48,53) group block, 53 restart head, 54 valid,
// [55,58) seqno bytes and [58,60) shared bytes of a header shape phase A has
// verified (0 = not verified: phase B decodes the header itself).
constexpr int kRecEndShift = 16, kRecKeyShift = 32, kRecBlockShift = 48, kRecN1Shift = 55, kRecN2Shift = 58;
constexpr uint64_t kRecRestart = 1ULL << 53, kRecValid = 1ULL << 54;

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

__device__ __forceinline__ void emit_global(const lsm_parsed_items& o, uint64_t i, const ItemFields& f) {
  if (o.seqno) gstore(o.seqno, i, f.seqno);
  if (o.key_off) gstore(o.key_off, i, f.key_off);
  if (o.val_off) gstore(o.val_off, i, f.val_off);
  if (o.val_len) gstore(o.val_len, i, f.val_len);
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
__device__ __forceinline__ void meta_trailer(const uint8_t* base, int32_t expect_type, uint32_t cap, BlockMeta& m) {
  if (m.st != ST_OK) return;
  const uint32_t plen = m.len - kHdrLen;
  if (m.item_count != plen) { m.st = ST_TRUNCATED; return; }   // data_length vs handle
  if (expect_type >= 0 && (int32_t)m.type != expect_type) { m.st = ST_TYPE_MISMATCH; return; }
  if (m.type == 2) { m.st = ST_UNSUPPORTED; return; }          // filter blocks are not KV blocks
  TrailerInfo t;
  int32_t st = read_trailer(base, m.hb + kHdrLen, plen, t);
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

__device__ __forceinline__ uint64_t rec_desc(uint32_t a, uint32_t end, uint32_t key, uint64_t tag) {
  return (uint64_t)a | ((uint64_t)end << kRecEndShift) | ((uint64_t)key << kRecKeyShift) | tag;
}

// Predicted header shape of a non-restart record: n1 seqno bytes, n2 shared
// bytes, 1 key-length byte.  msk = MSB bits of header bytes 1..hdr-1, pat =
// where their LEB terminators must be; a record matches iff (~h & msk) == pat.
struct Shape {
  uint32_t hdr, kshift;
  uint64_t msk, pat;
  uint64_t bits;  // descriptor shape bits
};
__device__ __forceinline__ Shape make_shape(uint32_t n1, uint32_t n2) {
  Shape s;
  s.bits = ((uint64_t)n1 << kRecN1Shift) | ((uint64_t)n2 << kRecN2Shift);
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
// Up to two groups walked by one wave: intervals [0, tot_a) belong to slot A,
// [tot_a, tot_a + tot_b) to slot B (the ring walker pairs groups so that all
// 64 lanes have an interval); each lane picks its slot's LDS arrays.
struct WalkSlots {
  const uint8_t* img[2];
  BlockMeta* meta[2];
  const uint8_t* owner[2];
  uint64_t* rec[2];
  uint32_t tot_a;
};

__device__ __forceinline__ void phase_a2(const WalkSlots& W, uint32_t c_first, uint32_t c_step, uint32_t total,
                                         uint32_t dummy, uint32_t diag_half = 0) {
  const int lane = threadIdx.x & (kWave - 1);
  for (uint32_t c0 = c_first; c0 < total; c0 += c_step) {
    const uint32_t cg = c0 + lane;
    const bool live = cg < total;
    const bool sel = cg >= W.tot_a;
    const uint32_t c = sel ? cg - W.tot_a : cg;
    const uint8_t* img = sel ? W.img[1] : W.img[0];
    BlockMeta* meta = sel ? W.meta[1] : W.meta[0];
    uint64_t* rec = sel ? W.rec[1] : W.rec[0];
    const uint32_t j = live ? (sel ? W.owner[1] : W.owner[0])[c] : 0;
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
    const uint64_t tag = ((uint64_t)j << kRecBlockShift) | kRecValid;
    const uint32_t stop = p0 + e_rel;
    uint32_t a = p0 + (ok ? s_rel : 0), key = a;
    uint32_t max_count = __builtin_amdgcn_readfirstlane(wave_max_u32(count));
    if (diag_half) max_count = (max_count + 1) / 2;  // diagnostic: price the walk's serial chain
    if (!max_count) continue;
    Shape sp;
    bool defer = false;  // a record shape the straight path does not take: whole block to the general path
    {  // restart head (full key: the value length is read separately)
      const Win16 w = read_win16(img, a);
      const RecHead hd = rec_head(w.lo, true);
      const uint32_t nxt = a + rec_len(hd.vt, hd.q, read_u16_unaligned(img, a + hd.q));
      key = a + hd.hdr;
      sp = make_shape(min(hd.e1 >> 3, 5u), 1);
      defer = count > 1 && !(hd.ok && valid_vtype(hd.vt));
      const bool act = count > 0 && !defer;
      if (count > 1 && act) ok = nxt < rec_end;
      const uint64_t rbits = (count > 1) ? ((uint64_t)(hd.e1 >> 3) << kRecN1Shift) : 0;  // verified only if walked
      rec[act ? ib0 : dummy] = rec_desc(a, count == 1 ? stop : nxt, key, tag | kRecRestart | rbits);
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
    uint32_t hi = (uint32_t)((((uint64_t)key << kRecKeyShift) | tag | sp.bits) >> 32);
    const uint32_t dmy = dummy;
    for (uint32_t jj = 1; jj < max_count; ++jj) {
      const uint64_t h = read_u64_unaligned(img, a);
      uint32_t z = read_u16_unaligned(img, a + qp);
      const uint32_t klen = (uint32_t)(h >> sp.kshift) & 0x7F;
      uint32_t q = sp.hdr + klen;
      uint32_t vt = (uint32_t)h & 0xFF;
      if (((~h & sp.msk) != sp.pat) | (q != qp)) {  // rare: header shape or key length changed
        const RecHead hd = rec_head(h, false);
        if (hd.ok) sp = make_shape(hd.e1 >> 3, (hd.e2 - hd.e1) >> 3);
        defer = defer || (jj < count && !hd.ok);  // seqno >= 2^49, shared >= 2^21 or key length >= 128
        q = hd.q;
        z = read_u16_unaligned(img, a + q);
        qp = q;
        hi = (uint32_t)((((uint64_t)key << kRecKeyShift) | tag | sp.bits) >> 32);
      }
      const uint32_t nxt = min(a + rec_len(vt, q, z), rec_end);
      const bool act = jj < count && !defer;
      const uint32_t end = jj + 1 == count ? stop : nxt;
      rec[act ? ib0 + jj : dmy] = ((uint64_t)hi << 32) | (uint64_t)(a | (end << kRecEndShift));
      a = act ? nxt : a;
    }
    if (defer) meta[j].st = ST_DEFER;                             // wins over PARSE
    else if (count && !ok) atomicCAS(&meta[j].st, ST_OK, ST_PARSE);  // walked off the record area
  }
}

// Phase A with two lanes per restart interval (adjacent lanes h = 0, 1): the
// dependent chain of the walk is the latency the group waits for, so lane
// h = 1 walks the second half of the interval from a PREDICTED start while
// h = 0 walks the first half.  h = 1 parses the head and record 1 like h = 0,
// then jumps to record ms at start(1) + (ms - 1) * len(1) (uniform records);
// the prediction holds iff h = 0 ends exactly there (lane-pair exchange).  If
// it does not, h = 0 walks the second half itself and overwrites h = 1's
// descriptors.  A verified split is a true parse, so phase B's checks are
// unchanged.  Work items: 2 per interval, item = c_first + lane + k c_step.
__device__ __forceinline__ void phase_a_split(const uint8_t* img, BlockMeta* meta, const uint8_t* owner,
                                              uint64_t* rec, uint32_t c_first, uint32_t c_step, uint32_t total,
                                              uint32_t dummy) {
  const int lane = threadIdx.x & (kWave - 1);
  for (uint32_t c0 = c_first; c0 < 2 * total; c0 += c_step) {
    const uint32_t item = c0 + lane;
    const uint32_t c = item >> 1;
    const bool h1 = (item & 1) != 0;
    const bool live = c < total;
    const uint32_t j = live ? owner[c] : 0;
    const BlockMeta& m = meta[j];
    const TrailerInfo t = trailer_of(m);
    const uint32_t p0 = m.p0, rec_end = m.rec_end;
    const uint32_t r = live ? c - m.chain0 : 0;
    const bool last_iv = r + 1 == t.bin_len;
    const uint32_t s_rel = bin_get(img, p0, t, r);
    const uint32_t e_rel = last_iv ? t.rec_end : bin_get(img, p0, t, r + 1);
    bool ok = s_rel < t.rec_end && e_rel <= t.rec_end && (r != 0 || s_rel == 0);
    const uint32_t count = (live && ok) ? (last_iv ? t.item_count - r * t.ri : t.ri) : 0;
    if (live && !ok && !h1) atomicCAS(&meta[j].st, ST_OK, ST_PARSE);
    const uint32_t ib0 = m.item0 + r * t.ri;
    const uint64_t tag = ((uint64_t)j << kRecBlockShift) | kRecValid;
    const uint32_t stop = p0 + e_rel;
    // split point: h0 takes records [0, ms), h1 records 1 and [ms, count)
    const uint32_t ms = count >= 4 ? (count + 3) >> 1 : count;
    const uint32_t steps = h1 ? (ms < count ? count - ms + 2 : 0) : ms;  // loop bound jj < steps
    uint32_t a = p0 + (ok ? s_rel : 0), key = a;
    const uint32_t max_steps = __builtin_amdgcn_readfirstlane(wave_max_u32(max(steps, min(count, 1u))));
    if (!max_steps) continue;
    Shape sp;
    bool defer = false;
    {  // restart head (both lanes parse it; h0 writes its descriptor)
      const Win16 w = read_win16(img, a);
      const RecHead hd = rec_head(w.lo, true);
      const uint32_t nxt = a + rec_len(hd.vt, hd.q, read_u16_unaligned(img, a + hd.q));
      key = a + hd.hdr;
      sp = make_shape(min(hd.e1 >> 3, 5u), 1);
      defer = count > 1 && !(hd.ok && valid_vtype(hd.vt));
      const bool act = count > 0 && !defer;
      if (count > 1 && act) ok = nxt < rec_end;
      const uint64_t rbits = (count > 1) ? ((uint64_t)(hd.e1 >> 3) << kRecN1Shift) : 0;
      rec[(act && !h1) ? ib0 : dummy] = rec_desc(a, count == 1 ? stop : nxt, key, tag | kRecRestart | rbits);
      a = (act && ok) ? nxt : a;
    }
    uint32_t qp = 0, pred = 0;
    uint32_t hi = (uint32_t)((((uint64_t)key << kRecKeyShift) | tag | sp.bits) >> 32);
    const uint32_t dmy = dummy;
    for (uint32_t jj = 1; jj < max_steps; ++jj) {
      const uint64_t h = read_u64_unaligned(img, a);
      uint32_t z = read_u16_unaligned(img, a + qp);
      const uint32_t klen = (uint32_t)(h >> sp.kshift) & 0x7F;
      uint32_t q = sp.hdr + klen;
      uint32_t vt = (uint32_t)h & 0xFF;
      if (((~h & sp.msk) != sp.pat) | (q != qp)) {  // rare: header shape or key length changed
        const RecHead hd = rec_head(h, false);
        if (hd.ok) sp = make_shape(hd.e1 >> 3, (hd.e2 - hd.e1) >> 3);
        const uint32_t idx_d = (h1 && jj > 1) ? jj + ms - 2 : jj;
        defer = defer || (jj < steps && idx_d < count && !hd.ok);
        q = hd.q;
        z = read_u16_unaligned(img, a + q);
        qp = q;
        hi = (uint32_t)((((uint64_t)key << kRecKeyShift) | tag | sp.bits) >> 32);
      }
      const uint32_t nxt = min(a + rec_len(vt, q, z), rec_end);
      const uint32_t idx = (h1 && jj > 1) ? jj + ms - 2 : jj;
      const bool act = jj < steps && idx < count && !defer;
      const uint32_t end = idx + 1 == count ? stop : nxt;
      rec[act ? ib0 + idx : dmy] = ((uint64_t)hi << 32) | (uint64_t)(a | (end << kRecEndShift));
      uint32_t an = act ? nxt : a;
      if (h1 && jj == 1 && act) {  // jump to record ms assuming records 1 .. ms-1 all have record 1's length
        an = min(nxt + (ms - 2) * (nxt - a), rec_end);
        pred = an;
      }
      a = an;
    }
    // h0 now sits at the start of record ms (if it walked that far)
    const uint32_t a0 = (uint32_t)__shfl_xor((int)a, 1);
    const bool split = ms < count;
    const bool hit = !split || pred == a0;  // (read on h1 lanes)
    const bool redo = (uint32_t)__shfl_xor((int)(hit ? 1 : 0), 1) == 0;  // on h0 lanes: h1 mispredicted
    const bool my_redo = !h1 && split && redo && !defer;
    // fallback: h0 walks records [ms, count) itself
    const uint32_t need = my_redo ? count - ms : 0;
    const uint32_t max_redo = __builtin_amdgcn_readfirstlane(wave_max_u32(need));
    for (uint32_t k = 0; k < max_redo; ++k) {
      const uint64_t h = read_u64_unaligned(img, a);
      const RecHead hd = rec_head(h, false);
      const uint32_t z = read_u16_unaligned(img, a + hd.q);
      if (hd.ok) sp = make_shape(hd.e1 >> 3, (hd.e2 - hd.e1) >> 3);
      const bool act = k < need && !defer;
      defer = defer || (k < need && !hd.ok);
      const uint32_t idx = ms + k;
      const uint32_t nxt = min(a + rec_len(hd.vt, hd.q, z), rec_end);
      const uint32_t end = idx + 1 == count ? stop : nxt;
      const uint32_t hb = (uint32_t)((((uint64_t)key << kRecKeyShift) | tag | sp.bits) >> 32);
      rec[(act && !defer) ? ib0 + idx : dmy] = ((uint64_t)hb << 32) | (uint64_t)(a | (end << kRecEndShift));
      a = act ? nxt : a;
    }
    const bool keep = !h1 || (split && hit);  // a mispredicted h1 lane's flags are void
    if (keep && defer) meta[j].st = ST_DEFER;                             // wins over PARSE
    else if (keep && count && !ok) atomicCAS(&meta[j].st, ST_OK, ST_PARSE);
  }
}

__device__ __forceinline__ void phase_a(const uint8_t* img, BlockMeta* meta, const uint8_t* owner, uint64_t* rec,
                                        uint32_t c_first, uint32_t c_step, uint32_t total, uint32_t dummy,
                                        uint32_t diag_half = 0) {
  WalkSlots W;
  W.img[0] = W.img[1] = img;
  W.meta[0] = W.meta[1] = meta;
  W.owner[0] = W.owner[1] = owner;
  W.rec[0] = W.rec[1] = rec;
  W.tot_a = total;
  phase_a2(W, c_first, c_step, total, dummy, diag_half);
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

__device__ __forceinline__ void store_fields(const DecodeParams& P, bool all_fields, uint64_t gi,
                                             const ItemFields& f) {
  if (all_fields) {  // every output array present: no per-field null checks
    gstore(P.out.seqno, gi, f.seqno);
    gstore(P.out.key_off, gi, f.key_off);
    gstore(P.out.val_off, gi, f.val_off);
    gstore(P.out.val_len, gi, f.val_len);
    gstore(P.out.key_len, gi, f.key_len);
    gstore(P.out.prefix_len, gi, f.prefix_len);
    gstore(P.out.vtype, gi, f.vtype);
    if (P.out.handle_off) gstore(P.out.handle_off, gi, f.handle_off);
  } else {
    emit_global(P.out, gi, f);
  }
}

// Phase B: thread = record.  Full parse + validation of every descriptor
// (the oracle's parse_data_item checks, and the record must end exactly at
// the descriptor's end), then coalesced stores of all fields.
template <bool kAllFields>
__device__ __forceinline__ void phase_b(const DecodeParams& P, const uint8_t* img, BlockMeta* meta,
                                        const uint64_t* rec, uint32_t n_items, uint32_t g_item0, uint32_t tid,
                                        uint32_t nthr) {
  constexpr bool all_fields = kAllFields;
  const bool store = !(P.flags & kDiagSkipStore);
  for (uint32_t i0 = 0; i0 < n_items; i0 += nthr) {
    const uint32_t i = i0 + tid;
    if (i >= n_items) break;
    const uint64_t d = rec[i];
    if (!(d & kRecValid)) continue;  // not reached: its block has failed
    const uint32_t j = (uint32_t)(d >> kRecBlockShift) & 31;
    const u32x4 hot = *reinterpret_cast<const u32x4*>(&meta[j]);  // p0, rec_end, st, type
    const uint32_t p0 = hot.x, end = hot.y - p0;
    if ((int32_t)hot.z != ST_OK) continue;  // block already failed: outputs unspecified
    const uint32_t a = ((uint32_t)d & 0xFFFF) - p0;
    const uint32_t want = ((uint32_t)(d >> kRecEndShift) & 0xFFFF) - p0;
    const uint32_t base_key = ((uint32_t)(d >> kRecKeyShift) & 0xFFFF) - p0;
    const bool restart = (d & kRecRestart) != 0;
    const uint64_t gi = (uint64_t)g_item0 + i;
    ItemFields f;
    uint32_t next;
    const uint32_t n1 = (uint32_t)(d >> kRecN1Shift) & 7, n2 = (uint32_t)(d >> kRecN2Shift) & 3;
    const int rc = n1 ? parse_data_shape(img, p0, a, end, restart, base_key, n1, n2, f, next)
                      : parse_data_fast(img, p0, a, end, restart, base_key, f, next);
    if (rc > 0 && store) store_fields(P, all_fields, gi, f);
    if (rc == 0) meta[j].st = ST_DEFER;  // wins over PARSE
    else if (rc < 0 || next != want) atomicCAS(&meta[j].st, ST_OK, ST_PARSE);
  }
}

// Interval walk straight from a span (direct path); emit(j, fields).
template <class Emit>
__device__ __forceinline__ bool walk_interval(const uint8_t* base, uint32_t p0, const BlockMeta& m, uint32_t r,
                                              Emit emit) {
  const TrailerInfo t = trailer_of(m);
  const bool last = r + 1 == t.bin_len;
  const uint32_t start = bin_get(base, p0, t, r);
  const uint32_t stop = last ? t.rec_end : bin_get(base, p0, t, r + 1);
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
  if (meta[0].st == ST_OK) {
    uint64_t lo, hi;
    xxh3_128_wave(base, hb + kHdrLen, meta[0].len - kHdrLen, &kLongSecret, lo, hi);
    if (lane == 0 && (lo != meta[0].ck_lo || hi != meta[0].ck_hi)) meta[0].st = ST_CKSUM;
  }
  wave_sync();
  if (lane == 0) meta_trailer(base, P.expect_type, cap, meta[0]);
  wave_sync();
  const BlockMeta m = meta[0];
  if (m.st == ST_OK) {
    bool ok = true;
    for (uint32_t r = lane; r < m.bin_len; r += kWave) {
      ok &= walk_interval(base, hb + kHdrLen, m, r,
                          [&](uint32_t j, const ItemFields& f) { emit_global(P.out, item_base + j, f); });
    }
    if (!ok) atomicCAS(&meta[0].st, ST_OK, ST_PARSE);
  }
  wave_sync();
  if (lane == 0) gstore(P.status, b, meta[0].st);
  wave_sync();
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

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
                                            uint32_t gmax, uint64_t offr, uint32_t itr) {
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
  const bool lone = ((G.end_j + 15) & ~15ULL) - (G.off_j & ~15ULL) > P.stage_bytes ||
                    G.it1_j - G.it0_j > P.tile_items;
  const bool fits = in_run && !lone && G.end_j >= G.off_j && G.off_j >= off_b &&
                    ((G.end_j + 15) & ~15ULL) - G.span0 <= P.stage_bytes && G.it1_j - G.g_item0 <= P.tile_items;
  G.k = (uint32_t)__builtin_ctzll(~__ballot(fits));  // lanes >= gmax never fit
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

// General path for the deferred blocks: one wave per block, straight from
// HBM, Cursor fallback for every record shape (decode_block_direct).
__global__ __launch_bounds__(kWave) void decode_deferred_kernel(DecodeParams P) {
  __shared__ BlockMeta meta[1];
  const uint32_t n = gload(P.defer_count, 0);
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) decode_block_direct(P, gload(P.defer_list, i), meta);
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
    if (span1 - span0 > kBigStage) {  // HBM path
      if (wave == 0) decode_block_direct(P, b, meta);
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
      meta_trailer(stage, P.expect_type, cap, meta[1]);
      *cks_bad = 0;
    }
    lds_barrier();
    // payload checksum: per-KiB contributions on all waves, then the chain on wave 0
    const bool hdr_ok = meta[0].st == ST_OK;
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
                              [&](uint32_t j, const ItemFields& f) { emit_global(P.out, item_base + j, f); });
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

// Workgroup = kGroupWaves waves sharing one LDS stage of up to 64 KiB (16
// 4-KiB blocks, ~64 restart intervals).  Per group:
//   all waves   LDS-DMA of the span (wave w moves 1-KiB pieces w, w+4, ...)
//   wave 0      headers + trailers (lane j = block j), interval numbering
//   wave pa     phase A over all intervals (every lane walks one interval)
//   other waves payload checksums (12 DPP rows, block j on row j mod 12)
//   all waves   phase B (thread = record), coalesced SoA stores
// pa rotates with the group index so the serial walk lands on each SIMD in
// turn.  Phase A needs only the trailer, not the checksum, so it runs
// concurrently with the hash; statuses merge in oracle order at the end.
#ifndef LSM_DEC_WAVES
#define LSM_DEC_WAVES 4
#endif
#ifndef LSM_DEC_WPE
#define LSM_DEC_WPE 3
#endif
constexpr uint32_t kGroupWaves = LSM_DEC_WAVES;

// Diagnostic phase timers (flag kDiagTimers): per workgroup clock64() deltas,
// summed over the grid; read back with lsm_diag_decode_timers (abi.hip).
constexpr uint32_t kDiagTimers = 0x2000;
enum : int { kTmForm, kTmDma, kTmHdr, kTmA, kTmHash, kTmSplit, kTmB, kTmTail, kTmGroups, kTmN };
__device__ unsigned long long g_decode_timers[kTmN];

template <bool kTimed, bool kAllFields>
__global__ __launch_bounds__(kGroupWaves * kWave) __attribute__((amdgpu_waves_per_eu(LSM_DEC_WPE))) void decode_blocks_kernel(DecodeParams P) {
  // LDS: [meta: G x 80 B][rec: u64 per item + 1 scratch][owner: u8 per item][staged bytes + pad]
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
  const bool dbl = (P.flags & kDecodeDouble) != 0;
  const uint32_t slot_stride = ((P.stage_bytes + 15) & ~15u) + kStagePad;
  LongSecret* ls = reinterpret_cast<LongSecret*>(img + (dbl ? 2 : 1) * slot_stride);
  if (tid < sizeof(LongSecret) / 8)
    reinterpret_cast<uint64_t*>(ls)[tid] = reinterpret_cast<const uint64_t*>(&kLongSecret)[tid];
  uint32_t iter = 0;
  constexpr bool timed = kTimed;
  uint64_t tm[kTmN] = {};
  uint64_t t0 = 0;
  if constexpr (timed) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
#define LSM_TICK(slot)                                                                     \
  if constexpr (timed) {                                                                   \
    uint64_t t1;                                                                           \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");             \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    tm[slot] += t1 - t0;                                                                   \
    t0 = t1;                                                                               \
  }
  // Next stageable group at or after bb (larger blocks go to the general path).
  auto next_group = [&](uint32_t bb) -> Group {
    for (;;) {
      if (bb >= b_end) {
        Group z;
        z.b = bb;
        z.k = 0;
        return z;
      }
      const Group g = form_group(P, bb, b_begin, b_end, gmax, offr, itr);
      if (g.k) return g;
      bb += 1;  // a lone block: listed for the general path before the loop
    }
  };
  // LDS-DMA of a group's span into a stage slot (wave w moves 1-KiB pieces
  // w, w + 8, ...).  Inline asm (lds_dma.hpp): invisible to the compiler's
  // waitcnt pass, so a prefetch stays in flight across the current group's
  // LDS work; the loop head waits for it with vmcnt(0).
  auto issue_dma = [&](const Group& g, uint8_t* dst) {
    const uint32_t chunks = (uint32_t)((g.span1 - g.span0) >> 4);
    const uint8_t* src = P.blocks + g.span0 + 16 * lane;
    const uint32_t d0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst);
    if (dbl) {
      for (uint32_t i = wave; i * kWave < chunks; i += kGroupWaves) {
        if (i * kWave + lane < chunks) dma16<false>(src + 1024 * i, d0 + 1024 * i);
      }
    } else {  // nothing to overlap: the compiler-visible builtin
      for (uint32_t i = wave; i * kWave < chunks; i += kGroupWaves) {
        if (i * kWave + lane < chunks)
          __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + 1024 * i), (lds_void_t*)(dst + 1024 * i), 16, 0, 0);
      }
    }
  };
  // Lone blocks (larger than the stage, or more items than a tile) go to the
  // general path, decode_deferred_staged_kernel (a 72 KiB stage, the block
  // hashed by four waves): listed here, one atomic per workgroup.
  if (wave == 0) {
    const uint64_t nx = wave_shfl_u64(offr, min(lane + 1, kWave - 1));
    const uint32_t ix = (uint32_t)__shfl((int)itr, min(lane + 1, kWave - 1));
    const bool in = b_begin + lane < b_end;
    const bool lone = in && (((nx + 15) & ~15ULL) - (offr & ~15ULL) > P.stage_bytes || ix - itr > P.tile_items);
    defer_blocks_wave(P, lone, b_begin + lane);
  }
  Group G = next_group(b_begin);
  uint32_t cur = 0;
  if (G.k) issue_dma(G, img);
  for (; G.k; ++iter) {
    const uint32_t b = G.b;
    const uint32_t k = G.k;
    uint8_t* const stage = img + cur * slot_stride;
    // ---- 1. this group's span has landed (issued one group ahead when
    //         double-buffered); clear the record descriptors; prefetch the next
    for (uint32_t i = tid; i < G.n_items; i += kGroupWaves * kWave) rec[i] = 0;
    vm_wait<0>();
    lds_barrier();
    LSM_TICK(kTmDma);
    const Group Gn = next_group(b + k);
    if (dbl && Gn.k) issue_dma(Gn, img + (cur ^ 1) * slot_stride);
    LSM_TICK(kTmForm);
    // ---- 2. wave 0: headers, trailers, restart-interval numbering; owner[c] = block of interval c
    if (wave == 0) {
      uint32_t chains = 0;
      BlockMeta m;
      if ((uint32_t)lane < k) {
        meta_header_fields(stage, (uint32_t)(G.off_j - G.span0), G.end_j - G.off_j, m);
        m.item0 = G.it0_j - G.g_item0;
        m.hdr_st = m.st;
        m.ck_bad = 0;
        m.hck_bad = 0;
        meta_trailer(stage, P.expect_type, G.it1_j - G.it0_j, m);
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
    LSM_TICK(kTmHdr);
    // ---- 3. phase A on nA waves (64 intervals each)  ||  payload checksums on the others
    {
      const uint32_t total = (P.flags & kDiagSkipParse) ? 0
                             : meta[k - 1].chain0 + (meta[k - 1].st == ST_OK ? meta[k - 1].bin_len : 0);
      const bool split = (P.flags & kDecodeSplitWalk) != 0;
      const uint32_t nA = min(((split ? 2 : 1) * total + kWave - 1) / kWave, kGroupWaves - 1);
      const uint32_t role = (wave + kGroupWaves - iter % kGroupWaves) % kGroupWaves;  // rotates per group
      if (role < nA) {
        // the serial walk is the group's critical path: let it win issue
        // arbitration against the other workgroup's waves on this SIMD
        if (P.flags & kPrioA) __builtin_amdgcn_s_setprio(3);
        if (split) phase_a_split(stage, meta, owner, rec, role * kWave, nA * kWave, total, P.tile_items);
        else phase_a(stage, meta, owner, rec, role * kWave, nA * kWave, total, P.tile_items, P.flags & kDiagHalfWalk);
        if (P.flags & kPrioA) __builtin_amdgcn_s_setprio(0);
        LSM_TICK(kTmA);
      } else if (!(P.flags & kDiagSkipHash) && k <= kGroupWaves - nA) {
        // few (large) blocks: one wave per block, the 64-lane XXH3 (1 KiB per step)
        const uint32_t jb = role - nA;
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
        LSM_TICK(kTmHash);
      } else if (!(P.flags & kDiagSkipHash)) {
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
        LSM_TICK(kTmHash);
      }
    }
    lds_barrier();
    LSM_TICK(kTmSplit);
    // ---- 4. phase B: thread = record; full parse + validation; coalesced stores
    if (!(P.flags & (kDiagSkipParse | kDiagSkipPhaseB))) phase_b<kAllFields>(P, stage, meta, rec, G.n_items, G.g_item0, threadIdx.x, blockDim.x);
    LSM_TICK(kTmB);
    lds_barrier();
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
    if (!dbl && Gn.k) issue_dma(Gn, img);  // single stage: refill after phase B
    G = Gn;
    if (dbl) cur ^= 1;
    if constexpr (timed) tm[kTmGroups] += 1;
    LSM_TICK(kTmTail);
  }
#undef LSM_TICK
  if (timed && lane == 0) {
    // each wave adds its own view; phase A / hash slots only from the waves that ran them
    for (int i = 0; i < kTmN; ++i) atomicAdd(&g_decode_timers[i], (unsigned long long)tm[i]);
  }
}

// ============================================================ ring kernel
// decode_ring_kernel: one persistent 16-wave workgroup per CU streams its
// share of the batch through an LDS ring of `ring_slots` slots; each slot
// holds one GROUP (the longest run of consecutive blocks that fits the slot).
// Roles (fixed per wave, synchronised through per-slot sequence words in LDS,
// never s_barrier, so every role runs at its own pace):
//   wave 0            loader: forms groups from the handles (scalar loads),
//                     issues the group's LDS-DMA and publishes FULL once its
//                     own counted vmcnt says the bytes have landed;
//   walker waves      headers + trailers (lane = block), interval numbering,
//                     phase A (lane = restart interval) -> record descriptors;
//   hasher waves      payload xxh3_128 (16-lane DPP rows) + header checksum;
//   parser waves      phase B (lane = record) -> SoA stores, block statuses,
//                     then FREE (the slot returns to the loader).
// Group g lives in slot g % S and is taken by walker g % nx, hasher g % nh and
// parser g % nb, so up to S groups are in flight at different stages and the
// DMA of later groups overlaps the compute of earlier ones.  The loader is the
// only wave with vector-memory loads (its DMA is inline asm, invisible to the
// compiler's waitcnt pass, which would otherwise drain it before every LDS
// access); parsers are the only waves with global stores.
constexpr uint32_t kRingMaxSlots = 8, kRingGroup = 16;

// Diagnostic ring timers (tuning flag kDiagTimers): s_memtime cycles per role
// phase summed over the grid, read back with lsm_diag_decode_timers.
enum : int { kRtLIssue, kRtLWait, kRtLIdle, kRtLand, kRtGroups, kRtXBusy, kRtXIdle, kRtHBusy, kRtHIdle, kRtBBusy,
             kRtBIdle, kRtN };
__device__ unsigned long long g_ring_timers[kRtN];
struct RingClock {
  bool on;
  uint64_t t, acc[kRtN];
  __device__ __forceinline__ explicit RingClock(bool en) : on(en), t(en ? __builtin_amdgcn_s_memtime() : 0) {
    for (int i = 0; i < kRtN; ++i) acc[i] = 0;
  }
  __device__ __forceinline__ void tick(int slot) {
    if (on) {
      const uint64_t n = __builtin_amdgcn_s_memtime();
      acc[slot] += n - t;
      t = n;
    }
  }
  __device__ __forceinline__ void flush() {
    if (on && (threadIdx.x & 63) == 0)
      for (int i = 0; i < kRtN; ++i)
        if (acc[i]) atomicAdd(&g_ring_timers[i], (unsigned long long)acc[i]);
  }
};

struct RingCtl {
  uint32_t full[kRingMaxSlots];   // g + 1 once group g's bytes are in slot g % S
  uint32_t xdone[kRingMaxSlots];  // g + 1 once its descriptors + block meta are written
  uint32_t bdone[kRingMaxSlots];  // g + 1 once parsed, stored and released
  uint32_t hcnt[kRingMaxSlots];   // hashers done with the group (team counter)
  uint32_t bcnt[kRingMaxSlots];   // parsers done with the group (team counter)
  uint32_t issue[kRingMaxSlots];  // g + 1 once the leader has formed group g (followers may issue)
  uint32_t lcnt[kRingMaxSlots];   // loaders whose share of group g has landed (team counter)
  uint32_t total;                 // groups of this workgroup (~0 until the leader has formed them all)
  uint32_t psync;                 // parser team barrier (monotonic arrivals)
  uint32_t ppend;                 // parser team: re-anchored intervals (monotonic)
  uint32_t pfail;                 // parser team: unverified records (monotonic)
  uint32_t fin[kRingMaxSlots];    // parts done with group g (parser team, hasher): the 2nd finishes it
};
struct SlotDesc {
  uint32_t b, k, g_item0, n_items, defer, bytes;  // bytes: the group's span (LDS-DMA length)
  uint32_t span0_lo, span0_hi;                    // span start in d_blocks (16-aligned)
  uint32_t n_iv, pad[3];                          // restart intervals (planner)
};
struct SlotBlk {
  uint32_t hb, len, item0, cap;  // header offset in the slot image, handle size, first item, item capacity
};
// One restart interval of a group (planner writes it, parsers advance it).
// Positions are payload-relative.  Records [first, anchor) are placed for
// certain; record k >= anchor is guessed at apos + (k - anchor) * stride.
// stride == 0: the interval is finished (or its block failed).
// Guess for record k (k > first): k < cut ? apos + (k - anchor) * stride
//                                          : apos2 + (k - cut) * stride2.
struct alignas(16) Iv {
  uint16_t s, e;         // head position, where the interval must end
  uint16_t first, last;  // group item indices of the head and the last record
  uint16_t p0, end;      // payload start in the slot image; record-area end (payload-relative)
  uint16_t key;          // the head's key (prefix of the truncated records)
  uint16_t live;         // 0: settled (or its block failed)
  uint16_t anchor, apos, stride, cut, apos2, stride2;
  uint16_t pad[2];
};
static_assert(sizeof(Iv) == 32, "Iv");
constexpr uint32_t kMaxIv = 96;  // intervals per group on the speculative path (more: general path)

__device__ __forceinline__ uint32_t iv_pos(const Iv& iv, uint32_t k) {
  return k == iv.first ? (uint32_t)iv.s
         : k < iv.cut  ? (uint32_t)iv.apos + (k - iv.anchor) * iv.stride
                       : (uint32_t)iv.apos2 + (k - iv.cut) * iv.stride2;
}
constexpr uint32_t kSlotBlkOff = sizeof(SlotDesc);
constexpr uint32_t kSlotMetaOff = kSlotBlkOff + kRingGroup * sizeof(SlotBlk);
constexpr uint32_t kSlotHresOff = kSlotMetaOff + kRingGroup * sizeof(BlockMeta);
constexpr uint32_t kSlotIvOff = kSlotHresOff + kRingGroup * 4;
constexpr uint32_t kSlotFailOff = kSlotIvOff + kMaxIv * sizeof(Iv);
constexpr uint32_t kSlotIvbOff = kSlotFailOff + kMaxIv * 4;
constexpr uint32_t kSlotOwnOff = kSlotIvbOff + kMaxIv;
constexpr uint32_t kSlotRecIvOff = kSlotOwnOff + kMaxIv;
static_assert(sizeof(RingCtl) <= 320, "RingCtl");
static_assert(kSlotMetaOff % 16 == 0 && kSlotIvOff % 16 == 0 && kSlotRecIvOff % 16 == 0, "slot layout");

struct RingLayout {
  uint32_t slot_meta;  // bytes of one slot's metadata block
  uint32_t meta_base, handles, secret, img, total;
};
// The loader streams the handles (block_off, item_start) of its blocks into two
// LDS chunk buffers, kHandleStep blocks apart, each holding kHandleEnt entries
// (a group formed anywhere in a chunk's first kHandleStep blocks sees its 17).
constexpr uint32_t kHandleStep = 112, kHandleEnt = kHandleStep + kRingGroup + 1;
constexpr uint32_t kHandleOffBytes = (8 * kHandleEnt + 15) & ~15u, kHandleItBytes = (4 * kHandleEnt + 15) & ~15u;
constexpr uint32_t kHandleBuf = kHandleOffBytes + kHandleItBytes;
__host__ __device__ __forceinline__ RingLayout ring_layout(uint32_t slots, uint32_t slot_bytes, uint32_t tile) {
  RingLayout L;
  L.slot_meta = kSlotRecIvOff + ((tile + 15) & ~15u);
  L.meta_base = 320;
  L.handles = L.meta_base + slots * L.slot_meta;
  L.secret = L.handles + 2 * kHandleBuf;
  L.img = (L.secret + (uint32_t)sizeof(LongSecret) + 15) & ~15u;
  L.total = L.img + slots * ((slot_bytes + 15) & ~15u) + kStagePad;
  return L;
}

__device__ __forceinline__ uint32_t lds_get(const uint32_t* p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
// Release (this wave's LDS writes first) and store a sequence word.
__device__ __forceinline__ void lds_publish(uint32_t* p, uint32_t v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Relaxed poll with s_sleep, one acquire.  false: the ring ended before group g.
__device__ __forceinline__ bool ring_wait(const uint32_t* p, uint32_t v, const RingCtl* ctl, uint32_t g) {
  uint32_t n = 0;
  while (lds_get(p) != v) {  // back off: polls cost issue slots of the busy waves on this SIMD
    if ((++n & 7) == 0 && lds_get(&ctl->total) <= g) return false;
    if (n < 4) __builtin_amdgcn_s_sleep(1);
    else __builtin_amdgcn_s_sleep(3);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  return true;
}

struct RingSlot {
  SlotDesc* desc;
  SlotBlk* blk;
  BlockMeta* meta;
  uint32_t* hres;
  Iv* iv;
  uint32_t* fail;   // per interval: first failing record of the round (atomicMin), ~0 = none
  uint8_t* ivb;     // per interval: its block
  uint8_t* owner;   // planner scratch: interval -> block
  uint8_t* rec_iv;  // per record: its interval (0xFF: not on the speculative path)
  uint8_t* img;
};
__device__ __forceinline__ RingSlot ring_slot(uint8_t* smem, const RingLayout& L, uint32_t s, uint32_t slot_bytes,
                                              uint32_t tile) {
  RingSlot r;
  uint8_t* m = smem + L.meta_base + s * L.slot_meta;
  r.desc = reinterpret_cast<SlotDesc*>(m);
  r.blk = reinterpret_cast<SlotBlk*>(m + kSlotBlkOff);
  r.meta = reinterpret_cast<BlockMeta*>(m + kSlotMetaOff);
  r.hres = reinterpret_cast<uint32_t*>(m + kSlotHresOff);
  r.iv = reinterpret_cast<Iv*>(m + kSlotIvOff);
  r.fail = reinterpret_cast<uint32_t*>(m + kSlotFailOff);
  r.ivb = m + kSlotIvbOff;
  r.owner = m + kSlotOwnOff;
  r.rec_iv = m + kSlotRecIvOff;
  r.img = smem + L.img + s * ((slot_bytes + 15) & ~15u);
  return r;
}

// Team arrival: the last of n waves to finish group g on slot s gets true
// (and resets the counter for group g + S).  Every wave releases its own LDS
// writes first; the last one acquires everybody's.
__device__ __forceinline__ bool team_arrive(uint32_t* cnt, uint32_t n) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  uint32_t old = 0;
  if ((threadIdx.x & (kWave - 1)) == 0)
    old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  old = __builtin_amdgcn_readfirstlane(old);
  if (old + 1 != n) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  if ((threadIdx.x & (kWave - 1)) == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return true;
}

// ---- loader waves [0, NL): LDS-DMA of every group, split piece-wise over NL
// waves (one wave's LDS-DMA issue caps near 1.4 TB/s chip-wide; scripts/dma_probe.py).
// Wave 0 leads: it streams the handles, forms group g in slot g % S once the
// slot is free and publishes ISSUE; every loader then issues pieces l, l + NL,
// ... of the group's span.  A loader waits for its own pieces (counted vmcnt)
// only when it cannot issue more; the last loader whose share has landed
// publishes FULL.
// Budget: a wave stalls at issue once 63 vector-memory ops are outstanding,
// which would also hold back its arrivals; a share is issued only if the ops
// not yet known to have landed still fit.
__device__ __forceinline__ uint32_t share_pieces(uint32_t bytes, uint32_t l, uint32_t nl) {
  const uint32_t pieces = (bytes + 1023) >> 10;
  return pieces > l ? (pieces - l + nl - 1) / nl : 0u;
}

template <bool kNt>
__device__ __forceinline__ uint32_t issue_share(const DecodeParams& P, uint32_t l, uint32_t nl, uint64_t span0,
                                                uint32_t bytes, uint32_t img) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t n = share_pieces(bytes, l, nl);
  if (!n) return 0;
  const uint32_t voff = 16 * (uint32_t)lane;
  uint64_t gb = (uint64_t)(uintptr_t)(P.blocks + span0 + 1024 * l);
  gb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)gb) |  // (readfirstlane is int:
       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(gb >> 32)) << 32);  //  no sign extension)
  uint32_t dst = __builtin_amdgcn_readfirstlane(img + 1024 * l);
  const uint32_t step = 1024 * nl;
  const uint32_t last = n - 1, last_bytes = bytes - 1024 * (l + nl * last);  // 1..1024
  for (uint32_t i = 0; i < last; ++i) {
    dma16s<kNt>(voff, gb, dst);
    gb += step;
    dst += step;
  }
  if (voff < last_bytes) dma16s<kNt>(voff, gb, dst);  // possibly partial last piece (stays inside the input)
  return n;
}

template <bool kNt>
__device__ __forceinline__ void ring_loader(KArgs Pk, uint8_t* smem, const RingLayout& L, uint32_t l, uint32_t nl) {
  const DecodeParams P = load_params(Pk);
  RingCtl* ctl = reinterpret_cast<RingCtl*>(smem);
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t S = P.ring_slots, SB = P.stage_bytes, tile = P.tile_items;
  const uint32_t G = gridDim.x, w = blockIdx.x;
  const uint32_t b_begin = (uint32_t)((uint64_t)P.n_blocks * w / G);
  const uint32_t b_end = (uint32_t)((uint64_t)P.n_blocks * (w + 1) / G);
  const bool leader = l == 0;
  uint32_t ops = 0;  // LDS-DMA instructions this wave has issued (its vmcnt stream)
  // handle chunk c (leader only): entries [b_begin + c * kHandleStep, + kHandleEnt) in buffer c & 1
  auto issue_chunk = [&](uint32_t c) {
    const uint32_t cb = b_begin + c * kHandleStep;
    if (cb > b_end) return;
    const uint32_t nent = min(kHandleEnt, P.n_blocks + 1 - cb);
    const uint32_t buf = (uint32_t)(uintptr_t)(smem + L.handles + (c & 1) * kHandleBuf);
    const uint8_t* so = reinterpret_cast<const uint8_t*>(P.block_off + cb);
    const uint8_t* si = reinterpret_cast<const uint8_t*>(P.item_start + cb);
    const uint32_t po = (2 * nent + 63) / 64, pi = (nent + 63) / 64;
    for (uint32_t i = 0; i < po; ++i)
      if (64 * i + (uint32_t)lane < 2 * nent) dma4(so + 256 * i + 4 * lane, __builtin_amdgcn_readfirstlane(buf + 256 * i));
    for (uint32_t i = 0; i < pi; ++i)
      if (64 * i + (uint32_t)lane < nent)
        dma4(si + 256 * i + 4 * lane, __builtin_amdgcn_readfirstlane(buf + kHandleOffBytes + 256 * i));
    ops += po + pi;
  };
  uint32_t mark_next = 0, cur = 0;
  if (leader) {
    issue_chunk(0);
    const uint32_t mark0 = ops;
    issue_chunk(1);
    mark_next = ops;  // ops after chunk cur + 1
    vm_wait_n(ops - mark0);
  }
  const uint32_t max_share = share_pieces(SB, 0, nl);
  const uint32_t budget = 63 - 8;
  uint32_t landed = ops;     // ops known to have landed (through this wave's last arrival)
  uint32_t mark[kRingMaxSlots];  // ops after this wave's share of the group in slot s
  uint32_t b = b_begin, g = 0, arr = 0;
  uint32_t total = ~0u;      // leader: groups formed once known
  RingClock clk((P.flags & kDiagTimers) != 0);
  for (;;) {
    const uint32_t s = g % S;
    const bool room = g - arr < S && (ops == landed || ops + max_share - landed <= budget);
    bool go = false;
    if (leader) go = room && b < b_end && (g < S || lds_get(&ctl->bdone[s]) == g - S + 1);
    else go = room && g < lds_get(&ctl->total) && lds_get(&ctl->issue[s]) == g + 1;
    if (go) {
      clk.tick(kRtLIdle);
      const RingSlot R = ring_slot(smem, L, s, SB, tile);
      uint64_t span0;
      uint32_t bytes;
      if (leader) {
        const uint32_t c = (b - b_begin) / kHandleStep;
        if (c != cur) {  // c == cur + 1: its chunk was issued one chunk ago
          vm_wait_n(ops - mark_next);
          issue_chunk(c + 1);
          mark_next = ops;
          cur = c;
        }
        const uint8_t* hb = smem + L.handles + (c & 1) * kHandleBuf;
        const uint32_t rel = b - (b_begin + c * kHandleStep);
        // lane j: block b + j (j <= 16)
        const uint32_t jl = min((uint32_t)lane, kRingGroup);
        const uint64_t off_j = reinterpret_cast<const uint64_t*>(hb)[rel + jl];
        const uint64_t end_j = reinterpret_cast<const uint64_t*>(hb)[rel + jl + (jl < kRingGroup ? 1 : 0)];
        const uint32_t it0_j = reinterpret_cast<const uint32_t*>(hb + kHandleOffBytes)[rel + jl];
        const uint32_t it1_j = reinterpret_cast<const uint32_t*>(hb + kHandleOffBytes)[rel + jl + (jl < kRingGroup ? 1 : 0)];
        const uint64_t off_b = wave_readlane_u64(off_j, 0);
        const uint32_t g_item0 = wave_readlane_u32(it0_j, 0);
        span0 = off_b & ~15ULL;
        const bool fits = (uint32_t)lane < kRingGroup && b + lane < b_end && end_j >= off_j && off_j >= off_b &&
                          ((end_j + 15) & ~15ULL) - span0 <= SB && it1_j - g_item0 <= tile && it1_j >= it0_j;
        const uint32_t k = (uint32_t)__builtin_ctzll(~__ballot(fits));
        const uint64_t span1 = k ? (wave_readlane_u64(end_j, k - 1) + 15) & ~15ULL : span0;
        const uint32_t n_items = k ? wave_readlane_u32(it1_j, k - 1) - g_item0 : 0;
        bytes = (uint32_t)(span1 - span0);
        if ((uint32_t)lane < k) {
          SlotBlk e;
          e.hb = (uint32_t)(off_j - span0);
          e.len = (uint32_t)(end_j - off_j);
          e.item0 = it0_j - g_item0;
          e.cap = it1_j - it0_j;
          R.blk[lane] = e;
        }
        if (lane == 0) {
          SlotDesc d;
          d.b = b;
          d.k = k ? k : 1;
          d.g_item0 = g_item0;
          d.n_items = n_items;
          d.defer = k == 0;
          d.bytes = bytes;
          d.span0_lo = (uint32_t)span0;
          d.span0_hi = (uint32_t)(span0 >> 32);
          *R.desc = d;
        }
        b += k ? k : 1;
        if (nl > 1) lds_publish(&ctl->issue[s], g + 1);
        if (b >= b_end) {  // every group is formed: followers and consumers learn the count
          total = g + 1;
          lds_publish(&ctl->total, total);
        }
      } else {
        bytes = lds_get(&R.desc->bytes);
        span0 = (uint64_t)lds_get(&R.desc->span0_lo) | ((uint64_t)lds_get(&R.desc->span0_hi) << 32);
      }
      ops += issue_share<kNt>(P, l, nl, span0, bytes, (uint32_t)(uintptr_t)R.img);
      mark[s] = ops;
      ++g;
      clk.tick(kRtLIssue);
      continue;
    }
    if (arr < g) {  // nothing to issue now: wait for the oldest share and arrive
      const uint32_t as = arr % S;
      clk.tick(kRtLIdle);
      landed = mark[as];
      vm_wait_n(ops - landed);
      if (team_arrive(&ctl->lcnt[as], nl)) lds_publish(&ctl->full[as], arr + 1);
      if (clk.on) clk.acc[kRtGroups] += 1;
      ++arr;
      clk.tick(kRtLWait);
      continue;
    }
    if (leader ? b >= b_end : g >= lds_get(&ctl->total)) break;
    __builtin_amdgcn_s_sleep(1);
  }
  vm_wait<0>();  // the leader's prefetched handle chunk
  clk.flush();
}

// ---- planner waves (group g % nx): headers and trailers (lane = block),
// interval numbering, then per restart interval (lane = interval): the head
// record and the one after it are parsed, which gives every record of the
// interval a guessed position (head end + i * second record's length).  No
// serial walk: the parser team verifies and corrects the guesses in parallel.
__device__ __forceinline__ void ring_planner(KArgs Pk, uint8_t* smem, const RingLayout& L, uint32_t first,
                                            uint32_t step) {
  const DecodeParams P = load_params(Pk);
  RingCtl* ctl = reinterpret_cast<RingCtl*>(smem);
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t S = P.ring_slots;
  RingClock clk((P.flags & kDiagTimers) != 0);
  for (uint32_t g = first;; g += step) {
    const uint32_t s = g % S;
    if (!ring_wait(&ctl->full[s], g + 1, ctl, g)) break;
    clk.tick(kRtXIdle);
    const RingSlot R = ring_slot(smem, L, s, P.stage_bytes, P.tile_items);
    const uint32_t k = lds_get(&R.desc->k), n_items = lds_get(&R.desc->n_items);
    uint32_t n_iv = 0;
    if (!lds_get(&R.desc->defer) && !(P.flags & kDiagSkipParse)) {
      uint32_t chains = 0;
      BlockMeta m;
      if ((uint32_t)lane < k) {
        const SlotBlk e = R.blk[lane];
        meta_header(R.img, e.hb, e.len, m);  // magic, type, length, header checksum (header.rs:116-169)
        m.item0 = e.item0;
        m.hdr_st = m.st;
        m.ck_bad = 0;
        m.hck_bad = 0;
        meta_trailer(R.img, P.expect_type, e.cap, m);
        if (m.st == ST_OK && m.type == 1) m.st = ST_DEFER;  // index blocks: general path
        chains = m.st == ST_OK ? m.bin_len : 0;
      }
      const uint32_t incl = wave_incl_scan_u32(chains);
      n_iv = wave_readlane_u32(incl, k - 1);
      if (n_iv > kMaxIv) {  // too many intervals for the table: the whole group takes the general path
        if ((uint32_t)lane < k && m.st == ST_OK) m.st = ST_DEFER;
        chains = 0;
        n_iv = 0;
      }
      if ((uint32_t)lane < k) {
        m.chain0 = incl - chains;
        R.meta[lane] = m;
        for (uint32_t r = 0; r < chains; ++r) R.owner[m.chain0 + r] = (uint8_t)lane;
      }
      for (uint32_t i = lane; i < n_items; i += kWave) R.rec_iv[i] = 0xFF;
      wave_sync();
      for (uint32_t c = lane; c < n_iv; c += kWave) {
        const uint32_t j = R.owner[c];
        BlockMeta* mj = &R.meta[j];
        const TrailerInfo t = trailer_of(*mj);
        const uint32_t p0 = mj->p0;
        const uint32_t r = c - mj->chain0;
        const bool last_iv = r + 1 == t.bin_len;
        const uint32_t s_rel = bin_get(R.img, p0, t, r);
        const uint32_t e_rel = last_iv ? t.rec_end : bin_get(R.img, p0, t, r + 1);
        // records lie before the marker; the first one at payload offset 0
        const bool ok = s_rel < t.rec_end && e_rel <= t.rec_end && (r != 0 || s_rel == 0);
        const uint32_t count = ok ? (last_iv ? t.item_count - r * t.ri : t.ri) : 0;
        const uint32_t fi = mj->item0 + r * t.ri;
        Iv iv;
        iv.s = (uint16_t)s_rel;
        iv.e = (uint16_t)e_rel;
        iv.first = (uint16_t)fi;
        iv.last = (uint16_t)(fi + (count ? count - 1 : 0));
        iv.p0 = (uint16_t)p0;
        iv.end = (uint16_t)t.rec_end;
        iv.key = 0;
        iv.live = 0;
        iv.anchor = (uint16_t)(fi + 1);
        iv.cut = (uint16_t)(fi + count);
        iv.apos = iv.stride = iv.apos2 = iv.stride2 = 0;
        iv.pad[0] = iv.pad[1] = 0;
        if (!ok) {
          atomicCAS(&mj->st, ST_OK, ST_PARSE);
        } else {
          for (uint32_t i = 0; i < count; ++i) R.rec_iv[fi + i] = (uint8_t)c;
          ItemFields f;
          uint32_t e0;
          const int rc0 = parse_data_fast(R.img, p0, s_rel, t.rec_end, true, 0, f, e0);
          if (rc0 == 0) mj->st = ST_DEFER;  // a record shape the fast parser does not take (wins over PARSE)
          else if (rc0 < 0) atomicCAS(&mj->st, ST_OK, ST_PARSE);
          if (rc0 > 0) {
            iv.live = 1;
            iv.key = (uint16_t)f.key_off;
            iv.apos = (uint16_t)e0;
            if (count > 1) {
              uint32_t e1;
              const int rc1 = parse_data_fast(R.img, p0, e0, t.rec_end, false, f.key_off, f, e1);
              const uint32_t len1 = rc1 > 0 ? e1 - e0 : 1;
              iv.stride = (uint16_t)len1;
              // Sorted fixed-size records only ever grow, by one byte, when the
              // key's shared prefix with the head shrinks: if the interval is d
              // bytes longer than count - 1 records of len1, guess that the last
              // d records are len1 + 1 (parsers verify every record either way).
              const int32_t d = (int32_t)e_rel - (int32_t)(e0 + (count - 1) * len1);
              if (d > 0 && d < (int32_t)count - 1) {
                iv.cut = (uint16_t)(fi + count - d);
                iv.apos2 = (uint16_t)(e0 + (count - 1 - d) * len1);
                iv.stride2 = (uint16_t)(len1 + 1);
              }
            }
          }
        }
        R.iv[c] = iv;
        R.ivb[c] = (uint8_t)j;
        R.fail[c] = ~0u;
      }
    }
    if (lane == 0) R.desc->n_iv = n_iv;
    lds_publish(&ctl->xdone[s], g + 1);
    clk.tick(kRtXBusy);
  }
  clk.tick(kRtXIdle);
  clk.flush();
}

// Parser-team barrier over LDS (never s_barrier: the other roles do not take part).
__device__ __forceinline__ void team_sync(uint32_t* cnt, uint32_t& target, uint32_t n) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if ((threadIdx.x & (kWave - 1)) == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  target += n;
  while ((int32_t)(lds_get(cnt) - target) < 0) __builtin_amdgcn_s_sleep(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Block statuses in oracle order, then FREE.  Run by whichever of the parser
// team and the group's hasher finishes second (both results are in LDS then).
__device__ __forceinline__ void finish_group(const DecodeParams& P, RingCtl* ctl, const RingSlot& R, uint32_t s,
                                             uint32_t g) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t b = lds_get(&R.desc->b), k = lds_get(&R.desc->k);
  if (lds_get(&R.desc->defer)) {
    if (lane == 0) defer_block(P, b);
  } else if ((uint32_t)lane < k) {
    const BlockMeta& m = R.meta[lane];
    const uint32_t hr = (P.flags & (kDiagSkipParse | kDiagSkipHash)) ? 0u : R.hres[lane];
    const int32_t st = (P.flags & kDiagSkipParse) ? (int32_t)ST_OK
                       : m.hdr_st != ST_OK        ? m.hdr_st  // incl. the header checksum
                       : (hr & 1)                 ? (int32_t)ST_CKSUM
                                                  : m.st;
    if (st == ST_DEFER) defer_block(P, b + lane);
    else gstore(P.status, b + lane, st);
  }
  lds_publish(&ctl->bdone[s], g + 1);
}
// The parser team (its wave 0) and the group's hasher each call this once
// per group; the second caller finishes the group.
__device__ __forceinline__ bool second_to_finish(RingCtl* ctl, uint32_t s) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  uint32_t old = 0;
  if ((threadIdx.x & (kWave - 1)) == 0)
    old = __hip_atomic_fetch_add(&ctl->fin[s], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  old = __builtin_amdgcn_readfirstlane(old);
  if (old == 0) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  if ((threadIdx.x & (kWave - 1)) == 0) __hip_atomic_store(&ctl->fin[s], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return true;
}

// ---- hasher waves (group g % nh): payload xxh3_128 of eight blocks at a time
// (one lane octet per block, xxh3_128_oct_long).  The header checksum is the
// planner's (lane per block).
__device__ __forceinline__ void ring_hasher(KArgs Pk, uint8_t* smem, const RingLayout& L, uint32_t first,
                                           uint32_t step) {
  const DecodeParams P = load_params(Pk);
  RingCtl* ctl = reinterpret_cast<RingCtl*>(smem);
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t S = P.ring_slots;
  const LongSecret* ls = reinterpret_cast<const LongSecret*>(smem + L.secret);
  RingClock clk((P.flags & kDiagTimers) != 0);
  for (uint32_t g = first;; g += step) {
    const uint32_t s = g % S;
    if (!ring_wait(&ctl->full[s], g + 1, ctl, g)) break;
    clk.tick(kRtHIdle);
    const RingSlot R = ring_slot(smem, L, s, P.stage_bytes, P.tile_items);
    const uint32_t k = lds_get(&R.desc->k);
    if (!lds_get(&R.desc->defer) && !(P.flags & kDiagSkipHash)) {
      for (uint32_t jb = lane >> 3; jb < k; jb += 8) {
        const SlotBlk e = R.blk[jb];
        uint32_t res = 0;
        if (e.len >= kHdrLen) {
          uint64_t lo, hi;
          const uint32_t plen = e.len - kHdrLen;
          if (plen > 240) xxh3_128_oct_long(R.img, e.hb + kHdrLen, plen, ls, lo, hi);
          else xxh3_128_short(plen, BaseReader8{R.img, e.hb + kHdrLen}, BaseReader64{R.img, e.hb + kHdrLen}, lo, hi);
          const BaseReader64 hr{R.img, e.hb};
          res = lo != hr(5) || hi != hr(13) ? 1u : 0u;
        }
        if ((lane & 7) == 0) R.hres[jb] = res;
      }
    }
    if (second_to_finish(ctl, s)) {
      ring_wait(&ctl->xdone[s], g + 1, ctl, g);  // (the parser team has waited for it already)
      finish_group(P, ctl, R, s, g);
    }
    clk.tick(kRtHBusy);
  }
  clk.tick(kRtHIdle);
  clk.flush();
}

// ---- parser team (every group, all nb waves): rounds of
//   1. parse: thread t takes records t, t + T, ... (T = 64 nb; the same thread
//      always owns the same record, so its later stores overwrite its earlier
//      ones in program order).  Record k of a live interval is parsed at its
//      guessed position and stored; it is verified iff it parsed and ends
//      exactly where record k + 1 is guessed (the interval end for the last).
//      The first unverified record of each interval is kept (LDS atomicMin).
//   2. advance (thread = interval): records before the first failure f end
//      where their successors start, so f's position is right: a parse error
//      there is the block's (PARSE / general path); f the last record means
//      the interval does not end where the binary index says (PARSE);
//      otherwise the interval is re-anchored at f + 1 = f's end with stride =
//      f's length, and another round runs.
// Every stored record of a good block is thus at its true position and every
// record ends where the next begins, as the serial iterator (decoder.rs:442-483)
// would find them.  After kRounds rounds a still-open interval sends its block
// to the general path.
constexpr uint32_t kRounds = 6;

template <bool kAllFields>
__device__ __forceinline__ void ring_parser(KArgs Pk, uint8_t* smem, const RingLayout& L, uint32_t p, uint32_t nb) {
  const DecodeParams P = load_params(Pk);
  RingCtl* ctl = reinterpret_cast<RingCtl*>(smem);
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t S = P.ring_slots;
  const uint32_t tid = p * kWave + lane, T = nb * kWave;
  const bool store = !(P.flags & kDiagSkipStore);
  uint32_t sync_target = 0;
  RingClock clk((P.flags & kDiagTimers) != 0);
  for (uint32_t g = 0;; ++g) {
    const uint32_t s = g % S;
    if (!ring_wait(&ctl->full[s], g + 1, ctl, g)) break;
    const RingSlot R = ring_slot(smem, L, s, P.stage_bytes, P.tile_items);
    const uint32_t defer = lds_get(&R.desc->defer);
    ring_wait(&ctl->xdone[s], g + 1, ctl, g);  // (also before a defer-only group is freed)
    if (defer) {
      if (p == 0 && second_to_finish(ctl, s)) finish_group(P, ctl, R, s, g);
      continue;
    }
    clk.tick(kRtBIdle);
    const uint32_t n_items = lds_get(&R.desc->n_items), g_item0 = lds_get(&R.desc->g_item0);
    const uint32_t n_iv = lds_get(&R.desc->n_iv);
    const bool parse = !(P.flags & (kDiagSkipParse | kDiagSkipPhaseB)) && n_iv;
    for (uint32_t round = 0; parse && round < kRounds; ++round) {
      // pfail only moves in step 1 and ppend only in step 2: read here, every
      // wave compares against the same values
      const uint32_t fail0 = lds_get(&ctl->pfail), pend0 = lds_get(&ctl->ppend);
      // 1. parse + verify at the guessed positions
      for (uint32_t kk = tid; kk < n_items; kk += T) {
        const uint32_t c = R.rec_iv[kk];
        if (c == 0xFF) continue;
        const Iv iv = R.iv[c];
        if (!iv.live || (round && kk < iv.anchor)) continue;
        const uint32_t p0 = iv.p0, end = iv.end;
        const bool head = kk == iv.first;
        const uint32_t pos = iv_pos(iv, kk);
        ItemFields f;
        uint32_t next;
        const int rc = parse_data_fast(R.img, p0, min(pos, end), end, head, iv.key, f, next);
        if (rc > 0 && store) store_fields(P, kAllFields, (uint64_t)g_item0 + kk, f);
        const uint32_t expect = kk == iv.last ? (uint32_t)iv.e : iv_pos(iv, kk + 1);
        if (!(rc > 0 && next == expect && pos < end)) {
          atomicMin(&R.fail[c], ((kk - iv.first) << 20) | ((uint32_t)(rc > 0 ? 0 : (rc == 0 ? 1 : 2)) << 18) |
                                    (next & 0xFFFF));
          __hip_atomic_fetch_add(&ctl->pfail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      team_sync(&ctl->psync, sync_target, nb);
      // every open record verified: all intervals settled after one barrier (nothing
      // may write the slot past this point: the group can be freed any moment now)
      if (lds_get(&ctl->pfail) == fail0) break;
      // 2. advance every interval (thread = interval)
      for (uint32_t c = tid; c < n_iv; c += T) {
        Iv* ivp = &R.iv[c];
        if (!ivp->live) continue;
        const uint32_t fw = R.fail[c];
        BlockMeta* mj = &R.meta[R.ivb[c]];
        if (fw == ~0u) {
          ivp->live = 0;  // every open record verified: settled
          continue;
        }
        R.fail[c] = ~0u;
        const Iv iv = *ivp;
        const uint32_t fk = iv.first + (fw >> 20), cls = (fw >> 18) & 3, nxt = fw & 0xFFFF;
        if (cls == 1) {
          mj->st = ST_DEFER;  // wins over PARSE
          ivp->live = 0;
        } else if (cls == 2 || fk == iv.last || round + 1 == kRounds) {
          if (cls == 2 || fk == iv.last) atomicCAS(&mj->st, ST_OK, ST_PARSE);
          else mj->st = ST_DEFER;  // still irregular after kRounds: general path
          ivp->live = 0;
        } else {
          const uint32_t pos_f = iv_pos(iv, fk);
          ivp->anchor = (uint16_t)(fk + 1);
          ivp->apos = (uint16_t)nxt;
          ivp->stride = (uint16_t)(nxt - pos_f);
          ivp->cut = (uint16_t)(iv.last + 1);
          __hip_atomic_fetch_add(&ctl->ppend, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      team_sync(&ctl->psync, sync_target, nb);
      if (lds_get(&ctl->ppend) == pend0) break;  // no interval re-anchored: all settled
    }
    clk.tick(kRtBBusy);
    // Every parser wave is past the team's last barrier: wave 0 reports the
    // team; the second of (team, hasher) writes the statuses and frees the slot.
    if (p == 0 && second_to_finish(ctl, s)) finish_group(P, ctl, R, s, g);
    clk.tick(kRtBBusy);
  }
  clk.tick(kRtBIdle);
  clk.flush();
}

template <bool kAllFields, bool kNt>
__global__ __launch_bounds__(kRingWaves * kWave) void decode_ring_kernel(DecodeParams P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const KArgs Pk = kargs();
  const RingLayout L = ring_layout(P.ring_slots, P.stage_bytes, P.tile_items);
  const uint32_t tid = threadIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  if (tid < sizeof(RingCtl) / 4)
    reinterpret_cast<uint32_t*>(smem)[tid] = (tid == offsetof(RingCtl, total) / 4) ? ~0u : 0u;
  if (tid < sizeof(LongSecret) / 8)
    reinterpret_cast<uint64_t*>(smem + L.secret)[tid] = reinterpret_cast<const uint64_t*>(&kLongSecret)[tid];
  __syncthreads();
  const uint32_t nl = P.ring_l, nx = P.ring_x, nh = P.ring_h, nb = kRingWaves - nl - nx - nh;
  if (wave < nl) ring_loader<kNt>(Pk, smem, L, wave, nl);
  else if (wave < nl + nx) ring_planner(Pk, smem, L, wave - nl, nx);
  else if (wave < nl + nx + nh) ring_hasher(Pk, smem, L, wave - nl - nx, nh);
  else ring_parser<kAllFields>(Pk, smem, L, wave - nl - nx - nh, nb);
}

uint32_t decode_ring_lds_bytes(uint32_t slots, uint32_t slot_bytes, uint32_t tile_items) {
  return ring_layout(slots, slot_bytes, tile_items).total;
}

// host[0 .. kTmN): legacy kernel phases; host[16 .. 16 + kRtN): ring roles.
hipError_t read_decode_timers(uint64_t* host, int n, bool reset) {
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_decode_timers), sizeof(uint64_t) * (n < kTmN ? n : kTmN));
  if (e == hipSuccess && n >= 16 + kRtN) e = hipMemcpyFromSymbol(host + 16, HIP_SYMBOL(g_ring_timers), sizeof(uint64_t) * kRtN);
  if (e != hipSuccess || !reset) return e;
  static const unsigned long long zero[16] = {};
  e = hipMemcpyToSymbol(HIP_SYMBOL(g_decode_timers), zero, sizeof(uint64_t) * kTmN);
  if (e != hipSuccess) return e;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_ring_timers), zero, sizeof(uint64_t) * kRtN);
}

// item counts from the trailers (trailer.rs:57-75), same rule as
// oracle/batch.c: 0 unless the handle holds header + a 32-byte minimum payload,
// and at most (payload - 32) / 3 (every record is >= 3 bytes), so a corrupt,
// not-yet-verified trailer cannot reserve more than its bytes could hold.
__global__ __launch_bounds__(256) void trailer_counts_kernel(const uint8_t* __restrict__ blocks,
                                                             const uint64_t* __restrict__ off, uint32_t n,
                                                             uint64_t* __restrict__ counts) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const uint64_t o = off[b], e = off[b + 1];
  uint64_t c = 0;
  if (e >= o && e - o >= kHdrLen + kTrailerLen + 1) {
    const uint8_t* p = blocks + e - 4;
    c = (uint64_t)p[0] | ((uint64_t)p[1] << 8) | ((uint64_t)p[2] << 16) | ((uint64_t)p[3] << 24);
    const uint64_t most = (e - o - kHdrLen - 32) / 3;  // records are >= 3 bytes each
    c = c < most ? c : most;
  }
  counts[b] = c;
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
static size_t defer_bytes(uint32_t n_blocks) { return ((size_t)n_blocks * 4 + 256 + 255) / 256 * 256; }

size_t decode_workspace_size(uint32_t n_blocks) {
  return counts_bytes(n_blocks) + tiles_bytes(n_blocks) + defer_bytes(n_blocks);
}

uint32_t decode_lds_bytes(uint32_t stage_bytes, uint32_t tile_items, uint32_t blocks_per_wave, uint32_t slots) {
  const uint32_t g = blocks_per_wave < kMaxGroup ? blocks_per_wave : kMaxGroup;
  return g * (uint32_t)sizeof(BlockMeta) + ((8 * (tile_items + 1) + 15) & ~15u) + ((tile_items + 15) & ~15u) +
         slots * (((stage_bytes + 15) & ~15u) + kStagePad) + (uint32_t)sizeof(LongSecret);
}

static hipError_t launch_ring(const DecodeParams& P, hipStream_t st);
static hipError_t launch_legacy(const DecodeParams& P, hipStream_t st);

hipError_t launch_decode(const DecodeParams& P0, void* ws, hipStream_t st) {
  DecodeParams P = P0;
  uint64_t* counts = (uint64_t*)ws;
  uint64_t* tiles = (uint64_t*)((uint8_t*)ws + counts_bytes(P.n_blocks));
  uint8_t* dws = (uint8_t*)ws + counts_bytes(P.n_blocks) + tiles_bytes(P.n_blocks);
  P.defer_count = (uint32_t*)dws;
  P.defer_list = (uint32_t*)(dws + 256);
  {
    hipError_t e = hipMemsetAsync(P.defer_count, 0, 4, st);
    if (e != hipSuccess) return e;
  }
  if (!(P.flags & LSM_DECODE_ITEM_START_VALID)) {
    hipLaunchKernelGGL(trailer_counts_kernel, dim3((P.n_blocks + 255) / 256), dim3(256), 0, st, P.blocks,
                       P.block_off, P.n_blocks, counts);
    hipError_t e = launch_excl_scan(counts, P.n_blocks, tiles, ItemStartOut{P.item_start_w, P.item_cap}, st);
    if (e != hipSuccess) return e;
  }
  if (!(P.flags & kDecodeLegacy)) {
    hipError_t e = launch_ring(P, st);
    if (e != hipSuccess) return e;
  } else {
    hipError_t e = launch_legacy(P, st);
    if (e != hipSuccess) return e;
  }
  const uint32_t dgrid = P.n_blocks < 1024 ? P.n_blocks : 1024;
  if (dgrid) {
    static const bool attr = hipFuncSetAttribute((const void*)decode_deferred_staged_kernel,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)(kBigStageOff + kBigStage + kStagePad)) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL(decode_deferred_staged_kernel, dim3(dgrid), dim3(kBigWaves * kWave),
                       kBigStageOff + kBigStage + kStagePad, st, P);
  }
  return hipGetLastError();
}

static hipError_t launch_legacy(const DecodeParams& P, hipStream_t st) {
  const uint32_t lds = decode_lds_bytes(P.stage_bytes, P.tile_items, P.blocks_per_wave, (P.flags & kDecodeDouble) ? 2 : 1);
  const bool timed = (P.flags & kDiagTimers) != 0, all = all_fields(P.out);
  const void* fn = timed ? (all ? (const void*)decode_blocks_kernel<true, true> : (const void*)decode_blocks_kernel<true, false>)
                         : (all ? (const void*)decode_blocks_kernel<false, true> : (const void*)decode_blocks_kernel<false, false>);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const uint32_t grid = (P.n_blocks + P.blocks_per_wave - 1) / P.blocks_per_wave;
  if (timed && all)
    hipLaunchKernelGGL((decode_blocks_kernel<true, true>), dim3(grid), dim3(kGroupWaves * kWave), lds, st, P);
  else if (timed)
    hipLaunchKernelGGL((decode_blocks_kernel<true, false>), dim3(grid), dim3(kGroupWaves * kWave), lds, st, P);
  else if (all)
    hipLaunchKernelGGL((decode_blocks_kernel<false, true>), dim3(grid), dim3(kGroupWaves * kWave), lds, st, P);
  else
    hipLaunchKernelGGL((decode_blocks_kernel<false, false>), dim3(grid), dim3(kGroupWaves * kWave), lds, st, P);
  return hipGetLastError();
}

// Persistent grid: as many ring workgroups as fit on the device at once.
static hipError_t launch_ring(const DecodeParams& P, hipStream_t st) {
  const uint32_t lds = decode_ring_lds_bytes(P.ring_slots, P.stage_bytes, P.tile_items);
  const bool all = all_fields(P.out), nt = (P.flags & kRingNt) != 0;
  const void* fn = all ? (nt ? (const void*)decode_ring_kernel<true, true> : (const void*)decode_ring_kernel<true, false>)
                       : (nt ? (const void*)decode_ring_kernel<false, true> : (const void*)decode_ring_kernel<false, false>);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  int dev = 0, cus = 0, per_cu = 0;
  if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
  if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
  if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kRingWaves * kWave, lds)) != hipSuccess) return e;
  if (per_cu < 1) return hipErrorInvalidConfiguration;
  const uint32_t grid = min((uint32_t)(cus * per_cu), P.n_blocks);
  if (all && nt) hipLaunchKernelGGL((decode_ring_kernel<true, true>), dim3(grid), dim3(kRingWaves * kWave), lds, st, P);
  else if (all) hipLaunchKernelGGL((decode_ring_kernel<true, false>), dim3(grid), dim3(kRingWaves * kWave), lds, st, P);
  else if (nt) hipLaunchKernelGGL((decode_ring_kernel<false, true>), dim3(grid), dim3(kRingWaves * kWave), lds, st, P);
  else hipLaunchKernelGGL((decode_ring_kernel<false, false>), dim3(grid), dim3(kRingWaves * kWave), lds, st, P);
  return hipGetLastError();
}

}  // namespace lsmgpu
