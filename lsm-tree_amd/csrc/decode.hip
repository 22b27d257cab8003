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
#include "scan.hpp"

namespace lsmgpu {

// Diagnostic-only flags (lsm_decode_tuning.flags high bits): drop one phase to
// price it in a profile.  Outputs are NOT valid with any of them set.
constexpr uint32_t kDiagSkipHash = 0x100, kDiagSkipParse = 0x200, kDiagSkipStore = 0x400,
                   kDiagSkipPhaseB = 0x800, kDiagNoPipe = 0x1000;

constexpr uint32_t kMaxGroup = 32;  // blocks per staged group
constexpr uint32_t kStagePad = 256;  // readable LDS bytes past the span (fast parsers read <= 138)

// Phase-A record descriptor (one u64 per group item, LDS): image offsets of
// the record start, of where it must end, and of its restart head's key.
constexpr int kRecEndShift = 16, kRecKeyShift = 32, kRecBlockShift = 48;
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
};
static_assert(sizeof(BlockMeta) == 80, "BlockMeta layout");

__device__ __forceinline__ void wave_sync() {
  // Single-wave workgroups: LDS operations of a wave complete in order, so a
  // compiler barrier is all cross-lane LDS hand-offs need (no s_barrier, and
  // no vmcnt(0) drain of the output stores as __syncthreads would imply).
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void emit_global(const lsm_parsed_items& o, uint64_t i, const ItemFields& f) {
  if (o.seqno) o.seqno[i] = f.seqno;
  if (o.key_off) o.key_off[i] = f.key_off;
  if (o.val_off) o.val_off[i] = f.val_off;
  if (o.val_len) o.val_len[i] = f.val_len;
  if (o.key_len) o.key_len[i] = f.key_len;
  if (o.prefix_len) o.prefix_len[i] = f.prefix_len;
  if (o.vtype) o.vtype[i] = f.vtype;
  if (o.handle_off) o.handle_off[i] = f.handle_off;
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

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

__device__ __forceinline__ uint64_t rec_desc(uint32_t a, uint32_t end, uint32_t key, uint64_t tag) {
  return (uint64_t)a | ((uint64_t)end << kRecEndShift) | ((uint64_t)key << kRecKeyShift) | tag;
}

// Phase A: lane = restart interval c of the group; one descriptor per record
// (start, required end, head key — image offsets) into rec[].  The walk only
// measures record lengths; phase B parses every record in full and checks
// the chain.  The step loop is wave-uniform: lanes past their interval's end
// compute on a harmless position and store to the scratch slot rec[dummy], so
// the only branches are the rare long-suffix read and the Cursor fallback.
__device__ __forceinline__ void phase_a(const uint8_t* img, BlockMeta* meta, const uint8_t* owner, uint64_t* rec,
                                        uint32_t total, uint32_t dummy) {
  const int lane = threadIdx.x;
  for (uint32_t c0 = 0; c0 < total; c0 += kWave) {
    const uint32_t c = c0 + lane;
    const bool live = c < total;
    const uint32_t j = live ? owner[c] : 0;
    const BlockMeta& m = meta[j];
    const TrailerInfo t = trailer_of(m);
    const uint32_t p0 = m.p0, rec_end = m.rec_end;
    const uint32_t r = live ? c - m.chain0 : 0;
    const bool last = r + 1 == t.bin_len;
    const uint32_t s_rel = bin_get(img, p0, t, r);
    const uint32_t e_rel = last ? t.rec_end : bin_get(img, p0, t, r + 1);
    bool ok = s_rel < t.rec_end && e_rel <= t.rec_end;  // records lie before the marker
    const uint32_t count = last ? t.item_count - r * t.ri : t.ri;
    const uint32_t steps = (live && ok) ? count - 1 : 0;  // record lengths to measure
    const uint32_t ib0 = m.item0 + r * t.ri;
    const uint64_t tag = ((uint64_t)j << kRecBlockShift) | kRecValid;
    uint32_t a = p0 + (ok ? s_rel : 0), key = a;
    const uint32_t max_steps = wave_max_u32(steps);
    if (max_steps) {
      // restart head (full key: value length read separately)
      {
        const bool act = steps > 0;
        const Win16u w = ld_win16u(img + a);
        const RecHead hd = rec_head(w.lo, true);
        const uint32_t z = ld_u16u(img + a + hd.q);
        uint32_t n4, vl;
        const bool vl_ok = rec_vlen(z, is_tombstone(hd.vt), n4, vl);
        uint32_t nxt = a + hd.q + n4 + vl;
        key = a + hd.hdr;
        if (act && !(hd.ok && vl_ok && valid_vtype(hd.vt))) {
          ItemFields tmp;
          uint32_t tnext;
          const bool sok = parse_data_slow(img, p0, a - p0, t.rec_end, true, 0, &tmp, &tnext);
          nxt = sok ? p0 + tnext : rec_end;
          key = p0 + tmp.key_off;
        }
        ok = ok && (!act || nxt < rec_end);
        const bool go = act && ok;
        rec[go ? ib0 : dummy] = rec_desc(a, nxt, key, tag | kRecRestart);
        a = go ? nxt : a;
      }
      for (uint32_t jj = 1; jj < max_steps; ++jj) {
        const bool act = jj < steps && ok;
        uint32_t len, hdr;
        uint32_t nxt = a;
        if (data_record_len_fast(img + a, false, len, hdr)) {
          nxt = a + len;
        } else if (act) {
          ItemFields tmp;
          uint32_t tnext;
          const bool sok = parse_data_slow(img, p0, a - p0, t.rec_end, false, key - p0, &tmp, &tnext);
          nxt = sok ? p0 + tnext : rec_end;
        }
        ok = ok && (!act || nxt < rec_end);
        const bool go = act && ok;
        rec[go ? ib0 + jj : dummy] = rec_desc(a, nxt, key, tag);
        a = go ? nxt : a;
      }
    }
    // the interval's last record must end where the next interval (or the marker) begins
    if (live && ok) rec[ib0 + count - 1] = rec_desc(a, p0 + e_rel, key, tag | (count == 1 ? kRecRestart : 0));
    if (live && !ok) atomicCAS(&meta[j].st, ST_OK, ST_PARSE);
  }
}

// Phase B: lane = record.  Full parse + validation of every descriptor, then
// coalesced stores of all fields (a failed block's outputs are unspecified,
// so lanes store unconditionally).
__device__ __forceinline__ void phase_b(const DecodeParams& P, const uint8_t* img, BlockMeta* meta,
                                        const uint64_t* rec, uint32_t n_items, uint32_t g_item0) {
  const int lane = threadIdx.x;
  const bool all_fields = P.out.seqno && P.out.key_off && P.out.val_off && P.out.val_len && P.out.key_len &&
                          P.out.prefix_len && P.out.vtype;
  const bool store = !(P.flags & kDiagSkipStore);
  for (uint32_t i0 = 0; i0 < n_items; i0 += kWave) {
    const uint32_t i = i0 + lane;
    if (i >= n_items) break;
    const uint64_t d = rec[i];
    const uint32_t j = (uint32_t)(d >> kRecBlockShift) & 31;
    const u32x4 hot = *reinterpret_cast<const u32x4*>(&meta[j]);  // p0, rec_end, st, type
    const uint32_t p0 = hot.x, end = hot.y - p0;
    const bool live = (d & kRecValid) && (int32_t)hot.z == ST_OK;
    const uint32_t a = ((uint32_t)d & 0xFFFF) - p0;
    const uint32_t want = ((uint32_t)(d >> kRecEndShift) & 0xFFFF) - p0;
    const uint32_t base_key = ((uint32_t)(d >> kRecKeyShift) & 0xFFFF) - p0;
    const bool restart = (d & kRecRestart) != 0;
    ItemFields f;
    uint32_t next;
    const int rc = parse_data_fast(img, p0, live ? a : 0, end, restart, base_key, f, next);
    bool good = rc > 0 && next == want && hot.w != 1;
    if (live && (rc == 0 || hot.w == 1)) {
      ItemFields tmp;  // only the out-of-line paths take an address (keeps f in registers)
      uint32_t tnext;
      const bool sok = hot.w == 1 ? parse_index_slow(img, p0, a, end, &tmp, &tnext)
                                  : parse_data_slow(img, p0, a, end, restart, base_key, &tmp, &tnext);
      good = sok && tnext == want;
      f = tmp;
    }
    if (live && !good) atomicCAS(&meta[j].st, ST_OK, ST_PARSE);
    if (!store) continue;
    const uint64_t gi = (uint64_t)g_item0 + i;
    if (all_fields) {  // common case: no per-field null checks
      P.out.seqno[gi] = f.seqno;
      P.out.key_off[gi] = f.key_off;
      P.out.val_off[gi] = f.val_off;
      P.out.val_len[gi] = f.val_len;
      P.out.key_len[gi] = f.key_len;
      P.out.prefix_len[gi] = f.prefix_len;
      P.out.vtype[gi] = f.vtype;
      if (P.out.handle_off) P.out.handle_off[gi] = f.handle_off;
    } else {
      emit_global(P.out, gi, f);
    }
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
  if (start > t.rec_end || stop > t.rec_end) return false;
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
__device__ __noinline__ void decode_block_direct(const DecodeParams& P, uint32_t b, BlockMeta* meta) {
  const int lane = threadIdx.x;
  const uint64_t off = P.block_off[b], end = P.block_off[b + 1];
  const uint8_t* base = P.blocks + (off & ~15ULL);
  const uint32_t hb = (uint32_t)(off & 15);
  const uint64_t len = end >= off ? end - off : 0;
  const uint64_t item_base = P.item_start[b];
  const uint32_t cap = P.item_start[b + 1] - P.item_start[b];
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
  if (lane == 0) P.status[b] = meta[0].st;
  wave_sync();
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

constexpr uint32_t kPipeChunks = 16;  // dwordx4 per lane held in flight: 16 KiB per wave

// A group: the longest run of consecutive blocks from b that fits the stage
// (k == 0: block b alone is too large and takes the direct path).  Lane j
// holds block b+j's handle and item range.
struct Group {
  uint32_t b, k, g_item0, n_items;
  uint64_t span0, span1;
  uint64_t off_j, end_j;
  uint32_t it0_j, it1_j;
};

// offr / itr: lane l holds block_off / item_start of block b_begin + l.
__device__ __forceinline__ Group form_group(const DecodeParams& P, uint32_t b, uint32_t b_begin, uint32_t b_end,
                                            uint32_t gmax, uint64_t offr, uint32_t itr) {
  const int lane = threadIdx.x;
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
  const bool fits = in_run && G.end_j >= G.off_j && G.off_j >= off_b &&
                    ((G.end_j + 15) & ~15ULL) - G.span0 <= P.stage_bytes && G.it1_j - G.g_item0 <= P.tile_items;
  G.k = (uint32_t)__builtin_ctzll(~__ballot(fits));  // lanes >= gmax never fit
  G.span1 = G.k ? (wave_readlane_u64(G.end_j, G.k - 1) + 15) & ~15ULL : G.span0;
  G.n_items = G.k ? wave_readlane_u32(G.it1_j, G.k - 1) - G.g_item0 : 0;
  return G;
}

// Steps 3-7 on a group whose bytes are in img.
__device__ __forceinline__ void process_group(const DecodeParams& P, const Group& G, const uint8_t* img,
                                              BlockMeta* meta, uint64_t* rec, uint8_t* owner) {
  const int lane = threadIdx.x;
  const uint32_t k = G.k;
  // ---- 3. lane j: header of block b+j
  if ((uint32_t)lane < k) {
    BlockMeta m;
    meta_header(img, (uint32_t)(G.off_j - G.span0), G.end_j - G.off_j, m);
    m.item0 = G.it0_j - G.g_item0;
    meta[lane] = m;
  }
  wave_sync();
  // ---- 4. payload checksums: DPP row g hashes blocks g, g+4, ...
  if (!(P.flags & kDiagSkipHash)) {
    const uint32_t g = lane >> 4;
    for (uint32_t j = g; j < k; j += 4) {
      if (meta[j].st != ST_OK) continue;
      const uint32_t hb = meta[j].hb, len = meta[j].len;
      uint64_t lo, hi;
      xxh3_128_row(img, hb + kHdrLen, len - kHdrLen, lo, hi);
      if ((lane & 15) == 0 && (lo != meta[j].ck_lo || hi != meta[j].ck_hi)) meta[j].st = ST_CKSUM;
    }
    wave_sync();
  }
  // ---- 5. trailers + restart-interval numbering; owner[c] = block of interval c
  uint32_t chains = 0;
  BlockMeta m;
  if ((uint32_t)lane < k) {
    m = meta[lane];
    meta_trailer(img, P.expect_type, G.it1_j - G.it0_j, m);
    chains = m.st == ST_OK ? m.bin_len : 0;
  }
  const uint32_t incl = wave_incl_scan_u32(chains);
  const uint32_t total = (P.flags & kDiagSkipParse) ? 0 : wave_readlane_u32(incl, 63);
  if ((uint32_t)lane < k) {
    m.chain0 = incl - chains;
    meta[lane] = m;
    if (total)
      for (uint32_t r = 0; r < chains; ++r) owner[m.chain0 + r] = (uint8_t)lane;
  }
  wave_sync();
  // ---- 6. phase A: lane = restart interval, record boundaries only
  phase_a(img, meta, owner, rec, total, P.tile_items);
  wave_sync();
  // ---- 7. phase B: lane = record; full parse + validation; coalesced stores
  if (!(P.flags & (kDiagSkipParse | kDiagSkipPhaseB))) phase_b(P, img, meta, rec, G.n_items, G.g_item0);
  wave_sync();
  if ((uint32_t)lane < k) P.status[G.b + lane] = meta[lane].st;
  wave_sync();
}

// kPipe (stage <= 16 KiB): the next group's span is loaded into registers
// (16 x dwordx4 per lane) while the current group is processed, so HBM
// latency overlaps the parse; the landed registers are written to LDS at the
// top of the next iteration.  !kPipe (larger stages): LDS-DMA, one wait.
template <bool kPipe>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 8))) void decode_blocks_kernel(DecodeParams P) {
  // LDS: [meta: G x 80 B][rec: u64 per item + 1 scratch][owner: u8 per item][staged bytes + pad]
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t gmax = min(kMaxGroup, P.blocks_per_wave);
  BlockMeta* meta = reinterpret_cast<BlockMeta*>(smem);
  uint64_t* rec = reinterpret_cast<uint64_t*>(smem + gmax * (uint32_t)sizeof(BlockMeta));
  uint8_t* owner = reinterpret_cast<uint8_t*>(rec) + ((8 * (P.tile_items + 1) + 15) & ~15u);
  uint8_t* img = owner + ((P.tile_items + 15) & ~15u);
  const int lane = threadIdx.x;
  const uint32_t b_begin = blockIdx.x * P.blocks_per_wave;
  const uint32_t b_end = min(b_begin + P.blocks_per_wave, P.n_blocks);
  // the wave's handles and item starts, once (blocks_per_wave <= 63)
  uint64_t offr = 0;
  uint32_t itr = 0;
  if (b_begin + lane <= b_end) {
    offr = P.block_off[b_begin + lane];
    itr = P.item_start[b_begin + lane];
  }
  u32x4 R[kPipeChunks];
  Group cur = form_group(P, b_begin, b_begin, b_end, gmax, offr, itr);
  if constexpr (kPipe) {
    if (cur.k) {
      const uint32_t chunks = (uint32_t)((cur.span1 - cur.span0) >> 4);
      const u32x4* src = reinterpret_cast<const u32x4*>(P.blocks + cur.span0) + lane;
#pragma unroll
      for (uint32_t i = 0; i < kPipeChunks; ++i)
        if (i * kWave + lane < chunks) R[i] = __builtin_nontemporal_load(src + i * kWave);
    }
  }
  while (cur.b < b_end) {
    if (cur.k == 0) {
      decode_block_direct(P, cur.b, meta);
      cur = form_group(P, cur.b + 1, b_begin, b_end, gmax, offr, itr);
      if constexpr (kPipe) {
        if (cur.k) {
          const uint32_t chunks = (uint32_t)((cur.span1 - cur.span0) >> 4);
          const u32x4* src = reinterpret_cast<const u32x4*>(P.blocks + cur.span0) + lane;
#pragma unroll
          for (uint32_t i = 0; i < kPipeChunks; ++i)
            if (i * kWave + lane < chunks) R[i] = __builtin_nontemporal_load(src + i * kWave);
        }
      }
      continue;
    }
    const uint32_t chunks = (uint32_t)((cur.span1 - cur.span0) >> 4);
    if constexpr (kPipe) {
      // land the prefetched span, then start the next one
      u32x4* dst = reinterpret_cast<u32x4*>(img) + lane;
#pragma unroll
      for (uint32_t i = 0; i < kPipeChunks; ++i)
        if (i * kWave + lane < chunks) dst[i * kWave] = R[i];
      const Group nxt = form_group(P, cur.b + cur.k, b_begin, b_end, gmax, offr, itr);
      if (nxt.b < b_end && nxt.k) {
        const uint32_t nchunks = (uint32_t)((nxt.span1 - nxt.span0) >> 4);
        const u32x4* src = reinterpret_cast<const u32x4*>(P.blocks + nxt.span0) + lane;
#pragma unroll
        for (uint32_t i = 0; i < kPipeChunks; ++i)
          if (i * kWave + lane < nchunks) R[i] = __builtin_nontemporal_load(src + i * kWave);
      }
      for (uint32_t i = lane; i < cur.n_items; i += kWave) rec[i] = 0;
      wave_sync();
      process_group(P, cur, img, meta, rec, owner);
      cur = nxt;
    } else {
      const uint8_t* src = P.blocks + cur.span0 + 16 * lane;
      for (uint32_t i = 0; i * kWave < chunks; ++i) {
        if (i * kWave + lane < chunks)
          __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + 1024 * i), (lds_void_t*)(img + 1024 * i), 16, 0, 0);
      }
      for (uint32_t i = lane; i < cur.n_items; i += kWave) rec[i] = 0;
      __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0): the DMA has landed
      wave_sync();
      process_group(P, cur, img, meta, rec, owner);
      cur = form_group(P, cur.b + cur.k, b_begin, b_end, gmax, offr, itr);
    }
  }
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

size_t decode_workspace_size(uint32_t n_blocks) {
  return ((size_t)n_blocks * 8 + 255) / 256 * 256 + (scan_tiles(n_blocks) * 8 + 255) / 256 * 256;
}

uint32_t decode_lds_bytes(uint32_t stage_bytes, uint32_t tile_items, uint32_t blocks_per_wave) {
  const uint32_t g = blocks_per_wave < kMaxGroup ? blocks_per_wave : kMaxGroup;
  return g * (uint32_t)sizeof(BlockMeta) + ((8 * (tile_items + 1) + 15) & ~15u) + ((tile_items + 15) & ~15u) +
         ((stage_bytes + 15) & ~15u) + kStagePad;
}

hipError_t launch_decode(const DecodeParams& P0, void* ws, hipStream_t st) {
  DecodeParams P = P0;
  uint64_t* counts = (uint64_t*)ws;
  uint64_t* tiles = (uint64_t*)((uint8_t*)ws + ((size_t)P.n_blocks * 8 + 255) / 256 * 256);
  if (!(P.flags & LSM_DECODE_ITEM_START_VALID)) {
    hipLaunchKernelGGL(trailer_counts_kernel, dim3((P.n_blocks + 255) / 256), dim3(256), 0, st, P.blocks,
                       P.block_off, P.n_blocks, counts);
    hipError_t e = launch_excl_scan(counts, P.n_blocks, tiles, ItemStartOut{P.item_start_w, P.item_cap}, st);
    if (e != hipSuccess) return e;
  }
  const uint32_t lds = decode_lds_bytes(P.stage_bytes, P.tile_items, P.blocks_per_wave);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)decode_blocks_kernel<false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const uint32_t grid = (P.n_blocks + P.blocks_per_wave - 1) / P.blocks_per_wave;
  if (P.stage_bytes <= kPipeChunks * 1024 && !(P.flags & kDiagNoPipe))
    hipLaunchKernelGGL(decode_blocks_kernel<true>, dim3(grid), dim3(64), lds, st, P);
  else
    hipLaunchKernelGGL(decode_blocks_kernel<false>, dim3(grid), dim3(64), lds, st, P);
  return hipGetLastError();
}

}  // namespace lsmgpu
