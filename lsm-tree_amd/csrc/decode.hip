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
                   kDiagSkipPhaseB = 0x800;

constexpr uint32_t kMaxGroup = 32;  // blocks per staged group
constexpr uint32_t kNoItem = 0xFFFFFFFFu;
constexpr uint32_t kInfoRestart = 1u << 21;

struct alignas(16) BlockMeta {
  uint64_t ck_lo, ck_hi;
  uint32_t hb;        // byte offset of the header in the image / span
  uint32_t len;       // handle size (header + payload)
  int32_t st;         // lsm_status
  uint32_t type;
  uint32_t ri, step, bin_len, bin_off, item_count, rec_end;
  uint32_t item0;     // first output index relative to the group base
  uint32_t chain0;    // exclusive prefix of restart intervals in the group
};
constexpr uint32_t kMetaBytes = kMaxGroup * sizeof(BlockMeta);

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
  m.item_count = t.item_count; m.rec_end = t.rec_end;
}

__device__ __forceinline__ TrailerInfo trailer_of(const BlockMeta& m) {
  TrailerInfo t;
  t.ri = m.ri; t.step = m.step; t.bin_len = m.bin_len; t.bin_off = m.bin_off;
  t.item_count = m.item_count; t.rec_end = m.rec_end;
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

// Phase A for restart interval r of group block j: record start positions
// (payload-relative, u16) into info[], the interval head's key offset into
// bkey[].  The last record's end is checked in phase B.
__device__ __forceinline__ bool walk_boundaries(const uint8_t* img, const BlockMeta& m, uint32_t j, uint32_t r,
                                                uint32_t* info, uint16_t* bkey) {
  const TrailerInfo t = trailer_of(m);
  const uint32_t p0 = m.hb + kHdrLen;
  const uint32_t start = bin_get(img, p0, t, r);
  const uint32_t count = (r + 1 == t.bin_len) ? t.item_count - r * t.ri : t.ri;
  const uint32_t ib0 = m.item0 + r * t.ri;
  if (start >= t.rec_end) return false;  // a record must start before the trailer marker
  info[ib0] = start | (j << 16) | kInfoRestart;
  if (m.type == 1) return true;          // index blocks: one record per restart interval
  uint32_t p = start;
  for (uint32_t jj = 0; jj + 1 < count; ++jj) {
    uint32_t next, key_off;
    const int rc = data_record_next_fast(img, p0, p, t.rec_end, jj == 0, next, key_off);
    if (rc < 0) return false;
    if (rc == 0) {
      ItemFields tmp;
      uint32_t tnext;
      if (!parse_data_slow(img, p0, p, t.rec_end, jj == 0, jj == 0 ? 0 : bkey[ib0], &tmp, &tnext)) return false;
      key_off = tmp.key_off;
      next = tnext;
    }
    if (jj == 0) bkey[ib0] = (uint16_t)key_off;
    p = next;
    if (p >= t.rec_end) return false;
    info[ib0 + jj + 1] = p | (j << 16);
  }
  return true;
}

// Phase B for group item i: full parse at its recorded start, checking that
// the record ends exactly where the next one (or the interval) begins.
__device__ __forceinline__ bool parse_item(const uint8_t* img, const BlockMeta& m, uint32_t i, uint32_t inf,
                                           const uint32_t* info, const uint16_t* bkey, ItemFields& f) {
  if (m.st != ST_OK) return false;
  const TrailerInfo t = trailer_of(m);
  const uint32_t p0 = m.hb + kHdrLen;
  const uint32_t p = inf & 0xFFFF;
  const uint32_t ib = i - m.item0;
  const uint32_t r = ib / t.ri, jj = ib - r * t.ri;
  const bool last = jj + 1 == t.ri || ib + 1 == t.item_count;
  const uint32_t base_key = jj ? bkey[m.item0 + r * t.ri] : 0;
  uint32_t next;
  if (!parse_record(img, p0, p, t, m.type, jj == 0, base_key, f, next)) return false;
  const uint32_t expect = last ? (r + 1 < t.bin_len ? bin_get(img, p0, t, r + 1) : t.rec_end)
                               : (info[i + 1] & 0xFFFF);
  return next == expect;
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

__global__ __launch_bounds__(64) void decode_blocks_kernel(DecodeParams P) {
  // LDS: [meta: kMaxGroup x 64 B][info: u32 per item][bkey: u16 per item][staged bytes]
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  BlockMeta* meta = reinterpret_cast<BlockMeta*>(smem);
  uint32_t* info = reinterpret_cast<uint32_t*>(smem + kMetaBytes);
  uint16_t* bkey = reinterpret_cast<uint16_t*>(smem + kMetaBytes + 4 * P.tile_items);
  uint8_t* img = smem + kMetaBytes + ((6 * P.tile_items + 15) & ~15u);
  const int lane = threadIdx.x;
  const uint32_t b_begin = blockIdx.x * P.blocks_per_wave;
  const uint32_t b_end = min(b_begin + P.blocks_per_wave, P.n_blocks);

  for (uint32_t b = b_begin; b < b_end;) {
    // ---- 1. group formation; lane j keeps block b+j's handle and item range
    const uint32_t bj = b + lane;
    const bool in_run = bj < b_end && (uint32_t)lane < kMaxGroup;
    uint64_t off_j = 0, end_j = 0;
    uint32_t it0_j = 0, it1_j = 0;
    if (in_run) {
      off_j = P.block_off[bj];
      end_j = P.block_off[bj + 1];
      it0_j = P.item_start[bj];
      it1_j = P.item_start[bj + 1];
    }
    const uint64_t off_b = wave_bcast_u64(off_j, 0);
    const uint32_t g_item0 = wave_bcast_u32(it0_j, 0);
    const uint64_t span0 = off_b & ~15ULL;
    const bool fits = in_run && end_j >= off_j && off_j >= off_b &&
                      ((end_j + 15) & ~15ULL) - span0 <= P.stage_bytes && it1_j - g_item0 <= P.tile_items;
    const uint64_t fit_mask = __ballot(fits);
    const uint32_t k = (uint32_t)__builtin_ctzll(~fit_mask);  // lanes >= kMaxGroup never fit
    if (k == 0) {
      decode_block_direct(P, b, meta);
      b += 1;
      continue;
    }
    const uint64_t span1 = (wave_bcast_u64(end_j, k - 1) + 15) & ~15ULL;
    const uint32_t n_items = wave_bcast_u32(it1_j, k - 1) - g_item0;
    // ---- 2. stage the group's bytes HBM -> LDS by LDS-DMA, one wait
    {
      const uint32_t chunks = (uint32_t)((span1 - span0) >> 4);
      const uint8_t* src = P.blocks + span0 + 16 * lane;
      for (uint32_t i = 0; i * kWave < chunks; ++i) {
        if (i * kWave + lane < chunks)
          __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + 1024 * i), (lds_void_t*)(img + 1024 * i), 16, 0, 0);
      }
      for (uint32_t i = lane; i < n_items; i += kWave) info[i] = kNoItem;
      __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0): the DMA has landed
      wave_sync();
    }
    // ---- 3. lane j: header of block b+j
    if ((uint32_t)lane < k) {
      BlockMeta m;
      meta_header(img, (uint32_t)(off_j - span0), end_j - off_j, m);
      m.item0 = it0_j - g_item0;
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
    // ---- 5. trailers + restart-interval numbering
    uint32_t chains = 0;
    if ((uint32_t)lane < k) {
      BlockMeta m = meta[lane];
      meta_trailer(img, P.expect_type, it1_j - it0_j, m);
      chains = m.st == ST_OK ? m.bin_len : 0;
      m.chain0 = 0;
      meta[lane] = m;
    }
    const uint32_t incl = wave_incl_scan_u32(chains);
    const uint32_t total = (P.flags & kDiagSkipParse) ? 0 : wave_bcast_u32(incl, 63);
    if ((uint32_t)lane < k) meta[lane].chain0 = incl - chains;
    wave_sync();
    // ---- 6. phase A: lane = restart interval, record boundaries only
    for (uint32_t c = lane; c < total; c += kWave) {
      uint32_t lo = 0, hi = k - 1;
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (meta[mid].chain0 <= c) lo = mid; else hi = mid - 1;
      }
      const uint32_t j = lo;
      if (!walk_boundaries(img, meta[j], j, c - meta[j].chain0, info, bkey)) atomicCAS(&meta[j].st, ST_OK, ST_PARSE);
    }
    wave_sync();
    // ---- 7. phase B: lane = record; full parse + validation; coalesced stores
    const uint32_t parse_items = (P.flags & (kDiagSkipParse | kDiagSkipPhaseB)) ? 0 : n_items;
    const bool all_fields = P.out.seqno && P.out.key_off && P.out.val_off && P.out.val_len && P.out.key_len &&
                            P.out.prefix_len && P.out.vtype;
    const bool store = !(P.flags & kDiagSkipStore);
    for (uint32_t i = lane; i < parse_items; i += kWave) {
      const uint32_t inf = info[i];
      if (inf == kNoItem) continue;
      const uint32_t j = (inf >> 16) & 31;
      ItemFields f;
      if (!parse_item(img, meta[j], i, inf, info, bkey, f)) {
        atomicCAS(&meta[j].st, ST_OK, ST_PARSE);
        continue;
      }
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
    wave_sync();
    if ((uint32_t)lane < k) P.status[b + lane] = meta[lane].st;
    wave_sync();
    b += k;
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

uint32_t decode_lds_bytes(uint32_t stage_bytes, uint32_t tile_items) {
  // the last DMA instruction of a group may land up to 1008 B past the span
  return kMetaBytes + ((6 * tile_items + 15) & ~15u) + ((stage_bytes + 1023) & ~1023u) + 64;
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
  const uint32_t lds = decode_lds_bytes(P.stage_bytes, P.tile_items);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)decode_blocks_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const uint32_t grid = (P.n_blocks + P.blocks_per_wave - 1) / P.blocks_per_wave;
  hipLaunchKernelGGL(decode_blocks_kernel, dim3(grid), dim3(64), lds, st, P);
  return hipGetLastError();
}

}  // namespace lsmgpu
